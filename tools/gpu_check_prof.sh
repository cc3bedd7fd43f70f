# GPU kernel + model parity tests, then a short rocprofv3 kernel-stats run of the default bench
set -o pipefail
export PYTHONPATH=$PWD/map-anything_amd:$PWD/tests TMPDIR=/tmp
mkdir -p gpurun_out/qprof
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/t_check.log 2>&1 || { tail -30 gpurun_out/t_check.log; exit 1; }
tail -2 gpurun_out/t_check.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 > gpurun_out/qprof_bench.json 2> gpurun_out/qprof.err || { tail -20 gpurun_out/qprof.err; exit 1; }
tail -c 300 gpurun_out/qprof_bench.json
