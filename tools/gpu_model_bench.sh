mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py > gpurun_out/tests_model.log 2>&1; rc=$?; tail -3 gpurun_out/tests_model.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -3 gpurun_out/bench.err; exit $rc
