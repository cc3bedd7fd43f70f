# Round-6 GPU check of the GPU resize: its kernel tests + the loader tests, then one short bench run (its
# from_files object carries the GPU-resize and PIL-resize loader legs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_resample.py tests/test_image_pipeline.py > gpurun_out/resize_tests.log 2>&1
rc=$?
tail -15 gpurun_out/resize_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_resize.json 2> gpurun_out/bench_resize.err
rc=$?
tail -c 2500 gpurun_out/bench_resize.json
exit $rc
