set -e
export PYTHONPATH=$PWD/map-anything_amd:$PWD/tests
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_modules.py > gpurun_out/t_model.log 2>&1
timeout -k 10 300 python -u tools/ab_model.py outconv 8 5 5 > gpurun_out/ab_outconv.log 2>&1
