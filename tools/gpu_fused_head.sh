set -e
export PYTHONPATH=$PWD/map-anything_amd:$PWD/tests
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "regressor_head or halo" > gpurun_out/t_head.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py > gpurun_out/t_model.log 2>&1
timeout -k 10 300 python -u tools/ab_model.py fusedhead 8 5 5 > gpurun_out/ab_fused.log 2>&1
