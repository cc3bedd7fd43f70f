set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./ab_libs/bl/bl || exit 1
MAPA_AB_LIB=$PWD/ab_libs/slow/libmapa.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k attention -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_slow.log 2>&1; tail -3 gpurun_out/attn_slow.log
