set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "bilinear" --timeout 120 --timeout-method thread > gpurun_out/bil_test.log 2>&1; tail -2 gpurun_out/bil_test.log
for i in 1 2; do for v in new old; do echo "== $v"; MAPA_AB_LIB=$PWD/ab_libs/$v/libmapa.so timeout -k 10 120 python tools/kbench.py bil 20 2>&1 | grep bil; done; done
