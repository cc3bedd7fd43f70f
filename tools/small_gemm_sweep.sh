set -o pipefail
export TMPDIR=/tmp KB_F16=1 KB_ROUNDS=3
export KB_SHAPES="10952,96,1024;10952,768,192;10952,192,768;10952,256,256;43808,256,256;175232,256,256;10952,1536,96;2888,256,256;10952,784,784;10952,384,768"
export KB_VARIANTS=0,1282,643,2571,2570,2568,2580,2581,2603,2600
timeout -k 10 600 python tools/kbench.py gemm 20 > gpurun_out/ksweep.log 2>&1 || { tail -20 gpurun_out/ksweep.log; exit 1; }
cat gpurun_out/ksweep.log
