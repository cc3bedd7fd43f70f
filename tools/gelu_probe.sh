mkdir -p gpurun_out; timeout -k 10 200 python -u tools/gelu_probe.py > gpurun_out/gelu_probe.log 2>&1; rc=$?; cat gpurun_out/gelu_probe.log | grep -v amdgpu.ids; exit $rc
