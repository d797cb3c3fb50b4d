set -u
mkdir -p gpurun_out/bisect
timeout -k 10 300 env VMAS_JIT_PRM_MASK=0x2 python tools/features_nan_probe.py > gpurun_out/bisect/nan_probe.log 2>&1; echo rc=$?
