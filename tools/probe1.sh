set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python tools/kworld_probe.py balance 32768 batch > gpurun_out/probe_batch.log 2>&1
timeout -k 10 240 python tools/kworld_probe.py balance 32768 env > gpurun_out/probe_env.log 2>&1
VMAS_JIT_PROFILE=200 timeout -k 10 240 python tools/kworld_probe.py balance 32768 batch > gpurun_out/probe_prof.log 2>&1
VMAS_JIT_GRID=host timeout -k 10 240 python tools/kworld_probe.py balance 32768 batch > gpurun_out/probe_host.log 2>&1
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/step_breakdown.log 2>&1
cat gpurun_out/probe_*.log
