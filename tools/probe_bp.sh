export TMPDIR=/tmp
timeout -k 10 240 env VMAS_JIT_PROFILE=0 python tools/kworld_probe.py balance 32768 batch > gpurun_out/kp_batch.log 2>&1 && \
timeout -k 10 240 env VMAS_JIT_PROFILE=0 python tools/kworld_probe.py balance 32768 env > gpurun_out/kp_env.log 2>&1 && \
timeout -k 10 240 python tools/kworld_probe.py balance 32768 env > gpurun_out/kp_env_noprof.log 2>&1 && \
timeout -k 10 240 python tools/kworld_probe.py balance 32768 batch > gpurun_out/kp_batch_noprof.log 2>&1
