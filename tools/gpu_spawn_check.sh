set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-steps 0 --scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw '{"use_agent_lidar": true}' > gpurun_out/c4.json 2> gpurun_out/c4.log; echo rc=$?; cat gpurun_out/c4.json
