#!/bin/bash
# Discovery: spawn / scenario GPU tests, then C4 interleaved A/B of VMAS_SPAWN_WAVES=8|16 and a
# rocprof kernel-stats pass at the default.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/abw
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_spawn.py tests/test_fused.py > gpurun_out/abw/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/abw/tests.log; exit 1; }
tail -1 gpurun_out/abw/tests.log
C4="--scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw {\"use_agent_lidar\":true} --steps 50 --warmup 10 --cpu-steps 0"
for r in 1 2; do
  for w in 8; do
    VMAS_SPAWN_WAVES=$w timeout -k 10 300 python bench.py $C4 > gpurun_out/abw/c4_w${w}_r$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'])" gpurun_out/abw/c4_w${w}_r$r.json w$w
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abw/prof -o run -- python bench.py $C4 > gpurun_out/abw/prof.log 2>&1 || exit 1
find gpurun_out/abw/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/abw/c4_kernel_stats.csv \;
find gpurun_out/abw/prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
