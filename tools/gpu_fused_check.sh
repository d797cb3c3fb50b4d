#!/bin/bash
# Fused scenario programs: parity tests against the torch programs, then fused vs torch benches.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fused.py tests/test_graph.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/pytest_fused.log | tail -n 40; [ $rc -eq 0 ] || exit $rc
for cfg in "balance||" "balance_torch|VMAS_FUSED_SCENARIOS=0|" "flocking||--scenario flocking --n-agents 8 --substeps 0" "flocking_torch|VMAS_FUSED_SCENARIOS=0|--scenario flocking --n-agents 8 --substeps 0" "transport||--scenario transport --n-agents 4 --substeps 0" "transport_torch|VMAS_FUSED_SCENARIOS=0|--scenario transport --n-agents 4 --substeps 0" "discovery||--scenario discovery --n-agents 8 --substeps 0 --envs 16384 --kw {\"use_agent_lidar\":true}" "discovery_torch|VMAS_FUSED_SCENARIOS=0|--scenario discovery --n-agents 8 --substeps 0 --envs 16384 --kw {\"use_agent_lidar\":true}"; do
  IFS='|' read -r name envs args <<< "$cfg"
  # shellcheck disable=SC2086
  env $envs timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 $args > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/bench_$name.json')); print('$name', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['roofline']['kernel_us_per_launch'], d['config']['step_mode'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flock -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-steps 0 --scenario flocking --n-agents 8 --substeps 0 > gpurun_out/prof_flock.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_disc -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-steps 0 --scenario discovery --n-agents 8 --substeps 0 --envs 16384 --kw '{"use_agent_lidar":true}' > gpurun_out/prof_disc.log 2>&1 || exit $?
echo done
python - <<'PY'
import csv
rows = list(csv.DictReader(open(__import__("glob").glob("gpurun_out/prof_flock/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_world"]
i0, i1 = idx[-8], idx[-7]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f} {r['Grid_Size_X']:>7}x{r['Grid_Size_Y']:>4} {r['Kernel_Name'][:70]}")
PY
