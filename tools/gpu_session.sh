#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace.  Stops at the first step that
# times out / crashes (exit 124, 134, 137, 139); plain test failures (exit 1) do not stop it.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-100}"
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
    return 0
}
rocm-smi --showproductname > gpurun_out/gpu_info.log 2>&1 || true
lscpu > gpurun_out/lscpu.log 2>&1 || true
for step in ${SESSION_STEPS:-tests bench prof}; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
    bench) run bench 600 python bench.py --steps "$STEPS" --warmup 10 ;;
    benchenv) run bench_env 600 python bench.py --steps "$STEPS" --warmup 10 --broadphase env --cpu-steps 0 ;;
    breakdown) run step_breakdown 300 python tools/step_breakdown.py ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-steps 0 ;;
  esac
done
echo "session done"
