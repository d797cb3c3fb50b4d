#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace.  Stops at the first step that
# times out / crashes (exit 124, 134, 137, 139); plain test failures (exit 1) do not stop it.
#   SESSION_STEPS="tests bench prof" OUT=gpurun_out/r5a bash tools/gpu_session.sh
# TESTS (for the "tests" step) narrows the pytest selection (default: the whole -m gpu suite).
set -u
OUT="${OUT:-gpurun_out}"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-100}"
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 12 "$OUT/$name.log"
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
    return 0
}
rocm-smi --showproductname > "$OUT/gpu_info.log" 2>&1 || true
lscpu > "$OUT/lscpu.log" 2>&1 || true
for step in ${SESSION_STEPS:-tests bench prof}; do
  case $step in
    tests) run pytest_gpu 1100 python -u -m pytest ${TESTS:-tests} -m gpu ${XFLAG--x} -v -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
    bench) run bench 600 python bench.py --steps "$STEPS" --warmup 10 ;;
    benchdef) run bench_default 600 python bench.py ;;
    bench_c3) run bench_c3 600 python bench.py --scenario transport --steps "$STEPS" --warmup 10 --cpu-steps 0 ;;
    bench_c4) run bench_c4 600 python bench.py --scenario discovery --steps "$STEPS" --warmup 10 --cpu-steps 0 ;;
    bench_c5) run bench_c5 600 python bench.py --scenario flocking --steps "$STEPS" --warmup 10 --cpu-steps 0 ;;
    bench_c5full) run bench_c5full 600 python bench.py --scenario flocking --envs 262144 --steps 50 --warmup 10 --cpu-steps 0 ;;
    bench_eager) run bench_eager 600 python bench.py --graph off --steps "$STEPS" --warmup 10 --cpu-steps 0 ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-steps 0 ;;
    profdef) run rocprof_default 900 rocprofv3 --kernel-trace --stats -d "$OUT/profdef" -o run --output-format csv -- python bench.py ;;
    bench20) run bench_20 600 python bench.py --steps 20 --warmup 5 --cpu-steps 0 ;;
    hostprof_eager) run hostprof_eager 600 python tools/host_profile.py balance 32768 200 eager ;;
  esac
done
echo "session done"
