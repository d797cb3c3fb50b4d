set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in exact relaxed exact relaxed; do
  VMAS_JIT_MATH=$m timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/bench_math_$m.json 2> gpurun_out/bench_math_$m.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/bench_math_$m.json')); print('$m', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['roofline']['kernel_us_per_launch'])"
done
VMAS_JIT_MATH=relaxed timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_jit.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_relaxed.log 2>&1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_relaxed.log | tail -40
