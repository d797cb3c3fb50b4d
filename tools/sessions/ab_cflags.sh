#!/bin/bash
# A/B of code-generation options for the specialised step kernel (VMAS_JIT_CFLAGS, appended to
# the defaults of csrc/vmas_jit.hip compile()) at C2, interleaved twice.  Prints per variant: the
# in-kernel launch time, the HIP-event launch time, M env-steps/s.
set -u
mkdir -p gpurun_out/abc
run() {  # tag, flags
  VMAS_JIT_CFLAGS="$2" timeout -k 10 200 python bench.py --steps 60 --warmup 10 --cpu-steps 0 > gpurun_out/abc/$1.json 2> gpurun_out/abc/$1.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/abc/$1.json')); r=d['roofline']; print('$1', r['kernel_us_per_launch'], r.get('kernel_us_event'), round(d['value']/1e6,1))"
}
for rep in 1 2; do
  run base$rep ""
  run maxilp$rep "-mllvm -amdgpu-sched-strategy=max-ilp"
  run iterilp$rep "-mllvm -amdgpu-sched-strategy=iterative-ilp"
  run bias0_$rep "-mllvm -amdgpu-schedule-metric-bias=0"
done
