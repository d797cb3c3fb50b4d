#!/bin/bash
# A/B of two library builds (abtmp/libvmas_{old,new}.so: default flags vs -fno-slp-vectorize for
# the AOT kernels), interleaved, with a rocprofv3 kernel-stats pass of each (stats CSV kept only).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/ab_lib
mkdir -p $OUT
LIB=vectorizedmultiagentsimulator_amd/libvmas_mi355x.so
CFGS=${CFGS:-"discovery|--scenario discovery --n-agents 8 --substeps 0 --kw {\"use_agent_lidar\":true}"}
for rep in 1 2; do
for v in old new; do
  cp abtmp/libvmas_$v.so $LIB
  while IFS= read -r cfg; do
    [ -z "$cfg" ] && continue
    name=${cfg%%|*}; args=${cfg#*|}
    timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-steps 0 $args > $OUT/${name}_${v}.json 2> $OUT/${name}_${v}.log || exit 1
    python -c "import json; d=json.load(open('$OUT/${name}_${v}.json')); print('$name $v', d['ms_per_step'], round(d['value']/1e6,1))"
    if [ $rep = 1 ]; then
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_${name}_${v} -o run -- python bench.py --steps 30 --warmup 5 --cpu-steps 0 $args > /dev/null 2>&1 || exit 1
      find /tmp/prof_${name}_${v} -name "*kernel_stats.csv" -exec cp {} $OUT/${name}_${v}_kernel_stats.csv \;
    fi
  done <<< "$CFGS"
done
done
cp abtmp/libvmas_new.so $LIB
