#!/bin/bash
# Interleaved A/B of two builds of the library (abtmp/libvmas_{new,old}.so, swapped into the package).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/ab_two
mkdir -p $OUT
LIB=vectorizedmultiagentsimulator_amd/libvmas_mi355x.so
for rep in 1 2 3; do
  for v in new old; do
    cp abtmp/libvmas_$v.so $LIB
    for cfg in "balance|" "flocking|--scenario flocking --n-agents 8 --substeps 0"; do
      name=${cfg%%|*}; args=${cfg#*|}
      timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-steps 0 $args > $OUT/${name}_${v}_${rep}.json 2> $OUT/${name}_${v}_${rep}.log || exit 1
      python -c "import json; d=json.load(open('$OUT/${name}_${v}_${rep}.json')); r=d['roofline']; print('$name $v', r['kernel_us_per_launch'], round(d['value']/1e6,1))"
    done
  done
done
cp abtmp/libvmas_new.so $LIB
