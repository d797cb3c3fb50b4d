#!/bin/bash
# Dependent-launch cost of small kernels in a replayed graph under runtime settings (one box).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/node_ab
run() {  # run <name> <env assignments...>
  local name=$1; shift
  timeout -k 10 120 env "$@" python tools/graph_node_probe.py 300 32768 > gpurun_out/node_ab/$name.json 2> gpurun_out/node_ab/$name.log
  local rc=$?; echo "$name rc=$rc $(cat gpurun_out/node_ab/$name.json)"
  case $rc in 0) ;; *) exit $rc;; esac
}
for rep in 1 2; do
  run default_$rep X=1
  run devkernarg1_$rep HIP_FORCE_DEV_KERNARG=1
  run devkernarg0_$rep HIP_FORCE_DEV_KERNARG=0
  run pktcap0_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run pktcap1_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
done
