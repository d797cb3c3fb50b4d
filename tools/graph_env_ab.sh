#!/bin/bash
# A/B of HIP runtime graph settings on graph-mode step time (balance 32k, 10 substeps)
set -u
for cfg in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 HIP_FORCE_DEV_KERNARG=1"; do
  echo "== [$cfg]"
  env $cfg timeout -k 10 120 python tools/graph_probe.py balance 2>&1 | grep -E "ms/step|FAILED" || exit $?
done
