#!/bin/bash
set -u
mkdir -p gpurun_out/stepk
export TMPDIR=/tmp
timeout -k 10 300 env STEP_GRAPH=0 python tools/step_kernels.py balance 32768 4 > gpurun_out/stepk/balance_eager.log 2>&1; echo rc=$?
timeout -k 10 300 python tools/step_kernels.py balance 32768 4 > gpurun_out/stepk/balance_graph.log 2>&1; echo rc=$?
