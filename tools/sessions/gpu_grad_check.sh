#!/bin/bash
# Autograd evidence: the gradient tests on the GPU (native VJPs vs the oracle's autograd, the
# restated test_vmas_differentiable), then the whole GPU suite.  Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_autograd.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/grad_tests.log 2>&1 || { echo "grad tests failed rc=$?"; tail -40 gpurun_out/grad_tests.log; exit 1; }
tail -3 gpurun_out/grad_tests.log
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu suite failed rc=$?"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
echo "grad check done"
