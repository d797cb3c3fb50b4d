#!/bin/bash
# Full GPU evidence session: the GPU test suite, the bench line, a rocprofv3 kernel trace and the
# PMC passes of the step kernel (tools/pmc_session.sh).  Stops at the first fatal step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SESSION_STEPS="${SESSION_STEPS:-tests bench prof}" bash tools/gpu_session.sh || exit $?
if [ "${PMC:-1}" = "1" ]; then
  TAG=final bash tools/pmc_session.sh || exit $?
fi
echo "full session done"
