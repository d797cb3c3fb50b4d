#!/bin/bash
# AddressSanitizer run of the library's HOST code (the device == -1 backend: host_step, the
# queries, the spawn resolver, the VJP host path, argument checks) -- device code is built as usual
# (GPU sanitizers are not available on the pool).  Builds build/asan/pkg/libvmas_mi355x.so and runs the
# CPU test files that drive the host backend with the clang ASAN runtime preloaded.
set -eu
cd "$(dirname "$0")/.."
# (laid out like the package: the specialised-step compiler finds its headers at <lib dir>/csrc and
# <lib dir>/../include)
mkdir -p build/asan/pkg
ln -sfn "$PWD/vectorizedmultiagentsimulator_amd/csrc" build/asan/pkg/csrc
ln -sfn "$PWD/include" build/asan/include
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
SRCS=(vectorizedmultiagentsimulator_amd/csrc/vmas_kernels.hip vectorizedmultiagentsimulator_amd/csrc/vmas_spawn.hip
      vectorizedmultiagentsimulator_amd/csrc/vmas_actions.hip vectorizedmultiagentsimulator_amd/csrc/vmas_jit.hip
      vectorizedmultiagentsimulator_amd/csrc/vmas_scenarios.hip vectorizedmultiagentsimulator_amd/csrc/vmas_copy.hip
      vectorizedmultiagentsimulator_amd/csrc/vmas_grad.hip)
"$HIPCC" --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -shared-libasan \
    -I include -o build/asan/pkg/libvmas_mi355x.so "${SRCS[@]}" -lhiprtc -ldl
echo "built build/asan/pkg/libvmas_mi355x.so (host code instrumented)"
export VMAS_LIB_PATH=$PWD/build/asan/pkg/libvmas_mi355x.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:print_summary=1
# every CPU test file but the build check (it rebuilds the normal library) and the multi-process
# gloo tests (child interpreters without the preload)
LD_PRELOAD=$RT python -m pytest -x -q -m "not gpu" -p no:cacheprovider tests \
    --ignore=tests/test_build.py --ignore=tests/test_distributed.py "$@"
