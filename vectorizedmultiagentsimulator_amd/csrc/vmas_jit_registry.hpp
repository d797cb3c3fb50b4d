// vmas_jit_registry.hpp -- what the library knows about the kernels of the loaded world modules
// (csrc/vmas_jit.hip registers them; vmas_graph_chain_build in vmas_kernels.hip reads them).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace vmas {

constexpr int kJitFnWorld = 0;    // k_world
constexpr int kJitFnProgram = 1;  // k_program_jit (modules compiled with a scenario program)

struct JitFnInfo {
    int kind;
    const void* world;    // the VmasJitWorld
    hipFunction_t world_fn;  // its k_world
    size_t arg_bytes;     // k_world's argument block
    long epi_offset;      // byte offset of Args.epi in it (-1: no epilogue)
    int batch;
    int epilogue;         // VMAS_EPILOGUE_*
    size_t io_bytes;      // the program's argument block (VmasBalanceIO / VmasTransportIO)
};

bool jit_fn_info(const void* f, JitFnInfo* out);

}  // namespace vmas
