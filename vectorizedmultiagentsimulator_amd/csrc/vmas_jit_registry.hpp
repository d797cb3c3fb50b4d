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
    long wbd_offset;      // byte offset of Args.wbd (the state write-back's backup delta, vmas_jit.hip wb_helpers)
    long tail_offset;     // byte offset of Args.tail (a VmasTail, vmas_tail.hpp; -1: the module has none)
    int batch;
    int epilogue;         // VMAS_EPILOGUE_*
    size_t io_bytes;      // the program's argument block (VmasBalanceIO / VmasTransportIO)
};

bool jit_fn_info(const void* f, JitFnInfo* out);

// Release the device copies of freed kernel chains (vmas_graph_chain_free defers them: a chain may
// be dropped while a stream is capturing, where hipFree is not allowed).  Called at the next chain
// build and when a world is destroyed (never during a capture: engines dropped while a stream
// captures are destroyed later, simulator/_engine.py drain_deferred).
void chain_free_drain();

}  // namespace vmas
