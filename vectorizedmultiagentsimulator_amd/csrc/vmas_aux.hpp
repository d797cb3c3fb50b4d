// vmas_aux.hpp -- shared host helpers of the auxiliary entry points (vmas_spawn.hip,
// vmas_actions.hip): the error channel behind vmas_aux_last_error and the host-side wait on a
// word of mapped pinned memory that a kernel publishes.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

namespace vmas_aux {

// record the message returned by vmas_aux_last_error; returns code (vmas_spawn.hip)
int32_t fail(int32_t code, const char* fmt, ...);

// Count a host wait on the device (a stream / event synchronisation or a spin on a published
// word) for vmas_host_waits: graph mode's check that a step can be captured (vmas_spawn.hip).
void note_host_wait();

// Spin until *word == seq (a kernel on `stream` stores it with system scope).  While waiting,
// the stream is polled every few thousand reads: an error, or an idle stream without the store,
// ends the wait with VMAS_E_HIP instead of spinning forever.
int32_t wait_host_word(const uint32_t* word, uint32_t seq, hipStream_t stream);
// The same for a 64-bit word whose high half is the sequence number (its low half is a payload
// published by the same single store); the whole word goes to *value.
int32_t wait_host_word64(const uint64_t* word, uint32_t seq, uint64_t* value, hipStream_t stream);

// Sets n_words 32-bit words at dst to value, stream-ordered, as a KERNEL launch (vmas_copy.hip).
// Used in place of hipMemsetAsync wherever the call can sit on a captured stream: a memset node
// of a captured graph misbehaved twice on ROCm 7.2 / MI355X ("Graph mode": a node
// found not complete before the next kernel, and words left holding pointer-like data), while a
// kernel node is ordered and parameterised like every other node of the graph.
hipError_t fill_u32_async(void* dst, uint32_t value, size_t n_words, hipStream_t stream);

}  // namespace vmas_aux

#define VMAS_AUX_HIP(x)                                                                               \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            (void)hipGetLastError();                                                                  \
            return vmas_aux::fail(VMAS_E_HIP, "%s: %s", #x, hipGetErrorString(e_));                   \
        }                                                                                             \
    } while (0)
