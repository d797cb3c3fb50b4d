// vmas_copy.hip -- one launch for a list of device-to-device byte copies (graph mode's carried
// state, output clones and per-step backups; simulator/environment/_graph.py).
//
// torch._foreach_copy_ over the handful of large tensors a step hands on launched PyTorch's
// multi-tensor-apply kernel once per dtype and call site (4 launches per balance step, 75-171
// workgroups each, 40 us of GPU time for ~14 MB).  Here every span of a call -- whatever its
// dtype -- goes in ONE launch: blockIdx.y = span, blockIdx.x grid-strides over the span in 16-byte
// (or, for unaligned spans, 4- / 1-byte) units, 256 threads x 4 units per workgroup round.
// HBM-bound: 2 x bytes of traffic.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"

namespace {

constexpr int kCopyThreads = 256, kCopyUnroll = 4, kMaxCopyBlocks = 1024;

struct CopyArgs {
    VmasCopySpan s[VMAS_COPY_MAX_SPANS];
    int n;
};
static_assert(sizeof(CopyArgs) <= 4096, "kernel argument block");

template <typename T>
__device__ __forceinline__ void copy_units(const T* __restrict__ src, T* __restrict__ dst, int64_t n) {
    const int64_t step = (int64_t)gridDim.x * kCopyThreads;
    int64_t i = (int64_t)blockIdx.x * kCopyThreads + threadIdx.x;
    for (; i + (kCopyUnroll - 1) * step < n; i += kCopyUnroll * step) {
        T v[kCopyUnroll];
#pragma unroll
        for (int k = 0; k < kCopyUnroll; ++k) v[k] = src[i + k * step];  // independent loads in flight
#pragma unroll
        for (int k = 0; k < kCopyUnroll; ++k) dst[i + k * step] = v[k];
    }
    for (; i < n; i += step) dst[i] = src[i];
}

__global__ void __launch_bounds__(kCopyThreads) k_copy_spans(CopyArgs a) {
    const VmasCopySpan& s = a.s[blockIdx.y];
    if (!s.src) {  // an increment span: dst[i] += 1.0f
        float* d = reinterpret_cast<float*>(s.dst);
        const int64_t n = s.nbytes / 4;
        for (int64_t i = (int64_t)blockIdx.x * kCopyThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kCopyThreads)
            d[i] = d[i] + 1.0f;
        return;
    }
    const uintptr_t al = (uintptr_t)s.src | (uintptr_t)s.dst | (uintptr_t)s.nbytes;
    if ((al & 15) == 0)
        copy_units(reinterpret_cast<const uint4*>(s.src), reinterpret_cast<uint4*>(s.dst), s.nbytes / 16);
    else if ((al & 3) == 0)
        copy_units(reinterpret_cast<const uint32_t*>(s.src), reinterpret_cast<uint32_t*>(s.dst), s.nbytes / 4);
    else
        copy_units(reinterpret_cast<const uint8_t*>(s.src), reinterpret_cast<uint8_t*>(s.dst), s.nbytes);
}

constexpr int kFillThreads = 256;

__global__ void __launch_bounds__(kFillThreads) k_fill_u32(uint32_t* __restrict__ dst, uint32_t value, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kFillThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kFillThreads)
        dst[i] = value;
}

}  // namespace

hipError_t vmas_aux::fill_u32_async(void* dst, uint32_t value, size_t n_words, hipStream_t stream) {
    if (n_words == 0) return hipSuccess;
    const int64_t n = (int64_t)n_words;
    const int gx = (int)std::min<int64_t>(1024, (n + kFillThreads - 1) / kFillThreads);
    hipLaunchKernelGGL(k_fill_u32, dim3(gx), dim3(kFillThreads), 0, stream, (uint32_t*)dst, value, n);
    return hipGetLastError();
}

extern "C" int32_t vmas_copy_spans(int32_t device, const VmasCopySpan* spans, int32_t n, void* stream) {
    if (n < 0 || (n > 0 && !spans) || device < 0) return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans: bad arguments");
    VMAS_AUX_HIP(hipSetDevice(device));
    for (int first = 0; first < n; first += VMAS_COPY_MAX_SPANS) {
        CopyArgs a{};
        a.n = 0;
        int64_t most = 0;  // units of the largest span (16-byte units: sets the grid)
        for (int i = first; i < std::min(n, first + VMAS_COPY_MAX_SPANS); ++i) {
            const VmasCopySpan& s = spans[i];
            if (s.nbytes < 0 || (s.nbytes > 0 && !s.dst) ||
                (!s.src && (s.nbytes % 4 != 0 || ((uintptr_t)s.dst & 3) != 0)))
                return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans: bad span %d", i);
            if (s.nbytes == 0 || s.src == s.dst) continue;
            a.s[a.n++] = s;
            most = std::max<int64_t>(most, (s.nbytes + 15) / 16);
        }
        if (a.n == 0) continue;
        const int64_t per_block = (int64_t)kCopyThreads * kCopyUnroll;
        const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxCopyBlocks, (most + per_block - 1) / per_block));
        hipLaunchKernelGGL(k_copy_spans, dim3(gx, a.n), dim3(kCopyThreads), 0, (hipStream_t)stream, a);
        VMAS_AUX_HIP(hipGetLastError());
    }
    return VMAS_OK;
}
