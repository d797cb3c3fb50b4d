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
#include <cstdio>
#include <cstdlib>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"
#include "vmas_uniform.hpp"

namespace {

constexpr int kCopyThreads = 256, kCopyUnroll = 4, kMaxCopyBlocks = 1024;

struct CopyArgs {
    VmasCopySpan s[VMAS_COPY_MAX_SPANS];
    int n;
    int nt;  // non-temporal stores (VMAS_COPY_NT=1, an A/B knob): the destinations are fresh tensors
};
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
static_assert(sizeof(CopyArgs) <= 4096, "kernel argument block");

// blk / nblk: this workgroup's index among the span's nblk workgroups (grid-stride over them)
template <typename T, bool NT = false>
__device__ __forceinline__ void copy_units(const T* __restrict__ src, T* __restrict__ dst, int64_t n, int blk, int nblk) {
    const int64_t step = (int64_t)nblk * kCopyThreads;
    int64_t i = (int64_t)blk * kCopyThreads + threadIdx.x;
    for (; i + (kCopyUnroll - 1) * step < n; i += kCopyUnroll * step) {
        T v[kCopyUnroll];
#pragma unroll
        for (int k = 0; k < kCopyUnroll; ++k) v[k] = src[i + k * step];  // independent loads in flight
#pragma unroll
        for (int k = 0; k < kCopyUnroll; ++k) {
            if constexpr (NT) __builtin_nontemporal_store(v[k], dst + i + k * step);
            else dst[i + k * step] = v[k];
        }
    }
    for (; i < n; i += step) dst[i] = src[i];
}

__device__ __forceinline__ void copy_span(const VmasCopySpan& s, bool nt, int blk, int nblk) {
    if (s.nbytes == VMAS_COPY_STORE64) {  // a store span: the 8-byte value src at dst
        if (blk == 0 && threadIdx.x == 0) *reinterpret_cast<uint64_t*>(s.dst) = (uint64_t)(uintptr_t)s.src;
        return;
    }
    if (!s.src) {  // an increment span: dst[i] += 1.0f
        float* d = reinterpret_cast<float*>(s.dst);
        const int64_t n = s.nbytes / 4;
        for (int64_t i = (int64_t)blk * kCopyThreads + threadIdx.x; i < n; i += (int64_t)nblk * kCopyThreads)
            d[i] = d[i] + 1.0f;
        return;
    }
    const uintptr_t al = (uintptr_t)s.src | (uintptr_t)s.dst | (uintptr_t)s.nbytes;
    if ((al & 15) == 0 && nt)
        copy_units<u32x4, true>(reinterpret_cast<const u32x4*>(s.src), reinterpret_cast<u32x4*>(s.dst), s.nbytes / 16,
                                blk, nblk);
    else if ((al & 15) == 0)
        copy_units(reinterpret_cast<const uint4*>(s.src), reinterpret_cast<uint4*>(s.dst), s.nbytes / 16, blk, nblk);
    else if ((al & 3) == 0)
        copy_units(reinterpret_cast<const uint32_t*>(s.src), reinterpret_cast<uint32_t*>(s.dst), s.nbytes / 4, blk, nblk);
    else
        copy_units(reinterpret_cast<const uint8_t*>(s.src), reinterpret_cast<uint8_t*>(s.dst), s.nbytes, blk, nblk);
}

__global__ void __launch_bounds__(kCopyThreads) k_copy_spans(CopyArgs a) {
    copy_span(a.s[blockIdx.y], a.nt != 0, (int)blockIdx.x, (int)gridDim.x);
}

// The post-replay copies and the next step's random-action draw in ONE launch (vmas_copy_spans_draw).
// Packed grid (default): item y (span y < n_spans, else draw column y - n_spans) owns the 1-D
// workgroups [first[y], first[y + 1]) -- a copy span as many as its bytes need (<= 1024), a column
// exactly torch's gx_draw -- so no workgroup is launched only to leave (the 2-D grid of
// max(copy, draw) x items launched ~10 000 of them per step for ~1 000 that work).  VMAS_COPY_PACKED=0:
// the 2-D grid (blockIdx.y = item, blocks beyond the item's share leave; an A/B knob).
constexpr int kMergedSpans = 96, kMergedCols = 16;
struct CopyDrawArgs {
    VmasCopySpan s[kMergedSpans];
    VmasUniformColumn c[kMergedCols];
    unsigned long long seed;
    long long numel, snap;
    const unsigned long long* off_dev;  // (non-null: the columns' offsets are relative to *off_dev)
    int n_spans, gx_draw, mode, n_items;
    int first[kMergedSpans + kMergedCols + 1];  // packed grid: the items' first workgroups (n_items + 1)
    int gx_copy, packed;
};
static_assert(sizeof(CopyDrawArgs) <= 4096, "kernel argument block");

__global__ void __launch_bounds__(kCopyThreads) k_copy_draw(CopyDrawArgs a) {
    int y, blk;
    if (a.packed) {  // the item owning this workgroup: the last y with first[y] <= blockIdx.x
        const int bx = (int)blockIdx.x;
        int lo = 0, hi = a.n_items - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.first[mid] <= bx) lo = mid;
            else hi = mid - 1;
        }
        y = lo;
        blk = bx - a.first[y];
    } else {
        y = (int)blockIdx.y;
        blk = (int)blockIdx.x;
        if (y < a.n_spans ? blk >= a.gx_copy : blk >= a.gx_draw) return;
    }
    if (y < a.n_spans) {
        copy_span(a.s[y], false, blk, a.packed ? a.first[y + 1] - a.first[y] : a.gx_copy);
        return;
    }
    VmasUniformColumn col = a.c[y - a.n_spans];
    if (a.off_dev) col.offset += *a.off_dev;  // (the generator offset a device launch left: see the ABI)
    vmas_uniform::draw_column(col, a.seed, a.numel, a.snap, a.mode, a.gx_draw, blk);
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

// a span the launch can run: a copy, an increment (src NULL: whole floats) or a store (STORE64)
static bool span_ok(const VmasCopySpan& s) {
    if (s.nbytes == VMAS_COPY_STORE64) return s.dst && ((uintptr_t)s.dst & 7) == 0;
    return s.nbytes >= 0 && (s.nbytes == 0 || s.dst) && (s.src || (s.nbytes % 4 == 0 && ((uintptr_t)s.dst & 3) == 0));
}

extern "C" int32_t vmas_copy_spans(int32_t device, const VmasCopySpan* spans, int32_t n, void* stream) {
    if (n < 0 || (n > 0 && !spans) || device < 0) return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans: bad arguments");
    VMAS_AUX_HIP(hipSetDevice(device));
    static const int nt = getenv("VMAS_COPY_NT") && getenv("VMAS_COPY_NT")[0] == '1';
    for (int first = 0; first < n; first += VMAS_COPY_MAX_SPANS) {
        CopyArgs a{};
        a.n = 0;
        a.nt = nt;
        int64_t most = 0;  // units of the largest span (16-byte units: sets the grid)
        for (int i = first; i < std::min(n, first + VMAS_COPY_MAX_SPANS); ++i) {
            const VmasCopySpan& s = spans[i];
            if (!span_ok(s)) return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans: bad span %d", i);
            if (s.nbytes == 0 || (s.nbytes > 0 && s.src == s.dst)) continue;
            a.s[a.n++] = s;
            most = std::max<int64_t>(most, s.nbytes > 0 ? (s.nbytes + 15) / 16 : 1);
        }
        if (a.n == 0) continue;
        const int64_t per_block = (int64_t)kCopyThreads * kCopyUnroll;
        const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxCopyBlocks, (most + per_block - 1) / per_block));
        hipLaunchKernelGGL(k_copy_spans, dim3(gx, a.n), dim3(kCopyThreads), 0, (hipStream_t)stream, a);
        VMAS_AUX_HIP(hipGetLastError());
    }
    return VMAS_OK;
}

extern "C" int32_t vmas_copy_spans_draw(int32_t device, const VmasCopySpan* spans, int32_t n_spans, int64_t numel,
                                        const VmasUniformColumn* cols, int32_t n_cols, uint64_t seed, uint64_t offset,
                                        const uint64_t* offset_dev, int32_t mode, int64_t u_snap_delta,
                                        uint64_t* increment, void* stream) {
    if (device < 0 || n_spans < 0 || n_spans > kMergedSpans || (n_spans > 0 && !spans) || n_cols <= 0 ||
        n_cols > kMergedCols || !cols || numel <= 0 || !increment || mode < 0 || mode > 3)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans_draw: bad arguments");
    VMAS_AUX_HIP(hipSetDevice(device));
    static int max_blocks[64] = {0};
    if (device >= 64) return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans_draw: device %d", device);
    if (!max_blocks[device]) {
        hipDeviceProp_t prop;
        VMAS_AUX_HIP(hipGetDeviceProperties(&prop, device));
        max_blocks[device] = prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / vmas_uniform::kThreads);
        if (max_blocks[device] <= 0) return vmas_aux::fail(VMAS_E_HIP, "vmas_copy_spans_draw: device properties");
    }
    int gx_draw = 0;
    unsigned long long inc = 0;
    vmas_uniform::grid_for(numel, max_blocks[device], &gx_draw, &inc);
    CopyDrawArgs a{};
    int64_t most = 0;
    int n = 0;
    for (int i = 0; i < n_spans; ++i) {
        const VmasCopySpan& sp = spans[i];
        if (!span_ok(sp)) return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans_draw: bad span %d", i);
        if (sp.nbytes == 0 || (sp.nbytes > 0 && sp.src == sp.dst)) continue;
        a.s[n++] = sp;
        most = std::max<int64_t>(most, sp.nbytes > 0 ? (sp.nbytes + 15) / 16 : 1);
    }
    for (int i = 0; i < n_cols; ++i) {
        if (!cols[i].out) return vmas_aux::fail(VMAS_E_INVALID, "vmas_copy_spans_draw: null column %d", i);
        a.c[i] = cols[i];
        a.c[i].offset = offset + inc * (unsigned long long)i;
    }
    a.seed = seed;
    a.numel = numel;
    a.snap = u_snap_delta;
    a.off_dev = reinterpret_cast<const unsigned long long*>(offset_dev);
    a.n_spans = n;
    a.gx_draw = gx_draw;
    a.mode = mode;
    const int64_t per_block = (int64_t)kCopyThreads * kCopyUnroll;
    const int gx_copy = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxCopyBlocks, (most + per_block - 1) / per_block));
    static const int packed = !(getenv("VMAS_COPY_PACKED") && getenv("VMAS_COPY_PACKED")[0] == '0');
    // packed grid: 16-byte units per thread a span's share is sized for (VMAS_COPY_UNITS, an A/B
    // knob: 1 = four times the workgroups, each thread one load in flight)
    static const int units_per_thread = getenv("VMAS_COPY_UNITS") ? std::max(1, std::min(kCopyUnroll, atoi(getenv("VMAS_COPY_UNITS")))) : kCopyUnroll;
    const int64_t per_share = (int64_t)kCopyThreads * units_per_thread;
    a.gx_copy = gx_copy;
    a.packed = packed;
    a.n_items = n + n_cols;
    int total = 0;
    for (int y = 0; y < n + n_cols; ++y) {
        a.first[y] = total;
        if (y < n) {  // a span's own share: its 16-byte units over 256 threads x 4, at least one
            const VmasCopySpan& sp = a.s[y];
            const int64_t units = sp.nbytes > 0 ? (sp.nbytes + 15) / 16 : 1;
            total += (int)std::max<int64_t>(1, std::min<int64_t>(kMaxCopyBlocks, (units + per_share - 1) / per_share));
        } else {
            total += gx_draw;
        }
    }
    a.first[n + n_cols] = total;
    static int trace = getenv("VMAS_COPY_TRACE") ? atoi(getenv("VMAS_COPY_TRACE")) : 0;
    if (trace > 0) {  // (a diagnostic: the first calls' span list, to stderr)
        --trace;
        int64_t bytes = 0;
        for (int i = 0; i < n; ++i) bytes += a.s[i].nbytes > 0 ? a.s[i].nbytes : 0;
        fprintf(stderr, "[vmas_copy_spans_draw] spans %d cols %d numel %lld bytes %lld grid %d x %d (copy %d draw %d) packed %d\n",
                n, n_cols, (long long)numel, (long long)bytes, std::max(gx_copy, gx_draw), n + n_cols, gx_copy, gx_draw,
                total);
        for (int i = 0; i < n; ++i)
            fprintf(stderr, "  span %d: %lld bytes%s\n", i, (long long)a.s[i].nbytes, a.s[i].src ? "" : " (increment)");
    }
    if (packed)
        hipLaunchKernelGGL(k_copy_draw, dim3((unsigned)total), dim3(kCopyThreads), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(k_copy_draw, dim3((unsigned)std::max(gx_copy, gx_draw), n + n_cols), dim3(kCopyThreads), 0,
                           (hipStream_t)stream, a);
    VMAS_AUX_HIP(hipGetLastError());
    *increment = inc * (unsigned long long)n_cols;
    return VMAS_OK;
}
