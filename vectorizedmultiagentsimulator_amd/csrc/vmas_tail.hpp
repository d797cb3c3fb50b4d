// vmas_tail.hpp -- a replay's post-replay work run by the step kernel's own workgroups after the
// fixed point's final decision (the "tail" of a fused k_world launch; vmas_jit.hip world_body,
// vmas_kernels.hip vmas_graph_chain_launch_tail).
//
// Graph mode ends every replay with one more launch (k_copy_draw, vmas_copy.hip): the carry of
// re-bound attributes, the next replay's output-buffer words, the step counter and the next step's
// random actions drawn ahead.  At C2 that launch is ~5.7 us of a ~48 us step, most of it the fixed
// cost of a second kernel.  In a single-launch chain (k_world with the scenario program as its
// epilogue) the same items can run inside k_world: once the final pass is decided no workgroup of
// the launch reads the step's inputs again, so every thread of the launch takes a share of the
// items' units.  A draw column's element keeps torch's grid and mapping (its philox subsequence is
// the torch thread that draws it), so any thread may compute it, bit for bit.
//
// Visibility inside the launch: a copy's source was written by other workgroups of this launch,
// possibly on another XCD, whose L2 is not coherent with this one.  The host admits a copy only
// when its source is written through (sc1: k_world's state outputs st_out*, the programs' carried
// outputs) and the tail loads it with agent-scope loads (L2 bypassed); everything the tail
// writes is read by later launches only (the kernel boundary orders it).
#pragma once

#ifndef __HIPCC_RTC__  // (hipRTC: vmas_physics.hpp provides the fixed-width types)
#include <stdint.h>
#endif

#include "../../include/vmas_mi355x.h"

constexpr int kTailSpans = 16, kTailCols = 12, kTailThreads = 256;

// The items of one tail (trivially copyable: packed into k_world's argument block per launch).
// Items y < n_spans are copy / increment / store spans (VmasCopySpan, as vmas_copy_spans), the
// rest draw columns (VmasUniformColumn, as vmas_uniform_columns_snap); item y owns the units
// [first[y], first[y + 1]) (a copy's 8- or 4-byte words, an increment's floats, one store word, a
// column's elements).  n_items == 0: no tail.
struct VmasTail {
    VmasCopySpan s[kTailSpans];
    VmasUniformColumn c[kTailCols];
    unsigned long long seed;
    long long numel, snap;
    const unsigned long long* off_dev;  // (non-null: the columns' offsets are relative to *off_dev)
    int n_spans, n_items, gx_draw, mode;
    int first[kTailSpans + kTailCols + 1];
    int pad;
};

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
namespace vmas_tail {

// rocrand's philox4x32-10 block function (as vmas_spawn.hip philox10)
__device__ __forceinline__ uint4 philox10(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const unsigned long long p0 = (unsigned long long)c.x * 0xD2511F53u;
        const unsigned long long p1 = (unsigned long long)c.z * 0xCD9E8D57u;
        const unsigned int hi0 = (unsigned int)(p0 >> 32), lo0 = (unsigned int)p0;
        const unsigned int hi1 = (unsigned int)(p1 >> 32), lo1 = (unsigned int)p1;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

// One unit of the tail: a draw column's element, a copy's word, an increment's float or a store
// word.  prep() computes it and issues its load (the copy's source at agent scope, the increment's
// float, the draw's previous action value for the snapshot); finish() stores.  run() preps two units
// before finishing either, so a thread's loads are in flight together.
struct Unit {
    int kind;  // 0 none, 1 draw, 2 copy u64, 3 copy u32, 4 increment, 5 store64
    float x, u;
    unsigned long long v;
    void* dst;
    float* out;
    float* uo;
};

// Element li of draw column `col` (vmas_uniform::draw_column's thread li % step, round-robin over
// torch's grid): rocrand_init(seed, subsequence idx, offset) + rocrand4 of round r = q / 4, output
// q % 4 (q = li / step) -- the counter (offset / 4 + r, idx) under key seed, shifted by offset % 4
// into the next block (rocrand's interleave).
__device__ __forceinline__ void prep_draw(const VmasTail& t, const VmasUniformColumn& col, long long li, Unit& w) {
    const long long step = (long long)kTailThreads * t.gx_draw;
    const long long q = li / step, idx = li - q * step;
    const unsigned long long off = col.offset + (t.off_dev ? *t.off_dev : 0ull);
    const unsigned long long c = off / 4 + (unsigned long long)(q / 4);
    const int k = (int)(q % 4) + (int)(off & 3ull);
    const uint2 key = make_uint2((unsigned int)t.seed, (unsigned int)(t.seed >> 32));
    const unsigned int ilo = (unsigned int)idx, ihi = (unsigned int)((unsigned long long)idx >> 32);
    const unsigned long long cc = c + (k >= 4 ? 1ull : 0ull);
    const uint4 v = philox10(make_uint4((unsigned int)cc, (unsigned int)(cc >> 32), ilo, ihi), key);
    const int kk = k & 3;
    const unsigned int bits = kk == 0 ? v.x : kk == 1 ? v.y : kk == 2 ? v.z : v.w;
    const float inv = 2.3283064e-10f;  // ROCRAND_2POW32_INV
    const float u01 = (t.mode & 1) ? __builtin_fmaf((float)bits, inv, inv) : inv + (float)bits * inv;
    const float from = col.from, to = col.to, range = to - from;
    const float val = (t.mode & 2) ? __builtin_fmaf(u01, range, from) : u01 * range + from;
    w.kind = 1;
    w.x = val == to ? from : val;  // (0, 1] -> [from, to)
    w.out = col.out + li * col.stride;
    w.uo = nullptr;
    if (col.u_out) {  // apply_one's operations on the same value (vmas_uniform.hpp)
        w.u = (col.u_clamp ? fminf(fmaxf(w.x, -col.u_range), col.u_range) : w.x) * col.u_mult;
        w.uo = col.u_out + li * col.u_stride;
        if (t.snap) w.v = __float_as_uint(*w.uo);  // (the previous value, for the snapshot)
    }
}

__device__ __forceinline__ void prep(const VmasTail& t, long long u, Unit& w) {
    w.kind = 0;
    if (u >= (long long)t.first[t.n_items]) return;
    int lo = 0, hi = t.n_items - 1;  // the item owning unit u: the last y with first[y] <= u
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((long long)t.first[mid] <= u) lo = mid;
        else hi = mid - 1;
    }
    const long long i = u - t.first[lo];
    if (lo >= t.n_spans) {
        prep_draw(t, t.c[lo - t.n_spans], i, w);
        return;
    }
    const VmasCopySpan& s = t.s[lo];
    if (s.nbytes == VMAS_COPY_STORE64) {
        w.kind = 5;
        w.dst = s.dst;
        w.v = (unsigned long long)s.src;
    } else if (!s.src) {  // an increment span: dst[i] += 1.0f
        w.kind = 4;
        w.dst = reinterpret_cast<float*>(s.dst) + i;
        w.x = *reinterpret_cast<const float*>(w.dst);
    } else if ((((unsigned long long)s.src | (unsigned long long)s.dst | (unsigned long long)s.nbytes) & 7) == 0) {
        w.kind = 2;
        w.dst = reinterpret_cast<unsigned long long*>(s.dst) + i;
        w.v = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(s.src) + i, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    } else {  // (4-byte aligned: the host's admission)
        w.kind = 3;
        w.dst = reinterpret_cast<uint32_t*>(s.dst) + i;
        w.v = __hip_atomic_load(reinterpret_cast<const uint32_t*>(s.src) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ void finish(const VmasTail& t, const Unit& w) {
    switch (w.kind) {
        case 1:
            *w.out = w.x;
            if (w.uo) {
                if (t.snap) *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(w.uo) + t.snap) = (uint32_t)w.v;
                *w.uo = w.u;
            }
            break;
        case 2: *reinterpret_cast<unsigned long long*>(w.dst) = w.v; break;
        case 3: *reinterpret_cast<uint32_t*>(w.dst) = (uint32_t)w.v; break;
        case 4: *reinterpret_cast<float*>(w.dst) = w.x + 1.0f; break;
        case 5: *reinterpret_cast<unsigned long long*>(w.dst) = w.v; break;
        default: break;
    }
}

// This thread's units of the tail: every thread of the launch strides over the units (first[] holds
// their prefix counts), two at a time.
__device__ __forceinline__ void run(const VmasTail& t) {
    const long long T = (long long)gridDim.x * blockDim.x, total = t.first[t.n_items];
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += 2 * T) {
        Unit a, b;
        prep(t, u, a);
        prep(t, u + T, b);
        finish(t, a);
        finish(t, b);
    }
}

}  // namespace vmas_tail
#endif
