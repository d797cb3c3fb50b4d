// vmas_uniform.hpp -- one column of PyTorch's uniform_ kernel on the device (vmas_actions.hip
// k_uniform_columns; vmas_copy.hip k_copy_draw): thread idx of torch's grid of `blocks` x 256
// threads initialises philox4x32-10 at (seed, subsequence = idx, column offset), draws 4 numbers
// per grid-stride round for elements idx + k * threads, maps them to (0, 1] and to [from, to)
// (the two float roundings fused or not: `mode`, probed against torch by the host).
#pragma once

#include <hip/hip_runtime.h>

#include <rocrand/rocrand_philox4x32_10.h>

#include "vmas_mi355x.h"

namespace vmas_uniform {

constexpr int kThreads = 256;

__device__ __forceinline__ float unit_float(unsigned int v, bool fused) {
    const float inv = 2.3283064e-10f;  // ROCRAND_2POW32_INV
    return fused ? __builtin_fmaf((float)v, inv, inv) : inv + (float)v * inv;
}

// Block `block` of the column's draw (blocks = torch's grid size for numel elements).  With a
// second output (col.u_out) the drawn value is also written as the action kernel applies it;
// snap != 0: that element's previous value is first stored snap bytes from it.
__device__ __forceinline__ void draw_column(const VmasUniformColumn& col, unsigned long long seed, long long numel,
                                            long long snap, int mode, int blocks, int block) {
    const long long idx = (long long)block * kThreads + threadIdx.x;
    rocrand_state_philox4x32_10 st;
    rocrand_init(seed, (unsigned long long)idx, col.offset, &st);
    const long long step = (long long)kThreads * blocks;
    const long long rounded = ((numel - 1) / (step * 4) + 1) * step * 4;
    const float from = col.from, to = col.to, range = to - from;
    const bool fused_unit = mode & 1, fused_affine = mode & 2;
    for (long long li0 = idx; li0 < rounded; li0 += step * 4) {
        const uint4 v = rocrand4(&st);
        const unsigned int vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long li = li0 + step * k;
            if (li < numel) {
                const float r = unit_float(vv[k], fused_unit);
                const float val = fused_affine ? __builtin_fmaf(r, range, from) : r * range + from;
                const float x = val == to ? from : val;  // (0, 1] -> [from, to)
                col.out[li * col.stride] = x;
                if (col.u_out) {  // apply_one's operations on the same value
                    const float u = col.u_clamp ? fminf(fmaxf(x, -col.u_range), col.u_range) : x;
                    float* uo = col.u_out + li * col.u_stride;
                    if (snap) *reinterpret_cast<float*>(reinterpret_cast<char*>(uo) + snap) = *uo;
                    *uo = u * col.u_mult;
                }
            }
        }
    }
}

// torch's distribution-kernel grid for numel elements and the per-call philox increment
// (counter_offset, rounded up to a multiple of 4); max_blocks = CUs x (maxThreadsPerCU / 256)
inline void grid_for(long long numel, int max_blocks, int* blocks, unsigned long long* inc) {
    const long long gx = (numel + kThreads - 1) / kThreads < max_blocks ? (numel + kThreads - 1) / kThreads : max_blocks;
    *blocks = (int)gx;
    *inc = (unsigned long long)((numel - 1) / (kThreads * gx * 4) + 1) * 4;
}

}  // namespace vmas_uniform
