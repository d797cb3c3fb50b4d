// vmas_actions.hip -- the continuous-action side of Environment.step for every agent in one pass
// (reference vmas/simulator/environment/environment.py:615-709, _set_action, continuous actions
// without communication): NaN check (621-623), optional clamp to u_range (636-640), range check
// (651-655) and u = physical * u_multiplier (709), gfx950 kernel + host backend + C ABI.
//
// The reference runs ~5 torch ops and one host sync per agent; here one launch covers all agents
// and the host learns the flags without a stream synchronisation: the kernel's last workgroup
// (device arrival counter) copies the OR-ed flags into mapped pinned host memory and then stores
// the call's sequence number there with system scope; the host spins on that word (checking the
// stream for errors while it waits).  The device flag words and the counter are reset by that
// same workgroup, so no memset is launched.  u is written for every env even when a flag is set
// (the caller raises and drops it, as the reference raises before it assigns u).
//
// Arithmetic: clamp = min(max(x, -r), r) and u = v * m in fp32, the element-wise torch ops.
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"

namespace {

constexpr int kMaxRefsPerLaunch = 8;  // refs travel in the kernel arguments
constexpr int kThreads = 256, kPerThread = 4;

struct ApplyArgs {
    VmasActionApplyRef r[kMaxRefsPerLaunch];
    float* out;
    uint32_t* dflags;   // [2 * kMaxRefsPerLaunch] device OR words, zero between calls
    uint32_t* counter;  // device arrival counter, zero between calls
    uint32_t* hsig;     // mapped host words: [0] sequence number, [1 + 2i], [2 + 2i] flags of ref i
    uint32_t seq;
    int B, n, total_blocks;
};

__host__ __device__ inline void apply_one(const VmasActionApplyRef& r, float* out, int b, int c,
                                          bool& nan_seen, bool& oor) {
    const float x = r.u[(long)b * r.s0 + (long)c * r.s1];
    nan_seen |= (x != x);
    if (c < r.n_phys) {
        const float rr = r.u_range[c];
        if (!r.clamp) oor |= fabsf(x) > rr;
        const float v = r.clamp ? fminf(fmaxf(x, -rr), rr) : x;
        out[r.out_offset + (long)b * r.n_phys + c] = v * r.u_mult[c];
    }
}

__global__ void __launch_bounds__(kThreads) k_apply_actions(ApplyArgs a) {
    const VmasActionApplyRef& r = a.r[blockIdx.y];
    const long n = (long)a.B * r.n_cols;
    bool nan_seen = false, oor = false;
    const long stride = (long)gridDim.x * kThreads;
    for (long idx = (long)blockIdx.x * kThreads + threadIdx.x; idx < n; idx += stride) {
        const int b = (int)(idx / r.n_cols), c = (int)(idx - (long)b * r.n_cols);
        apply_one(r, a.out, b, c, nan_seen, oor);
    }
    if (__any(nan_seen) && (threadIdx.x & 63) == 0) atomicOr(&a.dflags[2 * blockIdx.y], 1u);
    if (__any(oor) && (threadIdx.x & 63) == 0) atomicOr(&a.dflags[2 * blockIdx.y + 1], 1u);
    // last workgroup: publish the flags to the host, reset the device words
    __shared__ bool last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(a.counter, 1u) == (uint32_t)a.total_blocks - 1u;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    if ((int)threadIdx.x < 2 * a.n) {
        const uint32_t v = __hip_atomic_load(&a.dflags[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.hsig[1 + threadIdx.x], v ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        a.dflags[threadIdx.x] = 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        *a.counter = 0u;
        __threadfence_system();
        __hip_atomic_store(&a.hsig[0], a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

struct DevState {
    uint32_t* dflags = nullptr;
    uint32_t* counter = nullptr;
    uint32_t* hsig = nullptr;  // mapped, coherent pinned memory
    uint32_t seq = 0;
};
DevState g_dev[64];
std::mutex g_mu;

}  // namespace

extern "C" {

int32_t vmas_apply_actions(int32_t device, int32_t batch, const VmasActionApplyRef* refs, int32_t n_refs,
                           float* out, uint8_t* flags, void* stream) {
    if (n_refs <= 0 || batch <= 0) return VMAS_OK;
    if (!refs || !out || !flags) return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions: null argument");
    for (int i = 0; i < n_refs; ++i)
        if (!refs[i].u || !refs[i].u_range || !refs[i].u_mult || refs[i].n_phys > refs[i].n_cols ||
            refs[i].n_phys < 0 || refs[i].out_offset < 0)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions: bad ref %d", i);
    if (device < 0) {
        for (int i = 0; i < n_refs; ++i) {
            bool nan_seen = false, oor = false;
            for (int b = 0; b < batch; ++b)
                for (int c = 0; c < refs[i].n_cols; ++c) apply_one(refs[i], out, b, c, nan_seen, oor);
            flags[2 * i] = nan_seen;
            flags[2 * i + 1] = oor;
        }
        return VMAS_OK;
    }
    if (device >= 64) return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions: device %d", device);
    std::lock_guard<std::mutex> lk(g_mu);
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    DevState& d = g_dev[device];
    if (!d.dflags) {
        VMAS_AUX_HIP(hipMalloc((void**)&d.dflags, 2 * kMaxRefsPerLaunch * 4));
        VMAS_AUX_HIP(hipMalloc((void**)&d.counter, 4));
        VMAS_AUX_HIP(hipMemset(d.dflags, 0, 2 * kMaxRefsPerLaunch * 4));
        VMAS_AUX_HIP(hipMemset(d.counter, 0, 4));
        VMAS_AUX_HIP(hipHostMalloc((void**)&d.hsig, (1 + 2 * kMaxRefsPerLaunch) * 4,
                                   hipHostMallocMapped | hipHostMallocCoherent));
        d.hsig[0] = 0u;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int first = 0; first < n_refs; first += kMaxRefsPerLaunch) {
        const int n = std::min(kMaxRefsPerLaunch, n_refs - first);
        ApplyArgs a{};
        long max_elems = 0;
        for (int i = 0; i < n; ++i) {
            a.r[i] = refs[first + i];
            max_elems = std::max(max_elems, (long)batch * refs[first + i].n_cols);
        }
        const int gx = (int)std::max(1L, std::min(1024L, (max_elems + kThreads * kPerThread - 1) /
                                                               (kThreads * kPerThread)));
        a.out = out;
        a.dflags = d.dflags;
        a.counter = d.counter;
        a.hsig = d.hsig;
        a.seq = ++d.seq;
        if (a.seq == 0u) a.seq = ++d.seq;  // 0 is the "nothing published" value
        a.B = batch;
        a.n = n;
        a.total_blocks = gx * n;
        hipLaunchKernelGGL(k_apply_actions, dim3(gx, n), dim3(kThreads), 0, st, a);
        VMAS_AUX_HIP(hipGetLastError());
        if (int32_t rc = vmas_aux::wait_host_word(d.hsig, a.seq, st)) return rc;
        for (int i = 0; i < 2 * n; ++i) flags[2 * first + i] = d.hsig[1 + i] != 0u;
    }
    return VMAS_OK;
}

}  // extern "C"
