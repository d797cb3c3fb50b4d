// vmas_actions.hip -- the continuous-action side of Environment.step for every agent in one pass
// (reference vmas/simulator/environment/environment.py:615-709, _set_action, continuous actions
// without communication): NaN check (621-623), optional clamp to u_range (636-640), range check
// (651-655) and u = physical * u_multiplier (709), gfx950 kernel + host backend + C ABI.
//
// The reference runs ~5 torch ops and one host sync per agent; here one launch covers all agents
// and the host learns the flags without a stream synchronisation: every workgroup stores its
// flag bits into its own slot and arrives on a sharded device counter; the last to arrive ORs the slots
// and publishes (sequence number << 32 | flag bits) into mapped pinned host memory with ONE
// 64-bit system-scope store -- the number and the flags land together, so no system fence is
// needed -- and clears the counters.  The host spins on that word (checking the stream for errors
// while it waits).  Slots are overwritten by every call; nothing is memset per call.  u is
// written for every env even when a flag is set (the caller raises and drops it, as the
// reference raises before it assigns u).
//
// Arithmetic: clamp = min(max(x, -r), r) and u = v * m in fp32, the element-wise torch ops.
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>

#include <rocrand/rocrand_philox4x32_10.h>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"
#include "vmas_uniform.hpp"

namespace {

constexpr int kMaxRefsPerLaunch = 8;  // refs travel in the kernel arguments (16 flag bits)
// (kPerThread 2 / up to 256 workgroups per ref: 8 per thread and 64 per ref left most CUs idle
// and took 9.8 us per balance step in the kernel alone)
constexpr int kThreads = 256, kPerThread = 2, kMaxBlocksPerRef = 256;
constexpr uint32_t kShards = 32;  // arrival counter shards (+ the top counter), one line each

struct ApplyArgs {
    VmasActionApplyRef r[kMaxRefsPerLaunch];
    float* out;
    uint32_t* slots;    // [kMaxRefsPerLaunch][kMaxBlocksPerRef] flag bits of each workgroup
    uint32_t* counter;  // device arrival counter: [0] top, [32 * (1 + k)] shard k; zero between calls
    uint64_t* hsig;     // mapped host word: seq << 32 | flags (bit 2i NaN, 2i+1 out of range, ref i)
    uint32_t seq;
    int B, n, gx;
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

// Arrival of workgroup i of n on the sharded counter (one thread): shard i % kShards, each on a
// 128-byte line of its own, then the top counter for the arrival that completes its shard; true
// for the last arrival overall.  (One unsharded counter serialised the arrivals of all n
// workgroups at the memory side, ~11-13 ns each: 512 workgroups took 11 us per balance step;
// MI355X_MICROARCH.md "fanin".)
__device__ __forceinline__ bool arrive(uint32_t* counter, uint32_t i, uint32_t n) {
    const uint32_t k = i % kShards, n_k = (n + kShards - 1u - k) / kShards;
    const uint32_t n_top = n < (uint32_t)kShards ? n : (uint32_t)kShards;
    if (__hip_atomic_fetch_add(&counter[32 * (1 + k)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != n_k - 1u)
        return false;
    return __hip_atomic_fetch_add(&counter[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_top - 1u;
}

__global__ void __launch_bounds__(kThreads) k_apply_actions(ApplyArgs a) {
    const int ref = blockIdx.y;
    const VmasActionApplyRef& r = a.r[ref];
    const int n = a.B * r.n_cols;  // (< 2^31: checked by the host)
    bool nan_seen = false, oor = false;
    const int stride = (int)gridDim.x * kThreads;
    for (int idx = (int)blockIdx.x * kThreads + (int)threadIdx.x; idx < n; idx += stride) {
        const int b = idx / r.n_cols, c = idx - b * r.n_cols;
        apply_one(r, a.out, b, c, nan_seen, oor);
    }
    __shared__ uint32_t bits;
    __shared__ bool last;
    if (threadIdx.x == 0) bits = 0u;
    __syncthreads();
    const uint32_t mine = (__any(nan_seen) ? 1u : 0u) | (__any(oor) ? 2u : 0u);
    if ((threadIdx.x & 63) == 0 && mine) atomicOr(&bits, mine << (2 * ref));
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&a.slots[ref * kMaxBlocksPerRef + blockIdx.x], bits, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0);  // the slot store has completed before the arrival
        last = arrive(a.counter, (uint32_t)(ref * a.gx + (int)blockIdx.x), (uint32_t)(a.gx * a.n));
    }
    __syncthreads();
    if (!last) return;
    // the last workgroup: OR every slot, publish, clear the counter for the next call
    uint32_t f = 0u;
    for (int i = threadIdx.x; i < a.gx * a.n; i += kThreads) {
        const int rf = i / a.gx, bx = i - rf * a.gx;
        f |= __hip_atomic_load(&a.slots[rf * kMaxBlocksPerRef + bx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x == 0) bits = 0u;
    __syncthreads();
    if (f) atomicOr(&bits, f);
    __syncthreads();
    if (threadIdx.x <= kShards) __hip_atomic_store(&a.counter[32 * threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0)
        __hip_atomic_store(a.hsig, ((uint64_t)a.seq << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct DevState {
    uint32_t* slots = nullptr;
    uint32_t* counter = nullptr;
    uint64_t* hsig = nullptr;  // mapped, coherent pinned memory
    uint64_t* dsig = nullptr;  // its device address
    uint32_t seq = 0;
};
DevState g_dev[64];
std::mutex g_mu;

int32_t dev_init(DevState& d) {
    if (d.slots) return VMAS_OK;
    VMAS_AUX_HIP(hipMalloc((void**)&d.slots, kMaxRefsPerLaunch * kMaxBlocksPerRef * 4));
    VMAS_AUX_HIP(hipMalloc((void**)&d.counter, 4 * 32 * (kShards + 1)));
    VMAS_AUX_HIP(hipMemset(d.counter, 0, 4 * 32 * (kShards + 1)));
    VMAS_AUX_HIP(hipHostMalloc((void**)&d.hsig, 8, hipHostMallocMapped | hipHostMallocCoherent));
    VMAS_AUX_HIP(hipHostGetDevicePointer((void**)&d.dsig, d.hsig, 0));
    *d.hsig = 0u;
    return VMAS_OK;
}

// One launch over n <= kMaxRefsPerLaunch refs; returns the sequence number it publishes.
uint32_t launch_apply(DevState& d, int batch, const VmasActionApplyRef* refs, int n, float* out, hipStream_t st) {
    ApplyArgs a{};
    long max_elems = 0;
    for (int i = 0; i < n; ++i) {
        a.r[i] = refs[i];
        max_elems = std::max(max_elems, (long)batch * refs[i].n_cols);
    }
    const int gx = (int)std::max(1L, std::min((long)kMaxBlocksPerRef, (max_elems + kThreads * kPerThread - 1) /
                                                                           (kThreads * kPerThread)));
    a.out = out;
    a.slots = d.slots;
    a.counter = d.counter;
    a.hsig = d.dsig;
    a.seq = ++d.seq;
    if (a.seq == 0u) a.seq = ++d.seq;  // 0 is the "nothing published" value
    a.B = batch;
    a.n = n;
    a.gx = gx;
    hipLaunchKernelGGL(k_apply_actions, dim3(gx, n), dim3(kThreads), 0, st, a);
    return a.seq;
}

// Deferred assertion of one slot: AND of n condition bytes, published with the slot's next epoch.
__global__ void __launch_bounds__(256) k_assert_publish(const uint8_t* cond, int64_t n, uint32_t* epoch,
                                                        uint64_t* hsig) {
    __shared__ uint32_t bad;
    if (threadIdx.x == 0) bad = 0u;
    __syncthreads();
    bool mine = false;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) mine |= cond[i] == 0;
    // (the vote outside the lane-0 branch: a short-circuit `lane == 0 && __any(..)` would vote
    // with lane 0 alone)
    const bool wave_bad = __any(mine);
    if ((threadIdx.x & 63) == 0 && wave_bad) atomicOr(&bad, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t e = *epoch + 1u;
        if (e == 0u) e = 1u;  // 0 is the "nothing published" value
        *epoch = e;
        __hip_atomic_store(hsig, ((uint64_t)e << 32) | bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// A scripted agent's action range check (core.py:977-980: ((u / u_multiplier).abs() <= u_range)
// .all()) evaluated and published in one kernel: the element-wise test, the AND over the batch
// and the publish of k_assert_publish (instead of torch's divide / abs / compare / all-reduce
// kernels and a publish).  Workgroups OR their verdict into the slot's work line and arrive on
// its counter; the last one publishes and clears the line for the next launch.  (One 1024-thread
// workgroup over the 65 536 elements of flocking's target took 30 us.)
// (4 elements per thread, 32-bit index math where the element count fits: the grid-stride loop's
// serial chain of 64-bit divisions, not the bytes, set this kernel's ~6 us at flocking's 65 536
// elements with 8 per thread; more workgroups would add arrivals on the one counter line)
constexpr int kRangeThreads = 256, kRangePerThread = 4;
template <typename I>
__global__ void __launch_bounds__(kRangeThreads) k_assert_range(const float* u, int64_t s0, int64_t s1, int batch, int n,
                                                                const float* mult, const float* range, uint32_t* epoch,
                                                                uint64_t* hsig, uint32_t* work) {
    __shared__ uint32_t bad;
    __shared__ bool last;
    if (threadIdx.x == 0) bad = 0u;
    __syncthreads();
    bool mine = false;
    const I total = (I)batch * (I)n, step = (I)gridDim.x * kRangeThreads;
    for (I i = (I)blockIdx.x * kRangeThreads + (I)threadIdx.x; i < total; i += step) {
        const I b = i / (I)n;
        const int c = (int)(i - b * (I)n);
        const float x = u[(int64_t)b * s0 + (int64_t)c * s1];
        mine |= !(fabsf(x / mult[c]) <= range[c]);  // (NaN fails, as torch's comparison)
    }
    const bool wave_bad = __any(mine);  // (every lane takes part in the vote)
    if ((threadIdx.x & 63) == 0 && wave_bad) atomicOr(&bad, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (bad) (void)__hip_atomic_fetch_or(&work[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0);  // the verdict has landed before the arrival
        last = __hip_atomic_fetch_add(&work[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
    }
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    const uint32_t v = __hip_atomic_load(&work[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&work[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&work[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t e = *epoch + 1u;
    if (e == 0u) e = 1u;
    *epoch = e;
    __hip_atomic_store(hsig, ((uint64_t)e << 32) | (v ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- random actions: every agent's uniform_ columns in one launch ------------------------------
// The reference draws each action column with its own torch uniform_ call (environment.py:
// 524-606); on ROCm that is one philox kernel per column (PyTorch's distribution kernel: thread
// idx of a grid of min(ceil(n/256), CUs * maxThreadsPerCU/256) x 256 threads initialises
// philox4x32-10 at (seed, subsequence = idx, offset), draws 4 numbers per grid-stride round
// for elements idx + k * threads, maps them to floats in (0, 1] and to [from, to)).  Here one
// launch draws all columns (blockIdx.y = column, offset of column c = offset + c * increment), with
// rocrand's own philox engine.  The two float roundings whose contraction depends on how PyTorch
// was compiled (v * 2^-32 + 2^-32 and rand * range + from: separate or fused) are a mode; the
// host picks the mode that reproduces torch's draws bit for bit on this device (probe), or does
// not use the kernel.
constexpr int kMaxUniformCols = 32;
constexpr int kUniformThreads = vmas_uniform::kThreads;

struct UniformArgs {
    VmasUniformColumn c[kMaxUniformCols];
    unsigned long long seed;
    long long numel;
    long long snap;  // bytes from a pre-applied element to its snapshot slot (0: no snapshot)
    int mode;  // bit 0: fused (0, 1] mapping; bit 1: fused affine transform
};

__global__ void __launch_bounds__(kUniformThreads) k_uniform_columns(UniformArgs a) {
    vmas_uniform::draw_column(a.c[blockIdx.y], a.seed, a.numel, a.snap, a.mode, (int)gridDim.x, (int)blockIdx.x);
}

struct UniformGrid {
    int gx = 0;
    long long numel = -1;
};

}  // namespace

struct VmasDeviceAssert {
    int device = 0;
    int n_slots = 0;
    uint32_t* epoch = nullptr;  // [n_slots] device epochs
    uint32_t* work = nullptr;   // [n_slots][32] per-slot line: arrival counter, verdict (k_assert_range)
    uint64_t* hsig = nullptr;   // [n_slots] mapped, coherent pinned words
    uint64_t* dsig = nullptr;   // their device address
};

extern "C" {

int32_t vmas_apply_actions_launch(int32_t device, int32_t batch, const VmasActionApplyRef* refs, int32_t n_refs,
                                  float* out, uint32_t* seq, void* stream) {
    if (device < 0 || device >= 64 || n_refs <= 0 || n_refs > kMaxRefsPerLaunch || batch <= 0 || !refs || !out || !seq)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions_launch: bad arguments");
    for (int i = 0; i < n_refs; ++i)
        if (!refs[i].u || !refs[i].u_range || !refs[i].u_mult || refs[i].n_phys > refs[i].n_cols ||
            refs[i].n_phys < 0 || refs[i].out_offset < 0 || (long)batch * refs[i].n_cols > INT32_MAX)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions_launch: bad ref %d", i);
    std::lock_guard<std::mutex> lk(g_mu);
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    DevState& d = g_dev[device];
    if (int32_t rc = dev_init(d)) return rc;
    *seq = launch_apply(d, batch, refs, n_refs, out, (hipStream_t)stream);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_apply_actions_flags(int32_t device, uint32_t seq, int32_t n_refs, uint8_t* flags, void* stream) {
    if (device < 0 || device >= 64 || n_refs <= 0 || n_refs > kMaxRefsPerLaunch || !flags || seq == 0u)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions_flags: bad arguments");
    DevState& d = g_dev[device];
    if (!d.hsig) return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions_flags: nothing launched");
    uint64_t v = 0;
    if (int32_t rc = vmas_aux::wait_host_word64(d.hsig, seq, &v, (hipStream_t)stream)) return rc;
    for (int i = 0; i < n_refs; ++i) {
        flags[2 * i] = (v >> (2 * i)) & 1u;
        flags[2 * i + 1] = (v >> (2 * i + 1)) & 1u;
    }
    return VMAS_OK;
}

int32_t vmas_apply_actions(int32_t device, int32_t batch, const VmasActionApplyRef* refs, int32_t n_refs,
                           float* out, uint8_t* flags, void* stream) {
    if (n_refs <= 0 || batch <= 0) return VMAS_OK;
    if (!refs || !out || !flags) return vmas_aux::fail(VMAS_E_INVALID, "vmas_apply_actions: null argument");
    for (int i = 0; i < n_refs; ++i)
        if (!refs[i].u || !refs[i].u_range || !refs[i].u_mult || refs[i].n_phys > refs[i].n_cols ||
            refs[i].n_phys < 0 || refs[i].out_offset < 0 || (long)batch * refs[i].n_cols > INT32_MAX)
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
    if (int32_t rc = dev_init(d)) return rc;
    hipStream_t st = (hipStream_t)stream;
    for (int first = 0; first < n_refs; first += kMaxRefsPerLaunch) {
        const int n = std::min(kMaxRefsPerLaunch, n_refs - first);
        const uint32_t seq = launch_apply(d, batch, refs + first, n, out, st);
        VMAS_AUX_HIP(hipGetLastError());
        uint64_t v = 0;
        if (int32_t rc = vmas_aux::wait_host_word64(d.hsig, seq, &v, st)) return rc;
        for (int i = 0; i < n; ++i) {
            flags[2 * (first + i)] = (v >> (2 * i)) & 1u;
            flags[2 * (first + i) + 1] = (v >> (2 * i + 1)) & 1u;
        }
    }
    return VMAS_OK;
}

int32_t vmas_uniform_columns(int32_t device, int64_t numel, const VmasUniformColumn* cols, int32_t n_cols,
                             uint64_t seed, uint64_t offset, int32_t mode, uint64_t* increment, void* stream) {
    return vmas_uniform_columns_snap(device, numel, cols, n_cols, seed, offset, mode, 0, increment, stream);
}

int32_t vmas_uniform_columns_snap(int32_t device, int64_t numel, const VmasUniformColumn* cols, int32_t n_cols,
                                  uint64_t seed, uint64_t offset, int32_t mode, int64_t u_snap_delta,
                                  uint64_t* increment, void* stream) {
    if (device < 0 || device >= 64 || numel <= 0 || n_cols <= 0 || n_cols > kMaxUniformCols || !cols ||
        !increment || mode < 0 || mode > 3)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_uniform_columns: bad arguments");
    static int max_blocks[64] = {0};
    if (!max_blocks[device]) {
        hipDeviceProp_t prop;
        VMAS_AUX_HIP(hipGetDeviceProperties(&prop, device));
        max_blocks[device] = prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / kUniformThreads);
        if (max_blocks[device] <= 0) return vmas_aux::fail(VMAS_E_HIP, "vmas_uniform_columns: device properties");
    }
    const long long gx = std::min<long long>((numel + kUniformThreads - 1) / kUniformThreads, max_blocks[device]);
    // PyTorch's per-call philox increment (counter_offset, rounded up to a multiple of 4)
    const unsigned long long inc = (unsigned long long)((numel - 1) / (kUniformThreads * gx * 4) + 1) * 4;
    UniformArgs a{};
    for (int i = 0; i < n_cols; ++i) {
        if (!cols[i].out) return vmas_aux::fail(VMAS_E_INVALID, "vmas_uniform_columns: null column %d", i);
        a.c[i] = cols[i];
        a.c[i].offset = offset + inc * (unsigned long long)i;
    }
    a.seed = seed;
    a.numel = numel;
    a.snap = u_snap_delta;
    a.mode = mode;
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    hipLaunchKernelGGL(k_uniform_columns, dim3((unsigned)gx, n_cols), dim3(kUniformThreads), 0, (hipStream_t)stream, a);
    VMAS_AUX_HIP(hipGetLastError());
    *increment = inc * (unsigned long long)n_cols;
    return VMAS_OK;
}

int32_t vmas_assert_create(int32_t device, int32_t n_slots, VmasDeviceAssert** out) {
    if (!out || n_slots <= 0 || n_slots > 4096 || device < 0)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_assert_create: bad arguments");
    *out = nullptr;
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    VmasDeviceAssert* ch = new VmasDeviceAssert();
    ch->device = device;
    ch->n_slots = n_slots;
    hipError_t e = hipMalloc((void**)&ch->epoch, 4 * (size_t)n_slots);
    if (e == hipSuccess) e = hipMemset(ch->epoch, 0, 4 * (size_t)n_slots);
    if (e == hipSuccess) e = hipMalloc((void**)&ch->work, 128 * (size_t)n_slots);
    if (e == hipSuccess) e = hipMemset(ch->work, 0, 128 * (size_t)n_slots);
    if (e == hipSuccess) e = hipHostMalloc((void**)&ch->hsig, 8 * (size_t)n_slots, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&ch->dsig, ch->hsig, 0);
    if (e == hipSuccess) e = hipDeviceSynchronize();  // the epoch memset has landed before any capture
    if (cur != device) (void)hipSetDevice(cur);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        vmas_assert_destroy(ch);
        return vmas_aux::fail(VMAS_E_HIP, "vmas_assert_create: %s", hipGetErrorString(e));
    }
    for (int i = 0; i < n_slots; ++i) ch->hsig[i] = 0u;
    *out = ch;
    return VMAS_OK;
}

int32_t vmas_assert_destroy(VmasDeviceAssert* ch) {
    if (!ch) return VMAS_OK;
    if (ch->epoch) (void)hipFree(ch->epoch);
    if (ch->work) (void)hipFree(ch->work);
    if (ch->hsig) (void)hipHostFree(ch->hsig);
    delete ch;
    return VMAS_OK;
}

int32_t vmas_assert_publish(VmasDeviceAssert* ch, int32_t slot, const uint8_t* cond, int64_t n, void* stream) {
    if (!ch || !cond || slot < 0 || slot >= ch->n_slots || n <= 0)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_assert_publish: bad arguments");
    hipLaunchKernelGGL(k_assert_publish, dim3(1), dim3(256), 0, (hipStream_t)stream, cond, n, ch->epoch + slot,
                       ch->dsig + slot);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_assert_publish_range(VmasDeviceAssert* ch, int32_t slot, const float* u, int64_t s0, int64_t s1,
                                  int32_t batch, int32_t n, const float* mult, const float* range, void* stream) {
    if (!ch || !u || !mult || !range || slot < 0 || slot >= ch->n_slots || batch <= 0 || n <= 0)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_assert_publish_range: bad arguments");
    const int64_t total = (int64_t)batch * n;
    const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (total + kRangeThreads * kRangePerThread - 1) /
                                                                          (kRangeThreads * kRangePerThread)));
    if (total + (int64_t)gx * kRangeThreads < ((int64_t)1 << 31))
        hipLaunchKernelGGL(k_assert_range<int32_t>, dim3(gx), dim3(kRangeThreads), 0, (hipStream_t)stream, u, s0, s1, batch,
                           n, mult, range, ch->epoch + slot, ch->dsig + slot, ch->work + 32 * slot);
    else
        hipLaunchKernelGGL(k_assert_range<int64_t>, dim3(gx), dim3(kRangeThreads), 0, (hipStream_t)stream, u, s0, s1, batch,
                           n, mult, range, ch->epoch + slot, ch->dsig + slot, ch->work + 32 * slot);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_assert_wait(VmasDeviceAssert* ch, int32_t slot, uint32_t seq, int32_t* violated, void* stream) {
    if (!ch || !violated || slot < 0 || slot >= ch->n_slots || seq == 0u)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_assert_wait: bad arguments");
    uint64_t v = 0;
    if (int32_t rc = vmas_aux::wait_host_word64(ch->hsig + slot, seq, &v, (hipStream_t)stream)) return rc;
    *violated = (int32_t)(v & 1u);
    return VMAS_OK;
}

// Test utility: occupy CUs for `ticks` s_memrealtime ticks.  Every workgroup holds 144 KiB of
// the CU's 160 KiB LDS, so at most one fits per CU and no step workgroup (whose LDS is larger
// than the 16 KiB left) fits beside it: `blocks` CUs are closed to other kernels for the span.
// Every wave polls the wall clock and leaves once the span has passed (or after a poll bound),
// so the grid always drains.
__global__ void __launch_bounds__(256) k_hold(unsigned long long ticks, int* sink) {
    __shared__ int hog[144 * 1024 / 4];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    hog[threadIdx.x] = (int)threadIdx.x;
    for (uint32_t i = 0; i < (1u << 28); ++i) {
        if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
        __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
    if (sink && hog[(threadIdx.x * 7u) & 255u] < 0) sink[0] = 1;  // (never true: keeps the LDS)
}

int32_t vmas_test_hold(int32_t device, int32_t blocks, int64_t microseconds, void* stream) {
    if (device < 0 || blocks <= 0 || microseconds <= 0 || microseconds > 5000000)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_test_hold: bad arguments");
    VMAS_AUX_HIP(hipSetDevice(device));
    int khz = 0;
    VMAS_AUX_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
    const unsigned long long ticks = (unsigned long long)microseconds * (unsigned long long)(khz > 0 ? khz : 100000) / 1000ull;
    hipLaunchKernelGGL(k_hold, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ticks, (int*)nullptr);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

}  // extern "C"
