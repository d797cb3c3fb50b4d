// vmas_spawn.hip -- rejection-sampling resolver for ScenarioUtils.find_random_pos_for_entity
// (reference vmas/simulator/utils.py:272-319), gfx950 kernel + host backend + C ABI.
//
// The reference loop draws a full [B,1,2] proposal per try (x then y, torch uniform_), checks
// every env's current position against the occupied positions with torch.cdist, replaces the
// overlapping envs' positions with the new proposal, and stops at the first try where no env
// overlaps -- one host sync and ~10 kernels per try.  Per env, the accepted position is therefore
// the FIRST candidate that overlaps nothing (a non-overlapping position never changes again), and
// the number of tries the loop consumes is 1 if every env accepts candidate 0, else
// max_env(first accepted index) + 2.  The host side draws the candidates with the same torch
// calls (so the random numbers are the reference's), this kernel resolves a whole batch of tries
// at once, and the host rewinds the generator to exactly the reference's consumption.
//
// Distance: torch.cdist (p = 2) computes sqrt(fl(fl(d0^2) + fl(d1^2))) with d = a - b on both the
// CUDA/HIP kernel (per-dim squares, then a shuffle-reduction add) and the CPU kernel; the
// comparison `dist < min_dist` runs in fp32.  Compiled with -ffp-contract=off like the engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"

namespace vmas_aux {

namespace {
thread_local std::string g_aux_err;
}

int32_t fail(int32_t code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_aux_err = buf;
    return code;
}

const char* last_error() { return g_aux_err.c_str(); }

std::atomic<uint32_t> g_host_waits{0};
void note_host_wait() { g_host_waits.fetch_add(1u, std::memory_order_relaxed); }

int32_t wait_host_word(const uint32_t* word, uint32_t seq, hipStream_t stream) {
    note_host_wait();
    for (uint64_t i = 1;; ++i) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return VMAS_OK;
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {  // the stream drained: the store must be visible by now
                if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return VMAS_OK;
                return fail(VMAS_E_HIP, "kernel finished without publishing its result word");
            }
            if (q != hipErrorNotReady) return fail(VMAS_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

int32_t wait_host_word64(const uint64_t* word, uint32_t seq, uint64_t* value, hipStream_t stream) {
    note_host_wait();
    for (uint64_t i = 1;; ++i) {
        uint64_t v = __atomic_load_n(word, __ATOMIC_ACQUIRE);
        if ((uint32_t)(v >> 32) == seq) {
            *value = v;
            return VMAS_OK;
        }
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {
                v = __atomic_load_n(word, __ATOMIC_ACQUIRE);
                if ((uint32_t)(v >> 32) == seq) {
                    *value = v;
                    return VMAS_OK;
                }
                return fail(VMAS_E_HIP, "kernel finished without publishing its result word");
            }
            if (q != hipErrorNotReady) return fail(VMAS_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

}  // namespace vmas_aux

namespace {

std::mutex g_aux_mu;

struct SpawnArgs {
    int B, n_occ, occ_s0, occ_s1, occ_s2;
    const float* occ;
    const float* cand;  // [n_tries][2][B]: candidate k of env b = (cand[k*2B + b], cand[k*2B + B + b])
    int first_try, n_tries;
    float min_dist;
    float* pos;         // [B][2]
    int32_t* resolved;  // [B], -1 = not yet
};

__host__ __device__ inline bool overlaps(const SpawnArgs& a, int b, float x, float y) {
    bool hit = false;
    for (int j = 0; j < a.n_occ; ++j) {
        const float* o = a.occ + (long)b * a.occ_s0 + (long)j * a.occ_s1;
        const float d0 = o[0] - x, d1 = o[a.occ_s2] - y;
        const float dist = sqrtf(d0 * d0 + d1 * d1);
        hit = hit || (dist < a.min_dist);
    }
    return hit;
}

// resolve env b over this batch's candidates; returns its accepted index or -1
__host__ __device__ inline int resolve_env(const SpawnArgs& a, int b) {
    int r = a.resolved[b];
    if (r >= 0) return r;
    for (int k = 0; k < a.n_tries; ++k) {
        const float x = a.cand[(long)k * 2 * a.B + b], y = a.cand[(long)k * 2 * a.B + a.B + b];
        if (!overlaps(a, b, x, y)) {
            a.pos[2 * (long)b] = x;
            a.pos[2 * (long)b + 1] = y;
            a.resolved[b] = a.first_try + k;
            return a.first_try + k;
        }
    }
    return -1;
}

// out[0] = max accepted index over envs, out[1] = number of unresolved envs
__global__ void __launch_bounds__(256) k_spawn_resolve(SpawnArgs a, int32_t* out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int r = 0, unresolved = 0;
    if (b < a.B) {
        r = resolve_env(a, b);
        unresolved = r < 0;
    }
    // wave-level max / count, then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        r = max(r, __shfl_xor(r, off));
        unresolved += __shfl_xor(unresolved, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], r);
        if (unresolved) atomicAdd(&out[1], unresolved);
    }
}

// ---- the respawn loop of several entities, tries drawn on the device (vmas_spawn_targets) --------
constexpr int kUniformThreads = 256;  // PyTorch's distribution kernel block (vmas_actions.hip)

struct DrawGrid {
    long long step;  // threads of torch's uniform_ grid on B elements
    unsigned long long inc;
};

// rocrand's philox4x32-10 block function (rocrand_philox4x32_10.h ten_rounds / single_round).
__device__ __forceinline__ uint4 philox10(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const unsigned int hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const unsigned int hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

// Element b of torch's uniform_(lo, hi) on B floats at generator offset `off`: PyTorch's
// distribution kernel (k_uniform_columns of vmas_actions.hip, probed bit for bit against torch;
// `mode` bit 0 fused (0, 1] mapping, bit 1 fused affine transform) has thread t = b % step draw
// rocrand4 round q / 4 and take component q % 4, q = b / step, from a philox state initialised
// at (seed, subsequence t, offset off).  That state is counter (off / 4 + round, t) under key
// seed, its 4 outputs shifted by off % 4 into the next block (rocrand's interleave); computed
// here directly, one block function per draw.
__device__ __forceinline__ float uniform_at(unsigned long long seed, unsigned long long off, const DrawGrid& g, int b,
                                            float lo, float hi, int mode) {
    const int step = (int)g.step, t = b % step, q = b / step;
    const unsigned long long c = off / 4 + (unsigned long long)(q / 4);
    const uint2 key = make_uint2((unsigned int)seed, (unsigned int)(seed >> 32));
    const uint4 cur = philox10(make_uint4((unsigned int)c, (unsigned int)(c >> 32), (unsigned int)t, 0u), key);
    const int sub = (int)(off & 3ull), k = sub + q % 4;
    unsigned int u;
    if (k < 4) {
        u = k == 0 ? cur.x : k == 1 ? cur.y : k == 2 ? cur.z : cur.w;
    } else {
        const uint4 nxt = philox10(make_uint4((unsigned int)(c + 1), (unsigned int)((c + 1) >> 32), (unsigned int)t, 0u), key);
        u = k == 4 ? nxt.x : k == 5 ? nxt.y : nxt.z;
    }
    const float inv = 2.3283064e-10f;  // ROCRAND_2POW32_INV
    const float unit = (mode & 1) ? __builtin_fmaf((float)u, inv, inv) : inv + (float)u * inv;
    const float range = hi - lo;
    const float val = (mode & 2) ? __builtin_fmaf(unit, range, lo) : unit * range + lo;
    return val == hi ? lo : val;  // (0, 1] -> [lo, hi)
}

// torch.cdist(...) < min_dist with cdist = sqrt(fl(fl(d0^2) + fl(d1^2))): sqrtf is correctly
// rounded and monotone, so the test is d2 < d2_min, d2_min = the smallest float whose sqrtf
// reaches min_dist (computed on the host, spawn_d2_min) -- the same outcome without the sqrt.
__device__ __forceinline__ bool near(float ox, float oy, float x, float y, float d2_min) {
    const float d0 = ox - x, d1 = oy - y;
    return d0 * d0 + d1 * d1 < d2_min;
}

// The respawn loop of every target in ONE launch.  Work item (i, g) = target i for the 64 envs of
// group g: a workgroup of kSpawnWaves waves, wave w tries k = w, w + kSpawnWaves, ... for its lane's
// env and stops at the first accepted try or once another wave has accepted an earlier one (the
// per-lane minimum in LDS): the first accepted try of each env, as the reference's loop keeps it,
// with a kSpawnWaves times shorter serial chain.  The occupied positions are staged in LDS.
//
// Target i's generator offset follows from the earlier targets' max accepted tries over ALL envs,
// and its occupied set holds the earlier targets' new positions: item (i, g) starts once every
// item of target i - 1 is done.  Workgroups claim items in order from a counter and wait for the
// previous target's done count -- every item they wait for was claimed earlier by a running
// workgroup, so the launch needs no co-residency (the k_world claim pattern); the wait is bounded
// (kSpawnWaitTicks, then the error word and every workgroup leaves).  Before: a launch per target,
// 7 x 14.7 us at 16 384 envs.
//
// The grid is at most one workgroup per env group, so at most that many workgroups poll one done
// counter; each counter has a 128-byte line of its own (polls are sc1 loads served beyond the
// L2: on a shared line they delay the claims and the maxima -- 29 us per target when every
// word sat on one line and 1024 workgroups polled it).
//
// max_accepted words: [0, T) per-target max accepted try, [T] unresolved envs, [32] the claim
// counter, [64] error (1: a wait timed out), [96 + 32 i] target i's done items.
constexpr int kSpawnWaves = 8;
constexpr int kSpawnMaxOcc = 32 + VMAS_SPAWN_MAX_TARGETS - 1;  // agents + the other targets
constexpr unsigned long long kSpawnWaitTicks = 100000000ull;   // s_memrealtime (100 MHz): 1 s

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64 * kSpawnWaves) k_spawn_targets(VmasSpawnTargetsIO io, DrawGrid g, float d2_min,
                                                                  int n_groups) {
    __shared__ int best[64];
    __shared__ int item_s;
    __shared__ unsigned long long off_s;
    __shared__ float2 occ[kSpawnMaxOcc][64];  // the occupied positions of the item's 64 envs
    __shared__ float2 won[kSpawnWaves][64];   // each wave's accepted position (at most one per lane)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int T = io.n_targets, n_items = T * n_groups;
    int32_t* const W = io.max_accepted;
    int32_t* const claim = W + 32;
    int32_t* const err = W + 64;
    int32_t* const done = W + 96;  // target i's counter at done[32 * i]
    const unsigned long long per_try = 2ull * g.inc;
    const int n_occ = io.n_agents + T - 1;
    // (thread 0) the claim of the coming item, taken one item ahead so that the claim's round trip
    // overlaps the current item; still deadlock-free: the smallest unfinished item is always some
    // workgroup's current one, and it waits only for smaller items
    int next = threadIdx.x == 0 ? atomicAdd(claim, 1) : 0;
    for (;;) {
        if (threadIdx.x == 0) {
            int it = next;
            if (it < n_items) next = atomicAdd(claim, 1);
            if (it < n_items && it >= n_groups) {  // wait for every item of the previous target
                const int* dp = done + 32 * (it / n_groups - 1);
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (ld_agent(dp) < n_groups) {
                    if (ld_agent(err) || __builtin_amdgcn_s_memrealtime() - t0 > kSpawnWaitTicks) {
                        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        it = n_items;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            item_s = it;
            if (it < n_items) {  // target i's generator offset, from the earlier targets' maxima
                const int i = it / n_groups;
                int mv[VMAS_SPAWN_MAX_TARGETS];
#pragma unroll
                for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j) mv[j] = j < i ? ld_agent(W + j) : 0;  // (one round trip)
                unsigned long long off = io.offset;
#pragma unroll
                for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j)
                    if (j < i) off += (unsigned long long)(mv[j] == 0 ? 1 : mv[j] + 2) * per_try;
                off_s = off;
            }
        }
        __syncthreads();
        const int it = item_s;
        if (it >= n_items) return;
        const int i = it / n_groups, grp = it - i * n_groups;
        const int b = grp * 64 + lane;
        const bool valid = b < io.batch;
        const int bb = valid ? b : io.batch - 1;
        const bool cov = wave == 0 && valid && io.covered[(long)b * io.cov_s0 + (long)i * io.cov_s1];
        if (wave == 0) best[lane] = VMAS_SPAWN_MAX_TRIES;
        const unsigned long long off = off_s;
        // occupied: the agents, then every other target (earlier ones already moved, by items that
        // may have run on another XCD: loaded with agent-scope atomics, sc1, as they were stored)
        for (int m = wave; m < n_occ; m += kSpawnWaves) {
            if (m < io.n_agents) {
                const float* p = io.agents + (long)bb * io.ag_s0 + (long)m * io.ag_s1;
                occ[m][lane] = make_float2(p[0], p[io.ag_s2]);
            } else {
                const int j = m - io.n_agents + (m - io.n_agents >= i ? 1 : 0);
                const float* p = io.pos[j] + (long)bb * io.pos_s0[j];
                occ[m][lane] = make_float2(ld_agent(p), ld_agent(p + io.pos_s1[j]));
            }
        }
        __syncthreads();
        if (valid) {
            for (int k = wave; k < VMAS_SPAWN_MAX_TRIES; k += kSpawnWaves) {
                if (k >= __hip_atomic_load(&best[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                const unsigned long long o = off + (unsigned long long)k * per_try;
                const float x = uniform_at(io.seed, o, g, b, io.x_lo, io.x_hi, io.mode);
                const float y = uniform_at(io.seed, o + g.inc, g, b, io.y_lo, io.y_hi, io.mode);
                bool hit = false;
                for (int m = 0; m < n_occ; ++m) {
                    const float2 o2 = occ[m][lane];
                    hit = hit || near(o2.x, o2.y, x, y, d2_min);
                }
                if (!hit) {
                    won[wave][lane] = make_float2(x, y);
                    atomicMin(&best[lane], k);
                    break;
                }
            }
        }
        __syncthreads();
        if (wave == 0) {
            const int k = valid ? best[lane] : 0;
            const bool unresolved = valid && k == VMAS_SPAWN_MAX_TRIES;
            if (unresolved) atomicAdd(&W[T], 1);
            int km = unresolved ? 0 : k;  // one atomic per wave
            for (int s = 32; s > 0; s >>= 1) km = max(km, __shfl_xor(km, s));
            if (lane == 0 && km > 0) atomicMax(&W[i], km);
            if (cov && !unresolved) {  // try k was drawn and accepted by wave k % kSpawnWaves
                const float2 xy = won[k % kSpawnWaves][lane];
                float* p = io.pos[i] + (long)b * io.pos_s0[i];
                __hip_atomic_store(p, xy.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(p + io.pos_s1[i], xy.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the positions and the maxima have landed before the completion (the sc1 hand-off of
            // vmas_jit_ops.hpp: no agent fence, 1.7-6.5 us each)
            __builtin_amdgcn_s_waitcnt(0);
            if (lane == 0) atomicAdd(&done[32 * i], 1);
        }
        // (item_s is rewritten only after every wave has passed the barrier above)
    }
}

// The smallest float x >= 0 with sqrtf(x) >= min_dist (binary search over the ordered bit patterns
// of non-negative floats; sqrtf is correctly rounded on the host as on the device).
float spawn_d2_min(float min_dist) {
    if (!(min_dist > 0.f)) return 0.f;  // sqrt(d2) < min_dist never holds: neither does d2 < 0
    uint32_t lo = 0u, hi = 0x7f800000u;  // sqrtf(+inf) = inf >= min_dist
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        float x;
        memcpy(&x, &mid, 4);
        if (sqrtf(x) >= min_dist) hi = mid;
        else lo = mid + 1u;
    }
    float r;
    memcpy(&r, &lo, 4);
    return r;
}

struct DevScratch {
    int32_t* d_out = nullptr;
    int32_t* h_out = nullptr;
};
DevScratch g_scratch[64];

}  // namespace

extern "C" {

const char* vmas_aux_last_error(void) { return vmas_aux::last_error(); }

int32_t vmas_host_waits(void) { return (int32_t)vmas_aux::g_host_waits.load(std::memory_order_relaxed); }

int32_t vmas_spawn_resolve(int32_t device, int32_t batch, const float* occupied, int32_t n_occ,
                           int32_t occ_s0, int32_t occ_s1, int32_t occ_s2, const float* candidates,
                           int32_t first_try, int32_t n_tries, float min_dist, float* pos,
                           int32_t* resolved, int32_t* max_accepted, int32_t* n_unresolved,
                           void* stream) {
    std::lock_guard<std::mutex> lk(g_aux_mu);
    if (batch <= 0 || n_occ < 0 || n_tries <= 0 || first_try < 0 || !candidates || !pos || !resolved ||
        !max_accepted || !n_unresolved || (n_occ > 0 && !occupied))
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_resolve: bad argument");
    SpawnArgs a{batch, n_occ, occ_s0, occ_s1, occ_s2, occupied, candidates, first_try, n_tries, min_dist,
                pos, resolved};
    if (device < 0) {
        int mx = 0, un = 0;
        for (int b = 0; b < batch; ++b) {
            const int r = resolve_env(a, b);
            if (r < 0) ++un;
            else mx = r > mx ? r : mx;
        }
        *max_accepted = mx;
        *n_unresolved = un;
        return VMAS_OK;
    }
    if (device >= 64) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_resolve: device %d", device);
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    DevScratch& s = g_scratch[device];
    if (!s.d_out) {
        VMAS_AUX_HIP(hipMalloc((void**)&s.d_out, 2 * sizeof(int32_t)));
        VMAS_AUX_HIP(hipHostMalloc((void**)&s.h_out, 2 * sizeof(int32_t), hipHostMallocDefault));
    }
    hipStream_t st = (hipStream_t)stream;
    VMAS_AUX_HIP(hipMemsetAsync(s.d_out, 0, 2 * sizeof(int32_t), st));
    hipLaunchKernelGGL(k_spawn_resolve, dim3((batch + 255) / 256), dim3(256), 0, st, a, s.d_out);
    VMAS_AUX_HIP(hipGetLastError());
    VMAS_AUX_HIP(hipMemcpyAsync(s.h_out, s.d_out, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    vmas_aux::note_host_wait();
    VMAS_AUX_HIP(hipStreamSynchronize(st));
    *max_accepted = s.h_out[0];
    *n_unresolved = s.h_out[1];
    return VMAS_OK;
}

int32_t vmas_spawn_targets(int32_t device, const VmasSpawnTargetsIO* io, uint64_t* increment, void* stream) {
    if (!io || !increment || device < 0 || device >= 64 || io->batch <= 0 || io->n_agents < 0 || io->n_agents > 32 ||
        io->n_targets < 1 || io->n_targets > VMAS_SPAWN_MAX_TARGETS || !io->covered || !io->max_accepted ||
        (io->n_agents > 0 && !io->agents) || io->mode < 0 || io->mode > 3)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_targets: bad arguments");
    for (int i = 0; i < io->n_targets; ++i)
        if (!io->pos[i]) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_targets: null target %d", i);
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    static int max_blocks[64] = {0}, resident[64] = {0};
    if (!max_blocks[device]) {
        hipDeviceProp_t prop;
        VMAS_AUX_HIP(hipGetDeviceProperties(&prop, device));
        max_blocks[device] = prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / kUniformThreads);
        if (max_blocks[device] <= 0) return vmas_aux::fail(VMAS_E_HIP, "vmas_spawn_targets: device properties");
        int per_cu = 0;
        VMAS_AUX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spawn_targets, 64 * kSpawnWaves, 0));
        resident[device] = prop.multiProcessorCount * std::max(per_cu, 1);
    }
    // torch's distribution-kernel grid and per-call philox increment on B elements (as
    // vmas_uniform_columns)
    const long long B = io->batch;
    const long long gx = std::min<long long>((B + kUniformThreads - 1) / kUniformThreads, max_blocks[device]);
    DrawGrid g{kUniformThreads * gx, (unsigned long long)((B - 1) / (kUniformThreads * gx * 4) + 1) * 4};
    const float d2_min = spawn_d2_min(io->min_dist);
    hipStream_t st = (hipStream_t)stream;
    const int T = io->n_targets, n_groups = (int)((B + 63) / 64);
    VMAS_AUX_HIP(hipMemsetAsync(io->max_accepted, 0, sizeof(int32_t) * VMAS_SPAWN_WORDS(T), st));
    const long long grid = std::min<long long>(n_groups, resident[device]);
    hipLaunchKernelGGL(k_spawn_targets, dim3((unsigned)grid), dim3(64 * kSpawnWaves), 0, st, *io, g, d2_min, n_groups);
    VMAS_AUX_HIP(hipGetLastError());
    *increment = g.inc;
    return VMAS_OK;
}

}  // extern "C"
