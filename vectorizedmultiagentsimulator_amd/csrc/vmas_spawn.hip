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
        // (the 64-bit products: one v_mad_u64_u32 each instead of v_mul_hi_u32 + v_mul_lo_u32, both
        // quarter rate)
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
// counter, [40, 46) a channel's (seed, offset, seq) staged by k_spawn_clear, [64] error (1: a wait
// timed out), [96 + 32 i] target i's done items, then
// (k_spawn_targets_resident) kSpawnReplicas 64-bit words 128 bytes apart.
constexpr int kSpawnWaves = 16;
constexpr int kSpawnMaxOcc = 32 + VMAS_SPAWN_MAX_TARGETS - 1;  // agents + the other targets
constexpr int kSpawnReplicas = 32;  // (k_spawn_targets_resident) the published tries, one line each
constexpr unsigned long long kSpawnWaitTicks = 100000000ull;   // s_memrealtime (100 MHz): 1 s

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Spawn channel (vmas_spawn_channel_*): mapped pinned host words.  in: [0] seed, [1] offset, [2] seq.
// out: int32 [0, 16) maxima, [16] unresolved, [17] error; u64 word 12 (byte 96): seq << 32 | 1,
// stored last.
constexpr int kChanOutSeqWord = 12;
struct ChanArgs {
    const uint64_t* in;  // (device pointer of the mapped host words; null: no channel)
    uint64_t* out;
};

// With a channel, k_spawn_clear copies its (seed, offset, seq) into the launch's words at this
// int32 index (free words of the claim counter's line) and the spawn kernel's workgroups read them
// there: 256 workgroups each reading the mapped host words over PCIe took up to 54 us to all start
// (the reads serialise), one copy by one thread takes one round trip.
constexpr int kRngWord = VMAS_SPAWN_RNG_WORD;

// Generator state of a launch: the channel's (staged by k_spawn_clear) or the arguments'.
__device__ __forceinline__ void launch_rng(const VmasSpawnTargetsIO& io, const ChanArgs& ch, unsigned long long* seed,
                                           unsigned long long* off, unsigned long long* seq) {
    if (ch.in) {
        const unsigned long long* r = reinterpret_cast<const unsigned long long*>(io.max_accepted + kRngWord);
        *seed = r[0];
        *off = r[1];
        *seq = r[2];
    } else {
        *seed = io.seed;
        *off = io.offset;
        *seq = 0;
    }
}

// (the last workgroup done with the last target, one wave) the launch's words to the channel: every
// maximum and unresolved count has landed (each workgroup's before its completion).  Also the
// generator offset after the call (the launch's offset + the tries the reference loop consumes) into
// the launch's words at kOffEndWord, for a draw made ahead on the device (vmas_copy_spans_draw's
// offset_dev; meaningless when the call is unresolved -- the host then draws anew).
constexpr int kOffEndWord = VMAS_SPAWN_OFF_END_WORD;  // (int32 index; a u64, 8-byte aligned)
__device__ __forceinline__ void publish_channel(const ChanArgs& ch, int32_t* W, int T, unsigned long long seq,
                                                unsigned long long off0, unsigned long long per_try) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        unsigned long long tries = 0;
        for (int j = 0; j < T; ++j) {
            const int m = ld_agent(W + j);
            tries += m == 0 ? 1ull : (unsigned long long)m + 2ull;
        }
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(W + kOffEndWord), off0 + tries * per_try,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int32_t* o = reinterpret_cast<int32_t*>(ch.out);
    if (lane < T) __hip_atomic_store(o + lane, ld_agent(W + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 16) __hip_atomic_store(o + 16, ld_agent(W + T), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 17) __hip_atomic_store(o + 17, ld_agent(W + 64), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0)
        __hip_atomic_store(ch.out + kChanOutSeqWord, (seq << 32) | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64 * kSpawnWaves) k_spawn_targets(VmasSpawnTargetsIO io, DrawGrid g, float d2_min,
                                                                  int n_groups, unsigned long long* prof,
                                                                  ChanArgs ch) {
    __shared__ int best[64];
    __shared__ int item_s;
    __shared__ int abort_s;
    __shared__ unsigned long long off_s, t_claim_s, rng_s[3];
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
    const int MT = io.max_tries > 0 ? io.max_tries : VMAS_SPAWN_MAX_TRIES;
    if (threadIdx.x == 0) launch_rng(io, ch, &rng_s[0], &rng_s[1], &rng_s[2]);  // (read before the first barrier)
    // (Claiming one item ahead, to overlap the claim's round trip, made it slower: a workgroup
    // could hold two items of one target, serialising them -- 137 -> 218 us per call.)
    for (;;) {
        if (threadIdx.x == 0) {
            item_s = atomicAdd(claim, 1);
            if (prof) t_claim_s = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();
        const int it = item_s;
        if (it >= n_items) return;
        const int i = it / n_groups, grp = it - i * n_groups;
        const int b = grp * 64 + lane;
        const bool valid = b < io.batch;
        const int bb = valid ? b : io.batch - 1;
        // what does not depend on the earlier targets, loaded before the wait: the covered flag and
        // the agents' positions
        const bool cov = wave == 0 && valid && io.covered[(long)b * io.cov_s0 + (long)i * io.cov_s1];
        for (int m = wave; m < io.n_agents; m += kSpawnWaves) {
            const float* p = io.agents + (long)bb * io.ag_s0 + (long)m * io.ag_s1;
            occ[m][lane] = make_float2(p[0], p[io.ag_s2]);
        }
        if (threadIdx.x == 0) {
            bool ok = true;
            if (it >= n_groups) {  // wait for every item of the previous target
                const int* dp = done + 32 * (i - 1);
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (ld_agent(dp) < n_groups) {
                    if (ld_agent(err) || __builtin_amdgcn_s_memrealtime() - t0 > kSpawnWaitTicks) {
                        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            abort_s = ok ? 0 : 1;
            if (prof) {
                prof[(long)it * 6 + 0] = t_claim_s;
                prof[(long)it * 6 + 1] = __builtin_amdgcn_s_memrealtime();
                prof[(long)it * 6 + 5] = blockIdx.x;
            }
        }
        __syncthreads();
        if (abort_s) return;
        if (threadIdx.x == 0) {  // target i's generator offset, from the earlier targets' maxima
            int mv[VMAS_SPAWN_MAX_TARGETS];
#pragma unroll
            for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j) mv[j] = j < i ? ld_agent(W + j) : 0;  // (one round trip)
            unsigned long long off = rng_s[1];
#pragma unroll
            for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j)
                if (j < i) off += (unsigned long long)(mv[j] == 0 ? 1 : mv[j] + 2) * per_try;
            off_s = off;
        }
        if (wave == 0) best[lane] = MT;
        // the other targets (earlier ones already moved, by items that may have run on another XCD:
        // loaded with agent-scope atomics, sc1, as they were stored), with the maxima's round trip
        for (int m = io.n_agents + wave; m < n_occ; m += kSpawnWaves) {
            const int j = m - io.n_agents + (m - io.n_agents >= i ? 1 : 0);
            const float* p = io.pos[j] + (long)bb * io.pos_s0[j];
            occ[m][lane] = make_float2(ld_agent(p), ld_agent(p + io.pos_s1[j]));
        }
        __syncthreads();
        const unsigned long long off = off_s, seed = rng_s[0];
        if (prof && threadIdx.x == 0) prof[(long)it * 6 + 2] = __builtin_amdgcn_s_memrealtime();
        // rounds of kSpawnWaves tries, wave w drawing try base + w for the lanes still open; the
        // workgroup agrees after each round whether another is needed (one round unless an env
        // rejects 16 tries in a row).  (Without the rounds' barrier a wave whose try was rejected
        // went on to its next try before seeing another wave's earlier acceptance: 8 us per item
        // instead of one round's ~3.)
        for (int base = 0; base < MT; base += kSpawnWaves) {
            const int k = base + wave;
            if (valid && best[lane] == MT && k < MT) {
                const unsigned long long o = off + (unsigned long long)k * per_try;
                const float x = uniform_at(seed, o, g, b, io.x_lo, io.x_hi, io.mode);
                const float y = uniform_at(seed, o + g.inc, g, b, io.y_lo, io.y_hi, io.mode);
                bool hit = false;
                for (int m = 0; m < n_occ; ++m) {
                    const float2 o2 = occ[m][lane];
                    hit = hit || near(o2.x, o2.y, x, y, d2_min);
                }
                if (!hit) {
                    won[wave][lane] = make_float2(x, y);
                    atomicMin(&best[lane], k);
                }
            }
            if (!__syncthreads_or(valid && best[lane] == MT)) break;
        }
        if (prof && threadIdx.x == 0) prof[(long)it * 6 + 3] = __builtin_amdgcn_s_memrealtime();
        if (wave == 0) {
            const int k = valid ? best[lane] : 0;
            const bool unresolved = valid && k == MT;
            if (unresolved) atomicAdd(&W[T], 1);
            int km = unresolved ? 0 : k;  // one atomic per wave
            for (int s = 32; s > 0; s >>= 1) km = max(km, __shfl_xor(km, s));
            if (lane == 0 && km > 0) atomicMax(&W[i], km);
            if (io.backup && valid) {  // target i's position before the launch (only this item writes it)
                const float* p = io.pos[i] + (long)b * io.pos_s0[i];
                float* q = io.backup + ((long)i * io.batch + b) * 2;
                q[0] = p[0];
                q[1] = p[io.pos_s1[i]];
            }
            if (cov && !unresolved) {  // try k was drawn and accepted by wave k % kSpawnWaves
                const float2 xy = won[k % kSpawnWaves][lane];
                float* p = io.pos[i] + (long)b * io.pos_s0[i];
                __hip_atomic_store(p, xy.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(p + io.pos_s1[i], xy.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the positions and the maxima have landed before the completion (the sc1 hand-off of
            // vmas_jit_ops.hpp: no agent fence, 1.7-6.5 us each)
            __builtin_amdgcn_s_waitcnt(0);
            int last = 0;
            if (lane == 0) {
                last = atomicAdd(&done[32 * i], 1) == n_groups - 1;
                if (prof) prof[(long)it * 6 + 4] = __builtin_amdgcn_s_memrealtime();
            }
            if (ch.out && i == T - 1 && __shfl(last, 0)) publish_channel(ch, W, T, rng_s[2], rng_s[1], per_try);
        }
        // (item_s is rewritten only after every wave has passed the barrier above)
    }
}

// The same loop with a workgroup per 64-env group for every target (grid = the groups, used when
// they fit the device at once: the launch then needs every workgroup resident, which holds on an
// otherwise idle device -- stream order keeps the step's other kernels out -- and the bounded
// wait turns anything else into the error word rather than a hang).  The group's occupied
// positions stay in LDS from target to target (its own new positions included: no other
// workgroup reads them), so the only hand-off between workgroups per target is the maxima: the
// completion count, then one load of the maxima.  Per target ~6 us instead of the claimed
// items' ~11 (a claim round trip and the sc1 position loads on the critical path).
__global__ void __launch_bounds__(64 * kSpawnWaves) k_spawn_targets_resident(VmasSpawnTargetsIO io, DrawGrid g,
                                                                           float d2_min, unsigned long long* prof,
                                                                           ChanArgs ch) {
    __shared__ int best[64];
    __shared__ int abort_s;
    __shared__ unsigned long long off_s, rng_s[3];
    __shared__ float2 occ[32 + VMAS_SPAWN_MAX_TARGETS][64];  // agents, then every target
    __shared__ float2 won[kSpawnWaves][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int T = io.n_targets, A = io.n_agents, n_groups = (int)gridDim.x;
    int32_t* const W = io.max_accepted;
    int32_t* const err = W + 64;
    int32_t* const done = W + 96;
    unsigned long long* const rep = reinterpret_cast<unsigned long long*>(W + 96 + 32 * T);  // 128-byte lines
    const unsigned long long per_try = 2ull * g.inc;
    const int MT = io.max_tries > 0 ? io.max_tries : VMAS_SPAWN_MAX_TRIES;
    const int b = (int)blockIdx.x * 64 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    for (int m = wave; m < A + T; m += kSpawnWaves) {
        const float* p;
        int s1;
        if (m < A) {
            p = io.agents + (long)bb * io.ag_s0 + (long)m * io.ag_s1;
            s1 = io.ag_s2;
        } else {
            p = io.pos[m - A] + (long)bb * io.pos_s0[m - A];
            s1 = io.pos_s1[m - A];
        }
        occ[m][lane] = make_float2(p[0], p[s1]);
        if (m >= A && io.backup && valid) {  // the targets' positions before the launch
            float* q = io.backup + ((long)(m - A) * io.batch + b) * 2;
            q[0] = occ[m][lane].x;
            q[1] = occ[m][lane].y;
        }
    }
    if (threadIdx.x == 0) launch_rng(io, ch, &rng_s[0], &rng_s[1], &rng_s[2]);  // (read before the first barrier)
    uint32_t covm = 0u;  // (wave 0) the lane's covered targets
    if (wave == 0 && valid)
        for (int i = 0; i < T; ++i) covm |= io.covered[(long)b * io.cov_s0 + (long)i * io.cov_s1] ? (1u << i) : 0u;
    // (wave 0) the targets whose new position waits in occ[A + i]: stored after the last target (no
    // other workgroup reads them), so a target's completion waits only for its maximum
    uint32_t movm = 0u;
    auto store_moved = [&]() {
        for (int i = 0; i < T; ++i)
            if ((movm >> i) & 1u) {
                float* p = io.pos[i] + (long)b * io.pos_s0[i];
                p[0] = occ[A + i][lane].x;
                p[io.pos_s1[i]] = occ[A + i][lane].y;
            }
    };
    for (int i = 0; i < T; ++i) {
        const long it = (long)i * n_groups + blockIdx.x;
        if (threadIdx.x == 0) {
            const unsigned long long t_claim = __builtin_amdgcn_s_memrealtime();
            bool ok = true;
            unsigned long long tries = 0;  // tries the earlier targets consumed
            if (i > 0) {  // the last group done with target i - 1 publishes (i, tries) in our replica
                const unsigned long long* rp = rep + 16 * (blockIdx.x % kSpawnReplicas);
                unsigned long long v;
                while (((v = ld_agent(rp)) >> 32) != (unsigned long long)i) {
                    if (ld_agent(err) || __builtin_amdgcn_s_memrealtime() - t_claim > kSpawnWaitTicks) {
                        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
                tries = v & 0xFFFFFFFFull;
            }
            abort_s = ok ? 0 : 1;
            if (prof) {
                prof[it * 6 + 0] = t_claim;
                prof[it * 6 + 1] = __builtin_amdgcn_s_memrealtime();
                prof[it * 6 + 5] = blockIdx.x;
            }
            off_s = rng_s[1] + tries * per_try;
        }
        if (wave == 0) best[lane] = MT;
        __syncthreads();
        if (abort_s) {
            if (wave == 0) store_moved();  // (the targets done before the timeout, as they were)
            return;
        }
        if (prof && threadIdx.x == 0) prof[it * 6 + 2] = __builtin_amdgcn_s_memrealtime();
        const unsigned long long off = off_s, seed = rng_s[0];
        for (int base = 0; base < MT; base += kSpawnWaves) {  // (as k_spawn_targets)
            const int k = base + wave;
            if (valid && best[lane] == MT && k < MT) {
                const unsigned long long o = off + (unsigned long long)k * per_try;
                const float x = uniform_at(seed, o, g, b, io.x_lo, io.x_hi, io.mode);
                const float y = uniform_at(seed, o + g.inc, g, b, io.y_lo, io.y_hi, io.mode);
                bool hit = false;
                for (int m = 0; m < A + T; ++m) {
                    if (m == A + i) continue;  // (the target itself)
                    const float2 o2 = occ[m][lane];
                    hit = hit || near(o2.x, o2.y, x, y, d2_min);
                }
                if (!hit) {
                    won[wave][lane] = make_float2(x, y);
                    atomicMin(&best[lane], k);
                }
            }
            if (!__syncthreads_or(valid && best[lane] == MT)) break;
        }
        if (prof && threadIdx.x == 0) prof[it * 6 + 3] = __builtin_amdgcn_s_memrealtime();
        if (wave == 0) {
            const int k = valid ? best[lane] : 0;
            const bool unresolved = valid && k == MT;
            if (unresolved) atomicAdd(&W[T], 1);
            int km = unresolved ? 0 : k;
            for (int s = 32; s > 0; s >>= 1) km = max(km, __shfl_xor(km, s));
            if (lane == 0 && km > 0) atomicMax(&W[i], km);
            if (((covm >> i) & 1u) && !unresolved) {
                occ[A + i][lane] = won[k % kSpawnWaves][lane];  // (read by the next target's tries, after its barrier)
                movm |= 1u << i;
            }
            __builtin_amdgcn_s_waitcnt(0);  // the maxima have landed before the completion
            int last = 0;
            if (lane == 0) {
                last = atomicAdd(&done[32 * i], 1) == n_groups - 1;
                if (prof) prof[it * 6 + 4] = __builtin_amdgcn_s_memrealtime();
            }
            // the last group done: every maximum has landed (each group's before its completion);
            // it publishes the tries consumed so far to the replicas the others poll (kSpawnReplicas
            // lines: one line polled by every workgroup took ~6 us to see the count complete)
            if (ch.out && i == T - 1 && __shfl(last, 0)) publish_channel(ch, W, T, rng_s[2], rng_s[1], per_try);
            if (__shfl(last, 0) && i + 1 < T) {
                int mv[VMAS_SPAWN_MAX_TARGETS];
#pragma unroll
                for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j) mv[j] = j <= i ? ld_agent(W + j) : 0;
                unsigned long long tries = 0;
#pragma unroll
                for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j)
                    if (j <= i) tries += (unsigned long long)(mv[j] == 0 ? 1 : mv[j] + 2);
                if (lane < kSpawnReplicas)
                    __hip_atomic_store(rep + 16 * lane, ((unsigned long long)(i + 1) << 32) | tries, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (wave == 0) store_moved();
}

// Zeroes a launch's words (vmas_spawn_targets) ahead of the spawn kernel.  A kernel rather than
// hipMemsetAsync: inside a captured HIP graph a memset node in front of the spawn kernel was seen
// to leave the words holding a repeated 16-byte pattern of pointer-like values on some replays
// (ROCm 7.2 / MI355X; discovery's graph step then timed out in the kernel's bounded wait), and
// round 1 saw memset nodes in front of k_world's persistent launch that had not completed when the
// kernel ran.  A kernel node is ordered like every other node of the graph.
// (With a channel it also stages the channel's generator state at kRngWord, see launch_rng.)
constexpr int kWinNextWord = 38;  // (the windowed kernels' window for the next call: kept by the clear)
__global__ void __launch_bounds__(256) k_spawn_clear(int32_t* w, int n, const uint64_t* chan_in) {
    for (int i = (int)threadIdx.x; i < n; i += 256)
        if (i != kWinNextWord) w[i] = 0;
    __syncthreads();
    if (chan_in && threadIdx.x < 3)
        reinterpret_cast<unsigned long long*>(w + kRngWord)[threadIdx.x] =
            __hip_atomic_load(chan_in + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- the windowed respawn (k_spawn_cands + k_spawn_chain): no hand-off per target ---------------
//
// Every target draws from ONE stream of tries: try k of target i is pair p = P_i + k of the
// generator stream (x at offset o + p * per_try, y at + inc), P_0 = 0, P_{i+1} = P_i + consumed_i.
// So an env's candidates do not depend on the chain -- only WHICH pair each target starts at does,
// through the earlier targets' batch-global maxima.  The resident kernel resolves the targets one
// after another with a grid-wide hand-off per target (7 x ~9.5 us at C4).  Here k_spawn_cands
// evaluates the pairs [0, W) of every env once (W = the window, 128 by default: C4 consumes ~84),
// keeping per env and target a W-bit mask of the pairs that overlap nothing, and reduces per 64-env
// group, for every (target i, start pair P), the max over its envs of the first accepted try after
// P: k_e(i, P) = next_ok_e,i(P) - P.  k_spawn_chain (one workgroup) reduces those tables over the
// groups and walks the chain P_0 -> P_1 -> ... with table lookups.
//
// The masks hold target i's occupied set before the call except that an env with a covered target
// j < i ("dirty" for i) has j at its NEW position, which depends on P_j.  Those envs (every env with a
// covered target; ~0.6 % at C4) leave the tables for the targets after their first covered one and
// go to a list instead: their masks are taken against the agents and the targets that do not move
// before i, and the chain tests the surviving candidates against the moved targets while it walks,
// one thread per listed env, then writes every covered target's new position.  Nothing else
// moves; no co-residency, no bounded wait.  An env with no accepted pair inside the window, a list
// longer than the chain's capacity, or an env past max_tries marks the call unresolved: the caller
// redoes it with the reference loop (scenarios/discovery.py).
constexpr int kWinThreads = 1024, kWinWaves = kWinThreads / 64;
constexpr int kWinMaxPairs = 128;  // the masks' width
constexpr int kWinListWord = 33;   // (max_accepted words) listed envs
constexpr int kWinChainLds = 150 * 1024;

// listed envs the chain holds: masks (T x 16 B), new positions, two candidates (T x 3 x 8 B), their
// pairs (T x 4 B), env + covered bits
__host__ __device__ inline int win_list_cap(int T) {
    const int c = (kWinChainLds - T * kWinMaxPairs) / (T * 44 + 8);
    return (c > kWinThreads ? kWinThreads : c) & ~3;  // (even: the reduction buffer after it stays 16-byte aligned)
}

struct WinArgs {
    uint32_t* part;   // [groups][T * 32]: a group's table, 4 start pairs (bytes) per word
    uint32_t* crow;   // [clusters][T * 32]: a cluster's table
    uint32_t* list;   // [cap][2 + 4 T]: env, covered bits, T 128-bit masks
    int cap, pairs, q0;
};
constexpr int kWinCluster = 16;  // groups per cluster (the first reduction of the tables)
// The window of a call: the previous call's consumption + kWinMargin tries, rounded up to 16 (its
// chain kernel leaves it in the words at kWinNextWord; 0, or anything else, means the full window).
// C4 consumes ~74-84 tries over 7 targets (std ~3): 96 or 112 instead of 128 draws per env.
constexpr int kWinMargin = 24;
__device__ __forceinline__ int win_pairs(const int32_t* W, int full) {
    const int w = W[kWinNextWord];
    return (w >= 32 && w < full && (w & 15) == 0) ? w : full;  // (a multiple of 16: whole pairs per wave)
}
// (max_accepted words) cluster c's count: the per-target kernels' replica words, free here
__host__ __device__ inline int win_cluster_word(int T) { return 96 + 32 * T; }

__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// per-byte maximum of two words (two packed 16-bit maxima)
__device__ __forceinline__ uint32_t bytes_max(uint32_t a, uint32_t b) {
    const u16x2 lo = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a & 0x00FF00FFu),
                                               __builtin_bit_cast(u16x2, b & 0x00FF00FFu));
    const u16x2 hi = __builtin_elementwise_max(__builtin_bit_cast(u16x2, (a >> 8) & 0x00FF00FFu),
                                               __builtin_bit_cast(u16x2, (b >> 8) & 0x00FF00FFu));
    return __builtin_bit_cast(uint32_t, lo) | (__builtin_bit_cast(uint32_t, hi) << 8);
}

// max over the wave of non-negative v (DPP row shifts, then the row broadcasts)
__device__ __forceinline__ int wave_max_nonneg(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

// the first set bit >= P of a 128-bit mask (kWinMaxPairs when none)
__device__ __forceinline__ int next_bit128(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, int P) {
    if (P >= kWinMaxPairs) return kWinMaxPairs;
    const unsigned long long lo = ((unsigned long long)m1 << 32) | m0, hi = ((unsigned long long)m3 << 32) | m2;
    if (P < 64) {
        const unsigned long long x = lo & (~0ull << P);
        if (x) return __builtin_ctzll(x);
        return hi ? 64 + __builtin_ctzll(hi) : kWinMaxPairs;
    }
    const unsigned long long x = hi & (~0ull << (P - 64));
    return x ? 64 + __builtin_ctzll(x) : kWinMaxPairs;
}

// uniform_at when torch's grid covers the batch in one round (B <= step, so q = 0): one philox
// block, component off & 3 -- branch-free, so that the x and y draws of several pairs interleave
__device__ __forceinline__ float draw_q0(unsigned long long seed, unsigned long long off, int b, float lo, float hi,
                                         int mode) {
    const unsigned long long c = off / 4;
    const uint4 r = philox10(make_uint4((unsigned int)c, (unsigned int)(c >> 32), (unsigned int)b, 0u),
                             make_uint2((unsigned int)seed, (unsigned int)(seed >> 32)));
    const int sub = (int)(off & 3ull);
    const unsigned int u = sub == 0 ? r.x : sub == 1 ? r.y : sub == 2 ? r.z : r.w;
    const float inv = 2.3283064e-10f;  // ROCRAND_2POW32_INV
    const float unit = (mode & 1) ? __builtin_fmaf((float)u, inv, inv) : inv + (float)u * inv;
    const float range = hi - lo;
    const float val = (mode & 2) ? __builtin_fmaf(unit, range, lo) : unit * range + lo;
    return val == hi ? lo : val;
}

__device__ __forceinline__ float2 spawn_pair(const VmasSpawnTargetsIO& io, const DrawGrid& g, bool q0,
                                             unsigned long long seed, unsigned long long off0, int p, int b) {
    const unsigned long long o = off0 + (unsigned long long)p * 2ull * g.inc;
    if (q0)
        return make_float2(draw_q0(seed, o, b, io.x_lo, io.x_hi, io.mode),
                           draw_q0(seed, o + g.inc, b, io.y_lo, io.y_hi, io.mode));
    return make_float2(uniform_at(seed, o, g, b, io.x_lo, io.x_hi, io.mode),
                       uniform_at(seed, o + g.inc, g, b, io.y_lo, io.y_hi, io.mode));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// near() on packed pairs (v_pk_add_f32 / v_pk_mul_f32: each half rounds as the scalar form)
__device__ __forceinline__ bool near_pk(f32x2 o, f32x2 c, float d2_min) {
    const f32x2 d = o - c;
    const f32x2 q = d * d;
    return q.x + q.y < d2_min;
}

// (the chain's draws: one out-of-line copy -- the chain kernel runs on one CU, with a cold
// instruction cache every call, so its code size is its latency)
template <bool Q0>
__device__ __noinline__ float2 spawn_pair_call(float x_lo, float x_hi, float y_lo, float y_hi, int mode,
                                               long long step, unsigned long long inc, unsigned long long seed,
                                               unsigned long long off0, int p, int b) {
    const unsigned long long o = off0 + (unsigned long long)p * 2ull * inc;
    if (Q0) return make_float2(draw_q0(seed, o, b, x_lo, x_hi, mode), draw_q0(seed, o + inc, b, y_lo, y_hi, mode));
    const DrawGrid g{step, inc};
    return make_float2(uniform_at(seed, o, g, b, x_lo, x_hi, mode), uniform_at(seed, o + inc, g, b, y_lo, y_hi, mode));
}

// ---- every group: candidates, masks, the group's table (and its listed envs) ----------------------
// R pairs per wave (window 16 R); Q0: torch's grid covers the batch in one round (draw_q0)
template <int R, bool Q0>
__global__ void __launch_bounds__(kWinThreads) k_spawn_cands(VmasSpawnTargetsIO io, DrawGrid g, float d2_min,
                                                             WinArgs wa, unsigned long long* prof, ChanArgs ch) {
    extern __shared__ __align__(16) unsigned char win_lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int T = io.n_targets, A = io.n_agents, n_occ = A + T, cols = T * 32;
    const int b = (int)blockIdx.x * 64 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    if (prof && threadIdx.x == 0) {
        if (blockIdx.x == 0) prof[0] = __builtin_amdgcn_s_memrealtime();
        prof[32 + gridDim.x + blockIdx.x] = __builtin_amdgcn_s_memrealtime();  // (group g's start)
    }
    const int WP = win_pairs(io.max_accepted, wa.pairs);  // (the tries this call evaluates)
    float2* occ = reinterpret_cast<float2*>(win_lds);                // [n_occ][64]
    uint32_t* okw = reinterpret_cast<uint32_t*>(occ + n_occ * 64);   // [T][64][4] the masks
    uint32_t* covs = okw + T * 64 * 4;                               // [64] covered bits
    unsigned long long* rng = reinterpret_cast<unsigned long long*>(covs + 64);  // [3]
    for (int m = wave; m < n_occ; m += kWinWaves) {
        const float* p;
        int s1;
        if (m < A) {
            p = io.agents + (long)bb * io.ag_s0 + (long)m * io.ag_s1;
            s1 = io.ag_s2;
        } else {
            p = io.pos[m - A] + (long)bb * io.pos_s0[m - A];
            s1 = io.pos_s1[m - A];
        }
        const float2 v = make_float2(p[0], p[s1]);
        occ[m * 64 + lane] = v;
        if (m >= A && io.backup && valid) {  // the targets' positions before the call
            float* q = io.backup + ((long)(m - A) * io.batch + b) * 2;
            q[0] = v.x;
            q[1] = v.y;
        }
    }
    for (int q = (int)threadIdx.x; q < T * 64 * 4; q += kWinThreads) okw[q] = 0u;
    if (wave == 0) {
        uint32_t cm = 0u;
        if (valid)
            for (int i = 0; i < T; ++i) cm |= io.covered[(long)b * io.cov_s0 + (long)i * io.cov_s1] ? (1u << i) : 0u;
        covs[lane] = cm;
    }
    if (threadIdx.x == 0) launch_rng(io, ch, &rng[0], &rng[1], &rng[2]);
    __syncthreads();
    const unsigned long long seed = rng[0], off0 = rng[1];
    const uint32_t covm = covs[lane];
    {
        // this wave's R pairs, all drawn first (independent philox chains in flight), then tested
        // against each occupied position once
        // (this call's window spread over every wave: Rw <= R pairs each, so that no SIMD keeps
        // the full window's share when the window shrinks)
        const int Rw = (WP + kWinWaves - 1) / kWinWaves;
        const int p0 = __builtin_amdgcn_readfirstlane(wave) * Rw;
        f32x2 c[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float2 v = r < Rw ? spawn_pair(io, g, Q0, seed, off0, p0 + r, bb) : make_float2(0.f, 0.f);
            c[r] = f32x2{v.x, v.y};
        }
        uint32_t hit = 0u;  // bit r: pair r lands near an agent
        for (int m = 0; m < A; ++m) {
            const float2 o = occ[m * 64 + lane];
            const f32x2 o2{o.x, o.y};
#pragma unroll
            for (int r = 0; r < R; ++r) hit |= near_pk(o2, c[r], d2_min) ? (1u << r) : 0u;
        }
        uint32_t far[VMAS_SPAWN_MAX_TARGETS];  // bit r: pair r clear of target j's position before the call
#pragma unroll
        for (int j = 0; j < VMAS_SPAWN_MAX_TARGETS; ++j) {
            uint32_t f = ~0u;
            if (j < T) {
                const float2 o = occ[(A + j) * 64 + lane];
                const f32x2 o2{o.x, o.y};
                f = 0u;
#pragma unroll
                for (int r = 0; r < R; ++r) f |= near_pk(o2, c[r], d2_min) ? 0u : (1u << r);
            }
            far[j] = f;
        }
        // target i's occupied set: every target after it, the targets before it that do not move
        // (not covered), never itself -- prefix / suffix products of the clear-of bits
        uint32_t suf[VMAS_SPAWN_MAX_TARGETS + 1];
        suf[VMAS_SPAWN_MAX_TARGETS] = ~0u;
#pragma unroll
        for (int j = VMAS_SPAWN_MAX_TARGETS - 1; j >= 0; --j) suf[j] = suf[j + 1] & far[j];
        const uint32_t rmask = (1u << Rw) - 1u;
        const int s = p0, w0 = s >> 5, sh = s & 31;
        uint32_t pre = ~0u;
#pragma unroll
        for (int i = 0; i < VMAS_SPAWN_MAX_TARGETS; ++i) {
            const uint32_t ok = ~hit & rmask & pre & suf[i + 1];
            pre &= ((covm >> i) & 1u) ? ~0u : far[i];
            if (i < T && ok) {
                atomicOr(&okw[(i * 64 + lane) * 4 + w0], ok << sh);
                if (sh + Rw > 32) atomicOr(&okw[(i * 64 + lane) * 4 + w0 + 1], ok >> (32 - sh));
            }
        }
    }
    __syncthreads();
    if (prof && blockIdx.x == 0 && threadIdx.x == 0) prof[30] = __builtin_amdgcn_s_memrealtime();
    uint32_t mk0 = 0u, mk1 = 0u, mk2 = 0u, mk3 = 0u;  // (wave i < T) the lane's mask of target i
    if (wave < T) {
        const uint4 v = *reinterpret_cast<const uint4*>(&okw[(wave * 64 + lane) * 4]);
        mk0 = v.x;
        mk1 = v.y;
        mk2 = v.z;
        mk3 = v.w;
    }
    if (wave == 0 && valid && covm) {  // an env with a covered target: listed for the chain
        const int d = atomicAdd(&io.max_accepted[kWinListWord], 1);
        if (d < wa.cap) {
            uint32_t* e = wa.list + (long)d * (2 + 4 * T);
            e[0] = (uint32_t)b;
            e[1] = covm;
            for (int i = 0; i < T; ++i)
                *reinterpret_cast<uint4*>(e + 2 + 4 * i) = *reinterpret_cast<const uint4*>(&okw[(i * 64 + lane) * 4]);
        }
    }
    __syncthreads();  // (the masks are in registers: the space becomes the table)
    uint32_t* ktab = reinterpret_cast<uint32_t*>(win_lds);  // [64][cols + 1]: byte P & 3 of word (i, P >> 2)
    if (wave < T) {
        // k(P) = the first accepted pair at or after P, minus P, for P = 127 .. 0 (255: none in the
        // window); 0 for an env that is not in target i's table (dirty for i, or past the batch)
        const int i = wave;
        const bool in_table = valid && (covm & ((1u << i) - 1u)) == 0u;
        uint32_t k = 255u, packed = 0u;
#pragma unroll
        for (int P = kWinMaxPairs - 1; P >= 0; --P) {
            const uint32_t word = P < 32 ? mk0 : P < 64 ? mk1 : P < 96 ? mk2 : mk3;
            const bool ok = (word >> (P & 31)) & 1u;  // (pairs past the window never set)
            k = ok ? 0u : (k + 1u > 255u ? 255u : k + 1u);
            packed |= (in_table ? k : 0u) << (8 * (P & 3));
            if ((P & 3) == 0) {
                ktab[lane * (cols + 1) + i * 32 + (P >> 2)] = packed;
                packed = 0u;
            }
        }
    }
    __syncthreads();
    if (prof && blockIdx.x == 0 && threadIdx.x == 0) prof[31] = __builtin_amdgcn_s_memrealtime();
    for (int c = (int)threadIdx.x; c < cols; c += kWinThreads) {  // the group's table: max over its 64 envs
        uint32_t acc = 0u;
#pragma unroll 8
        for (int l = 0; l < 64; ++l) acc = bytes_max(acc, ktab[l * (cols + 1) + c]);
        st_agent(wa.part + (long)blockIdx.x * cols + c, acc);
    }
    // The last group of each cluster of kWinCluster reduces the cluster's tables into one row (the
    // chain then reads G / kWinCluster rows, not G: one workgroup pulls ~10 B per cycle from HBM).
    // The rows go out as agent-scope stores and come back as agent-scope loads (another XCD's L2
    // may hold the lines), landed before the cluster's count.
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    __shared__ int last_s;
    const int cl = (int)blockIdx.x / kWinCluster, first = cl * kWinCluster;
    const int members = min(kWinCluster, (int)gridDim.x - first);
    if (threadIdx.x == 0) last_s = atomicAdd(&io.max_accepted[win_cluster_word(T) + cl], 1) == members - 1;
    __syncthreads();
    if (prof && blockIdx.x == 0 && threadIdx.x == 0) prof[29] = __builtin_amdgcn_s_memrealtime();
    if (last_s) {
        const int per = kWinThreads / cols, c = (int)threadIdx.x % cols, r0 = (int)threadIdx.x / cols;
        uint32_t acc = 0u;
        if (r0 < per) {
            uint32_t v[kWinCluster];
#pragma unroll
            for (int u = 0; u < kWinCluster; ++u) {
                const int r = r0 + u * per;
                v[u] = r < members ? ld_agent(wa.part + (long)(first + r) * cols + c) : 0u;
            }
#pragma unroll
            for (int u = 0; u < kWinCluster; ++u) acc = bytes_max(acc, v[u]);
        }
        uint32_t* red = ktab;  // (the table space is free again)
        red[threadIdx.x] = acc;
        __syncthreads();
        if ((int)threadIdx.x < cols) {
            for (int r = 1; r < per; ++r) acc = bytes_max(acc, red[r * cols + threadIdx.x]);
            wa.crow[(long)cl * cols + threadIdx.x] = acc;
        }
    }
    if (prof && threadIdx.x == 0) prof[32 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

// ---- one workgroup: the tables over every group, then the chain of targets ------------------------
// Chain of the targets.  (a) The clean chain: P_i from the reduced tables alone.  (b) Every listed
// env's candidates at the first two accepted pairs (against the targets that do not move) at or
// after P_i, one thread per (env, target).  (c) The first of them clear of the env's moved targets
// (more, drawn in place, if both land on one): one thread per (env, target) for an env with one
// covered target (its moved target's position is its first candidate there), one thread per env,
// in target order, for an env with several.  (d) Where no listed env needs more tries than a
// target's clean maximum, the clean chain is the chain; else it is rebuilt from the first such
// target with the listed envs' maxima, one target at a time (P_j for the targets before it are
// right: their maxima held).
template <bool Q0>
__global__ void __launch_bounds__(kWinThreads) k_spawn_chain(VmasSpawnTargetsIO io, DrawGrid g, float d2_min,
                                                             WinArgs wa, int n_rows, unsigned long long* prof,
                                                             ChanArgs ch) {
    extern __shared__ __align__(16) unsigned char win_lds[];
    __shared__ unsigned long long rng_s[3];
    __shared__ int red_s[2][kWinWaves];  // (double-buffered: one barrier per step)
    __shared__ int ps_s[VMAS_SPAWN_MAX_TARGETS + 1], mc_s[VMAS_SPAWN_MAX_TARGETS], lmax_s[VMAS_SPAWN_MAX_TARGETS];
    __shared__ int bad_s, i0_s;
    __shared__ unsigned long long stamp_s[8];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int T = io.n_targets, c4 = T * 8;  // (uint4 columns of a table row)
    int32_t* const W = io.max_accepted;
    const int MT = io.max_tries > 0 ? io.max_tries : VMAS_SPAWN_MAX_TRIES;
    const int WP = win_pairs(W, wa.pairs);  // (as the candidates kernel evaluated them)
    const int cap = win_list_cap(T);
    uint32_t* lmask = reinterpret_cast<uint32_t*>(win_lds);             // [cap][T][4]
    float2* newpos = reinterpret_cast<float2*>(lmask + cap * T * 4);      // [cap][T]
    float2* cand1 = newpos + cap * T;                                     // [cap][T]
    float2* cand2 = cand1 + cap * T;                                      // [cap][T]
    uint32_t* pp = reinterpret_cast<uint32_t*>(cand2 + cap * T);          // [cap][T] p1 | p2 << 16
    uint32_t* linfo = pp + cap * T;                                       // [cap][2]
    uint8_t* mclean = reinterpret_cast<uint8_t*>(linfo + cap * 2);        // [T][128]
    const bool stamp = prof && threadIdx.x == 0;
    if (stamp) stamp_s[0] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) launch_rng(io, ch, &rng_s[0], &rng_s[1], &rng_s[2]);
    const int n_listed = W[kWinListWord];
    const int n_list = n_listed < cap ? n_listed : cap;
    if ((int)threadIdx.x < c4) {  // column c of the tables: max over every cluster's row, 16 loads in flight
        const uint4* src = reinterpret_cast<const uint4*>(wa.crow) + threadIdx.x;
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        for (int r0 = 0; r0 < n_rows; r0 += 16) {
            uint4 v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = r0 + u < n_rows ? src[(long)(r0 + u) * c4] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                acc.x = bytes_max(acc.x, v[u].x);
                acc.y = bytes_max(acc.y, v[u].y);
                acc.z = bytes_max(acc.z, v[u].z);
                acc.w = bytes_max(acc.w, v[u].w);
            }
        }
        reinterpret_cast<uint4*>(mclean)[threadIdx.x] = acc;  // byte P of row i = max over groups of k(i, P)
    }
    {
        // the listed envs: entry d = [env, covered, T masks], 4 loads in flight per thread
        const int E = 2 + 4 * T;
        for (int q0i = 0; q0i < n_list * E; q0i += 4 * kWinThreads) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0i + u * kWinThreads + (int)threadIdx.x;
                v[u] = q < n_list * E ? wa.list[q] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0i + u * kWinThreads + (int)threadIdx.x;
                if (q < n_list * E) {
                    const int d = q / E, f = q - d * E;
                    if (f < 2) linfo[d * 2 + f] = v[u];
                    else lmask[d * T * 4 + (f - 2)] = v[u];
                }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // (a) the clean chain
        if (stamp) stamp_s[1] = __builtin_amdgcn_s_memrealtime();
        int P = 0, bad = T;
        for (int i = 0; i < T; ++i) {
            const int M = P < kWinMaxPairs ? (int)mclean[i * kWinMaxPairs + P] : 255;
            ps_s[i] = P;
            mc_s[i] = M;
            lmax_s[i] = 0;
            if (M >= 255 || M >= MT) {
                bad = i;
                break;
            }
            P += M == 0 ? 1 : M + 2;
        }
        bad_s = bad;
    }
    __syncthreads();
    const int bad = bad_s;
    const unsigned long long seed = rng_s[0], off0 = rng_s[1];
    // (b) the candidates of every (listed env, target after its first covered one or covered)
    for (int it = (int)threadIdx.x; it < n_list * T; it += kWinThreads) {
        const int d = it / T, i = it - d * T;
        const uint32_t cov = linfo[d * 2 + 1];
        const int j0 = __builtin_ctz(cov);
        if (i >= bad || !(i > j0 || ((cov >> i) & 1u))) continue;
        const uint4 m = *reinterpret_cast<const uint4*>(&lmask[(d * T + i) * 4]);
        const int p1 = next_bit128(m.x, m.y, m.z, m.w, ps_s[i]);
        const int p2 = i > j0 ? next_bit128(m.x, m.y, m.z, m.w, p1 + 1) : kWinMaxPairs;
        const int db = (int)linfo[d * 2];
        const float2 c1 = spawn_pair(io, g, Q0, seed, off0, p1 < WP ? p1 : 0, db);  // (both drawn: in flight together)
        const float2 c2 = spawn_pair(io, g, Q0, seed, off0, p2 < WP ? p2 : 0, db);
        cand1[d * T + i] = c1;
        cand2[d * T + i] = c2;
        pp[d * T + i] = (uint32_t)p1 | ((uint32_t)p2 << 16);
        if (i == j0) newpos[d * T + i] = c1;  // (its first covered target: the first accepted try)
    }
    __syncthreads();
    if (stamp) stamp_s[2] = __builtin_amdgcn_s_memrealtime();
    // target i's first accepted try of listed env d at start pair P (255: none within the window or
    // max_tries); covered: its new position.  pre: the precomputed candidates at P (else drawn).
    auto walk = [&](int d, int i, int P, bool pre) -> int {
        const uint4 m = *reinterpret_cast<const uint4*>(&lmask[(d * T + i) * 4]);
        const uint32_t dcov = linfo[d * 2 + 1];
        const uint32_t moved = dcov & ((1u << i) - 1u);
        const bool cov_i = (dcov >> i) & 1u;
        const uint32_t pw = pp[d * T + i];
        int p = pre ? (int)(pw & 0xFFFFu) : next_bit128(m.x, m.y, m.z, m.w, P);
        for (int n = 0; p < WP && p - P < MT; ++n) {
            const float2 cnd = pre && n == 0   ? cand1[d * T + i]
                               : pre && n == 1 ? cand2[d * T + i]
                                               : spawn_pair_call<Q0>(io.x_lo, io.x_hi, io.y_lo, io.y_hi, io.mode,
                                                                     g.step, g.inc, seed, off0, p, (int)linfo[d * 2]);
            bool hit = false;
            for (uint32_t mv = moved; mv; mv &= mv - 1u) {
                const float2 q = newpos[d * T + __builtin_ctz(mv)];
                hit = hit || near(q.x, q.y, cnd.x, cnd.y, d2_min);
            }
            if (!hit) {
                if (cov_i) newpos[d * T + i] = cnd;
                return p - P;
            }
            p = pre && n == 0 ? (int)(pw >> 16) : next_bit128(m.x, m.y, m.z, m.w, p + 1);
        }
        return 255;
    };
    // (c) one covered target: per (env, target after it), in parallel; several: per env, in order
    for (int it = (int)threadIdx.x; it < n_list * T; it += kWinThreads) {
        const int d = it / T, i = it - d * T;
        const uint32_t cov = linfo[d * 2 + 1];
        const int j0 = __builtin_ctz(cov);
        if ((cov & (cov - 1u)) == 0u) {
            if (i > j0 && i < bad) atomicMax(&lmax_s[i], walk(d, i, ps_s[i], true));
        } else if (i == j0) {
            for (int t = j0 + 1; t < bad; ++t) atomicMax(&lmax_s[t], walk(d, t, ps_s[t], true));
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // (d) the first target whose maximum a listed env raises
        int i0 = T;
        for (int i = 0; i < bad; ++i)
            if (lmax_s[i] > mc_s[i]) {
                i0 = i;
                break;
            }
        i0_s = i0;
        if (stamp) stamp_s[3] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const int i0 = i0_s;
    const int d = (int)threadIdx.x;
    const bool has = d < n_list;
    const uint32_t dcov = has ? linfo[d * 2 + 1] : 0u;
    const int j0 = has ? __builtin_ctz(dcov) : 32;  // the first covered target
    bool unresolved = n_listed > cap || (i0 == T && bad < T);
    if (!unresolved && i0 < T) {
        // rebuild from target i0: its maximum with the listed envs' (computed at the right P), then
        // one target at a time
        int P = ps_s[i0];
        int M = max(mc_s[i0], lmax_s[i0]);
        if (M >= 255 || M >= MT) unresolved = true;
        __syncthreads();  // (every thread has read mc_s[i0])
        if (threadIdx.x == 0) mc_s[i0] = M;
        for (int i = i0 + 1; i < T && !unresolved; ++i) {
            P += M == 0 ? 1 : M + 2;
            int kd = 0;
            if (has && (i > j0 || ((dcov >> i) & 1u))) {
                const int k = walk(d, i, P, false);
                if (i > j0) kd = k;
            }
            const int wm = wave_max_nonneg(kd);
            if (lane == 0) red_s[i & 1][wave] = wm;
            __syncthreads();
            M = P < kWinMaxPairs ? (int)mclean[i * kWinMaxPairs + P] : 255;
#pragma unroll
            for (int w = 0; w < kWinWaves; ++w) M = max(M, red_s[i & 1][w]);
            if (M >= 255 || M >= MT) unresolved = true;
            else if (threadIdx.x == 0) mc_s[i] = M;
        }
    }
    if (!unresolved && has) {  // every covered target of a listed env to its new position
        const int db = (int)linfo[d * 2];
        for (int i = 0; i < T; ++i)
            if ((dcov >> i) & 1u) {
                float* p = io.pos[i] + (long)db * io.pos_s0[i];
                p[0] = newpos[d * T + i].x;
                p[io.pos_s1[i]] = newpos[d * T + i].y;
            }
    }
    // the words the next call's candidates count on, back to zero (a prestaged call has no clear
    // kernel): the listed envs and every cluster's count (read above; the candidates are done)
    if (threadIdx.x == 0) W[kWinListWord] = 0;
    for (int c = (int)threadIdx.x; c < n_rows; c += kWinThreads) W[win_cluster_word(T) + c] = 0;
    if (threadIdx.x == 0) {
        int used = 0;  // (the tries the reference loop consumes: the next call's window from it)
        if (!unresolved)
            for (int i = 0; i < T; ++i) {
                W[i] = mc_s[i];
                used += mc_s[i] == 0 ? 1 : mc_s[i] + 2;
            }
        W[T] = unresolved ? 1 : 0;
        const int next = (used + kWinMargin + 15) & ~15;
        W[kWinNextWord] = unresolved || next >= wa.pairs ? 0 : max(next, 32);
    }
    if (stamp) {
        stamp_s[4] = __builtin_amdgcn_s_memrealtime();
        stamp_s[5] = (unsigned long long)i0;
        for (int k = 0; k < 6; ++k) prof[1 + k] = stamp_s[k];
    }
    if (ch.out) {  // (publish_channel reads the words with agent-scope loads: stored above by this group)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (wave == 0) publish_channel(ch, W, T, rng_s[2], rng_s[1], 2ull * g.inc);
    }
}

size_t win_cands_lds_bytes(int A, int T) {
    const size_t p1a = (size_t)(A + T) * 64 * 8 + (size_t)T * 64 * 16 + 64 * 4 + 3 * 8;
    const size_t p1b = (size_t)64 * (T * 32 + 1) * 4;
    return std::max(p1a, p1b);
}

size_t win_chain_lds_bytes(int T) {
    const size_t cap = (size_t)win_list_cap(T);
    return cap * (44 * T + 8) + (size_t)T * kWinMaxPairs;
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

}  // namespace

struct VmasSpawnChannel {
    int device = 0;
    uint64_t* h_in = nullptr;  // mapped pinned: seed, offset, seq
    uint64_t* d_in = nullptr;
    uint64_t* h_out = nullptr;  // mapped pinned: 16 maxima + unresolved + error (int32), seq word (u64 12)
    uint64_t* d_out = nullptr;
};

namespace {

unsigned long long* g_spawn_prof = nullptr;  // (VMAS_SPAWN_PROFILE) the last launch's item stamps
size_t g_spawn_prof_n = 0;

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
    VMAS_AUX_HIP(vmas_aux::fill_u32_async(s.d_out, 0u, 2, st));
    hipLaunchKernelGGL(k_spawn_resolve, dim3((batch + 255) / 256), dim3(256), 0, st, a, s.d_out);
    VMAS_AUX_HIP(hipGetLastError());
    VMAS_AUX_HIP(hipMemcpyAsync(s.h_out, s.d_out, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    vmas_aux::note_host_wait();
    VMAS_AUX_HIP(hipStreamSynchronize(st));
    *max_accepted = s.h_out[0];
    *n_unresolved = s.h_out[1];
    return VMAS_OK;
}

int32_t vmas_spawn_channel_create(int32_t device, VmasSpawnChannel** out) {
    if (!out || device < 0 || device >= 64) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_channel_create: bad arguments");
    *out = nullptr;
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    VmasSpawnChannel* ch = new VmasSpawnChannel();
    ch->device = device;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e = hipHostMalloc((void**)&ch->h_in, 4 * sizeof(uint64_t), fl);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&ch->d_in, ch->h_in, 0);
    if (e == hipSuccess) e = hipHostMalloc((void**)&ch->h_out, 16 * sizeof(uint64_t), fl);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&ch->d_out, ch->h_out, 0);
    if (cur != device) (void)hipSetDevice(cur);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        vmas_spawn_channel_destroy(ch);
        return vmas_aux::fail(VMAS_E_HIP, "vmas_spawn_channel_create: %s", hipGetErrorString(e));
    }
    for (int i = 0; i < 4; ++i) ch->h_in[i] = 0;
    for (int i = 0; i < 16; ++i) ch->h_out[i] = 0;
    *out = ch;
    return VMAS_OK;
}

int32_t vmas_spawn_channel_destroy(VmasSpawnChannel* ch) {
    if (!ch) return VMAS_OK;
    if (ch->h_in) (void)hipHostFree(ch->h_in);
    if (ch->h_out) (void)hipHostFree(ch->h_out);
    delete ch;
    return VMAS_OK;
}

int32_t vmas_spawn_channel_in(VmasSpawnChannel* ch, const uint64_t** d_in) {
    if (!ch || !d_in) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_channel_in: bad arguments");
    *d_in = ch->d_in;
    return VMAS_OK;
}

int32_t vmas_spawn_channel_arm(VmasSpawnChannel* ch, uint64_t seed, uint64_t offset, uint32_t seq) {
    if (!ch || seq == 0u) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_channel_arm: bad arguments");
    __atomic_store_n(&ch->h_in[0], seed, __ATOMIC_RELAXED);
    __atomic_store_n(&ch->h_in[1], offset, __ATOMIC_RELAXED);
    __atomic_store_n(&ch->h_in[2], (uint64_t)seq, __ATOMIC_RELEASE);
    return VMAS_OK;
}

int32_t vmas_spawn_channel_wait(VmasSpawnChannel* ch, uint32_t seq, int32_t* words, int32_t n_targets, void* stream) {
    if (!ch || !words || seq == 0u || n_targets < 1 || n_targets > VMAS_SPAWN_MAX_TARGETS)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_channel_wait: bad arguments");
    uint64_t v = 0;
    if (int32_t rc = vmas_aux::wait_host_word64(ch->h_out + kChanOutSeqWord, seq, &v, (hipStream_t)stream)) return rc;
    const int32_t* o = reinterpret_cast<const int32_t*>(ch->h_out);
    for (int i = 0; i < n_targets; ++i) words[i] = __atomic_load_n(o + i, __ATOMIC_RELAXED);
    words[n_targets] = __atomic_load_n(o + 16, __ATOMIC_RELAXED);
    words[n_targets + 1] = __atomic_load_n(o + 17, __ATOMIC_RELAXED);
    return VMAS_OK;
}

// (probe) copy the last profiled vmas_spawn_targets launch's item stamps (n words at most)
int32_t vmas_spawn_profile(uint64_t* out, int64_t n) {
    if (!g_spawn_prof || !out || n <= 0) return 0;
    const size_t k = std::min<size_t>((size_t)n, g_spawn_prof_n);
    VMAS_AUX_HIP(hipDeviceSynchronize());
    VMAS_AUX_HIP(hipMemcpy(out, g_spawn_prof, k * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return (int32_t)k;
}

int64_t vmas_spawn_scratch_words(int32_t batch, int32_t n_targets) {
    if (batch <= 0 || n_targets < 1 || n_targets > VMAS_SPAWN_MAX_TARGETS) return -1;
    const int64_t groups = (batch + 63) / 64;
    const int64_t clusters = (groups + kWinCluster - 1) / kWinCluster;
    return (groups + clusters) * n_targets * 32 + (int64_t)win_list_cap(n_targets) * (2 + 4 * n_targets);
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
    static int max_blocks[64] = {0}, resident[64] = {0}, resident_static[64] = {0};
    if (!max_blocks[device]) {
        hipDeviceProp_t prop;
        VMAS_AUX_HIP(hipGetDeviceProperties(&prop, device));
        max_blocks[device] = prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / kUniformThreads);
        if (max_blocks[device] <= 0) return vmas_aux::fail(VMAS_E_HIP, "vmas_spawn_targets: device properties");
        int per_cu = 0;
        VMAS_AUX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spawn_targets, 64 * kSpawnWaves, 0));
        resident[device] = prop.multiProcessorCount * std::max(per_cu, 1);
        per_cu = 0;
        VMAS_AUX_HIP(
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spawn_targets_resident, 64 * kSpawnWaves, 0));
        resident_static[device] = prop.multiProcessorCount * per_cu;
    }
    // torch's distribution-kernel grid and per-call philox increment on B elements (as
    // vmas_uniform_columns)
    const long long B = io->batch;
    const long long gx = std::min<long long>((B + kUniformThreads - 1) / kUniformThreads, max_blocks[device]);
    DrawGrid g{kUniformThreads * gx, (unsigned long long)((B - 1) / (kUniformThreads * gx * 4) + 1) * 4};
    const float d2_min = spawn_d2_min(io->min_dist);
    hipStream_t st = (hipStream_t)stream;
    const int T = io->n_targets, n_groups = (int)((B + 63) / 64);
    const char* kn = getenv("VMAS_SPAWN_KERNEL");
    const bool group_resident = n_groups <= resident_static[device] && !getenv("VMAS_SPAWN_CLAIMED") &&
                                !(kn && strcmp(kn, "claimed") == 0);
    const long long grid = std::min<long long>(n_groups, resident[device]);
    // VMAS_SPAWN_PROFILE=1 (a probe's knob): per item s_memrealtime stamps [claimed, wait over,
    // occupied loaded, tries done, completion added, workgroup] into g_spawn_prof (vmas_spawn_profile)
    unsigned long long* prof = nullptr;
    static const bool want_prof = getenv("VMAS_SPAWN_PROFILE") && getenv("VMAS_SPAWN_PROFILE")[0] == '1';
    if (want_prof) {
        const size_t need = std::max<size_t>((size_t)T * n_groups * 6, 32 + 2 * (size_t)n_groups);  // (window: [0] cands start, [1, 7) the chain's stamps, group 0's [30] pairs drawn, [31] sweep done, [29] tables stored, [32 + g] group g done, [32 + G + g] its start)
        if (g_spawn_prof_n < need) {
            if (g_spawn_prof) (void)hipFree(g_spawn_prof);
            VMAS_AUX_HIP(hipMalloc((void**)&g_spawn_prof, need * sizeof(unsigned long long)));
            g_spawn_prof_n = need;
        }
        prof = g_spawn_prof;
    }
    ChanArgs ch{nullptr, nullptr};
    if (io->channel) {
        if (io->channel->device != device) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_targets: channel of another device");
        ch.in = io->channel->d_in;
        ch.out = io->channel->d_out;
    }
    // the kernel: the windowed one when the caller gave it its scratch (VMAS_SPAWN_KERNEL=resident /
    // claimed selects the per-target hand-off kernels, an A/B knob)
    const bool per_target = kn && (strcmp(kn, "resident") == 0 || strcmp(kn, "claimed") == 0);
    const int64_t need = vmas_spawn_scratch_words(io->batch, T);
    if (!per_target && io->scratch && need > 0 && io->scratch_words >= need &&
        (n_groups + kWinCluster - 1) / kWinCluster <= 32 * 32) {  // (the cluster counts: the replica words)
        const char* wv = getenv("VMAS_SPAWN_WINDOW");
        const int pairs = wv ? atoi(wv) : kWinMaxPairs;
        if (pairs != 16 && pairs != 64 && pairs != 96 && pairs != 128)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_targets: VMAS_SPAWN_WINDOW=%d (16, 64, 96 or 128)", pairs);
        const int cap = win_list_cap(T);
        const size_t lds1 = win_cands_lds_bytes(io->n_agents, T), lds2 = win_chain_lds_bytes(T);
        const bool q0 = g.step >= B;
        using CandsFn = void (*)(VmasSpawnTargetsIO, DrawGrid, float, WinArgs, unsigned long long*, ChanArgs);
        CandsFn cands = nullptr;
        switch (pairs * 2 + (q0 ? 1 : 0)) {
            case 16 * 2 + 1: cands = k_spawn_cands<1, true>; break;
            case 16 * 2: cands = k_spawn_cands<1, false>; break;
            case 64 * 2 + 1: cands = k_spawn_cands<4, true>; break;
            case 64 * 2: cands = k_spawn_cands<4, false>; break;
            case 96 * 2 + 1: cands = k_spawn_cands<6, true>; break;
            case 96 * 2: cands = k_spawn_cands<6, false>; break;
            case 128 * 2 + 1: cands = k_spawn_cands<8, true>; break;
            default: cands = k_spawn_cands<8, false>; break;
        }
        static bool attr[64] = {false};
        if (!attr[device]) {  // (as k_step: > 64 KiB of dynamic LDS; HIP on gfx950 may refuse the attribute and
                              // launch anyway -- the launch's own error check below is the one that counts)
            (void)hipFuncSetAttribute((const void*)k_spawn_chain<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds2);
            (void)hipFuncSetAttribute((const void*)k_spawn_chain<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds2);
            (void)hipGetLastError();
            attr[device] = true;
        }
        const int n_clusters = (n_groups + kWinCluster - 1) / kWinCluster;
        uint32_t* sw = reinterpret_cast<uint32_t*>(io->scratch);
        WinArgs wa{sw, sw + (size_t)n_groups * T * 32, sw + (size_t)(n_groups + n_clusters) * T * 32, cap, pairs,
                   q0 ? 1 : 0};
        if (!(io->prestaged && ch.in))  // (prestaged: cleaned by the previous call, staged by the step)
            hipLaunchKernelGGL(k_spawn_clear, dim3(1), dim3(256), 0, st, io->max_accepted, (int)VMAS_SPAWN_WORDS(T),
                               ch.in);
        hipLaunchKernelGGL(cands, dim3((unsigned)n_groups), dim3(kWinThreads), lds1, st, *io, g, d2_min, wa, prof, ch);
        if (q0)
            hipLaunchKernelGGL(k_spawn_chain<true>, dim3(1), dim3(kWinThreads), lds2, st, *io, g, d2_min, wa, n_clusters,
                               prof, ch);
        else
            hipLaunchKernelGGL(k_spawn_chain<false>, dim3(1), dim3(kWinThreads), lds2, st, *io, g, d2_min, wa,
                               n_clusters, prof, ch);
        VMAS_AUX_HIP(hipGetLastError());
        *increment = g.inc;
        return VMAS_OK;
    }
    hipLaunchKernelGGL(k_spawn_clear, dim3(1), dim3(256), 0, st, io->max_accepted, (int)VMAS_SPAWN_WORDS(T), ch.in);
    if (group_resident)
        hipLaunchKernelGGL(k_spawn_targets_resident, dim3((unsigned)n_groups), dim3(64 * kSpawnWaves), 0, st, *io, g,
                           d2_min, prof, ch);
    else
        hipLaunchKernelGGL(k_spawn_targets, dim3((unsigned)grid), dim3(64 * kSpawnWaves), 0, st, *io, g, d2_min,
                           n_groups, prof, ch);
    VMAS_AUX_HIP(hipGetLastError());
    *increment = g.inc;
    return VMAS_OK;
}

}  // extern "C"
