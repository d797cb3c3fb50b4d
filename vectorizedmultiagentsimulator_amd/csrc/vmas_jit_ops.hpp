// vmas_jit_ops.hpp -- per-entity force terms and integration for the world-specialised kernels
// (csrc/vmas_jit.hip, compiled by hipRTC).  Same operations, same order as pre_forces /
// integrate in vmas_kernels.hip (tests/test_jit.py checks the two paths are bit-identical).
#pragma once

#include "vmas_physics.hpp"

namespace vmas {

// (pre_forces / integrate: vmas_physics.hpp, shared with k_step and the gradient path)

#ifndef __HIP_MEMORY_SCOPE_AGENT
#define __HIP_MEMORY_SCOPE_AGENT 4
#endif

// Sticky error bits of the device-side fixed point (vmas_jit.hip reads them back lazily).
// (kGridErrStateTimeout belonged to an earlier spin-waiting launch; no code sets it.)
constexpr uint32_t kGridErrNoConverge = 2u, kGridErrStateTimeout = 4u;

// Device-side fixed point of the batch-global broadphase (core.py:2796) in ONE persistent launch
// whose only cross-workgroup wait is for work that a RUNNING workgroup has claimed -- so nothing
// assumes that the workgroups of the launch are co-resident.
//
//   * Work items are the 64-env groups.  Group g is claimed for pass p by a compare-and-swap of
//     claim[g] from p to p + 1 (one word per group, each on its own 128-byte line: no contended
//     address).  A workgroup first claims its own groups (g = blockIdx.x + k * gridDim.x), then
//     scans the claim words for groups still unclaimed in this pass and steals them (normally
//     none: every workgroup has started long before the first one finishes).  Claims are never
//     taken back within a pass, so a scan that sees no unclaimed group proves that every group
//     is claimed: no claim counter (its adds, 64 per address at 32 768 envs, serialised at the
//     memory side and delayed the first group of every workgroup by 2-6 us).
//   * Processing a group ends with its R/Z activity row stored in blk[g] and one completion on a
//     two-level counter (shard g % 32, one 128-byte line each, then the top counter; cumulative
//     over the passes of a step).  The workgroup whose completion is the last of the
//     pass is the DECIDER: it ORs the rows, applies the k_jit_flags_reduce test (was the mask a
//     fixed point?), stores the next mask (inverted: zero means "all pairs active") and publishes
//     dec[p] = 2 | continue.
//   * A workgroup that finds nothing left to claim in pass p waits for dec[p].  Every group of
//     pass p is then claimed, and a group is claimed only by a workgroup that is executing, which
//     finishes it without waiting for anyone: the decision always comes, whichever workgroups
//     are resident (a workgroup that only becomes resident later finds every group claimed and
//     the decisions published, and follows them to the exit).
//   * The last workgroup to exit (exit counter == gridDim.x: nobody reads the control words any
//     more) resets claims, counters, decisions and the mask for the next step: no host memset,
//     so the step stays one capturable kernel node.
// Memory order (MI355X_MICROARCH.md, the sc1 hand-off forms): every byte handed between
// workgroups inside the launch -- activity rows, mask words, claims, counters, decisions -- is
// stored and loaded with agent-scope atomics (sc1: L1 bypassed, L2 dropped / written through);
// every storing wave waits for its stores (s_waitcnt 0) and the workgroup synchronises before
// lane 0 signals (a completion add, a decision store); a consumer loads only after its add
// returned last or its poll matched, and its other waves after a barrier.  No agent fences
// (1.7-6.5 us each on the critical path).  The step outputs are stored sc1 as well, so a group
// re-run in a later pass by a workgroup on another XCD never races a dirty line of the earlier
// pass: the earlier stores have completed (s_waitcnt) before the completion that precedes the
// decision that precedes the re-run.
//
// ctl (uint32), every counter shard on a 128-byte line of its own (the adds of hundreds of
// workgroups arriving together on one address serialise at the memory side: 32 shards):
// [0] top completion counter, [1] top exit counter, [2] passes run by the last step,
// [32 * (1 + k)] completion shard k (groups g % 32 == k, cumulative over the passes of a step),
// [32 * (33 + k)] exit shard k (workgroups blockIdx % 32 == k), [32 * 65 .. 32 * 73) unused,
// [32 * 73 + p] dec[p] (p < kGridMaxPasses); then the mask words (nwords) and the claim words
// (one per group, kClaimStride apart).
constexpr int kGridMaxPasses = 64, kGridShards = 32;
constexpr int kGridDone = 32, kGridExit = 32 * 33, kGridDec = 32 * 73;
constexpr int kGridCtlWords = kGridDec + kGridMaxPasses;

// Two-level sharded arrival: add one to shard (i % kGridShards) of `base`; the arrival that
// completes its shard adds one to the top counter; true for the arrival that completes the top
// (n arrivals per round, `round` rounds so far including this one).  One thread.
__device__ __forceinline__ bool sharded_arrive(uint32_t* shard0, uint32_t* top, uint32_t i, uint32_t n, uint32_t round) {
    const uint32_t k = i % kGridShards, n_k = (n + kGridShards - 1u - k) / kGridShards;
    const uint32_t n_top = n < (uint32_t)kGridShards ? n : (uint32_t)kGridShards;
    if (__hip_atomic_fetch_add(&shard0[32 * k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != n_k * round - 1u)
        return false;
    return __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_top * round - 1u;
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool cas_agent(uint32_t* p, uint32_t expect, uint32_t v) {
    return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
// step outputs, stored sc1 (write-through: no dirty copy stays in the XCD's L2)
__device__ __forceinline__ void st_out1(float* p, size_t i, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p) + i, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_out2(float* p, size_t i, V2 v) {
    const unsigned long long bits = (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p) + i, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Device timer (timing on, persistent launches): workgroup 0 stamps s_memrealtime into tm[0] at
// its start; the last workgroup to exit (grid_exit) adds (now - tm[0]) to tm[2] and counts the
// launch in tm[4] -- the launch's span bar the dispatch of workgroup 0 and the completion signal.
// Two stores per launch instead of per-workgroup atomics (measured: ~10 us on a 512-workgroup
// launch).  The last workgroup also adds its own s_memtime (shader clock) and s_memrealtime
// (100 MHz-class wall clock) spans to tm[5] / tm[6]: their ratio is the in-kernel shader clock
// (MI355X_MICROARCH.md, DVFS give-back item 6).
struct TimerStart {
    unsigned long long rt, sc;
};
__device__ __forceinline__ TimerStart device_timer_start(unsigned long long* tm, bool stamp_start) {
    TimerStart t{0ull, 0ull};
    if (tm && threadIdx.x == 0) {
        t.rt = __builtin_amdgcn_s_memrealtime();
        t.sc = __builtin_amdgcn_s_memtime();
        if (stamp_start && blockIdx.x == 0)
            __hip_atomic_store(&tm[0], t.rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return t;
}

// Sticky error bits: OR-ed into the device word, and the OR so far stored into the mapped host
// word (system scope, no fence: any nonzero value means failure), so the host sees a failure
// without a copy in the stream.
__device__ __forceinline__ void report_err(uint32_t* err, uint32_t* herr, uint32_t bit) {
    const uint32_t v = atomicOr(err, bit) | bit;
    if (herr) __hip_atomic_store(herr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Claim words: one per group, each on a 128-byte line of its own (the claims of hundreds of
// workgroups arriving together serialise per line at the memory side).
constexpr int kClaimStride = 32;

// Claim group g for pass `pass` (one thread): claim[g] p -> p + 1.  A workgroup's own groups are
// normally free: one compare-and-swap, no load first and no counter.
__device__ __forceinline__ bool grid_claim(uint32_t* claim, int g, int pass) {
    return cas_agent(&claim[(size_t)g * kClaimStride], (uint32_t)pass, (uint32_t)pass + 1u);
}

// Steal round (all threads): scan the claim words of `pass` and claim up to 64 groups still
// unclaimed.  LIST: 65 words of LDS; returns the number of entries in LIST[0..n) (an entry whose
// claim lost a race holds ~0u) and sets *seen when any unclaimed group was seen.  Claims are
// never taken back within a pass, so a scan that sees none unclaimed proves every group of the
// pass is claimed (by a running workgroup, which will complete it).
__device__ __forceinline__ int grid_steal(uint32_t* claim, int ngrp, int pass, uint32_t* LIST, bool* seen) {
    if (threadIdx.x == 0) LIST[64] = 0u;
    __syncthreads();
    for (int g = (int)threadIdx.x; g < ngrp; g += (int)blockDim.x) {
        uint32_t* w = &claim[(size_t)g * kClaimStride];
        if (ld_agent(w) != (uint32_t)pass) continue;
        const uint32_t i = atomicAdd(&LIST[64], 1u);  // reserve a slot before claiming
        if (i < 64u) LIST[i] = cas_agent(w, (uint32_t)pass, (uint32_t)pass + 1u) ? (uint32_t)g : ~0u;
    }
    __syncthreads();
    const uint32_t r = LIST[64];
    __syncthreads();
    *seen = r != 0u;
    return r < 64u ? (int)r : 64;
}

// Completion of group g in `pass` (all threads; the group's row and outputs are stored).
// Returns true in the workgroup that completed the pass (the decider).
__device__ __forceinline__ bool grid_complete(uint32_t* ctl, int g, int ngrp, int pass, uint32_t* FLAG) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's stores have completed
    __syncthreads();
    if (threadIdx.x == 0)
        *FLAG = sharded_arrive(&ctl[kGridDone], &ctl[0], (uint32_t)g, (uint32_t)ngrp, (uint32_t)(pass + 1)) ? 1u : 0u;
    __syncthreads();
    const bool last = *FLAG != 0u;
    __syncthreads();
    return last;
}

// The decider of pass `pass` (all threads): every group's row is in blk.  RED: 2 * nwords + 2
// words of LDS.  Returns true when the final pass did NOT converge (the caller then poisons the
// step's outputs with NaN, so that the bad step is visible in its own results; the sticky error
// bit also fails the next step).
__device__ inline bool grid_decide(const uint32_t* blk, uint32_t* nmask, uint32_t* ctl, uint32_t* err, uint32_t* herr,
                                   int nwords, int ngrp, int pass, int max_pass, uint32_t* RED) {
    const int nw2 = 2 * nwords;
    for (int w = threadIdx.x; w < nw2 + 2; w += blockDim.x) RED[w] = 0u;
    __syncthreads();
    {
        const int rows = ngrp, t = (int)threadIdx.x;
        if (nw2 <= (int)blockDim.x) {  // rows split over blockDim / nw2 thread groups per word
            const int per = (int)blockDim.x / nw2, w = t % nw2, g0 = t / nw2;
            if (g0 < per) {
                uint32_t r0 = 0u, r1 = 0u, r2 = 0u, r3 = 0u;  // independent loads in flight
                int i = g0;
                for (; i + 3 * per < rows; i += 4 * per) {
                    r0 |= ld_agent(&blk[(size_t)i * nw2 + w]);
                    r1 |= ld_agent(&blk[(size_t)(i + per) * nw2 + w]);
                    r2 |= ld_agent(&blk[(size_t)(i + 2 * per) * nw2 + w]);
                    r3 |= ld_agent(&blk[(size_t)(i + 3 * per) * nw2 + w]);
                }
                for (; i < rows; i += per) r0 |= ld_agent(&blk[(size_t)i * nw2 + w]);
                const uint32_t r = r0 | r1 | r2 | r3;
                if (r) atomicOr(&RED[w], r);
            }
        } else {
            for (int w = t; w < nw2; w += blockDim.x) {
                uint32_t r = 0u;
                for (int i = 0; i < rows; ++i) r |= ld_agent(&blk[(size_t)i * nw2 + w]);
                RED[w] = r;
            }
        }
    }
    __syncthreads();
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
        const uint32_t m = ~ld_agent(&nmask[w]), r = RED[w], z = RED[nwords + w];
        if ((m & ~r & z) | (~m & r)) atomicOr(&RED[nw2 + 1], 1u);
    }
    __syncthreads();
    const bool viol = RED[nw2 + 1] != 0u;
    const bool more = viol && pass + 1 < max_pass;
    if (more)
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) st_agent(&nmask[w], ~RED[w]);
    __builtin_amdgcn_s_waitcnt(0);  // the new mask words have completed before the publish
    __syncthreads();
    if (threadIdx.x == 0) {
        if (viol && !more) report_err(err, herr, kGridErrNoConverge);
        st_agent(&ctl[2], (uint32_t)(pass + 1));
        st_agent(&ctl[kGridDec + pass], more ? 3u : 2u);
    }
    __syncthreads();
    return viol && !more;
}

// Wait for the decision of `pass` (all threads): true when another pass follows.
__device__ __forceinline__ bool grid_wait(const uint32_t* ctl, int pass, uint32_t* FLAG) {
    if (threadIdx.x == 0) {
        uint32_t d;
        while ((d = ld_agent(&ctl[kGridDec + pass])) == 0u) __builtin_amdgcn_s_sleep(4);
        *FLAG = d;
    }
    __syncthreads();
    const bool more = (*FLAG & 1u) != 0u;
    __syncthreads();
    return more;
}

#ifdef VMAS_JIT_PROFILE_SLOTS
// profile builds: the per-workgroup record array (set by the kernel's prologue; 24 words per
// workgroup, csrc/vmas_jit.hip kProfRec)
__device__ unsigned long long* vmas_prof_blk;
#endif

// Per-workgroup cursor of the persistent launch (LDS; thread 0 writes it, behind barriers).
struct GridCursor {
    int pass, own, nl, il;
};

// The next group this workgroup processes, or -1 once the step is done (all threads).  Host-driven
// launches (persistent false): the workgroup's own groups.  Persistent launches: own groups
// claimed for the current pass, then the steal list, then steal rounds while a scan sees an
// unclaimed group, then the pass decision -- another pass restarts the cursor and
// reloads MSK from the (inverted) mask words.  Not inlined: its loop-invariant addresses would be
// hoisted around the group body and spill its registers (measured: +125 SGPR spills on balance).
__device__ __attribute__((noinline)) int grid_next(bool persistent, uint32_t* ctl, uint32_t* claim, const uint32_t* mask,
                                                   uint32_t* MSK, int nwords, int ngrp, GridCursor* CUR, uint32_t* QL) {
    GridCursor c = *CUR;
    int g = -1;
    for (;;) {
        if (c.own < ngrp) {
            const int own = c.own;
            c.own += (int)gridDim.x;
            if (!persistent) {
                g = own;
                break;
            }
#ifdef VMAS_JIT_PROFILE_SLOTS
            if (threadIdx.x == 0 && blockIdx.x < 4096u) vmas_prof_blk[blockIdx.x * 24 + 6] = __builtin_amdgcn_s_memrealtime();
#endif
            if (threadIdx.x == 0) QL[65] = grid_claim(claim, own, c.pass) ? 1u : 0u;
#ifdef VMAS_JIT_PROFILE_SLOTS
            if (threadIdx.x == 0 && blockIdx.x < 4096u) vmas_prof_blk[blockIdx.x * 24 + 7] = __builtin_amdgcn_s_memrealtime();
#endif
            __syncthreads();
            const bool mine = QL[65] != 0u;
            __syncthreads();
            if (mine) {
                g = own;
                break;
            }
        } else if (!persistent) {
            break;
        } else if (c.il < c.nl) {
            const uint32_t q = QL[c.il++];
            if (q != ~0u) {
                g = (int)q;
                break;
            }
        } else {
            bool seen;
            c.nl = grid_steal(claim, ngrp, c.pass, QL, &seen);
            c.il = 0;
            if (seen) continue;  // stolen groups in QL (or lost races: scan again)
            if (!grid_wait(ctl, c.pass, &QL[65])) break;
            ++c.pass;
            c.own = (int)blockIdx.x;
            c.nl = c.il = 0;
            for (int i = threadIdx.x; i < nwords; i += blockDim.x) MSK[i] = ~ld_agent(&mask[i]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *CUR = c;
    __syncthreads();
    return g;
}

// End of group g (all threads; persistent launches): its activity row FL into blk[g], the
// completion, and -- in the decider -- the pass decision.  Returns true when the step's final
// pass did not converge (the caller poisons the outputs).  Not inlined (see grid_next).
__device__ __attribute__((noinline)) bool grid_finish(int g, const uint32_t* FL, int nfl, uint32_t* blk, uint32_t* nmask,
                                                      uint32_t* ctl, uint32_t* err, uint32_t* herr, int nwords, int ngrp,
                                                      int pass, int max_pass, uint32_t* RED, uint32_t* FLAG) {
    __syncthreads();
    for (int i = threadIdx.x; i < nfl; i += blockDim.x) st_agent(&blk[(size_t)g * nfl + i], FL[i]);
    return grid_complete(ctl, g, ngrp, pass, FLAG) &&
           grid_decide(blk, nmask, ctl, err, herr, nwords, ngrp, pass, max_pass, RED);
}

// Exit (all threads): the last workgroup out resets the control words for the next step.
__device__ __forceinline__ void grid_exit(uint32_t* ctl, uint32_t* nmask, uint32_t* claim, int nwords, int ngrp,
                                          int max_pass, uint32_t* FLAG, unsigned long long* tm, TimerStart t0s) {
    __syncthreads();
    if (threadIdx.x == 0) *FLAG = sharded_arrive(&ctl[kGridExit], &ctl[1], blockIdx.x, gridDim.x, 1u) ? 1u : 0u;
    __syncthreads();
    if (*FLAG == 0u) return;
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) st_agent(&nmask[w], 0u);
    for (int g = threadIdx.x; g < ngrp; g += blockDim.x) st_agent(&claim[(size_t)g * kClaimStride], 0u);
    for (int p = threadIdx.x; p < max_pass; p += blockDim.x) st_agent(&ctl[kGridDec + p], 0u);
    const int t = (int)threadIdx.x;
    if (t < 2) st_agent(&ctl[t], 0u);
    if (t >= 64 && t < 64 + kGridShards) st_agent(&ctl[kGridDone + 32 * (t - 64)], 0u);
    if (t >= 128 && t < 128 + kGridShards) st_agent(&ctl[kGridExit + 32 * (t - 128)], 0u);
    if (tm && t == 0) {  // the launch's span: workgroup 0's start -> the last workgroup out
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        const unsigned long long t0 = __hip_atomic_load(&tm[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        (void)__hip_atomic_fetch_add(&tm[2], t1 > t0 ? t1 - t0 : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        (void)__hip_atomic_fetch_add(&tm[4], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c1 > t0s.sc && t1 > t0s.rt) {  // (thread 0 holds this workgroup's start stamps)
            (void)__hip_atomic_fetch_add(&tm[5], c1 - t0s.sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            (void)__hip_atomic_fetch_add(&tm[6], t1 - t0s.rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (threadIdx.x == 9) st_agent(&ctl[kGridExit], 0u);
}

}  // namespace vmas
