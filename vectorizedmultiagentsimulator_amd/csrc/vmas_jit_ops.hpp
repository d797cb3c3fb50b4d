// vmas_jit_ops.hpp -- per-entity force terms and integration for the world-specialised kernels
// (csrc/vmas_jit.hip, compiled by hipRTC).  Same operations, same order as pre_forces /
// integrate in vmas_kernels.hip (tests/test_jit.py checks the two paths are bit-identical).
#pragma once

#include "vmas_physics.hpp"
#include "vmas_tail.hpp"

namespace vmas {

// (pre_forces / integrate: vmas_physics.hpp, shared with k_step and the gradient path)

#ifndef __HIP_MEMORY_SCOPE_AGENT
#define __HIP_MEMORY_SCOPE_AGENT 4
#endif

// Sticky error bits of the device-side fixed point (vmas_jit.hip reads them back lazily):
// kGridErrNoConverge -- the fixed point did not converge within max_pass passes;
// kGridErrStateTimeout -- the final decider waited kGridStartWaitTicks for a workgroup of the
// launch to be dispatched (grid_decide).  Both NaN-poison the step's outputs.
constexpr uint32_t kGridErrNoConverge = 2u, kGridErrStateTimeout = 4u;
// Bound of the final decider's wait for the dispatcher, in s_memrealtime ticks (100 MHz): 10 s.
// Far above any real dispatch delay (a kernel of another stream holding the CUs for 0.5 s is
// tested), low enough that a stuck dispatch fails the step instead of hanging it.
constexpr unsigned long long kGridStartWaitTicks = 1000000000ull;

// Device-side fixed point of the batch-global broadphase (core.py:2796) in ONE persistent launch
// whose only cross-workgroup waits are for work that a RUNNING workgroup has claimed -- so nothing
// assumes that the workgroups of the launch are co-resident.
//
//   * Pass numbers are GLOBAL and only grow: a launch's first pass is E = ctl[kGridEpoch] (the
//     passes of every earlier step), and every per-pass word -- claims, completion counters,
//     the candidate word, decisions -- is compared against the global pass index G = E + p.
//     Nothing is ever reset: no exit counter and no reset work at the end of a launch.
//   * Work items are the 64-env groups.  Group g is claimed for pass G by a compare-and-swap of
//     claim[g] (u64) from G to G + 1 (one word per group, each on its own 128-byte line: no
//     contended address).  A workgroup first claims its own groups (g = blockIdx.x + k *
//     gridDim.x), then scans the claim words for groups still unclaimed in this pass and steals
//     them (normally none: every workgroup has started long before the first one finishes).
//     Claims are never taken back within a pass, so a scan that sees no unclaimed group proves
//     that every group is claimed: no claim counter (its adds, 64 per address at 32 768 envs,
//     serialised at the memory side and delayed the first group of every workgroup by 2-6 us).
//   * Processing a group ends with its R/Z activity row stored in blk[g]; a group whose OWN row
//     could break the fixed point (the k_jit_flags_reduce rule applied to its row alone: a
//     masked pair in range, or an active pair with an out-of-range force and no env of the
//     group in range) raises the candidate word to G + 1.  Then one completion on a two-level
//     counter (shard g % 32, one 128-byte line each, then the top counter; cumulative: n * (G + 1)
//     arrivals once pass G is complete).
//   * The workgroup whose completion is the last of the pass is the DECIDER.  A candidate word
//     below G + 1 proves the mask a fixed point without reading a row (the rule's violations
//     are ORs of per-group candidate bits: an in-range masked pair is one group's bit; an
//     out-of-range force with no env in range anywhere is a bit of the group that saw the force).
//     Otherwise it ORs the rows and applies the rule, and on a violation stores the next mask
//     (inverted: zero means "all pairs active").  It publishes dec[G % 64] = ((G + 1) << 1) |
//     continue.
//   * A workgroup that finds nothing left to claim in pass G waits for dec[G % 64].  Every group
//     of the pass is then claimed, and a group is claimed only by a workgroup that is executing,
//     which finishes it without waiting for anyone: the decision always comes, whichever
//     workgroups are resident (a workgroup that only becomes resident later finds every group
//     claimed and the decisions published, and follows them to the exit).
//   * The decider of the final pass then waits until every workgroup of the launch has read E
//     (a start counter sharded like the completions; a workgroup adds its start before its first
//     wait for a decision -- off its critical path -- and the decider counts itself), advances E
//     past the launch's passes and clears the mask if a re-run changed it.  The starts are
//     cumulative over launches, so the wait is for an ABSOLUTE count: the sum of the shards equal
//     to kGridStartBase (the starts of every earlier launch, advanced by each launch's final
//     decider) + gridDim.x.  (A per-shard residue test cannot tell a shard nobody has started
//     in from a full one.)  The wait is bounded (kGridStartWaitTicks): past it the step fails
//     with kGridErrStateTimeout and NaN outputs instead of hanging.  The decision is published before that wait, so every other
//     workgroup is leaving and the slots the remaining ones need are free: this wait is for the
//     dispatcher, never for another workgroup's progress.
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
// ctl (uint32 words; each 64-bit word on a 128-byte line of its own): [2] passes run by the last
// step (u32, read by the host); u64 words: kGridEpoch (E), kGridStartBase (starts of every
// earlier launch), kGridCand (candidate word), kGridTop
// (top completion counter), kGridDone + 32 * k (completion shard k: groups g % 32 == k),
// kGridDec + 2 * p (dec[p], contiguous), kGridStart + 32 * k (start shard k: workgroups
// blockIdx % 32 == k).  Then the mask words and, from the next multiple of 32 words, the claim
// words (u64, kClaimStride words apart).
constexpr int kGridMaxPasses = 64, kGridShards = 32;
constexpr int kGridEpoch = 32, kGridStartBase = 64, kGridCand = 96, kGridTop = 128, kGridDone = 160;
constexpr int kGridDec = kGridDone + 32 * kGridShards;
constexpr int kGridStart = kGridDec + 2 * kGridMaxPasses;
constexpr int kGridCtlWords = kGridStart + 32 * kGridShards;
static_assert(kGridCtlWords % 32 == 0, "mask words start on a 128-byte line");

// offset of the claim words from the mask words
__host__ __device__ constexpr long grid_claim_offset(long mask_words) { return (mask_words + 31) / 32 * 32; }

typedef unsigned long long u64;
__device__ __forceinline__ u64 ld64(const uint32_t* p) {
    return __hip_atomic_load(reinterpret_cast<const u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st64(uint32_t* p, u64 v) {
    __hip_atomic_store(reinterpret_cast<u64*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 add64(uint32_t* p, u64 v) {
    return __hip_atomic_fetch_add(reinterpret_cast<u64*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool cas64(uint32_t* p, u64 expect, u64 v) {
    return __hip_atomic_compare_exchange_strong(reinterpret_cast<u64*>(p), &expect, v, __ATOMIC_RELAXED,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Two-level cumulative arrival of group g at the end of global pass G (one thread): add one to
// shard g % kGridShards; the arrival that completes its shard's pass adds one to the top
// counter; true for the arrival that completes the top (the decider).
__device__ __forceinline__ bool grid_arrive(uint32_t* ctl, uint32_t g, uint32_t ngrp, u64 G) {
    const uint32_t k = g % kGridShards, n_k = (ngrp + kGridShards - 1u - k) / kGridShards;
    const uint32_t n_top = ngrp < (uint32_t)kGridShards ? ngrp : (uint32_t)kGridShards;
    if (add64(&ctl[kGridDone + 32 * k], 1ull) != (u64)n_k * (G + 1ull) - 1ull) return false;
    return add64(&ctl[kGridTop], 1ull) == (u64)n_top * (G + 1ull) - 1ull;
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
// its start; the decider of the step's final pass, once every workgroup has started, adds (now -
// tm[0]) to tm[2] and counts the launch in tm[4] (grid_time) -- the launch's span bar the
// dispatch of workgroup 0, the other workgroups' exit after the published decision and the
// completion signal.  Two stores per launch instead of per-workgroup atomics (measured: ~10 us
// on a 512-workgroup launch).  The decider also adds its own s_memtime (shader clock) and
// s_memrealtime (100 MHz-class wall clock) spans to tm[5] / tm[6]: their ratio is the in-kernel
// shader clock (MI355X_MICROARCH.md, DVFS give-back item 6).
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

// Claim group g for global pass G (one thread): claim[g] G -> G + 1.  A workgroup's own groups
// are normally free: one compare-and-swap, no load first and no counter.
__device__ __forceinline__ bool grid_claim(uint32_t* claim, int g, u64 G) {
    return cas64(&claim[(size_t)g * kClaimStride], G, G + 1ull);
}

// Steal round (all threads): scan the claim words of pass G and claim up to 64 groups still
// unclaimed.  LIST: 65 words of LDS; returns the number of entries in LIST[0..n) (an entry whose
// claim lost a race holds ~0u) and sets *seen when any unclaimed group was seen.  Claims are
// never taken back within a pass, so a scan that sees none unclaimed proves every group of the
// pass is claimed (by a running workgroup, which will complete it).
__device__ __forceinline__ int grid_steal(uint32_t* claim, int ngrp, u64 G, uint32_t* LIST, bool* seen) {
    if (threadIdx.x == 0) LIST[64] = 0u;
    __syncthreads();
    for (int g = (int)threadIdx.x; g < ngrp; g += (int)blockDim.x) {
        uint32_t* w = &claim[(size_t)g * kClaimStride];
        if (ld64(w) != G) continue;
        const uint32_t i = atomicAdd(&LIST[64], 1u);  // reserve a slot before claiming
        if (i < 64u) LIST[i] = cas64(w, G, G + 1ull) ? (uint32_t)g : ~0u;
    }
    __syncthreads();
    const uint32_t r = LIST[64];
    __syncthreads();
    *seen = r != 0u;
    return r < 64u ? (int)r : 64;
}

// This workgroup has read E (one thread; it read E and the mask words in the prologue): count
// it in start shard blockIdx % 32 (the final decider waits for every start before advancing E).
__device__ __forceinline__ void grid_started(uint32_t* ctl) {
    __builtin_amdgcn_s_waitcnt(0);  // (workgroup 0: its timer stamp has landed)
    (void)add64(&ctl[kGridStart + 32 * (int)(blockIdx.x % kGridShards)], 1ull);
}

// Starts counted so far over every launch (the first 64 threads; wave-uniform result): the sum
// of the start shards.
__device__ __forceinline__ u64 grid_starts(const uint32_t* ctl) {
    const uint32_t nsh = gridDim.x < (uint32_t)kGridShards ? gridDim.x : (uint32_t)kGridShards;
    u64 v = threadIdx.x < nsh ? ld64(&ctl[kGridStart + 32 * (int)threadIdx.x]) : 0ull;
    for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return __shfl(v, 0, 64);
}

// Completion of group g in global pass G (all threads; the group's row and outputs are stored).
// Returns true in the workgroup that completed the pass (the decider).
__device__ __forceinline__ bool grid_complete(uint32_t* ctl, int g, int ngrp, u64 G, uint32_t* FLAG) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's stores have completed
    __syncthreads();
    if (threadIdx.x == 0) *FLAG = grid_arrive(ctl, (uint32_t)g, (uint32_t)ngrp, G) ? 1u : 0u;
    __syncthreads();
    const bool last = *FLAG != 0u;
    __syncthreads();
    return last;
}

// The decider's timer update (see device_timer_start).
__device__ __forceinline__ void grid_time(unsigned long long* tm, TimerStart t0s) {
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

// Per-workgroup cursor of the persistent launch (LDS; thread 0 writes it, behind barriers):
// pass within the launch, next own group, steal list length / position, start counted,
// E of the launch.
struct GridCursor {
    int pass, own, nl, il, started;
    u64 base;
};

// Test knob (VMAS_JIT_TEST_PASSES=<n>, compiled into the generated source): every step runs at least
// n passes -- the decider treats the earlier passes as violated, with the mask re-derived from the
// rows as for a real violation -- so the re-run path (and a fused scenario program re-run after each
// pass, vmas_jit.hip epi_text) is exercised; the results must equal the one-pass step's.
#ifndef VMAS_GRID_MIN_PASSES
#define VMAS_GRID_MIN_PASSES 1
#endif

// The decider of global pass G = E + pass (all threads): every group's row is in blk and the
// pass's mask is MSK (LDS, 1 = active).  RED: 2 * nwords + 2 words of LDS.  Returns true when the
// final pass did NOT converge (the caller then poisons the step's outputs with NaN, so that the
// bad step is visible in its own results; the sticky error bit also fails the next step).
__device__ inline bool grid_decide(const uint32_t* blk, uint32_t* nmask, const uint32_t* MSK, uint32_t* ctl, uint32_t* err,
                                   uint32_t* herr, int nwords, int ngrp, u64 G, int pass, int max_pass, uint32_t* RED,
                                   unsigned long long* tm, TimerStart t0s, GridCursor* CUR) {
    const int nw2 = 2 * nwords;
    const bool force = pass + 1 < VMAS_GRID_MIN_PASSES;  // (test knob: another pass regardless)
    if (threadIdx.x == 0) RED[nw2] = (force || ld64(&ctl[kGridCand]) == G + 1ull) ? 1u : 0u;
    for (int w = threadIdx.x; w < nw2; w += blockDim.x) RED[w] = 0u;
    if (threadIdx.x == 0) RED[nw2 + 1] = 0u;
    __syncthreads();
    if (RED[nw2] != 0u) {  // some group's own bits could break the fixed point: OR the rows
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
        __syncthreads();
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
            const uint32_t m = MSK[w], r = RED[w], z = RED[nwords + w];
            if ((m & ~r & z) | (~m & r)) atomicOr(&RED[nw2 + 1], 1u);
        }
    }
    __syncthreads();
    const bool viol = RED[nw2 + 1] != 0u || force;
    const bool more = viol && pass + 1 < max_pass;
    if (more)
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) st_agent(&nmask[w], ~RED[w]);
    __builtin_amdgcn_s_waitcnt(0);  // the new mask words have completed before the publish
    __syncthreads();
    if (threadIdx.x == 0) {
        if (viol && !more) report_err(err, herr, kGridErrNoConverge);
        if (!more) st_agent(&ctl[2], (uint32_t)(pass + 1));
        st64(&ctl[kGridDec + 2 * (int)(G % (u64)kGridMaxPasses)], ((G + 1ull) << 1) | (more ? 1ull : 0ull));
    }
    if (!more) {  // the step's final pass: wait for every start, then advance E (see the header)
        const bool self = CUR->started != 0;
        if (threadIdx.x < 64) {
            const u64 base = ld64(&ctl[kGridStartBase]);
            const u64 want = base + (u64)gridDim.x - (self ? 0ull : 1ull);
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            bool late = false;
            while (grid_starts(ctl) != want) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > kGridStartWaitTicks) {
                    late = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
            if (threadIdx.x == 0) {
                st64(&ctl[kGridStartBase], base + (u64)gridDim.x);
                RED[nw2 + 1] = late ? 2u : (viol ? 1u : 0u);
            }
        }
        if (threadIdx.x == 0) {
            if (RED[nw2 + 1] == 2u) report_err(err, herr, kGridErrStateTimeout);
            st64(&ctl[kGridEpoch], G + 1ull);
            if (!self) {
                grid_started(ctl);
                CUR->started = 1;
            }
            if (tm) grid_time(tm, t0s);
        }
        __syncthreads();
        if (pass > 0)  // a re-run changed the mask: all pairs active again for the next step
            for (int w = threadIdx.x; w < nwords; w += blockDim.x) st_agent(&nmask[w], 0u);
    }
    __syncthreads();
    return RED[nw2 + 1] == 2u || (viol && !more);
}

// Wait for the decision of global pass G (all threads): true when another pass follows.  The
// workgroup's first wait counts its start first (*started).
__device__ __forceinline__ bool grid_wait(uint32_t* ctl, u64 G, uint32_t* FLAG, int* started) {
    if (threadIdx.x == 0) {
        if (!*started) grid_started(ctl);
        const uint32_t* dec = &ctl[kGridDec + 2 * (int)(G % (u64)kGridMaxPasses)];
        u64 d;
        while (((d = ld64(dec)) >> 1) != G + 1ull) __builtin_amdgcn_s_sleep(4);
        *FLAG = (uint32_t)(d & 1ull);
    }
    *started = 1;
    __syncthreads();
    const bool more = *FLAG != 0u;
    __syncthreads();
    return more;
}

#ifdef VMAS_JIT_PROFILE_SLOTS
// profile builds: the per-workgroup record array (set by the kernel's prologue; 24 words per
// workgroup, csrc/vmas_jit.hip kProfRec)
__device__ unsigned long long* vmas_prof_blk;
#endif

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
            if (threadIdx.x == 0) QL[65] = grid_claim(claim, own, c.base + (u64)c.pass) ? 1u : 0u;
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
            c.nl = grid_steal(claim, ngrp, c.base + (u64)c.pass, QL, &seen);
            c.il = 0;
            if (seen) continue;  // stolen groups in QL (or lost races: scan again)
            if (!grid_wait(ctl, c.base + (u64)c.pass, &QL[65], &c.started)) break;
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

// End of group g (all threads; persistent launches): its activity row FL into blk[g], its
// candidate bits (see the header), the completion, and -- in the decider -- the pass decision.
// Returns true when the step's final pass did not converge (the caller poisons the outputs).
// Not inlined (see grid_next).
__device__ __attribute__((noinline)) bool grid_finish(int g, const uint32_t* FL, int nfl, uint32_t* blk, uint32_t* nmask,
                                                      const uint32_t* MSK, uint32_t* ctl, uint32_t* err, uint32_t* herr,
                                                      int nwords, int ngrp, GridCursor* CUR, int max_pass,
                                                      uint32_t* RED, uint32_t* FLAG, unsigned long long* tm,
                                                      unsigned long long t0_rt, unsigned long long t0_sc) {
    const TimerStart t0s{t0_rt, t0_sc};
    __syncthreads();
    const int pass = CUR->pass;
    const u64 G = CUR->base + (u64)pass;
    for (int i = threadIdx.x; i < nfl; i += blockDim.x) st_agent(&blk[(size_t)g * nfl + i], FL[i]);
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
        const uint32_t m = MSK[w], r = FL[w], z = FL[nwords + w];
        if ((m & ~r & z) | (~m & r))
            (void)__hip_atomic_fetch_max(reinterpret_cast<u64*>(&ctl[kGridCand]), G + 1ull, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    }
    return grid_complete(ctl, g, ngrp, G, FLAG) &&
           grid_decide(blk, nmask, MSK, ctl, err, herr, nwords, ngrp, G, pass, max_pass, RED, tm, t0s, CUR);
}

}  // namespace vmas
