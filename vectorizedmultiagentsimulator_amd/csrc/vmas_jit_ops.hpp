// vmas_jit_ops.hpp -- per-entity force terms and integration for the world-specialised kernels
// (csrc/vmas_jit.hip, compiled by hipRTC).  Same operations, same order as pre_forces /
// integrate in vmas_kernels.hip (tests/test_jit.py checks the two paths are bit-identical).
#pragma once

#include "vmas_physics.hpp"

namespace vmas {

// Action force/torque clamps + friction + gravity of one entity (core.py:1994-2003, 2017-2101).
// af/at: the agent's current state.force/torque, updated in place (the reference writes the
// clamped value back to agent.state.force each substep).
__device__ __forceinline__ void pre_forces(const VmasEntityDesc& d, bool is_agent, V2& af, float& at, V2 vel,
                                           float w, V2 eg, bool has_eg, float gx, float gy, bool has_g,
                                           float sdt, float& fx, float& fy, float& tq) {
    fx = 0.f;
    fy = 0.f;
    tq = 0.f;
    const bool mov = d.flags & VMAS_F_MOVABLE, rotb = d.flags & VMAS_F_ROTATABLE;
    if (is_agent) {
        if (mov) {  // _apply_action_force (core.py:2017-2027)
            V2 f = af;
            if (d.flags & VMAS_F_MAX_F) f = clamp_with_norm(f, d.max_f);
            if (d.flags & VMAS_F_F_RANGE) f = mk(tclamp(f.x, -d.f_range, d.f_range), tclamp(f.y, -d.f_range, d.f_range));
            af = f;
            fx = fx + f.x;
            fy = fy + f.y;
        }
        if (rotb) {  // _apply_action_torque (core.py:2029-2040)
            float t = at;
            if (d.flags & VMAS_F_MAX_T) t = clamp_with_norm1(t, d.max_t);
            if (d.flags & VMAS_F_T_RANGE) t = tclamp(t, -d.t_range, d.t_range);
            at = t;
            tq = tq + t;
        }
    }
    if (d.flags & VMAS_F_LIN_FRIC) {  // _apply_friction_force (core.py:2053-2101)
        const V2 f = friction2(vel, d.lin_fric, d.mass, sdt);
        fx = fx + f.x;
        fy = fy + f.y;
    }
    if (d.flags & VMAS_F_ANG_FRIC) tq = tq + friction1(w, d.ang_fric, d.inertia, sdt);
    if (mov) {  // _apply_gravity (core.py:2042-2051)
        if (has_g) {
            fx = fx + d.mass * gx;
            fy = fy + d.mass * gy;
        }
        if (has_eg) {
            fx = fx + d.mass * eg.x;
            fy = fy + d.mass * eg.y;
        }
    }
}

// _integrate_state (core.py:2859-2907)
__device__ __forceinline__ void integrate(const VmasEntityDesc& d, int substep, float sdt, float fx, float fy,
                                          float tq, bool has_xs, float xs, bool has_ys, float ys, V2& p, V2& v,
                                          float& rot, float& w) {
    if (d.flags & VMAS_F_MOVABLE) {
        if (substep == 0) v = mk(v.x * d.one_minus_drag, v.y * d.one_minus_drag);
        const V2 acc = mk(fx / d.mass, fy / d.mass);
        v = mk(v.x + acc.x * sdt, v.y + acc.y * sdt);
        if (d.flags & VMAS_F_MAX_SPEED) v = clamp_with_norm(v, d.max_speed);
        if (d.flags & VMAS_F_V_RANGE) v = mk(tclamp(v.x, -d.v_range, d.v_range), tclamp(v.y, -d.v_range, d.v_range));
        V2 np = mk(p.x + v.x * sdt, p.y + v.y * sdt);
        if (has_xs) np.x = tclamp(np.x, -xs, xs);
        if (has_ys) np.y = tclamp(np.y, -ys, ys);
        p = np;
    }
    if (d.flags & VMAS_F_ROTATABLE) {
        if (substep == 0) w = w * d.one_minus_drag;
        w = w + (tq / d.inertia) * sdt;
        rot = rot + w * sdt;
    }
}

#ifndef __HIP_MEMORY_SCOPE_AGENT
#define __HIP_MEMORY_SCOPE_AGENT 4
#endif

// Sticky error bits of the device-side fixed point (vmas_jit.hip reads them back lazily).
// (kGridErrStateTimeout belonged to the former spin-waiting persistent launch; no code sets it.)
constexpr uint32_t kGridErrNoConverge = 2u, kGridErrStateTimeout = 4u;

// Device-side fixed point of the batch-global broadphase as a RELAY of launches, with no
// workgroup ever waiting for another (so nothing assumes that the workgroups of a launch are
// co-resident).  The step enqueues L launches on one stream: pass 0 (k_world) and passes
// 1..L-1 (k_world_rerun).  Every launch is an ordinary grid over the 64-env groups:
//   * each workgroup stores the OR of its R/Z activity words in blk[blockIdx.x] ([2][nwords])
//     and arrives on a two-level counter;
//   * the LAST workgroup to arrive ORs every row, applies the k_jit_flags_reduce test (was the
//     mask a fixed point?) and publishes the decision in ctl[1] = (epoch << 8 | (pass+1) << 1 |
//     continue), with the next mask (stored inverted, so zero means "all pairs active");
//   * a rerun launch reads ctl[1] first and exits at once unless the previous pass asked for it.
// Stream order between the launches is the only synchronisation: a launch starts after the
// previous one has completed, with its memory visible (kernel-boundary release / acquire).
// ctl: [0] top arrival counter, [1] published word, [2] passes run, [3] launch epoch, [32 * (1 +
// k)] arrival counter of the workgroups with blockIdx % 8 == k (one 128-byte line each: 512
// arrivals on one address serialise at the memory side).  No host memset: the final pass's
// reducer, which runs after every workgroup of the step has arrived, clears the counters and the
// mask words for the next step and advances the epoch, which keeps the previous step's
// published word from being read as this step's.
//
// Why no spin-wait any more (the former single persistent launch): its waiting workgroups needed
// every workgroup of the grid resident at once, which a plain launch does not guarantee (a kernel
// of another stream or process holding CUs delays some workgroups; the resident ones then spun
// until their bound and the step completed with a non-fixed-point mask).  The relay has no such
// assumption.  The graph-replay timeouts seen with a memset node in front of the persistent
// kernel are consistent with the same cause: the waits could only time out if an arrival never
// came, i.e. a workgroup of the grid was not running (or its counter increment was zeroed by a
// memset that had not completed when the first workgroups arrived).  Neither can stall a relay.
//
// RED: workgroup LDS of 2 * nwords + 2 words.  Returns true in the reducer of a final pass that
// did NOT converge (the caller then poisons the step's outputs with NaN, so that the bad step is
// visible in its own results; the sticky error bit also fails the next step).
constexpr int kGridCtlWords = 32 * 9;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Device timer (timing on, persistent launches): workgroup 0 stamps s_memrealtime into tm[0] at
// its start; the final pass's reducer -- the last workgroup to arrive, after which every
// workgroup only reads the published word and exits -- adds (now - tm[0]) to tm[2] and counts
// the launch in tm[4].  Two stores per launch instead of per-workgroup atomics (measured: ~10 us
// on a 512-workgroup launch).  The reducer also adds its own s_memtime (shader clock) and
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

// Whether a rerun launch of pass `pass` (>= 1) was requested by the previous pass of this step.
__device__ __forceinline__ bool relay_requested(const uint32_t* ctl, uint32_t epoch, int pass) {
    return ld_agent(&ctl[1]) == (((epoch & 0xFFFFFFu) << 8) | ((uint32_t)pass << 1) | 1u);
}

// Sticky error bits: OR-ed into the device word, and the OR so far stored into the mapped host
// word (system scope, no fence: any nonzero value means failure), so the host sees a failure
// without a copy in the stream.
__device__ __forceinline__ void report_err(uint32_t* err, uint32_t* herr, uint32_t bit) {
    const uint32_t v = atomicOr(err, bit) | bit;
    if (herr) __hip_atomic_store(herr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline bool relay_arrive(const uint32_t* blk, uint32_t* nmask, uint32_t* ctl, uint32_t* err, uint32_t* herr,
                                    int nwords, int pass, int max_pass, uint32_t* RED, uint32_t epoch,
                                    unsigned long long* tm, TimerStart t0s) {
    const uint32_t tag = ((epoch & 0xFFFFFFu) << 8) | ((uint32_t)(pass + 1) << 1);
    const uint32_t G = gridDim.x, k = blockIdx.x & 7u;
    const uint32_t n_k = (G + 7u - k) / 8u, n_sub = G < 8u ? G : 8u;  // workgroups in sub-counter k
    const int nw2 = 2 * nwords;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's blk stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        bool last = false;
        if (add_agent(&ctl[32 * (1 + k)], 1u) == n_k * (uint32_t)(pass + 1) - 1u)
            last = add_agent(&ctl[0], 1u) == n_sub * (uint32_t)(pass + 1) - 1u;
        RED[nw2] = last ? 1u : 0u;
    }
    __syncthreads();
    const bool reducer = RED[nw2] != 0u;
    __syncthreads();
    if (!reducer) return false;  // nothing to wait for: the next launch reads the decision
    // the reducer: every row has arrived
    for (int w = threadIdx.x; w < nw2 + 2; w += blockDim.x) RED[w] = 0u;
    __syncthreads();
    {
        const int rows = (int)G, t = (int)threadIdx.x;
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
        st_agent(&ctl[1], tag | (more ? 1u : 0u));
    }
    if (!more) {  // the final pass: every workgroup of the step has arrived; reset for the next step
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) st_agent(&nmask[w], 0u);
        if (threadIdx.x == 0) st_agent(&ctl[0], 0u);
        if (threadIdx.x >= 1 && threadIdx.x <= 8) st_agent(&ctl[32 * threadIdx.x], 0u);
        if (threadIdx.x == 9) st_agent(&ctl[3], epoch + 1u);
        if (tm && threadIdx.x == 0) {  // (thread 0 holds this workgroup's start stamps)
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long c1 = __builtin_amdgcn_s_memtime();
            const unsigned long long t0 = __hip_atomic_load(&tm[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            (void)__hip_atomic_fetch_add(&tm[2], t1 > t0 ? t1 - t0 : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            (void)__hip_atomic_fetch_add(&tm[4], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c1 > t0s.sc && t1 > t0s.rt) {
                (void)__hip_atomic_fetch_add(&tm[5], c1 - t0s.sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                (void)__hip_atomic_fetch_add(&tm[6], t1 - t0s.rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    return viol && !more;
}

}  // namespace vmas
