// vmas_programs.hpp -- scenario per-step programs as per-env device functions: balance
// (balance.py:205-262) and transport (transport.py:130-190), shared by the library kernels
// k_balance / k_transport (vmas_scenarios.hip) and a world module's k_program_jit and k_world
// epilogue (vmas_jit.hip).  Their arithmetic is IEEE in any translation unit (xdiv / xsqrt below),
// so the library launch, the module's launch in an eager step and a replay whose k_world runs the
// program as its epilogue (vmas_graph_chain_build) give the same bits -- the reference's.
//
// Also the small helpers every fused scenario kernel uses (direct outputs, strided vector loads,
// torch.remainder).
#pragma once

#include "vmas_mi355x.h"
#include "vmas_query.hpp"

namespace vmas {

__device__ __forceinline__ V2 ld_vec2(const VmasVec& v, int b) {
    return mk(v.p[(long)b * v.s0], v.p[(long)b * v.s0 + v.s1]);
}
__device__ __forceinline__ float ld_vec1(const VmasVec& v, int b) { return v.p[(long)b * v.s0]; }

// torch.remainder(a, b) for floating point (ATen's remainder kernel): fmod, moved into the sign
// of the divisor
__device__ __forceinline__ float torch_remainder(float a, float b) {
    float mod = fmodf(a, b);
    if ((mod != 0.f) && ((b < 0.f) != (mod < 0.f))) mod = mod + b;
    return mod;
}

// Graph mode's direct outputs (simulator/environment/_graph.py DirectOutputs): the byte offsets from
// the captured step's obs / rewards / done buffers to this replay's fresh output tensors, written by
// the previous post-replay launch; out_delta NULL (every eager launch): in place.
struct OutDelta {
    long long obs, rew, done;
};
template <class IO>
__device__ __forceinline__ OutDelta load_out_delta(const IO& io) {
    OutDelta o{0, 0, 0};
    if (io.out_delta) {
        o.obs = io.out_delta[0];
        o.rew = io.out_delta[1];
        o.done = io.out_delta[2];
    }
    return o;
}
template <class T>
__device__ __forceinline__ T* moved(T* p, long long d) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(p) + d);
}
// A store written through to memory (sc1): an output that graph mode carries or copies after the
// replay -- in a fused launch its tail (vmas_tail.hpp) does that inside the same launch, possibly on
// another XCD, loading the value at agent scope.  The same value as a plain store.
__device__ __forceinline__ void st_wt(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<unsigned int*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt8(uint8_t* p, uint8_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- flag-independent IEEE arithmetic ---------------------------------------------------------------
// A world module is compiled with the relaxed options (-fno-hip-fp32-correctly-rounded-divide-sqrt,
// -fapprox-func; vmas_jit.hip codegen_flags), under which `/` and sqrtf are ~1-ulp approximations.
// The scenario programs below must give the reference's fp32 results bit for bit in any
// translation unit (the library's k_balance, a module's k_program_jit and its k_world epilogue), so
// they divide and take square roots through these: the correctly rounded sequences LLVM itself
// emits for fp32 fdiv / sqrt on gfx9 with denormals on (HIP's mode), spelled with the builtins the
// options do not touch.  tests/test_fused.py checks the programs bit for bit against the reference's
// torch program (eager and replayed); test_exact_math_gpu checks these against IEEE `/` and sqrtf.
__device__ __forceinline__ float xdiv(float a, float b) {
    bool num_scaled, den_scaled;
    const float d = __builtin_amdgcn_div_scalef(a, b, false, &den_scaled);  // the scaled denominator
    const float n = __builtin_amdgcn_div_scalef(a, b, true, &num_scaled);   // the scaled numerator
    const float r = __builtin_amdgcn_rcpf(d);
    const float e0 = __builtin_fmaf(-d, r, 1.0f);
    const float r1 = __builtin_fmaf(e0, r, r);
    const float q0 = n * r1;
    const float e1 = __builtin_fmaf(-d, q0, n);
    const float q1 = __builtin_fmaf(e1, r1, q0);
    const float e2 = __builtin_fmaf(-d, q1, n);
    return __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(e2, r1, q1, num_scaled), b, a);
}
__device__ __forceinline__ float xsqrt(float x) {
    const bool scale = x < 0x1.0p-96f;  // (v_sqrt_f32 is 1 ulp on normal inputs)
    const float sx = scale ? x * 0x1.0p+32f : x;
    float s = __builtin_amdgcn_sqrtf(sx);
    const float dn = __int_as_float(__float_as_int(s) - 1), up = __int_as_float(__float_as_int(s) + 1);
    const float vp = __builtin_fmaf(-dn, s, sx), vs = __builtin_fmaf(-up, s, sx);
    s = vp <= 0.f ? dn : s;
    s = vs > 0.f ? up : s;
    s = scale ? s * 0x1.0p-16f : s;
    return (sx == 0.f || sx == __builtin_huge_valf()) ? sx : s;
}
__device__ __forceinline__ float xnorm(V2 v) { return xsqrt(v.x * v.x + v.y * v.y); }

// physics._get_closest_points_line_line (physics.py:143-218) with IEEE division / norms; otherwise
// the operations of vmas_physics.hpp closest_points_line_line, in its order
__device__ __forceinline__ void xclosest_points_line_line(Seg l1, Seg l2, V2* out1, V2* out2) {
    const V2 xy1 = mk(l1.half * l1.dir.x, l1.half * l1.dir.y);
    const V2 xy2 = mk(l2.half * l2.dir.x, l2.half * l2.dir.y);
    const V2 a1 = l1.p + xy1, a2 = l1.p - xy1;
    const V2 b1 = l2.p + xy2, b2 = l2.p - xy2;
    const V2 r = a2 - a1, s = b2 - b1;
    const V2 qp = b1 - a1;
    const float cqpr = cross(qp, r), cqps = cross(qp, s), crs = cross(r, s);
    const float u = xdiv(cqpr, crs), t = xdiv(cqps, crs);
    const bool cond = (crs != 0.f) && (0.f <= u) && (u <= 1.f) && (0.f <= t) && (t <= 1.f);
    const V2 a1b = closest_point_line(l2.p, l2.dir, l2.half, a1, true);
    const V2 a2b = closest_point_line(l2.p, l2.dir, l2.half, a2, true);
    const V2 b1a = closest_point_line(l1.p, l1.dir, l1.half, b1, true);
    const V2 b2a = closest_point_line(l1.p, l1.dir, l1.half, b2, true);
    V2 c1 = mk(INFINITY, INFINITY), c2 = mk(INFINITY, INFINITY);
    float md = INFINITY, d;
    d = xnorm(a1 - a1b);
    if (d < md) { md = d; c1 = a1; c2 = a1b; }
    d = xnorm(a2 - a2b);
    if (d < md) { md = d; c1 = a2; c2 = a2b; }
    d = xnorm(b1a - b1);
    if (d < md) { md = d; c1 = b1a; c2 = b1; }
    d = xnorm(b2a - b2);
    if (d < md) { md = d; c1 = b2a; c2 = b2; }
    if (cond) {
        const V2 pi = a1 + r * t;
        c1 = pi;
        c2 = pi;
    }
    *out1 = c1;
    *out2 = c2;
}
// cos / sin of rot and of rot + pi / 2 (physics.py:299-301) with the library functions
__device__ __forceinline__ Trig xtrig(float rot) {
    const float r2 = rot + kHalfPi;
    return Trig{cosf(rot), sinf(rot), cosf(r2), sinf(r2)};
}
// physics._get_closest_point_box (physics.py:262-294): first strict minimum over the 4 sides
__device__ __forceinline__ V2 xclosest_point_box(V2 pos, Trig t, float hl, float hw, V2 tp) {
    V2 best = mk(INFINITY, INFINITY);
    float bd = INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const Seg sd = box_side(pos, t, hl, hw, i);
        const V2 p = closest_point_line(sd.p, sd.dir, sd.half, tp, true);
        const float d = xnorm(tp - p);
        if (d < bd) {
            bd = d;
            best = p;
        }
    }
    return best;
}
// is_overlapping for (box, sphere) (core.py:1932-1963)
__device__ __forceinline__ bool xoverlap_box_sphere(const VmasShapeRef& bx, const VmasShapeRef& sp, int b) {
    const V2 pb = ref_pos(bx, b), ps = ref_pos(sp, b);
    const V2 cp = xclosest_point_box(pb, xtrig(ref_rot(bx, b)), bx.length * 0.5f, bx.width * 0.5f, ps);
    const float dsc = xnorm(ps - cp), dsb = xnorm(ps - pb), dcb = xnorm(pb - cp);
    return (dsb < dcb) || (dsc < sp.radius_lmd);
}
// get_distance of two spheres (core.py:1821-1830): |pa - pb| - r_a - r_b
__device__ __forceinline__ float xdist_spheres(const VmasShapeRef& a, const VmasShapeRef& c, int b) {
    return (xnorm(ref_pos(a, b) - ref_pos(c, b)) - a.radius) - c.radius;
}

// ---- the programs ------------------------------------------------------------------------------------
// Each function takes its argument block as a template IO: `const VmasBalanceIO&` through the k_world
// epilogue's pointer, or -- in the kernels that receive it by value (k_balance, k_transport,
// k_program_jit) -- the block read in place from the kernel argument segment (VMAS_PROGRAM_ARGS; a
// loop indexing the by-value parameter's arrays copies the whole block to scratch).  Structs are
// copied out of it before they meet the non-template helpers.
#ifdef __HIP_DEVICE_COMPILE__
#define VMAS_PROGRAM_ARGS(T, name)                                                                  \
    const T __attribute__((address_space(4)))& io =                                                 \
        *(const T __attribute__((address_space(4)))*)__builtin_amdgcn_kernarg_segment_ptr();        \
    (void)name
#else
#define VMAS_PROGRAM_ARGS(T, name) const T& io = name
#endif

// ---- balance (balance.py:205-262; restated in scenarios/balance.py) -------------------------------
// Q: kBalQRows rows of 64 floats: [0, 16) side s of closest_line_box(floor, line) as (q1.x, q1.y,
// q2.x, q2.y); [16, 28) side s of closest_point_box(floor, package.pos) as (p.x, p.y, |pos - p|).
// The four sides of both are computed by four waves in parallel; the first strict minimum over
// them, in side order, is taken after the barrier (the reference's selection order).
constexpr int kBalQRows = 28;
__device__ __forceinline__ float* bal_q(float* Q, int row) { return Q + row * 64; }

// Where the program reads the step's state.  Every launch outside k_world: the argument block's
// tensors.  As k_world's epilogue (vmas_jit.hip epi_text): the LDS rows k_world already holds the
// group's integrated state in (positions, rotations, velocities; a row index per field, -1 = read
// the tensor), found by comparing the argument block's pointers with k_world's own output / input
// tensors -- the same fp32 values, without the round trip to HBM that re-reading the step's just
// written (write-through) outputs costs.
enum BalField {
    kBalPkgPos, kBalGoalPos, kBalLinePos, kBalFloorPos, kBalLineRot, kBalFloorRot, kBalPkgVel, kBalLineVel,
    kBalLineAng, kBalAgPos, kBalAgVel = kBalAgPos + VMAS_SCN_MAX_AGENTS, kBalFields = kBalAgVel + VMAS_SCN_MAX_AGENTS
};
struct BalRows {
    const float* L;  // the row buffer ([row][lane], 64 floats per row)
    const int* row;  // kBalFields row indices
    int lane;
};
template <class IO>
__device__ __forceinline__ V2 bal_v2(IO& io, const BalRows* s, int f, int b) {
    if (s) {
        const int r = __builtin_amdgcn_readfirstlane(s->row[f]);  // (one value for the workgroup)
        if (r >= 0) return mk(s->L[r * 64 + s->lane], s->L[(r + 1) * 64 + s->lane]);
    }
    switch (f) {
        case kBalPkgPos: { const VmasShapeRef x = io.package; return ref_pos(x, b); }
        case kBalGoalPos: { const VmasShapeRef x = io.goal; return ref_pos(x, b); }
        case kBalLinePos: { const VmasShapeRef x = io.line; return ref_pos(x, b); }
        case kBalFloorPos: { const VmasShapeRef x = io.floor; return ref_pos(x, b); }
        case kBalPkgVel: { const VmasVec v = io.package_vel; return ld_vec2(v, b); }
        case kBalLineVel: { const VmasVec v = io.line_vel; return ld_vec2(v, b); }
        default:
            if (f >= kBalAgVel) { const VmasVec v = io.agent_vel[f - kBalAgVel]; return ld_vec2(v, b); }
            { const VmasVec v = io.agent_pos[f - kBalAgPos]; return ld_vec2(v, b); }
    }
}
template <class IO>
__device__ __forceinline__ float bal_f1(IO& io, const BalRows* s, int f, int b) {
    if (s) {
        const int r = __builtin_amdgcn_readfirstlane(s->row[f]);
        if (r >= 0) return s->L[r * 64 + s->lane];
    }
    switch (f) {
        case kBalLineRot: { const VmasShapeRef x = io.line; return ref_rot(x, b); }
        case kBalFloorRot: { const VmasShapeRef x = io.floor; return ref_rot(x, b); }
        default: { const VmasVec v = io.line_ang_vel; return ld_vec1(v, b); }
    }
}

// side `side` of both box queries, env bb
template <class IO>
__device__ __forceinline__ void bal_side(IO& io, int bb, int side, int lane, float* Q, const BalRows* src = nullptr) {
    const VmasShapeRef fl = io.floor, ln = io.line;
    const float rb = bal_f1(io, src, kBalLineRot, bb);
    const V2 pf = bal_v2(io, src, kBalFloorPos, bb);
    const Trig tf = xtrig(bal_f1(io, src, kBalFloorRot, bb));
    const Seg sd = box_side(pf, tf, fl.length * 0.5f, fl.width * 0.5f, side);
    Pts q;
    xclosest_points_line_line(sd, Seg{bal_v2(io, src, kBalLinePos, bb), mk(cosf(rb), sinf(rb)), ln.length * 0.5f}, &q.p1,
                              &q.p2);
    bal_q(Q, 4 * side + 0)[lane] = q.p1.x;
    bal_q(Q, 4 * side + 1)[lane] = q.p1.y;
    bal_q(Q, 4 * side + 2)[lane] = q.p2.x;
    bal_q(Q, 4 * side + 3)[lane] = q.p2.y;
    const V2 ps = bal_v2(io, src, kBalPkgPos, bb);  // closest_point_box (physics.py:262-294), this side's candidate
    const V2 p = closest_point_line(sd.p, sd.dir, sd.half, ps, true);
    bal_q(Q, 16 + 3 * side + 0)[lane] = p.x;
    bal_q(Q, 16 + 3 * side + 1)[lane] = p.y;
    bal_q(Q, 16 + 3 * side + 2)[lane] = xnorm(ps - p);
}

// done = on_the_ground + is_overlapping(package, goal)
template <class IO>
__device__ __forceinline__ void bal_done(IO& io, int b, bool og, const OutDelta& od, const BalRows* src = nullptr) {
    const VmasShapeRef pk = io.package, gl = io.goal;
    // xdist_spheres' arithmetic: (|pa - pb| - r_a) - r_b
    const float d = (xnorm(bal_v2(io, src, kBalPkgPos, b) - bal_v2(io, src, kBalGoalPos, b)) - pk.radius) - gl.radius;
    moved(io.done, od.done)[b] = (og || d < 0.f) ? 1 : 0;
}

// (an A/B knob of the package / floor preload: -DVMAS_BAL_PRELOAD_POS=0 through VMAS_JIT_CFLAGS)
#ifndef VMAS_BAL_PRELOAD_POS
#define VMAS_BAL_PRELOAD_POS 1
#endif
// wave 0's own inputs of the reward block, loaded before the barrier (their latency under the
// four waves' box queries instead of after them): the previous shaping, the goal, package and
// floor positions
struct BalPre {
    float gs;
    V2 goal, pkg, pf;
};
template <class IO>
__device__ __forceinline__ BalPre bal_preload(IO& io, int bb, const BalRows* src = nullptr) {
    return BalPre{io.global_shaping[(long)bb * io.gs_s0], bal_v2(io, src, kBalGoalPos, bb), bal_v2(io, src, kBalPkgPos, bb),
                  bal_v2(io, src, kBalFloorPos, bb)};
}

// The reward block of env b from the sides in Q: closest_line_box's and closest_point_box's
// first strict minima over the sides in order, compute_on_the_ground, the package-goal distance,
// ground / position rewards, the global shaping update, every agent's reward; then done.
template <class IO>
__device__ __forceinline__ void bal_reward(IO& io, int b, int lane, const OutDelta& od, float* Q, const BalPre& pre) {
    V2 c1 = mk(INFINITY, INFINITY), c2 = mk(INFINITY, INFINITY), cp = mk(INFINITY, INFINITY);
    float bd = INFINITY, bp = INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const V2 q1 = mk(bal_q(Q, 4 * i)[lane], bal_q(Q, 4 * i + 1)[lane]);
        const V2 q2 = mk(bal_q(Q, 4 * i + 2)[lane], bal_q(Q, 4 * i + 3)[lane]);
        const float d = xnorm(q1 - q2);
        if (d < bd) {
            bd = d;
            c1 = q1;
            c2 = q2;
        }
        const float dp = bal_q(Q, 16 + 3 * i + 2)[lane];
        if (dp < bp) {
            bp = dp;
            cp = mk(bal_q(Q, 16 + 3 * i)[lane], bal_q(Q, 16 + 3 * i + 1)[lane]);
        }
    }
    const VmasShapeRef pk = io.package;
#if VMAS_BAL_PRELOAD_POS
    const V2 pkg = pre.pkg, goal = pre.goal, pf = pre.pf;  // (b == bb: wave 0's valid lanes only)
#else
    const V2 pkg = ref_pos(pk, b), goal = pre.goal, pf = ref_pos(io.floor, b);
#endif
    // compute_on_the_ground: is_overlapping(line, floor) + is_overlapping(package, floor)
    // (canonical (box, line) / (box, sphere) branches, core.py:1932-1968)
    const float dsc = xnorm(pkg - cp), dsb = xnorm(pkg - pf), dcb = xnorm(pf - cp);
    const bool og = (xnorm(c1 - c2) - kLineMinDist < 0.f) || (dsb < dcb) || (dsc < pk.radius_lmd);
    io.on_the_ground[b] = og ? 1 : 0;
    const float dist = xnorm(pkg - goal);  // vector_norm(package.pos - goal.pos, dim=1)
    io.package_dist[b] = dist;
    const float ground = og ? io.fall_reward : 0.f;  // zeros, masked_fill_(on_the_ground, fall)
    st_wt(io.ground_rew + b, ground);  // (ground_rew, global_shaping, pos_rew: copied after the replay)
    const float gs = dist * io.shaping_factor;
    const float pos_rew = pre.gs - gs;
    st_wt(io.global_shaping_out + b, gs);
    if (io.pos_rew_prev) io.pos_rew_prev[b] = 0.f;  // pos_rew[:] = 0 on the tensor being replaced
    st_wt(io.pos_rew + b, pos_rew);
    const float r = ground + pos_rew;  // reward(agent) = ground_rew + pos_rew
    for (int i = 0; i < io.n_agents; ++i) moved(io.rewards[i], od.rew)[b] = r;
    if (io.what & VMAS_SCN_DONE) {  // bal_done on the loaded positions (xdist_spheres' arithmetic)
        const VmasShapeRef gl = io.goal;
        moved(io.done, od.done)[b] = (og || (xnorm(pkg - goal) - pk.radius) - gl.radius < 0.f) ? 1 : 0;
    }
}

// agent i's 16-entry observation in env b
template <class IO>
__device__ __forceinline__ void bal_obs(IO& io, int b, int i, const OutDelta& od, const BalRows* src = nullptr) {
    const V2 pkg = bal_v2(io, src, kBalPkgPos, b), goal = bal_v2(io, src, kBalGoalPos, b);
    const V2 lpos = bal_v2(io, src, kBalLinePos, b), pv = bal_v2(io, src, kBalPkgVel, b), lv = bal_v2(io, src, kBalLineVel, b);
    const float law = bal_f1(io, src, kBalLineAng, b);
    const float lrot = torch_remainder(bal_f1(io, src, kBalLineRot, b), io.pi);
    const V2 pg = pkg - goal;
    const V2 p = bal_v2(io, src, kBalAgPos + i, b), v = bal_v2(io, src, kBalAgVel + i, b);
    const V2 dp = p - pkg, dl = p - lpos;
    float4* dst = reinterpret_cast<float4*>(moved(io.obs[i], od.obs) + (long)b * 16);
    dst[0] = make_float4(p.x, p.y, v.x, v.y);
    dst[1] = make_float4(dp.x, dp.y, dl.x, dl.y);
    dst[2] = make_float4(pg.x, pg.y, pv.x, pv.y);
    dst[3] = make_float4(lv.x, lv.y, law, lrot);
}

// The whole program for 64-env group g, by every thread of a workgroup of nwave >= 5 waves (a
// barrier inside): waves 0-3 the four box sides, waves 4.. the observations, then wave 0 the
// reward block and done.  Q: kBalQRows x 64 floats of LDS.
template <class IO>
__device__ __forceinline__ void balance_group(IO& io, int g, int wave, int nwave, int lane, float* Q,
                                              const BalRows* src = nullptr) {
    const int b = g * 64 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    const OutDelta od = load_out_delta(io);
    const bool rew = io.what & VMAS_SCN_REWARD;
    const BalPre pre = rew && wave == 0 ? bal_preload(io, bb, src) : BalPre{0.f, mk(0.f, 0.f), mk(0.f, 0.f), mk(0.f, 0.f)};
    if (rew && wave < 4) bal_side(io, bb, wave, lane, Q, src);
    if ((io.what & VMAS_SCN_OBS) && wave >= 4 && valid)
        for (int i = wave - 4; i < io.n_agents; i += nwave - 4) bal_obs(io, b, i, od, src);
    __syncthreads();
    if (wave != 0 || !valid) return;
    if (rew) bal_reward(io, b, lane, od, Q, pre);
    else if (io.what & VMAS_SCN_DONE) bal_done(io, b, io.on_the_ground[b] != 0, od, src);
}

// ---- transport (transport.py:130-190; restated in scenarios/transport.py) -------------------------
// The reward (every package) and done of env b
template <class IO>
__device__ __forceinline__ void tr_reward_done(IO& io, int b, const OutDelta& od) {
    const int np = io.n_packages;
    bool all_on = true;
    if (io.what & VMAS_SCN_REWARD) {
        float rew = 0.f;  // self.rew = zeros
#pragma unroll 1  // (one copy of the box-sphere test: compiled into k_world too)
        for (int i = 0; i < np; ++i) {
            const VmasShapeRef pk = io.package[i], gl = io.goal[i];
            const float dist = xnorm(ref_pos(pk, b) - ref_pos(gl, b));
            const bool on = xoverlap_box_sphere(pk, gl, b);
            // (dist_to_goal, on_goal, colour, global_shaping: carried after the replay, written through)
            st_wt(io.dist_to_goal[i] + b, dist);
            st_wt8(io.on_goal[i] + b, on ? 1 : 0);
            float* col = io.color[i] + (long)b * 3;  // where(on_goal, green, red)
            st_wt(col, on ? io.green[0] : io.red[0]);
            st_wt(col + 1, on ? io.green[1] : io.red[1]);
            st_wt(col + 2, on ? io.green[2] : io.red[2]);
            const float shaping = dist * io.shaping_factor;
            rew = rew + (on ? 0.f : io.global_shaping[i][(long)b * io.gs_s0[i]] - shaping);
            st_wt(io.global_shaping_out[i] + b, shaping);
            all_on = all_on && on;
        }
        moved(io.rew, od.rew)[b] = rew;
    } else if (io.what & VMAS_SCN_DONE) {
        for (int i = 0; i < np; ++i) all_on = all_on && io.on_goal_in[i][b] != 0;
    }
    if (io.what & VMAS_SCN_DONE) moved(io.done, od.done)[b] = all_on ? 1 : 0;  // all(stack(on_goal), -1)
}

// agent a's observation in env b.  With REWARD in the same launch on_goal is recomputed
// (is_overlapping, deterministic) rather than read back from the reward's output.
template <class IO>
__device__ __forceinline__ void tr_obs(IO& io, int b, int a, const OutDelta& od) {
    const int np = io.n_packages;
    const VmasVec apv = io.agent_pos[a], avv = io.agent_vel[a];
    const V2 p = ld_vec2(apv, b), v = ld_vec2(avv, b);
    float* o = moved(io.obs[a], od.obs) + (long)b * (4 + 7 * np);
    o[0] = p.x;
    o[1] = p.y;
    o[2] = v.x;
    o[3] = v.y;
#pragma unroll 1  // (one copy of the box-sphere test: compiled into k_world too)
    for (int i = 0; i < np; ++i) {
        const VmasShapeRef pk = io.package[i], gl = io.goal[i];
        const VmasVec pvv = io.package_vel[i];
        const V2 pp = ref_pos(pk, b), gp = ref_pos(gl, b), pv = ld_vec2(pvv, b);
        const bool on = (io.what & VMAS_SCN_REWARD) ? xoverlap_box_sphere(pk, gl, b) : io.on_goal_in[i][b] != 0;
        float* q = o + 4 + 7 * i;
        q[0] = pp.x - gp.x;
        q[1] = pp.y - gp.y;
        q[2] = pp.x - p.x;
        q[3] = pp.y - p.y;
        q[4] = pv.x;
        q[5] = pv.y;
        q[6] = on ? 1.f : 0.f;
    }
}

// The whole program for 64-env group g by a workgroup of nwave >= 2 waves: wave 0 the reward and
// done, the other waves the observations (no barrier inside).
template <class IO>
__device__ __forceinline__ void transport_group(IO& io, int g, int wave, int nwave, int lane) {
    const int b = g * 64 + lane;
    if (b >= io.batch) return;
    const OutDelta od = load_out_delta(io);
    if (wave == 0) {
        if (io.what & (VMAS_SCN_REWARD | VMAS_SCN_DONE)) tr_reward_done(io, b, od);
    } else if (io.what & VMAS_SCN_OBS) {
        for (int a = wave - 1; a < io.n_agents; a += nwave - 1) tr_obs(io, b, a, od);
    }
}

}  // namespace vmas
