// vmas_physics.hpp -- scalar fp32 physics of one environment, compiled for both gfx950 (kernels in
// vmas_kernels.hip) and the host (the device == -1 backend in the same translation unit).
//
// Every function restates a PyTorch op sequence of the reference in the same left-to-right order
// and with the same fp32 roundings (python scalars are cast to fp32 before they meet a tensor, as
// torch's wrapped-number promotion does), so that with -ffp-contract=off the only differences
// from torch-CPU are the last-ulp differences of sin/cos/exp/log1p/sqrt-of-reductions.
// Citations are file:line in the reference checkout.
#pragma once

// Under hipRTC (the world-specialised step kernels of csrc/vmas_jit.hip) the HIP runtime, device
// math and fixed-width integer types are provided by the runtime compiler itself.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#else
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
#ifndef INFINITY
#define INFINITY __builtin_huge_valf()
#endif
#endif

#include "../../include/vmas_mi355x.h"

#define VHD __host__ __device__ __forceinline__

// The scalar type is a parameter: Real = float everywhere the step runs; the gradient path
// (csrc/vmas_grad.hip) includes this header once more, in its own namespace, with Real = a
// forward-mode dual number (value + tangents), so that the derivatives follow exactly the
// operations, branches and selections of the forward step.
#ifndef VMAS_PHYS_NS
#define VMAS_PHYS_NS vmas
#define VMAS_PHYS_REAL float
#endif

namespace VMAS_PHYS_NS {

using Real = VMAS_PHYS_REAL;

// utils.py:27 LINE_MIN_DIST = 4 / 6e2, as the f32 value torch uses when it meets a f32 tensor
constexpr float kLineMinDist = (float)(4.0 / 6e2);
constexpr float kHalfPi = (float)(3.141592653589793 / 2.0);  // torch.pi / 2 -> f32

struct V2 {
    Real x, y;
};
VHD V2 mk(Real x, Real y) { return V2{x, y}; }
VHD V2 operator+(V2 a, V2 b) { return V2{a.x + b.x, a.y + b.y}; }
VHD V2 operator-(V2 a, V2 b) { return V2{a.x - b.x, a.y - b.y}; }
VHD V2 operator-(V2 a) { return V2{-a.x, -a.y}; }
VHD V2 operator*(V2 a, Real s) { return V2{a.x * s, a.y * s}; }
VHD V2 operator*(Real s, V2 a) { return V2{s * a.x, s * a.y}; }
VHD V2 operator/(V2 a, Real s) { return V2{a.x / s, a.y / s}; }

// torch.linalg.vector_norm(v, dim=-1) of a length-2 vector
VHD Real norm(V2 v) { return sqrtf(v.x * v.x + v.y * v.y); }
// TorchUtils.cross (utils.py:194-197): a.x*b.y - a.y*b.x
VHD Real cross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
// torch.sign: (0 < x) - (x < 0); NaN -> 0
VHD Real tsign(Real x) { return Real((float)((0.f < x) - (x < 0.f))); }
// torch.minimum / torch.maximum / torch.min(dim) / torch.max(dim): NaN propagating.  Relaxed
// builds (the world-specialised kernels) use gfx950's v_minimum3_f32 / v_maximum3_f32 (IEEE 754-2019
// minimum / maximum: NaN propagating, one instruction instead of three compares and three selects);
// they differ from the selects only in the sign of a zero result of comparing +0 with -0.
#ifdef VMAS_PHYS_RELAXED
VHD Real tmin(Real a, Real b) { return __builtin_elementwise_minimum(a, b); }
VHD Real tmax(Real a, Real b) { return __builtin_elementwise_maximum(a, b); }
#else
VHD Real tmin(Real a, Real b) { return (a != a) ? a : ((b != b) ? b : (a < b ? a : b)); }
VHD Real tmax(Real a, Real b) { return (a != a) ? a : ((b != b) ? b : (a > b ? a : b)); }
#endif
// torch.clamp(x, lo, hi).  Its backward passes the gradient where lo <= x <= hi, bounds
// included; the gradient build (VMAS_PHYS_GRAD, csrc/vmas_grad.hip) keeps x itself there so a value
// sitting exactly on a bound (an action clamped last step) carries its tangent as torch's does.
#ifdef VMAS_PHYS_GRAD
VHD Real tclamp(Real x, Real lo, Real hi) { return (x >= lo && x <= hi) ? x : tmin(tmax(x, lo), hi); }
#else
VHD Real tclamp(Real x, Real lo, Real hi) { return tmin(tmax(x, lo), hi); }
#endif

// Transcendentals.  Relaxed builds (VMAS_PHYS_RELAXED: the world-specialised kernels of jointless
// worlds, csrc/vmas_jit.hip relaxed_math) use the hardware instructions: v_sin/v_cos_f32 for the
// entity trig and Kahan's log1p(y) = log(u) * y / (u - 1), u = 1 + y, with v_log_f32 for the
// soft-contact penetration (y = exp(-|x|) in (0, 1]) -- a few ulp instead of ocml's
// double-float log1pf (~110 VALU instructions per contact) and its range-reduced sin/cos
// (~100 each).  Every other build keeps the correctly rounded library functions.
#ifdef VMAS_PHYS_RELAXED
// v_sin / v_cos_f32 take revolutions: the x * (1 / 2 pi) product rounds to |x| * 2^-24 rad (1e-6
// rad at 16 rad) and the instructions' domain ends at 256 revolutions.  The reference never wraps
// an entity's rotation (core.py:2907), so a spinning body's angle grows without bound: the
// argument is first reduced by 2 pi (Cody-Waite, 2 pi as three floats, fused multiply-adds, so
// no product k * C is ever rounded; the first part has 8 significant bits, which makes x - k * C1
// exact), branch-free.  |x| < pi gives k = 0 and r = x exactly: the same value as the unreduced
// instruction.  Range (host emulation of these three steps against the double-precision remainder
// of the float angle, 2e4 angles per magnitude): |sin error| <= 2.3e-7 up to 1e7 rad,
// 4.4e-7 at 1e8 rad, 6.8e-6 at 1e9 rad (where the third part's truncation shows) --
// tests/test_fused.py::test_relaxed_trig_large_rotation_gpu runs bodies turned by up to 1e6 rad.  (Round 4's lane-divergent branch to the library sin / cos beyond 16 rad
// kept the library's Payne-Hanek code and its registers in every world's kernel: +10 VGPRs and
// +12.5 % VALU instructions per balance launch)
#ifdef VMAS_TRIG_GUARD
VHD Real tsin(Real x) { return fabsf(x) < 16.f ? __sinf(x) : sinf(x); }
VHD Real tcos(Real x) { return fabsf(x) < 16.f ? __cosf(x) : cosf(x); }
#else
VHD Real red2pi(Real x) {
    const Real k = rintf(x * 0x1.45f306p-3f);
    Real r = __builtin_fmaf(-k, 6.28125f, x);
    r = __builtin_fmaf(-k, 0x1.fb5444p-10f, r);
    return __builtin_fmaf(-k, 0x1.68c234p-37f, r);
}
VHD Real tsin(Real x) { return __sinf(red2pi(x)); }
VHD Real tcos(Real x) { return __cosf(red2pi(x)); }
#endif
VHD Real tlog1p(Real y) {
    const Real u = 1.f + y;
    return u == 1.f ? y : __logf(u) * (y / (u - 1.f));
}
#else
VHD Real tsin(Real x) { return sinf(x); }
VHD Real tcos(Real x) { return cosf(x); }
VHD Real tlog1p(Real y) { return log1pf(y); }
#endif

// Angle trig of one entity: cos/sin(rot) and cos/sin(rot + pi/2) (physics.py:299-301)
struct Trig {
    Real c0, s0, c1, s1;
};
VHD Trig make_trig(Real rot) {
    const Real r2 = rot + kHalfPi;
    return Trig{tcos(rot), tsin(rot), tcos(r2), tsin(r2)};
}
// Lines and joint anchors only use cos/sin(rot); boxes also use the side normal rot + pi/2.
VHD Trig make_trig_for(Real rot, bool box) {
    if (box) return make_trig(rot);
    return Trig{tcos(rot), tsin(rot), 0.f, 0.f};
}

// Wave-uniform vote used for exact early-outs: on gfx950 true iff the predicate holds in every
// active lane of the wave (so a skipped computation is skipped for all of them); on the host
// backend (one environment at a time) it is the predicate itself.
__device__ __forceinline__ bool vote_all(bool b) { return __all(b); }
__host__ __forceinline__ bool vote_all(bool b) { return b; }

// TorchUtils.clamp_with_norm (utils.py:168-173)
VHD V2 clamp_with_norm(V2 t, Real max_norm) {
    const Real n = norm(t);
    const V2 nt = (t / n) * max_norm;
    return (n > max_norm) ? nt : t;
}
VHD Real clamp_with_norm1(Real t, Real max_norm) {  // [B,1] variant: norm = |t|
    const Real n = fabsf(t);
    const Real nt = (t / n) * max_norm;
    return (n > max_norm) ? nt : t;
}

// torch.logaddexp(0, x) (ATen logaddexp kernel: m + log1p(exp(-|a-b|)))
VHD Real logaddexp0(Real x) {
    const Real m = tmax(0.f, x);
    return m + tlog1p(expf(-fabsf(0.f - x)));
}

// World._get_constraint_forces (core.py:2804-2838).  Returns the force on a; b gets -force.
// `sc` = f32(sign * force_multiplier) (a python Real product), `k` = f32(contact_margin).
VHD V2 constraint_force(V2 pa, V2 pb, Real dmin, Real sc, Real k, bool attractive) {
    const V2 delta = pa - pb;
    const Real dist = norm(delta);
    // The reference zeroes the force where dist < 1e-6 or (repulsive) dist > dmin /
    // (attractive) dist < dmin; when that holds in every lane the softplus is not needed.
    const bool zero = (dist < 1e-6f) || (attractive ? (dist < dmin) : (dist > dmin));
    if (vote_all(zero)) return mk(0.f, 0.f);
    const Real x = attractive ? (-(dmin - dist)) / k : (dmin - dist) / k;  // (dmin-dist)*sign/k
    const Real pen = logaddexp0(x) * k;
    const Real dsafe = (dist > 0.f) ? dist : 1e-8f;
    V2 f = mk(((sc * delta.x) / dsafe) * pen, ((sc * delta.y) / dsafe) * pen);
    if (dist < 1e-6f) f = mk(0.f, 0.f);
    if (!attractive) {
        if (dist > dmin) f = mk(0.f, 0.f);
    } else {
        if (dist < dmin) f = mk(0.f, 0.f);
    }
    return f;
}

// physics._get_closest_point_line (physics.py:399-428); dir = (cos, sin) of the line rot.
VHD V2 closest_point_line(V2 lp, V2 dir, Real half, V2 tp, bool limit) {
    const V2 d = lp - tp;
    const Real dot = d.x * dir.x + d.y * dir.y;
    const Real sg = tsign(dot);
    const Real dfc = limit ? tmin(fabsf(dot), half) : fabsf(dot);
    const Real m = sg * dfc;
    return lp - dir * m;
}

// One side of a box as a line (physics._get_all_lines_box, physics.py:297-324)
struct Seg {
    V2 p;       // centre
    V2 dir;     // (cos, sin) of the side's rot
    Real half; // half length
};
VHD Seg box_side(V2 pos, Trig t, Real hl, Real hw, int i) {
    const V2 rv = mk(t.c0, t.s0);
    const V2 rv2 = mk(t.c1, t.s1);
    switch (i) {
        case 0: return Seg{pos + rv * hl, rv2, hw};
        case 1: return Seg{pos - rv * hl, rv2, hw};
        case 2: return Seg{pos + rv2 * hw, rv, hl};
        default: return Seg{pos - rv2 * hw, rv, hl};
    }
}

// physics._get_closest_point_box (physics.py:262-294): first strict minimum over the 4 sides.
VHD V2 closest_point_box(V2 pos, Trig t, Real hl, Real hw, V2 tp) {
    V2 best = mk(INFINITY, INFINITY);
    Real bd = INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const Seg s = box_side(pos, t, hl, hw, i);
        const V2 p = closest_point_line(s.p, s.dir, s.half, tp, true);
        const Real d = norm(tp - p);
        if (d < bd) {
            bd = d;
            best = p;
        }
    }
    return best;
}

// physics._get_inner_point_box (physics.py:12-22)
VHD V2 inner_point_box(V2 outside, V2 surface, V2 box_pos, Real* dmag) {
    const V2 v = surface - outside;
    const V2 u = box_pos - surface;
    const Real vn = norm(v);
    Real xm = (v.x * u.x + v.y * u.y) / vn;
    V2 x = (v / vn) * xm;
    if (vn == 0.f) {
        x = surface;  // reference quirk: x = surface_point when v_norm == 0
        xm = 0.f;
    }
    *dmag = fabsf(xm);
    return surface + x;
}

// physics._get_closest_points_line_line (physics.py:143-218) incl. _get_line_extrema and
// _get_intersection_point_line_line (physics.py:131-140, 221-259).  Line 1 = (p1,dir1,h1).
VHD void closest_points_line_line(Seg l1, Seg l2, V2* out1, V2* out2) {
    const V2 xy1 = mk(l1.half * l1.dir.x, l1.half * l1.dir.y);
    const V2 xy2 = mk(l2.half * l2.dir.x, l2.half * l2.dir.y);
    const V2 a1 = l1.p + xy1, a2 = l1.p - xy1;  // line 1 extrema
    const V2 b1 = l2.p + xy2, b2 = l2.p - xy2;  // line 2 extrema
    // intersection
    const V2 r = a2 - a1, s = b2 - b1;
    const V2 qp = b1 - a1;
    const Real cqpr = cross(qp, r), cqps = cross(qp, s), crs = cross(r, s);
    const Real u = cqpr / crs, t = cqps / crs;
    const bool cond = (crs != 0.f) && (0.f <= u) && (u <= 1.f) && (0.f <= t) && (t <= 1.f);
    // end points projected on the other segment
    const V2 a1b = closest_point_line(l2.p, l2.dir, l2.half, a1, true);
    const V2 a2b = closest_point_line(l2.p, l2.dir, l2.half, a2, true);
    const V2 b1a = closest_point_line(l1.p, l1.dir, l1.half, b1, true);
    const V2 b2a = closest_point_line(l1.p, l1.dir, l1.half, b2, true);
    V2 c1 = mk(INFINITY, INFINITY), c2 = mk(INFINITY, INFINITY);
    Real md = INFINITY, d;
    d = norm(a1 - a1b);
    if (d < md) { md = d; c1 = a1; c2 = a1b; }
    d = norm(a2 - a2b);
    if (d < md) { md = d; c1 = a2; c2 = a2b; }
    d = norm(b1a - b1);
    if (d < md) { md = d; c1 = b1a; c2 = b1; }
    d = norm(b2a - b2);
    if (d < md) { md = d; c1 = b2a; c2 = b2; }
    if (cond) {
        const V2 pi = a1 + r * t;  // p + t * r
        c1 = pi;
        c2 = pi;
    }
    *out1 = c1;
    *out2 = c2;
}

// physics._get_closest_line_box (physics.py:327-381): returns (point on box, point on line)
VHD void closest_line_box(V2 bpos, Trig bt, Real hl, Real hw, Seg line, V2* pbox, V2* pline) {
    V2 c1 = mk(INFINITY, INFINITY), c2 = mk(INFINITY, INFINITY);
    Real bd = INFINITY;
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        V2 q1, q2;
        closest_points_line_line(box_side(bpos, bt, hl, hw, i), line, &q1, &q2);
        const Real d = norm(q1 - q2);
        if (d < bd) {
            bd = d;
            c1 = q1;
            c2 = q2;
        }
    }
    *pbox = c1;
    *pline = c2;
}

// physics._get_closest_box_box (physics.py:25-128): (point on A, point on B)
VHD void closest_box_box(V2 pa, Trig ta, Real hla, Real hwa, V2 pb, Trig tb, Real hlb,
                         Real hwb, V2* out_a, V2* out_b) {
    V2 c1 = mk(INFINITY, INFINITY), c2 = mk(INFINITY, INFINITY);
    Real bd = INFINITY;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        V2 p1, p2;
        if (i < 4) {  // side i of A vs box B: closest_line_box(B, sideA) -> (on B, on A side)
            closest_line_box(pb, tb, hlb, hwb, box_side(pa, ta, hla, hwa, i), &p2, &p1);
        } else {      // box A vs side j of B: closest_line_box(A, sideB) -> (on A, on B side)
            closest_line_box(pa, ta, hla, hwa, box_side(pb, tb, hlb, hwb, i - 4), &p1, &p2);
        }
        const Real d = norm(p1 - p2);
        if (d < bd) {
            bd = d;
            c1 = p1;
            c2 = p2;
        }
    }
    *out_a = c1;
    *out_b = c2;
}

// ---------------------------------------------------------------------------------------------
// Pair narrowphases.  Result convention: force on entity a (entity b receives exactly -fa, as
// _get_constraint_forces returns (force, -force)), torque on a, torque on b.
struct PairOut {
    V2 fa;
    Real ta, tb;
};

struct Body {  // one entity's state in one env plus its static shape numbers
    V2 p, v;
    Real rot, w;
};

struct WorldK {  // f32 world constants used by the narrowphases
    float k;     // contact_margin
    float c;     // collision_force
    float cj;    // joint_force
    float ct;    // torque_constraint_force
};

// _sphere_sphere_vectorized_collision (core.py:2293-2338)
VHD PairOut pair_ss(V2 pa, V2 pb, Real dmin, const WorldK& w) {
    return PairOut{constraint_force(pa, pb, dmin, w.c, w.k, false), 0.f, 0.f};
}

// _sphere_line_vectorized_collision (core.py:2340-2391); a = line, b = sphere
VHD PairOut pair_ls(V2 pl, Trig tl, Real hl, V2 ps, Real dmin, const WorldK& w) {
    const V2 cp = closest_point_line(pl, mk(tl.c0, tl.s0), hl, ps, true);
    const V2 fs = constraint_force(ps, cp, dmin, w.c, w.k, false);
    const V2 fl = -fs;
    const V2 r = cp - pl;
    return PairOut{fl, cross(r, fl), 0.f};
}

// _line_line_vectorized_collision (core.py:2393-2456)
VHD PairOut pair_ll(V2 pa, Trig ta, Real hla, V2 pb, Trig tb, Real hlb, Real dmin,
                    const WorldK& w) {
    V2 qa, qb;
    closest_points_line_line(Seg{pa, mk(ta.c0, ta.s0), hla}, Seg{pb, mk(tb.c0, tb.s0), hlb}, &qa, &qb);
    const V2 fa = constraint_force(qa, qb, dmin, w.c, w.k, false);
    const V2 fb = -fa;
    return PairOut{fa, cross(qa - pa, fa), cross(qb - pb, fb)};
}

// _box_sphere_vectorized_collision (core.py:2458-2551); a = box, b = sphere
VHD PairOut pair_bs(V2 pbx, Trig tbx, Real hl, Real hw, bool hollow, V2 ps, Real dmin_rl,
                    const WorldK& w) {
    const V2 cpb = closest_point_box(pbx, tbx, hl, hw, ps);
    V2 inner = cpb;
    Real d = 0.f;
    if (!hollow) inner = inner_point_box(ps, cpb, pbx, &d);
    const V2 fs = constraint_force(ps, inner, dmin_rl + d, w.c, w.k, false);
    const V2 fb = -fs;
    return PairOut{fb, cross(cpb - pbx, fb), 0.f};
}

// Box-line / box-box narrowphases split into independent parts (one box side / one
// side-vs-box test each) plus a finish step, so that several waves can evaluate one pair.  The
// finish step replays the reference's "first strict minimum" selection over the parts in order,
// hence split and fused evaluation are bit-identical.
struct Pts {
    V2 p1, p2;
};
VHD Pts bl_part(V2 pbx, Trig tbx, Real hl, Real hw, V2 pl, Trig tl, Real hll, int side) {
    Pts r;
    closest_points_line_line(box_side(pbx, tbx, hl, hw, side), Seg{pl, mk(tl.c0, tl.s0), hll}, &r.p1, &r.p2);
    return r;
}
VHD Pts bb_part(V2 pa, Trig ta, Real hla, Real hwa, V2 pb, Trig tb, Real hlb, Real hwb, int i) {
    Pts r;
    if (i < 4) closest_line_box(pb, tb, hlb, hwb, box_side(pa, ta, hla, hwa, i), &r.p2, &r.p1);
    else closest_line_box(pa, ta, hla, hwa, box_side(pb, tb, hlb, hwb, i - 4), &r.p1, &r.p2);
    return r;
}
template <class PartFn>
VHD Pts select_min(int n, PartFn part) {
    Pts best{mk(INFINITY, INFINITY), mk(INFINITY, INFINITY)};
    Real bd = INFINITY;
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
        const Pts q = part(i);
        const Real d = norm(q.p1 - q.p2);
        if (d < bd) {
            bd = d;
            best = q;
        }
    }
    return best;
}
VHD PairOut bl_finish(V2 pbx, bool hollow, V2 pl, Pts q, Real dmin, const WorldK& w) {
    const V2 pb = q.p1, plp = q.p2;
    V2 inner = pb;
    Real d = 0.f;
    if (!hollow) inner = inner_point_box(plp, pb, pbx, &d);
    const V2 fbox = constraint_force(inner, plp, dmin + d, w.c, w.k, false);
    const V2 fline = -fbox;
    return PairOut{fbox, cross(pb - pbx, fbox), cross(plp - pl, fline)};
}
VHD PairOut bb_finish(V2 pa, bool hol_a, V2 pb, bool hol_b, Pts q, Real dmin, const WorldK& w) {
    const V2 qa = q.p1, qb = q.p2;
    V2 ia = qa, ib = qb;
    Real da = 0.f, db = 0.f;
    if (!hol_a) ia = inner_point_box(qb, qa, pa, &da);
    if (!hol_b) ib = inner_point_box(qa, qb, pb, &db);
    const V2 fa = constraint_force(ia, ib, (da + db) + dmin, w.c, w.k, false);
    const V2 fb = -fa;
    return PairOut{fa, cross(qa - pa, fa), cross(qb - pb, fb)};
}

// _box_line_vectorized_collision (core.py:2553-2652); a = box, b = line
VHD PairOut pair_bl(V2 pbx, Trig tbx, Real hl, Real hw, bool hollow, V2 pl, Trig tl, Real hll,
                    Real dmin, const WorldK& w) {
    const Pts q = select_min(4, [&](int i) { return bl_part(pbx, tbx, hl, hw, pl, tl, hll, i); });
    return bl_finish(pbx, hollow, pl, q, dmin, w);
}

// _box_box_vectorized_collision (core.py:2654-2785)
VHD PairOut pair_bb(V2 pa, Trig ta, Real hla, Real hwa, bool hol_a, V2 pb, Trig tb, Real hlb,
                    Real hwb, bool hol_b, Real dmin, const WorldK& w) {
    const Pts q = select_min(8, [&](int i) { return bb_part(pa, ta, hla, hwa, pb, tb, hlb, hwb, i); });
    return bb_finish(pa, hol_a, pb, hol_b, q, dmin, w);
}

// TorchUtils.rotate_vector (utils.py:176-191) with precomputed cos/sin of the angle
VHD V2 rotate(V2 v, Real c, Real s) { return mk(v.x * c - v.y * s, v.x * s + v.y * c); }

// _vectorized_joint_constraints + _get_constraint_torques (core.py:2200-2291, 2840-2857)
// fixed_rot = JointConstraint.fixed_rotation for this env.
VHD PairOut pair_joint(V2 pa, Real rota, Trig ta, V2 pb, Real rotb, Trig tb, V2 da, V2 db,
                       Real dist, bool rotate_ok, Real fixed_rot, const WorldK& w) {
    const V2 pja = pa + rotate(da, ta.c0, ta.s0);
    const V2 pjb = pb + rotate(db, tb.c0, tb.s0);
    const V2 fat = constraint_force(pja, pjb, dist, -w.cj, w.k, true);
    const V2 far = constraint_force(pja, pjb, dist, w.cj, w.k, false);
    const V2 fa = fat + far;
    const V2 fb = (-fat) + (-far);
    Real tra = cross(pja - pa, fa);
    Real trb = cross(pjb - pb, fb);
    if (!rotate_ok) {
        const Real delta = rota - (rotb + fixed_rot);
        const Real ad = fabsf(delta);
        const Real pen = expf(ad) - 1.f;
        Real tq = (w.ct * tsign(delta)) * pen;
        if (ad < 1e-9f) tq = 0.f;
        tra = tra + (-tq);
        trb = trb + tq;
    }
    return PairOut{fa, tra, trb};
}

// get_friction_force (core.py:2054-2072) for a 2-vector
VHD V2 friction2(V2 v, Real coeff, Real mass, Real sdt) {
    const Real speed = norm(v);
    const Real ffc = coeff * mass;
    const Real den = (speed == 0.f) ? 1e-8f : speed;
    V2 f = mk(-(v.x / den) * tmin(ffc, (fabsf(v.x) / sdt) * mass),
              -(v.y / den) * tmin(ffc, (fabsf(v.y) / sdt) * mass));
    if (speed == 0.f) f = mk(0.f, 0.f);
    return f;
}
VHD Real friction1(Real v, Real coeff, Real mass, Real sdt) {
    const Real speed = fabsf(v);
    const Real ffc = coeff * mass;
    const Real den = (speed == 0.f) ? 1e-8f : speed;
#ifdef VMAS_PHYS_RELAXED
    // v / |v| is exactly +-1 in IEEE arithmetic for every finite v != 0, denormals included.
    // The relaxed build's division is x * v_rcp_f32(y), and v_rcp_f32 of a denormal is inf: an
    // angular velocity that friction has brought to a denormal residue would make the torque
    // inf (measured: features world, 16 384 envs).  So the sign is taken directly (NaN and 0
    // keep the division, whose result is the same there).
    const Real dir = (speed == 0.f || speed != speed) ? v / den : copysignf(1.f, v);
    Real f = -dir * tmin(ffc, (fabsf(v) / sdt) * mass);
#else
    Real f = -(v / den) * tmin(ffc, (fabsf(v) / sdt) * mass);
#endif
    if (speed == 0.f) f = 0.f;
    return f;
}

// Action force/torque clamps + friction + gravity of one entity (core.py:1994-2003, 2017-2101).
// af/at: the agent's current state.force/torque, updated in place (the reference writes the
// clamped value back to agent.state.force each substep).
VHD void pre_forces(const VmasEntityDesc& d, bool is_agent, V2& af, Real& at, V2 vel,
                                           Real w, V2 eg, bool has_eg, Real gx, Real gy, bool has_g,
                                           Real sdt, Real& fx, Real& fy, Real& tq) {
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
            Real t = at;
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
VHD void integrate(const VmasEntityDesc& d, int substep, Real sdt, Real fx, Real fy,
                                          Real tq, bool has_xs, Real xs, bool has_ys, Real ys, V2& p, V2& v,
                                          Real& rot, Real& w) {
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

// ---------------------------------------------------------------------------------------------
// Ray casts (core.py:1280-1625), one ray against one target.  `o` ray origin, (dc, ds) ray dir.
VHD Real ray_box(V2 o, Real ang, Real dc, Real ds, V2 bp, Real brot, Real L, Real W,
                  Real max_range) {
    const V2 po = o - bp;
    const Real nc = cosf(-brot), ns = sinf(-brot);
    const V2 pa = rotate(po, nc, ns);
    const V2 da = rotate(mk(dc, ds), nc, ns);
    (void)ang;
    const Real tx1 = ((-L) / 2.f - pa.x) / da.x;
    const Real tx2 = (L / 2.f - pa.x) / da.x;
    Real tmn = tmin(tx1, tx2), tmx = tmax(tx1, tx2);
    const Real ty1 = ((-W) / 2.f - pa.y) / da.y;
    const Real ty2 = (W / 2.f - pa.y) / da.y;
    const Real tymn = tmin(ty1, ty2), tymx = tmax(ty1, ty2);
    tmn = tmax(tmn, tymn);
    tmx = tmin(tmx, tymx);
    const V2 ia = da * tmn + pa;  // tmin * dir_aabb + pos_aabb
    const V2 iw = rotate(ia, cosf(brot), sinf(brot)) + bp;
    const bool hit = (tmx >= tmn) && (tmn > 0.f);
    const Real d = norm(o - iw);
    return hit ? d : max_range;
}

VHD Real ray_sphere(V2 o, Real dc, Real ds, V2 sp, Real r, Real max_range) {
    const V2 dir = mk(dc, ds);
    const V2 lp = o + dir * (max_range / 2.f);
    const V2 cp = closest_point_line(lp, dir, 0.f, sp, false);
    const Real dn = norm(sp - cp);
    const bool inter = dn < r;
    const Real a = r * r - dn * dn;
    const Real m = sqrtf((a > 0.f) ? a : 1e-8f);
    const V2 u = sp - o;
    const V2 u1 = cp - o;
    const Real udot = u.x * dir.x + u.y * dir.y;
    const bool front = udot > 0.f;
    const Real d = norm(u1) - m;
    return (inter && front) ? d : max_range;
}

// The same distance in its direct form (the fused scenario programs' fast LIDAR): u = centre -
// origin, t = u . dir (the foot point's distance along the ray; the reference's |cp - o| and its
// `front` test udot > 0), dn^2 = |u|^2 - t^2 (the reference's |sp - cp|^2), d = t - sqrt(r^2 - dn^2)
// on a hit.  Mathematically the reference's value; in fp32 within the LIDAR parity tolerance,
// and at a tangent ray or the front boundary the hit / miss decision can flip (certified by a
// ray turned by ~1e-6 rad, tests/_parity.py lidar_parity).  `u` is the centre relative to the
// origin, `r2` the squared radius.
VHD Real ray_sphere_fast(V2 u, Real dc, Real ds, Real r2, Real max_range) {
    const Real t = u.x * dc + u.y * ds;
    const Real a = r2 - (u.x * u.x + u.y * u.y - t * t);
    const Real m = sqrtf(a > 0.f ? a : 1e-8f);
    return (a > 0.f && t > 0.f) ? t - m : max_range;
}

// ray_sphere_fast without compares (the fused programs' inner loop: 6 VALU + the hardware square
// root per (ray, sphere) instead of ~26 with the compares, selects and the NaN-propagating min as
// divergent branches).  c = r^2 - |u|^2 per sphere; returns t - sqrt(min(a, t * 1e30)), a = t^2 + c
// = r^2 - dn^2: NaN on a miss (a < 0, or t < 0 making the root's argument negative), which the
// caller's fminf drops (IEEE minNum keeps the other operand) -- so the running minimum starts at
// max_range and never becomes NaN, as the reference's where(hit, d, max_range) before its min
// (non-finite positions fail its comparisons: max_range; here: NaN, dropped).  Differs from
// ray_sphere_fast only on the measure-zero boundaries a == 0 and t == 0 (and t * 1e30 < a, t below
// ~1e-32), the hit / miss flips the LIDAR certification covers.
VHD float ray_sphere_fast_nan(float ux, float uy, float c, float dc, float ds) {
    const float t = __builtin_fmaf(ux, dc, uy * ds);
    const float a = __builtin_fmaf(t, t, c);
    return t - __builtin_amdgcn_sqrtf(__builtin_fminf(a, t * 1e30f));
}
#if defined(__HIP_DEVICE_COMPILE__)
// v_min_f32 as is (IEEE mode: a quiet NaN operand yields the other one).  fminf makes the compiler
// quieten a running minimum that crosses a basic block (v_max_f32 x, x) on every update.
__device__ __forceinline__ float min_drop_nan(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
#else
VHD float min_drop_nan(float a, float b) { return fminf(a, b); }
#endif

VHD Real ray_line(V2 o, Real dc, Real ds, V2 lp, Real lrot, Real L, Real max_range) {
    const V2 r = mk(cosf(lrot) * L, sinf(lrot) * L);
    const V2 s = mk(dc, ds);
    const Real rxs = cross(r, s);
    const V2 qp = o - lp;
    const Real t = cross(qp, s / rxs);
    const Real u = cross(qp, r / rxs);
    const Real d = norm(mk(u * s.x, u * s.y));
    const bool miss = (rxs == 0.f) || (t > 0.5f) || (t < -0.5f) || (u < 0.f);
    return miss ? max_range : d;
}

}  // namespace VMAS_PHYS_NS
