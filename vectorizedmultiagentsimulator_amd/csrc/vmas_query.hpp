// vmas_query.hpp -- per-env distance / overlap queries (World.get_distance_from_point,
// get_distance, is_overlapping; core.py:1787-1968), shared by k_distance (vmas_kernels.hip) and
// the fused scenario kernels (vmas_scenarios.hip).
#pragma once

#include "vmas_physics.hpp"

namespace vmas {

__host__ __device__ __forceinline__ V2 ref_pos(const VmasShapeRef& s, int b) {
    return mk(s.pos[(long)b * s.pos_s0], s.pos[(long)b * s.pos_s0 + s.pos_s1]);
}
__host__ __device__ __forceinline__ float ref_rot(const VmasShapeRef& s, int b) {
    return s.rot ? s.rot[(long)b * s.rot_s0] : 0.f;
}

// get_distance_from_point (core.py:1787-1819)
__host__ __device__ __forceinline__ float dist_point(const VmasShapeRef& a, int b, V2 tp) {
    const V2 p = ref_pos(a, b);
    if (a.shape == VMAS_SPHERE) return norm(p - tp) - a.radius;
    if (a.shape == VMAS_BOX) {
        const V2 cp = closest_point_box(p, make_trig(ref_rot(a, b)), a.length / 2.f, a.width / 2.f, tp);
        return norm(tp - cp) - kLineMinDist;
    }
    const float r = ref_rot(a, b);
    const V2 cp = closest_point_line(p, mk(cosf(r), sinf(r)), a.length / 2.f, tp, true);
    return norm(tp - cp) - kLineMinDist;
}

// is_overlapping for (box, sphere) (core.py:1932-1963)
__host__ __device__ __forceinline__ bool overlap_box_sphere(const VmasShapeRef& bx, const VmasShapeRef& sp, int b) {
    const V2 pb = ref_pos(bx, b), ps = ref_pos(sp, b);
    const V2 cp = closest_point_box(pb, make_trig(ref_rot(bx, b)), bx.length / 2.f, bx.width / 2.f, ps);
    const float dsc = norm(ps - cp), dsb = norm(ps - pb), dcb = norm(pb - cp);
    return (dsb < dcb) || (dsc < sp.radius_lmd);
}

// get_distance (core.py:1821-1904); a/b are canonicalised by the caller as the reference does
__host__ __device__ __forceinline__ float dist_pair(const VmasShapeRef& a, const VmasShapeRef& bref, int b) {
    const int sa = a.shape, sb = bref.shape;
    if (sa == VMAS_SPHERE && sb == VMAS_SPHERE) return dist_point(a, b, ref_pos(bref, b)) - bref.radius;
    if (sa == VMAS_BOX && sb == VMAS_SPHERE) {
        float d = dist_point(a, b, ref_pos(bref, b)) - bref.radius;
        if (overlap_box_sphere(a, bref, b)) d = -1.f;
        return d;
    }
    if (sa == VMAS_LINE && sb == VMAS_SPHERE) return dist_point(a, b, ref_pos(bref, b)) - bref.radius;
    const float ra = ref_rot(a, b), rb = ref_rot(bref, b);
    const V2 pa = ref_pos(a, b), pb = ref_pos(bref, b);
    V2 qa, qb;
    if (sa == VMAS_LINE && sb == VMAS_LINE) {
        closest_points_line_line(Seg{pa, mk(cosf(ra), sinf(ra)), a.length / 2.f},
                                 Seg{pb, mk(cosf(rb), sinf(rb)), bref.length / 2.f}, &qa, &qb);
    } else if (sa == VMAS_BOX && sb == VMAS_LINE) {
        closest_line_box(pa, make_trig(ra), a.length / 2.f, a.width / 2.f,
                         Seg{pb, mk(cosf(rb), sinf(rb)), bref.length / 2.f}, &qa, &qb);
    } else {  // box, box
        closest_box_box(pa, make_trig(ra), a.length / 2.f, a.width / 2.f, pb, make_trig(rb),
                        bref.length / 2.f, bref.width / 2.f, &qa, &qb);
    }
    return norm(qa - qb) - kLineMinDist;
}

__host__ __device__ __forceinline__ float distance_query(int kind, const VmasShapeRef& a,
                                                         const VmasShapeRef& bref, const float* tp,
                                                         int tp_s0, int tp_s1, int b) {
    if (kind == VMAS_DIST_POINT) return dist_point(a, b, mk(tp[(long)b * tp_s0], tp[(long)b * tp_s0 + tp_s1]));
    if (kind == VMAS_DIST_PAIR) return dist_pair(a, bref, b);
    // overlap
    if (a.shape == VMAS_BOX && bref.shape == VMAS_SPHERE) return overlap_box_sphere(a, bref, b) ? 1.f : 0.f;
    return (dist_pair(a, bref, b) < 0.f) ? 1.f : 0.f;
}

__host__ __device__ __forceinline__ void store_query(void* out, int kind, int b, float v) {
    if (kind == VMAS_OVERLAP_PAIR) reinterpret_cast<uint8_t*>(out)[b] = v != 0.f;  // torch.bool
    else reinterpret_cast<float*>(out)[b] = v;
}

// World.cast_rays of one (env, ray) (core.py:1661-1785): min over the targets of the ray-shape
// distances, from max_range.  Shared by k_cast_rays (vmas_kernels.hip) and the fused scenario
// kernels (vmas_scenarios.hip).
__host__ __device__ __forceinline__ float cast_one(const VmasRayTarget* tg, int nt, V2 o, float ang,
                                                   int b, float max_range) {
    const float dc = cosf(ang), ds = sinf(ang);
    float best = max_range;
    for (int t = 0; t < nt; ++t) {
        const VmasRayTarget& x = tg[t];
        const V2 tp = mk(x.pos[(long)b * x.pos_s0], x.pos[(long)b * x.pos_s0 + x.pos_s1]);
        float d;
        if (x.shape == VMAS_SPHERE) {
            d = ray_sphere(o, dc, ds, tp, x.radius, max_range);
        } else if (x.shape == VMAS_BOX) {
            d = ray_box(o, ang, dc, ds, tp, x.rot[(long)b * x.rot_s0], x.length, x.width, max_range);
        } else {
            d = ray_line(o, dc, ds, tp, x.rot[(long)b * x.rot_s0], x.length, max_range);
        }
        best = tmin(best, d);
    }
    return best;
}

}  // namespace vmas
