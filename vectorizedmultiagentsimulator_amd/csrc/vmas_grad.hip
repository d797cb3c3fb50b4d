// vmas_grad.hip -- the gradient of the physics step (autograd through World.step, reference
// test_vmas.py:277-304 / environment.py grad_enabled), gfx950 kernels + host backend + C ABI.
//
// vmas_world_step_vjp computes the vector-Jacobian product of one World.step: given the step's
// inputs (the same VmasStepIO the forward took) and the gradient of a loss with respect to the
// step's outputs (laid out as the forward's output buffer), it writes the gradient with respect
// to every entity's pos / vel / rot / ang_vel and every agent's force / torque.
//
// Method: forward-mode dual numbers (vmas_dual.hpp) through the SAME physics functions as the
// forward (vmas_physics.hpp, included here a second time with Real = Dual, in its own
// namespace).  One pass of the per-env step carries 8 tangents, i.e. 8 columns of the env's
// Jacobian; ceil(n_in / 8) passes per env (n_in = 6 per entity + 3 per agent) give every column,
// contracted on the fly with the output gradient.  The batch-global broadphase mask is the
// forward's fixed point, recomputed here with the same R/Z rule (a host-driven loop of value
// passes).  The value part of a dual pass equals the forward step's fp32 results.  Entity
// gravity and joint fixed rotations enter as constants.
//
// Cost: ~9 x (value + 8 tangents) x ceil(n_in / 8) forward steps -- a training-time path, not
// the benchmark's.  One thread per (env, column block) on the GPU, a thread pool on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"

#include "vmas_dual.hpp"
#define VMAS_PHYS_NS vmas_dual
#define VMAS_PHYS_GRAD 1
#define VMAS_PHYS_REAL vmas_dual::Dual
#include "vmas_physics.hpp"

namespace {

using vmas_dual::Dual;
using vmas_dual::kTangents;
using DV2 = vmas_dual::V2;
using DTrig = vmas_dual::Trig;
using DOut = vmas_dual::PairOut;

// Static tables of a world (device copies for the GPU path)
struct Tables {
    VmasWorldConfig cfg;
    const VmasEntityDesc* ed;
    const VmasPairDesc* pd;
    const VmasJointDesc* jd;
    const int32_t* dyn;       // dynamic entities
    const int32_t* item_off;  // [n_dyn + 1]
    const int32_t* items;     // (pair << 2) | (side << 1) | torque, in pair order (as k_step)
    int n_dyn, W;
};

struct Work {  // one env's dual state (pointers into a workspace slice)
    DV2 *pos, *vel;
    Dual *rot, *ang, *af;
    DTrig* tr;
    DOut* res;
};

__host__ __device__ inline size_t work_duals(int E, int A, int P) { return (size_t)E * 10 + (size_t)A * 3 + (size_t)P * 4; }

__host__ __device__ inline Work carve(Dual* ws, int E, int A) {
    Work w;
    w.pos = reinterpret_cast<DV2*>(ws);
    w.vel = w.pos + E;
    w.rot = reinterpret_cast<Dual*>(w.vel + E);
    w.ang = w.rot + E;
    w.tr = reinterpret_cast<DTrig*>(w.ang + E);
    w.af = reinterpret_cast<Dual*>(w.tr + E);
    w.res = reinterpret_cast<DOut*>(w.af + A * 3);
    return w;
}

__host__ __device__ inline float ld(const float* p, long i) { return p[i]; }

// Input column c of an env: entity e = c / 6 (pos.x, pos.y, vel.x, vel.y, rot, ang) for
// c < 6E, then agent a = (c - 6E) / 3 (force.x, force.y, torque).
// One pass of env b with tangent slot k seeded on column col0 + k.  Returns the contraction of
// the outputs' tangents with the output gradient in g[kTangents] (when gout is set), and the
// broadphase activity bits in R / Z (when set, value passes).
__host__ __device__ void dual_step_env(const Tables& T, const VmasStepIO& io, const uint32_t* mask, int b, int col0,
                                       Dual* ws, bool tangents, const VmasStepIO* gout, float* g, uint32_t* R,
                                       uint32_t* Z) {
    using namespace vmas_dual;
    const int E = T.cfg.n_entities, A = T.cfg.n_agents, P = T.cfg.n_pairs, S = io.substeps, Wd = T.W;
    Work w = carve(ws, E, A);
    auto sd = [&](float x, int col) { return tangents ? seed(x, col - col0) : Dual(x); };
    for (int e = 0; e < E; ++e) {
        const VmasEntityIO& x = io.entities[e];
        const int c = 6 * e;
        w.pos[e] = mk(sd(ld(x.pos, (long)b * x.pos_s0), c), sd(ld(x.pos, (long)b * x.pos_s0 + x.pos_s1), c + 1));
        w.vel[e] = mk(sd(ld(x.vel, (long)b * x.vel_s0), c + 2), sd(ld(x.vel, (long)b * x.vel_s0 + x.vel_s1), c + 3));
        w.rot[e] = sd(ld(x.rot, (long)b * x.rot_s0), c + 4);
        w.ang[e] = sd(ld(x.ang_vel, (long)b * x.ang_s0), c + 5);
        w.tr[e] = make_trig_for(w.rot[e], T.ed[e].shape == VMAS_BOX);
    }
    for (int a = 0; a < A; ++a) {
        const VmasAgentIO& x = io.agents[a];
        const int c = 6 * E + 3 * a;
        w.af[3 * a] = sd(ld(x.force, (long)b * x.force_s0), c);
        w.af[3 * a + 1] = sd(ld(x.force, (long)b * x.force_s0 + x.force_s1), c + 1);
        w.af[3 * a + 2] = sd(ld(x.torque, (long)b * x.torque_s0), c + 2);
    }
    const WorldK wk{T.cfg.contact_margin, T.cfg.collision_force, T.cfg.joint_force, T.cfg.torque_constraint_force};
    const Dual sdt(io.sub_dt);
    for (int s = 0; s < S; ++s) {
        for (int p = 0; p < P; ++p) {
            const VmasPairDesc& pd = T.pd[p];
            bool inr = true;
            if (pd.cls != VMAS_PAIR_JOINT) inr = norm(w.pos[pd.ea] - w.pos[pd.eb]) <= pd.bp_radius;
            if (R && inr) R[s * Wd + (p >> 5)] |= 1u << (p & 31);
            if (!((mask[s * Wd + (p >> 5)] >> (p & 31)) & 1u)) continue;
            const int ea = pd.ea, eb = pd.eb;
            const VmasEntityDesc &da = T.ed[ea], &db = T.ed[eb];
            DOut o;
            switch (pd.cls) {  // eval_pair of vmas_kernels.hip
                case VMAS_PAIR_SS: o = pair_ss(w.pos[ea], w.pos[eb], pd.dmin, wk); break;
                case VMAS_PAIR_LS: o = pair_ls(w.pos[ea], w.tr[ea], da.half_length, w.pos[eb], pd.dmin, wk); break;
                case VMAS_PAIR_LL:
                    o = pair_ll(w.pos[ea], w.tr[ea], da.half_length, w.pos[eb], w.tr[eb], db.half_length, pd.dmin, wk);
                    break;
                case VMAS_PAIR_BS:
                    o = pair_bs(w.pos[ea], w.tr[ea], da.half_length, da.half_width, (da.flags & VMAS_F_HOLLOW) != 0,
                                w.pos[eb], pd.dmin, wk);
                    break;
                case VMAS_PAIR_BL:
                    o = pair_bl(w.pos[ea], w.tr[ea], da.half_length, da.half_width, (da.flags & VMAS_F_HOLLOW) != 0,
                                w.pos[eb], w.tr[eb], db.half_length, pd.dmin, wk);
                    break;
                case VMAS_PAIR_BB:
                    o = pair_bb(w.pos[ea], w.tr[ea], da.half_length, da.half_width, (da.flags & VMAS_F_HOLLOW) != 0,
                                w.pos[eb], w.tr[eb], db.half_length, db.half_width, (db.flags & VMAS_F_HOLLOW) != 0,
                                pd.dmin, wk);
                    break;
                default: {
                    const VmasJointDesc j = T.jd[pd.joint];
                    const VmasJointIO* ji = io.joints ? &io.joints[pd.joint] : nullptr;
                    const float fr = (ji && ji->fixed_rotation) ? ji->fixed_rotation[(long)b * ji->s0] : j.fixed_rotation;
                    o = pair_joint(w.pos[ea], w.rot[ea], w.tr[ea], w.pos[eb], w.rot[eb], w.tr[eb], mk(Dual(j.delta_a_x), Dual(j.delta_a_y)),
                                   mk(Dual(j.delta_b_x), Dual(j.delta_b_y)), j.dist, j.rotate != 0, fr, wk);
                }
            }
            w.res[p] = o;
            if (Z && pd.cls != VMAS_PAIR_JOINT && !inr && (o.fa.x != 0.f || o.fa.y != 0.f || o.ta != 0.f || o.tb != 0.f))
                Z[s * Wd + (p >> 5)] |= 1u << (p & 31);
        }
        for (int i = 0; i < T.n_dyn; ++i) {
            const int e = T.dyn[i];
            const VmasEntityDesc& d = T.ed[e];
            DV2 a2 = mk(Dual(0.f), Dual(0.f));
            Dual at(0.f);
            if (d.agent_index >= 0) {
                a2 = mk(w.af[d.agent_index * 3], w.af[d.agent_index * 3 + 1]);
                at = w.af[d.agent_index * 3 + 2];
            }
            DV2 eg = mk(Dual(0.f), Dual(0.f));
            const bool has_eg = (d.flags & VMAS_F_GRAVITY) != 0;
            if (has_eg) {
                const VmasEntityIO& x = io.entities[e];
                eg = mk(Dual(ld(x.gravity, (long)b * x.grav_s0)), Dual(ld(x.gravity, (long)b * x.grav_s0 + x.grav_s1)));
            }
            Dual fx, fy, tq;
            pre_forces(d, d.agent_index >= 0, a2, at, w.vel[e], w.ang[e], eg, has_eg, T.cfg.gravity_x, T.cfg.gravity_y,
                       T.cfg.has_world_gravity != 0, sdt, fx, fy, tq);
            if (d.agent_index >= 0) {
                w.af[d.agent_index * 3] = a2.x;
                w.af[d.agent_index * 3 + 1] = a2.y;
                w.af[d.agent_index * 3 + 2] = at;
            }
            const bool mov = d.flags & VMAS_F_MOVABLE, rotb = d.flags & VMAS_F_ROTATABLE;
            for (int q = T.item_off[i]; q < T.item_off[i + 1]; ++q) {
                const int it = T.items[q], p = it >> 2;
                if (!((mask[s * Wd + (p >> 5)] >> (p & 31)) & 1u)) continue;
                const bool side = (it >> 1) & 1;
                if (mov) {
                    fx = fx + (side ? -w.res[p].fa.x : w.res[p].fa.x);
                    fy = fy + (side ? -w.res[p].fa.y : w.res[p].fa.y);
                }
                if (rotb && (it & 1)) tq = tq + (side ? w.res[p].tb : w.res[p].ta);
            }
            DV2 p2 = w.pos[e], v2 = w.vel[e];
            Dual r2 = w.rot[e], w2 = w.ang[e];
            integrate(d, s, sdt, fx, fy, tq, T.cfg.has_x_semidim != 0, T.cfg.x_semidim, T.cfg.has_y_semidim != 0,
                      T.cfg.y_semidim, p2, v2, r2, w2);
            w.pos[e] = p2;
            w.vel[e] = v2;
            w.rot[e] = r2;
            w.ang[e] = w2;
            if (d.flags & VMAS_F_ROTATABLE) w.tr[e] = make_trig_for(r2, d.shape == VMAS_BOX);
        }
    }
    if (!gout) return;
    // contraction with the output gradient (the forward's output layout: [slot][B][2] / [slot][B])
    const int B = T.cfg.batch;
#pragma unroll
    for (int k = 0; k < kTangents; ++k) g[k] = 0.f;
    auto acc = [&](const float* gp, const Dual& x) {
        const float gv = *gp;
        if (gv != 0.f)
            for (int k = 0; k < kTangents; ++k) g[k] += gv * x.d[k];
    };
    for (int i = 0; i < T.n_dyn; ++i) {
        const int e = T.dyn[i];
        const VmasEntityDesc& d = T.ed[e];
        if (d.out_lin >= 0) {
            const size_t o = ((size_t)d.out_lin * B + b) * 2;
            acc(gout->out_pos + o, w.pos[e].x);
            acc(gout->out_pos + o + 1, w.pos[e].y);
            acc(gout->out_vel + o, w.vel[e].x);
            acc(gout->out_vel + o + 1, w.vel[e].y);
        }
        if (d.out_rot >= 0) {
            const size_t o = (size_t)d.out_rot * B + b;
            acc(gout->out_rot + o, w.rot[e]);
            acc(gout->out_ang_vel + o, w.ang[e]);
        }
        if (d.agent_index >= 0) {
            if (d.out_force >= 0) {
                const size_t o = ((size_t)d.out_force * B + b) * 2;
                acc(gout->out_force + o, w.af[d.agent_index * 3]);
                acc(gout->out_force + o + 1, w.af[d.agent_index * 3 + 1]);
            }
            if (d.out_torque >= 0) acc(gout->out_torque + (size_t)d.out_torque * B + b, w.af[d.agent_index * 3 + 2]);
        }
    }
}

// Scatter the contracted column block of env b into the per-input gradient buffers.
__host__ __device__ inline void scatter(const VmasGradIO& gio, int E, int A, int B, int b, int col0, int n_in,
                                        const float* g) {
    for (int k = 0; k < kTangents && col0 + k < n_in; ++k) {
        const int c = col0 + k;
        if (c < 6 * E) {
            const int e = c / 6, f = c % 6;
            float* dst = f < 2 ? gio.pos[e] : f < 4 ? gio.vel[e] : f == 4 ? gio.rot[e] : gio.ang_vel[e];
            if (!dst) continue;
            if (f < 4) dst[(long)b * 2 + (f & 1)] = g[k];
            else dst[b] = g[k];
        } else {
            const int a = (c - 6 * E) / 3, f = (c - 6 * E) % 3;
            float* dst = f < 2 ? gio.force[a] : gio.torque[a];
            if (!dst) continue;
            if (f < 2) dst[(long)b * 2 + f] = g[k];
            else dst[b] = g[k];
        }
    }
    (void)B;
}

struct GradArgs {
    Tables T;
    VmasStepIO io, gout;
    VmasGradIO gio;
    const uint32_t* mask;
    uint32_t *R, *Z;
    Dual* ws;
    int n_in, n_blocks;
    bool value_pass;
};

__global__ void __launch_bounds__(64) k_grad(GradArgs a) {
    const long t = (long)blockIdx.x * 64 + threadIdx.x;
    const int B = a.T.cfg.batch;
    const int E = a.T.cfg.n_entities, A = a.T.cfg.n_agents, P = a.T.cfg.n_pairs;
    Dual* ws = a.ws + (size_t)t * work_duals(E, A, P);
    if (a.value_pass) {
        if (t >= B) return;
        const int S = a.io.substeps, Wd = a.T.W;
        // per-env activity bits, OR-ed into the batch words
        uint32_t r[256], z[256];
        const int nw = S * Wd;
        for (int i = 0; i < nw; ++i) r[i] = z[i] = 0u;
        dual_step_env(a.T, a.io, a.mask, (int)t, 0, ws, false, nullptr, nullptr, r, z);
        for (int i = 0; i < nw; ++i) {
            if (r[i]) atomicOr(&a.R[i], r[i]);
            if (z[i]) atomicOr(&a.Z[i], z[i]);
        }
        return;
    }
    if (t >= (long)B * a.n_blocks) return;
    const int b = (int)(t / a.n_blocks), col0 = (int)(t % a.n_blocks) * kTangents;
    float g[kTangents];
    dual_step_env(a.T, a.io, a.mask, b, col0, ws, true, &a.gout, g, nullptr, nullptr);
    scatter(a.gio, E, A, B, b, col0, a.n_in, g);
}

thread_local std::vector<char> g_scratch;

// ---- distance queries (core.py:1787-1904) with dual operands ------------------------------------
// An entity as seen by a query: its shape numbers (VmasShapeRef) and its dual pose.
struct DEnt {
    const VmasShapeRef* s;
    DV2 p;
    Dual r;
};

__host__ __device__ inline Dual ddist_point(const DEnt& a, DV2 tp) {  // get_distance_from_point
    using namespace vmas_dual;
    if (a.s->shape == VMAS_SPHERE) return norm(a.p - tp) - a.s->radius;
    if (a.s->shape == VMAS_BOX) {
        const DV2 cp = closest_point_box(a.p, make_trig(a.r), a.s->length / 2.f, a.s->width / 2.f, tp);
        return norm(tp - cp) - kLineMinDist;
    }
    const DV2 cp = closest_point_line(a.p, mk(cosf(a.r), sinf(a.r)), a.s->length / 2.f, tp, true);
    return norm(tp - cp) - kLineMinDist;
}

__host__ __device__ inline bool doverlap_box_sphere(const DEnt& bx, const DEnt& sp) {
    using namespace vmas_dual;
    const DV2 cp = closest_point_box(bx.p, make_trig(bx.r), bx.s->length / 2.f, bx.s->width / 2.f, sp.p);
    const Dual dsc = norm(sp.p - cp), dsb = norm(sp.p - bx.p), dcb = norm(bx.p - cp);
    return (dsb < dcb) || (dsc < sp.s->radius_lmd);
}

__host__ __device__ inline Dual ddist_pair(const DEnt& a, const DEnt& b) {  // get_distance (canonical order)
    using namespace vmas_dual;
    const int sa = a.s->shape, sb = b.s->shape;
    if (sa == VMAS_SPHERE && sb == VMAS_SPHERE) return ddist_point(a, b.p) - b.s->radius;
    if (sa == VMAS_BOX && sb == VMAS_SPHERE) {
        Dual d = ddist_point(a, b.p) - b.s->radius;
        if (doverlap_box_sphere(a, b)) d = Dual(-1.f);
        return d;
    }
    if (sa == VMAS_LINE && sb == VMAS_SPHERE) return ddist_point(a, b.p) - b.s->radius;
    DV2 qa, qb;
    if (sa == VMAS_LINE && sb == VMAS_LINE) {
        closest_points_line_line(Seg{a.p, mk(cosf(a.r), sinf(a.r)), Dual(a.s->length / 2.f)},
                                 Seg{b.p, mk(cosf(b.r), sinf(b.r)), Dual(b.s->length / 2.f)}, &qa, &qb);
    } else if (sa == VMAS_BOX && sb == VMAS_LINE) {
        closest_line_box(a.p, make_trig(a.r), a.s->length / 2.f, a.s->width / 2.f,
                         Seg{b.p, mk(cosf(b.r), sinf(b.r)), Dual(b.s->length / 2.f)}, &qa, &qb);
    } else {
        closest_box_box(a.p, make_trig(a.r), a.s->length / 2.f, a.s->width / 2.f, b.p, make_trig(b.r),
                        b.s->length / 2.f, b.s->width / 2.f, &qa, &qb);
    }
    return norm(qa - qb) - kLineMinDist;
}

// inputs of one env: a.pos (0, 1), a.rot (2), b.pos (3, 4), b.rot (5), test point (6, 7): one pass
struct DistArgs {
    VmasShapeRef a, b;
    int32_t kind, has_b, batch, pad;
    const float* tp;
    int32_t tp_s0, tp_s1;
    const float* gout;
    float *ga_pos, *ga_rot, *gb_pos, *gb_rot, *gtp;
};

__host__ __device__ inline void dist_vjp_env(const DistArgs& x, int b) {
    using vmas_dual::seed;
    const float g = x.gout[b];
    auto pose = [&](const VmasShapeRef& s, int c0) {
        DEnt e;
        e.s = &s;
        e.p = vmas_dual::mk(seed(s.pos[(long)b * s.pos_s0], c0), seed(s.pos[(long)b * s.pos_s0 + s.pos_s1], c0 + 1));
        e.r = seed(s.rot ? s.rot[(long)b * s.rot_s0] : 0.f, c0 + 2);
        return e;
    };
    const DEnt ea = pose(x.a, 0);
    Dual d;
    if (x.kind == VMAS_DIST_POINT) {
        const DV2 tp = vmas_dual::mk(seed(x.tp[(long)b * x.tp_s0], 6), seed(x.tp[(long)b * x.tp_s0 + x.tp_s1], 7));
        d = ddist_point(ea, tp);
    } else {
        d = ddist_pair(ea, pose(x.b, 3));
    }
    if (x.ga_pos) {
        x.ga_pos[(long)b * 2] = g * d.d[0];
        x.ga_pos[(long)b * 2 + 1] = g * d.d[1];
    }
    if (x.ga_rot) x.ga_rot[b] = g * d.d[2];
    if (x.gb_pos) {
        x.gb_pos[(long)b * 2] = g * d.d[3];
        x.gb_pos[(long)b * 2 + 1] = g * d.d[4];
    }
    if (x.gb_rot) x.gb_rot[b] = g * d.d[5];
    if (x.gtp) {
        x.gtp[(long)b * 2] = g * d.d[6];
        x.gtp[(long)b * 2 + 1] = g * d.d[7];
    }
}

__global__ void __launch_bounds__(64) k_dist_vjp(DistArgs x) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b < x.batch) dist_vjp_env(x, b);
}

// ---- ray casts (core.py:1280-1785) with dual operands -------------------------------------------
// inputs of one env: origin (0, 1), rot offset (2), target t pos / rot (3 + 3t ..), angles (3 + 3nt + r)
struct RayVjpArgs {
    const VmasRayTarget* tg;  // (device copy on the GPU)
    int32_t nt, B, R, n_in, n_blocks;
    const float* origin;
    int32_t o_s0, o_s1;
    const float* ang;
    int32_t a_s0, a_s1;
    const float* rot;
    int32_t r_s0;
    float max_range;
    const float* gout;        // [B, R] contiguous
    float *g_origin, *g_rot, *g_ang;       // [B,2], [B], [B,R]
    float* const* g_tpos;     // per target [B,2] (device array on the GPU)
    float* const* g_trot;     // per target [B]
};

__host__ __device__ inline void ray_vjp_env(const RayVjpArgs& x, int b, int col0) {
    using namespace vmas_dual;
    auto sd = [&](float v, int c) { return seed(v, c - col0); };
    const DV2 o = mk(sd(x.origin[(long)b * x.o_s0], 0), sd(x.origin[(long)b * x.o_s0 + x.o_s1], 1));
    const Dual roff = sd(x.rot ? x.rot[(long)b * x.r_s0] : 0.f, 2);
    float g[kTangents];
    for (int k = 0; k < kTangents; ++k) g[k] = 0.f;
    for (int r = 0; r < x.R; ++r) {
        const float gr = x.gout[(long)b * x.R + r];
        if (gr == 0.f) continue;
        Dual a = sd(x.ang[(long)b * x.a_s0 + (long)r * x.a_s1], 3 + 3 * x.nt + r);
        if (x.rot) a = a + roff;
        const Dual dc = cosf(a), ds = sinf(a);
        Dual best(x.max_range);
        for (int t = 0; t < x.nt; ++t) {  // cast_one of vmas_query.hpp
            const VmasRayTarget& q = x.tg[t];
            const DV2 tp = mk(sd(q.pos[(long)b * q.pos_s0], 3 + 3 * t), sd(q.pos[(long)b * q.pos_s0 + q.pos_s1], 4 + 3 * t));
            Dual d;
            if (q.shape == VMAS_SPHERE) {
                d = ray_sphere(o, dc, ds, tp, q.radius, x.max_range);
            } else {
                const Dual tr = sd(q.rot[(long)b * q.rot_s0], 5 + 3 * t);
                if (q.shape == VMAS_BOX) d = ray_box(o, a, dc, ds, tp, tr, q.length, q.width, x.max_range);
                else d = ray_line(o, dc, ds, tp, tr, q.length, x.max_range);
            }
            best = tmin(best, d);
        }
        for (int k = 0; k < kTangents; ++k) g[k] += gr * best.d[k];
    }
    for (int k = 0; k < kTangents && col0 + k < x.n_in; ++k) {
        const int c = col0 + k;
        if (c < 2) {
            if (x.g_origin) x.g_origin[(long)b * 2 + c] = g[k];
        } else if (c == 2) {
            if (x.g_rot) x.g_rot[b] = g[k];
        } else if (c < 3 + 3 * x.nt) {
            const int t = (c - 3) / 3, f = (c - 3) % 3;
            if (f < 2) {
                if (x.g_tpos[t]) x.g_tpos[t][(long)b * 2 + f] = g[k];
            } else if (x.g_trot[t]) {
                x.g_trot[t][b] = g[k];
            }
        } else if (x.g_ang) {
            x.g_ang[(long)b * x.R + (c - 3 - 3 * x.nt)] = g[k];
        }
    }
}

__global__ void __launch_bounds__(64) k_ray_vjp(RayVjpArgs x) {
    const long t = (long)blockIdx.x * 64 + threadIdx.x;
    if (t >= (long)x.B * x.n_blocks) return;
    ray_vjp_env(x, (int)(t / x.n_blocks), (int)(t % x.n_blocks) * kTangents);
}

}  // namespace

extern "C" int32_t vmas_distance_vjp(int32_t device, int32_t batch, int32_t kind, const VmasShapeRef* a,
                                     const VmasShapeRef* b, const float* test_point, int32_t tp_s0, int32_t tp_s1,
                                     const float* grad_out, float* grad_a_pos, float* grad_a_rot, float* grad_b_pos,
                                     float* grad_b_rot, float* grad_point, void* stream) {
    if (!a || batch <= 0 || !grad_out || (kind == VMAS_DIST_POINT && !test_point) || (kind == VMAS_DIST_PAIR && !b) ||
        (kind != VMAS_DIST_POINT && kind != VMAS_DIST_PAIR))
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_distance_vjp: bad arguments");
    DistArgs x{};
    x.a = *a;
    if (b) x.b = *b;
    x.kind = kind;
    x.has_b = b != nullptr;
    x.batch = batch;
    x.tp = test_point;
    x.tp_s0 = tp_s0;
    x.tp_s1 = tp_s1;
    x.gout = grad_out;
    x.ga_pos = grad_a_pos;
    x.ga_rot = grad_a_rot;
    x.gb_pos = grad_b_pos;
    x.gb_rot = grad_b_rot;
    x.gtp = grad_point;
    if (device < 0) {
        for (int e = 0; e < batch; ++e) dist_vjp_env(x, e);
        return VMAS_OK;
    }
    VMAS_AUX_HIP(hipSetDevice(device));
    hipLaunchKernelGGL(k_dist_vjp, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream, x);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

extern "C" int32_t vmas_cast_rays_vjp(int32_t device, int32_t batch, int32_t n_rays, const float* origin, int32_t o_s0,
                                      int32_t o_s1, const float* angles, int32_t a_s0, int32_t a_s1, const float* rot,
                                      int32_t r_s0, const VmasRayTarget* targets, int32_t n_targets, float max_range,
                                      const float* grad_out, float* grad_origin, float* grad_rot, float* grad_angles,
                                      float* const* grad_target_pos, float* const* grad_target_rot, void* stream_) {
    if (batch <= 0 || n_rays <= 0 || n_targets < 0 || (n_targets > 0 && !targets) || !origin || !angles || !grad_out)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_cast_rays_vjp: bad arguments");
    RayVjpArgs x{};
    x.nt = n_targets;
    x.B = batch;
    x.R = n_rays;
    x.n_in = 3 + 3 * n_targets + n_rays;
    x.n_blocks = (x.n_in + kTangents - 1) / kTangents;
    x.origin = origin;
    x.o_s0 = o_s0;
    x.o_s1 = o_s1;
    x.ang = angles;
    x.a_s0 = a_s0;
    x.a_s1 = a_s1;
    x.rot = rot;
    x.r_s0 = r_s0;
    x.max_range = max_range;
    x.gout = grad_out;
    x.g_origin = grad_origin;
    x.g_rot = grad_rot;
    x.g_ang = grad_angles;
    if (device < 0) {
        x.tg = targets;
        x.g_tpos = grad_target_pos;
        x.g_trot = grad_target_rot;
        for (int e = 0; e < batch; ++e)
            for (int k = 0; k < x.n_blocks; ++k) ray_vjp_env(x, e, k * kTangents);
        return VMAS_OK;
    }
    hipStream_t stream = (hipStream_t)stream_;
    VMAS_AUX_HIP(hipSetDevice(device));
    const size_t nt = (size_t)std::max(n_targets, 1);
    const size_t bytes = sizeof(VmasRayTarget) * nt + 2 * sizeof(float*) * nt;
    char* d = nullptr;
    VMAS_AUX_HIP(hipMallocAsync((void**)&d, bytes, stream));
    std::vector<char> h(bytes, 0);
    if (n_targets) memcpy(h.data(), targets, sizeof(VmasRayTarget) * n_targets);
    float** hp = reinterpret_cast<float**>(h.data() + sizeof(VmasRayTarget) * nt);
    for (int t = 0; t < n_targets; ++t) {
        hp[t] = grad_target_pos ? grad_target_pos[t] : nullptr;
        hp[nt + t] = grad_target_rot ? grad_target_rot[t] : nullptr;
    }
    VMAS_AUX_HIP(hipMemcpyAsync(d, h.data(), bytes, hipMemcpyHostToDevice, stream));
    x.tg = reinterpret_cast<const VmasRayTarget*>(d);
    x.g_tpos = reinterpret_cast<float* const*>(d + sizeof(VmasRayTarget) * nt);
    x.g_trot = x.g_tpos + nt;
    hipLaunchKernelGGL(k_ray_vjp, dim3((unsigned)(((long)batch * x.n_blocks + 63) / 64)), dim3(64), 0, stream, x);
    const hipError_t le = hipGetLastError();
    VMAS_AUX_HIP(hipFreeAsync(d, stream));
    vmas_aux::note_host_wait();
    VMAS_AUX_HIP(hipStreamSynchronize(stream));  // (the host table must outlive its upload)
    if (le != hipSuccess) return vmas_aux::fail(VMAS_E_HIP, "vmas_cast_rays_vjp: %s", hipGetErrorString(le));
    return VMAS_OK;
}

extern "C" int32_t vmas_world_step_vjp(const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                                       const VmasPairDesc* pairs, const VmasJointDesc* joints, const VmasStepIO* io,
                                       const VmasStepIO* grad_out, const VmasGradIO* grad_in, void* stream_) {
    if (!cfg || !entities || !io || !grad_out || !grad_in || cfg->n_entities <= 0 || cfg->batch <= 0 ||
        io->substeps <= 0 || (cfg->n_pairs > 0 && !pairs) || (cfg->n_joints > 0 && !joints))
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_world_step_vjp: bad arguments");
    const int E = cfg->n_entities, A = cfg->n_agents, P = cfg->n_pairs, B = cfg->batch, S = io->substeps;
    const int Wd = std::max(1, (P + 31) / 32), nwords = S * Wd;
    if (nwords > 256) return vmas_aux::fail(VMAS_E_INVALID, "vmas_world_step_vjp: substeps x ceil(pairs/32) > 256");
    // contribution lists in pair order (as vmas_world_create)
    std::vector<int32_t> dyn, off, items;
    for (int e = 0; e < E; ++e)
        if (entities[e].flags & (VMAS_F_MOVABLE | VMAS_F_ROTATABLE)) dyn.push_back(e);
    off.push_back(0);
    for (int e : dyn) {
        for (int p = 0; p < P; ++p)
            for (int side = 0; side < 2; ++side) {
                if ((side ? pairs[p].eb : pairs[p].ea) != e) continue;
                int tq = 1;
                if (pairs[p].cls == VMAS_PAIR_SS) tq = 0;
                if ((pairs[p].cls == VMAS_PAIR_LS || pairs[p].cls == VMAS_PAIR_BS) && side == 1) tq = 0;
                items.push_back((p << 2) | (side << 1) | tq);
            }
        off.push_back((int32_t)items.size());
    }
    const int n_in = 6 * E + 3 * A, n_blocks = (n_in + kTangents - 1) / kTangents;
    const size_t wsd = work_duals(E, A, P);
    const bool batch_bp = io->broadphase == VMAS_BROADPHASE_BATCH;
    std::vector<uint32_t> mask(nwords, 0u), R(nwords), Z(nwords);
    // all candidate pairs active (the forward's pass 0 / broadphase "env")
    for (int p = 0; p < P; ++p)
        for (int s = 0; s < S; ++s) mask[s * Wd + (p >> 5)] |= 1u << (p & 31);

    if (cfg->device < 0) {  // host backend: per env, sequentially per thread chunk
        Tables T{*cfg, entities, pairs, joints, dyn.data(), off.data(), items.data(), (int)dyn.size(), Wd};
        const int nthreads = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
        auto run = [&](auto&& body, int n) {
            std::vector<std::thread> th;
            for (int t = 0; t < nthreads; ++t)
                th.emplace_back([&, t] {
                    std::vector<Dual> ws(wsd);
                    for (int i = t; i < n; i += nthreads) body(i, ws.data());
                });
            for (auto& x : th) x.join();
        };
        for (int it = 0; batch_bp && it < S + 2; ++it) {  // the forward's fixed point (R/Z rule)
            std::vector<std::vector<uint32_t>> rr(B, std::vector<uint32_t>(nwords, 0u)), zz = rr;
            run([&](int b, Dual* ws) { dual_step_env(T, *io, mask.data(), b, 0, ws, false, nullptr, nullptr, rr[b].data(), zz[b].data()); }, B);
            std::fill(R.begin(), R.end(), 0u);
            std::fill(Z.begin(), Z.end(), 0u);
            for (int b = 0; b < B; ++b)
                for (int i = 0; i < nwords; ++i) {
                    R[i] |= rr[b][i];
                    Z[i] |= zz[b][i];
                }
            bool viol = false;
            for (int i = 0; i < nwords; ++i)
                if ((mask[i] & ~R[i] & Z[i]) | (~mask[i] & R[i])) viol = true;
            if (!viol) break;
            mask = R;
        }
        run([&](int t, Dual* ws) {
            const int b = t / n_blocks, col0 = (t % n_blocks) * kTangents;
            float g[kTangents];
            dual_step_env(T, *io, mask.data(), b, col0, ws, true, grad_out, g, nullptr, nullptr);
            scatter(*grad_in, E, A, B, b, col0, n_in, g);
        }, B * n_blocks);
        return VMAS_OK;
    }

    // GPU: device copies of the tables and pointer arrays, a dual workspace per thread
    hipStream_t stream = (hipStream_t)stream_;
    VMAS_AUX_HIP(hipSetDevice(cfg->device));
    auto bytes = [](size_t n, size_t a) { return (n + a - 1) / a * a; };
    const size_t n_threads = std::max<size_t>((size_t)B, (size_t)B * n_blocks);
    size_t o = 0;
    const size_t o_ed = o; o += bytes(sizeof(VmasEntityDesc) * E, 256);
    const size_t o_pd = o; o += bytes(sizeof(VmasPairDesc) * std::max(P, 1), 256);
    const size_t o_jd = o; o += bytes(sizeof(VmasJointDesc) * std::max(cfg->n_joints, 1), 256);
    const size_t o_dyn = o; o += bytes(4 * std::max<size_t>(dyn.size(), 1), 256);
    const size_t o_off = o; o += bytes(4 * off.size(), 256);
    const size_t o_it = o; o += bytes(4 * std::max<size_t>(items.size(), 1), 256);
    const size_t o_eio = o; o += bytes(sizeof(VmasEntityIO) * E, 256);
    const size_t o_aio = o; o += bytes(sizeof(VmasAgentIO) * std::max(A, 1), 256);
    const size_t o_jio = o; o += bytes(sizeof(VmasJointIO) * std::max(cfg->n_joints, 1), 256);
    const size_t o_gptr = o; o += bytes(sizeof(float*) * (4 * E + 2 * std::max(A, 1)), 256);
    const size_t o_mask = o; o += bytes(4 * 3 * nwords, 256);
    const size_t o_ws = o; o += sizeof(Dual) * wsd * n_threads;
    char* d = nullptr;
    VMAS_AUX_HIP(hipMallocAsync((void**)&d, o, stream));
    std::vector<char>& h = g_scratch;
    h.assign(o_ws, 0);
    memcpy(h.data() + o_ed, entities, sizeof(VmasEntityDesc) * E);
    if (P) memcpy(h.data() + o_pd, pairs, sizeof(VmasPairDesc) * P);
    if (cfg->n_joints) memcpy(h.data() + o_jd, joints, sizeof(VmasJointDesc) * cfg->n_joints);
    if (!dyn.empty()) memcpy(h.data() + o_dyn, dyn.data(), 4 * dyn.size());
    memcpy(h.data() + o_off, off.data(), 4 * off.size());
    if (!items.empty()) memcpy(h.data() + o_it, items.data(), 4 * items.size());
    memcpy(h.data() + o_eio, io->entities, sizeof(VmasEntityIO) * E);
    if (A) memcpy(h.data() + o_aio, io->agents, sizeof(VmasAgentIO) * A);
    if (cfg->n_joints && io->joints) memcpy(h.data() + o_jio, io->joints, sizeof(VmasJointIO) * cfg->n_joints);
    float** gp = reinterpret_cast<float**>(h.data() + o_gptr);
    for (int e = 0; e < E; ++e) {
        gp[e] = grad_in->pos[e];
        gp[E + e] = grad_in->vel[e];
        gp[2 * E + e] = grad_in->rot[e];
        gp[3 * E + e] = grad_in->ang_vel[e];
    }
    for (int a = 0; a < A; ++a) {
        gp[4 * E + a] = grad_in->force[a];
        gp[4 * E + A + a] = grad_in->torque[a];
    }
    memcpy(h.data() + o_mask, mask.data(), 4 * nwords);
    VMAS_AUX_HIP(hipMemcpyAsync(d, h.data(), o_ws, hipMemcpyHostToDevice, stream));
    GradArgs ga{};
    ga.T = Tables{*cfg, (const VmasEntityDesc*)(d + o_ed), (const VmasPairDesc*)(d + o_pd),
                  (const VmasJointDesc*)(d + o_jd), (const int32_t*)(d + o_dyn), (const int32_t*)(d + o_off),
                  (const int32_t*)(d + o_it), (int)dyn.size(), Wd};
    ga.io = *io;
    ga.io.entities = (const VmasEntityIO*)(d + o_eio);
    ga.io.agents = (const VmasAgentIO*)(d + o_aio);
    ga.io.joints = (cfg->n_joints && io->joints) ? (const VmasJointIO*)(d + o_jio) : nullptr;
    ga.gout = *grad_out;
    float** dgp = reinterpret_cast<float**>(d + o_gptr);
    ga.gio = VmasGradIO{dgp, dgp + E, dgp + 2 * E, dgp + 3 * E, dgp + 4 * E, dgp + 4 * E + A};
    uint32_t* dmask = reinterpret_cast<uint32_t*>(d + o_mask);
    ga.mask = dmask;
    ga.R = dmask + nwords;
    ga.Z = dmask + 2 * nwords;
    ga.ws = reinterpret_cast<Dual*>(d + o_ws);
    ga.n_in = n_in;
    ga.n_blocks = n_blocks;
    int32_t rc = VMAS_OK;
    for (int it = 0; batch_bp && it < S + 2; ++it) {  // the forward's fixed point (R/Z rule)
        VMAS_AUX_HIP(vmas_aux::fill_u32_async(ga.R, 0u, 2 * (size_t)nwords, stream));
        ga.value_pass = true;
        hipLaunchKernelGGL(k_grad, dim3((B + 63) / 64), dim3(64), 0, stream, ga);
        VMAS_AUX_HIP(hipGetLastError());
        VMAS_AUX_HIP(hipMemcpyAsync(R.data(), ga.R, 4 * nwords, hipMemcpyDeviceToHost, stream));
        VMAS_AUX_HIP(hipMemcpyAsync(Z.data(), ga.Z, 4 * nwords, hipMemcpyDeviceToHost, stream));
        vmas_aux::note_host_wait();
        VMAS_AUX_HIP(hipStreamSynchronize(stream));
        bool viol = false;
        for (int i = 0; i < nwords; ++i)
            if ((mask[i] & ~R[i] & Z[i]) | (~mask[i] & R[i])) viol = true;
        if (!viol) break;
        mask = R;
        VMAS_AUX_HIP(hipMemcpyAsync(dmask, mask.data(), 4 * nwords, hipMemcpyHostToDevice, stream));
    }
    ga.value_pass = false;
    hipLaunchKernelGGL(k_grad, dim3((unsigned)((n_threads + 63) / 64)), dim3(64), 0, stream, ga);
    if (hipGetLastError() != hipSuccess) rc = vmas_aux::fail(VMAS_E_HIP, "vmas_world_step_vjp: launch failed");
    VMAS_AUX_HIP(hipFreeAsync(d, stream));
    vmas_aux::note_host_wait();
    VMAS_AUX_HIP(hipStreamSynchronize(stream));  // (the host copies above must outlive the uploads)
    return rc;
}
