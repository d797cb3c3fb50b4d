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

}  // namespace vmas
