// vmas_scenarios.hip -- fused observation / reward / done programs of the benchmark scenarios
// (SURVEY.md §8(f) row 4), gfx950 kernels + C ABI.
//
// The reference computes a scenario's per-step outputs as an eager tensor program: balance's
// rewards, observations and dones (balance.py:222-262) are ~37 small kernels per step, each a few
// microseconds of launch latency for a few hundred KB of traffic -- more GPU time than the physics
// step itself.  Each entry point here computes one scenario's program in ONE launch, one thread
// per environment, with the reference's fp32 operations in the reference's order (no FMA
// contraction: -ffp-contract=off as the engine; norms as torch.linalg.vector_norm of a length-2
// vector; `%` as torch.remainder; is_overlapping / get_distance as vmas_query.hpp).  The host
// side (the restated scenario) keeps every attribute the reference's program leaves behind.
#include <hip/hip_runtime.h>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"
#include "vmas_query.hpp"

using namespace vmas;

namespace {

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

// balance.py:205-262 (restated in scenarios/balance.py): reward of the first agent (on-the-ground
// test, package-goal distance, ground / position rewards and the global shaping update), every
// agent's reward (ground_rew + pos_rew), every agent's 16-entry observation, and done
// (on_the_ground + is_overlapping(package, goal)).  Grid: x = 64-env groups, y = part: 0 the
// reward / done part, 1 + i agent i's observation (one 64-thread workgroup per (group, part): at
// 32 768 envs 512 x 5 workgroups instead of 128 x 1, whose long per-thread chains -- the box-line
// distance -- left half the chip idle and took 16 us).
__global__ void __launch_bounds__(64) k_balance(VmasBalanceIO io) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    const int part = blockIdx.y;
    const V2 pkg = ref_pos(io.package, b), goal = ref_pos(io.goal, b);
    if (part == 0) {
        bool og = false;
        if (io.what & VMAS_SCN_REWARD) {
            // compute_on_the_ground: is_overlapping(line, floor) + is_overlapping(package, floor)
            // (canonical (box, line) / (box, sphere) branches, core.py:1932-1968)
            og = (dist_pair(io.floor, io.line, b) < 0.f) || overlap_box_sphere(io.floor, io.package, b);
            io.on_the_ground[b] = og ? 1 : 0;
            const float dist = norm(pkg - goal);  // vector_norm(package.pos - goal.pos, dim=1)
            io.package_dist[b] = dist;
            const float ground = og ? io.fall_reward : 0.f;  // zeros, masked_fill_(on_the_ground, fall)
            io.ground_rew[b] = ground;
            const float gs = dist * io.shaping_factor;
            const float pos_rew = io.global_shaping[(long)b * io.gs_s0] - gs;
            io.global_shaping_out[b] = gs;
            if (io.pos_rew_prev) io.pos_rew_prev[b] = 0.f;  // pos_rew[:] = 0 on the tensor being replaced
            io.pos_rew[b] = pos_rew;
            const float r = ground + pos_rew;  // reward(agent) = ground_rew + pos_rew
            for (int i = 0; i < io.n_agents; ++i) io.rewards[i][b] = r;
        } else if (io.what & VMAS_SCN_DONE) {
            og = io.on_the_ground[b] != 0;
        }
        if (io.what & VMAS_SCN_DONE)  // done = on_the_ground + is_overlapping(package, goal)
            io.done[b] = (og || dist_pair(io.package, io.goal, b) < 0.f) ? 1 : 0;
        return;
    }
    // part 1 + i: agent i's observation
    const int i = part - 1;
    const V2 lpos = ref_pos(io.line, b), pv = ld_vec2(io.package_vel, b), lv = ld_vec2(io.line_vel, b);
    const float law = ld_vec1(io.line_ang_vel, b);
    const float lrot = torch_remainder(ref_rot(io.line, b), io.pi);
    const V2 pg = pkg - goal;
    const V2 p = ld_vec2(io.agent_pos[i], b), v = ld_vec2(io.agent_vel[i], b);
    const V2 dp = p - pkg, dl = p - lpos;
    float4* dst = reinterpret_cast<float4*>(io.obs[i] + (long)b * 16);
    dst[0] = make_float4(p.x, p.y, v.x, v.y);
    dst[1] = make_float4(dp.x, dp.y, dl.x, dl.y);
    dst[2] = make_float4(pg.x, pg.y, pv.x, pv.y);
    dst[3] = make_float4(lv.x, lv.y, law, lrot);
}

// The flocking separation term sums n floats in the order of torch's .mean(-1) over a contiguous
// last dim: `acc` strided accumulators (acc_i = x_i + x_{i+acc} + ...), combined by an
// adjacent-pair tree ((a0+a1)+(a2+a3))...  The host probes which accumulator count torch uses on
// this device for n (simulator/_fused.py reduce_order; measured on MI355X / ROCm 7.2: the largest
// power of two <= n) and passes it as sum_mode.

// flocking.py:149-206 (restated in scenarios/flocking.py).  Grid: x = 64-env groups, y = (policy
// agent p, part): part 0 is p's reward and the first six observation entries, part 1 + r is ray r
// of p's LIDAR (one (env, agent, ray) per thread: a thread per (env, agent) casting all 12 rays
// left the chip latency-bound at 3 waves per SIMD, 95 us per step at 32 768 envs x 8 agents).
// Positions are loaded up front with independent loads (unrolled over the static bounds).
__global__ void __launch_bounds__(64) k_flocking(VmasFlockingIO io) {
    constexpr int MA = VMAS_FLOCK_MAX_AGENTS, MT = VMAS_SCN_MAX_RAY_TARGETS;
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    const int parts = (io.what & VMAS_SCN_OBS) ? 1 + io.n_rays : 1;
    const int p = blockIdx.y / parts, part = blockIdx.y - p * parts, k = io.policy[p], na = io.n_all;
    const V2 pk = ref_pos(io.agents[k], b);
    const int W = 6 + io.n_rays;
    if (part > 0) {  // LIDAR ray r: Lidar.measure = World.cast_rays(angles + agent rot) (cast_one)
        const int r = part - 1, nt = io.n_ray_targets;
        V2 T[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const VmasRayTarget& x = io.ray_targets[t];
            T[t] = t < nt ? mk(x.pos[(long)b * x.pos_s0], x.pos[(long)b * x.pos_s0 + x.pos_s1]) : mk(0.f, 0.f);
        }
        const float a = io.angles[p][(long)b * io.ang_s0[p] + (long)r * io.ang_s1[p]] + ld_vec1(io.rot[p], b);
        const float dc = cosf(a), ds = sinf(a);
        float best = io.max_range;
#pragma unroll
        for (int t = 0; t < MT; ++t)  // (sphere targets: checked by the host entry point)
            if (t < nt) best = tmin(best, ray_sphere(pk, dc, ds, T[t], io.ray_targets[t].radius, io.max_range));
        io.lidar[p][(long)b * io.n_rays + r] = best;
        io.obs[p][(long)b * W + 6 + r] = best;
        return;
    }
    V2 P[MA];
#pragma unroll
    for (int j = 0; j < MA; ++j) P[j] = j < na ? ref_pos(io.agents[j], b) : mk(0.f, 0.f);
    if (io.what & VMAS_SCN_REWARD) {
        if (p == 0) io.t[b] = io.t[b] + 1.f;  // self.t += 1 (first policy agent's call)
        // collision rewards: pairs (i < j) of world.agents in loop order; agent k meets them
        // as j = 0 .. k-1, k+1 .. n-1 (get_distance of spheres: |p_lo - p_hi| - r_lo - r_hi)
        float cr = 0.f;  // a.collision_rew[:] = 0
        if (io.collide_reward_on) {
#pragma unroll
            for (int j = 0; j < MA; ++j) {
                if (j >= na || j == k) continue;
                const int lo = j < k ? j : k, hi = j < k ? k : j;
                const V2 plo = j < k ? P[j] : pk, phi = j < k ? pk : P[j];
                const float d = (norm(plo - phi) - io.agents[lo].radius) - io.agents[hi].radius;
                cr = cr + ((d <= io.min_collision_distance) ? io.collision_reward : 0.f);
            }
            io.collision_rew[p][b] = cr;
        } else {
            cr = io.collision_rew[p][b];
        }
        // separation: (stack(|p_k - p_j| for j != k) - desired).pow(2).mean(-1) * factor, summed
        // in torch's order (static register indices: element n goes to accumulator n % acc, every
        // value >= +0 so 0 + e == e)
        float y[MA];
#pragma unroll
        for (int i = 0; i < MA; ++i) y[i] = 0.f;
        int n = 0;
        const int accm = io.sum_mode - 1;
#pragma unroll
        for (int j = 0; j < MA; ++j) {
            if (j >= na || j == k) continue;
            const float d = norm(pk - P[j]) - io.desired_distance;
            const float e = d * d;
            const int slot = n & accm;
#pragma unroll
            for (int i = 0; i < MA; ++i)
                if (i == slot) y[i] = y[i] + e;
            ++n;
        }
        const int m = n < io.sum_mode ? n : io.sum_mode;
#pragma unroll
        for (int w = 1; w < MA; w *= 2)
#pragma unroll
            for (int i = 0; i + w < MA; i += 2 * w)
                if (i + w < m) y[i] = y[i] + y[i + w];
        const float shaping = (y[0] * (1.f / (float)n)) * io.dist_shaping_factor;
        const float dr = io.shaping_in[p][b] - shaping;
        io.shaping_out[p][b] = shaping;
        io.dist_rew[p][b] = dr;
        io.rewards[p][b] = cr + dr;
    }
    if (io.what & VMAS_SCN_OBS) {
        const V2 v = ld_vec2(io.vel[p], b);
        V2 tp = mk(0.f, 0.f);
#pragma unroll
        for (int j = 0; j < MA; ++j)
            if (j == io.target) tp = P[j];
        float* o = io.obs[p] + (long)b * W;
        o[0] = pk.x;
        o[1] = pk.y;
        o[2] = v.x;
        o[3] = v.y;
        o[4] = pk.x - tp.x;
        o[5] = pk.y - tp.y;
    }
}

}  // namespace

extern "C" {

int32_t vmas_balance_outputs(int32_t device, const VmasBalanceIO* io, void* stream) {
    if (!io || device < 0 || io->batch <= 0 || io->n_agents < 0 || io->n_agents > VMAS_SCN_MAX_AGENTS)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_balance_outputs: bad arguments");
    if (io->package.shape != VMAS_SPHERE || io->goal.shape != VMAS_SPHERE || io->line.shape != VMAS_LINE ||
        io->floor.shape != VMAS_BOX)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_balance_outputs: unexpected entity shapes");
    VMAS_AUX_HIP(hipSetDevice(device));
    const int parts = 1 + ((io->what & VMAS_SCN_OBS) ? io->n_agents : 0);
    hipLaunchKernelGGL(k_balance, dim3((io->batch + 63) / 64, parts), dim3(64), 0, (hipStream_t)stream, *io);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_flocking_outputs(int32_t device, const VmasFlockingIO* io, void* stream) {
    if (!io || device < 0 || io->batch <= 0 || io->n_all < 2 || io->n_all > VMAS_FLOCK_MAX_AGENTS || io->n_policy < 1 ||
        io->n_policy > io->n_all || io->target < 0 || io->target >= io->n_all || io->n_rays < 0 ||
        io->n_ray_targets < 0 || io->n_ray_targets > VMAS_SCN_MAX_RAY_TARGETS || io->sum_mode < 1 || io->sum_mode > VMAS_FLOCK_MAX_AGENTS || (io->sum_mode & (io->sum_mode - 1)))
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_flocking_outputs: bad arguments");
    for (int i = 0; i < io->n_all; ++i)
        if (io->agents[i].shape != VMAS_SPHERE) return vmas_aux::fail(VMAS_E_INVALID, "vmas_flocking_outputs: agent %d is not a sphere", i);
    for (int t = 0; t < io->n_ray_targets; ++t)
        if (io->ray_targets[t].shape != VMAS_SPHERE)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_flocking_outputs: LIDAR target %d is not a sphere", t);
    for (int p = 0; p < io->n_policy; ++p)
        if (io->policy[p] < 0 || io->policy[p] >= io->n_all)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_flocking_outputs: bad policy index %d", p);
    VMAS_AUX_HIP(hipSetDevice(device));
    static_assert(sizeof(VmasFlockingIO) <= 4096, "kernel argument block");
    const int parts = (io->what & VMAS_SCN_OBS) ? 1 + io->n_rays : 1;
    hipLaunchKernelGGL(k_flocking, dim3((io->batch + 63) / 64, io->n_policy * parts), dim3(64), 0, (hipStream_t)stream, *io);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

}  // extern "C"
