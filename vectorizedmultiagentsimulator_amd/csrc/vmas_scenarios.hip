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

}  // extern "C"
