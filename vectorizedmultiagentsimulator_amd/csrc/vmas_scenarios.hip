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
#include "vmas_programs.hpp"
#include "vmas_query.hpp"

using namespace vmas;

namespace {

// __sinf / __cosf (v_sin_f32 / v_cos_f32) take the angle in revolutions: x * (1 / 2 pi) rounds to
// |x| * 2^-24 rad, i.e. 1e-6 rad at 16 rad (the LIDAR certification's turn, tests/_parity.py) and
// 1.5e-5 rad at 256.  Below this bound the fast LIDAR programs use them; above it ocml's
// range-reduced sincosf.  (Ray angles are the sensor's [0, 2 pi) plus the agent's rotation.)
constexpr float kFastTrigMaxAngle = 16.f;

// balance.py:205-262 (restated in scenarios/balance.py): reward of the first agent (on-the-ground
// test, package-goal distance, ground / position rewards and the global shaping update), every
// agent's reward (ground_rew + pos_rew), every agent's 16-entry observation, and done
// (on_the_ground + is_overlapping(package, goal)).  Grid: x = 64-env groups, y = part, 4 waves
// per workgroup.  Part 0 is the reward / done part: the (floor, line) box-line distance of the
// on-the-ground test is split over the 4 waves, one box side each (bl_part), and wave 0 picks the
// first strict minimum over the sides in order, as closest_line_box does, then finishes.  Parts
// 1 + k are the observations of agents 4k .. 4k + 3, one per wave.  (One 64-thread workgroup per
// (group, part), the box-line distance in one chain: 11 us per step at 32 768 envs, the chain's
// latency at two waves per CU; before that 128 x 1 workgroups took 16 us.)
__global__ void __launch_bounds__(256) k_balance(VmasBalanceIO io_arg) {
    VMAS_PROGRAM_ARGS(VmasBalanceIO, io_arg);
    __shared__ float Q[kBalQRows * 64];  // the box queries' sides (vmas_programs.hpp bal_q)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x * 64 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    const OutDelta od = load_out_delta(io);
    if (blockIdx.y == 0) {
        if (!(io.what & VMAS_SCN_REWARD)) {
            if (wave != 0 || !valid || !(io.what & VMAS_SCN_DONE)) return;
            bal_done(io, b, io.on_the_ground[b] != 0, od);
            return;
        }
        const BalPre pre = wave == 0 ? bal_preload(io, bb) : BalPre{0.f, mk(0.f, 0.f)};
        bal_side(io, bb, wave, lane, Q);  // side `wave` of the floor's two box queries
        __syncthreads();
        if (wave != 0 || !valid) return;
        bal_reward(io, b, lane, od, Q, pre);
        return;
    }
    // agent i's observation
    const int i = (blockIdx.y - 1) * 4 + wave;
    if (i >= io.n_agents || !valid) return;
    bal_obs(io, b, i, od);
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
// Part 0 of policy agent p in env b: the reward block (REWARD) and the first six observation
// entries (OBS).
struct FlockHead {
    float v[6];
};
// IO: the argument block by value, or (k_flocking_fast) read in place through the kernel
// argument segment pointer -- structs copied out before use, see k_flocking_fast.
template <class IO>
__device__ __forceinline__ FlockHead flock_part0(IO& io, int b, int p, const OutDelta& od, bool ret = false) {
    FlockHead h{};
    constexpr int MA = VMAS_FLOCK_MAX_AGENTS;
    const int k = io.policy[p], na = io.n_all;
    const VmasShapeRef ak = io.agents[k];
    const V2 pk = ref_pos(ak, b);
    const int W = 6 + io.n_rays;
    V2 P[MA];
#pragma unroll
    for (int j = 0; j < MA; ++j) {
        const VmasShapeRef aj = io.agents[j];
        P[j] = j < na ? ref_pos(aj, b) : mk(0.f, 0.f);
    }
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
        moved(io.rewards[p], od.rew)[b] = cr + dr;
    }
    if (io.what & VMAS_SCN_OBS) {
        const VmasVec vp = io.vel[p];
        const V2 v = ld_vec2(vp, b);
        V2 tp = mk(0.f, 0.f);
#pragma unroll
        for (int j = 0; j < MA; ++j)
            if (j == io.target) tp = P[j];
        h = FlockHead{{pk.x, pk.y, v.x, v.y, pk.x - tp.x, pk.y - tp.y}};
        if (!ret) {
            float* o = moved(io.obs[p], od.obs) + (long)b * W;
#pragma unroll
            for (int i = 0; i < 6; ++i) o[i] = h.v[i];
        }
    }
    return h;
}

// flocking.py:149-206 (restated in scenarios/flocking.py), LIDAR bit-identical to k_cast_rays
// (io.fast_lidar == 0).  Grid: x = 64-env groups, y = (policy agent p, part): part 0 is p's
// reward and the first six observation entries, part 1 + r is ray r of p's LIDAR (one (env,
// agent, ray) per thread: a thread per (env, agent) casting all 12 rays with the exact ray code
// left the chip latency-bound at 3 waves per SIMD, 95 us per step at 32 768 envs x 8 agents).
// Positions are loaded up front with independent loads (unrolled over the static bounds).
__global__ void __launch_bounds__(64) k_flocking(VmasFlockingIO io) {
    constexpr int MT = VMAS_SCN_MAX_RAY_TARGETS;
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    const int parts = (io.what & VMAS_SCN_OBS) ? 1 + io.n_rays : 1;
    const int p = blockIdx.y / parts, part = blockIdx.y - p * parts, k = io.policy[p];
    const OutDelta od = load_out_delta(io);
    if (part == 0) {
        flock_part0(io, b, p, od);
        return;
    }
    // LIDAR ray r: Lidar.measure = World.cast_rays(angles + agent rot) (cast_one)
    const V2 pk = ref_pos(io.agents[k], b);
    const int W = 6 + io.n_rays;
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
    moved(io.obs[p], od.obs)[(long)b * W + 6 + r] = best;
}

// The same program with the fast LIDAR (io.fast_lidar, the default): the ray-sphere distance in
// its direct form (ray_sphere_fast), hardware sin / cos / sqrt.  Grid: x = 64-env groups, y =
// groups of 4 policy agents; a wave per (64 envs, agent): its reward / head (flock_part0) and all
// of its rays (angles and targets loaded up front), the observation rows staged in LDS and
// written out as contiguous blocks (a lane per env writes 4-byte values 4 * W bytes apart
// otherwise: twice the output bytes reached HBM).  History (32 768 envs x 8 agents): a thread per
// ray of the exact program, 53 us; a thread per (env, agent) with ocml sincosf and per-ray angle
// loads, 89 us; waves over ray subsets with wave 0 also doing the reward, 48 us.
constexpr int kFlockFastRays = 16, kFlockFastTargets = 8, kFlockFastW = 6 + kFlockFastRays;
#ifdef __HIP_DEVICE_COMPILE__
typedef const VmasFlockingIO __attribute__((address_space(4))) KFlockingIO;  // (the device pass)
#else
typedef const VmasFlockingIO KFlockingIO;  // (the host pass only parses the kernel)
#endif
// NR / NT > 0: the ray and target counts fixed at compile time (flocking's 12 rays; instantiated
// for 1..8 targets): every ray unrolled with its angle in a register, so the rays' chains
// interleave (the rolled loop left each wave one ray's dependent chain at a time, at 4 waves per
// SIMD), no per-target branch, and the LIDAR row split by a constant.  Same operations per ray
// in the same order as the runtime form (bit-identical).
template <int NR, int NT>
__global__ void __launch_bounds__(256) k_flocking_fast(VmasFlockingIO io_arg) {
    constexpr int RM = NR > 0 ? NR : kFlockFastRays, TM = NT > 0 ? NT : kFlockFastTargets;
    // The argument block read in place (s_load from the kernel argument segment): indexed by the
    // wave's agent, the by-value parameter was copied to scratch (3.5 KiB per lane)
#ifdef __HIP_DEVICE_COMPILE__
    KFlockingIO& io = *(KFlockingIO*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)io_arg;
#else
    KFlockingIO& io = io_arg;
#endif
    __shared__ float S[4][64 * kFlockFastW];
    const int lane = (int)(threadIdx.x & 63u), w = (int)(threadIdx.x >> 6);
    // (p made wave-uniform for the compiler: indexing the argument block's arrays with a per-lane
    // index copies the whole 3.5 KiB block to scratch)
    const int g0 = (int)blockIdx.x * 64, b = g0 + lane;
    const int p = __builtin_amdgcn_readfirstlane((int)blockIdx.y * 4 + w);
    if (p >= io.n_policy) return;  // (wave-uniform; no workgroup barrier below)
    const bool valid = b < io.batch;
    const int nr = NR > 0 ? NR : io.n_rays, nt = NT > 0 ? NT : io.n_ray_targets, W = 6 + nr;
    const int bb = valid ? b : io.batch - 1;
    const int row = lane * W;
    const OutDelta od = load_out_delta(io);
    if (io.what & VMAS_SCN_OBS) {
        // loads first (independent): angles, rotation, position, targets
        const float* ang = io.angles[p] + (long)bb * io.ang_s0[p];
        const int as1 = io.ang_s1[p];
        float A[RM];
#pragma unroll
        for (int r = 0; r < RM; ++r) A[r] = r < nr ? ang[(long)r * as1] : 0.f;
        const VmasVec rv = io.rot[p];
        const float rot = ld_vec1(rv, bb);
        const VmasShapeRef ak = io.agents[io.policy[p]];
        const V2 pk = ref_pos(ak, bb);
        V2 T[TM];
        float R2[TM];
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            const float* xp = io.ray_targets[t].pos;
            const int s0 = io.ray_targets[t].pos_s0, s1 = io.ray_targets[t].pos_s1;
            const float rad = io.ray_targets[t].radius;
            T[t] = t < nt ? mk(xp[(long)bb * s0], xp[(long)bb * s0 + s1]) - pk : mk(0.f, 0.f);
            R2[t] = t < nt ? rad * rad : 0.f;
        }
        if (valid) {
            const FlockHead h = flock_part0(io, b, p, od, true);
#pragma unroll
            for (int i = 0; i < 6; ++i) S[w][row + i] = h.v[i];
        }
        // (loops fully unrolled with guarded bodies, never `break`: a partly unrolled loop indexes
        // A / T dynamically, which puts them in scratch)
        float C[TM];
#pragma unroll
        for (int t = 0; t < TM; ++t) C[t] = R2[t] - (T[t].x * T[t].x + T[t].y * T[t].y);
        if constexpr (NR > 0 && NT > 0) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float a = A[r] + rot;
                // hardware sin / cos (v_sin / v_cos_f32) below kFastTrigMaxAngle, ocml's
                // range-reduced sincosf above (see kFastTrigMaxAngle)
                float ds, dc;
                if (fabsf(a) < kFastTrigMaxAngle) {
                    ds = __sinf(a);
                    dc = __cosf(a);
                } else {
                    sincosf(a, &ds, &dc);
                }
                float best = io.max_range;
#pragma unroll
                for (int t = 0; t < NT; ++t) best = min_drop_nan(best, ray_sphere_fast_nan(T[t].x, T[t].y, C[t], dc, ds));
                S[w][row + 6 + r] = best;
            }
        } else {
            // rays in a rolled loop, targets unrolled inside (see k_discovery_obs_fast)
            // (the angles wait in the rays' own LDS slots: a register array indexed at run time
            // goes to scratch)
#pragma unroll
            for (int r = 0; r < RM; ++r)
                if (r < nr) S[w][row + 6 + r] = A[r] + rot;
#pragma unroll 1
            for (int r = 0; r < nr; ++r) {
                const float a = S[w][row + 6 + r];
                float ds, dc;
                if (fabsf(a) < kFastTrigMaxAngle) {
                    ds = __sinf(a);
                    dc = __cosf(a);
                } else {
                    sincosf(a, &ds, &dc);
                }
                float best = io.max_range;
#pragma unroll
                for (int t = 0; t < TM; ++t) {
                    if (t >= nt) continue;
                    best = min_drop_nan(best, ray_sphere_fast_nan(T[t].x, T[t].y, C[t], dc, ds));
                }
                S[w][row + 6 + r] = best;
            }
        }
        // the wave's rows out as contiguous blocks: obs [64 x W], the LIDAR [64 x nr]
        const int nv = io.batch - g0 < 64 ? io.batch - g0 : 64;
        float* obs = moved(io.obs[p], od.obs) + (long)g0 * W;
        for (int i = lane; i < nv * W; i += 64) obs[i] = S[w][i];
        float* lid = io.lidar[p] + (long)g0 * nr;
        for (int i = lane; i < nv * nr; i += 64) {
            const int e = i / nr;
            lid[i] = S[w][e * W + 6 + (i - e * nr)];
        }
    } else if (valid) {
        flock_part0(io, b, p, od);
    }
}

// flocking's scripted target: u = stack([cos(t / period), sin(t / period)], dim=1) (the division
// by a Python scalar as torch's divide kernel computes it: t * (1 / period) in fp32).
__global__ void __launch_bounds__(256) k_flocking_target(const float* t, int batch, float inv, float* u) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= batch) return;
    const float x = t[b] * inv;
    reinterpret_cast<float2*>(u)[b] = make_float2(cosf(x), sinf(x));
}

// transport.py:130-190 (restated in scenarios/transport.py).  Grid: x = 64-env groups, y = part:
// 0 the reward (every package) + done, 1 + i agent i's observation.  An observation part of a
// launch that also computes the reward recomputes on_goal (is_overlapping, deterministic) rather
// than reading part 0's output.
__global__ void __launch_bounds__(64) k_transport(VmasTransportIO io_arg) {
    VMAS_PROGRAM_ARGS(VmasTransportIO, io_arg);
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    const OutDelta od = load_out_delta(io);
    if (blockIdx.y == 0) tr_reward_done(io, b, od);
    else tr_obs(io, b, blockIdx.y - 1, od);
}

// (the REWARD launch, workgroup 0) a spawn channel's armed words into the step's respawn words
// (VmasDiscoveryIO.stage_in / stage_out): one PCIe read while the reward runs, instead of a clear
// kernel of the respawn's own on the step's critical path
template <class IO>
__device__ __forceinline__ void disc_stage(IO& io) {
    if (io.stage_in && blockIdx.x == 0 && threadIdx.x < 3)
        io.stage_out[threadIdx.x] = __hip_atomic_load(io.stage_in + threadIdx.x, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM);
}

// The optional reductions over the targets (VmasDiscoveryIO.covered_count / done): the count of
// covered targets (an integer sum: exact) and all() of the all-time covered flags.
template <class IO>
__device__ __forceinline__ void disc_reductions(IO& io, int b, int T, int n_cov) {
    if (io.covered_count) io.covered_count[b] = (int64_t)n_cov;
    if (io.done) {
        bool all = true;
        for (int j = 0; j < T; ++j) all = all && io.all_time[(long)b * T + j] != 0;
        moved(io.done, load_out_delta(io).done)[b] = all ? 1 : 0;
    }
}

// discovery.py:146-246 (restated in scenarios/discovery.py), REWARD part: one thread per env.
__global__ void __launch_bounds__(64) k_discovery_reward(VmasDiscoveryIO io) {
    constexpr int MA = VMAS_DISC_MAX_AGENTS, MT = VMAS_DISC_MAX_TARGETS;
    disc_stage(io);
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    const int A = io.n_agents, T = io.n_targets;
    V2 PA[MA], PT[MT];
#pragma unroll
    for (int i = 0; i < MA; ++i) PA[i] = i < A ? ld_vec2(io.pos[io.agent_entity[i]], b) : mk(0.f, 0.f);
#pragma unroll
    for (int j = 0; j < MT; ++j) PT[j] = j < T ? ld_vec2(io.pos[io.target_entity[j]], b) : mk(0.f, 0.f);
    // the stacks and the time reward
#pragma unroll
    for (int i = 0; i < MA; ++i)
        if (i < A) reinterpret_cast<float2*>(io.agents_pos)[(long)b * A + i] = make_float2(PA[i].x, PA[i].y);
#pragma unroll
    for (int j = 0; j < MT; ++j)
        if (j < T) reinterpret_cast<float2*>(io.targets_pos)[(long)b * T + j] = make_float2(PT[j].x, PT[j].y);
    if (io.time_int) reinterpret_cast<int64_t*>(io.time_rew)[b] = io.time_penalty_i;  // torch.full(int)
    else reinterpret_cast<float*>(io.time_rew)[b] = io.time_penalty;
    // torch.cdist (p = 2): sqrt(fl(fl(d0^2) + fl(d1^2))); per target the count of agents in range
    int cnt[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) cnt[j] = 0;
#pragma unroll
    for (int i = 0; i < MA; ++i) {
        if (i >= A) continue;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            if (j >= T) continue;
            const float d0 = PA[i].x - PT[j].x, d1 = PA[i].y - PT[j].y;
            const float d = sqrtf(d0 * d0 + d1 * d1);
            io.dists[((long)b * A + i) * T + j] = d;
            cnt[j] += (d < io.covering_range) ? 1 : 0;
        }
    }
    bool cov[MT];
    int n_cov = 0;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
        cov[j] = cnt[j] >= io.agents_per_target;
        if (j < T) {
            io.per_target[(long)b * T + j] = (int64_t)cnt[j];
            io.covered[(long)b * T + j] = cov[j] ? 1 : 0;
            n_cov += cov[j] ? 1 : 0;
        }
    }
    disc_reductions(io, b, T, n_cov);
    // agent_reward: covering_reward[:] = 0; += (count of covered targets in range) * coeff;
    // shared[:] = 0; += each agent's covering reward in agent order; halved where nonzero
    float shared = 0.f;
    float covr[MA];
#pragma unroll
    for (int i = 0; i < MA; ++i) {
        covr[i] = 0.f;
        if (i >= A) continue;
        int n = 0;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            if (j >= T) continue;
            const float d0 = PA[i].x - PT[j].x, d1 = PA[i].y - PT[j].y;
            n += (sqrtf(d0 * d0 + d1 * d1) < io.covering_range && cov[j]) ? 1 : 0;
        }
        covr[i] = 0.f + (float)n * io.covering_rew_coeff;
        io.covering[i][b] = covr[i];
        shared = shared + covr[i];
    }
    if (shared != 0.f) shared = shared / 2.f;
    io.shared[b] = shared;
#pragma unroll
    for (int i = 0; i < MA; ++i) {
        if (i >= A) continue;
        io.collision[i][b] = 0.f;  // collision_rew[:] = 0 (penalty 0: nothing added)
        const float cv = io.shared_reward ? shared : covr[i];
        moved(io.rewards[i], load_out_delta(io).rew)[b] = (0.f + cv) + io.time_penalty;  // collision_rew + covering_rew + time_rew
    }
}

// discovery.py:248-255, OBS part: one thread per (env, agent, part).
__global__ void __launch_bounds__(64) k_discovery_obs(VmasDiscoveryIO io) {
    constexpr int ME = VMAS_DISC_MAX_ENTITIES;
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    int rays = 0;
    for (int s = 0; s < io.n_lidars; ++s) rays += io.n_rays[s];
    const int parts = 1 + rays, a = blockIdx.y / parts, part = blockIdx.y - a * parts;
    const int self = io.agent_entity[a], W = 4 + rays;
    const V2 p = ld_vec2(io.pos[self], b);
    float* o = moved(io.obs[a], load_out_delta(io).obs) + (long)b * W;
    if (part == 0) {
        const V2 v = ld_vec2(io.vel[a], b);
        o[0] = p.x;
        o[1] = p.y;
        o[2] = v.x;
        o[3] = v.y;
        return;
    }
    int r = part - 1, s = 0, col = 4;
    while (s + 1 < io.n_lidars && r >= io.n_rays[s]) {
        r -= io.n_rays[s];
        col += io.n_rays[s];
        ++s;
    }
    const uint32_t mask = io.mask[s] & ~(1u << self);  // World.cast_rays skips the entity itself
    const float ang = io.angles[s][a][(long)b * io.ang_s0[s][a] + (long)r * io.ang_s1[s][a]] + ld_vec1(io.rot[a], b);
    const float dc = cosf(ang), ds = sinf(ang), mr = io.max_range[s];
    float best = mr;
#pragma unroll
    for (int e = 0; e < ME; ++e)  // (spheres: checked by the host entry point)
        if (e < io.n_entities && ((mask >> e) & 1u)) best = tmin(best, ray_sphere(p, dc, ds, ld_vec2(io.pos[e], b), io.radius[e], mr));
    io.lidar[s][a][(long)b * io.n_rays[s] + r] = best;
    o[col + r] = best;
}

#ifdef __HIP_DEVICE_COMPILE__
typedef const VmasDiscoveryIO __attribute__((address_space(4))) KDiscoveryIO;  // (see k_flocking_fast)
#define VMAS_KARG(T, name) T& io = *(T*)__builtin_amdgcn_kernarg_segment_ptr(); (void)name
#else
typedef const VmasDiscoveryIO KDiscoveryIO;
#define VMAS_KARG(T, name) T& io = name
#endif

// REWARD with a wave per agent (k_discovery_reward has one thread per env: 256 waves for 16 384
// envs, 31.5 us): lane = env of the workgroup's 64, wave i = agent i.  The agents' in-range bits
// meet in LDS for the per-target counts; wave 0 sums the covering rewards in agent order (the
// reference's loop order: bit-identical); the [64 x A x T] distances and the stacks are staged in
// LDS and written out as contiguous blocks.
constexpr int kDiscFastAgents = 16, kDiscFastTargets = 16;
__global__ void __launch_bounds__(1024) k_discovery_reward_fast(VmasDiscoveryIO io_arg) {
    VMAS_KARG(KDiscoveryIO, io_arg);
    disc_stage(io);
    constexpr int MT = kDiscFastTargets;
    __shared__ float D[64 * kDiscFastAgents * kDiscFastTargets];  // dists rows of the 64 envs (64 KiB)
    __shared__ uint32_t IN[kDiscFastAgents][64];                  // agent i's in-range target bits
    __shared__ float CR[kDiscFastAgents][64];                     // agent i's covering reward
    __shared__ float SH[64];
    const int lane = (int)(threadIdx.x & 63u);
    const int i = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int A = io.n_agents, T = io.n_targets, g0 = (int)blockIdx.x * 64, b = g0 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    const int nv = io.batch - g0 < 64 ? io.batch - g0 : 64;
    V2 PT[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
        const VmasVec pv = io.pos[io.target_entity[j < T ? j : 0]];
        PT[j] = j < T ? ld_vec2(pv, bb) : mk(0.f, 0.f);
    }
    const VmasVec av = io.pos[io.agent_entity[i]];
    const V2 pa = ld_vec2(av, bb);
    // torch.cdist (p = 2): sqrt(fl(fl(d0^2) + fl(d1^2))); agent i's distances and in-range bits
    uint32_t in = 0u;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
        if (j >= T) continue;
        const float d0 = pa.x - PT[j].x, d1 = pa.y - PT[j].y;
        const float d = sqrtf(d0 * d0 + d1 * d1);
        D[(lane * A + i) * T + j] = d;
        in |= (d < io.covering_range) ? (1u << j) : 0u;
    }
    IN[i][lane] = in;
    __syncthreads();
    // per target: the count of agents in range, covered when >= agents_per_target
    uint32_t covm = 0u;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
        if (j >= T) continue;
        int cnt = 0;
        for (int k = 0; k < A; ++k) cnt += (IN[k][lane] >> j) & 1u;
        covm |= cnt >= io.agents_per_target ? (1u << j) : 0u;
        if (i == 0 && valid) {
            io.per_target[(long)b * T + j] = (int64_t)cnt;
            io.covered[(long)b * T + j] = cnt >= io.agents_per_target ? 1 : 0;
        }
    }
    if (i == 1 % A && valid) disc_reductions(io, b, T, __builtin_popcount(covm));
    // agent i's covering reward: (count of covered targets in range) * coeff
    const float covr = 0.f + (float)__builtin_popcount(in & covm) * io.covering_rew_coeff;
    CR[i][lane] = covr;
    if (valid) {
        io.covering[i][b] = covr;
        io.collision[i][b] = 0.f;  // collision_rew[:] = 0 (penalty 0: nothing added)
    }
    __syncthreads();
    if (i == 0) {  // shared[:] = 0; += each agent's covering reward in agent order; halved where nonzero
        float shared = 0.f;
        for (int k = 0; k < A; ++k) shared = shared + CR[k][lane];
        if (shared != 0.f) shared = shared / 2.f;
        SH[lane] = shared;
        if (valid) {
            io.shared[b] = shared;
            if (io.time_int) reinterpret_cast<int64_t*>(io.time_rew)[b] = io.time_penalty_i;  // torch.full(int)
            else reinterpret_cast<float*>(io.time_rew)[b] = io.time_penalty;
        }
    }
    __syncthreads();
    if (valid) {
        const float cv = io.shared_reward ? SH[lane] : covr;
        moved(io.rewards[i], load_out_delta(io).rew)[b] = (0.f + cv) + io.time_penalty;  // collision_rew + covering_rew + time_rew
    }
    // the stacks and the distances as contiguous blocks of the workgroup's envs
    const int tid = (int)threadIdx.x, nth = (int)blockDim.x;
    float* dists = io.dists + (long)g0 * A * T;
    for (int k = tid; k < nv * A * T; k += nth) dists[k] = D[k];
    float2* ap = reinterpret_cast<float2*>(io.agents_pos) + (long)g0 * A;
    float2* tp = reinterpret_cast<float2*>(io.targets_pos) + (long)g0 * T;
    for (int k = tid; k < nv * A; k += nth) {
        const int e = k / A, a = k - e * A;
        const VmasVec v = io.pos[io.agent_entity[a]];
        ap[k] = make_float2(v.p[(long)(g0 + e) * v.s0], v.p[(long)(g0 + e) * v.s0 + v.s1]);
    }
    for (int k = tid; k < nv * T; k += nth) {
        const int e = k / T, j = k - e * T;
        const VmasVec v = io.pos[io.target_entity[j]];
        tp[k] = make_float2(v.p[(long)(g0 + e) * v.s0], v.p[(long)(g0 + e) * v.s0 + v.s1]);
    }
}

// OBS with the fast LIDAR (io.fast_lidar): a wave per (64 envs, agent), every ray of its LIDARs
// from the entity positions loaded once, the direct ray-sphere form with hardware sin / cos /
// sqrt (as k_flocking_fast), the observation rows staged in LDS and written as contiguous blocks.
constexpr int kDiscFastEntities = 16, kDiscFastRays = 16;  // per LIDAR
constexpr int kDiscFastW = 4 + VMAS_DISC_MAX_LIDARS * kDiscFastRays;
__global__ void __launch_bounds__(256) k_discovery_obs_fast(VmasDiscoveryIO io_arg) {
    VMAS_KARG(KDiscoveryIO, io_arg);
    constexpr int ME = kDiscFastEntities, RM = kDiscFastRays;
    __shared__ float S[4][64 * kDiscFastW];
    const int lane = (int)(threadIdx.x & 63u), w = (int)(threadIdx.x >> 6);
    const int a = __builtin_amdgcn_readfirstlane((int)blockIdx.y * 4 + w);
    if (a >= io.n_agents) return;  // (wave-uniform; no workgroup barrier below)
    const int g0 = (int)blockIdx.x * 64, b = g0 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    const int nv = io.batch - g0 < 64 ? io.batch - g0 : 64;
    const int self = io.agent_entity[a], ne = io.n_entities;
    int rays = 0;
    for (int s = 0; s < io.n_lidars; ++s) rays += io.n_rays[s];
    const int W = 4 + rays, row = lane * W;
    const VmasVec sp = io.pos[self], vv = io.vel[a], rv = io.rot[a];
    const V2 p = ld_vec2(sp, bb), v = ld_vec2(vv, bb);
    const float rot = ld_vec1(rv, bb);
    V2 T[ME];
    float R2[ME];
#pragma unroll
    for (int e = 0; e < ME; ++e) {
        const VmasVec ev = io.pos[e < ne ? e : 0];
        const float rad = io.radius[e < ne ? e : 0];
        T[e] = e < ne ? ld_vec2(ev, bb) - p : mk(0.f, 0.f);
        R2[e] = rad * rad;
    }
    S[w][row + 0] = p.x;
    S[w][row + 1] = p.y;
    S[w][row + 2] = v.x;
    S[w][row + 3] = v.y;
    float C[ME];
#pragma unroll
    for (int e = 0; e < ME; ++e) C[e] = R2[e] - (T[e].x * T[e].x + T[e].y * T[e].y);
    int col = 4;
    for (int s = 0; s < io.n_lidars; ++s) {
        const uint32_t mask = io.mask[s] & ~(1u << self);  // World.cast_rays skips the entity itself
        const int nr = io.n_rays[s];
        const float mr = io.max_range[s];
        const float* ang = io.angles[s][a] + (long)bb * io.ang_s0[s][a];
        const int as1 = io.ang_s1[s][a];
        // rays in a rolled loop (entities unrolled inside, a uniform branch on the LIDAR's mask):
        // the fully unrolled rays x entities body was ~35 KiB of straight-line code, each wave
        // streaming it through the instruction cache once
        // (the angles, loaded together up front, wait in the rays' own LDS slots)
        // (rays in pairs: two rays' independent chains interleave -- at 4 waves per SIMD one chain
        // at a time left the SIMDs waiting; the same operations per ray, in the same order)
#pragma unroll
        for (int r = 0; r < RM; ++r)
            if (r < nr) S[w][row + col + r] = ang[(long)r * as1] + rot;
        auto sc = [](float th, float& ds, float& dc) {
            if (fabsf(th) < kFastTrigMaxAngle) {
                ds = __sinf(th);
                dc = __cosf(th);
            } else {
                sincosf(th, &ds, &dc);
            }
        };
        int r = 0;
#pragma unroll 1
        for (; r + 1 < nr; r += 2) {
            float dc0, ds0, dc1, ds1;
            sc(S[w][row + col + r], ds0, dc0);
            sc(S[w][row + col + r + 1], ds1, dc1);
            float b0 = mr, b1 = mr;
#pragma unroll
            for (int e = 0; e < ME; ++e) {
                if (e >= ne || !((mask >> e) & 1u)) continue;
                b0 = min_drop_nan(b0, ray_sphere_fast_nan(T[e].x, T[e].y, C[e], dc0, ds0));
                b1 = min_drop_nan(b1, ray_sphere_fast_nan(T[e].x, T[e].y, C[e], dc1, ds1));
            }
            S[w][row + col + r] = b0;
            S[w][row + col + r + 1] = b1;
        }
        if (r < nr) {
            float dc, ds;
            sc(S[w][row + col + r], ds, dc);
            float best = mr;
#pragma unroll
            for (int e = 0; e < ME; ++e) {
                if (e >= ne || !((mask >> e) & 1u)) continue;
                best = min_drop_nan(best, ray_sphere_fast_nan(T[e].x, T[e].y, C[e], dc, ds));
            }
            S[w][row + col + r] = best;
        }
        float* lid = io.lidar[s][a] + (long)g0 * nr;
        for (int k = lane; k < nv * nr; k += 64) {
            const int e = k / nr;
            lid[k] = S[w][e * W + col + (k - e * nr)];
        }
        col += nr;
    }
    float* obs = moved(io.obs[a], load_out_delta(io).obs) + (long)g0 * W;
    for (int k = lane; k < nv * W; k += 64) obs[k] = S[w][k];
}

// The same program with a wave per (64 envs, agent, LIDAR) instead of per (64 envs, agent): L
// waves of one workgroup share an agent's observation rows in LDS, each casting one LIDAR's rays
// (the same operations per ray, in the same order: bit-identical), and write the rows out together
// after one barrier.  At C4 (16 384 envs, 8 agents, 2 LIDARs) the per-agent form ran 2 048 waves,
// 2 per SIMD, too few to hide the trig / sqrt / LDS latencies; this runs 4 096.
template <int L>
__global__ void __launch_bounds__(256) k_discovery_obs_split(VmasDiscoveryIO io_arg) {
    VMAS_KARG(KDiscoveryIO, io_arg);
    constexpr int ME = kDiscFastEntities, RM = kDiscFastRays, AP = 4 / L;
    __shared__ float S[AP][64 * kDiscFastW];
    const int lane = (int)(threadIdx.x & 63u), w = (int)(threadIdx.x >> 6);
    const int sub = w / L, s = w - sub * L;
    const int a = __builtin_amdgcn_readfirstlane((int)blockIdx.y * AP + sub);
    const bool active = a < io.n_agents;  // (no early return: the barrier below)
    const int g0 = (int)blockIdx.x * 64, b = g0 + lane;
    const bool valid = b < io.batch;
    const int bb = valid ? b : io.batch - 1;
    const int nv = io.batch - g0 < 64 ? io.batch - g0 : 64;
    int rays = 0, col = 4;
    for (int k = 0; k < L; ++k) {
        rays += io.n_rays[k];
        if (k < s) col += io.n_rays[k];
    }
    const int W = 4 + rays, row = lane * W;
    if (active) {
        const int self = io.agent_entity[a], ne = io.n_entities;
        const VmasVec sp = io.pos[self], rv = io.rot[a];
        const V2 p = ld_vec2(sp, bb);
        const float rot = ld_vec1(rv, bb);
        if (s == 0) {
            const V2 v = ld_vec2(io.vel[a], bb);
            S[sub][row + 0] = p.x;
            S[sub][row + 1] = p.y;
            S[sub][row + 2] = v.x;
            S[sub][row + 3] = v.y;
        }
        V2 T[ME];
        float C[ME];
#pragma unroll
        for (int e = 0; e < ME; ++e) {
            const VmasVec ev = io.pos[e < ne ? e : 0];
            const float rad = io.radius[e < ne ? e : 0];
            T[e] = e < ne ? ld_vec2(ev, bb) - p : mk(0.f, 0.f);
            C[e] = rad * rad - (T[e].x * T[e].x + T[e].y * T[e].y);
        }
        const uint32_t mask = io.mask[s] & ~(1u << self);  // World.cast_rays skips the entity itself
        const int nr = io.n_rays[s];
        const float mr = io.max_range[s];
        const float* ang = io.angles[s][a] + (long)bb * io.ang_s0[s][a];
        const int as1 = io.ang_s1[s][a];
#pragma unroll
        for (int r = 0; r < RM; ++r)
            if (r < nr) S[sub][row + col + r] = ang[(long)r * as1] + rot;
        auto sc = [](float th, float& ds, float& dc) {
            if (fabsf(th) < kFastTrigMaxAngle) {
                ds = __sinf(th);
                dc = __cosf(th);
            } else {
                sincosf(th, &ds, &dc);
            }
        };
        int r = 0;
#pragma unroll 1
        for (; r + 1 < nr; r += 2) {
            float dc0, ds0, dc1, ds1;
            sc(S[sub][row + col + r], ds0, dc0);
            sc(S[sub][row + col + r + 1], ds1, dc1);
            float b0 = mr, b1 = mr;
#pragma unroll
            for (int e = 0; e < ME; ++e) {
                if (e >= ne || !((mask >> e) & 1u)) continue;
                b0 = min_drop_nan(b0, ray_sphere_fast_nan(T[e].x, T[e].y, C[e], dc0, ds0));
                b1 = min_drop_nan(b1, ray_sphere_fast_nan(T[e].x, T[e].y, C[e], dc1, ds1));
            }
            S[sub][row + col + r] = b0;
            S[sub][row + col + r + 1] = b1;
        }
        if (r < nr) {
            float dc, ds;
            sc(S[sub][row + col + r], ds, dc);
            float best = mr;
#pragma unroll
            for (int e = 0; e < ME; ++e) {
                if (e >= ne || !((mask >> e) & 1u)) continue;
                best = min_drop_nan(best, ray_sphere_fast_nan(T[e].x, T[e].y, C[e], dc, ds));
            }
            S[sub][row + col + r] = best;
        }
        float* lid = io.lidar[s][a] + (long)g0 * nr;  // (this wave's own columns: no barrier needed)
        for (int k = lane; k < nv * nr; k += 64) {
            const int e = k / nr;
            lid[k] = S[sub][e * W + col + (k - e * nr)];
        }
    }
    __syncthreads();
    if (!active) return;
    float* obs = moved(io.obs[a], load_out_delta(io).obs) + (long)g0 * W;
    for (int k = lane + s * 64; k < nv * W; k += 64 * L) obs[k] = S[sub][k];
}

// Test kernel (tests/test_fused.py test_exact_math_gpu): the flag-independent division / square
// root of vmas_programs.hpp next to this translation unit's IEEE `/` and sqrtf.
__global__ void k_test_exact_math(const float* a, const float* b, float* out, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = xdiv(a[i], b[i]);
    out[n + i] = a[i] / b[i];
    out[2 * n + i] = xsqrt(a[i]);
    out[3 * n + i] = sqrtf(a[i]);
}

// The fast LIDAR programs' direction instructions (v_sin_f32 / v_cos_f32 through __sinf / __cosf,
// as k_flocking_fast / k_discovery_obs_fast compute a ray's (cos, sin)): out[i] = sin, out[n + i] = cos.
__global__ void k_test_fast_trig(const float* x, float* out, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = __sinf(x[i]);
    out[n + i] = __cosf(x[i]);
}

}  // namespace

extern "C" {

int32_t vmas_test_fast_trig(int32_t device, const float* x, float* out, int64_t n, void* stream) {
    if (device < 0 || !x || !out || n <= 0) return vmas_aux::fail(VMAS_E_INVALID, "vmas_test_fast_trig: bad arguments");
    VMAS_AUX_HIP(hipSetDevice(device));
    hipLaunchKernelGGL(k_test_fast_trig, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, out, (long)n);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_test_exact_math(int32_t device, const float* a, const float* b, float* out, int64_t n, void* stream) {
    if (device < 0 || !a || !b || !out || n <= 0) return vmas_aux::fail(VMAS_E_INVALID, "vmas_test_exact_math: bad arguments");
    VMAS_AUX_HIP(hipSetDevice(device));
    hipLaunchKernelGGL(k_test_exact_math, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, b, out, (long)n);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_balance_outputs(int32_t device, const VmasBalanceIO* io, void* stream) {
    if (!io || device < 0 || io->batch <= 0 || io->n_agents < 0 || io->n_agents > VMAS_SCN_MAX_AGENTS)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_balance_outputs: bad arguments");
    if (io->package.shape != VMAS_SPHERE || io->goal.shape != VMAS_SPHERE || io->line.shape != VMAS_LINE ||
        io->floor.shape != VMAS_BOX)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_balance_outputs: unexpected entity shapes");
    VMAS_AUX_HIP(hipSetDevice(device));
    const int parts = 1 + ((io->what & VMAS_SCN_OBS) ? (io->n_agents + 3) / 4 : 0);
    hipLaunchKernelGGL(k_balance, dim3((io->batch + 63) / 64, parts), dim3(256), 0, (hipStream_t)stream, *io);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_flocking_target_action(int32_t device, const float* t, int32_t batch, float period, float* u,
                                    void* stream) {
    if (device < 0 || !t || !u || batch <= 0 || period == 0.f)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_flocking_target_action: bad arguments");
    const float inv = 1.0f / period;
    hipLaunchKernelGGL(k_flocking_target, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, t, batch, inv, u);
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
    if (io->fast_lidar && io->n_rays <= kFlockFastRays && io->n_ray_targets <= kFlockFastTargets) {
        const dim3 grid((io->batch + 63) / 64, (io->n_policy + 3) / 4);
        const hipStream_t st = (hipStream_t)stream;
        // flocking's 12 rays with 1..8 targets: the unrolled instantiation (VMAS_FLOCK_UNROLL=0: runtime form)
        static const bool unroll = !getenv("VMAS_FLOCK_UNROLL") || getenv("VMAS_FLOCK_UNROLL")[0] != '0';
        const int nt = unroll && io->n_rays == 12 ? io->n_ray_targets : 0;
        switch (nt) {
#define VMAS_FLOCK_CASE(k) \
    case k: hipLaunchKernelGGL((k_flocking_fast<12, k>), grid, dim3(256), 0, st, *io); break;
            VMAS_FLOCK_CASE(1) VMAS_FLOCK_CASE(2) VMAS_FLOCK_CASE(3) VMAS_FLOCK_CASE(4)
            VMAS_FLOCK_CASE(5) VMAS_FLOCK_CASE(6) VMAS_FLOCK_CASE(7) VMAS_FLOCK_CASE(8)
#undef VMAS_FLOCK_CASE
            default: hipLaunchKernelGGL((k_flocking_fast<0, 0>), grid, dim3(256), 0, st, *io); break;
        }
    } else
        hipLaunchKernelGGL(k_flocking, dim3((io->batch + 63) / 64, io->n_policy * parts), dim3(64), 0, (hipStream_t)stream,
                           *io);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_transport_outputs(int32_t device, const VmasTransportIO* io, void* stream) {
    if (!io || device < 0 || io->batch <= 0 || io->n_agents < 0 || io->n_agents > VMAS_TRANSPORT_MAX_AGENTS ||
        io->n_packages < 0 || io->n_packages > VMAS_TRANSPORT_MAX_PACKAGES)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_transport_outputs: bad arguments");
    for (int i = 0; i < io->n_packages; ++i)
        if (io->package[i].shape != VMAS_BOX || io->goal[i].shape != VMAS_SPHERE)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_transport_outputs: package %d is not (box, sphere goal)", i);
    VMAS_AUX_HIP(hipSetDevice(device));
    static_assert(sizeof(VmasTransportIO) <= 4096, "kernel argument block");
    const int parts = 1 + ((io->what & VMAS_SCN_OBS) ? io->n_agents : 0);
    hipLaunchKernelGGL(k_transport, dim3((io->batch + 63) / 64, parts), dim3(64), 0, (hipStream_t)stream, *io);
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_discovery_outputs(int32_t device, const VmasDiscoveryIO* io, void* stream) {
    if (!io || device < 0 || io->batch <= 0 || io->n_agents < 1 || io->n_agents > VMAS_DISC_MAX_AGENTS ||
        io->n_targets < 0 || io->n_targets > VMAS_DISC_MAX_TARGETS || io->n_entities < 1 ||
        io->n_entities > VMAS_DISC_MAX_ENTITIES || io->n_lidars < 0 || io->n_lidars > VMAS_DISC_MAX_LIDARS ||
        (io->done && !io->all_time))
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_discovery_outputs: bad arguments");
    for (int i = 0; i < io->n_agents; ++i)
        if (io->agent_entity[i] < 0 || io->agent_entity[i] >= io->n_entities)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_discovery_outputs: bad agent index %d", i);
    for (int j = 0; j < io->n_targets; ++j)
        if (io->target_entity[j] < 0 || io->target_entity[j] >= io->n_entities)
            return vmas_aux::fail(VMAS_E_INVALID, "vmas_discovery_outputs: bad target index %d", j);
    int rays = 0;
    for (int s = 0; s < io->n_lidars; ++s) {
        if (io->n_rays[s] < 0) return vmas_aux::fail(VMAS_E_INVALID, "vmas_discovery_outputs: bad ray count");
        rays += io->n_rays[s];
    }
    VMAS_AUX_HIP(hipSetDevice(device));
    static_assert(sizeof(VmasDiscoveryIO) <= 4096, "kernel argument block");
    const unsigned gx = (unsigned)((io->batch + 63) / 64);
    if (io->what & VMAS_SCN_REWARD) {
        if (io->n_agents <= kDiscFastAgents && io->n_targets <= kDiscFastTargets && io->n_targets >= 1)
            hipLaunchKernelGGL(k_discovery_reward_fast, dim3(gx), dim3(64 * io->n_agents), 0, (hipStream_t)stream, *io);
        else
            hipLaunchKernelGGL(k_discovery_reward, dim3(gx), dim3(64), 0, (hipStream_t)stream, *io);
    }
    if (io->what & VMAS_SCN_OBS) {
        bool fast = io->fast_lidar && io->n_entities <= kDiscFastEntities;
        for (int s = 0; s < io->n_lidars; ++s) fast = fast && io->n_rays[s] <= kDiscFastRays;
        // a wave per (64 envs, agent, LIDAR) with two LIDARs (VMAS_DISC_OBS_SPLIT=0: per agent, A/B)
        static const bool split = !(getenv("VMAS_DISC_OBS_SPLIT") && getenv("VMAS_DISC_OBS_SPLIT")[0] == '0');
        if (fast && split && io->n_lidars == 2)
            hipLaunchKernelGGL(k_discovery_obs_split<2>, dim3(gx, (io->n_agents + 1) / 2), dim3(256), 0,
                               (hipStream_t)stream, *io);
        else if (fast)
            hipLaunchKernelGGL(k_discovery_obs_fast, dim3(gx, (io->n_agents + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                               *io);
        else
            hipLaunchKernelGGL(k_discovery_obs, dim3(gx, io->n_agents * (1 + rays)), dim3(64), 0, (hipStream_t)stream,
                               *io);
    }
    VMAS_AUX_HIP(hipGetLastError());
    return VMAS_OK;
}

}  // extern "C"
