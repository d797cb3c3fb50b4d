// vmas_jit.hip -- world-specialised step kernels (hipRTC) for the VMAS physics step.
//
// vmas_world_step's k_step is generic: every pair and entity is a table row, dispatched at run
// time.  For a fixed world (VMAS worlds are fixed after make_env), this module generates one HIP
// kernel for that world and compiles it with hipRTC for gfx950.  It keeps k_step's decomposition
// and arithmetic:
//   * one workgroup = 64 envs (lane = env) x 8 waves; per substep a pair phase (each wave its
//     statically scheduled pair tasks), a barrier, an entity phase (each wave its dynamic
//     entities: action clamps / friction / gravity, then the pair results in the reference's
//     summation order, then semi-implicit Euler), a barrier;
//   * the same vmas_physics.hpp functions with the same fp32 operation order, so results are
//     bit-identical to k_step and the host backend (tests/test_jit.py);
// and specialises what k_step looks up at run time:
//   * per-wave straight-line code for exactly its pair tasks and entities (no descriptor loads,
//     no class switch); entity/pair/joint/world constants are constexpr, so flag tests fold;
//   * a dynamic entity's state, velocity and agent force/torque live in its owner wave's
//     registers for the whole launch; positions, rotations and trig rows are published to LDS;
//   * box-line / box-box pairs are split into their per-side parts (4 / 8 tasks) on several
//     waves; a finish task (last in its wave's list) waits for the parts on an LDS counter,
//     replays the reference's first-strict-minimum selection and finishes the contact.  Every
//     wave runs all its parts before any finish, so the waits cannot deadlock;
//   * tasks are placed by longest-processing-time with class costs measured with
//     tools/jit_phase_profile.py (a contact pair costs several times an out-of-contact one; the
//     costs are for the contact case);
//   * the per-call tensor pointers and strides are kernel arguments (no staging upload); static
//     entities are loaded once; entities in no pair and not dynamic are never read.
// A single work queue shared by the waves was measured slower (one switch over every pair in the
// substep loop: the hoisted constants spilled 114 SGPRs, +37 % pair-phase work).
// Worlds beyond the kernel-argument or LDS budget return VMAS_E_INVALID from
// vmas_jit_world_create and the caller uses vmas_world_step.
//
// Batch-global broadphase (core.py:2796): the fixed-point scheme of vmas_world_step (R/Z flags
// per group, a reduction that checks the mask, a re-run on violation), run on the device inside
// ONE persistent launch: the 64-env groups are claimed per pass, the last completion of a pass
// reduces the flags and publishes the decision, and a workgroup only ever waits for groups that
// running workgroups have claimed -- never for another workgroup to become resident
// (vmas_jit_ops.hpp grid_*).  The host only launches.  VMAS_JIT_GRID=host keeps the host-driven
// loop (one launch + reduction + host read per pass).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <hip/hip_ext.h>
#include <dlfcn.h>

#include "vmas_aux.hpp"
#include "vmas_jit_ops.hpp"
#include "vmas_jit_registry.hpp"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "vmas_mi355x.h"

namespace {

thread_local std::string g_jit_err;

int32_t jfail(int32_t code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_jit_err = buf;
    return code;
}

#define JHIP(x)                                                                                 \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            (void)hipGetLastError();                                                            \
            return jfail(VMAS_E_HIP, "%s: %s", #x, hipGetErrorString(e_));                      \
        }                                                                                       \
    } while (0)

// exact fp32 literal
std::string fl(float v) {
    if (v != v) return "__builtin_nanf(\"\")";
    if (v == __builtin_huge_valf()) return "__builtin_huge_valf()";
    if (v == -__builtin_huge_valf()) return "(-__builtin_huge_valf())";
    char b[64];
    snprintf(b, sizeof b, "%af", (double)v);
    return b;
}
std::string it(long v) { return std::to_string(v); }
std::string bl(bool v) { return v ? "true" : "false"; }

// Relaxed fp32 math for a world's kernel (default for worlds without joints, whose joint torque
// exp(|dtheta|) - 1 left the parity tolerance in round 1; VMAS_JIT_MATH=exact turns it off):
// fp32 division and sqrt without the correctly-rounded sequences (v_rcp / v_sqrt, ~1 ulp), exp
// from the hardware approximation.  Still fp32 throughout; the results are within the oracle
// tolerance (tests/test_gpu_parity.py, full size included), not bit-identical to k_step.
// Measured on balance 32 768 x 10 substeps: k_world 66.3 -> 51.8 us.
constexpr const char* kRelaxedTag = "// vmas-math: relaxed";
// The generated source carries its own code-generation options on this line (compile() reads
// them from there), so the source text -- and its sha256, which keys the bench's PMC record --
// pins the code object.
constexpr const char* kFlagsTag = "// vmas-cflags:";

// -fno-slp-vectorize: the SLP vectoriser pairs independent scalar ops of the per-lane physics
// into v_pk_add/v_pk_mul_f32, which on gfx950 costs more than it saves: register-pair moves
// (v_mov) and hazard s_nops around the packed ops (balance C2: 4490 -> 4905 VALU in the substep
// loops but 395 -> 123 s_nop, 494 -> 172 v_mov; k_world 55.4 -> 48.8 us,
// profiles/r02/run9_noslp).  Packed ops round per element, so results are unchanged.
// Relaxed worlds add the approximate-function / fast divide-sqrt options.  VMAS_JIT_CFLAGS
// (space separated) appends options for A/B measurements.
std::string codegen_flags(bool relaxed) {
    std::string f = " -fno-slp-vectorize";
    if (relaxed) f += " -fapprox-func -fno-hip-fp32-correctly-rounded-divide-sqrt";
    if (const char* x = getenv("VMAS_JIT_CFLAGS")) f += std::string(" ") + x;
    return f;
}


// Largest float x with sqrtf(x) <= r (sqrtf correctly rounded on both the host and gfx950 with
// -fno-fast-math, hence monotonic): for d2 = fl(fl(dx*dx) + fl(dy*dy)),
// norm(d) <= r  <=>  d2 <= sq_limit(r), and norm(d) > r <=> d2 > sq_limit(r); NaN compares false
// both ways, as in the reference.
float sq_limit(float r) {
    if (!(r >= 0.f)) return -1.f;  // no finite d2 qualifies (NaN / negative radius)
    if (r == __builtin_huge_valf()) return __builtin_huge_valf();
    float x = r * r;
    while (x > 0.f && std::sqrt(x) > r) x = std::nextafter(x, 0.f);
    while (std::sqrt(std::nextafter(x, __builtin_huge_valf())) <= r) x = std::nextafter(x, __builtin_huge_valf());
    return x;
}

constexpr int kNW = 8;      // waves per workgroup (VMAS_JIT_WAVES overrides: 8 or 16)
constexpr int kMaxNW = 16;  // column stride of the phase-profile buffer
constexpr int kProfBlocks = 4096;  // workgroups with a per-workgroup record in profile builds
constexpr int kProfRec = 24;       // words per record (16 waves' HW_ID at most)
constexpr int kMaxArgBytes = 3584;        // HIP kernel argument block limit is 4 KiB
static_assert(sizeof(VmasBalanceIO) % 8 == 0 && sizeof(VmasTransportIO) % 8 == 0,
              "a scenario program's argument block is copied into LDS in 8-byte words");
constexpr int kEpiQRows = 28;             // LDS rows of a scenario program (vmas_programs.hpp kBalQRows)
constexpr int kLdsTwoPerCu = 64 * 1024;   // keeps two 512-thread workgroups per CU
constexpr int kLdsOnePerCu = 150 * 1024;  // big worlds: one workgroup per CU (160 KiB LDS)

// pointer-table sources of the kernel argument block
enum Src { S_POS, S_VEL, S_ROT, S_ANG, S_GRAV, S_FORCE, S_TORQUE, S_JFIX };
constexpr unsigned kPrmMaskDefault = 0x7FFu;
// value fields of VmasEntityDesc passed as kernel arguments (Gen::value_fields)
enum Prm { kPrmMass, kPrmInertia, kPrmDrag, kPrmLinFric, kPrmAngFric, kPrmMaxSpeed, kPrmVRange, kPrmMaxF, kPrmFRange,
           kPrmMaxT, kPrmTRange };
inline float prm_value(const VmasEntityDesc& d, int k) {
    switch (k) {
        case kPrmMass: return d.mass;
        case kPrmInertia: return d.inertia;
        case kPrmDrag: return d.one_minus_drag;
        case kPrmLinFric: return d.lin_fric;
        case kPrmAngFric: return d.ang_fric;
        case kPrmMaxSpeed: return d.max_speed;
        case kPrmVRange: return d.v_range;
        case kPrmMaxF: return d.max_f;
        case kPrmFRange: return d.f_range;
        case kPrmMaxT: return d.max_t;
        default: return d.t_range;
    }
}
inline float prm_world_value(const VmasWorldConfig& c, int k) {
    return k == 0 ? c.gravity_x : k == 1 ? c.gravity_y : k == 2 ? c.x_semidim : c.y_semidim;
}

struct Item {
    int pair, side, torque;
};
constexpr int kWhole = -1, kFinish = -2;
struct Task {
    int pair, part;  // kWhole, 0..n-1 (one part of a split pair) or kFinish
    float cost;
};

struct Gen {
    const VmasWorldConfig& cfg;
    const std::vector<VmasEntityDesc>& ed;
    const std::vector<VmasPairDesc>& pd;
    const std::vector<VmasJointDesc>& jd;
    int E, P, A, J, W, nfl;
    bool split_boxes = true;
    long lds_budget = kLdsTwoPerCu;
    // rows in a global-memory slab (one per workgroup, a.rows) instead of LDS: worlds whose rows
    // exceed one workgroup's LDS (hundreds of box pairs) still run the world-specialised step and
    // its persistent fixed point; the rows' traffic then goes through L1 / L2
    bool global_rows = false;
    int nw = kNW;         // waves per 64-env group
    // 64-env groups per claimed work item (VMAS_JIT_NG, A/B): ng > 1 runs ng groups in one
    // workgroup of nw * ng waves in lockstep -- waves [k * nw, (k + 1) * nw) run group k's copy of
    // the per-wave code on its own LDS rows, all sharing the workgroup's barriers -- so the groups a
    // CU holds finish together instead of the second workgroup of a CU trailing the first
    int ng = 1;
    int prof_block = -1;  // >= 0: stamp s_memtime at every phase boundary of this workgroup
    bool relaxed = false;  // relaxed fp32 math (VMAS_JIT_MATH=relaxed, worlds without joints; see compile())
    int prio_mode = 1;     // VMAS_JIT_PRIO=0 turns off the wave issue priority falling with the substep
    bool entity_preload = true;  // VMAS_JIT_PRELOAD=0 (A/B): contribution reads inside their branches
    bool pair_preload = true;    // VMAS_JIT_PAIR_PRELOAD=0 (A/B): other waves' entity rows read at each use
    std::vector<char> dyn, in_pair, need_trig, need_rot, split;
    std::vector<int> owner;  // wave owning a dynamic entity / loading a static pair entity
    std::vector<std::vector<int>> wave_ents, wave_static;
    std::vector<std::vector<Task>> wave_tasks;
    std::vector<std::vector<Item>> items;  // per entity, reference order
    std::vector<int> split_idx;            // per split pair: its LDS completion counter
    int n_split = 0;
    // LDS rows (64 floats each)
    std::vector<int> r_p, r_rot, r_trig, r_res;
    // balance's epilogue reads the group's state from the rows (epi_src): velocity rows of the
    // dynamic entities, published after the last substep; Q (its scratch) then sits on the pair
    // result rows, dead by then
    std::vector<int> r_v, r_w;
    int res_first = 0, res_end = 0;
    bool epi_src = false;  // (VMAS_JIT_EPI_SRC=1, A/B: measured slower so far, profiles/r06/)
    int n_rows = 0;
    // argument block
    std::vector<std::pair<int, int>> ptr_src, str_src;  // (Src, index); strides: (Src*4 + k, index)
    std::vector<int> ptr_of[8], str_of[8][2];
    std::string src;

    Gen(const VmasWorldConfig& c, const std::vector<VmasEntityDesc>& e, const std::vector<VmasPairDesc>& p,
        const std::vector<VmasJointDesc>& j)
        : cfg(c), ed(e), pd(p), jd(j) {
        E = c.n_entities;
        P = c.n_pairs;
        A = c.n_agents;
        J = c.n_joints;
        W = std::max(1, (P + 31) / 32);
        nfl = 2 * c.max_substeps * W;
    }

    static int parts(int cls) { return cls == VMAS_PAIR_BL ? 4 : 8; }

    int ptr(Src s, int idx) {
        int& slot = ptr_of[s][idx];
        if (slot < 0) {
            slot = (int)ptr_src.size();
            ptr_src.push_back({s, idx});
        }
        return slot;
    }
    int str(Src s, int k, int idx) {
        int& slot = str_of[s][k][idx];
        if (slot < 0) {
            slot = (int)str_src.size();
            str_src.push_back({s * 4 + k, idx});
        }
        return slot;
    }
    int rows(int n) {
        const int r = n_rows;
        n_rows += n;
        return r;
    }

    bool plan(std::string* why) {
        dyn.assign(E, 0);
        in_pair.assign(E, 0);
        need_trig.assign(E, 0);
        need_rot.assign(E, 0);
        split.assign(P, 0);
        split_idx.assign(P, -1);
        for (int e = 0; e < E; ++e) dyn[e] = (ed[e].flags & (VMAS_F_MOVABLE | VMAS_F_ROTATABLE)) != 0;
        for (const auto& q : pd) {
            in_pair[q.ea] = in_pair[q.eb] = 1;
            if (q.cls == VMAS_PAIR_JOINT) need_trig[q.ea] = need_trig[q.eb] = need_rot[q.ea] = need_rot[q.eb] = 1;
        }
        for (int e = 0; e < E; ++e) {
            if (in_pair[e] && ed[e].shape != VMAS_SPHERE) need_trig[e] = 1;
            if (need_trig[e]) need_rot[e] = 1;
        }
        for (int p = 0; p < P; ++p) {
            split[p] = split_boxes && (pd[p].cls == VMAS_PAIR_BL || pd[p].cls == VMAS_PAIR_BB);
            if (split[p]) split_idx[p] = n_split++;
        }
        items.assign(E, {});
        for (int p = 0; p < P; ++p) {
            for (int side = 0; side < 2; ++side) {
                const int e = side ? pd[p].eb : pd[p].ea;
                if (!dyn[e]) continue;
                int tq = 1;  // spheres in SS/LS/BS receive no torque (core.py:2330-2338, 2383-2391, 2543-2551)
                if (pd[p].cls == VMAS_PAIR_SS) tq = 0;
                if ((pd[p].cls == VMAS_PAIR_LS || pd[p].cls == VMAS_PAIR_BS) && side == 1) tq = 0;
                items[e].push_back({p, side, tq});
            }
        }
        // pair tasks: longest-processing-time over the waves.  Contact-case costs in units of a
        // sphere-sphere contact, measured per wave with tools/jit_phase_profile.py.
        // A sphere-sphere pair mostly takes the exact early-out (out of contact in all 64 envs), so
        // it is priced at half a contact; a split pair's finish is placed by the LPT with the
        // other tasks (last in its wave), priced at 3.  Measured (profiles/r01/run27_schedule):
        // k_world balance 66.3 -> 64.4 us, transport 10.2 -> 9.9 us against SS 1.0 and the
        // finish placed after all other tasks.  VMAS_JIT_COST_SS / VMAS_JIT_COST_FINISH /
        // VMAS_JIT_COST_PART (a box-line part) / VMAS_JIT_FINISH_LPT=0 override (A/B).
        float kCost[7] = {1.5f, 0.5f, 2.0f, 1.8f, 2.2f, 7.4f, 30.f};
        float finish_cost = 3.0f;
        // (measured and rejected, profiles/r02/run10_sched: a table rescaled to relaxed-math VALU
        // counts and SIMD-aware placement (waves w and w + 4 share a SIMD) -- balance C2 k_world
        // 40.8 -> 42.6-45.7 us: the two workgroups on a CU map waves to SIMDs with different
        // rotations, so per-SIMD sums even out, and the per-wave makespan is what binds)
        if (const char* c = getenv("VMAS_JIT_COST_SS")) kCost[VMAS_PAIR_SS] = (float)atof(c);
        if (const char* c = getenv("VMAS_JIT_COST_FINISH")) finish_cost = (float)atof(c);
        float bl_part_cost = 1.8f, bb_part_cost = 3.8f;  // a split box-line / box-box pair's part
        if (const char* c = getenv("VMAS_JIT_COST_PART")) bl_part_cost = (float)atof(c);
        const char* fl_lpt = getenv("VMAS_JIT_FINISH_LPT");
        const bool finish_in_lpt = !(fl_lpt && fl_lpt[0] == '0');
        std::vector<Task> all, finishes;
        for (int p = 0; p < P; ++p) {
            if (split[p]) {
                for (int k = 0; k < parts(pd[p].cls); ++k)
                    all.push_back({p, k, pd[p].cls == VMAS_PAIR_BL ? bl_part_cost : bb_part_cost});
                (finish_in_lpt ? all : finishes).push_back({p, kFinish, finish_cost});
            } else {
                all.push_back({p, kWhole, kCost[pd[p].cls]});
            }
        }
        std::stable_sort(all.begin(), all.end(), [](const Task& a, const Task& b) { return a.cost > b.cost; });
        wave_tasks.assign(nw, {});
        std::vector<float> load(nw, 0.f);
        auto place = [&](const Task& t) {
            const int w = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            wave_tasks[w].push_back(t);
            load[w] += t.cost;
        };
        for (const Task& t : all) place(t);
        // parts first in their waves (a finish waits for them), finishes last: a wave waiting in
        // a finish has run all of its parts
        for (auto& v : wave_tasks)
            std::stable_sort(v.begin(), v.end(), [](const Task& a, const Task& b) {
                const int ra = a.part >= 0 ? 0 : a.part == kFinish ? 2 : 1;  // parts, wholes, finishes
                const int rb = b.part >= 0 ? 0 : b.part == kFinish ? 2 : 1;
                return ra != rb ? ra < rb : a.pair < b.pair;
            });
        for (const Task& t : finishes) place(t);
        // entity phase: dynamic entities over the waves by contribution count (LPT)
        owner.assign(E, -1);
        wave_ents.assign(nw, {});
        wave_static.assign(nw, {});
        {
            std::vector<int> order;
            for (int e = 0; e < E; ++e)
                if (dyn[e]) order.push_back(e);
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return items[a].size() > items[b].size(); });
            std::vector<float> eload(nw, 0.f);
            for (int e : order) {
                const int w = (int)(std::min_element(eload.begin(), eload.end()) - eload.begin());
                owner[e] = w;
                wave_ents[w].push_back(e);
                eload[w] += 4.f + items[e].size();
            }
            int rr = 0;
            for (int e = 0; e < E; ++e)
                if (!dyn[e] && in_pair[e]) {
                    owner[e] = rr % nw;
                    wave_static[rr % nw].push_back(e);
                    ++rr;
                }
        }
        // LDS rows: published entity state, then per pair 4 result rows (a split pair first holds
        // its parts' (p1, p2) and the pre-integration centres)
        r_p.assign(E, -1);
        r_rot.assign(E, -1);
        r_trig.assign(E, -1);
        r_res.assign(P, -1);
        for (int e = 0; e < E; ++e) {
            if (!in_pair[e]) continue;
            r_p[e] = rows(2);
            if (need_rot[e]) r_rot[e] = rows(1);
            if (need_trig[e]) r_trig[e] = rows(4);
        }
        res_first = n_rows;
        for (int p = 0; p < P; ++p) r_res[p] = rows(split[p] ? 4 * parts(pd[p].cls) + 8 : res_rows(p));
        res_end = n_rows;
        r_v.assign(E, -1);
        r_w.assign(E, -1);
        if (use_src())
            for (int e = 0; e < E; ++e)
                if (dyn[e]) {
                    r_v[e] = rows(2);
                    r_w[e] = rows(1);
                }
        // rows + FL + DONE + the pass's mask words + the fixed point's reduction words (in the
        // row buffer when it is large enough)
        const long red = (!global_rows && (long)std::max(n_rows, 1) * 64 * ng >= nfl + 2) ? 0 : nfl + 2;
        const long lds = (global_rows ? 0L : (long)n_rows * 256 * ng) + (long)nfl * 4 + 4 * (n_split * ng + 1) +
                         4L * (nfl / 2) + 4 * red + (has_epi() && !epi_q_in_rows() ? (long)kEpiQRows * 256 * ng : 0L) +
                         (has_epi() && epi_lds ? (long)(cfg.epilogue == VMAS_EPILOGUE_BALANCE ? sizeof(VmasBalanceIO)
                                                                                            : sizeof(VmasTransportIO)) : 0L);
        if (lds > lds_budget) {
            *why = "LDS budget exceeded (" + it(lds) + " B)";
            return false;
        }
        // argument block slots
        for (auto& v : ptr_of) v.assign(std::max(E, std::max(A, J)) + 1, -1);
        for (auto& a : str_of)
            for (auto& v : a) v.assign(std::max(E, std::max(A, J)) + 1, -1);
        for (int e = 0; e < E; ++e) {
            if (!(dyn[e] || in_pair[e])) continue;
            ptr(S_POS, e), str(S_POS, 0, e), str(S_POS, 1, e);
            if (need_rot[e] || dyn[e]) ptr(S_ROT, e), str(S_ROT, 0, e);
            if (dyn[e]) {
                ptr(S_VEL, e), str(S_VEL, 0, e), str(S_VEL, 1, e);
                ptr(S_ANG, e), str(S_ANG, 0, e);
                if (ed[e].flags & VMAS_F_GRAVITY) ptr(S_GRAV, e), str(S_GRAV, 0, e), str(S_GRAV, 1, e);
                if (ed[e].agent_index >= 0) {
                    const int a = ed[e].agent_index;
                    ptr(S_FORCE, a), str(S_FORCE, 0, a), str(S_FORCE, 1, a);
                    ptr(S_TORQUE, a), str(S_TORQUE, 0, a);
                }
            }
        }
        for (int p = 0; p < P; ++p)
            if (pd[p].cls == VMAS_PAIR_JOINT) ptr(S_JFIX, pd[p].joint), str(S_JFIX, 0, pd[p].joint);
        if (str_src.size() % 2) str_src.push_back({-1, 0});  // keep the int block 8-byte aligned
        plan_params();
        {
            const char* tl = getenv("VMAS_JIT_TAIL");
            tail = has_epi() && !(tl && tl[0] == '0');
            if (tail && arg_bytes() > kMaxArgBytes) tail = false;
        }
        if (arg_bytes() > kMaxArgBytes) {
            *why = "kernel argument block too large (" + it(arg_bytes()) + " B)";
            return false;
        }
        return true;
    }

    // output pointers: pos, vel, rot, ang_vel, force, torque (+ forces_dict, torques_dict rows)
    size_t n_out() const { return cfg.export_forces ? 8 : 6; }

    // a scenario program compiled into the module (VmasWorldConfig.epilogue): its own kernel and
    // k_world's optional epilogue, whose argument block pointer is Args.epi
    bool has_epi() const { return cfg.epilogue == VMAS_EPILOGUE_BALANCE || cfg.epilogue == VMAS_EPILOGUE_TRANSPORT; }
    // the program's argument block (vmas_programs.hpp program_group overloads)
    const char* epi_type() const { return cfg.epilogue == VMAS_EPILOGUE_BALANCE ? "VmasBalanceIO" : "VmasTransportIO"; }
    // the call running the program for group g (vmas_programs.hpp balance_group / transport_group)
    std::string epi_call(const std::string& io, const std::string& g, const std::string& wave, const std::string& lane,
                         const std::string& q, const std::string& src = "") const {
        if (cfg.epilogue == VMAS_EPILOGUE_BALANCE)
            return "balance_group(" + io + ", " + g + ", " + wave + ", " + it(nw) + ", " + lane + ", " + q + src + ")";
        return "transport_group(" + io + ", " + g + ", " + wave + ", " + it(nw) + ", " + lane + ")";
    }
    bool epi_q_in_rows() const {
        return !global_rows && (use_src() ? res_end - res_first >= kEpiQRows : n_rows >= kEpiQRows);
    }
    // the epilogue's state from the rows (balance only; not with rows in global memory)
    bool use_src() const { return epi_src && cfg.epilogue == VMAS_EPILOGUE_BALANCE && !global_rows; }
    // Q's first row in the row buffer (epi_q_in_rows)
    long epi_q_row() const { return use_src() ? res_first : 0; }
    // byte offset of Args.epi (after the fixed pointers: the value slots follow it)
    size_t epi_offset() const { return 8 * (std::max<size_t>(ptr_src.size(), 1) + n_out() + 7 + (global_rows ? 1 : 0)); }
    // byte offset of Args.wbd (after epi): the state write-back's backup delta (0: off; see wb_text)
    size_t wbd_offset() const { return epi_offset() + (has_epi() ? 8 : 0); }

    size_t tail_offset() const {  // byte offset of Args.tail (after the value slots)
        // (+4 ints: B, S, sdt, max_pass; then the value slots; padded to the 8-byte alignment)
        const size_t n = 8 * (std::max<size_t>(ptr_src.size(), 1) + n_out() + 7 + (global_rows ? 1 : 0) + (has_epi() ? 1 : 0) + 1) +
                         4 * (std::max<size_t>(str_src.size(), 2) + 4) +
                         4 * std::max<size_t>(prm_src.size(), 1);
        return (n + 7) & ~(size_t)7;
    }
    size_t arg_bytes() const {  // layout of the generated struct Args
        return tail_offset() + (tail ? sizeof(VmasTail) : 0);
    }

    // expressions for entity e as seen by wave w (registers when w owns it)
    static std::string row(int r, int k = 0) { return "L[" + it((long)(r + k) * 64) + " + lane]"; }
    bool mine(int e, int w) const { return dyn[e] && owner[e] == w; }
    // Other waves' entities a wave's pair tasks read: with pair_preload, held in registers (q/u/o
    // <e>) -- static ones loaded once per group, dynamic ones at the top of each pair phase, all
    // reads in flight together -- instead of LDS reads at each use (inside the pairs' branches).
    std::vector<char> pre_pos, pre_trig, pre_rot;  // of the wave being generated
    std::string pos(int e, int w) const {
        if (mine(e, w)) return "p" + it(e);
        if (!pre_pos.empty() && pre_pos[e]) return "q" + it(e);
        return "mk(" + row(r_p[e]) + ", " + row(r_p[e], 1) + ")";
    }
    std::string rot(int e, int w) const {
        if (mine(e, w)) return "r" + it(e);
        if (!pre_rot.empty() && pre_rot[e]) return "o" + it(e);
        return row(r_rot[e]);
    }
    std::string trig(int e, int w) const {
        if (mine(e, w)) return "t" + it(e);
        if (!pre_trig.empty() && pre_trig[e]) return "u" + it(e);
        return "Trig{" + row(r_trig[e]) + ", " + row(r_trig[e], 1) + ", " + row(r_trig[e], 2) + ", " +
               row(r_trig[e], 3) + "}";
    }
    // the entities (and which of their rows) wave w's pair tasks read, outside its own registers
    void task_reads(int w, std::vector<char>& rp, std::vector<char>& rt, std::vector<char>& rr) const {
        rp.assign(E, 0);
        rt.assign(E, 0);
        rr.assign(E, 0);
        for (const Task& k : wave_tasks[w]) {
            if (k.part == kFinish) continue;
            const VmasPairDesc& q = pd[k.pair];
            for (int side = 0; side < 2; ++side) {
                const int e = side ? q.eb : q.ea;
                if (mine(e, w)) continue;
                rp[e] = 1;
                const bool t = q.cls == VMAS_PAIR_LL || q.cls == VMAS_PAIR_BL || q.cls == VMAS_PAIR_BB ||
                               q.cls == VMAS_PAIR_JOINT ||
                               (side == 0 && (q.cls == VMAS_PAIR_LS || q.cls == VMAS_PAIR_BS));
                if (t && r_trig[e] >= 0) rt[e] = 1;
                if (q.cls == VMAS_PAIR_JOINT && r_rot[e] >= 0) rr[e] = 1;
            }
        }
    }
    std::string preload(int e, bool p, bool t, bool r) const {
        std::string o;
        if (p) o += "        const V2 q" + it(e) + " = mk(" + row(r_p[e]) + ", " + row(r_p[e], 1) + ");\n";
        if (t)
            o += "        const Trig u" + it(e) + " = Trig{" + row(r_trig[e]) + ", " + row(r_trig[e], 1) + ", " +
                 row(r_trig[e], 2) + ", " + row(r_trig[e], 3) + "};\n";
        if (r) o += "        const float o" + it(e) + " = " + row(r_rot[e]) + ";\n";
        return o;
    }
    std::string P_(Src s, int i) const { return "a.ptr[" + it(ptr_of[s][i]) + "]"; }
    std::string S_(Src s, int k, int i) const { return "a.str[" + it(str_of[s][k][i]) + "]"; }
    // rb: a field the state write-back overwrites, read from the backup in a re-run pass (rbd)
    std::string ld2(Src s, int i, bool rb = false) const {
        return "ld2(" + (rb ? "rbp(" + P_(s, i) + ", rbd)" : P_(s, i)) + ", " + S_(s, 0, i) + ", " + S_(s, 1, i) + ", bb)";
    }
    std::string ld1(Src s, int i, bool rb = false) const {
        return (rb ? "rbp(" + P_(s, i) + ", rbd)" : P_(s, i)) + "[(long)bb * " + S_(s, 0, i) + "]";
    }
    std::string mbit(int p) const { return "(m" + it(p >> 5) + " & " + it(1u << (p & 31)) + "u)"; }
    // first of the 4 result rows (fa.x, fa.y, ta, tb) of pair p
    int res(int p) const { return split[p] ? r_res[p] + 4 * parts(pd[p].cls) + 4 : r_res[p]; }

    // timestamp slot: per substep s, k = 0 pair phase done, 1 after its barrier, 2 entity phase
    // done, 3 after its barrier; prologue: slots max_substeps*4 + {0, 1}
    std::string stamp(int w, const std::string& slot) const {
        if (prof_block < 0) return "";
        return "if ((b >> 6) == " + it(prof_block) + " && lane == 0) a.prof[(" + slot + ") * " + it(kMaxNW) + " + " +
               it(w) + "] = __builtin_amdgcn_s_memtime();\n";
    }

    // per-workgroup record (profile builds, kProfRec words): slot 0 start (s_memrealtime), 1 HW_ID,
    // 2 XCC_ID, 3 leaving the group loop, 4 / 5 start / end of its last group, 6 / 7 around the
    // first claim (vmas_jit_ops.hpp), 8 + w HW_ID of wave w; after the phase stamps
    std::string block_stamp(int k, const std::string& v) const {
        if (prof_block < 0) return "";
        return "    if (threadIdx.x == 0 && blockIdx.x < " + it(kProfBlocks) + ") a.prof[" +
               it((long)(cfg.max_substeps * 4 + 2) * kMaxNW) + " + blockIdx.x * " + it(kProfRec) + " + " + it(k) +
               "] = " + v + ";\n";
    }

    // The STRUCTURE of a dynamic entity (shape, flags, slots, dimensions) is constexpr; its
    // VALUES (mass, inertia, drag, frictions, speed / force / torque limits) are zero here and
    // come from the kernel arguments (a.prm, prm_slots), so a world whose values change (a mass
    // re-rolled on every reset, ref scenarios/debug/het_mass.py:48-54) keeps its code object.
    // Which values are kernel arguments: bit k = entity value field k (kPrm*), bit 11 = the
    // world's gravity and semidims.  Default 0x7FF: every entity value an argument, the world's
    // values folded -- as arguments they cost balance's k_world ~0.8 us (+2.4 %; a folded zero
    // gravity component and semidim clamps simplify; interleaved A/B, profiles/r03/run8_prm_ab),
    // and scenarios change world values far more rarely than entity masses (a change rebuilds).
    // VMAS_JIT_PRM_MASK overrides (A/B).
    unsigned prm_mask = kPrmMaskDefault;
    std::string desc(int e) const {
        const VmasEntityDesc& d = ed[e];
        auto v = [&](int k) { return (prm_mask >> k) & 1u ? std::string("0.f") : fl(prm_value(d, k)); };
        std::string o = "{" + it(d.shape) + ", " + it(d.flags) + "u, " + it(d.agent_index) + ", " + it(d.out_lin) + ", " +
                        it(d.out_rot) + ", " + it(d.out_force) + ", " + it(d.out_torque) + ", " + fl(d.radius) + ", " +
                        fl(d.half_length) + ", " + fl(d.half_width);
        for (int k = 0; k <= kPrmTRange; ++k) o += ", " + v(k);
        return o + "}";
    }
    // the value fields a dynamic entity's code reads (by its flags), in VmasEntityDesc order
    std::vector<int> value_fields(const VmasEntityDesc& d) const {
        std::vector<int> f = value_fields_all(d), out;
        for (int k : f)
            if ((prm_mask >> k) & 1u) out.push_back(k);
        return out;
    }
    static std::vector<int> value_fields_all(const VmasEntityDesc& d) {
        std::vector<int> f;
        const bool mov = d.flags & VMAS_F_MOVABLE, rotb = d.flags & VMAS_F_ROTATABLE;
        if (mov) f.push_back(kPrmMass);
        if (rotb) f.push_back(kPrmInertia);
        if (mov || rotb) f.push_back(kPrmDrag);
        if (d.flags & VMAS_F_LIN_FRIC) f.push_back(kPrmLinFric);
        if (d.flags & VMAS_F_ANG_FRIC) f.push_back(kPrmAngFric);
        if (d.flags & VMAS_F_MAX_SPEED) f.push_back(kPrmMaxSpeed);
        if (d.flags & VMAS_F_V_RANGE) f.push_back(kPrmVRange);
        if (d.flags & VMAS_F_MAX_F) f.push_back(kPrmMaxF);
        if (d.flags & VMAS_F_F_RANGE) f.push_back(kPrmFRange);
        if (d.flags & VMAS_F_MAX_T) f.push_back(kPrmMaxT);
        if (d.flags & VMAS_F_T_RANGE) f.push_back(kPrmTRange);
        return f;
    }
    static const char* field_name(int k) {
        static const char* n[] = {"mass", "inertia", "one_minus_drag", "lin_fric", "ang_fric", "max_speed",
                                  "v_range", "max_f", "f_range", "max_t", "t_range"};
        return n[k];
    }
    // kernel-argument value slots: (entity, field) pairs, then the world's gravity x / y and
    // semidims (kPrmWorld + 0..3); laid out once in plan()
    std::vector<std::pair<int, int>> prm_src;
    std::vector<int> prm_of;  // first slot of entity e's fields (-1 if none)
    int prm_world = -1;
    void plan_params() {
        prm_src.clear();
        prm_of.assign(E, -1);
        for (int e = 0; e < E; ++e) {
            if (!dyn[e]) continue;
            prm_of[e] = (int)prm_src.size();
            for (int k : value_fields(ed[e])) prm_src.push_back({e, k});
        }
        prm_world = (int)prm_src.size();
        for (int k = 0; k < 4; ++k) prm_src.push_back({-1, k});
    }
    // prologue: the value slots into LDS, constant indices only (a loop indexing a.prm
    // dynamically makes the compiler keep the whole by-value argument block addressable:
    // balance static VALU +27 %)
    std::string prm_copy() const {
        std::string o = "    if (threadIdx.x == 0) {";
        for (size_t i = 0; i < prm_src.size(); ++i) o += " PRM[" + it((long)i) + "] = a.prm[" + it((long)i) + "];";
        return o + " }\n";
    }
    // the entity's runtime desc: the constexpr structure with its value fields from a.prm
    std::string runtime_desc(int e, const std::string& I) const {
        const std::string s = it(e);
        std::string o = I + "VmasEntityDesc D" + s + " = D" + s + "c;\n";
        int slot = prm_of[e];
        for (int k : value_fields(ed[e])) o += I + "D" + s + "." + field_name(k) + " = PRM[" + it(slot++) + "];\n";
        return o;
    }

    void publish(std::string& o, int e, const std::string& ind, bool with_pos, bool with_rot) const {
        if (!in_pair[e]) return;
        if (with_pos) o += ind + row(r_p[e]) + " = p" + it(e) + ".x; " + row(r_p[e], 1) + " = p" + it(e) + ".y;\n";
        if (with_rot && r_rot[e] >= 0) o += ind + row(r_rot[e]) + " = r" + it(e) + ";\n";
        if (with_rot && r_trig[e] >= 0)
            o += ind + row(r_trig[e]) + " = t" + it(e) + ".c0; " + row(r_trig[e], 1) + " = t" + it(e) + ".s0; " +
                 row(r_trig[e], 2) + " = t" + it(e) + ".c1; " + row(r_trig[e], 3) + " = t" + it(e) + ".s1;\n";
    }

    std::string pair_call(int p, int w) const {
        const VmasPairDesc& q = pd[p];
        const int a = q.ea, b = q.eb;
        const VmasEntityDesc &da = ed[a], &db = ed[b];
        const std::string ha = bl(da.flags & VMAS_F_HOLLOW), hb = bl(db.flags & VMAS_F_HOLLOW);
        const std::string dm = fl(q.dmin);
        switch (q.cls) {
            case VMAS_PAIR_SS: return "pair_ss(" + pos(a, w) + ", " + pos(b, w) + ", " + dm + ", WK)";
            case VMAS_PAIR_LS:
                return "pair_ls(" + pos(a, w) + ", " + trig(a, w) + ", " + fl(da.half_length) + ", " + pos(b, w) +
                       ", " + dm + ", WK)";
            case VMAS_PAIR_LL:
                return "pair_ll(" + pos(a, w) + ", " + trig(a, w) + ", " + fl(da.half_length) + ", " + pos(b, w) +
                       ", " + trig(b, w) + ", " + fl(db.half_length) + ", " + dm + ", WK)";
            case VMAS_PAIR_BS:
                return "pair_bs(" + pos(a, w) + ", " + trig(a, w) + ", " + fl(da.half_length) + ", " +
                       fl(da.half_width) + ", " + ha + ", " + pos(b, w) + ", " + dm + ", WK)";
            case VMAS_PAIR_BL:
                return "pair_bl(" + pos(a, w) + ", " + trig(a, w) + ", " + fl(da.half_length) + ", " +
                       fl(da.half_width) + ", " + ha + ", " + pos(b, w) + ", " + trig(b, w) + ", " +
                       fl(db.half_length) + ", " + dm + ", WK)";
            case VMAS_PAIR_BB:
                return "pair_bb(" + pos(a, w) + ", " + trig(a, w) + ", " + fl(da.half_length) + ", " +
                       fl(da.half_width) + ", " + ha + ", " + pos(b, w) + ", " + trig(b, w) + ", " +
                       fl(db.half_length) + ", " + fl(db.half_width) + ", " + hb + ", " + dm + ", WK)";
            default: {
                const VmasJointDesc& j = jd[q.joint];
                return "pair_joint(" + pos(a, w) + ", " + rot(a, w) + ", " + trig(a, w) + ", " + pos(b, w) + ", " +
                       rot(b, w) + ", " + trig(b, w) + ", mk(" + fl(j.delta_a_x) + ", " + fl(j.delta_a_y) + "), mk(" +
                       fl(j.delta_b_x) + ", " + fl(j.delta_b_y) + "), " + fl(j.dist) + ", " + bl(j.rotate) +
                       ", fixed_rot, WK)";
            }
        }
    }

    // Broadphase activity bits of a pair, gathered in wave-uniform words (fr<k> / fz<k>) over the
    // wave's pair phase and ORed into the workgroup's LDS words once per substep (flag_flush).
    std::string flag_r(int p, const std::string& ind) const {  // R: some env within the broadphase radius
        return ind + "if (a.blk && __ballot(inr && valid)) fr" + it(p >> 5) + " |= " + it(1u << (p & 31)) + "u;\n";
    }
    std::string flag_z(int p, const std::string& ind) const {  // Z: an out-of-range env got a force
        return ind + "if (a.blk && __ballot(valid && !inr && (o.fa.x != 0.f || o.fa.y != 0.f || o.ta != 0.f || "
                     "o.tb != 0.f))) fz" + it(p >> 5) + " |= " + it(1u << (p & 31)) + "u;\n";
    }
    std::string flag_flush(const std::vector<char>& words) const {
        std::string o;
        for (int k = 0; k < W; ++k)
            if (words[k])
                o += "        if (lane == 0) {\n"
                     "            if (fr" + it(k) + ") atomicOr(&FL[s * " + it(W) + " + " + it(k) + "], fr" + it(k) + ");\n"
                     "            if (fz" + it(k) + ") atomicOr(&FL[(a.S + s) * " + it(W) + " + " + it(k) + "], fz" +
                     it(k) + ");\n        }\n";
        return o;
    }
    // result rows a whole pair needs: no torque is ever read from a sphere-sphere result, and
    // none for the sphere side of a line/box-sphere result (the entity items' torque flags)
    int res_rows(int p) const {
        const int c = pd[p].cls;
        return c == VMAS_PAIR_SS ? 2 : (c == VMAS_PAIR_LS || c == VMAS_PAIR_BS) ? 3 : 4;
    }
    std::string store_res(int p, const std::string& ind) const {
        const int r = res(p), n = split[p] ? 4 : res_rows(p);
        std::string o = ind + row(r) + " = o.fa.x; " + row(r, 1) + " = o.fa.y;";
        if (n > 2) o += " " + row(r, 2) + " = o.ta;";
        if (n > 3) o += " " + row(r, 3) + " = o.tb;";
        return o + "\n";
    }

    void task_code(std::string& o, const Task& k, int w) const {
        const int p = k.pair;
        const VmasPairDesc& q = pd[p];
        const std::string I = "            ";
        o += "        {  // pair " + it(p) + " class " + it(q.cls) + " (" + it(q.ea) + ", " + it(q.eb) + ")" +
             (k.part >= 0 ? " part " + it(k.part) : k.part == kFinish ? std::string(" finish") : std::string()) +
             "\n";
        if (k.part == kFinish) {  // wait for the parts, select, finish the contact, store the result
            const int n = parts(q.cls), base = r_res[p], c = base + 4 * n;
            o += I + "if " + mbit(p) + " {\n";
            o += I + "    if (lane == 0) {\n" + I + "        while (atomicAdd(&DONE[" + it(split_idx[p]) + "], 0u) < " +
                 it(n) + "u) __builtin_amdgcn_s_sleep(1);\n" + I + "    }\n";
            o += I + "    __builtin_amdgcn_wave_barrier();\n" + I + "    __threadfence_block();\n";
            o += I + "    const V2 ca = mk(" + row(c) + ", " + row(c, 1) + "), cb = mk(" + row(c, 2) + ", " + row(c, 3) +
                 ");\n";
            o += I + "    const Pts q = select_min(" + it(n) + ", [&](int i) { const float* x = L + " +
                 it((long)base * 64) + " + i * 256 + lane; return Pts{mk(x[0], x[64]), mk(x[128], x[192])}; });\n";
            if (q.cls == VMAS_PAIR_BL)
                o += I + "    const PairOut o = bl_finish(ca, " + bl(ed[q.ea].flags & VMAS_F_HOLLOW) + ", cb, q, " +
                     fl(q.dmin) + ", WK);\n";
            else
                o += I + "    const PairOut o = bb_finish(ca, " + bl(ed[q.ea].flags & VMAS_F_HOLLOW) + ", cb, " +
                     bl(ed[q.eb].flags & VMAS_F_HOLLOW) + ", q, " + fl(q.dmin) + ", WK);\n";
            o += I + "    const bool inr = norm(ca - cb) <= " + fl(q.bp_radius) + ";\n";
            o += flag_z(p, I + "    ");
            o += store_res(p, I + "    ");
            o += I + "}\n        }\n";
            return;
        }
        const bool needs_d2 = q.cls != VMAS_PAIR_JOINT && (k.part == kWhole || k.part == 0);
        if (needs_d2)  // squared centre distance, rounded as inside norm()
            o += I + "const V2 dl = " + pos(q.ea, w) + " - " + pos(q.eb, w) + ";\n" + I +
                 "const float d2 = dl.x * dl.x + dl.y * dl.y;\n";
        if (k.part == kWhole || k.part == 0) {
            if (q.cls != VMAS_PAIR_JOINT)  // norm(pa - pb) <= bp_radius, without the sqrt
                o += I + "const bool inr = d2 <= " + fl(sq_limit(q.bp_radius)) + ";\n";
            else
                o += I + "const bool inr = true;\n";
            o += flag_r(p, I);
        }
        o += I + "if " + mbit(p) + " {\n";
        if (k.part == kWhole) {
            if (q.cls == VMAS_PAIR_JOINT) {
                const int j = q.joint;
                o += I + "    const float* frp = " + P_(S_JFIX, j) + ";\n";
                o += I + "    const float fixed_rot = frp ? frp[(long)bb * " + S_(S_JFIX, 0, j) + "] : " +
                     fl(jd[j].fixed_rotation) + ";\n";
            }
            if (q.cls == VMAS_PAIR_SS)  // every lane beyond d_min: the reference's force is 0
                o += I + "    const PairOut o = vote_all(d2 > " + fl(sq_limit(q.dmin)) +
                     ") ? PairOut{mk(0.f, 0.f), 0.f, 0.f} : " + pair_call(p, w) + ";\n";
            else
                o += I + "    const PairOut o = " + pair_call(p, w) + ";\n";
            o += store_res(p, I + "    ");
            // A sphere pair whose squared broadphase limit is at or beyond its contact limit: an env
            // out of range gets exactly zero force (core.py:2832, dist > dist_min) unless its
            // distance is NaN (then the force is NaN), so Z reduces to "some valid env has a NaN
            // distance" -- no dependency on the force.
            const bool z_nan_only = q.cls == VMAS_PAIR_SS && sq_limit(q.bp_radius) >= sq_limit(q.dmin);
            if (z_nan_only)
                o += I + "    if (a.blk && __ballot(valid && d2 != d2)) fz" + it(p >> 5) + " |= " + it(1u << (p & 31)) +
                     "u;\n";
            else if (q.cls != VMAS_PAIR_JOINT)
                o += flag_z(p, I + "    ");
            o += I + "}\n        }\n";
            return;
        }
        const VmasEntityDesc &da = ed[q.ea], &db = ed[q.eb];
        if (q.cls == VMAS_PAIR_BL)
            o += I + "    const Pts q = bl_part(" + pos(q.ea, w) + ", " + trig(q.ea, w) + ", " + fl(da.half_length) + ", " +
                 fl(da.half_width) + ", " + pos(q.eb, w) + ", " + trig(q.eb, w) + ", " + fl(db.half_length) + ", " +
                 it(k.part) + ");\n";
        else
            o += I + "    const Pts q = bb_part(" + pos(q.ea, w) + ", " + trig(q.ea, w) + ", " + fl(da.half_length) + ", " +
                 fl(da.half_width) + ", " + pos(q.eb, w) + ", " + trig(q.eb, w) + ", " + fl(db.half_length) + ", " +
                 fl(db.half_width) + ", " + it(k.part) + ");\n";
        const int r = r_res[p] + 4 * k.part;
        o += I + "    " + row(r) + " = q.p1.x; " + row(r, 1) + " = q.p1.y; " + row(r, 2) + " = q.p2.x; " + row(r, 3) +
             " = q.p2.y;\n";
        if (k.part == 0) {  // the finish needs the pre-integration centres
            const int c = r_res[p] + 4 * parts(q.cls);
            const std::string pa = pos(q.ea, w), pb = pos(q.eb, w);
            o += I + "    { const V2 ca = " + pa + ", cb = " + pb + "; " + row(c) + " = ca.x; " + row(c, 1) + " = ca.y; " +
                 row(c, 2) + " = cb.x; " + row(c, 3) + " = cb.y; }\n";
        }
        o += I + "}\n";
        o += I + "__threadfence_block();\n" + I + "if (lane == 0) atomicAdd(&DONE[" + it(split_idx[p]) + "], 1u);\n";
        o += "        }\n";
    }

    void wave_body(std::string& o, int w) {
        o += "template <> __device__ __forceinline__ bool run<" + it(w) +
             ">(const Args& a, float* L, uint32_t* FL, uint32_t* DONE, const uint32_t* MSK, int lane, int b, int bb, "
             "bool valid, long long rbd, bool bk, bool wbk, bool spec, bool spec_ok, uint32_t* QL" +
             std::string(use_src() ? ", const VmasBalanceIO* prog" : "") + ") {\n";
        // prologue: static pair entities (loaded once), dynamic entities into registers
        std::string bk_code;  // the state write-back's backup stores (wb_helpers)
        for (int e : wave_static[w]) {
            o += "    {  // static entity " + it(e) + "\n";
            o += "        const V2 p" + it(e) + " = " + ld2(S_POS, e) + ";\n";
            if (need_rot[e]) o += "        const float r" + it(e) + " = " + ld1(S_ROT, e) + ";\n";
            if (need_trig[e])
                o += "        const Trig t" + it(e) + " = make_trig_for(r" + it(e) + ", " + bl(ed[e].shape == VMAS_BOX) +
                     ");\n";
            publish(o, e, "        ", true, true);
            o += "    }\n";
        }
        for (int e : wave_ents[w]) {
            const VmasEntityDesc& d = ed[e];
            const std::string s = it(e);
            const bool lin = d.out_lin >= 0, rotf = d.out_rot >= 0;  // (the fields a write-back overwrites)
            o += "    V2 p" + s + " = " + ld2(S_POS, e, lin) + ", v" + s + " = " + ld2(S_VEL, e, lin) + ";\n";
            o += "    float r" + s + " = " + ld1(S_ROT, e, rotf) + ", w" + s + " = " + ld1(S_ANG, e, rotf) + ";\n";
            if (lin || rotf) {  // (stored after the first barrier, once the group is known to be ours)
                if (lin)
                    bk_code += "        bk2(" + P_(S_POS, e) + ", " + S_(S_POS, 0, e) + ", " + S_(S_POS, 1, e) + ", bb, a.wbd, p" + s +
                               ");\n        bk2(" + P_(S_VEL, e) + ", " + S_(S_VEL, 0, e) + ", " + S_(S_VEL, 1, e) +
                               ", bb, a.wbd, v" + s + ");\n";
                if (rotf)
                    bk_code += "        bk1(" + P_(S_ROT, e) + ", " + S_(S_ROT, 0, e) + ", bb, a.wbd, r" + s + ");\n        bk1(" +
                               P_(S_ANG, e) + ", " + S_(S_ANG, 0, e) + ", bb, a.wbd, w" + s + ");\n";
            }
            if (d.agent_index >= 0)
                o += "    V2 af" + s + " = " + ld2(S_FORCE, d.agent_index) + "; float at" + s + " = " +
                     ld1(S_TORQUE, d.agent_index) + ";\n";
            else
                o += "    V2 af" + s + " = mk(0.f, 0.f); float at" + s + " = 0.f;\n";
            if (d.flags & VMAS_F_GRAVITY) o += "    const V2 eg" + s + " = " + ld2(S_GRAV, e) + ";\n";
            else o += "    const V2 eg" + s + " = mk(0.f, 0.f);\n";
            if (need_trig[e])
                o += "    Trig t" + s + " = make_trig_for(r" + s + ", " + bl(d.shape == VMAS_BOX) + ");\n";
            publish(o, e, "    ", true, true);
            // World.forces_dict / torques_dict: the totals of the last substep (core.py:1975-1992)
            if (cfg.export_forces) o += "    float lfx" + s + " = 0.f, lfy" + s + " = 0.f, ltq" + s + " = 0.f;\n";
            // its parameter values, read from LDS once per group (registers for the substeps)
            o += runtime_desc(e, "    ");
        }
        const std::string pro = it((long)cfg.max_substeps * 4);
        // the speculative first claim (loop_text): its result, waited for only here -- after this
        // wave's state loads are in flight -- and handed to every wave by the barrier below
        if (w == 0) o += "    if (spec && threadIdx.x == 0) QL[65] = spec_ok ? 1u : 0u;\n";
        // the epilogue's row table (src_fns), behind the same barrier, after wave 0's loads are in flight
        if (w == 0 && use_src()) o += "    if (prog) src_rows(a, prog, lane);\n";
        o += "    " + stamp(w, pro);
        o += "    __syncthreads();\n";
        o += "    const bool own = !spec || QL[65] != 0u;  // (a lost speculative claim: compute, store nothing)\n";
        if (!bk_code.empty()) o += "    if (bk && valid && own) {\n" + bk_code + "    }\n";
        o += "    " + stamp(w, pro + " + 1");
        std::vector<char> rp, rt, rr;
        if (pair_preload) {
            task_reads(w, rp, rt, rr);
            for (int e = 0; e < E; ++e)  // static entities: once per group
                if (!dyn[e] && (rp[e] || rt[e] || rr[e])) o += preload(e, rp[e], rt[e], rr[e]).substr(4);
        }
        o += "    for (int s = 0; s < a.S; ++s) {\n";
        // Issue priority falling with the substep: of the two workgroups on a CU the one behind
        // gets the issue slots, so they finish together instead of the second running its last
        // substeps alone at half occupancy (balance 40.6-41.0 -> 39.7-40.0 us, flocking 38.2 ->
        // 37.1 us, interleaved; priority by wave load measured no gain: profiles/r02/run14_prio)
        if (prio_mode == 1)
            o += "        if (4 * s < a.S) __builtin_amdgcn_s_setprio(3); else if (2 * s < a.S) __builtin_amdgcn_s_setprio(2);"
                 " else if (4 * s < 3 * a.S) __builtin_amdgcn_s_setprio(1); else __builtin_amdgcn_s_setprio(0);\n";
        std::vector<char> word(W, 0);  // mask words this wave reads
        for (const Task& t : wave_tasks[w]) word[t.pair >> 5] = 1;
        for (int e : wave_ents[w])
            for (const Item& x : items[e]) word[x.pair >> 5] = 1;
        for (int k = 0; k < W; ++k)
            if (word[k]) o += "        const uint32_t m" + it(k) + " = MSK[s * " + it(W) + " + " + it(k) + "];\n";
        std::vector<char> fword(W, 0);  // flag words this wave's tasks set
        for (const Task& t : wave_tasks[w]) fword[t.pair >> 5] = 1;
        for (int k = 0; k < W; ++k)
            if (fword[k]) o += "        uint32_t fr" + it(k) + " = 0u, fz" + it(k) + " = 0u;\n";
        if (pair_preload) {
            for (int e = 0; e < E; ++e)  // dynamic entities: at the top of each pair phase
                if (dyn[e] && (rp[e] || rt[e] || rr[e])) o += preload(e, rp[e], rt[e], rr[e]);
            pre_pos = rp;
            pre_trig = rt;
            pre_rot = rr;
        }
        for (const Task& t : wave_tasks[w]) task_code(o, t, w);
        pre_pos.clear();
        pre_trig.clear();
        pre_rot.clear();
        o += flag_flush(fword);
        o += "        " + stamp(w, "s * 4");
        o += "        __syncthreads();\n";
        o += "        " + stamp(w, "s * 4 + 1");
        if (w == 0 && n_split)  // no part signals before the next pair phase
            o += "        for (int i = lane; i < " + it(n_split) + "; i += 64) DONE[i] = 0u;\n";
        // entity phase
        for (int e : wave_ents[w]) {
            const VmasEntityDesc& d = ed[e];
            const std::string s = it(e);
            const bool mov = d.flags & VMAS_F_MOVABLE, rotb = d.flags & VMAS_F_ROTATABLE;
            o += "        {  // entity " + s + "\n";
            o += "            float fx, fy, tq;\n";
            o += "            pre_forces(D" + s + ", " + bl(d.agent_index >= 0) + ", af" + s + ", at" + s + ", v" + s +
                 ", w" + s + ", eg" + s + ", " + bl(d.flags & VMAS_F_GRAVITY) + ", GX, GY, HAS_G, a.sdt, fx, fy, tq);\n";
            // every contribution row read up front (independent LDS reads in flight together),
            // then added in the reference's order where its pair is active (a select: the same
            // sums as the branch)
            if (entity_preload) {
                int k = 0;
                for (const Item& x : items[e]) {
                    const int r = res(x.pair);
                    const std::string c = "c" + it(k++);
                    if (mov) o += "            const float " + c + "x = " + row(r) + ", " + c + "y = " + row(r, 1) + ";\n";
                    if (rotb && x.torque) o += "            const float " + c + "t = " + row(r, x.side ? 3 : 2) + ";\n";
                }
                k = 0;
                for (const Item& x : items[e]) {
                    const std::string c = "c" + it(k++), m = mbit(x.pair);
                    if (mov) {
                        const std::string sx = x.side ? "-" + c + "x" : c + "x", sy = x.side ? "-" + c + "y" : c + "y";
                        o += "            fx = " + m + " ? fx + " + sx + " : fx; fy = " + m + " ? fy + " + sy + " : fy;\n";
                    }
                    if (rotb && x.torque) o += "            tq = " + m + " ? tq + " + c + "t : tq;\n";
                }
            } else {
                for (const Item& x : items[e]) {
                    const int r = res(x.pair);
                    std::string body;
                    if (mov)
                        body += x.side ? "fx = fx + -" + row(r) + "; fy = fy + -" + row(r, 1) + "; "
                                       : "fx = fx + " + row(r) + "; fy = fy + " + row(r, 1) + "; ";
                    if (rotb && x.torque) body += "tq = tq + " + row(r, x.side ? 3 : 2) + "; ";
                    if (!body.empty()) o += "            if " + mbit(x.pair) + " { " + body + "}\n";
                }
            }
            if (cfg.export_forces) o += "            lfx" + s + " = fx; lfy" + s + " = fy; ltq" + s + " = tq;\n";
            o += "            integrate(D" + s + ", s, a.sdt, fx, fy, tq, HAS_XS, XS, HAS_YS, YS, p" + s + ", v" + s +
                 ", r" + s + ", w" + s + ");\n";
            if (need_trig[e] && rotb)
                o += "            t" + s + " = make_trig_for(r" + s + ", " + bl(d.shape == VMAS_BOX) + ");\n";
            publish(o, e, "            ", mov, rotb);
            o += "        }\n";
        }
        o += "        " + stamp(w, "s * 4 + 2");
        o += "        __syncthreads();\n";
        o += "        " + stamp(w, "s * 4 + 3");
        o += "    }\n";
        // the velocity rows balance's epilogue reads (use_src)
        if (use_src()) {
            std::string vr;
            for (int e : wave_ents[w])
                if (r_v[e] >= 0)
                    vr += "        " + row(r_v[e]) + " = v" + it(e) + ".x; " + row(r_v[e], 1) + " = v" + it(e) + ".y; " +
                          row(r_w[e]) + " = w" + it(e) + ";\n";
            if (!vr.empty()) o += "    if (a.epi) {\n" + vr + "    }\n";
        }
        // epilogue: the integrated fields into the fresh output tensors
        if (!wave_ents[w].empty()) {
            o += "    if (valid && own) {\n";
            for (int e : wave_ents[w]) {
                const VmasEntityDesc& d = ed[e];
                const std::string s = it(e);
                // sc1 (write-through) stores: a group re-run in a later fixed-point pass by a
                // workgroup on another XCD must not race a dirty line of the earlier pass
                // (vmas_jit_ops.hpp, memory order of the persistent launch)
                if (d.out_lin >= 0)
                    o += "        st_out2(a.out[0], (size_t)" + it(d.out_lin) + " * a.B + b, p" + s + ");\n        st_out2(a.out[1], (size_t)" +
                         it(d.out_lin) + " * a.B + b, v" + s + ");\n";
                if (d.out_rot >= 0)
                    o += "        st_out1(a.out[2], (size_t)" + it(d.out_rot) + " * a.B + b, r" + s + ");\n        st_out1(a.out[3], (size_t)" +
                         it(d.out_rot) + " * a.B + b, w" + s + ");\n";
                if (d.agent_index >= 0) {
                    if (d.out_force >= 0)
                        o += "        st_out2(a.out[4], (size_t)" + it(d.out_force) + " * a.B + b, af" + s + ");\n";
                    if (d.out_torque >= 0)
                        o += "        st_out1(a.out[5], (size_t)" + it(d.out_torque) + " * a.B + b, at" + s + ");\n";
                }
                if (cfg.export_forces)
                    o += "        st_out2(a.out[6], (size_t)" + s + " * a.B + b, mk(lfx" + s + ", lfy" + s +
                         "));\n        st_out1(a.out[7], (size_t)" + s + " * a.B + b, ltq" + s + ");\n";
                if (d.out_lin >= 0 || d.out_rot >= 0) {  // the state write-back into this step's inputs
                    o += "        if (wbk) {\n";
                    if (d.out_lin >= 0)
                        o += "            wb2(" + P_(S_POS, e) + ", " + S_(S_POS, 0, e) + ", " + S_(S_POS, 1, e) + ", b, p" + s +
                             ");\n            wb2(" + P_(S_VEL, e) + ", " + S_(S_VEL, 0, e) + ", " + S_(S_VEL, 1, e) + ", b, v" +
                             s + ");\n";
                    if (d.out_rot >= 0)
                        o += "            wb1(" + P_(S_ROT, e) + ", " + S_(S_ROT, 0, e) + ", b, r" + s + ");\n            wb1(" +
                             P_(S_ANG, e) + ", " + S_(S_ANG, 0, e) + ", b, w" + s + ");\n";
                    o += "        }\n";
                }
            }
            o += "    }\n";
        }
        o += "    return own;\n}\n\n";
    }

    // The state write-back (Args.wbd != 0; graph mode's rollback-free replays, vmas_graph_chain_set_writeback):
    // the step writes its integrated fields into its own inputs as well as into the fresh outputs, so
    // the replay needs no post-replay carry of the state (outputs -> inputs, simulator/environment/
    // _graph.py).  A group re-run in a later fixed-point pass must read the PRE-step state, which the
    // write-back has overwritten: the first pass stores each group's loaded state into a backup at
    // the same offsets (input + wbd; sc1, handed between workgroups like the outputs) and a re-run pass
    // reads it from there (rbp); the re-run's write-back lands last.  Stores only -- no extra loads on
    // the path that runs (one pass).
    std::string wb_helpers() const {
        return "__device__ __forceinline__ const float* rbp(const float* p, long long d) {\n"
               "    return reinterpret_cast<const float*>(reinterpret_cast<const char*>(p) + d);\n}\n"
               "__device__ __forceinline__ void bk1(const float* p, int s0, int b, long long d, float v) {\n"
               "    st_out1(const_cast<float*>(rbp(p, d)), (size_t)((long)b * s0), v);\n}\n"
               "__device__ __forceinline__ void bk2(const float* p, int s0, int s1, int b, long long d, V2 v) {\n"
               "    float* q = const_cast<float*>(rbp(p, d));\n"
               "    st_out1(q, (size_t)((long)b * s0), v.x);\n    st_out1(q, (size_t)((long)b * s0 + s1), v.y);\n}\n"
               "__device__ __forceinline__ void wb1(const float* p, int s0, int b, float v) {\n"
               "    const_cast<float*>(p)[(long)b * s0] = v;\n}\n"
               "__device__ __forceinline__ void wb2(const float* p, int s0, int s1, int b, V2 v) {\n"
               "    float* q = const_cast<float*>(p);\n    q[(long)b * s0] = v.x;\n    q[(long)b * s0 + s1] = v.y;\n}\n\n";
    }

    // Balance's epilogue reads the group's state from the rows (use_src): which row holds the
    // tensor an argument-block pointer names -- a dynamic entity's output (the fresh output buffer,
    // this launch's a.out) or a static entity's input (a.ptr) -- compared pointer and strides, once
    // per workgroup by thread 0 (prologue); -1: not held in a row, the program reads the tensor.
    std::string src_fns() const {
        std::string rp = "__device__ __forceinline__ int row_pos(const Args& a, const float* p, int s0, int s1) {\n";
        std::string rv = "__device__ __forceinline__ int row_vel(const Args& a, const float* p, int s0, int s1) {\n";
        std::string rr = "__device__ __forceinline__ int row_rot(const Args& a, const float* p, int s0) {\n";
        std::string rw = "__device__ __forceinline__ int row_ang(const Args& a, const float* p, int s0) {\n";
        for (int e = 0; e < E; ++e) {
            const VmasEntityDesc& d = ed[e];
            if (r_p[e] >= 0) {
                if (dyn[e] && d.out_lin >= 0)
                    rp += "    if (p == a.out[0] + (size_t)" + it(d.out_lin) + " * a.B * 2 && s0 == 2 && s1 == 1) return " +
                          it(r_p[e]) + ";\n";
                else if (!dyn[e] || d.out_lin < 0)
                    rp += "    if (p == " + P_(S_POS, e) + " && s0 == " + S_(S_POS, 0, e) + " && s1 == " + S_(S_POS, 1, e) +
                          ") return " + it(r_p[e]) + ";\n";
            }
            if (r_rot[e] >= 0) {
                if (dyn[e] && d.out_rot >= 0)
                    rr += "    if (p == a.out[2] + (size_t)" + it(d.out_rot) + " * a.B && s0 == 1) return " + it(r_rot[e]) + ";\n";
                else if (!dyn[e] || d.out_rot < 0)
                    rr += "    if (p == " + P_(S_ROT, e) + " && s0 == " + S_(S_ROT, 0, e) + ") return " + it(r_rot[e]) + ";\n";
            }
            if (r_v[e] >= 0 && d.out_lin >= 0)
                rv += "    if (p == a.out[1] + (size_t)" + it(d.out_lin) + " * a.B * 2 && s0 == 2 && s1 == 1) return " +
                      it(r_v[e]) + ";\n";
            if (r_w[e] >= 0 && d.out_rot >= 0)
                rw += "    if (p == a.out[3] + (size_t)" + it(d.out_rot) + " * a.B && s0 == 1) return " + it(r_w[e]) + ";\n";
        }
        const std::string end = "    return -1;\n}\n";
        return rp + end + rv + end + rr + "    (void)a; (void)p; (void)s0;\n" + end + rw + "    (void)a; (void)p; (void)s0;\n" + end +
               "__shared__ int ESRC[kBalFields];\n"
               "// (wave 0, a field per lane: thread 0 alone walking the fields held every workgroup ~3 us)\n"
               "__device__ __forceinline__ void src_rows(const Args& a, const VmasBalanceIO* io, int lane) {\n"
               "    for (int f = lane; f < kBalFields; f += 64) {\n"
               "        const float* p = nullptr;\n"
               "        int s0 = 0, s1 = 0, kind = 0;  // 0 position, 1 velocity, 2 rotation, 3 angular velocity\n"
               "        if (f < kBalLineRot) {\n"
               "            const VmasShapeRef* x = f == kBalPkgPos ? &io->package : f == kBalGoalPos ? &io->goal\n"
               "                                   : f == kBalLinePos ? &io->line : &io->floor;\n"
               "            p = x->pos; s0 = x->pos_s0; s1 = x->pos_s1;\n"
               "        } else if (f <= kBalFloorRot) {\n"
               "            const VmasShapeRef* x = f == kBalLineRot ? &io->line : &io->floor;\n"
               "            p = x->rot; s0 = x->rot_s0; kind = 2;\n"
               "        } else if (f < kBalAgPos) {\n"
               "            const VmasVec* v = f == kBalPkgVel ? &io->package_vel : f == kBalLineVel ? &io->line_vel : &io->line_ang_vel;\n"
               "            p = v->p; s0 = v->s0; s1 = v->s1; kind = f == kBalLineAng ? 3 : 1;\n"
               "        } else {\n"
               "            const int i = f < kBalAgVel ? f - kBalAgPos : f - kBalAgVel;\n"
               "            if (i < io->n_agents) {\n"
               "                const VmasVec* v = f < kBalAgVel ? &io->agent_pos[i] : &io->agent_vel[i];\n"
               "                p = v->p; s0 = v->s0; s1 = v->s1; kind = f < kBalAgVel ? 0 : 1;\n"
               "            }\n"
               "        }\n"
               "        ESRC[f] = !p ? -1 : kind == 0 ? row_pos(a, p, s0, s1) : kind == 1 ? row_vel(a, p, s0, s1)\n"
               "                              : kind == 2 ? row_rot(a, p, s0) : row_ang(a, p, s0);\n"
               "    }\n}\n\n";
    }

    // The group loop: one copy per wave (loop_per_wave, the default), each calling its own run<w>,
    // or one loop around a switch over the waves (VMAS_JIT_LOOP_PER_WAVE=0).  With one loop the
    // compiler hoists the loop-invariant address / stride values of EVERY wave's body above it,
    // all live at once (balance: 106 SGPRs and 163 v_writelane spills of them into VGPR lanes,
    // read back with v_readlane -- VALU instructions); with a loop per wave only that wave's are.
    bool loop_per_wave = true;  // (required by ng > 1)
    // the launch's first group run before its claim is confirmed (loop_text; VMAS_JIT_SPEC_CLAIM=0: claimed first)
    bool spec_claim = true;
    // Args.tail (vmas_tail.hpp): a replay's post-replay work run after the final decision, for the
    // modules whose k_world a kernel chain can fuse into one launch (a scenario program); dropped
    // when the argument block would outgrow kMaxArgBytes.  VMAS_JIT_TAIL=0: none (A/B).
    bool tail = false;
    // the scenario program's argument block copied into LDS at the launch's start (epi_lds, the
    // default; VMAS_JIT_EPI_LDS=0: read through Args.epi): the epilogue's field reads are LDS reads
    // instead of a cold scalar-cache miss per group
    bool epi_lds = true;
    std::string epi_text(const std::string& io) const {
        if (!has_epi()) return "";
        // The scenario program of this group (vmas_graph_chain_build fuses a replay's k_world and
        // k_program_jit into this launch): it reads the group's fields the waves just stored --
        // visible to the whole workgroup after the barrier (its workgroup-scope release / acquire;
        // agent-scope fences here write back L2 per group: 38 -> 159 us per launch) -- each pass of
        // the fixed point re-running it after its group, the final pass's writes last (as the
        // state outputs).  Q: the row buffer, idle between groups.
        const std::string lb = ng > 1 ? "Ls" : "L";
        const std::string q = epi_q_in_rows() ? lb + (epi_q_row() ? " + " + it(epi_q_row() * 64) : std::string())
                                               : (ng > 1 ? "EQ + sub * " + it((long)kEpiQRows * 64) : "EQ");
        // (balance: the group's state from the rows -- use_src, BalRows)
        const std::string src = use_src() ? ", &SRC" : "";
        return "        if (a.epi) {\n"
               "            __syncthreads();\n"
               + std::string(use_src() ? "            const BalRows SRC{" + lb + ", ESRC, lane};\n" : "") +
               "            " + (ng > 1 ? epi_call(io, "g * " + it(ng) + " + sub", "WAVE", "lane", q, src)
                                        : epi_call(io, "g", "wave", "lane", q, src)) + ";\n"
               "            __syncthreads();\n"
               "        }\n";
    }
    std::string loop_text(const std::string& run, const std::string& cur, const std::string& io) const {
        // The launch's first group is this workgroup's own (g = blockIdx.x), run speculatively: its
        // claim's compare-and-swap is issued here and its result read only after the group's state
        // loads (run<0>), so the claim's round trip overlaps them; a lost claim (another workgroup
        // stole the group before this one started) discards the group -- no store, no epilogue, no
        // completion.  The cursor already points past it (world_body).
        return "    bool spec = persistent && spec_first, spec_ok = true, own = true;\n"
               "    if (spec && threadIdx.x == 0) spec_ok = grid_claim(claim, (int)blockIdx.x, (" + cur + ")->base);\n"
               "    for (;;) {\n"
               "        const int g = spec ? (int)blockIdx.x : grid_next(persistent, a.ctl, claim, a.mask, MSK, nwords, ngrp, " + cur + ", QL);\n"
               "        if (g < 0) break;\n" + block_stamp(4, "__builtin_amdgcn_s_memrealtime()") +
               "        if (persistent) {\n"
               "            for (int i = threadIdx.x; i < nfl; i += blockDim.x) FL[i] = 0u;\n"
               "            __syncthreads();\n"
               "        }\n"
               "        {\n"
               "            const int b = " + std::string(ng > 1 ? "(g * " + it(ng) + " + sub) * 64 + lane" : "g * 64 + lane") + ";\n"
               "            const bool valid = b < a.B;\n"
               "            const int bb = valid ? b : (a.B - 1);\n"
               "            // the state write-back (Args.wbd, wb_text): this pass's inputs, its backup\n"
               "            const bool wbx = persistent && a.wbd != 0;\n"
               "            const long long rbd = (wbx && (" + cur + ")->pass > 0) ? a.wbd : 0ll;\n"
               "            const bool bk = wbx && (" + cur + ")->pass == 0;\n" + run + "        }\n"
               "        spec = false;\n"
               "        if (!own) continue;\n" + epi_text(io) +
               "        if (persistent && grid_finish(g, FL, nfl, a.blk, a.mask, MSK, a.ctl, a.err, a.herr, nwords, ngrp, " + cur + ",\n"
               "                                      a.max_pass, RED, &QL[65], a.tm, t0s.rt, t0s.sc))\n"
               "            poison_outputs(a);\n" + block_stamp(5, "__builtin_amdgcn_s_memrealtime()") +
               "    }\n";
    }

    void generate() {
        std::string& o = src;
        o += "// generated by vmas_jit.hip for one world\n";
        if (relaxed) o += std::string(kRelaxedTag) + "\n#define VMAS_PHYS_RELAXED 1\n";
        // A/B knob: VMAS_JIT_TRIG=guard generates round 4's entity trig (a lane-divergent branch to
        // the library sin / cos beyond 16 rad) instead of the branch-free reduction (vmas_physics.hpp)
        if (relaxed && getenv("VMAS_JIT_TRIG") && std::string(getenv("VMAS_JIT_TRIG")) == "guard")
            o += "#define VMAS_TRIG_GUARD 1\n";
        o += std::string(kFlagsTag) + codegen_flags(relaxed) + "\n";
        if (prof_block >= 0) o += "#define VMAS_JIT_PROFILE_SLOTS 1\n";
        if (const char* mp = getenv("VMAS_JIT_TEST_PASSES"))  // (test knob: vmas_jit_ops.hpp grid_decide)
            o += "#define VMAS_GRID_MIN_PASSES " + it(std::max(1, atoi(mp))) + "\n";
        o += "#include \"vmas_jit_ops.hpp\"\n";
        if (has_epi()) o += "#include \"vmas_programs.hpp\"\n";
        o += "using namespace vmas;\n\n";
        o += "struct Args {\n    const float* ptr[" + it(std::max<size_t>(ptr_src.size(), 1)) +
             "];\n    float* out[" + it(n_out()) + "];\n    uint32_t* mask;\n    uint32_t* blk;\n    unsigned long long* prof;\n"
             "    uint32_t* ctl;\n    uint32_t* err;\n    uint32_t* herr;\n    unsigned long long* tm;\n" +
             std::string(global_rows ? "    float* rows;\n" : "") +
             std::string(has_epi() ? std::string("    const ") + epi_type() + "* epi;\n" : std::string()) +
             "    long long wbd;\n" +
             "    int str[" + it(std::max<size_t>(str_src.size(), 2)) + "];\n    int B, S;\n    float sdt;\n    int max_pass;\n"
             "    float prm[" + it(std::max<size_t>(prm_src.size(), 1)) + "];\n" +
             std::string(tail ? "    VmasTail tail;\n" : "") + "};\n"
             "static_assert(sizeof(Args) == " + it((long)arg_bytes()) + ", \"argument block layout\");\n\n";
        o += "__device__ __forceinline__ V2 ld2(const float* p, int s0, int s1, int b) {\n"
             "    return mk(p[(long)b * s0], p[(long)b * s0 + s1]);\n}\n\n";
        o += wb_helpers();
        o += "constexpr WorldK WK{" + fl(cfg.contact_margin) + ", " + fl(cfg.collision_force) + ", " +
             fl(cfg.joint_force) + ", " + fl(cfg.torque_constraint_force) + "};\n";
        // world gravity and semidims: whether they apply is structure, their values are arguments
        const std::string pw = it(prm_world);
        // (the values are copied from the kernel arguments into LDS in the prologue and read from
        // there where used: held in SGPRs for the whole launch they raised balance's SGPR
        // spills 193 -> 289 and the static VALU count by 11 %)
        o += "__shared__ float PRM[" + it(std::max<size_t>(prm_src.size(), 1)) + "];\n";
        if ((prm_mask >> 11) & 1u) {
            o += "#define GX PRM[" + pw + "]\n#define GY PRM[" + pw + " + 1]\n";
            o += "#define XS PRM[" + pw + " + 2]\n#define YS PRM[" + pw + " + 3]\n";
        } else {
            o += "constexpr float GX = " + fl(cfg.gravity_x) + ", GY = " + fl(cfg.gravity_y) + ";\n";
            o += "constexpr float XS = " + fl(cfg.x_semidim) + ", YS = " + fl(cfg.y_semidim) + ";\n";
        }
        o += "constexpr bool HAS_G = " + bl(cfg.has_world_gravity) + ";\n";
        o += "constexpr bool HAS_XS = " + bl(cfg.has_x_semidim) + ", HAS_YS = " + bl(cfg.has_y_semidim) + ";\n";
        for (int e = 0; e < E; ++e)
            if (dyn[e]) o += "constexpr VmasEntityDesc D" + it(e) + "c" + desc(e) + ";\n";
        o += "\ntemplate <int WAVE>\n__device__ __forceinline__ bool run(const Args& a, float* L, uint32_t* FL, "
             "uint32_t* DONE, const uint32_t* MSK, int lane, int b, int bb, bool valid, long long rbd, bool bk, bool wbk, "
             "bool spec, bool spec_ok, uint32_t* QL" + std::string(use_src() ? ", const VmasBalanceIO* prog" : "") +
             ");\n\n";
        if (use_src()) o += src_fns();
        for (int w = 0; w < nw; ++w) wave_body(o, w);
        // waves per SIMD the register budget must allow: 2 workgroups per CU (4) or 1 (2)
        const int waves_per_eu = (lds_budget <= kLdsTwoPerCu ? 2 : 1) * nw * ng / 4;
        // NaN over every output field of the step (one workgroup; only after a fixed point that
        // did not converge within max_pass passes): the bad step is visible in its own results
        {
            const int n_lin = cfg.n_out_lin, n_rot = cfg.n_out_rot, n_f = cfg.n_out_force, n_t = cfg.n_out_torque;
            const int per_env[6] = {2 * n_lin, 2 * n_lin, n_rot, n_rot, 2 * n_f, n_t};
            o += "__device__ __forceinline__ void poison_outputs(const Args& a) {\n"
                 "    const float nan = __builtin_nanf(\"\");\n";
            for (int k = 0; k < 6; ++k)
                if (per_env[k] > 0)
                    o += "    for (size_t i = threadIdx.x; i < (size_t)" + it(per_env[k]) +
                         " * a.B; i += blockDim.x) a.out[" + it(k) + "][i] = nan;\n";
            o += "}\n\n";
        }
        // wave w's group loop (loop_per_wave): its copy of the persistent loop around run<w>
        if (loop_per_wave) {
            o += "template <int WAVE>\n__device__ __forceinline__ void group_loop(const Args& a, float* L, uint32_t* FL, uint32_t* DONE, "
                 "uint32_t* MSK, uint32_t* QL, uint32_t* RED, float* EQ, GridCursor* CURP, uint32_t* claim, TimerStart t0s, "
                 "bool persistent, bool spec_first, int nfl, int nwords, int ngrp, int lane, int wave" +
                 std::string(ng > 1 ? ", int sub" : "") +
                 std::string(has_epi() ? std::string(", const ") + epi_type() + "* PROG_IOP" : std::string()) + ") {\n    (void)EQ;\n";
            if (ng > 1)  // (this wave's group: its rows and split-pair counters)
                o += "    float* const Ls = L + sub * " + it((long)std::max(n_rows, 1) * 64) + ";\n"
                     "    uint32_t* const DONEs = DONE + sub * " + it(n_split) + ";\n    (void)Ls;\n";
            o += loop_text(ng > 1 ? "            own = run<WAVE>(a, Ls, FL, DONEs, MSK, lane, b, bb, valid, rbd, bk, wbx, spec, spec_ok, QL" + std::string(use_src() ? ", a.epi ? PROG_IOP : nullptr" : "") + ");\n"
                                  : "            own = run<WAVE>(a, L, FL, DONE, MSK, lane, b, bb, valid, rbd, bk, wbx, spec, spec_ok, QL" + std::string(use_src() ? ", a.epi ? PROG_IOP : nullptr" : "") + ");\n",
                           "CURP", "*PROG_IOP");
            o += "}\n\n";
        }
        o += "__device__ __forceinline__ void world_body(const Args& a) {\n";
        if (global_rows)  // (this workgroup's slab: the same [row][lane] layout as the LDS rows)
            o += "    float* L = a.rows + (size_t)blockIdx.x * " + it((long)std::max(n_rows, 1) * 64) + ";\n";
        else
            o += "    __shared__ __attribute__((aligned(16))) float L[" + it(std::max(n_rows, 1) * 64 * ng) + "];\n";
        o += "    __shared__ uint32_t FL[" + it(nfl) + "];\n";
        if (has_epi() && !epi_q_in_rows()) o += "    __shared__ float EQ[" + it((long)kEpiQRows * 64 * ng) + "];\n";
        if (has_epi() && epi_lds) o += std::string("    __shared__ __attribute__((aligned(16))) ") + epi_type() + " PROG_IO;\n";
        o += "    __shared__ uint32_t DONE[" + it(std::max(n_split * ng, 1)) + "];\n";
        // LDS of the device-side fixed point: the row buffer when it is large enough (it is
        // idle between groups), else its own array; QL: steal list + broadcast word
        const int red_words = nfl + 2;
        o += "    __shared__ uint32_t MSK[" + it(std::max(nfl / 2, 1)) + "];\n";
        o += "    __shared__ uint32_t QL[66];\n";
        if (!global_rows && (long)std::max(n_rows, 1) * 64 * ng >= red_words)
            o += "    uint32_t* RED = reinterpret_cast<uint32_t*>(L);\n";
        else
            o += "    __shared__ uint32_t RED[" + it(red_words) + "];\n";
        o += "    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;\n";
        o += "    const int nfl = 2 * a.S * " + it(W) + ", nwords = a.S * " + it(W) + ", ngrp = " +
             (ng > 1 ? "(a.B + " + it(64 * ng - 1) + ") / " + it(64 * ng) : std::string("(a.B + 63) >> 6")) + ";\n"
             "    for (int i = threadIdx.x; i < " + it(n_split * ng) + "; i += blockDim.x) DONE[i] = 0u;\n";
        // Host-driven loop (a.ctl null): one pass per launch, each workgroup strides over the
        // 64-env groups and ORs their activity words into its own blk row (read by
        // k_jit_flags_reduce).  Persistent launch (a.ctl set): the broadphase fixed point on the
        // device; groups are claimed per pass (own groups, then steals), each completion stores
        // the group's row, the last completion of a pass decides, waits are only for claimed
        // work (vmas_jit_ops.hpp grid_*).  One call site of the group body (a second one would
        // duplicate the per-wave code).  DONE is back to zero at the end of every substep's pair
        // phase, so it carries over between groups.
        o += "    const bool persistent = a.ctl != nullptr;\n"
             "    uint32_t* claim = a.mask + " + it(vmas::grid_claim_offset((long)cfg.max_substeps * W)) + ";\n"
             "    const TimerStart t0s = device_timer_start(persistent ? a.tm : nullptr, true);\n"
             "    __shared__ GridCursor CUR;\n"
             "    const bool spec_first = " + std::string(spec_claim ? "persistent && (int)blockIdx.x < ngrp" : "false") +
             ";  // (the speculative first group: loop_text)\n"
             "    if (threadIdx.x == 0)\n"
             "        CUR = GridCursor{0, (int)blockIdx.x + (spec_first ? (int)gridDim.x : 0), 0, 0, 0, persistent ? ld64(&a.ctl[kGridEpoch]) : 0ull};\n"
             "    for (int i = threadIdx.x; i < nfl; i += blockDim.x) FL[i] = 0u;\n"
             "    for (int i = threadIdx.x; i < nwords; i += blockDim.x) MSK[i] = ~ld_agent(&a.mask[i]);\n" +
             std::string(has_epi() && epi_lds ?
                 "    if (a.epi)\n"
                 "        for (int i = threadIdx.x; i < (int)(sizeof(PROG_IO) / 8); i += blockDim.x)\n"
                 "            reinterpret_cast<unsigned long long*>(&PROG_IO)[i] = reinterpret_cast<const unsigned long long*>(a.epi)[i];\n"
                 : "") +
             prm_copy() +
             "    __syncthreads();\n" +
             block_stamp(0, "__builtin_amdgcn_s_memrealtime()") + block_stamp(1, "__builtin_amdgcn_s_getreg(63492)") +
             block_stamp(2, "__builtin_amdgcn_s_getreg(30740)") +
             (prof_block >= 0 ? "    if (lane == 0 && blockIdx.x < " + it(kProfBlocks) + ") a.prof[" +
                                    it((long)(cfg.max_substeps * 4 + 2) * kMaxNW) + " + blockIdx.x * " + it(kProfRec) +
                                    " + 8 + wave] = __builtin_amdgcn_s_getreg(63492);\n"
                              : "") +
             (prof_block >= 0 ? "    if (threadIdx.x == 0) vmas_prof_blk = a.prof + " + it((long)(cfg.max_substeps * 4 + 2) * kMaxNW) + ";\n" : "") +
             "";
        // the group loop (loop_text): one copy per wave (loop_per_wave), or one around a switch
        if (loop_per_wave) {
            // (ng > 1: one call site per wave body, the group index a run-time value)
            std::string sw = ng > 1 ? "    switch (wave % " + it(nw) + ") {\n" : "    switch (wave) {\n";
            for (int w = 0; w < nw; ++w)
                sw += "        case " + it(w) + ": group_loop<" + it(w) + ">(a, L, FL, DONE, MSK, QL, RED, " +
                      std::string(has_epi() && !epi_q_in_rows() ? "EQ" : "nullptr") +
                      ", &CUR, claim, t0s, persistent, spec_first, nfl, nwords, ngrp, lane, wave" +
                      std::string(ng > 1 ? ", wave / " + it(nw) : "") +
                      std::string(has_epi() ? (epi_lds ? ", &PROG_IO" : ", a.epi") : "") + "); break;\n";
            o += sw + "        default: break;\n    }\n";
        } else {
            std::string sw = "            switch (wave) {\n";
            for (int w = 0; w < nw; ++w)
                sw += "                case " + it(w) + ": run<" + it(w) + ">(a, L, FL, DONE, MSK, lane, b, bb, valid, rbd, bk, wbx, spec, spec_ok, QL" + std::string(use_src() ? (epi_lds ? ", a.epi ? &PROG_IO : nullptr" : ", a.epi") : "") + "); break;\n";
            o += loop_text(sw + "                default: break;\n            }\n", "&CUR", epi_lds ? "PROG_IO" : "*a.epi");
        }
        o += block_stamp(3, "__builtin_amdgcn_s_memrealtime()") +
             std::string(tail ? "    // the replay's post-replay work (vmas_tail.hpp): every group's final pass is decided\n"
                                "    if (persistent && a.tail.n_items > 0) vmas_tail::run(a.tail);\n" : "") +
             "    if (!persistent) {\n"
             "        if (!a.blk) return;\n"
             "        __syncthreads();\n"
             "        for (int i = threadIdx.x; i < nfl; i += blockDim.x) st_agent(&a.blk[(size_t)blockIdx.x * nfl + i], FL[i]);\n"
             "        return;\n"
             "    }\n"
             "}\n\n";
        const std::string bounds = "__launch_bounds__(" + it(nw * ng * 64) + ", " + it(waves_per_eu) + ")";
        o += "extern \"C\" __global__ void " + bounds + " k_world(Args a) {\n    world_body(a);\n}\n";
        if (has_epi())  // the eager step's launch of the same program (vmas_jit_program_outputs)
            o += "\nextern \"C\" __global__ void __launch_bounds__(" + it(nw * 64) + ") k_program_jit(" + epi_type() + " io_arg) {\n"
                 "    VMAS_PROGRAM_ARGS(" + epi_type() + ", io_arg);\n"
                 "    __shared__ float Q[" + it((long)kEpiQRows * 64) + "];\n"
                 "    " + epi_call("io", "blockIdx.x", "(int)(threadIdx.x >> 6)", "(int)(threadIdx.x & 63)", "Q") + ";\n}\n";
    }
};

// Code-generation A/B knobs (environment): VMAS_JIT_PRIO, VMAS_JIT_PRELOAD, VMAS_JIT_PAIR_PRELOAD,
// VMAS_JIT_LOOP_PER_WAVE, VMAS_JIT_EPI_LDS.
void codegen_knobs(Gen& g) {
    if (const char* pr = getenv("VMAS_JIT_PRIO")) g.prio_mode = atoi(pr);
    if (const char* pl = getenv("VMAS_JIT_PRELOAD")) g.entity_preload = atoi(pl) != 0;
    if (const char* pp = getenv("VMAS_JIT_PAIR_PRELOAD")) g.pair_preload = atoi(pp) != 0;
    if (const char* lw = getenv("VMAS_JIT_LOOP_PER_WAVE")) g.loop_per_wave = atoi(lw) != 0 || g.ng > 1;
    if (const char* el = getenv("VMAS_JIT_EPI_LDS")) g.epi_lds = atoi(el) != 0;
    if (const char* sc = getenv("VMAS_JIT_SPEC_CLAIM")) g.spec_claim = atoi(sc) != 0;
}

// Plan a world: box pairs split with two workgroups per CU, else unsplit, else unsplit with the
// whole LDS (one workgroup per CU).  VMAS_JIT_SPLIT=0 disables splitting.
std::unique_ptr<Gen> make_plan(const VmasWorldConfig& cfg, const std::vector<VmasEntityDesc>& ed,
                               const std::vector<VmasPairDesc>& pd, const std::vector<VmasJointDesc>& jd,
                               std::string* why, int force_nw = 0) {
    const char* sp = getenv("VMAS_JIT_SPLIT");
    const bool allow_split = !(sp && sp[0] == '0');
    const struct {
        bool split;
        long budget;
        bool global_rows;
    } tries[] = {{true, kLdsTwoPerCu, false}, {false, kLdsTwoPerCu, false}, {false, kLdsOnePerCu, false},
                 {false, kLdsOnePerCu, true}};
    // VMAS_JIT_NG=2 (A/B): two 64-env groups per workgroup in lockstep (Gen::ng), LDS rows of both,
    // one workgroup per CU; not for worlds whose rows live in global memory
    const char* ngs = getenv("VMAS_JIT_NG");
    const int ng_want = ngs && atoi(ngs) == 2 ? 2 : 1;
    for (int ng = ng_want; ng >= 1; --ng)  // (a world too big for two groups' rows plans with one)
    for (const auto& t : tries) {
        if (t.split && !allow_split) continue;
        if (ng > 1 && t.global_rows) continue;
        std::unique_ptr<Gen> g(new Gen(cfg, ed, pd, jd));
        g->ng = ng;
        if (const char* es = getenv("VMAS_JIT_EPI_SRC")) g->epi_src = atoi(es) != 0;  // (read before plan: rows)
        if (const char* pm = getenv("VMAS_JIT_PRM_MASK")) g->prm_mask = (unsigned)strtoul(pm, nullptr, 0) & 0xFFFu;
        if ((size_t)cfg.max_substeps * g->W > 1024) {
            *why = "too many substeps x pairs";
            return nullptr;
        }
        g->split_boxes = t.split;
        g->lds_budget = ng > 1 ? kLdsOnePerCu : t.budget;  // (ng > 1: one workgroup per CU)
        g->global_rows = t.global_rows;
        // 16 waves per workgroup once there are enough pair tasks to spread (measured: flocking
        // 81 pairs 72 -> 59 us, discovery 19.2 -> 16.3 us; balance's 24 tasks 67.7 -> 69.7 us)
        int n_tasks = 0;
        for (const auto& q : pd)
            n_tasks += (t.split && (q.cls == VMAS_PAIR_BL || q.cls == VMAS_PAIR_BB)) ? Gen::parts(q.cls) + 1 : 1;
        g->nw = n_tasks >= 32 ? 16 : kNW;
        if (const char* nws = getenv("VMAS_JIT_WAVES")) g->nw = atoi(nws) == 16 ? 16 : kNW;
        if (force_nw) g->nw = force_nw;
        if (g->ng > 1) g->nw = kNW;  // (8 waves per group: 16 per workgroup)
        why->clear();
        if (g->plan(why)) return g;
    }
    return nullptr;
}

// OR the per-block activity words, decide whether the mask was a fixed point, update it if not
// (same scheme as vmas_world_step's reduction).  blk: [nblk][2][S][W]; one workgroup.
__global__ void __launch_bounds__(1024) k_jit_flags_reduce(const uint32_t* blk, int nblk, int S, int W,
                                                           uint32_t* mask, uint32_t* viol_out) {
    __shared__ uint32_t R[1024], Z[1024];
    __shared__ uint32_t viol;
    const int nwords = S * W;
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
        R[w] = 0u;
        Z[w] = 0u;
    }
    if (threadIdx.x == 0) viol = 0u;
    __syncthreads();
    const int groups = max(1, (int)blockDim.x / nwords);
    if ((int)threadIdx.x < groups * nwords) {
        const int w = threadIdx.x % nwords, g0 = threadIdx.x / nwords;
        uint32_t r = 0u, z = 0u;
        for (int i = g0; i < nblk; i += groups) {
            r |= blk[(size_t)i * 2 * nwords + w];
            z |= blk[(size_t)i * 2 * nwords + nwords + w];
        }
        if (r) atomicOr(&R[w], r);
        if (z) atomicOr(&Z[w], z);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
        const uint32_t m = ~mask[w];  // stored inverted (zero memset = all pairs active)
        if ((m & ~R[w] & Z[w]) | (~m & R[w])) atomicOr(&viol, 1u);
    }
    __syncthreads();
    if (viol)
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) mask[w] = ~R[w];
    if (threadIdx.x == 0) *viol_out = viol;
}

// Math mode of a world's kernel: relaxed (the default) for worlds without joints, exact with
// joints or with VMAS_JIT_MATH=exact (then bit-identical to k_step and the host backend).
bool relaxed_math(const VmasWorldConfig& cfg) {
    const char* m = getenv("VMAS_JIT_MATH");
    return !(m && std::string(m) == "exact") && cfg.n_joints == 0;
}

// hipRTC compile with an in-process cache (identical world structures share one code object;
// parameter values are kernel arguments, so a world whose masses / drags / limits change keeps
// its entry).  Bounded: the kCodeCacheMax most recently used code objects (VMAS_JIT_CACHE).
std::mutex g_cache_mu;
std::unordered_map<std::string, std::pair<std::vector<char>, uint64_t>> g_code_cache;  // src -> (code, last use)
uint64_t g_cache_tick = 0;
constexpr size_t kCodeCacheMax = 32;
size_t code_cache_max() {
    const char* c = getenv("VMAS_JIT_CACHE");
    return c ? (size_t)std::max(1, atoi(c)) : kCodeCacheMax;
}

std::string module_dir() {
    Dl_info info{};
    if (dladdr((const void*)&jfail, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        const size_t k = p.rfind('/');
        return k == std::string::npos ? std::string(".") : p.substr(0, k);
    }
    return ".";
}

int64_t g_jit_compiles = 0;  // hipRTC compiles so far (vmas_jit_stats)

int32_t compile(const std::string& src, std::vector<char>* code) {
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        auto f = g_code_cache.find(src);
        if (f != g_code_cache.end()) {
            *code = f->second.first;
            f->second.second = ++g_cache_tick;
            return VMAS_OK;
        }
    }
    const std::string dir = module_dir();
    const std::string inc1 = "-I" + dir + "/csrc", inc2 = "-I" + dir + "/../include";
    std::vector<const char*> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                                     inc1.c_str(), inc2.c_str()};
    // the code-generation options the generator wrote into the source (kFlagsTag line)
    std::vector<std::string> extra;
    const size_t at = src.find(kFlagsTag);
    if (at != std::string::npos) {
        const size_t b = at + strlen(kFlagsTag), e = src.find('\n', b);
        const std::string line = src.substr(b, e == std::string::npos ? std::string::npos : e - b);
        std::string t;
        for (char c : line + " ") {
            if (c == ' ') {
                if (!t.empty()) extra.push_back(t);
                t.clear();
            } else {
                t += c;
            }
        }
    }
    for (const std::string& x : extra) opts.push_back(x.c_str());
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "vmas_world.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return jfail(VMAS_E_HIP, "hiprtcCreateProgram failed");
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        return jfail(VMAS_E_HIP, "hipRTC compile failed: %.900s", log.c_str());
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code->resize(n);
    hiprtcGetCode(prog, code->data());
    hiprtcDestroyProgram(&prog);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    ++g_jit_compiles;
    while (!g_code_cache.empty() && g_code_cache.size() >= code_cache_max()) {  // evict the least recently used
        auto lru = g_code_cache.begin();
        for (auto it2 = g_code_cache.begin(); it2 != g_code_cache.end(); ++it2)
            if (it2->second.second < lru->second.second) lru = it2;
        g_code_cache.erase(lru);
    }
    g_code_cache[src] = {*code, ++g_cache_tick};
    return VMAS_OK;
}

}  // namespace

// The kernels of the loaded world modules (k_world, k_program_jit): a kernel node of a captured
// step graph whose function is one of these is a module launch, and a k_world node followed by its
// module's k_program_jit node can run as one launch (vmas_graph_chain_build, vmas_kernels.hip).
namespace vmas {
namespace {
std::mutex g_fn_mu;
std::unordered_map<const void*, JitFnInfo> g_live_fns;
}  // namespace
void fn_register(hipFunction_t f, const JitFnInfo& info) {
    std::lock_guard<std::mutex> lk(g_fn_mu);
    g_live_fns[(const void*)f] = info;
}
void fn_unregister(hipFunction_t f) {
    if (!f) return;
    std::lock_guard<std::mutex> lk(g_fn_mu);
    g_live_fns.erase((const void*)f);
}
bool jit_fn_info(const void* f, JitFnInfo* out) {
    std::lock_guard<std::mutex> lk(g_fn_mu);
    auto it = g_live_fns.find(f);
    if (it == g_live_fns.end()) return false;
    if (out) *out = it->second;
    return true;
}
}  // namespace vmas

struct VmasJitWorld {
    VmasWorldConfig cfg{};
    std::vector<VmasEntityDesc> ed;
    std::vector<VmasPairDesc> pd;
    std::vector<VmasJointDesc> jd;
    std::string src;
    std::vector<std::pair<int, int>> ptr_src, str_src, prm_src;
    unsigned prm_mask = kPrmMaskDefault;  // value fields passed as arguments (the others are folded in)
    size_t arg_bytes = 0;
    int W = 1, nblk = 0, nw = kNW;
    int ng = 1;  // 64-env groups per work item (k_world runs nw * ng waves per workgroup)
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;  // k_world
    hipFunction_t fn_prog = nullptr;  // k_program_jit (cfg.epilogue: the scenario program's own kernel)
    size_t epi_offset = 0;           // byte offset of Args.epi (epilogue modules)
    uint32_t *d_mask = nullptr, *d_blk = nullptr, *d_viol = nullptr, *h_viol = nullptr;
    // persistent launches: d_ctl = [kGridCtlWords control words | inverted mask words | claim word
    // per group (u64, kClaimStride apart, from grid_claim_offset)], zeroed at create and never
    // reset (global pass numbers, vmas_jit_ops.hpp);
    // d_err: sticky error bits; h_err: mapped host word the kernel stores them into (dh_err: its
    // device address)
    uint32_t *d_ctl = nullptr, *d_err = nullptr, *h_err = nullptr, *dh_err = nullptr;
    int grid = 0;          // workgroups of a persistent launch (0: host-driven loop, one pass per launch)
    int max_passes = 0;    // fixed-point passes per step (0: substeps + 2, the bound; VMAS_JIT_MAX_PASSES)
    hipStream_t last_stream = nullptr;
    int last_passes = 0;   // passes of the last host-driven step (persistent: read on demand)
    bool last_persistent = false;
    unsigned long long* d_prof = nullptr;  // phase timestamps of one workgroup (VMAS_JIT_PROFILE)
    size_t n_prof = 0;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending, ev_free;
    double timed_ms = 0.0;
    long timed_launches = 0;
    // device timer (timing on, persistent launches): [0] workgroup 0's start, [2] accumulated
    // ticks, [4] launches -- s_memrealtime, kept by the kernel itself so that launches replayed
    // from a HIP graph are timed too (HIP records no events inside a graph; vmas_jit_ops.hpp)
    unsigned long long* d_tm = nullptr;
    int wall_khz = 0;
    // rows in global memory (Gen::global_rows): one slab of n_rows x 64 floats per workgroup
    bool global_rows = false;
    float* d_rows = nullptr;
};

extern "C" {

const char* vmas_jit_last_error(void) { return g_jit_err.c_str(); }

int32_t vmas_jit_stats(int64_t* compiles, int64_t* cached) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    if (compiles) *compiles = g_jit_compiles;
    if (cached) *cached = (int64_t)g_code_cache.size();
    return VMAS_OK;
}

int32_t vmas_jit_world_destroy(VmasJitWorld* W) {
    if (!W) return VMAS_OK;
    if (W->cfg.device >= 0) {
        (void)hipSetDevice(W->cfg.device);
        vmas::chain_free_drain();
        vmas::fn_unregister(W->fn);
        vmas::fn_unregister(W->fn_prog);
        if (W->mod) (void)hipModuleUnload(W->mod);
        if (W->d_mask) (void)hipFree(W->d_mask);
        if (W->d_blk) (void)hipFree(W->d_blk);
        if (W->d_viol) (void)hipFree(W->d_viol);
        if (W->h_viol) (void)hipHostFree(W->h_viol);
        if (W->d_prof) (void)hipFree(W->d_prof);
        if (W->d_rows) (void)hipFree(W->d_rows);
        if (W->d_ctl) (void)hipFree(W->d_ctl);
        if (W->d_err) (void)hipFree(W->d_err);
        if (W->h_err) (void)hipHostFree(W->h_err);
        for (auto& ev : W->ev_pending) { (void)hipEventDestroy(ev.first); (void)hipEventDestroy(ev.second); }
        for (auto& ev : W->ev_free) { (void)hipEventDestroy(ev.first); (void)hipEventDestroy(ev.second); }
        if (W->d_tm) (void)hipFree(W->d_tm);
    }
    delete W;
    return VMAS_OK;
}

int32_t vmas_jit_world_create(const VmasWorldConfig* cfg, const VmasEntityDesc* entities, const VmasPairDesc* pairs,
                              const VmasJointDesc* joints, VmasJitWorld** out_world) {
    if (!cfg || !out_world) return jfail(VMAS_E_INVALID, "null argument");
    if (cfg->device < 0) return jfail(VMAS_E_INVALID, "the specialised step is a GPU path (device >= 0)");
    if (cfg->batch <= 0 || cfg->n_entities <= 0 || cfg->n_pairs < 0 || cfg->max_substeps <= 0)
        return jfail(VMAS_E_INVALID, "bad world config");
    auto* W = new VmasJitWorld();
    W->cfg = *cfg;
    W->ed.assign(entities, entities + cfg->n_entities);
    W->pd.assign(pairs, pairs + cfg->n_pairs);
    if (cfg->n_joints) W->jd.assign(joints, joints + cfg->n_joints);
    for (const auto& q : W->pd)
        if (q.ea < 0 || q.ea >= cfg->n_entities || q.eb < 0 || q.eb >= cfg->n_entities || q.cls < 0 || q.cls > 6 ||
            (q.cls == VMAS_PAIR_JOINT && (q.joint < 0 || q.joint >= cfg->n_joints))) {
            delete W;
            return jfail(VMAS_E_INVALID, "bad pair table");
        }
    auto cleanup = [&](int32_t rc) {
        vmas_jit_world_destroy(W);
        return rc;
    };
    JHIP(hipSetDevice(cfg->device));
    std::string why;
    std::unique_ptr<Gen> gp;
    // A 16-wave kernel whose register budget (8 waves/SIMD -> 64 VGPRs) makes it spill is
    // regenerated with 8 waves (measured: pollock 154 spilled VGPRs at 16 waves).
    for (int force_nw : {0, kNW}) {
        gp = make_plan(W->cfg, W->ed, W->pd, W->jd, &why, force_nw);
        if (!gp) {
            delete W;
            return jfail(VMAS_E_INVALID, "world not specialised: %s", why.c_str());
        }
        Gen& g = *gp;
        if (const char* pb = getenv("VMAS_JIT_PROFILE")) g.prof_block = std::max(0, atoi(pb));
        codegen_knobs(g);
        g.relaxed = relaxed_math(W->cfg);
        g.generate();
        std::vector<char> code;
        if (int32_t rc = compile(g.src, &code)) return cleanup(rc);
        if (W->mod) {
            W->fn = nullptr;
            (void)hipModuleUnload(W->mod);
            W->mod = nullptr;
        }
        if (hipModuleLoadData(&W->mod, code.data()) != hipSuccess)
            return cleanup(jfail(VMAS_E_HIP, "hipModuleLoadData"));
        if (hipModuleGetFunction(&W->fn, W->mod, "k_world") != hipSuccess)
            return cleanup(jfail(VMAS_E_HIP, "hipModuleGetFunction"));
        int scratch = 0;
        (void)hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, W->fn);
        if (scratch == 0 || g.nw == kNW || g.ng > 1) break;
    }
    Gen& g = *gp;
    W->src = g.src;
    W->ptr_src = g.ptr_src;
    W->str_src = g.str_src;
    W->prm_src = g.prm_src;
    W->prm_mask = g.prm_mask;
    W->arg_bytes = g.arg_bytes();
    W->W = g.W;
    W->nw = g.nw;
    W->ng = g.ng;
    W->nblk = (cfg->batch + 64 * g.ng - 1) / (64 * g.ng);
    if (g.has_epi()) {
        if (hipModuleGetFunction(&W->fn_prog, W->mod, "k_program_jit") != hipSuccess)
            return cleanup(jfail(VMAS_E_HIP, "hipModuleGetFunction(k_program_jit)"));
        W->epi_offset = g.epi_offset();
    }
    {
        vmas::JitFnInfo info{};
        info.kind = vmas::kJitFnWorld;
        info.world = W;
        info.world_fn = W->fn;
        info.arg_bytes = W->arg_bytes;
        info.epi_offset = W->fn_prog ? (long)W->epi_offset : -1L;
        info.wbd_offset = (long)g.wbd_offset();
        info.tail_offset = g.tail ? (long)g.tail_offset() : -1L;
        info.batch = cfg->batch;
        info.epilogue = g.has_epi() ? cfg->epilogue : VMAS_EPILOGUE_NONE;
        info.io_bytes = cfg->epilogue == VMAS_EPILOGUE_BALANCE ? sizeof(VmasBalanceIO)
                        : cfg->epilogue == VMAS_EPILOGUE_TRANSPORT ? sizeof(VmasTransportIO) : 0;
        vmas::fn_register(W->fn, info);
        if (W->fn_prog) {
            info.kind = vmas::kJitFnProgram;
            vmas::fn_register(W->fn_prog, info);
        }
    }
    const size_t nwords = (size_t)cfg->max_substeps * W->W;
    if (hipMalloc((void**)&W->d_mask, nwords * 4) != hipSuccess ||
        hipMalloc((void**)&W->d_blk, (size_t)W->nblk * 2 * nwords * 4) != hipSuccess ||
        hipMalloc((void**)&W->d_viol, 4) != hipSuccess ||
        hipHostMalloc((void**)&W->h_viol, 4, hipHostMallocDefault) != hipSuccess)
        return cleanup(jfail(VMAS_E_NOMEM, "hipMalloc broadphase scratch"));
    const size_t ctl_words = vmas::kGridCtlWords + (size_t)vmas::grid_claim_offset((long)nwords) +
                             (size_t)W->nblk * vmas::kClaimStride;
    if (hipMalloc((void**)&W->d_ctl, ctl_words * 4) != hipSuccess || hipMalloc((void**)&W->d_err, 4) != hipSuccess ||
        hipHostMalloc((void**)&W->h_err, 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&W->dh_err, W->h_err, 0) != hipSuccess ||
        hipMemset(W->d_err, 0, 4) != hipSuccess ||
        hipMemset(W->d_ctl, 0, ctl_words * 4) != hipSuccess)
        return cleanup(jfail(VMAS_E_NOMEM, "hipMalloc fixed-point control words"));
    *W->h_err = 0u;
    if (hipMalloc((void**)&W->d_tm, 8 * 8) != hipSuccess || hipMemset(W->d_tm, 0, 8 * 8) != hipSuccess ||
        hipDeviceGetAttribute(&W->wall_khz, hipDeviceAttributeWallClockRate, cfg->device) != hipSuccess ||
        W->wall_khz <= 0)
        return cleanup(jfail(VMAS_E_HIP, "device timer (hipMalloc / wall clock rate)"));
    // Persistent grid (vmas_jit_ops.hpp grid_*): as many workgroups as can be resident at once
    // (occupancy x CUs), capped by the number of 64-env groups; each claims its own groups, then
    // steals.  Waits are only for claimed work, so residency is a performance choice, not a
    // requirement.  VMAS_JIT_GRID=host keeps the host-driven loop (one launch + reduction + host
    // read per pass); VMAS_JIT_MAX_PASSES=<n> caps the passes per step (default substeps + 2, the
    // fixed point's bound; at most kGridMaxPasses).
    {
        const char* gm = getenv("VMAS_JIT_GRID");
        const std::string mode = gm ? gm : "persistent";
        int per_cu = 0, cus = 0;
        if (mode != "host" &&
            hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, W->fn, W->nw * W->ng * 64, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess &&
            per_cu > 0 && cus > 0) {
            W->grid = std::min(W->nblk, per_cu * cus);
            if (const char* cap = getenv("VMAS_JIT_GRID_CAP")) W->grid = std::max(1, std::min(W->grid, atoi(cap)));
            if (const char* r = getenv("VMAS_JIT_MAX_PASSES")) W->max_passes = std::max(1, atoi(r));
        }
    }
    W->global_rows = g.global_rows;
    if (g.global_rows) {  // (a slab per workgroup of the largest grid: the host-driven loop's nblk)
        const size_t slab = (size_t)std::max(W->nblk, W->grid) * (size_t)std::max(g.n_rows, 1) * 64 * 4;
        if (hipMalloc((void**)&W->d_rows, slab) != hipSuccess) return cleanup(jfail(VMAS_E_NOMEM, "hipMalloc row slabs"));
    }
    if (g.prof_block >= 0) {
        W->n_prof = ((size_t)cfg->max_substeps * 4 + 2) * kMaxNW + (size_t)kProfBlocks * kProfRec;
        if (hipMalloc((void**)&W->d_prof, W->n_prof * 8) != hipSuccess ||
            hipMemset(W->d_prof, 0, W->n_prof * 8) != hipSuccess)
            return cleanup(jfail(VMAS_E_NOMEM, "hipMalloc profile buffer"));
    }
    *out_world = W;
    return VMAS_OK;
}

// Phase timestamps of the profiled workgroup from the last launch (VMAS_JIT_PROFILE=<block> at
// create): [max_substeps*4 + 2][NW] s_memtime values (see Gen::stamp); returns the count.
int32_t vmas_jit_world_profile(VmasJitWorld* W, uint64_t* out, int64_t cap) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    if (!W->d_prof) return 0;
    JHIP(hipSetDevice(W->cfg.device));
    JHIP(hipDeviceSynchronize());
    const size_t n = std::min<size_t>(W->n_prof, cap > 0 ? (size_t)cap : 0);
    if (out && n) JHIP(hipMemcpy(out, W->d_prof, n * 8, hipMemcpyDeviceToHost));
    return (int32_t)W->n_prof;
}

// Generate and compile (hipRTC, gfx950) the specialised kernel of a world without a device:
// returns the source length (copied into buf when given) or a negative VMAS_E_* code.
int32_t vmas_jit_compile_check(const VmasWorldConfig* cfg, const VmasEntityDesc* entities, const VmasPairDesc* pairs,
                               const VmasJointDesc* joints, char* buf, int64_t cap) {
    if (!cfg || cfg->n_entities <= 0 || cfg->max_substeps <= 0) return jfail(VMAS_E_INVALID, "bad world config");
    std::vector<VmasEntityDesc> ed(entities, entities + cfg->n_entities);
    std::vector<VmasPairDesc> pd(pairs, pairs + cfg->n_pairs);
    std::vector<VmasJointDesc> jd;
    if (cfg->n_joints) jd.assign(joints, joints + cfg->n_joints);
    std::string why;
    std::unique_ptr<Gen> gp = make_plan(*cfg, ed, pd, jd, &why);
    if (!gp) return jfail(VMAS_E_INVALID, "world not specialised: %s", why.c_str());
    Gen& g = *gp;
    codegen_knobs(g);
    g.relaxed = relaxed_math(*cfg);
    g.generate();
    std::vector<char> code;
    if (int32_t rc = compile(g.src, &code)) return rc;
    if (buf && cap > 0) {
        const size_t k = std::min<size_t>(g.src.size(), (size_t)cap - 1);
        memcpy(buf, g.src.data(), k);
        buf[k] = '\0';
    }
    return (int32_t)g.src.size();
}

int32_t vmas_jit_world_source(const VmasJitWorld* W, char* buf, int64_t cap) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    const int64_t n = (int64_t)W->src.size();
    if (buf && cap > 0) {
        const int64_t k = std::min(n, cap - 1);
        memcpy(buf, W->src.data(), (size_t)k);
        buf[k] = '\0';
    }
    return (int32_t)std::min<int64_t>(n, INT32_MAX);
}

int32_t vmas_jit_world_step(VmasJitWorld* W, const VmasStepIO* io, void* stream_, int32_t* iterations) {
    if (!W || !io) return jfail(VMAS_E_INVALID, "null argument");
    const VmasWorldConfig& cfg = W->cfg;
    if (io->substeps <= 0 || io->substeps > cfg.max_substeps)
        return jfail(VMAS_E_INVALID, "substeps %d outside [1, %d]", io->substeps, cfg.max_substeps);
    int cur = -1;
    JHIP(hipGetDevice(&cur));
    if (cur != cfg.device) JHIP(hipSetDevice(cfg.device));
    hipStream_t stream = (hipStream_t)stream_;
    // kernel argument block (layout of the generated `struct Args`)
    std::vector<char> buf(W->arg_bytes, 0);
    char* p = buf.data();
    auto put_ptr = [&](const void* v) {
        memcpy(p, &v, 8);
        p += 8;
    };
    auto put_i32 = [&](int32_t v) {
        memcpy(p, &v, 4);
        p += 4;
    };
    for (const auto& s : W->ptr_src) {
        const int i = s.second;
        const VmasEntityIO* e = io->entities + (s.first <= S_GRAV ? i : 0);
        switch (s.first) {
            case S_POS: put_ptr(e->pos); break;
            case S_VEL: put_ptr(e->vel); break;
            case S_ROT: put_ptr(e->rot); break;
            case S_ANG: put_ptr(e->ang_vel); break;
            case S_GRAV: put_ptr(e->gravity); break;
            case S_FORCE: put_ptr(io->agents[i].force); break;
            case S_TORQUE: put_ptr(io->agents[i].torque); break;
            default: put_ptr(io->joints ? io->joints[i].fixed_rotation : nullptr); break;
        }
    }
    if (W->ptr_src.empty()) put_ptr(nullptr);
    put_ptr(io->out_pos);
    put_ptr(io->out_vel);
    put_ptr(io->out_rot);
    put_ptr(io->out_ang_vel);
    put_ptr(io->out_force);
    put_ptr(io->out_torque);
    if (W->cfg.export_forces) {
        put_ptr(io->out_fdict);
        put_ptr(io->out_tdict);
    }
    const bool batch_bp = io->broadphase == VMAS_BROADPHASE_BATCH;
    const bool persistent = batch_bp && W->grid > 0;
    uint32_t* nmask = persistent ? W->d_ctl + vmas::kGridCtlWords : W->d_mask;
    put_ptr(nmask);
    put_ptr(batch_bp ? W->d_blk : nullptr);
    put_ptr(W->d_prof);
    put_ptr(persistent ? W->d_ctl : nullptr);
    put_ptr(W->d_err);
    put_ptr(W->dh_err);
    put_ptr(W->timing && persistent ? W->d_tm : nullptr);
    if (W->global_rows) put_ptr(W->d_rows);
    if (W->fn_prog) put_ptr(nullptr);  // Args.epi: no epilogue (the chain replay's fused launch sets it)
    put_ptr(nullptr);                  // Args.wbd: no state write-back (the chain's write-back variant sets it)
    for (const auto& s : W->str_src) {
        const int kind = s.first / 4, k = s.first % 4, i = s.second;
        int32_t v = 0;
        if (s.first >= 0) {
            const VmasEntityIO* e = io->entities + (kind <= S_GRAV ? i : 0);
            switch (kind) {
                case S_POS: v = k ? e->pos_s1 : e->pos_s0; break;
                case S_VEL: v = k ? e->vel_s1 : e->vel_s0; break;
                case S_ROT: v = e->rot_s0; break;
                case S_ANG: v = e->ang_s0; break;
                case S_GRAV: v = k ? e->grav_s1 : e->grav_s0; break;
                case S_FORCE: v = k ? io->agents[i].force_s1 : io->agents[i].force_s0; break;
                case S_TORQUE: v = io->agents[i].torque_s0; break;
                default: v = io->joints ? io->joints[i].s0 : 0; break;
            }
        }
        put_i32(v);
    }
    if (W->str_src.empty()) {
        put_i32(0);
        put_i32(0);
    }
    put_i32(cfg.batch);
    put_i32(io->substeps);
    memcpy(p, &io->sub_dt, 4);
    p += 4;
    const int max_it = batch_bp ? io->substeps + 2 : 1;
    const int max_pass = std::min(W->max_passes > 0 ? std::min(W->max_passes, max_it) : max_it, vmas::kGridMaxPasses);
    put_i32(persistent ? max_pass : max_it);
    for (const auto& q : W->prm_src) {
        const float v = q.first >= 0 ? prm_value(W->ed[q.first], q.second) : prm_world_value(W->cfg, q.second);
        memcpy(p, &v, 4);
        p += 4;
    }
    size_t size = ((size_t)(p - buf.data()) + 7) & ~(size_t)7;
    if (size > buf.size()) return jfail(VMAS_E_INVALID, "kernel argument block overflow");
    size = buf.size();  // (Args.tail, when the module has one: zero -- no tail; a chain replay sets it)
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, buf.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                     HIP_LAUNCH_PARAM_END};

    // a fixed-point failure of an earlier step (sticky error bits, which the kernel
    // stores into mapped host memory) surfaces here
    if (uint32_t e = *(volatile uint32_t*)W->h_err)
        return jfail(e & vmas::kGridErrNoConverge ? VMAS_E_NOCONVERGE : VMAS_E_HIP,
                     "device-side broadphase fixed point failed in an earlier step (error bits 0x%x)", e);
    W->last_stream = stream;
    W->last_persistent = persistent;
    const size_t nwords = (size_t)io->substeps * W->W;
    // (the persistent kernel's control words need no reset: global pass numbers, vmas_jit_ops.hpp)
    if (!persistent) JHIP(vmas_aux::fill_u32_async(W->d_mask, 0u, nwords, stream));
    // Timing (vmas_jit_world_set_timing): the events ride on the kernel's own dispatch packet
    // (hipExtModuleLaunchKernel), so they bracket its execution alone, as rocprofv3's kernel
    // trace does -- events recorded around a launch on an idle queue also count the dispatch gap.
    auto ev_pair = [&](std::pair<hipEvent_t, hipEvent_t>* ev) -> int32_t {
        if (W->ev_free.empty()) {
            JHIP(hipEventCreate(&ev->first));
            JHIP(hipEventCreate(&ev->second));
        } else {
            *ev = W->ev_free.back();
            W->ev_free.pop_back();
        }
        return VMAS_OK;
    };
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    JHIP(hipStreamIsCapturing(stream, &cap));
    const bool capturing = cap == hipStreamCaptureStatusActive;
    auto launch_plain = [&](int blocks, hipFunction_t fn, bool timed) -> int32_t {
        const uint32_t threads = (uint32_t)(W->nw * W->ng) * 64;
        if (!W->timing || capturing || !timed) {  // (a captured launch is timed by the device timer)
            JHIP(hipModuleLaunchKernel(fn, blocks, 1, 1, threads, 1, 1, 0, stream, nullptr, extra));
            return VMAS_OK;
        }
        std::pair<hipEvent_t, hipEvent_t> ev{};
        if (int32_t rc = ev_pair(&ev)) return rc;
        JHIP(hipExtModuleLaunchKernel(fn, (uint32_t)blocks * threads, 1, 1, threads, 1, 1, 0, stream, nullptr,
                                      extra, ev.first, ev.second, 0));
        W->ev_pending.push_back(ev);
        return VMAS_OK;
    };
    if (persistent) {
        // one launch runs every pass of the fixed point; nothing waits on the host
        if (int32_t rc = launch_plain(W->grid, W->fn, true)) return rc;
        if (iterations) *iterations = 0;  // not known without a sync: vmas_jit_world_passes
        return VMAS_OK;
    }
    for (int it = 0; it < max_it; ++it) {
        if (int32_t rc = launch_plain(W->nblk, W->fn, true)) return rc;
        W->last_passes = it + 1;
        if (iterations) *iterations = it + 1;
        if (!batch_bp) return VMAS_OK;
        hipLaunchKernelGGL(k_jit_flags_reduce, dim3(1), dim3(1024), 0, stream, (const uint32_t*)W->d_blk, W->nblk,
                           io->substeps, W->W, W->d_mask, W->d_viol);
        JHIP(hipGetLastError());
        JHIP(hipMemcpyAsync(W->h_viol, W->d_viol, 4, hipMemcpyDeviceToHost, stream));
        vmas_aux::note_host_wait();
        JHIP(hipStreamSynchronize(stream));
        if (*W->h_viol == 0u) return VMAS_OK;
    }
    return jfail(VMAS_E_NOCONVERGE, "broadphase fixed point did not converge");
}

// The scenario program a world module was compiled with (VMAS_EPILOGUE_*).
int32_t vmas_jit_world_epilogue(const VmasJitWorld* W) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    return W->fn_prog ? W->cfg.epilogue : VMAS_EPILOGUE_NONE;
}

// A scenario program (VMAS_EPILOGUE_*: balance.py:205-262, transport.py:130-190) by the module's
// k_program_jit: the code k_world runs as its epilogue when a replay fuses the two launches, so the
// eager step and the replay agree bit for bit (both IEEE: vmas_programs.hpp).
int32_t vmas_jit_program_outputs(VmasJitWorld* W, int32_t kind, const void* io_, void* stream) {
    if (!W || !io_) return jfail(VMAS_E_INVALID, "null argument");
    if (!W->fn_prog || kind != W->cfg.epilogue) return jfail(VMAS_E_INVALID, "the world module has no program %d", kind);
    size_t size = 0;
    alignas(16) char buf[sizeof(VmasBalanceIO) > sizeof(VmasTransportIO) ? sizeof(VmasBalanceIO) : sizeof(VmasTransportIO)];
    if (kind == VMAS_EPILOGUE_BALANCE) {
        const VmasBalanceIO* io = (const VmasBalanceIO*)io_;
        if (io->batch != W->cfg.batch || io->n_agents < 0 || io->n_agents > VMAS_SCN_MAX_AGENTS)
            return jfail(VMAS_E_INVALID, "vmas_jit_program_outputs(balance): bad arguments");
        if (io->package.shape != VMAS_SPHERE || io->goal.shape != VMAS_SPHERE || io->line.shape != VMAS_LINE ||
            io->floor.shape != VMAS_BOX)
            return jfail(VMAS_E_INVALID, "vmas_jit_program_outputs(balance): unexpected entity shapes");
        size = sizeof *io;
    } else {
        const VmasTransportIO* io = (const VmasTransportIO*)io_;
        if (io->batch != W->cfg.batch || io->n_agents < 0 || io->n_agents > VMAS_TRANSPORT_MAX_AGENTS ||
            io->n_packages < 0 || io->n_packages > VMAS_TRANSPORT_MAX_PACKAGES)
            return jfail(VMAS_E_INVALID, "vmas_jit_program_outputs(transport): bad arguments");
        for (int i = 0; i < io->n_packages; ++i)
            if (io->package[i].shape != VMAS_BOX || io->goal[i].shape != VMAS_SPHERE)
                return jfail(VMAS_E_INVALID, "vmas_jit_program_outputs(transport): package %d is not (box, sphere goal)", i);
        if (io->n_agents > 0 && W->nw < 2) return jfail(VMAS_E_INVALID, "vmas_jit_program_outputs: too few waves");
        size = sizeof *io;
    }
    memcpy(buf, io_, size);
    int cur = -1;
    JHIP(hipGetDevice(&cur));
    if (cur != W->cfg.device) JHIP(hipSetDevice(W->cfg.device));
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, buf, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
    JHIP(hipModuleLaunchKernel(W->fn_prog, (W->cfg.batch + 63) / 64, 1, 1, (uint32_t)W->nw * 64, 1, 1, 0,
                               (hipStream_t)stream, nullptr, extra));
    return VMAS_OK;
}

// Passes the last step ran (waits for it).  Also reports a device-side fixed-point failure.
int32_t vmas_jit_world_passes(VmasJitWorld* W, int32_t* passes) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    if (!W->last_persistent) {
        if (passes) *passes = W->last_passes;
        return VMAS_OK;
    }
    JHIP(hipSetDevice(W->cfg.device));
    JHIP(hipStreamSynchronize(W->last_stream));
    uint32_t ctl[3] = {0, 0, 0}, err = 0;
    JHIP(hipMemcpy(ctl, W->d_ctl, sizeof ctl, hipMemcpyDeviceToHost));
    JHIP(hipMemcpy(&err, W->d_err, 4, hipMemcpyDeviceToHost));
    if (passes) *passes = (int32_t)ctl[2];
    if (err)
        return jfail(err & vmas::kGridErrNoConverge ? VMAS_E_NOCONVERGE : VMAS_E_HIP,
                     "device-side broadphase fixed point failed (error bits 0x%x)", err);
    return VMAS_OK;
}

int32_t vmas_jit_world_set_params(VmasJitWorld* W, const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                                  const VmasPairDesc* pairs, const VmasJointDesc* joints) {
    if (!W || !cfg || !entities || (cfg->n_pairs && !pairs) || (cfg->n_joints && !joints))
        return jfail(VMAS_E_INVALID, "null argument");
    const VmasWorldConfig& c = W->cfg;
    if (cfg->n_entities != c.n_entities || cfg->n_agents != c.n_agents || cfg->n_pairs != c.n_pairs ||
        cfg->n_joints != c.n_joints || cfg->batch != c.batch || cfg->device != c.device ||
        cfg->n_out_lin != c.n_out_lin || cfg->n_out_rot != c.n_out_rot || cfg->n_out_force != c.n_out_force ||
        cfg->n_out_torque != c.n_out_torque || cfg->contact_margin != c.contact_margin ||
        cfg->collision_force != c.collision_force || cfg->joint_force != c.joint_force ||
        cfg->torque_constraint_force != c.torque_constraint_force || cfg->has_world_gravity != c.has_world_gravity ||
        cfg->has_x_semidim != c.has_x_semidim || cfg->has_y_semidim != c.has_y_semidim ||
        cfg->max_substeps != c.max_substeps || cfg->export_forces != c.export_forces || cfg->epilogue != c.epilogue)
        return jfail(VMAS_E_INVALID, "set_params: the world configuration differs in structure");
    for (int e = 0; e < c.n_entities; ++e) {
        const VmasEntityDesc &a = W->ed[e], &b = entities[e];
        if (a.shape != b.shape || a.flags != b.flags || a.agent_index != b.agent_index || a.out_lin != b.out_lin ||
            a.out_rot != b.out_rot || a.out_force != b.out_force || a.out_torque != b.out_torque ||
            a.radius != b.radius || a.half_length != b.half_length || a.half_width != b.half_width)
            return jfail(VMAS_E_INVALID, "set_params: entity %d differs in structure", e);
        for (int k = 0; k <= kPrmTRange; ++k)  // (fields folded into the code: VMAS_JIT_PRM_MASK)
            if (!((W->prm_mask >> k) & 1u) && prm_value(a, k) != prm_value(b, k))
                return jfail(VMAS_E_INVALID, "set_params: entity %d field %d is folded into the code", e, k);
    }
    if (!((W->prm_mask >> 11) & 1u))
        for (int k = 0; k < 4; ++k)
            if (prm_world_value(c, k) != prm_world_value(*cfg, k))
                return jfail(VMAS_E_INVALID, "set_params: the world values are folded into the code");
    // pairs (classes, order, broadphase radii, d_min) and joints (anchors, dist, fixed rotation)
    // are folded into the code
    if (c.n_pairs && memcmp(pairs, W->pd.data(), sizeof(VmasPairDesc) * (size_t)c.n_pairs) != 0)
        return jfail(VMAS_E_INVALID, "set_params: the pair table differs");
    if (c.n_joints && memcmp(joints, W->jd.data(), sizeof(VmasJointDesc) * (size_t)c.n_joints) != 0)
        return jfail(VMAS_E_INVALID, "set_params: the joint table differs");
    W->ed.assign(entities, entities + c.n_entities);
    W->cfg.gravity_x = cfg->gravity_x;
    W->cfg.gravity_y = cfg->gravity_y;
    W->cfg.x_semidim = cfg->x_semidim;
    W->cfg.y_semidim = cfg->y_semidim;
    return VMAS_OK;
}

// Error bits the kernel has reported so far (no wait: launches replayed from a HIP graph surface
// a fixed-point failure through this check).
int32_t vmas_jit_world_check(VmasJitWorld* W) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    if (uint32_t e = *(volatile uint32_t*)W->h_err)
        return jfail(e & vmas::kGridErrNoConverge ? VMAS_E_NOCONVERGE : VMAS_E_HIP,
                     "device-side broadphase fixed point failed in an earlier step (error bits 0x%x)", e);
    return VMAS_OK;
}

// 0: host-driven passes; otherwise the persistent grid size (returned negative: plain launches)
int32_t vmas_jit_world_grid(const VmasJitWorld* W) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    return -W->grid;
}

int32_t vmas_jit_world_set_timing(VmasJitWorld* W, int32_t enable) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    W->timing = enable != 0;
    return VMAS_OK;
}

// Device timer totals (timing on, persistent launches): every launch -- eager or replayed from a
// HIP graph -- adds (final decision - workgroup 0 start) in s_memrealtime ticks; *clock_ghz is
// the in-kernel shader clock of the reducing workgroups.  Waits for the device.
int32_t vmas_jit_world_device_timing(VmasJitWorld* W, int32_t reset, double* total_ms, int64_t* launches,
                                     double* clock_ghz) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    JHIP(hipSetDevice(W->cfg.device));
    JHIP(hipDeviceSynchronize());
    unsigned long long tm[7] = {0, 0, 0, 0, 0, 0, 0};
    JHIP(hipMemcpy(tm, W->d_tm, sizeof tm, hipMemcpyDeviceToHost));
    if (total_ms) *total_ms = (double)tm[2] / (double)W->wall_khz;
    if (launches) *launches = (int64_t)tm[4];
    if (clock_ghz) *clock_ghz = tm[6] ? (double)tm[5] / (double)tm[6] * (double)W->wall_khz * 1e-6 : 0.0;
    if (reset) JHIP(hipMemset(W->d_tm, 0, 8 * 8));
    return VMAS_OK;
}

int32_t vmas_jit_world_get_timing(VmasJitWorld* W, int32_t reset, double* total_ms, int64_t* launches) {
    if (!W) return jfail(VMAS_E_INVALID, "null world");
    JHIP(hipSetDevice(W->cfg.device));
    for (auto& ev : W->ev_pending) {
        float ms = 0.f;
        JHIP(hipEventSynchronize(ev.second));
        JHIP(hipEventElapsedTime(&ms, ev.first, ev.second));
        W->timed_ms += ms;
        W->timed_launches += 1;
        W->ev_free.push_back(ev);
    }
    W->ev_pending.clear();
    if (total_ms) *total_ms = W->timed_ms;
    if (launches) *launches = W->timed_launches;
    if (reset) {
        W->timed_ms = 0.0;
        W->timed_launches = 0;
    }
    return VMAS_OK;
}

}  // extern "C"
