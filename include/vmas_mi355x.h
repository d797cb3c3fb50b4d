/*
 * vmas_mi355x.h -- C ABI of the MI355X-native VMAS physics engine.
 *
 * The reference (robj0nes/VectorizedMultiAgentSimulator, pure Python + PyTorch) has no FFI; its
 * hot path is a sequence of PyTorch tensor ops behind three Python seams.  Each entry point below
 * replaces one of those seams (file:line relative to the reference checkout):
 *
 *   vmas_world_step      <- World.step                         vmas/simulator/core.py:1971-2014
 *                           (force/torque accumulation 2017-2101, broadphase + 6 narrowphases +
 *                            joints 2103-2838, semi-implicit Euler 2859-2907)
 *   vmas_cast_rays       <- World.cast_rays / World.cast_ray     vmas/simulator/core.py:1627-1785
 *                           (Lidar.measure, vmas/simulator/sensors.py:100-122)
 *   vmas_distance        <- World.get_distance_from_point / get_distance / is_overlapping
 *                                                                vmas/simulator/core.py:1787-1968
 *
 * Conventions
 *   - Plain pointers and sizes only; every float is IEEE fp32 (the reference computes in
 *     torch.float32, core.py:304-315).
 *   - `device` >= 0 selects a HIP device (gfx950); pointers are then device pointers and the call
 *     is stream-ordered on `stream` (a hipStream_t, NULL = default stream).  `device` == -1 runs
 *     the same arithmetic on host threads over host pointers (`stream` ignored).
 *   - Every call returns 0 on success or a negative VMAS_E_* code; nothing throws across the ABI.
 *   - The library allocates device memory only in vmas_world_create (tables, broadphase flag
 *     scratch) and in a process-wide pinned staging ring used to upload the per-call pointer
 *     tables; per-call it allocates nothing.
 *   - State tensors are addressed through per-call pointer tables with explicit element strides,
 *     so the caller's tensors (views, user-replaced tensors, in-place mutated tensors) are read
 *     exactly where they live.  Outputs go to caller-provided fresh buffers, mirroring the
 *     reference's "every integrated field is a new tensor" semantics (core.py:2866-2907).
 */
#ifndef VMAS_MI355X_H
#define VMAS_MI355X_H

#ifndef __HIPCC_RTC__ /* under hipRTC the types come from csrc/vmas_physics.hpp */
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* v3: VmasDiscoveryIO gained covered_count / all_time / done; increment spans (src NULL) in
 * vmas_copy_spans; VMAS_COPY_MAX_SPANS 160
 * v4: VmasSpawnTargetsIO max_tries / backup; vmas_uniform_columns_snap
 * v5: VmasSpawnTargetsIO scratch / scratch_words (the windowed respawn), vmas_spawn_scratch_words;
 *     the fused programs' out_delta (direct outputs) and VMAS_COPY_STORE64 spans */
#define VMAS_ABI_VERSION 6

/* error codes */
#define VMAS_OK 0
#define VMAS_E_INVALID (-1)
#define VMAS_E_HIP (-2)
#define VMAS_E_NOMEM (-3)
#define VMAS_E_NOCONVERGE (-4)
#define VMAS_E_UNSUPPORTED (-5) /* vmas_graph_chain_build: the graph is not a short chain of kernel nodes */

/* shapes: vmas/simulator/core.py:102-202 */
#define VMAS_SPHERE 0
#define VMAS_BOX 1
#define VMAS_LINE 2

/* pair classes in the reference's dispatch order (core.py:2174-2188) */
#define VMAS_PAIR_JOINT 0
#define VMAS_PAIR_SS 1
#define VMAS_PAIR_LS 2 /* (line, sphere)  canonicalised as core.py:2134-2139 */
#define VMAS_PAIR_LL 3
#define VMAS_PAIR_BS 4 /* (box, sphere)   core.py:2150-2155 */
#define VMAS_PAIR_BL 5 /* (box, line)     core.py:2162-2167 */
#define VMAS_PAIR_BB 6

/* entity flags */
#define VMAS_F_MOVABLE (1u << 0)
#define VMAS_F_ROTATABLE (1u << 1)
#define VMAS_F_HOLLOW (1u << 2)
#define VMAS_F_AGENT (1u << 3)
#define VMAS_F_MAX_F (1u << 4)
#define VMAS_F_F_RANGE (1u << 5)
#define VMAS_F_MAX_T (1u << 6)
#define VMAS_F_T_RANGE (1u << 7)
#define VMAS_F_MAX_SPEED (1u << 8)
#define VMAS_F_V_RANGE (1u << 9)
#define VMAS_F_LIN_FRIC (1u << 10) /* linear friction applies (entity value or world > 0) */
#define VMAS_F_ANG_FRIC (1u << 11)
#define VMAS_F_GRAVITY (1u << 12) /* entity gravity tensor present (core.py:2048-2051) */

/* broadphase semantics */
#define VMAS_BROADPHASE_BATCH 0 /* reference: pair simulated iff ANY env in range (core.py:2796) */
#define VMAS_BROADPHASE_ENV 1   /* every static candidate pair simulated in every env */

/* Static per-entity parameters (host array; uploaded once by vmas_world_create). */
typedef struct VmasEntityDesc {
    int32_t shape;         /* VMAS_SPHERE / VMAS_BOX / VMAS_LINE */
    uint32_t flags;        /* VMAS_F_* */
    int32_t agent_index;   /* index into VmasStepIO.agents, -1 for landmarks */
    int32_t out_lin;       /* slot in out_pos/out_vel, -1 if not movable */
    int32_t out_rot;       /* slot in out_rot/out_ang_vel, -1 if not rotatable */
    int32_t out_force;     /* slot in out_force (agent force clamps write back), -1 if none */
    int32_t out_torque;    /* slot in out_torque, -1 if none */
    float radius;          /* f32(Sphere.radius) */
    float half_length;     /* f32(length) / 2  (box / line) */
    float half_width;      /* f32(width) / 2   (box) */
    float mass;            /* f32(mass) */
    float inertia;         /* f32(moment_of_inertia(mass)) computed in double (core.py:122-187) */
    float one_minus_drag;  /* f32(1 - (entity.drag or world.drag)) (core.py:2864-2868) */
    float lin_fric;        /* f32(linear friction coefficient) */
    float ang_fric;        /* f32(angular friction coefficient) */
    float max_speed, v_range, max_f, f_range, max_t, t_range;
} VmasEntityDesc;

/* Static candidate pair (host array in the reference's accumulation order). */
typedef struct VmasPairDesc {
    int32_t cls;       /* VMAS_PAIR_* */
    int32_t ea, eb;    /* entity indices; for joints: JointConstraint.entity_a / entity_b */
    int32_t joint;     /* joint index for VMAS_PAIR_JOINT, else -1 */
    float bp_radius;   /* f32(circumscribed_radius(a) + circumscribed_radius(b)) (core.py:2796-2800) */
    float dmin;        /* class part of dist_min: SS f32(ra)+f32(rb); LS/BS f32(r)+f32(LINE_MIN_DIST);
                          LL/BL/BB f32(LINE_MIN_DIST); joints f32(dist) */
} VmasPairDesc;

/* Static joint constraint (joints.py:147-215, core.py:2200-2291). */
typedef struct VmasJointDesc {
    float delta_a_x, delta_a_y; /* shape.get_delta_from_anchor(anchor_a) as f32 */
    float delta_b_x, delta_b_y;
    float dist;
    int32_t rotate;
    float fixed_rotation;       /* used when VmasJointIO.fixed_rotation is NULL */
    int32_t pad;
} VmasJointDesc;

/* World-level constants (World.__init__, core.py:1090-1149). */
typedef struct VmasWorldConfig {
    int32_t n_entities, n_agents, n_pairs, n_joints;
    int32_t batch;            /* num_envs */
    int32_t device;           /* HIP ordinal, or -1 for host */
    int32_t n_out_lin, n_out_rot, n_out_force, n_out_torque;
    float contact_margin, collision_force, joint_force, torque_constraint_force;
    float gravity_x, gravity_y;
    int32_t has_world_gravity; /* not (gravity == 0).all()  (core.py:2044) */
    float x_semidim, y_semidim;
    int32_t has_x_semidim, has_y_semidim;
    int32_t max_substeps;     /* capacity of the broadphase flag scratch */
    int32_t export_forces;    /* 1: the step fills VmasStepIO.out_fdict / out_tdict (World.forces_dict /
                                 torques_dict, core.py:1975-1992); 0: those pointers must be NULL */
    int32_t epilogue;         /* (v6) VMAS_EPILOGUE_*: a scenario program the world-specialised module
                                 also compiles, as its own kernel and as an optional k_world epilogue
                                 (vmas_jit_program_outputs, vmas_graph_chain_build); ignored by
                                 vmas_world_create */
    int32_t pad_cfg;
} VmasWorldConfig;
#define VMAS_EPILOGUE_NONE 0
#define VMAS_EPILOGUE_BALANCE 1 /* balance.py:205-262 (VmasBalanceIO) */
#define VMAS_EPILOGUE_TRANSPORT 2 /* transport.py:130-190 (VmasTransportIO) */

/* Per-call input pointers.  Strides are in elements (torch .stride()). */
typedef struct VmasEntityIO {
    const float* pos;     /* [B,2] */
    const float* vel;     /* [B,2] */
    const float* rot;     /* [B,1] */
    const float* ang_vel; /* [B,1] */
    const float* gravity; /* entity gravity broadcast to [B,2] (strides may be 0), or NULL */
    int32_t pos_s0, pos_s1, vel_s0, vel_s1;
    int32_t rot_s0, ang_s0, grav_s0, grav_s1;
} VmasEntityIO;

typedef struct VmasAgentIO {
    const float* force;  /* agent.state.force  [B,2] */
    const float* torque; /* agent.state.torque [B,1] */
    int32_t force_s0, force_s1, torque_s0, pad;
} VmasAgentIO;

typedef struct VmasJointIO {
    const float* fixed_rotation; /* per-env [B,1] tensor (Joint.notify), or NULL */
    int32_t s0, pad;
} VmasJointIO;

typedef struct VmasStepIO {
    const VmasEntityIO* entities; /* host array [n_entities] */
    const VmasAgentIO* agents;    /* host array [n_agents] */
    const VmasJointIO* joints;    /* host array [n_joints] or NULL */
    float* out_pos;    /* [n_out_lin][B][2] */
    float* out_vel;    /* [n_out_lin][B][2] */
    float* out_rot;    /* [n_out_rot][B] */
    float* out_ang_vel;/* [n_out_rot][B] */
    float* out_force;  /* [n_out_force][B][2] */
    float* out_torque; /* [n_out_torque][B] */
    int32_t substeps;
    float sub_dt;      /* f32(dt / substeps) */
    int32_t broadphase;/* VMAS_BROADPHASE_* */
    int32_t pad;
    /* World.forces_dict / torques_dict (core.py:1975-1992, 2027-2198): each dynamic entity's force
     * and torque totals of the LAST substep, [n_entities][B][2] / [n_entities][B] in entity
     * order; rows of entities that neither move nor rotate are not written.  NULL = not exported
     * (required when VmasWorldConfig.export_forces is 0). */
    float* out_fdict;
    float* out_tdict;
} VmasStepIO;

typedef struct VmasWorld VmasWorld;

/* Ray target (one filtered entity of World.cast_rays, core.py:1677-1690). */
typedef struct VmasRayTarget {
    int32_t shape;
    float radius, length, width; /* f32 of the python shape sizes */
    const float* pos;            /* [B,2] */
    const float* rot;            /* [B,1] */
    int32_t pos_s0, pos_s1, rot_s0, pad;
} VmasRayTarget;

/* Distance query operand (core.py:1787-1968). */
typedef struct VmasShapeRef {
    int32_t shape;
    int32_t pad0;
    float radius, length, width; /* f32 of the python shape sizes */
    float radius_lmd;            /* f32(radius + LINE_MIN_DIST) summed in double (core.py:1960) */
    const float* pos;
    const float* rot;
    int32_t pos_s0, pos_s1, rot_s0, pad;
} VmasShapeRef;

#define VMAS_DIST_POINT 0   /* get_distance_from_point(a, test_point) */
#define VMAS_DIST_PAIR 1    /* get_distance(a, b) */
#define VMAS_OVERLAP_PAIR 2 /* is_overlapping(a, b) -> out_dist holds 1.0f / 0.0f */

int32_t vmas_abi_version(void);
/* Number of HIP devices visible (0 if none / no driver). */
int32_t vmas_device_count(void);
const char* vmas_last_error(void);
/* Ends a stream capture left open by a failed HIP-graph capture (1 if one was ended) and clears
 * the last HIP error (graph mode's fallback to the eager step; no reference counterpart). */
int32_t vmas_stream_abort_capture(void* stream);
/* Launches an instantiated HIP graph (hipGraphExec_t) on a stream: graph mode's replay of a step
 * graph that draws no random numbers, without torch's generator-state prologue (no reference
 * counterpart). */
int32_t vmas_graph_launch(void* graph_exec, void* stream);
/* A captured step graph (hipGraph_t, torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()) that
 * is a chain of 1..max_nodes (<= VMAS_GRAPH_CHAIN_MAX) kernel nodes, replayed as plain kernel
 * launches on a stream: a replayed graph costs the GPU ~5 us more per launch than its kernels
 * launched on the stream (graph mode's replay; no reference counterpart).  build: VMAS_E_UNSUPPORTED
 * when the graph is not such a chain (the caller keeps vmas_graph_launch).  The nodes' arguments
 * stay owned by the graph, which must outlive the chain. */
#define VMAS_GRAPH_CHAIN_MAX 16
typedef struct VmasKernelChain VmasKernelChain;
int32_t vmas_graph_chain_build(void* graph, int32_t max_nodes, VmasKernelChain** out_chain);
int32_t vmas_graph_chain_launch(const VmasKernelChain* chain, void* stream);
int32_t vmas_graph_chain_nodes(const VmasKernelChain* chain); /* launches per replay (0: null chain) */
/* k_world + k_program_jit node pairs of the graph that run as ONE launch (k_world with its module's
 * scenario program as the epilogue, Args.epi set; VMAS_GRAPH_FUSE=0 disables) */
int32_t vmas_graph_chain_fused(const VmasKernelChain* chain);
int32_t vmas_graph_chain_free(VmasKernelChain* chain);
/* The state write-back variant of a chain (graph mode's rollback-free replays; no reference
 * counterpart): the chain's k_world launch with its backup delta set, so the step also writes its
 * integrated state into its own input tensors (a re-run fixed-point pass reads the pre-step state
 * from input + backup_delta, which the first pass stores) and the replay needs no post-replay carry
 * of that state.  set: VMAS_E_UNSUPPORTED when the chain has no k_world launch; 0 removes it.
 * launch_wb: vmas_graph_chain_launch with that variant. */
int32_t vmas_graph_chain_set_writeback(VmasKernelChain* chain, int64_t backup_delta);
int32_t vmas_graph_chain_launch_wb(const VmasKernelChain* chain, void* stream);
/* Host waits on the device performed by the library so far (stream / event synchronisations and
 * spins on published words; wraps around): graph mode runs one step between two reads of it to
 * tell whether the step can be captured (no reference counterpart). */
int32_t vmas_host_waits(void);

/* Test utility (no reference counterpart): launches `blocks` workgroups of 256 threads on
 * `stream` that each occupy their CU for `microseconds` (<= 5 s) -- a kernel of another stream
 * holding CUs while a step runs (tests/test_jit.py). */
int32_t vmas_test_hold(int32_t device, int32_t blocks, int64_t microseconds, void* stream);

int32_t vmas_world_create(const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                          const VmasPairDesc* pairs, const VmasJointDesc* joints,
                          VmasWorld** out_world);
int32_t vmas_world_destroy(VmasWorld* world);

/* One World.step(): all substeps.  Under VMAS_BROADPHASE_BATCH the call returns after the
 * broadphase fixed point has been verified (one host<->device handshake per iteration);
 * *iterations (may be NULL) receives the number of kernel passes used. */
int32_t vmas_world_step(VmasWorld* world, const VmasStepIO* io, void* stream, int32_t* iterations);

/* Measurement hooks (no reference counterpart): when enabled, every k_step launch of this world
 * is bracketed by HIP events on its launch stream; get_timing resolves them (synchronising on the
 * events) and returns the accumulated kernel milliseconds and launch count. */
int32_t vmas_world_set_timing(VmasWorld* world, int32_t enable);
int32_t vmas_world_get_timing(VmasWorld* world, int32_t reset, double* total_ms, int64_t* launches);

/* World.cast_rays(entity, angles, max_range, entity_filter) with the filter already applied:
 * out[b, r] = min(max_range, min over targets of the ray distance).  angle[b, r] =
 * angles[b*ang_s0 + r*ang_s1] (+ rot_offset[b*rot_s0] when rot_offset != NULL, the Lidar's
 * `self._angles + agent.state.rot`). */
int32_t vmas_cast_rays(int32_t device, int32_t batch, int32_t n_rays, const float* origin,
                       int32_t origin_s0, int32_t origin_s1, const float* angles, int32_t ang_s0,
                       int32_t ang_s1, const float* rot_offset, int32_t rot_s0,
                       const VmasRayTarget* targets, int32_t n_targets, float max_range,
                       float* out, void* stream);

/* Action validation of Environment.step (environment.py:621-623 and 653-655) for all agents in
 * one pass: flags[2*i] = any NaN in agent i's action, flags[2*i+1] = any |u| > u_range in its
 * physical columns (after the optional clamp, i.e. never when clamp != 0).  `flags` is a HOST
 * array; the call returns after the flags are known (one device->host handshake). */
typedef struct VmasActionRef {
    const float* u;       /* [B, n_cols] action tensor (any strides) */
    const float* u_range; /* [n_phys] u_range_tensor on the same device */
    int32_t s0, s1;
    int32_t n_cols;       /* columns checked for NaN */
    int32_t n_phys;       /* leading columns range-checked */
    int32_t clamp;        /* clamp_actions: the range check cannot fail */
    int32_t pad;
} VmasActionRef;

int32_t vmas_check_actions(int32_t device, int32_t batch, const VmasActionRef* refs,
                           int32_t n_refs, uint8_t* flags, void* stream);

/* Continuous actions of Environment._set_action (environment.py:615-709) for all agents in one
 * pass (csrc/vmas_actions.hip), the no-communication case: per agent i, flags[2*i] = any NaN
 * in its n_cols action columns, flags[2*i+1] = any |u| > u_range in its n_phys physical columns
 * (never when clamp != 0), and the agent's new action.u, u[b, c] = (clamp ? min(max(x, -r), r)
 * : x) * u_mult[c], is written to out[out_offset + b*n_phys + c] (fp32).  `flags` is a HOST
 * array, known when the call returns: the kernel publishes them to mapped pinned memory and the
 * host waits on a sequence word, without a stream synchronisation.  Supersedes
 * vmas_check_actions for this case (same flags, plus u, one launch). */
typedef struct VmasActionApplyRef {
    const float* u;       /* [B, n_cols] action tensor (any strides) */
    const float* u_range; /* [n_phys] u_range_tensor on the same device */
    const float* u_mult;  /* [n_phys] u_multiplier_tensor on the same device */
    int64_t out_offset;   /* floats into out of this agent's [B, n_phys] u */
    int32_t s0, s1;
    int32_t n_cols;
    int32_t n_phys;
    int32_t clamp;
    int32_t pad;
} VmasActionApplyRef;

int32_t vmas_apply_actions(int32_t device, int32_t batch, const VmasActionApplyRef* refs,
                           int32_t n_refs, float* out, uint8_t* flags, void* stream);
/* The same split in two (GPU only, n_refs <= 8): _launch enqueues the kernel and returns the
 * sequence number it will publish; _flags waits for it and fills flags as above.  Graph mode
 * launches the replay between the two and rolls the step back when a flag is set. */
int32_t vmas_apply_actions_launch(int32_t device, int32_t batch, const VmasActionApplyRef* refs,
                                  int32_t n_refs, float* out, uint32_t* seq, void* stream);
int32_t vmas_apply_actions_flags(int32_t device, uint32_t seq, int32_t n_refs, uint8_t* flags,
                                 void* stream);

/* Random actions (Environment.get_random_actions, environment.py:524-606): the uniform_ draws
 * of every agent's action columns in one launch (csrc/vmas_actions.hip).  Column i gets
 * numel floats in [from, to) written to out[k * stride], drawn exactly as a torch uniform_ call
 * on a contiguous [numel] tensor would with the CUDA generator at (seed, offset + i * inc), where
 * inc is that call's philox increment; *increment = n_cols * inc is what the caller adds to the
 * generator's offset.  mode selects the fp contraction of two roundings (bit 0: the (0, 1]
 * mapping, bit 1: rand * range + from); the host keeps the mode that reproduces torch on the
 * device (probe) and otherwise draws with torch.  GPU only. */
typedef struct VmasUniformColumn {
    float* out;
    int64_t stride;      /* elements between consecutive draws */
    float from, to;      /* f32(low), f32(high) as torch casts them */
    uint64_t offset;     /* set by the library */
    /* Optional second output (u_out != NULL): the drawn value x as the step's action kernel
     * applies it (vmas_apply_actions: x clamped to +-u_range when u_clamp, times u_mult; the same
     * fp32 operations), at u_out[i * u_stride] -- the random actions of a graph-mode step drawn
     * and applied in one launch (environment.py:615-709 on values that pass its checks by
     * construction: uniform draws in [-u_range, u_range]). */
    float* u_out;
    int64_t u_stride;
    float u_range, u_mult;
    int32_t u_clamp, pad;
} VmasUniformColumn;

int32_t vmas_uniform_columns(int32_t device, int64_t numel, const VmasUniformColumn* cols,
                             int32_t n_cols, uint64_t seed, uint64_t offset, int32_t mode,
                             uint64_t* increment, void* stream);
/* The same draw; with u_snap_delta != 0 every pre-applied element's previous value (u_out[i *
 * u_stride] before this launch) is first stored u_snap_delta bytes from it: graph mode keeps the
 * values agents' action.u / state.force show until the step that consumes the draw (the reference's
 * get_random_action has no side effect on the agents, environment.py:524-582). */
int32_t vmas_uniform_columns_snap(int32_t device, int64_t numel, const VmasUniformColumn* cols,
                                  int32_t n_cols, uint64_t seed, uint64_t offset, int32_t mode,
                                  int64_t u_snap_delta, uint64_t* increment, void* stream);

/* Deferred device assertions for graph mode (csrc/vmas_actions.hip).  Replaces the host sync of
 * a reference assert on a device tensor inside the step -- Agent.action_callback's range check of
 * a scripted action (core.py:977-980) -- when the step is captured into a HIP graph.
 * vmas_assert_publish enqueues one kernel (capturable) that ANDs the n bytes of `cond` (torch.bool,
 * nonzero = holds) and publishes (epoch << 32 | violated) for `slot` into mapped host memory with
 * one system-scope store; every execution advances the slot's device epoch by one (0 skipped).
 * vmas_assert_wait spins on the host until the slot shows epoch `seq` and returns its violated
 * bit (polling the stream: an error or an idle stream without the store ends the wait with
 * VMAS_E_HIP).  No reference counterpart beyond the assert it defers. */
typedef struct VmasDeviceAssert VmasDeviceAssert;
int32_t vmas_assert_create(int32_t device, int32_t n_slots, VmasDeviceAssert** out);
int32_t vmas_assert_destroy(VmasDeviceAssert* ch);
int32_t vmas_assert_publish(VmasDeviceAssert* ch, int32_t slot, const uint8_t* cond, int64_t n,
                            void* stream);
int32_t vmas_assert_wait(VmasDeviceAssert* ch, int32_t slot, uint32_t seq, int32_t* violated,
                         void* stream);
/* The scripted-action range check itself (Agent.action_callback, core.py:977-980:
 * ((u / u_multiplier).abs() <= u_range).all(), u [batch, n] fp32 with element strides s0 / s1,
 * u_multiplier / u_range [n] fp32 device arrays) evaluated, reduced and published into `slot` by
 * one kernel, as vmas_assert_publish publishes a precomputed condition. */
int32_t vmas_assert_publish_range(VmasDeviceAssert* ch, int32_t slot, const float* u, int64_t s0,
                                  int64_t s1, int32_t batch, int32_t n, const float* mult,
                                  const float* range, void* stream);

/* Distance queries; out has B floats, or B bytes of 0/1 (torch.bool) for VMAS_OVERLAP_PAIR. */
int32_t vmas_distance(int32_t device, int32_t batch, int32_t kind, const VmasShapeRef* a,
                      const VmasShapeRef* b, const float* test_point, int32_t tp_s0,
                      int32_t tp_s1, void* out, void* stream);

/* Spawn sampler: one batch of tries of ScenarioUtils.find_random_pos_for_entity
 * (vmas/simulator/utils.py:272-319; rows "next" #3 of SURVEY.md §8f).  Implemented in
 * csrc/vmas_spawn.hip.
 *   occupied    [B, n_occ, 2] (element strides occ_s0/s1/s2); n_occ may be 0
 *   candidates  [n_tries][2][B]: try k of env b = (x, y) = (c[k*2B + b], c[k*2B + B + b]), drawn by
 *               the caller with the reference's torch uniform_ calls
 *   resolved    [B] int32, -1 for envs still searching; set to the global try index (first_try + k)
 *               of the first candidate whose torch.cdist distance to every occupied position is
 *               >= min_dist (fp32), whose (x, y) is then written to pos [B][2]
 *   max_accepted / n_unresolved: host int32 outputs (max accepted index, envs still searching);
 *               the call synchronises `stream` to return them.
 * The reference loop consumes 1 try if every env accepts try 0, else max_accepted + 2 tries. */
int32_t vmas_spawn_resolve(int32_t device, int32_t batch, const float* occupied, int32_t n_occ,
                           int32_t occ_s0, int32_t occ_s1, int32_t occ_s2, const float* candidates,
                           int32_t first_try, int32_t n_tries, float min_dist, float* pos,
                           int32_t* resolved, int32_t* max_accepted, int32_t* n_unresolved,
                           void* stream);

/* Spawn sampler for a sequence of entities in one stream-ordered call: the loop of
 * discovery's target respawn (discovery.py:237-252 of the reference; scenarios/discovery.py
 * _respawn) -- for target i = 0 .. n_targets-1, find_random_pos_for_entity over
 * occupied = [agents, every other target] (targets before i already moved), then
 * target_i.pos = where(covered[:, i], new, old).  The tries are drawn on the device with the
 * reference's numbers: try k of target i is torch's uniform_ on [B] for x at generator offset
 * o_i + k * per_try and for y at o_i + k * per_try + inc, per_try = 2 * inc, with inc, the element
 * to (philox subsequence, offset) mapping and the float mapping (`mode`, vmas_uniform_columns) of
 * PyTorch's distribution kernel; o_0 = offset and o_{i+1} = o_i + consumed_i * per_try, consumed_i
 * = 1 if every env accepts try 0, else max accepted try + 2 (the reference loop).  ONE launch on
 * `stream` (workgroups claim (target, 64 envs) items in order; target i's items start once target
 * i - 1's are done), no host wait inside.  The caller reads max_accepted once afterwards and
 * advances the generator by sum_i consumed_i * per_try (*increment returns inc).
 * max_accepted[n_targets] counts envs that found no position within max_tries tries (the
 * reference loops on), max_accepted[VMAS_SPAWN_ERR_WORD] is nonzero when the launch's bounded
 * wait timed out (a workgroup never ran); either way the caller restores the targets from
 * `backup` and redoes the respawn with the reference's unbounded loop. */
#define VMAS_SPAWN_MAX_TARGETS 16
#define VMAS_SPAWN_MAX_TRIES 65536
typedef struct VmasSpawnTargetsIO {
    int32_t batch, n_agents, n_targets, mode;
    const float* agents;                  /* [B, n_agents, 2] */
    int32_t ag_s0, ag_s1, ag_s2;
    int32_t max_tries;                    /* tries per target before an env counts as unresolved (0:
                                             VMAS_SPAWN_MAX_TRIES) */
    float* pos[VMAS_SPAWN_MAX_TARGETS];   /* target i's [B, 2] position, updated in place */
    int32_t pos_s0[VMAS_SPAWN_MAX_TARGETS], pos_s1[VMAS_SPAWN_MAX_TARGETS];
    const uint8_t* covered;               /* [B, n_targets] torch.bool */
    int32_t cov_s0, cov_s1;
    float min_dist, x_lo, x_hi, y_lo, y_hi, pad1;
    uint64_t seed, offset;
    int32_t* max_accepted;                /* VMAS_SPAWN_WORDS(n_targets) device int32: [0, T) per-target max
                                             accepted try, [T] envs with no position found, [64] 1 when the
                                             launch's bounded wait timed out (the rest: its counters) */
    struct VmasSpawnChannel* channel;     /* optional (vmas_spawn_channel_create): the launch reads seed and
                                             offset from it at run time (a captured launch replays with the
                                             generator state armed before each replay) and publishes its
                                             maxima there; seed / offset above are then ignored */
    float* backup;                        /* optional [n_targets][B][2]: every target's position before the
                                             launch (written by it), so that the caller can undo the launch:
                                             an unresolved env or a timed-out wait is then redone by the
                                             reference's unbounded loop (scenarios/discovery.py) */
    int32_t* scratch;                     /* optional (v5) device words for the windowed kernel (one hand-off
                                             between workgroups per call instead of one per target): at least
                                             vmas_spawn_scratch_words(batch, n_targets); null: the per-target
                                             kernels.  An env left without an accepted try inside the window
                                             (128 tries of the call's shared stream, VMAS_SPAWN_WINDOW) counts
                                             as unresolved, as past max_tries */
    int64_t scratch_words;
    int32_t prestaged;                    /* (v5, with a channel and the windowed kernels) the launch's words
                                             were cleaned by the previous call through them and the channel's
                                             words staged by an earlier launch on the stream (the discovery
                                             REWARD launch's stage_out): no clear kernel */
    int32_t pad2;
} VmasSpawnTargetsIO;
/* (int32 index of the words) where a channel's (seed, offset, seq) are staged for the launch */
#define VMAS_SPAWN_RNG_WORD 40
#define VMAS_SPAWN_WORDS(n_targets) (96 + 32 * (n_targets) + 32 * 32)
#define VMAS_SPAWN_ERR_WORD 64
/* (u64 at int32 index 36 of the words) the generator offset after a call through a channel: the
 * call's offset plus the tries the reference loop consumes (valid when the call resolved) */
#define VMAS_SPAWN_OFF_END_WORD 36
/* scratch words of the windowed kernel for (batch, n_targets); -1 for bad arguments */
int64_t vmas_spawn_scratch_words(int32_t batch, int32_t n_targets);
int32_t vmas_spawn_targets(int32_t device, const VmasSpawnTargetsIO* io, uint64_t* increment, void* stream);
/* Spawn channel: mapped pinned host words between the host and a (captured) vmas_spawn_targets
 * launch, so that a graph-mode step keeps the respawn inside its one graph: the host arms the
 * channel with the generator state before each replay, the launch reads it at run time, and its
 * last workgroup publishes the per-target maxima, the unresolved count and the error word with one
 * final system-scope sequence word; the host waits on that word once per step (after the rest of
 * the step is queued) and advances the generator.  Replaces the graph-mode host hole (a graph
 * break, a device->host read and a second graph launch in the middle of every discovery step). */
typedef struct VmasSpawnChannel VmasSpawnChannel;
int32_t vmas_spawn_channel_create(int32_t device, VmasSpawnChannel** out);
int32_t vmas_spawn_channel_destroy(VmasSpawnChannel* ch);
/* (v5) the device address of the channel's armed words (seed, offset, seq): what an earlier launch of
 * the step copies into the respawn's words (VmasDiscoveryIO.stage_in) */
int32_t vmas_spawn_channel_in(VmasSpawnChannel* ch, const uint64_t** d_in);
/* the generator state the next launch through the channel reads; seq != 0, new per launch */
int32_t vmas_spawn_channel_arm(VmasSpawnChannel* ch, uint64_t seed, uint64_t offset, uint32_t seq);
/* waits (host spin, checking `stream` for errors) for the launch armed with seq; words[0, T) the
 * maxima, [T] unresolved envs, [T + 1] error word (nonzero: the launch's bounded wait timed out;
 * the launch then publishes nothing and this returns VMAS_E_HIP once the stream has drained) */
int32_t vmas_spawn_channel_wait(VmasSpawnChannel* ch, uint32_t seq, int32_t* words, int32_t n_targets, void* stream);

/* Probe support: with VMAS_SPAWN_PROFILE=1 in the environment, vmas_spawn_targets records per
 * (target, 64-env group) item six u64 words (s_memrealtime when claimed, wait over, occupied
 * positions loaded, tries done, completion added; the workgroup); this copies up to n words of
 * the last launch's record to host memory and returns the count (0: none recorded). */
int32_t vmas_spawn_profile(uint64_t* out, int64_t n);

/* ---- fused scenario programs (csrc/vmas_scenarios.hip) -------------------
 * One launch computes a benchmark scenario's per-step observation / reward / done tensor program
 * (one thread per env, the reference's fp32 operations in its order).  Error reporting as the
 * other auxiliary entry points (vmas_aux_last_error). */
typedef struct VmasVec { /* a [B, 2] or [B, 1] fp32 tensor: element (b, k) at p[b * s0 + k * s1] */
    const float* p;
    int32_t s0, s1;
} VmasVec;

#define VMAS_SCN_MAX_AGENTS 32
#define VMAS_SCN_REWARD 1 /* the first agent's reward call and every agent's reward */
#define VMAS_SCN_OBS 2    /* every agent's observation */
#define VMAS_SCN_DONE 4   /* done() */

/* balance (reference vmas/scenarios/balance.py:205-262): replaces, for all agents at once,
 * Scenario.reward (compute_on_the_ground, the package-goal norm, ground / position rewards, the
 * global shaping update, ground_rew + pos_rew per agent), Scenario.observation (torch.cat of 9
 * pieces, 16 entries) and Scenario.done. */
typedef struct VmasBalanceIO {
    int32_t batch, n_agents, what, pad0;
    float shaping_factor, fall_reward, pi, pad1; /* pi: f32(math.pi), the `% torch.pi` divisor */
    VmasShapeRef package, goal, line, floor;     /* shapes + pos / rot, as for vmas_distance */
    VmasVec package_vel, line_vel, line_ang_vel;
    VmasVec agent_pos[VMAS_SCN_MAX_AGENTS], agent_vel[VMAS_SCN_MAX_AGENTS];
    const float* global_shaping; /* [B] (stride gs_s0) in: the previous shaping */
    int32_t gs_s0, pad2;
    float* global_shaping_out;   /* [B] REWARD outputs (fresh tensors) */
    float* package_dist;
    float* pos_rew;
    float* ground_rew;           /* [B] written in place (the reference's [:] = 0 + masked_fill_) */
    uint8_t* on_the_ground;      /* [B] torch.bool: REWARD output, DONE input */
    float* rewards[VMAS_SCN_MAX_AGENTS]; /* [B] per agent (REWARD) */
    float* obs[VMAS_SCN_MAX_AGENTS];     /* [B, 16] contiguous per agent (OBS) */
    uint8_t* done;                       /* [B] torch.bool (DONE) */
    float* pos_rew_prev; /* [B] the previous pos_rew, zeroed in place (REWARD; the reference's
                            `pos_rew[:] = 0` before re-binding it); may be NULL */
    const int64_t* out_delta;            /* optional (v5; graph mode's direct outputs): three device words,
                                             the byte offsets added to the obs / rewards / done pointers
                                             (simulator/environment/_graph.py DirectOutputs); NULL: none */
} VmasBalanceIO;
int32_t vmas_balance_outputs(int32_t device, const VmasBalanceIO* io, void* stream);
/* Test utility (no reference counterpart): out[0, n) = the scenario programs' flag-independent
 * IEEE division a / b (csrc/vmas_balance.hpp xdiv), out[n, 2n) = this build's `/`, out[2n, 3n) =
 * xsqrt(a), out[3n, 4n) = sqrtf(a) -- equal bit for bit (tests/test_fused.py). */
int32_t vmas_test_exact_math(int32_t device, const float* a, const float* b, float* out, int64_t n, void* stream);
/* Test entry point (no reference counterpart): the fast LIDAR programs' ray-direction instructions
 * (hardware sin / cos, as k_flocking_fast and k_discovery_obs_fast use them below |x| 16) over x:
 * out[i] = sin, out[n + i] = cos -- the parity tests' scan certification derives its angle bound
 * from them (tests/_scenario_parity.py SCAN_DELTA). */
int32_t vmas_test_fast_trig(int32_t device, const float* x, float* out, int64_t n, void* stream);

/* flocking (reference vmas/scenarios/flocking.py:149-206): replaces, for every policy agent at
 * once, Scenario.reward (the first policy agent's `t += 1` and pairwise collision rewards over
 * world.agents via get_distance, then per agent the mean squared distance error to every other
 * agent, dist_rew and the re-bound distance_shaping) and Scenario.observation (pos, vel, pos -
 * target pos and the agent's LIDAR, cast as World.cast_rays does).  Sphere agents and sphere LIDAR
 * targets only (checked; the scenario keeps its torch program otherwise).
 * Grid: one thread per (env, policy agent, part): the reward + observation head, or one LIDAR ray. */
#define VMAS_SCN_MAX_RAY_TARGETS 16
#define VMAS_FLOCK_MAX_AGENTS 16 /* the struct travels as kernel arguments (< 4 KiB) */
typedef struct VmasFlockingIO {
    int32_t batch, n_all, n_policy, what;
    int32_t target, n_rays, n_ray_targets, sum_mode; /* target: index in agents[]; sum_mode: accumulators of
                                                        the mean's sum order (vmas_scenarios.hip ordered_sum) */
    float min_collision_distance, collision_reward, desired_distance, dist_shaping_factor;
    float max_range, pad0;
    int32_t collide_reward_on;             /* the scenario's `collision_reward != 0` */
    int32_t fast_lidar;                    /* 1: one thread per (env, agent), direct ray-sphere
                                              form (k_flocking_fast; LIDAR within the parity
                                              tolerance); 0: bit-identical to k_cast_rays */
    VmasShapeRef agents[VMAS_FLOCK_MAX_AGENTS]; /* world.agents, in order (spheres) */
    int32_t scripted[VMAS_FLOCK_MAX_AGENTS];    /* action_script is not None */
    int32_t policy[VMAS_FLOCK_MAX_AGENTS];      /* world.policy_agents[p] = agents[policy[p]] */
    VmasVec vel[VMAS_FLOCK_MAX_AGENTS];         /* [B,2] per policy agent */
    VmasVec rot[VMAS_FLOCK_MAX_AGENTS];         /* [B,1] per policy agent: the LIDAR's angle offset */
    const float* angles[VMAS_FLOCK_MAX_AGENTS]; /* [B, n_rays] per policy agent (Lidar._angles) */
    int32_t ang_s0[VMAS_FLOCK_MAX_AGENTS], ang_s1[VMAS_FLOCK_MAX_AGENTS];
    VmasRayTarget ray_targets[VMAS_SCN_MAX_RAY_TARGETS];
    float* t;                                  /* [B] in place (REWARD: t += 1) */
    const float* shaping_in[VMAS_FLOCK_MAX_AGENTS];  /* [B] contiguous per policy agent */
    float* shaping_out[VMAS_FLOCK_MAX_AGENTS];   /* [B] fresh */
    float* dist_rew[VMAS_FLOCK_MAX_AGENTS];      /* [B] fresh */
    float* collision_rew[VMAS_FLOCK_MAX_AGENTS]; /* [B] in place */
    float* rewards[VMAS_FLOCK_MAX_AGENTS];       /* [B] fresh */
    float* obs[VMAS_FLOCK_MAX_AGENTS];           /* [B, 6 + n_rays] fresh (OBS) */
    float* lidar[VMAS_FLOCK_MAX_AGENTS];         /* [B, n_rays] fresh (OBS): Lidar._last_measurement */
    const int64_t* out_delta;            /* optional (v5; graph mode's direct outputs): three device words,
                                             the byte offsets added to the obs / rewards / done pointers
                                             (simulator/environment/_graph.py DirectOutputs); NULL: none */
} VmasFlockingIO;
int32_t vmas_flocking_outputs(int32_t device, const VmasFlockingIO* io, void* stream);
/* flocking's scripted target (flocking.py:81-87 action_script): u[b] = (cos(t[b] / period),
 * sin(t[b] / period)) written into u [batch, 2] (contiguous), the division as torch computes a
 * tensor / Python-scalar division (t * f32(1 / period)). */
int32_t vmas_flocking_target_action(int32_t device, const float* t, int32_t batch, float period, float* u,
                                    void* stream);

/* transport (reference vmas/scenarios/transport.py:130-190): replaces Scenario.reward (for the
 * first agent: per package dist_to_goal, on_goal = is_overlapping(package, goal), the colour,
 * the shaping reward and the re-bound global_shaping; the shared rew), Scenario.observation
 * (pos, vel, then per package: package - goal, package - agent, package vel, on_goal) and
 * Scenario.done.  Grid: one thread per (env, part): part 0 the reward + done, 1 + i agent i's
 * observation. */
#define VMAS_TRANSPORT_MAX_PACKAGES 8
#define VMAS_TRANSPORT_MAX_AGENTS 16
typedef struct VmasTransportIO {
    int32_t batch, n_agents, n_packages, what;
    float shaping_factor, red[3], green[3], pad0;
    VmasShapeRef package[VMAS_TRANSPORT_MAX_PACKAGES], goal[VMAS_TRANSPORT_MAX_PACKAGES];
    VmasVec package_vel[VMAS_TRANSPORT_MAX_PACKAGES];
    VmasVec agent_pos[VMAS_TRANSPORT_MAX_AGENTS], agent_vel[VMAS_TRANSPORT_MAX_AGENTS];
    const float* global_shaping[VMAS_TRANSPORT_MAX_PACKAGES]; /* [B] (stride gs_s0) in */
    int32_t gs_s0[VMAS_TRANSPORT_MAX_PACKAGES];
    float* global_shaping_out[VMAS_TRANSPORT_MAX_PACKAGES];   /* [B] fresh (REWARD) */
    float* dist_to_goal[VMAS_TRANSPORT_MAX_PACKAGES];         /* [B] fresh (REWARD) */
    uint8_t* on_goal[VMAS_TRANSPORT_MAX_PACKAGES];            /* [B] torch.bool fresh (REWARD) */
    float* color[VMAS_TRANSPORT_MAX_PACKAGES];                /* [B, 3] fresh (REWARD) */
    const uint8_t* on_goal_in[VMAS_TRANSPORT_MAX_PACKAGES];   /* [B] the attribute (OBS / DONE
                                                                 without REWARD) */
    float* rew;                                               /* [B] fresh (REWARD) */
    float* obs[VMAS_TRANSPORT_MAX_AGENTS];                    /* [B, 4 + 7 n_packages] (OBS) */
    uint8_t* done;                                            /* [B] torch.bool (DONE) */
    const int64_t* out_delta;            /* optional (v5; graph mode's direct outputs): three device words,
                                             the byte offsets added to the obs / rewards / done pointers
                                             (simulator/environment/_graph.py DirectOutputs); NULL: none */
} VmasTransportIO;
int32_t vmas_transport_outputs(int32_t device, const VmasTransportIO* io, void* stream);

/* discovery (reference vmas/scenarios/discovery.py:146-246), two launches per step:
 *   REWARD (the first agent's reward call): agents_pos / targets_pos stacks, the torch.cdist
 *     agent-target distances, agents_per_target (int64), covered_targets, every agent's
 *     covering_reward (in place), the shared covering reward (in place, halved where nonzero),
 *     time_rew and every agent's reward (collision_rew + covering + time_rew; the agent
 *     collision penalty must be 0: the scenario checks);
 *   OBS (the first observation call, after the last agent's reward has respawned the targets):
 *     every agent's observation (pos, vel, then each LIDAR, cast as World.cast_rays does).
 * Entities are spheres (checked): a compact table in world.entities order; each LIDAR sees the
 * table entries of its mask but never its own agent.  Grid: REWARD one thread per env; OBS one
 * thread per (env, agent, part): part 0 the pos / vel head, then one per LIDAR ray. */
#define VMAS_DISC_MAX_AGENTS 16
#define VMAS_DISC_MAX_TARGETS 16
#define VMAS_DISC_MAX_ENTITIES 32
#define VMAS_DISC_MAX_LIDARS 2
typedef struct VmasDiscoveryIO {
    int32_t batch, n_agents, n_targets, what;
    float covering_range, covering_rew_coeff, time_penalty;
    int32_t agents_per_target, shared_reward, n_entities, n_lidars;
    int32_t time_int;             /* time_rew is int64 (torch.full of a python int), value time_penalty_i */
    int32_t fast_lidar;           /* 1: OBS with the direct ray-sphere form (k_discovery_obs_fast; within
                                     the LIDAR parity tolerance); 0: bit-identical to k_cast_rays */
    int64_t time_penalty_i;
    int32_t agent_entity[VMAS_DISC_MAX_AGENTS];  /* table index of agent i */
    int32_t target_entity[VMAS_DISC_MAX_TARGETS]; /* table index of target j (scenario order) */
    VmasVec pos[VMAS_DISC_MAX_ENTITIES];          /* entity table: [B,2] positions */
    float radius[VMAS_DISC_MAX_ENTITIES];
    VmasVec vel[VMAS_DISC_MAX_AGENTS], rot[VMAS_DISC_MAX_AGENTS];
    int32_t n_rays[VMAS_DISC_MAX_LIDARS];
    float max_range[VMAS_DISC_MAX_LIDARS];
    uint32_t mask[VMAS_DISC_MAX_LIDARS];          /* entity-table bits each LIDAR sees */
    const float* angles[VMAS_DISC_MAX_LIDARS][VMAS_DISC_MAX_AGENTS]; /* [B, n_rays] */
    int32_t ang_s0[VMAS_DISC_MAX_LIDARS][VMAS_DISC_MAX_AGENTS], ang_s1[VMAS_DISC_MAX_LIDARS][VMAS_DISC_MAX_AGENTS];
    float* lidar[VMAS_DISC_MAX_LIDARS][VMAS_DISC_MAX_AGENTS];        /* [B, n_rays] fresh (OBS) */
    float* obs[VMAS_DISC_MAX_AGENTS];             /* [B, 4 + sum n_rays] fresh (OBS) */
    float* agents_pos;                            /* [B, A, 2] fresh (REWARD) */
    float* targets_pos;                           /* [B, T, 2] fresh */
    float* dists;                                 /* [B, A, T] fresh */
    int64_t* per_target;                          /* [B, T] fresh */
    uint8_t* covered;                             /* [B, T] torch.bool fresh */
    void* time_rew;                               /* [B] fresh: float32, or int64 when time_int */
    float* shared;                                /* [B] in place */
    float* covering[VMAS_DISC_MAX_AGENTS];        /* [B] in place */
    float* collision[VMAS_DISC_MAX_AGENTS];       /* [B] in place (zeroed) */
    float* rewards[VMAS_DISC_MAX_AGENTS];         /* [B] fresh */
    /* (REWARD, optional: NULL skips) the step's other reductions over the targets, computed where
     * covered_targets is: info's targets_covered = covered_targets.sum(-1) (discovery.py:247-255)
     * and done() = all_time_covered_targets.all(-1) (discovery.py:264-265) */
    int64_t* covered_count;                       /* [B] fresh */
    const uint8_t* all_time;                      /* [B, T] torch.bool, contiguous */
    uint8_t* done;                                /* [B] torch.bool fresh */
    const int64_t* out_delta;            /* optional (v5; graph mode's direct outputs): three device words,
                                             the byte offsets added to the obs / rewards / done pointers
                                             (simulator/environment/_graph.py DirectOutputs); NULL: none */
    const uint64_t* stage_in;            /* optional (v5): a spawn channel's armed words (seed, offset,
                                             seq), copied by the REWARD launch into stage_out -- the step's
                                             respawn launch then needs no clear kernel of its own
                                             (VmasSpawnTargetsIO.prestaged) */
    uint64_t* stage_out;
} VmasDiscoveryIO;
int32_t vmas_discovery_outputs(int32_t device, const VmasDiscoveryIO* io, void* stream);

/* Device-to-device byte copies, all spans in one launch (csrc/vmas_copy.hip): graph mode's carried
 * state, output clones and per-step backups (simulator/environment/_graph.py; no reference
 * counterpart -- the reference returns fresh tensors from its eager ops).  Spans must not
 * overlap one another's destinations; more than VMAS_COPY_MAX_SPANS spans take several launches.
 * A span with src == NULL is an increment, not a copy: 1.0f is added to each of the nbytes / 4
 * floats at dst (4-byte aligned) -- graph mode's `Environment.steps += 1` (ref environment.py:397),
 * folded into the post-replay launch instead of a kernel node of its own.  A span with nbytes ==
 * VMAS_COPY_STORE64 stores the 8-byte value (uint64_t)src at dst (8-byte aligned): graph mode's
 * direct-output offsets for the next replay (the fused programs' out_delta words). */
#define VMAS_COPY_STORE64 (-8)
#define VMAS_COPY_MAX_SPANS 160 /* (spans travel as kernel arguments: 160 x 24 B < 4 KiB) */
typedef struct VmasCopySpan {
    const void* src;
    void* dst;
    int64_t nbytes;
} VmasCopySpan;
int32_t vmas_copy_spans(int32_t device, const VmasCopySpan* spans, int32_t n, void* stream);
/* The copies of vmas_copy_spans (at most 96 spans) and the draw of vmas_uniform_columns_snap (at
 * most 16 columns) in ONE launch: graph mode's post-replay copies together with the next step's
 * random actions drawn ahead (simulator/environment/_graph.py); the numbers and the generator
 * increment are those of vmas_uniform_columns (no reference counterpart beyond those two).
 * offset_dev (optional, v5): a device word holding the generator offset to draw at, read when the
 * launch runs (`offset` is then added to it): the offset a spawn launch earlier on the stream leaves
 * (max_accepted words at VMAS_SPAWN_OFF_END_WORD), unknown to the host when it queues the draw. */
int32_t vmas_copy_spans_draw(int32_t device, const VmasCopySpan* spans, int32_t n_spans, int64_t numel,
                             const VmasUniformColumn* cols, int32_t n_cols, uint64_t seed, uint64_t offset,
                             const uint64_t* offset_dev, int32_t mode, int64_t u_snap_delta, uint64_t* increment,
                             void* stream);
/* (round 6, no reference counterpart) The same items as vmas_copy_spans_draw run as the tail of a
 * graph replay's single fused k_world launch (csrc/vmas_tail.hpp), by its workgroups once the
 * broadphase fixed point's final pass is decided -- one launch per step instead of two.  wb: the
 * chain's write-back variant (vmas_graph_chain_set_writeback).  Returns 1 when the launch is
 * queued, 0 when the chain or the items do not admit a tail (nothing queued: launch the chain and
 * vmas_copy_spans_draw), < 0 on error.  The caller passes only copies whose sources the launch
 * writes through (k_world's state outputs, the scenario program's write-through outputs). */
int32_t vmas_graph_chain_launch_tail(const VmasKernelChain* chain, int32_t wb, const VmasCopySpan* spans,
                                     int32_t n_spans, int64_t numel, const VmasUniformColumn* cols, int32_t n_cols,
                                     uint64_t seed, uint64_t offset, const uint64_t* offset_dev, int32_t mode,
                                     int64_t u_snap_delta, uint64_t* increment, void* stream);
/* (round 6, test utility) The tail's draw alone: n_cols columns of numel elements at (seed, offset),
 * as vmas_uniform_columns draws them (its unit test compares the two bit for bit). */
int32_t vmas_test_tail_draw(int32_t device, const VmasUniformColumn* cols, int32_t n_cols, int64_t numel, uint64_t seed,
                            uint64_t offset, int32_t mode, uint64_t* increment, void* stream);

/* Error message of the last failed auxiliary call (vmas_spawn_resolve). */
const char* vmas_aux_last_error(void);

/* Gradient of one World.step (csrc/vmas_grad.hip; autograd through the step, reference
 * test_vmas.py:277-304, environment.py grad_enabled): the vector-Jacobian product.  `io` is the
 * forward's VmasStepIO (inputs; its out_* pointers are ignored); `grad_out`'s out_* pointers hold
 * the loss gradient with respect to the forward's outputs, in the forward's output layout;
 * `grad_in` receives the gradient with respect to each entity's pos [B,2] / vel [B,2] /
 * rot [B] / ang_vel [B] and each agent's force [B,2] / torque [B] (contiguous; a NULL entry is
 * skipped).  Forward-mode dual numbers through the same physics functions as the forward,
 * with the forward's batch-global broadphase mask.  device -1: host backend.  Synchronises
 * `stream`. */
typedef struct VmasGradIO {
    float* const* pos;     /* [n_entities] */
    float* const* vel;
    float* const* rot;
    float* const* ang_vel;
    float* const* force;   /* [n_agents] */
    float* const* torque;
} VmasGradIO;
int32_t vmas_world_step_vjp(const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                            const VmasPairDesc* pairs, const VmasJointDesc* joints,
                            const VmasStepIO* io, const VmasStepIO* grad_out,
                            const VmasGradIO* grad_in, void* stream);
/* Gradient of a distance query (vmas_distance's VMAS_DIST_POINT / VMAS_DIST_PAIR; core.py:1787-1904)
 * with respect to a's pos [B,2] / rot [B], b's pos / rot and the test point [B,2] (outputs may be
 * NULL), given grad_out [B].  Same dual-number method as vmas_world_step_vjp. */
int32_t vmas_distance_vjp(int32_t device, int32_t batch, int32_t kind, const VmasShapeRef* a,
                          const VmasShapeRef* b, const float* test_point, int32_t tp_s0, int32_t tp_s1,
                          const float* grad_out, float* grad_a_pos, float* grad_a_rot, float* grad_b_pos,
                          float* grad_b_rot, float* grad_point, void* stream);
/* Gradient of vmas_cast_rays (core.py:1661-1785) with respect to the origin [B,2], the angle offset
 * `rot` [B], the angles [B,R] and every target's pos [B,2] / rot [B] (host arrays of device
 * pointers, entries may be NULL), given grad_out [B,R] contiguous.  Synchronises `stream`. */
int32_t vmas_cast_rays_vjp(int32_t device, int32_t batch, int32_t n_rays, const float* origin,
                           int32_t o_s0, int32_t o_s1, const float* angles, int32_t a_s0,
                           int32_t a_s1, const float* rot, int32_t r_s0,
                           const VmasRayTarget* targets, int32_t n_targets, float max_range,
                           const float* grad_out, float* grad_origin, float* grad_rot,
                           float* grad_angles, float* const* grad_target_pos,
                           float* const* grad_target_rot, void* stream);

/* World-specialised step (csrc/vmas_jit.hip): same seam and semantics as vmas_world_create /
 * vmas_world_step (World.step, core.py:1971-2014), GPU only.  vmas_jit_world_create generates a
 * gfx950 kernel for this exact world structure (shapes, pairs and flags folded, per-wave
 * straight-line pair/entity code; parameter values are kernel arguments, see
 * vmas_jit_world_set_params) and compiles it with hipRTC (an in-process cache of the most
 * recently used code objects, keyed by the generated source, serves identical structures); it
 * returns VMAS_E_INVALID for worlds beyond its argument-block or LDS budget, in which case the
 * caller uses vmas_world_step.  With VMAS_JIT_MATH=exact (always for worlds with joints) results
 * are bit-identical to vmas_world_step. */
typedef struct VmasJitWorld VmasJitWorld;
int32_t vmas_jit_world_create(const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                              const VmasPairDesc* pairs, const VmasJointDesc* joints,
                              VmasJitWorld** out_world);
int32_t vmas_jit_world_destroy(VmasJitWorld* world);
/* With the batch broadphase the step is ONE persistent launch on `stream` that runs every
 * fixed-point pass on the device (no host wait; workgroups claim the 64-env groups per pass and
 * only ever wait for groups that running workgroups have claimed, so co-residency of the grid is
 * not assumed).  *iterations is then 0 and vmas_jit_world_passes reports the count.  A fixed
 * point that did not converge within substeps + 2 passes writes NaN over the step's outputs and
 * is returned by vmas_jit_world_passes and by the next vmas_jit_world_step. */
int32_t vmas_jit_world_step(VmasJitWorld* world, const VmasStepIO* io, void* stream,
                            int32_t* iterations);
/* New parameter VALUES for a world of the same structure (the entity attributes a scenario may
 * change between steps -- mass and inertia (ref scenarios/debug/het_mass.py:48-54 re-rolls them on
 * every reset), drag, frictions, max_speed, v_range, force / torque limits; Entity setters,
 * core.py:537-1085).  They are kernel arguments of the generated kernel, so no recompilation: the
 * next vmas_jit_world_step uses them.  Returns VMAS_E_INVALID (and changes nothing) when anything
 * else differs from the world's tables: shapes and dimensions, flags (which limits / frictions /
 * gravity apply), slots, pairs, joints, world constants and the world's gravity / semidims (folded
 * into the code; the caller then creates a new world), batch, device.  A graph that captured a
 * step keeps the values it captured. */
int32_t vmas_jit_world_set_params(VmasJitWorld* world, const VmasWorldConfig* cfg,
                                  const VmasEntityDesc* entities, const VmasPairDesc* pairs,
                                  const VmasJointDesc* joints);
/* Error bits the kernel has reported so far, without waiting (VMAS_OK if none): how a launch
 * replayed from a HIP graph surfaces a device-side fixed-point failure. */
int32_t vmas_jit_world_check(VmasJitWorld* world);
/* Fixed-point passes of the last step (waits for it on its stream). */
int32_t vmas_jit_world_passes(VmasJitWorld* world, int32_t* passes);
/* Persistent grid size, returned negative (plain launches); 0: host-driven passes
 * (VMAS_JIT_GRID=persistent|host at create). */
int32_t vmas_jit_world_grid(const VmasJitWorld* world);
int32_t vmas_jit_world_set_timing(VmasJitWorld* world, int32_t enable);
int32_t vmas_jit_world_get_timing(VmasJitWorld* world, int32_t reset, double* total_ms,
                                  int64_t* launches);
/* Device timer (timing on; batch-broadphase persistent launches): the kernel itself accumulates,
 * per step, the span from workgroup 0's start to the last workgroup's exit
 * (s_memrealtime, converted with the device's wall-clock rate);
 * *clock_ghz (may be NULL) is the in-kernel shader clock (s_memtime / s_memrealtime spans).  It also times launches replayed from a HIP graph, where HIP records
 * no events.  Waits for the device.  (bench.py's roofline timer; no reference counterpart.) */
int32_t vmas_jit_world_device_timing(VmasJitWorld* world, int32_t reset, double* total_ms,
                                     int64_t* launches, double* clock_ghz);
/* Generated source of a world (length returned; copied into buf when buf != NULL). */
int32_t vmas_jit_world_source(const VmasJitWorld* world, char* buf, int64_t cap);
/* The scenario program the world's module was compiled with (VmasWorldConfig.epilogue; 0: none). */
int32_t vmas_jit_world_epilogue(const VmasJitWorld* world);
/* A scenario's per-step program launched from the world's module (kind = VmasWorldConfig.epilogue:
 * VMAS_EPILOGUE_BALANCE with a VmasBalanceIO, reference balance.py:205-262, as vmas_balance_outputs;
 * VMAS_EPILOGUE_TRANSPORT with a VmasTransportIO, transport.py:130-190, as vmas_transport_outputs):
 * the same compiled code k_world runs as its epilogue when a replayed step graph fuses k_world and
 * this launch (vmas_graph_chain_build); IEEE arithmetic, bit-identical to the library kernels. */
int32_t vmas_jit_program_outputs(VmasJitWorld* world, int32_t kind, const void* io, void* stream);
/* Generate + compile a world's kernel without a device (build checks); returns the source length. */
int32_t vmas_jit_compile_check(const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                               const VmasPairDesc* pairs, const VmasJointDesc* joints, char* buf,
                               int64_t cap);
/* Phase timestamps (s_memtime) of one workgroup from the last launch when the world was created
 * with VMAS_JIT_PROFILE=<workgroup> set: [max_substeps*4 + 2][8 waves]; returns the count. */
int32_t vmas_jit_world_profile(VmasJitWorld* world, uint64_t* out, int64_t cap);
const char* vmas_jit_last_error(void);
/* hipRTC compiles done by this process so far and the code objects held by the bounded cache
 * (at most 32, VMAS_JIT_CACHE overrides).  Test / diagnostics entry point, no reference
 * counterpart. */
int32_t vmas_jit_stats(int64_t* compiles, int64_t* cached);

#ifdef __cplusplus
}
#endif

#endif /* VMAS_MI355X_H */
