// vmas_kernels.hip -- MI355X (gfx950) kernels + host backend + C ABI for the VMAS physics step.
//
// Layout of the work:
//   * one workgroup = 64 environments (one env per lane) x NW waves;
//   * the environment's entity state lives in LDS as [entity][field][lane] fp32 rows, so every
//     LDS access of a wave is 64 consecutive dwords (conflict free) and every HBM access is a
//     coalesced 256/512-B line;
//   * per substep: "pair phase" -- waves stride over the candidate pairs of a chunk (a pair is one
//     wave-uniform task: same narrowphase class for all 64 lanes, no divergence) and store
//     (force on a, torque on a, torque on b) rows in LDS; barrier; "entity phase" -- waves stride
//     over the dynamic entities, accumulate action/friction/gravity and then the pair results in
//     the reference's order (bit-identical summation order, no atomics), integrate; barrier;
//   * all substeps run inside one launch; the reference's batch-global broadphase (a pair is
//     simulated iff ANY env has it in range, core.py:2796) is honoured exactly by a fixed-point
//     iteration over a [substep][pair] activity mask (see vmas_world_step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "vmas_aux.hpp"
#include "vmas_physics.hpp"
#include "vmas_query.hpp"
#include "vmas_jit_registry.hpp"
#include "vmas_tail.hpp"
#include "vmas_uniform.hpp"

using namespace vmas;

// ------------------------------------------------------------------------------------------------
// error reporting
static thread_local std::string g_err;
static int32_t fail(int32_t code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIP_TRY(x)                                                                        \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            (void)hipGetLastError(); /* not left for the caller's next launch check */    \
            return fail(VMAS_E_HIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                              \
        }                                                                                 \
    } while (0)

// ------------------------------------------------------------------------------------------------
// host thread pool for the device == -1 backend
class Pool {
  public:
    static Pool& get() {
        static Pool p;
        return p;
    }
    int size() const { return (int)workers_.size() + 1; }
    // run fn(chunk_index) for chunk_index in [0, n)
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 1 || workers_.empty()) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        std::unique_lock<std::mutex> lk(m_);
        job_ = &fn;
        njobs_ = n;
        next_.store(0);
        done_ = 0;
        ++gen_;
        cv_.notify_all();
        lk.unlock();
        work();
        lk.lock();
        cv_done_.wait(lk, [&] { return done_ == (int)workers_.size(); });
        job_ = nullptr;
    }

  private:
    Pool() {
        int n = (int)std::thread::hardware_concurrency();
        if (const char* s = getenv("OMP_NUM_THREADS")) n = std::max(1, atoi(s));
        if (const char* s = getenv("VMAS_HOST_THREADS")) n = std::max(1, atoi(s));
        n = std::min(n, 64);
        for (int i = 0; i + 1 < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void work() {
        for (;;) {
            int i = next_.fetch_add(1);
            if (i >= njobs_) break;
            (*job_)(i);
        }
    }
    void loop() {
        long seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            lk.unlock();
            work();
            lk.lock();
            ++done_;
            cv_done_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, cv_done_;
    const std::function<void(int)>* job_ = nullptr;
    int njobs_ = 0, done_ = 0;
    long gen_ = 0;
    bool stop_ = false;
    std::atomic<int> next_{0};
};

// ------------------------------------------------------------------------------------------------
// Pinned staging ring: per-call pointer tables are copied host -> pinned slot -> device slot with
// one stream-ordered hipMemcpyAsync; slots are recycled in segments guarded by events.
namespace {
constexpr size_t kSlot = 16384;   // bytes per slot
constexpr int kSlots = 256;
constexpr int kSegs = 8;          // kSlots / kSegs slots per segment
// Uploads issued while the stream is being captured into a HIP graph get a slot of their own that
// is never recycled: the captured memcpy node re-reads its pinned source at every replay.
constexpr int kFrozen = 128;
struct Ring {
    int device = -1;
    char* host = nullptr;
    char* dev = nullptr;
    hipEvent_t ev[kSegs];
    bool ev_live[kSegs] = {};
    int next = 0;
    char* frozen_host = nullptr;
    char* frozen_dev = nullptr;
    int frozen_next = 0;
};
std::mutex g_ring_mu;
std::vector<Ring*> g_rings;

int32_t ring_upload(int device, const void* src, size_t n, hipStream_t stream, const void** out) {
    if (n > kSlot) return fail(VMAS_E_INVALID, "pointer table of %zu bytes exceeds %zu", n, kSlot);
    std::lock_guard<std::mutex> lk(g_ring_mu);
    Ring* r = nullptr;
    for (Ring* x : g_rings)
        if (x->device == device) r = x;
    if (!r) {
        r = new Ring();
        r->device = device;
        HIP_TRY(hipHostMalloc((void**)&r->host, kSlot * kSlots, hipHostMallocDefault));
        HIP_TRY(hipMalloc((void**)&r->dev, kSlot * kSlots));
        for (int i = 0; i < kSegs; ++i) HIP_TRY(hipEventCreateWithFlags(&r->ev[i], hipEventDisableTiming));
        HIP_TRY(hipHostMalloc((void**)&r->frozen_host, kSlot * kFrozen, hipHostMallocDefault));
        HIP_TRY(hipMalloc((void**)&r->frozen_dev, kSlot * kFrozen));
        g_rings.push_back(r);
    }
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(stream, &cap));
    if (cap == hipStreamCaptureStatusActive) {
        if (!r->frozen_host) return fail(VMAS_E_HIP, "graph-capture staging slots not allocated");
        if (r->frozen_next >= kFrozen) return fail(VMAS_E_NOMEM, "graph-capture staging slots exhausted (%d)", kFrozen);
        const size_t off = (size_t)r->frozen_next++ * kSlot;
        memcpy(r->frozen_host + off, src, n);
        HIP_TRY(hipMemcpyAsync(r->frozen_dev + off, r->frozen_host + off, n, hipMemcpyHostToDevice, stream));
        *out = r->frozen_dev + off;
        return VMAS_OK;
    }
    const int per = kSlots / kSegs;
    const int slot = r->next;
    const int seg = slot / per;
    if (slot % per == 0 && r->ev_live[seg]) {
        // (not counted by vmas_host_waits: a ring wrap waits for old work only, and a captured
        // step takes frozen slots instead, so it does not make a step uncapturable)
        HIP_TRY(hipEventSynchronize(r->ev[seg]));
    }
    memcpy(r->host + (size_t)slot * kSlot, src, n);
    HIP_TRY(hipMemcpyAsync(r->dev + (size_t)slot * kSlot, r->host + (size_t)slot * kSlot, n,
                           hipMemcpyHostToDevice, stream));
    if (slot % per == per - 1) {
        HIP_TRY(hipEventRecord(r->ev[seg], stream));
        r->ev_live[seg] = true;
    }
    r->next = (slot + 1) % kSlots;
    *out = r->dev + (size_t)slot * kSlot;
    return VMAS_OK;
}

int32_t use_device(int device) {
    int cur = -1;
    HIP_TRY(hipGetDevice(&cur));
    if (cur != device) HIP_TRY(hipSetDevice(device));
    return VMAS_OK;
}
}  // namespace

// ------------------------------------------------------------------------------------------------
// World: static tables (host copies + device copies) and broadphase scratch.
struct VmasWorld {
    VmasWorldConfig cfg;
    std::vector<VmasEntityDesc> ed;
    std::vector<VmasPairDesc> pd;
    std::vector<VmasJointDesc> jd;
    std::vector<int32_t> dyn;         // dynamic entity indices
    std::vector<int32_t> trig_slot;   // [E], -1 = no trig row
    int n_trig = 0;
    // per-dynamic-entity contribution items ((pair << 2) | (side << 1) | torque), reference order
    std::vector<std::vector<int32_t>> items;
    // GPU launch geometry
    int nw = 8, n_chunks = 1, rs_rows = 0;
    std::vector<int32_t> chunk_p;      // [n_chunks + 1] first pair of each chunk
    std::vector<int32_t> prow;         // [P] first result row of each pair within its chunk
    std::vector<int32_t> fin;          // split pairs to finish, per (chunk, wave)
    std::vector<int32_t> fin_off;      // [n_chunks][nw + 1]
    std::vector<int32_t> contrib;      // flattened items
    std::vector<int32_t> contrib_off;  // [n_dyn][n_chunks + 1]
    std::vector<int32_t> sched;        // tasks (pair << 4) | part, LPT-balanced per (chunk, wave)
    std::vector<int32_t> sched_off;    // [n_chunks][nw + 1]
    size_t lds_state_floats = 0;       // per block, in floats (state/trig/results/acc/agent rows)
    bool global_scratch = false;
    // device allocations
    char* d_tables = nullptr;
    const VmasEntityDesc* d_ed = nullptr;
    const VmasPairDesc* d_pd = nullptr;
    const VmasJointDesc* d_jd = nullptr;
    const int32_t* d_dyn = nullptr;
    const int32_t* d_trig = nullptr;
    const int32_t* d_contrib = nullptr;
    const int32_t* d_contrib_off = nullptr;
    const int32_t* d_sched = nullptr;
    const int32_t* d_sched_off = nullptr;
    const int32_t* d_prow = nullptr;
    const int32_t* d_fin = nullptr;
    const int32_t* d_fin_off = nullptr;
    uint32_t* d_mask = nullptr;     // [max_substeps][W]
    uint32_t* d_blk = nullptr;       // [nblk][2][max_substeps][W]
    uint32_t* d_viol = nullptr;      // 1 word
    uint32_t* h_viol = nullptr;      // pinned
    float* d_scratch = nullptr;      // global-memory state rows when LDS is too small
    int W = 1, nblk = 0;
    // optional kernel timing (HIP events around every k_step launch, on the launch stream)
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending, ev_free;
    double timed_ms = 0.0;
    long timed_launches = 0;
};

// ------------------------------------------------------------------------------------------------
// device-side parameter block
struct StepK {
    const VmasEntityDesc* ed;
    const VmasPairDesc* pd;
    const VmasJointDesc* jd;
    const int32_t* dyn;
    const int32_t* trig;
    const int32_t* contrib;
    const int32_t* contrib_off;
    const int32_t* sched;
    const int32_t* sched_off;
    const int32_t* prow;
    const int32_t* fin;
    const int32_t* fin_off;
    const VmasEntityIO* eio;
    const VmasAgentIO* aio;
    const VmasJointIO* jio;
    float* out_pos;
    float* out_vel;
    float* out_rot;
    float* out_ang;
    float* out_force;
    float* out_torque;
    float* out_fd;  // [E][B][2] or NULL (VmasStepIO.out_fdict)
    float* out_td;  // [E][B]
    const uint32_t* mask;
    uint32_t* blk;
    float* scratch;
    int B, E, A, P, W, S, n_dyn, n_trig, rs_rows, n_chunks;
    size_t scratch_floats;
    float sdt;
    WorldK wk;
    float gx, gy, xs, ys;
    int has_g, has_xs, has_ys;
};

__device__ __forceinline__ V2 load2(const float* p, int s0, int s1, int b) {
    if (s0 == 2 && s1 == 1) {
        const float2 v = reinterpret_cast<const float2*>(p)[b];
        return mk(v.x, v.y);
    }
    return mk(p[(long)b * s0], p[(long)b * s0 + s1]);
}

// LDS (or global scratch) row accessor for the kernel
struct RowsK {
    float* SB;
    float* TR;
    const int32_t* trig;
    int lane;
    __device__ __forceinline__ V2 pos(int e) const {
        return mk(SB[(e * 6 + 0) * 64 + lane], SB[(e * 6 + 1) * 64 + lane]);
    }
    __device__ __forceinline__ float rot(int e) const { return SB[(e * 6 + 4) * 64 + lane]; }
    __device__ __forceinline__ Trig tr(int e) const {
        const int s = trig[e];
        const float* t = TR + s * 4 * 64 + lane;
        return Trig{t[0], t[64], t[128], t[192]};
    }
};

// Evaluate one candidate pair (shared by the kernel and the host backend)
template <class G>
__host__ __device__ __forceinline__ PairOut eval_pair(const VmasPairDesc& pd,
                                                      const VmasEntityDesc* ed,
                                                      const VmasJointDesc* jd, const G& g,
                                                      const WorldK& w, float fixed_rot) {
    const int ea = pd.ea, eb = pd.eb;
    switch (pd.cls) {
        case VMAS_PAIR_SS:
            return pair_ss(g.pos(ea), g.pos(eb), pd.dmin, w);
        case VMAS_PAIR_LS:
            return pair_ls(g.pos(ea), g.tr(ea), ed[ea].half_length, g.pos(eb), pd.dmin, w);
        case VMAS_PAIR_LL:
            return pair_ll(g.pos(ea), g.tr(ea), ed[ea].half_length, g.pos(eb), g.tr(eb),
                           ed[eb].half_length, pd.dmin, w);
        case VMAS_PAIR_BS:
            return pair_bs(g.pos(ea), g.tr(ea), ed[ea].half_length, ed[ea].half_width,
                           (ed[ea].flags & VMAS_F_HOLLOW) != 0, g.pos(eb), pd.dmin, w);
        case VMAS_PAIR_BL:
            return pair_bl(g.pos(ea), g.tr(ea), ed[ea].half_length, ed[ea].half_width,
                           (ed[ea].flags & VMAS_F_HOLLOW) != 0, g.pos(eb), g.tr(eb),
                           ed[eb].half_length, pd.dmin, w);
        case VMAS_PAIR_BB:
            return pair_bb(g.pos(ea), g.tr(ea), ed[ea].half_length, ed[ea].half_width,
                           (ed[ea].flags & VMAS_F_HOLLOW) != 0, g.pos(eb), g.tr(eb),
                           ed[eb].half_length, ed[eb].half_width,
                           (ed[eb].flags & VMAS_F_HOLLOW) != 0, pd.dmin, w);
        default: {  // VMAS_PAIR_JOINT
            const VmasJointDesc j = jd[pd.joint];
            return pair_joint(g.pos(ea), g.rot(ea), g.tr(ea), g.pos(eb), g.rot(eb), g.tr(eb),
                              mk(j.delta_a_x, j.delta_a_y), mk(j.delta_b_x, j.delta_b_y), j.dist,
                              j.rotate != 0, fixed_rot, w);
        }
    }
}

// (pre_forces / integrate: vmas_physics.hpp)

__device__ __forceinline__ bool mask_bit(const uint32_t* m, int W, int s, int p) {
    return (m[s * W + (p >> 5)] >> (p & 31)) & 1u;
}

// Pair-phase task = (pair << 4) | part; part kWholePair evaluates the whole narrowphase, parts
// 0..split_parts-1 one box side (box-line) or one side-vs-box test (box-box) of a split pair.
// A split pair's result rows: split_parts x (p1.x, p1.y, p2.x, p2.y), then (pa.x, pa.y, pb.x, pb.y).
constexpr int kWholePair = 15;
__host__ __device__ __forceinline__ int split_parts(int cls) { return cls == VMAS_PAIR_BL ? 4 : 8; }

// Finish step of split pair p from its rows r (this lane's column): overwrites the first four rows
// with the whole-pair result (fa.x, fa.y, ta, tb) and raises the pair's Z bit in zwords
// (out-of-range pair with a nonzero result) like the pair phase does for whole pairs.
__device__ __forceinline__ void finish_split(const StepK& k, float* r, int p, bool valid,
                                             int lane, uint32_t* zwords) {
    const VmasPairDesc pd = k.pd[p];
    const int n = split_parts(pd.cls);
    const float* ctr = r + n * 4 * 64;
    const V2 pa = mk(ctr[0], ctr[64]), pb = mk(ctr[128], ctr[192]);
    const Pts q = select_min(n, [&](int i) {
        const float* x = r + i * 4 * 64;
        return Pts{mk(x[0], x[64]), mk(x[128], x[192])};
    });
    const bool ha = (k.ed[pd.ea].flags & VMAS_F_HOLLOW) != 0;
    const bool hb = (k.ed[pd.eb].flags & VMAS_F_HOLLOW) != 0;
    const PairOut o = pd.cls == VMAS_PAIR_BL ? bl_finish(pa, ha, pb, q, pd.dmin, k.wk)
                                             : bb_finish(pa, ha, pb, hb, q, pd.dmin, k.wk);
    if (k.blk) {
        const bool nz = valid && !(norm(pa - pb) <= pd.bp_radius) &&
                        (o.fa.x != 0.f || o.fa.y != 0.f || o.ta != 0.f || o.tb != 0.f);
        const unsigned long long bal = __ballot(nz);
        if (lane == 0 && bal) atomicOr(&zwords[p >> 5], 1u << (p & 31));
    }
    r[0] = o.fa.x; r[64] = o.fa.y; r[128] = o.ta; r[192] = o.tb;
}

// ------------------------------------------------------------------------------------------------
// The fused step kernel.  kGlobalRows = false keeps every row in LDS (the pointers are then
// provably LDS and compile to ds_read/ds_write); true places the rows of big worlds in a per-block
// global scratch slab (same layout) when they exceed the LDS budget.
template <bool kGlobalRows>
__global__ void __launch_bounds__(512, 4) k_step(StepK k) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const int b = blockIdx.x * 64 + lane;
    const bool valid = b < k.B;
    const int bb = valid ? b : (k.B - 1);

    uint32_t* FL = reinterpret_cast<uint32_t*>(lds);
    const int nfl = 2 * k.S * k.W;
    float* base;
    if constexpr (kGlobalRows) base = k.scratch + (size_t)blockIdx.x * k.scratch_floats;
    else base = lds + ((nfl + 3) & ~3);
    float* SB = base;
    float* TR = SB + k.E * 6 * 64;
    float* RS = TR + k.n_trig * 4 * 64;
    float* AC = RS + k.rs_rows * 64;
    float* AF = AC + k.n_dyn * 3 * 64;
    const RowsK g{SB, TR, k.trig, lane};

    for (int i = threadIdx.x; i < nfl; i += blockDim.x) FL[i] = 0u;
    // ---- load state rows
    for (int e = wave; e < k.E; e += nw) {
        const VmasEntityIO io = k.eio[e];
        const V2 p = load2(io.pos, io.pos_s0, io.pos_s1, bb);
        const V2 v = load2(io.vel, io.vel_s0, io.vel_s1, bb);
        const float r = io.rot[(long)bb * io.rot_s0];
        const float w = io.ang_vel[(long)bb * io.ang_s0];
        float* s = SB + e * 6 * 64 + lane;
        s[0] = p.x; s[64] = p.y; s[128] = v.x; s[192] = v.y; s[256] = r; s[320] = w;
        const int ts = k.trig[e];
        if (ts >= 0) {
            const Trig t = make_trig_for(r, k.ed[e].shape == VMAS_BOX);
            float* tt = TR + ts * 4 * 64 + lane;
            tt[0] = t.c0; tt[64] = t.s0; tt[128] = t.c1; tt[192] = t.s1;
        }
    }
    for (int a = wave; a < k.A; a += nw) {
        const VmasAgentIO io = k.aio[a];
        const V2 f = load2(io.force, io.force_s0, io.force_s1, bb);
        float* s = AF + a * 3 * 64 + lane;
        s[0] = f.x; s[64] = f.y; s[128] = io.torque[(long)bb * io.torque_s0];
    }
    __syncthreads();

    for (int s = 0; s < k.S; ++s) {
        for (int c = 0; c < k.n_chunks; ++c) {
            // ---- pair phase: this wave's LPT-balanced share of the chunk's tasks (a whole pair,
            // or one part of a split box-line / box-box pair)
            const int t0 = k.sched_off[c * (nw + 1) + wave], t1 = k.sched_off[c * (nw + 1) + wave + 1];
            for (int t = t0; t < t1; ++t) {
                const int task = k.sched[t];
                const int p = task >> 4, part = task & 15;
                const VmasPairDesc pd = k.pd[p];
                float* r = RS + k.prow[p] * 64 + lane;
                const bool head = part == kWholePair || part == 0;
                bool inr = true;
                if (head && pd.cls != VMAS_PAIR_JOINT) inr = norm(g.pos(pd.ea) - g.pos(pd.eb)) <= pd.bp_radius;
                if (k.blk && head) {
                    const unsigned long long bal = __ballot(inr && valid);
                    if (lane == 0 && bal) atomicOr(&FL[s * k.W + (p >> 5)], 1u << (p & 31));
                }
                if (!mask_bit(k.mask, k.W, s, p)) continue;
                if (part != kWholePair) {
                    const VmasEntityDesc& da = k.ed[pd.ea];
                    const VmasEntityDesc& db = k.ed[pd.eb];
                    const V2 pa = g.pos(pd.ea), pb = g.pos(pd.eb);
                    const Pts q = pd.cls == VMAS_PAIR_BL
                        ? bl_part(pa, g.tr(pd.ea), da.half_length, da.half_width, pb, g.tr(pd.eb), db.half_length, part)
                        : bb_part(pa, g.tr(pd.ea), da.half_length, da.half_width, pb, g.tr(pd.eb),
                                  db.half_length, db.half_width, part);
                    float* x = r + part * 4 * 64;
                    x[0] = q.p1.x; x[64] = q.p1.y; x[128] = q.p2.x; x[192] = q.p2.y;
                    if (part == 0) {  // the finish step needs the pre-integration centres
                        float* ctr = r + split_parts(pd.cls) * 4 * 64;
                        ctr[0] = pa.x; ctr[64] = pa.y; ctr[128] = pb.x; ctr[192] = pb.y;
                    }
                    continue;
                }
                float fixed_rot = 0.f;
                if (pd.cls == VMAS_PAIR_JOINT) {
                    const VmasJointIO jio = k.jio[pd.joint];
                    fixed_rot = jio.fixed_rotation ? jio.fixed_rotation[(long)bb * jio.s0]
                                                   : k.jd[pd.joint].fixed_rotation;
                }
                const PairOut o = eval_pair(pd, k.ed, k.jd, g, k.wk, fixed_rot);
                r[0] = o.fa.x; r[64] = o.fa.y; r[128] = o.ta; r[192] = o.tb;
                if (k.blk && pd.cls != VMAS_PAIR_JOINT) {
                    const bool nz = valid && !inr &&
                                    (o.fa.x != 0.f || o.fa.y != 0.f || o.ta != 0.f || o.tb != 0.f);
                    const unsigned long long bal = __ballot(nz);
                    if (lane == 0 && bal)
                        atomicOr(&FL[(k.S + s) * k.W + (p >> 5)], 1u << (p & 31));
                }
            }
            __syncthreads();
            // ---- finish phase of the chunk's split pairs (if any)
            if (k.fin_off[c * (nw + 1) + nw] > k.fin_off[c * (nw + 1)]) {
                const int f0 = k.fin_off[c * (nw + 1) + wave], f1 = k.fin_off[c * (nw + 1) + wave + 1];
                for (int t = f0; t < f1; ++t) {
                    const int p = k.fin[t];
                    if (!mask_bit(k.mask, k.W, s, p)) continue;
                    finish_split(k, RS + k.prow[p] * 64 + lane, p, valid, lane, FL + (k.S + s) * k.W);
                }
                __syncthreads();
            }
            // ---- entity phase
            for (int i = wave; i < k.n_dyn; i += nw) {
                const int e = k.dyn[i];
                const VmasEntityDesc d = k.ed[e];
                float fx, fy, tq;
                float* acc = AC + i * 3 * 64 + lane;
                float* sb = SB + e * 6 * 64 + lane;
                if (c == 0) {
                    V2 af = mk(0.f, 0.f);
                    float at = 0.f;
                    float* afp = nullptr;
                    if (d.agent_index >= 0) {
                        afp = AF + d.agent_index * 3 * 64 + lane;
                        af = mk(afp[0], afp[64]);
                        at = afp[128];
                    }
                    V2 eg = mk(0.f, 0.f);
                    const bool has_eg = (d.flags & VMAS_F_GRAVITY) != 0;
                    if (has_eg) {
                        const VmasEntityIO io = k.eio[e];
                        eg = load2(io.gravity, io.grav_s0, io.grav_s1, bb);
                    }
                    pre_forces(d, d.agent_index >= 0, af, at, mk(sb[128], sb[192]), sb[320], eg,
                               has_eg, k.gx, k.gy, k.has_g != 0, k.sdt, fx, fy, tq);
                    if (afp) { afp[0] = af.x; afp[64] = af.y; afp[128] = at; }
                } else {
                    fx = acc[0]; fy = acc[64]; tq = acc[128];
                }
                const int j0 = k.contrib_off[i * (k.n_chunks + 1) + c];
                const int j1 = k.contrib_off[i * (k.n_chunks + 1) + c + 1];
                const bool mov = d.flags & VMAS_F_MOVABLE, rotb = d.flags & VMAS_F_ROTATABLE;
                for (int j = j0; j < j1; ++j) {
                    const int it = k.contrib[j];
                    const int p = it >> 2;
                    if (!mask_bit(k.mask, k.W, s, p)) continue;
                    const float* r = RS + k.prow[p] * 64 + lane;
                    const bool side = (it >> 1) & 1;
                    if (mov) {
                        const float rx = r[0], ry = r[64];
                        fx = fx + (side ? -rx : rx);
                        fy = fy + (side ? -ry : ry);
                    }
                    if (rotb && (it & 1)) tq = tq + (side ? r[192] : r[128]);
                }
                if (c + 1 < k.n_chunks) {
                    acc[0] = fx; acc[64] = fy; acc[128] = tq;
                } else {
                    if (k.out_fd && s == k.S - 1 && valid) {  // World.forces_dict / torques_dict
                        reinterpret_cast<float2*>(k.out_fd)[(size_t)e * k.B + b] = make_float2(fx, fy);
                        k.out_td[(size_t)e * k.B + b] = tq;
                    }
                    V2 p = mk(sb[0], sb[64]), v = mk(sb[128], sb[192]);
                    float rot = sb[256], w = sb[320];
                    integrate(d, s, k.sdt, fx, fy, tq, k.has_xs != 0, k.xs, k.has_ys != 0, k.ys,
                              p, v, rot, w);
                    sb[0] = p.x; sb[64] = p.y; sb[128] = v.x; sb[192] = v.y; sb[256] = rot; sb[320] = w;
                    const int ts = k.trig[e];
                    if (ts >= 0 && (d.flags & VMAS_F_ROTATABLE)) {
                        const Trig t = make_trig_for(rot, d.shape == VMAS_BOX);
                        float* tt = TR + ts * 4 * 64 + lane;
                        tt[0] = t.c0; tt[64] = t.s0; tt[128] = t.c1; tt[192] = t.s1;
                    }
                }
            }
            __syncthreads();
        }
    }
    // ---- write back the integrated fields into fresh tensors
    if (valid) {
        for (int i = wave; i < k.n_dyn; i += nw) {
            const int e = k.dyn[i];
            const VmasEntityDesc d = k.ed[e];
            const float* sb = SB + e * 6 * 64 + lane;
            if (d.out_lin >= 0) {
                reinterpret_cast<float2*>(k.out_pos)[(size_t)d.out_lin * k.B + b] = make_float2(sb[0], sb[64]);
                reinterpret_cast<float2*>(k.out_vel)[(size_t)d.out_lin * k.B + b] = make_float2(sb[128], sb[192]);
            }
            if (d.out_rot >= 0) {
                k.out_rot[(size_t)d.out_rot * k.B + b] = sb[256];
                k.out_ang[(size_t)d.out_rot * k.B + b] = sb[320];
            }
            if (d.agent_index >= 0) {
                const float* af = AF + d.agent_index * 3 * 64 + lane;
                if (d.out_force >= 0)
                    reinterpret_cast<float2*>(k.out_force)[(size_t)d.out_force * k.B + b] = make_float2(af[0], af[64]);
                if (d.out_torque >= 0) k.out_torque[(size_t)d.out_torque * k.B + b] = af[128];
            }
        }
    }
    if (k.blk) {
        __syncthreads();
        uint32_t* dst = k.blk + (size_t)blockIdx.x * nfl;
        for (int i = threadIdx.x; i < nfl; i += blockDim.x) dst[i] = FL[i];
    }
}

// OR the per-block activity words, decide whether the mask was a fixed point, update it if not.
// blk: [nblk][2][S][W]  (R words then Z words).  One workgroup.
__global__ void __launch_bounds__(1024) k_flags_reduce(const uint32_t* blk, int nblk, int S, int W,
                                                       uint32_t* mask, uint32_t* viol_out) {
    __shared__ uint32_t R[1024], Z[1024];
    __shared__ uint32_t viol;
    const int nwords = S * W;
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) { R[w] = 0u; Z[w] = 0u; }
    if (threadIdx.x == 0) viol = 0u;
    __syncthreads();
    // thread -> (word, block group): every thread issues independent loads for one word
    // (nwords <= 1024 = blockDim is enforced by vmas_world_create)
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
        const uint32_t m = mask[w];
        if ((m & ~R[w] & Z[w]) | (~m & R[w])) atomicOr(&viol, 1u);
    }
    __syncthreads();
    if (viol)
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) mask[w] = R[w];
    if (threadIdx.x == 0) *viol_out = viol;
}

// ------------------------------------------------------------------------------------------------
// Host backend: identical arithmetic, one environment at a time.
struct RowsH {
    const V2* P;
    const float* ROT;
    const Trig* T;
    V2 pos(int e) const { return P[e]; }
    float rot(int e) const { return ROT[e]; }
    Trig tr(int e) const { return T[e]; }
};

static inline V2 hload2(const float* p, int s0, int s1, int b) {
    return mk(p[(long)b * s0], p[(long)b * s0 + s1]);
}

static void host_step_env(const VmasWorld& W, const VmasStepIO& io, const uint32_t* mask,
                          uint32_t* R, uint32_t* Z, int b, std::vector<float>& scratch) {
    const int E = W.cfg.n_entities, A = W.cfg.n_agents, P = W.cfg.n_pairs;
    const int S = io.substeps;
    scratch.resize((size_t)E * 16 + (size_t)A * 3 + (size_t)P * 4);
    V2* pos = reinterpret_cast<V2*>(scratch.data());
    V2* vel = pos + E;
    float* rot = reinterpret_cast<float*>(vel + E);
    float* ang = rot + E;
    Trig* tr = reinterpret_cast<Trig*>(ang + E);
    float* af = reinterpret_cast<float*>(tr + E);  // [A][3]
    PairOut* res = reinterpret_cast<PairOut*>(af + A * 3);
    const WorldK wk{W.cfg.contact_margin, W.cfg.collision_force, W.cfg.joint_force,
                    W.cfg.torque_constraint_force};
    for (int e = 0; e < E; ++e) {
        const VmasEntityIO& x = io.entities[e];
        pos[e] = hload2(x.pos, x.pos_s0, x.pos_s1, b);
        vel[e] = hload2(x.vel, x.vel_s0, x.vel_s1, b);
        rot[e] = x.rot[(long)b * x.rot_s0];
        ang[e] = x.ang_vel[(long)b * x.ang_s0];
        if (W.trig_slot[e] >= 0) tr[e] = make_trig_for(rot[e], W.ed[e].shape == VMAS_BOX);
    }
    for (int a = 0; a < A; ++a) {
        const VmasAgentIO& x = io.agents[a];
        const V2 f = hload2(x.force, x.force_s0, x.force_s1, b);
        af[a * 3 + 0] = f.x;
        af[a * 3 + 1] = f.y;
        af[a * 3 + 2] = x.torque[(long)b * x.torque_s0];
    }
    const RowsH g{pos, rot, tr};
    const int Wd = W.W;
    for (int s = 0; s < S; ++s) {
        for (int p = 0; p < P; ++p) {
            const VmasPairDesc& pd = W.pd[p];
            bool inr = true;
            if (pd.cls != VMAS_PAIR_JOINT) inr = norm(pos[pd.ea] - pos[pd.eb]) <= pd.bp_radius;
            if (R && inr) R[s * Wd + (p >> 5)] |= 1u << (p & 31);
            if (!((mask[s * Wd + (p >> 5)] >> (p & 31)) & 1u)) continue;
            float fixed_rot = 0.f;
            if (pd.cls == VMAS_PAIR_JOINT) {
                const VmasJointIO* j = io.joints ? &io.joints[pd.joint] : nullptr;
                fixed_rot = (j && j->fixed_rotation) ? j->fixed_rotation[(long)b * j->s0]
                                                     : W.jd[pd.joint].fixed_rotation;
            }
            const PairOut o = eval_pair(pd, W.ed.data(), W.jd.data(), g, wk, fixed_rot);
            res[p] = o;
            if (Z && pd.cls != VMAS_PAIR_JOINT && !inr &&
                (o.fa.x != 0.f || o.fa.y != 0.f || o.ta != 0.f || o.tb != 0.f))
                Z[s * Wd + (p >> 5)] |= 1u << (p & 31);
        }
        for (size_t i = 0; i < W.dyn.size(); ++i) {
            const int e = W.dyn[i];
            const VmasEntityDesc& d = W.ed[e];
            V2 a2 = mk(0.f, 0.f);
            float at = 0.f;
            if (d.agent_index >= 0) {
                a2 = mk(af[d.agent_index * 3], af[d.agent_index * 3 + 1]);
                at = af[d.agent_index * 3 + 2];
            }
            V2 eg = mk(0.f, 0.f);
            const bool has_eg = (d.flags & VMAS_F_GRAVITY) != 0;
            if (has_eg) {
                const VmasEntityIO& x = io.entities[e];
                eg = hload2(x.gravity, x.grav_s0, x.grav_s1, b);
            }
            float fx, fy, tq;
            pre_forces(d, d.agent_index >= 0, a2, at, vel[e], ang[e], eg, has_eg,
                       W.cfg.gravity_x, W.cfg.gravity_y, W.cfg.has_world_gravity != 0, io.sub_dt,
                       fx, fy, tq);
            if (d.agent_index >= 0) {
                af[d.agent_index * 3] = a2.x;
                af[d.agent_index * 3 + 1] = a2.y;
                af[d.agent_index * 3 + 2] = at;
            }
            const bool mov = d.flags & VMAS_F_MOVABLE, rotb = d.flags & VMAS_F_ROTATABLE;
            for (int it : W.items[i]) {
                const int p = it >> 2;
                if (!((mask[s * Wd + (p >> 5)] >> (p & 31)) & 1u)) continue;
                const bool side = (it >> 1) & 1;
                if (mov) {
                    fx = fx + (side ? -res[p].fa.x : res[p].fa.x);
                    fy = fy + (side ? -res[p].fa.y : res[p].fa.y);
                }
                if (rotb && (it & 1)) tq = tq + (side ? res[p].tb : res[p].ta);
            }
            if (io.out_fdict && s == S - 1) {  // World.forces_dict / torques_dict (core.py:1975-1992)
                const size_t r = (size_t)e * W.cfg.batch + b;
                io.out_fdict[r * 2] = fx;
                io.out_fdict[r * 2 + 1] = fy;
                io.out_tdict[r] = tq;
            }
            // integration must not disturb other entities' substep-start state: stage it
            V2 p2 = pos[e], v2 = vel[e];
            float r2 = rot[e], w2 = ang[e];
            integrate(d, s, io.sub_dt, fx, fy, tq, W.cfg.has_x_semidim != 0, W.cfg.x_semidim,
                      W.cfg.has_y_semidim != 0, W.cfg.y_semidim, p2, v2, r2, w2);
            // pairs of this substep are already evaluated; entity pre-forces read only own state
            pos[e] = p2;
            vel[e] = v2;
            rot[e] = r2;
            ang[e] = w2;
            if (W.trig_slot[e] >= 0 && (d.flags & VMAS_F_ROTATABLE)) tr[e] = make_trig_for(r2, d.shape == VMAS_BOX);
        }
    }
    const int B = W.cfg.batch;
    for (size_t i = 0; i < W.dyn.size(); ++i) {
        const int e = W.dyn[i];
        const VmasEntityDesc& d = W.ed[e];
        if (d.out_lin >= 0) {
            io.out_pos[((size_t)d.out_lin * B + b) * 2] = pos[e].x;
            io.out_pos[((size_t)d.out_lin * B + b) * 2 + 1] = pos[e].y;
            io.out_vel[((size_t)d.out_lin * B + b) * 2] = vel[e].x;
            io.out_vel[((size_t)d.out_lin * B + b) * 2 + 1] = vel[e].y;
        }
        if (d.out_rot >= 0) {
            io.out_rot[(size_t)d.out_rot * B + b] = rot[e];
            io.out_ang_vel[(size_t)d.out_rot * B + b] = ang[e];
        }
        if (d.agent_index >= 0) {
            if (d.out_force >= 0) {
                io.out_force[((size_t)d.out_force * B + b) * 2] = af[d.agent_index * 3];
                io.out_force[((size_t)d.out_force * B + b) * 2 + 1] = af[d.agent_index * 3 + 1];
            }
            if (d.out_torque >= 0) io.out_torque[(size_t)d.out_torque * B + b] = af[d.agent_index * 3 + 2];
        }
    }
}

static int32_t host_step(VmasWorld& W, const VmasStepIO& io, int32_t* iterations) {
    const int B = W.cfg.batch, S = io.substeps, Wd = W.W;
    const int nwords = S * Wd;
    std::vector<uint32_t> mask(nwords, 0xFFFFFFFFu);
    const bool batch_bp = io.broadphase == VMAS_BROADPHASE_BATCH;
    Pool& pool = Pool::get();
    const int nchunks = std::min(B, pool.size() * 4);
    const int per = (B + nchunks - 1) / nchunks;
    std::vector<uint32_t> RZ((size_t)nchunks * 2 * nwords);
    const int max_it = S + 2;
    for (int it = 0; it < max_it; ++it) {
        std::fill(RZ.begin(), RZ.end(), 0u);
        pool.run(nchunks, [&](int c) {
            std::vector<float> scratch;
            uint32_t* R = batch_bp ? &RZ[(size_t)c * 2 * nwords] : nullptr;
            uint32_t* Z = batch_bp ? R + nwords : nullptr;
            const int b0 = c * per, b1 = std::min(B, b0 + per);
            for (int b = b0; b < b1; ++b) host_step_env(W, io, mask.data(), R, Z, b, scratch);
        });
        if (iterations) *iterations = it + 1;
        if (!batch_bp) return VMAS_OK;
        std::vector<uint32_t> Rt(nwords, 0u), Zt(nwords, 0u);
        for (int c = 0; c < nchunks; ++c)
            for (int w = 0; w < nwords; ++w) {
                Rt[w] |= RZ[(size_t)c * 2 * nwords + w];
                Zt[w] |= RZ[(size_t)c * 2 * nwords + nwords + w];
            }
        bool viol = false;
        for (int w = 0; w < nwords; ++w)
            if ((mask[w] & ~Rt[w] & Zt[w]) | (~mask[w] & Rt[w])) viol = true;
        if (!viol) return VMAS_OK;
        mask = Rt;
    }
    return fail(VMAS_E_NOCONVERGE, "broadphase fixed point did not converge");
}

// ------------------------------------------------------------------------------------------------
// Ray casting: one thread per (env, ray)
struct RayK {
    const VmasRayTarget* tg;
    int nt, B, R;
    const float* origin;
    int o_s0, o_s1;
    const float* ang;
    int a_s0, a_s1;
    const float* rot;
    int r_s0;
    float max_range;
    float* out;
};

__global__ void __launch_bounds__(256) k_cast_rays(RayK k) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)k.B * k.R) return;
    const int b = (int)(idx / k.R), r = (int)(idx - (long)b * k.R);
    const V2 o = mk(k.origin[(long)b * k.o_s0], k.origin[(long)b * k.o_s0 + k.o_s1]);
    float a = k.ang[(long)b * k.a_s0 + (long)r * k.a_s1];
    if (k.rot) a = a + k.rot[(long)b * k.r_s0];
    k.out[idx] = cast_one(k.tg, k.nt, o, a, b, k.max_range);
}

// ------------------------------------------------------------------------------------------------
// Distance queries: one thread per env (the per-env functions are in vmas_query.hpp)
__global__ void __launch_bounds__(256) k_distance(int B, int kind, VmasShapeRef a, VmasShapeRef bref,
                                                  const float* tp, int tp_s0, int tp_s1, void* out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    store_query(out, kind, b, distance_query(kind, a, bref, tp, tp_s0, tp_s1, b));
}

// ------------------------------------------------------------------------------------------------
// Action validation: grid (agent, slice of envs); per-block OR then one atomicOr per flag word.
__global__ void __launch_bounds__(256) k_check_actions(const VmasActionRef* refs, int B, uint32_t* flags) {
    const VmasActionRef r = refs[blockIdx.y];
    uint32_t nan_seen = 0u, out_of_range = 0u;
    const long n = (long)B * r.n_cols;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
        const int b = (int)(idx / r.n_cols), c = (int)(idx - (long)b * r.n_cols);
        const float x = r.u[(long)b * r.s0 + (long)c * r.s1];
        nan_seen |= (x != x);
        if (c < r.n_phys && !r.clamp) out_of_range |= (fabsf(x) > r.u_range[c]);
    }
    if (__any(nan_seen) && (threadIdx.x & 63) == 0) atomicOr(&flags[2 * blockIdx.y], 1u);
    if (__any(out_of_range) && (threadIdx.x & 63) == 0) atomicOr(&flags[2 * blockIdx.y + 1], 1u);
}

namespace {
struct CheckScratch {
    int device = -1;
    uint32_t* d_flags = nullptr;
    uint32_t* h_flags = nullptr;
};
std::mutex g_check_mu;
std::vector<CheckScratch*> g_checks;
}  // namespace

// ================================================================================================
// C ABI
constexpr int kChainMaxNodes = VMAS_GRAPH_CHAIN_MAX;

extern "C" {

int32_t vmas_abi_version(void) { return VMAS_ABI_VERSION; }

int32_t vmas_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* vmas_last_error(void) { return g_err.c_str(); }

// Ends a stream capture that a failed capture left open (returns 1 if one was ended, 0 if none)
// and clears the thread's last HIP error, so that the eager step that follows can launch.
int32_t vmas_stream_abort_capture(void* stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    int32_t ended = 0;
    if (st != hipStreamCaptureStatusNone) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(stream, &g);
        if (g) (void)hipGraphDestroy(g);
        ended = 1;
    }
    (void)hipGetLastError();
    return ended;
}

// Launches an instantiated graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()) on a stream
// without torch's replay prologue, whose two generator-state fill kernels serve only graphs
// that draw random numbers (graph mode checks that the step's graph does not).
int32_t vmas_graph_launch(void* graph_exec, void* stream) {
    if (!graph_exec) return fail(VMAS_E_INVALID, "vmas_graph_launch: null graph");
    const hipError_t e = hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(VMAS_E_HIP, "vmas_graph_launch: %s", hipGetErrorString(e));
    }
    return VMAS_OK;
}

// A captured step graph that is a short chain of kernel nodes, replayed as plain launches on the
// stream.  Measured on MI355X (tools/launch_gap_probe.py, profiles/r05/run7_launch_gap): a replayed
// graph costs ~5 us of GPU time more than the same kernel launched on the stream (a 20 us kernel:
// 24.9 vs 20.0 us per iteration, back to back, GPU-bound), and a stream kernel after a graph
// starts ~2.3 us later than after a stream kernel -- ~7 us of every C2 step of ~56 us.  The
// nodes' parameters (function, grid, kernel arguments) stay owned by the kept graph
// (torch.cuda.CUDAGraph(keep_graph=True)), which must outlive the chain.
struct ChainNode {
    hipFunction_t fn;
    dim3 grid, block;
    unsigned shmem;
    void** kernel_params;  // the graph node's (owned by the graph)
    void** extra;          // the graph node's, or a FusedArgs' below
};
// A k_world launch that also runs its module's scenario program as the epilogue: the node's argument
// block with Args.epi pointing at a device copy of the k_program_jit node's argument block.
struct FusedArgs {
    std::vector<char> buf;
    size_t size = 0;
    void* extra[5];
};
struct VmasKernelChain {
    int n = 0, fused = 0;
    ChainNode node[kChainMaxNodes];
    std::vector<std::unique_ptr<FusedArgs>> args;
    std::vector<void*> dev;  // device copies of the epilogue argument blocks
    // the chain's k_world launch (-1: none), its argument block (the node's, or its FusedArgs') and
    // registry entry; wb: the same block with Args.wbd set (vmas_graph_chain_set_writeback)
    int world = -1;
    const char* world_args = nullptr;
    vmas::JitFnInfo world_info{};
    std::unique_ptr<FusedArgs> wb;
    // (vmas_graph_chain_launch_tail: the argument block of the launch being queued, Args.tail set)
    mutable std::vector<char> tail_buf;
    mutable size_t tail_size = 0;
    mutable void* tail_extra[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
};

namespace {
// Device copies of chains freed since: released at the next build (a chain may be dropped while
// another stream is being captured, where hipFree is not allowed).
std::mutex g_chain_free_mu;
std::vector<void*> g_chain_free;
}  // namespace

extern "C++" {
namespace vmas {
void chain_free_drain() {
    std::lock_guard<std::mutex> lk(g_chain_free_mu);
    for (void* d : g_chain_free) (void)hipFree(d);
    g_chain_free.clear();
}
}  // namespace vmas
}

namespace {

// The argument block of a captured kernel node whose kernel takes one struct by value: from the
// node's `extra` buffer (module launches with HIP_LAUNCH_PARAM_BUFFER_POINTER) or its first
// kernel parameter.  NULL if neither holds at least `expect` bytes.
const char* node_arg_block(const hipKernelNodeParams& p, size_t expect) {
    if (p.extra) {
        const void* buf = nullptr;
        size_t sz = 0;
        for (int i = 0; i < 8 && p.extra[i] != HIP_LAUNCH_PARAM_END; i += 2) {
            if (p.extra[i] == HIP_LAUNCH_PARAM_BUFFER_POINTER) buf = p.extra[i + 1];
            else if (p.extra[i] == HIP_LAUNCH_PARAM_BUFFER_SIZE) sz = *(const size_t*)p.extra[i + 1];
            else return nullptr;
        }
        return buf && sz >= expect ? (const char*)buf : nullptr;
    }
    return p.kernelParams && p.kernelParams[0] ? (const char*)p.kernelParams[0] : nullptr;
}

// A program may run as k_world's epilogue when every per-env input it reads is a per-env row (no
// stride-0 view: a row k_world writes for one env must not be read for another).
bool balance_io_fusable(const VmasBalanceIO& io, int batch) {
    if (io.batch != batch || io.n_agents < 0 || io.n_agents > VMAS_SCN_MAX_AGENTS) return false;
    if (io.package.shape != VMAS_SPHERE || io.goal.shape != VMAS_SPHERE || io.line.shape != VMAS_LINE ||
        io.floor.shape != VMAS_BOX)
        return false;
    for (const VmasShapeRef* r : {&io.package, &io.goal, &io.line, &io.floor})
        if (!r->pos || r->pos_s0 == 0 || (r->rot && r->rot_s0 == 0)) return false;
    if ((io.what & VMAS_SCN_REWARD) && io.gs_s0 == 0) return false;
    if (io.what & VMAS_SCN_OBS) {
        for (const VmasVec* v : {&io.package_vel, &io.line_vel, &io.line_ang_vel})
            if (!v->p || v->s0 == 0) return false;
        for (int i = 0; i < io.n_agents; ++i)
            if (!io.agent_pos[i].p || io.agent_pos[i].s0 == 0 || !io.agent_vel[i].p || io.agent_vel[i].s0 == 0)
                return false;
    }
    return true;
}
bool transport_io_fusable(const VmasTransportIO& io, int batch) {
    if (io.batch != batch || io.n_agents < 0 || io.n_agents > VMAS_TRANSPORT_MAX_AGENTS || io.n_packages < 0 ||
        io.n_packages > VMAS_TRANSPORT_MAX_PACKAGES)
        return false;
    for (int i = 0; i < io.n_packages; ++i) {
        for (const VmasShapeRef* r : {&io.package[i], &io.goal[i]})
            if (!r->pos || r->pos_s0 == 0 || (r->rot && r->rot_s0 == 0)) return false;
        if (io.package[i].shape != VMAS_BOX || io.goal[i].shape != VMAS_SPHERE) return false;
        if ((io.what & VMAS_SCN_REWARD) && io.gs_s0[i] == 0) return false;
        if ((io.what & VMAS_SCN_OBS) && (!io.package_vel[i].p || io.package_vel[i].s0 == 0)) return false;
    }
    if (io.what & VMAS_SCN_OBS)
        for (int i = 0; i < io.n_agents; ++i)
            if (!io.agent_pos[i].p || io.agent_pos[i].s0 == 0 || !io.agent_vel[i].p || io.agent_vel[i].s0 == 0)
                return false;
    return true;
}
bool program_io_fusable(int kind, const char* io, int batch) {
    if (kind == VMAS_EPILOGUE_BALANCE) {
        VmasBalanceIO x;
        memcpy(&x, io, sizeof x);
        return balance_io_fusable(x, batch);
    }
    if (kind == VMAS_EPILOGUE_TRANSPORT) {
        VmasTransportIO x;
        memcpy(&x, io, sizeof x);
        return transport_io_fusable(x, batch);
    }
    return false;
}
}  // namespace

int32_t vmas_graph_chain_build(void* graph_, int32_t max_nodes, VmasKernelChain** out) {
    if (!graph_ || !out) return fail(VMAS_E_INVALID, "vmas_graph_chain_build: null argument");
    *out = nullptr;
    vmas::chain_free_drain();
    const hipGraph_t graph = (hipGraph_t)graph_;
    max_nodes = std::min<int32_t>(max_nodes, kChainMaxNodes);
    size_t n = 0;
    if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess) {
        (void)hipGetLastError();
        return fail(VMAS_E_HIP, "vmas_graph_chain_build: hipGraphGetNodes");
    }
    if (n == 0 || (int64_t)n > max_nodes) return fail(VMAS_E_UNSUPPORTED, "graph of %zu nodes (chain: 1..%d)", n, max_nodes);
    std::vector<hipGraphNode_t> nodes(n);
    if (hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) {
        (void)hipGetLastError();
        return fail(VMAS_E_HIP, "vmas_graph_chain_build: hipGraphGetNodes");
    }
    // every node a kernel node; one root, every other node with exactly one dependency and every
    // node with at most one dependent: a chain, walked from the root
    std::vector<hipGraphNode_t> dep(n, nullptr);
    int root = -1;
    for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess || t != hipGraphNodeTypeKernel) {
            (void)hipGetLastError();
            return fail(VMAS_E_UNSUPPORTED, "graph node %zu is not a kernel node", i);
        }
        size_t nd = 0;
        if (hipGraphNodeGetDependencies(nodes[i], nullptr, &nd) != hipSuccess) {
            (void)hipGetLastError();
            return fail(VMAS_E_HIP, "hipGraphNodeGetDependencies");
        }
        if (nd > 1) return fail(VMAS_E_UNSUPPORTED, "graph node %zu has %zu dependencies", i, nd);
        if (nd == 1) {
            if (hipGraphNodeGetDependencies(nodes[i], &dep[i], &nd) != hipSuccess) {
                (void)hipGetLastError();
                return fail(VMAS_E_HIP, "hipGraphNodeGetDependencies");
            }
        } else {
            if (root >= 0) return fail(VMAS_E_UNSUPPORTED, "graph has more than one root");
            root = (int)i;
        }
    }
    if (root < 0) return fail(VMAS_E_UNSUPPORTED, "graph has no root");
    // the nodes in chain order, their functions resolved
    std::vector<hipKernelNodeParams> prm(n);
    std::vector<hipFunction_t> fns(n);
    std::vector<char> used(n, 0);
    int cur = root;
    for (size_t k = 0; k < n; ++k) {
        if (cur < 0 || used[cur]) return fail(VMAS_E_UNSUPPORTED, "graph is not a chain");
        used[cur] = 1;
        hipKernelNodeParams p{};
        if (hipGraphKernelNodeGetParams(nodes[cur], &p) != hipSuccess) {
            (void)hipGetLastError();
            return fail(VMAS_E_HIP, "hipGraphKernelNodeGetParams");
        }
        if (!p.func || (!p.kernelParams && !p.extra)) return fail(VMAS_E_UNSUPPORTED, "kernel node without function / arguments");
        // a registered host stub (hipLaunchKernelGGL, torch's kernels) or a world module's kernel
        hipFunction_t f = nullptr;
        if (hipGetFuncBySymbol(&f, p.func) != hipSuccess || !f) {
            (void)hipGetLastError();
            if (!vmas::jit_fn_info(p.func, nullptr)) return fail(VMAS_E_UNSUPPORTED, "kernel node %d: unknown function", (int)k);
            f = (hipFunction_t)p.func;
        }
        prm[k] = p;
        fns[k] = f;
        int next = -1;  // the node whose dependency is this one (at most one)
        for (size_t i = 0; i < n; ++i)
            if (dep[i] == nodes[cur]) {
                if (next >= 0) return fail(VMAS_E_UNSUPPORTED, "graph node has two dependents");
                next = (int)i;
            }
        if (k + 1 < n && next < 0) return fail(VMAS_E_UNSUPPORTED, "graph is not a chain");
        cur = next;
    }
    std::unique_ptr<VmasKernelChain> c(new VmasKernelChain());
    const char* fz = getenv("VMAS_GRAPH_FUSE");  // 0: no k_world epilogue (A/B)
    const bool fuse = !(fz && fz[0] == '0');
    for (size_t k = 0; k < n; ++k) {
        const hipKernelNodeParams& p = prm[k];
        ChainNode nd{fns[k], p.gridDim, p.blockDim, p.sharedMemBytes, p.kernelParams, p.extra};
        vmas::JitFnInfo a{}, b{};
        if (fuse && k + 1 < n && vmas::jit_fn_info(p.func, &a) && a.kind == vmas::kJitFnWorld && a.epi_offset >= 0 &&
            vmas::jit_fn_info(prm[k + 1].func, &b) && b.kind == vmas::kJitFnProgram && b.world == a.world) {
            const char* wa = node_arg_block(p, a.arg_bytes);
            const char* io = node_arg_block(prm[k + 1], b.io_bytes);
            if (wa && io && program_io_fusable(a.epilogue, io, a.batch)) {
                void* d = nullptr;
                if (hipMalloc(&d, b.io_bytes) != hipSuccess || hipMemcpy(d, io, b.io_bytes, hipMemcpyHostToDevice) != hipSuccess) {
                    (void)hipGetLastError();
                    if (d) (void)hipFree(d);
                    for (void* x : c->dev) (void)hipFree(x);
                    return fail(VMAS_E_HIP, "vmas_graph_chain_build: epilogue argument copy");
                }
                c->dev.push_back(d);
                std::unique_ptr<FusedArgs> fa(new FusedArgs());
                fa->buf.assign(wa, wa + a.arg_bytes);
                memcpy(fa->buf.data() + a.epi_offset, &d, sizeof d);
                fa->size = a.arg_bytes;
                fa->extra[0] = HIP_LAUNCH_PARAM_BUFFER_POINTER;
                fa->extra[1] = fa->buf.data();
                fa->extra[2] = HIP_LAUNCH_PARAM_BUFFER_SIZE;
                fa->extra[3] = &fa->size;
                fa->extra[4] = HIP_LAUNCH_PARAM_END;
                nd.fn = a.world_fn;
                nd.kernel_params = nullptr;
                nd.extra = fa->extra;
                if (c->world < 0) {
                    c->world = c->n;
                    c->world_args = fa->buf.data();
                    c->world_info = a;
                }
                c->args.push_back(std::move(fa));
                c->node[c->n++] = nd;
                ++c->fused;
                ++k;  // (the balance node runs inside this launch)
                continue;
            }
        }
        if (c->world < 0 && vmas::jit_fn_info(p.func, &a) && a.kind == vmas::kJitFnWorld) {
            const char* wa = node_arg_block(p, a.arg_bytes);
            if (wa) {
                c->world = c->n;
                c->world_args = wa;
                c->world_info = a;
            }
        }
        c->node[c->n++] = nd;
    }
    *out = c.release();
    return VMAS_OK;
}

// The state write-back variant of a chain (graph mode's rollback-free replays): the chain's k_world
// launch with Args.wbd = backup_delta, so the step also writes its integrated state into its own
// inputs (and backs them up at input + backup_delta for a re-run pass; vmas_jit.hip wb_helpers) --
// the replay then needs no post-replay carry of that state.  backup_delta 0 removes the variant.
int32_t vmas_graph_chain_set_writeback(VmasKernelChain* c, int64_t backup_delta) {
    if (!c) return fail(VMAS_E_INVALID, "vmas_graph_chain_set_writeback: null chain");
    if (backup_delta == 0) {
        c->wb.reset();
        return VMAS_OK;
    }
    if (c->world < 0 || !c->world_args || c->world_info.wbd_offset <= 0 ||
        (size_t)c->world_info.wbd_offset + 8 > c->world_info.arg_bytes)
        return fail(VMAS_E_UNSUPPORTED, "vmas_graph_chain_set_writeback: the chain has no k_world launch");
    std::unique_ptr<FusedArgs> fa(new FusedArgs());
    fa->buf.assign(c->world_args, c->world_args + c->world_info.arg_bytes);
    memcpy(fa->buf.data() + c->world_info.wbd_offset, &backup_delta, sizeof backup_delta);
    fa->size = c->world_info.arg_bytes;
    fa->extra[0] = HIP_LAUNCH_PARAM_BUFFER_POINTER;
    fa->extra[1] = fa->buf.data();
    fa->extra[2] = HIP_LAUNCH_PARAM_BUFFER_SIZE;
    fa->extra[3] = &fa->size;
    fa->extra[4] = HIP_LAUNCH_PARAM_END;
    c->wb = std::move(fa);
    return VMAS_OK;
}

static int32_t chain_launch(const VmasKernelChain* c, void* stream, bool wb) {
    if (!c || c->n <= 0) return fail(VMAS_E_INVALID, "vmas_graph_chain_launch: empty chain");
    if (wb && !c->wb) return fail(VMAS_E_INVALID, "vmas_graph_chain_launch_wb: no write-back variant");
    for (int k = 0; k < c->n; ++k) {
        const ChainNode& d = c->node[k];
        const bool w = wb && k == c->world;
        const hipError_t e = hipModuleLaunchKernel(d.fn, d.grid.x, d.grid.y, d.grid.z, d.block.x, d.block.y, d.block.z,
                                                   d.shmem, (hipStream_t)stream, w ? nullptr : d.kernel_params,
                                                   w ? c->wb->extra : d.extra);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(VMAS_E_HIP, "vmas_graph_chain_launch: node %d: %s", k, hipGetErrorString(e));
        }
    }
    return VMAS_OK;
}

int32_t vmas_graph_chain_launch(const VmasKernelChain* c, void* stream) { return chain_launch(c, stream, false); }

// The chain with its write-back variant of the k_world launch (vmas_graph_chain_set_writeback).
int32_t vmas_graph_chain_launch_wb(const VmasKernelChain* c, void* stream) { return chain_launch(c, stream, true); }

// The chain (one fused k_world launch) with the replay's post-replay work as its tail: the spans of
// vmas_copy_spans and the draw of vmas_uniform_columns_snap (the arguments of
// vmas_copy_spans_draw), run by k_world's workgroups once the fixed point's final pass is decided
// (vmas_tail.hpp).  Returns 1 when the launch is queued, 0 when this chain or these items cannot take
// the tail (nothing queued: the caller launches the chain and vmas_copy_spans_draw), < 0 on error.
// The caller admits only copies whose sources the launch writes through (vmas_tail.hpp).
int32_t vmas_graph_chain_launch_tail(const VmasKernelChain* c, int32_t wb, const VmasCopySpan* spans, int32_t n_spans,
                                     int64_t numel, const VmasUniformColumn* cols, int32_t n_cols, uint64_t seed,
                                     uint64_t offset, const uint64_t* offset_dev, int32_t mode, int64_t u_snap_delta,
                                     uint64_t* increment, void* stream) {
    if (!c || !increment || n_spans < 0 || (n_spans > 0 && !spans) || n_cols < 0 || (n_cols > 0 && !cols) || mode < 0 ||
        mode > 3)
        return fail(VMAS_E_INVALID, "vmas_graph_chain_launch_tail: bad arguments");
    *increment = 0;
    static const bool off = getenv("VMAS_GRAPH_TAIL") && getenv("VMAS_GRAPH_TAIL")[0] == '0';  // (A/B knob)
    const vmas::JitFnInfo& a = c->world_info;
    if (off || c->n != 1 || c->world != 0 || c->fused != 1 || c->args.empty() || a.tail_offset <= 0 ||
        (size_t)a.tail_offset + sizeof(VmasTail) > a.arg_bytes || n_cols > kTailCols || (wb && !c->wb))
        return 0;
    VmasTail t;
    memset(&t, 0, sizeof t);
    // (diagnostic only, VMAS_TAIL_DIAG=nocopy / nodraw: drop the copies / the draw from the tail to
    // time its parts -- the step's results are then wrong; never set outside a timing probe)
    static const char* diag = getenv("VMAS_TAIL_DIAG");
    const bool no_copy = diag && strcmp(diag, "nocopy") == 0, no_draw = diag && strcmp(diag, "nodraw") == 0;
    if (no_draw) n_cols = 0;
    int n = 0;
    for (int i = 0; i < n_spans; ++i) {
        const VmasCopySpan& sp = spans[i];
        if (sp.nbytes == 0 || (sp.nbytes > 0 && sp.src == sp.dst)) continue;
        if (no_copy && sp.src && sp.nbytes != VMAS_COPY_STORE64) continue;
        if (sp.nbytes == VMAS_COPY_STORE64) {
            if (!sp.dst || ((uintptr_t)sp.dst & 7)) return 0;
        } else if (sp.nbytes < 0 || !sp.dst || (((uintptr_t)sp.src | (uintptr_t)sp.dst | (uintptr_t)sp.nbytes) & 3)) {
            return 0;  // (copies and increments in whole 4-byte words)
        }
        if (n == kTailSpans) return 0;
        t.s[n++] = sp;
    }
    int gx = 0;
    unsigned long long inc = 0;
    if (n_cols > 0) {
        if (numel <= 0) return fail(VMAS_E_INVALID, "vmas_graph_chain_launch_tail: numel %lld", (long long)numel);
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
            (void)hipGetLastError();
            return fail(VMAS_E_HIP, "vmas_graph_chain_launch_tail: device");
        }
        static int max_blocks[64] = {0};
        if (!max_blocks[dev]) {
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
                (void)hipGetLastError();
                return fail(VMAS_E_HIP, "vmas_graph_chain_launch_tail: device properties");
            }
            max_blocks[dev] = prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / vmas_uniform::kThreads);
        }
        vmas_uniform::grid_for(numel, max_blocks[dev], &gx, &inc);  // (torch's grid: vmas_copy_spans_draw)
    }
    for (int i = 0; i < n_cols; ++i) {
        if (!cols[i].out) return fail(VMAS_E_INVALID, "vmas_graph_chain_launch_tail: null column %d", i);
        t.c[i] = cols[i];
        t.c[i].offset = offset + inc * (unsigned long long)i;
    }
    t.seed = seed;
    t.numel = numel;
    t.snap = u_snap_delta;
    t.off_dev = reinterpret_cast<const unsigned long long*>(offset_dev);
    t.n_spans = n;
    t.gx_draw = gx;
    t.mode = mode;
    t.n_items = n + n_cols;
    if (t.n_items == 0) return 0;
    // the items' units (vmas_tail.hpp): a copy's 8-byte (or 4-byte) words, an increment's floats,
    // one store word, a column's elements -- spread over every thread of the launch
    int64_t total = 0;
    for (int y = 0; y < n; ++y) {
        t.first[y] = (int)total;
        const VmasCopySpan& sp = t.s[y];
        const bool w8 = sp.src && ((((uintptr_t)sp.src | (uintptr_t)sp.dst | (uintptr_t)sp.nbytes) & 7) == 0);
        total += sp.nbytes == VMAS_COPY_STORE64 ? 1 : sp.nbytes / (w8 ? 8 : 4);
    }
    for (int y = n; y < n + n_cols; ++y) {
        t.first[y] = (int)total;
        total += numel;
    }
    if (total >= (int64_t)1 << 30) return 0;
    t.first[n + n_cols] = (int)total;
    const FusedArgs* base = wb ? c->wb.get() : c->args.front().get();
    c->tail_buf.assign(base->buf.begin(), base->buf.begin() + a.arg_bytes);
    memcpy(c->tail_buf.data() + a.tail_offset, &t, sizeof t);
    c->tail_size = a.arg_bytes;
    c->tail_extra[0] = HIP_LAUNCH_PARAM_BUFFER_POINTER;
    c->tail_extra[1] = c->tail_buf.data();
    c->tail_extra[2] = HIP_LAUNCH_PARAM_BUFFER_SIZE;
    c->tail_extra[3] = &c->tail_size;
    c->tail_extra[4] = HIP_LAUNCH_PARAM_END;
    const ChainNode& d = c->node[0];
    const hipError_t e = hipModuleLaunchKernel(d.fn, d.grid.x, d.grid.y, d.grid.z, d.block.x, d.block.y, d.block.z,
                                               d.shmem, (hipStream_t)stream, nullptr, c->tail_extra);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(VMAS_E_HIP, "vmas_graph_chain_launch_tail: %s", hipGetErrorString(e));
    }
    *increment = inc * (unsigned long long)n_cols;
    return 1;
}

namespace {
__global__ void __launch_bounds__(256) k_test_tail(VmasTail t) { vmas_tail::run(t); }
}  // namespace

// (test utility) The tail's draw items alone (vmas_tail.hpp run / prep / finish) launched by a plain
// 1-D grid: `n_cols` columns of `numel` elements at (seed, offset), as vmas_uniform_columns draws them
// -- its unit test compares the two bit for bit at every offset residue and over several rounds.
int32_t vmas_test_tail_draw(int32_t device, const VmasUniformColumn* cols, int32_t n_cols, int64_t numel, uint64_t seed,
                            uint64_t offset, int32_t mode, uint64_t* increment, void* stream) {
    if (device < 0 || device >= 64 || !cols || n_cols < 1 || n_cols > kTailCols || numel <= 0 || !increment || mode < 0 ||
        mode > 3 || numel * n_cols >= ((int64_t)1 << 30))
        return fail(VMAS_E_INVALID, "vmas_test_tail_draw: bad arguments");
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    int gx = 0;
    unsigned long long inc = 0;
    vmas_uniform::grid_for(numel, prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / vmas_uniform::kThreads),
                           &gx, &inc);
    VmasTail t;
    memset(&t, 0, sizeof t);
    for (int i = 0; i < n_cols; ++i) {
        t.c[i] = cols[i];
        t.c[i].offset = offset + inc * (unsigned long long)i;
        t.first[i] = (int)(numel * i);
    }
    t.first[n_cols] = (int)(numel * n_cols);
    t.seed = seed;
    t.numel = numel;
    t.gx_draw = gx;
    t.mode = mode;
    t.n_items = n_cols;
    hipLaunchKernelGGL(k_test_tail, dim3(512), dim3(256), 0, (hipStream_t)stream, t);
    HIP_TRY(hipGetLastError());
    *increment = inc * (unsigned long long)n_cols;
    return VMAS_OK;
}

int32_t vmas_graph_chain_nodes(const VmasKernelChain* c) { return c ? c->n : 0; }

int32_t vmas_graph_chain_fused(const VmasKernelChain* c) { return c ? c->fused : 0; }

int32_t vmas_graph_chain_free(VmasKernelChain* c) {
    if (c && !c->dev.empty()) {
        std::lock_guard<std::mutex> lk(g_chain_free_mu);
        g_chain_free.insert(g_chain_free.end(), c->dev.begin(), c->dev.end());
    }
    delete c;
    return VMAS_OK;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int32_t vmas_world_create(const VmasWorldConfig* cfg, const VmasEntityDesc* entities,
                          const VmasPairDesc* pairs, const VmasJointDesc* joints,
                          VmasWorld** out_world) {
    if (!cfg || !out_world) return fail(VMAS_E_INVALID, "null argument");
    if (cfg->batch <= 0 || cfg->n_entities < 0 || cfg->n_pairs < 0 || cfg->n_agents < 0 ||
        cfg->n_joints < 0 || cfg->max_substeps <= 0)
        return fail(VMAS_E_INVALID, "bad world config");
    auto* W = new VmasWorld();
    W->cfg = *cfg;
    W->ed.assign(entities, entities + cfg->n_entities);
    W->pd.assign(pairs, pairs + cfg->n_pairs);
    if (cfg->n_joints) W->jd.assign(joints, joints + cfg->n_joints);
    const int E = cfg->n_entities, P = cfg->n_pairs;
    for (int p = 0; p < P; ++p) {
        const VmasPairDesc& pd = W->pd[p];
        if (pd.ea < 0 || pd.ea >= E || pd.eb < 0 || pd.eb >= E || pd.cls < 0 || pd.cls > 6 ||
            (pd.cls == VMAS_PAIR_JOINT && (pd.joint < 0 || pd.joint >= cfg->n_joints))) {
            delete W;
            return fail(VMAS_E_INVALID, "bad pair %d", p);
        }
    }
    W->trig_slot.assign(E, -1);
    auto need_trig = [&](int e) {
        if (W->trig_slot[e] < 0) W->trig_slot[e] = W->n_trig++;
    };
    for (int e = 0; e < E; ++e)
        if (W->ed[e].shape != VMAS_SPHERE) need_trig(e);
    for (int p = 0; p < P; ++p)
        if (W->pd[p].cls == VMAS_PAIR_JOINT) { need_trig(W->pd[p].ea); need_trig(W->pd[p].eb); }
    for (int e = 0; e < E; ++e)
        if (W->ed[e].flags & (VMAS_F_MOVABLE | VMAS_F_ROTATABLE)) W->dyn.push_back(e);
    // contribution lists in pair order
    W->items.resize(W->dyn.size());
    for (size_t i = 0; i < W->dyn.size(); ++i) {
        const int e = W->dyn[i];
        for (int p = 0; p < P; ++p) {
            const VmasPairDesc& pd = W->pd[p];
            for (int side = 0; side < 2; ++side) {
                if ((side ? pd.eb : pd.ea) != e) continue;
                // which side carries a torque (spheres in SS/LS/BS receive torque 0, core.py:2330-2338,2383-2391,2543-2551)
                int tq = 1;
                if (pd.cls == VMAS_PAIR_SS) tq = 0;
                if ((pd.cls == VMAS_PAIR_LS || pd.cls == VMAS_PAIR_BS) && side == 1) tq = 0;
                W->items[i].push_back((p << 2) | (side << 1) | tq);
            }
        }
    }
    W->W = std::max(1, (P + 31) / 32);
    if ((size_t)cfg->max_substeps * W->W > 1024) {
        delete W;
        return fail(VMAS_E_INVALID, "max_substeps * ceil(pairs/32) must be <= 1024");
    }
    const int B = cfg->batch;
    const int n_dyn = (int)W->dyn.size();
    if (cfg->device >= 0) {
        if (int32_t rc = use_device(cfg->device)) { delete W; return rc; }
        // launch geometry: chunk of pairs whose result rows fit the LDS budget
        W->nw = 8;
        const size_t fixed_rows = (size_t)E * 6 + (size_t)W->n_trig * 4 + (size_t)n_dyn * 3 +
                                  (size_t)cfg->n_agents * 3;
        const size_t flags_bytes = align_up((size_t)2 * cfg->max_substeps * W->W * 4, 16);
        const size_t budget = 96 * 1024;
        // static instruction-cost model per narrowphase class (box pairs are 3-35x a sphere
        // pair) and per part of a split pair
        static const float kCost[7] = {2.5f, 1.0f, 1.4f, 3.0f, 3.0f, 9.0f, 36.0f};
        auto part_cost = [](int cls) { return cls == VMAS_PAIR_BL ? 2.5f : 5.0f; };
        // Optionally split the box-line / box-box pairs across waves (VMAS_SPLIT_PAIRS=1; the
        // tests run both layouts).  Off by default: on balance (one box-line pair = 9 of 41 cost
        // units on 8 waves) the extra finish barrier cost more than the shorter pair phase saved
        // (k_step 112 -> 128 us, SQ_WAIT_ANY +16 %; profiles/r01/run4).
        bool split = false;
        if (const char* env = getenv("VMAS_SPLIT_PAIRS")) split = env[0] == '1';
        auto is_split = [&](int p) {
            return split && (W->pd[p].cls == VMAS_PAIR_BL || W->pd[p].cls == VMAS_PAIR_BB);
        };
        auto rows_of = [&](int p) { return is_split(p) ? 4 * split_parts(W->pd[p].cls) + 4 : 4; };
        // chunks: consecutive pair ranges whose result rows fit the LDS budget
        const long room = ((long)budget - (long)flags_bytes) / 256 - (long)fixed_rows;
        const int row_budget = (int)std::max<long>(32, room);
        W->prow.assign(P, 0);
        W->chunk_p.assign(1, 0);
        W->rs_rows = 0;
        int rows = 0;
        for (int p = 0; p < P; ++p) {
            if (rows > 0 && rows + rows_of(p) > row_budget) {
                W->chunk_p.push_back(p);
                rows = 0;
            }
            W->prow[p] = rows;
            rows += rows_of(p);
            W->rs_rows = std::max(W->rs_rows, rows);
        }
        W->chunk_p.push_back(P);
        W->n_chunks = (int)W->chunk_p.size() - 1;
        W->lds_state_floats = (fixed_rows + (size_t)W->rs_rows) * 64;
        W->global_scratch = W->lds_state_floats * 4 + flags_bytes > 160 * 1024 - 1024;
        // per-(dyn entity, chunk) item ranges
        W->contrib_off.assign((size_t)n_dyn * (W->n_chunks + 1), 0);
        for (int i = 0; i < n_dyn; ++i) {
            const auto& it = W->items[i];
            size_t j = 0;
            for (int c = 0; c <= W->n_chunks; ++c) {
                const int plim = W->chunk_p[c];
                while (j < it.size() && (it[j] >> 2) < plim) ++j;
                W->contrib_off[(size_t)i * (W->n_chunks + 1) + c] = (int32_t)(W->contrib.size() + j);
            }
            W->contrib.insert(W->contrib.end(), it.begin(), it.end());
        }
        // longest-processing-time assignment of each chunk's tasks to the block's waves
        W->sched_off.assign((size_t)W->n_chunks * (W->nw + 1), 0);
        for (int c = 0; c < W->n_chunks; ++c) {
            std::vector<std::pair<int, float>> tasks;  // (task, cost)
            for (int p = W->chunk_p[c]; p < W->chunk_p[c + 1]; ++p) {
                if (is_split(p)) {
                    for (int i = 0; i < split_parts(W->pd[p].cls); ++i)
                        tasks.push_back({(p << 4) | i, part_cost(W->pd[p].cls)});
                } else {
                    tasks.push_back({(p << 4) | kWholePair, kCost[W->pd[p].cls]});
                }
            }
            std::stable_sort(tasks.begin(), tasks.end(),
                             [](const std::pair<int, float>& a, const std::pair<int, float>& b) { return a.second > b.second; });
            std::vector<std::vector<int>> per(W->nw);
            std::vector<float> load(W->nw, 0.f);
            for (const auto& t : tasks) {
                const int w = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                per[w].push_back(t.first);
                load[w] += t.second;
            }
            for (int w = 0; w < W->nw; ++w) {
                W->sched_off[(size_t)c * (W->nw + 1) + w] = (int32_t)W->sched.size();
                W->sched.insert(W->sched.end(), per[w].begin(), per[w].end());
            }
            W->sched_off[(size_t)c * (W->nw + 1) + W->nw] = (int32_t)W->sched.size();
        }
        // finish tasks of split pairs: round-robin over the waves, box-box (2 inner points) first
        W->fin_off.assign((size_t)W->n_chunks * (W->nw + 1), 0);
        for (int c = 0; c < W->n_chunks; ++c) {
            std::vector<int> order;
            for (int p = W->chunk_p[c]; p < W->chunk_p[c + 1]; ++p)
                if (is_split(p)) order.push_back(p);
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return W->pd[a].cls > W->pd[b].cls; });
            std::vector<std::vector<int>> per(W->nw);
            for (size_t i = 0; i < order.size(); ++i) per[i % W->nw].push_back(order[i]);
            for (int w = 0; w < W->nw; ++w) {
                W->fin_off[(size_t)c * (W->nw + 1) + w] = (int32_t)W->fin.size();
                W->fin.insert(W->fin.end(), per[w].begin(), per[w].end());
            }
            W->fin_off[(size_t)c * (W->nw + 1) + W->nw] = (int32_t)W->fin.size();
        }
        // one allocation for all tables
        size_t off = 0;
        const size_t o_ed = off; off = align_up(off + sizeof(VmasEntityDesc) * std::max(E, 1), 64);
        const size_t o_pd = off; off = align_up(off + sizeof(VmasPairDesc) * std::max(P, 1), 64);
        const size_t o_jd = off; off = align_up(off + sizeof(VmasJointDesc) * std::max(cfg->n_joints, 1), 64);
        const size_t o_dyn = off; off = align_up(off + 4 * std::max(n_dyn, 1), 64);
        const size_t o_trig = off; off = align_up(off + 4 * std::max(E, 1), 64);
        const size_t o_c = off; off = align_up(off + 4 * std::max<size_t>(W->contrib.size(), 1), 64);
        const size_t o_co = off; off = align_up(off + 4 * std::max<size_t>(W->contrib_off.size(), 1), 64);
        const size_t o_s = off; off = align_up(off + 4 * std::max<size_t>(W->sched.size(), 1), 64);
        const size_t o_so = off; off = align_up(off + 4 * std::max<size_t>(W->sched_off.size(), 1), 64);
        const size_t o_pr = off; off = align_up(off + 4 * std::max(P, 1), 64);
        const size_t o_f = off; off = align_up(off + 4 * std::max<size_t>(W->fin.size(), 1), 64);
        const size_t o_fo = off; off = align_up(off + 4 * W->fin_off.size(), 64);
        std::vector<char> h(off, 0);
        memcpy(h.data() + o_pr, W->prow.data(), 4 * P);
        memcpy(h.data() + o_f, W->fin.data(), 4 * W->fin.size());
        memcpy(h.data() + o_fo, W->fin_off.data(), 4 * W->fin_off.size());
        memcpy(h.data() + o_ed, W->ed.data(), sizeof(VmasEntityDesc) * E);
        memcpy(h.data() + o_pd, W->pd.data(), sizeof(VmasPairDesc) * P);
        if (cfg->n_joints) memcpy(h.data() + o_jd, W->jd.data(), sizeof(VmasJointDesc) * cfg->n_joints);
        memcpy(h.data() + o_dyn, W->dyn.data(), 4 * n_dyn);
        memcpy(h.data() + o_trig, W->trig_slot.data(), 4 * E);
        memcpy(h.data() + o_c, W->contrib.data(), 4 * W->contrib.size());
        memcpy(h.data() + o_co, W->contrib_off.data(), 4 * W->contrib_off.size());
        memcpy(h.data() + o_s, W->sched.data(), 4 * W->sched.size());
        memcpy(h.data() + o_so, W->sched_off.data(), 4 * W->sched_off.size());
        auto cleanup = [&](int32_t rc) { vmas_world_destroy(W); return rc; };
        if (hipMalloc((void**)&W->d_tables, off) != hipSuccess) return cleanup(fail(VMAS_E_NOMEM, "hipMalloc tables"));
        if (hipMemcpy(W->d_tables, h.data(), off, hipMemcpyHostToDevice) != hipSuccess)
            return cleanup(fail(VMAS_E_HIP, "hipMemcpy tables"));
        W->d_ed = (const VmasEntityDesc*)(W->d_tables + o_ed);
        W->d_pd = (const VmasPairDesc*)(W->d_tables + o_pd);
        W->d_jd = (const VmasJointDesc*)(W->d_tables + o_jd);
        W->d_dyn = (const int32_t*)(W->d_tables + o_dyn);
        W->d_trig = (const int32_t*)(W->d_tables + o_trig);
        W->d_contrib = (const int32_t*)(W->d_tables + o_c);
        W->d_contrib_off = (const int32_t*)(W->d_tables + o_co);
        W->d_sched = (const int32_t*)(W->d_tables + o_s);
        W->d_sched_off = (const int32_t*)(W->d_tables + o_so);
        W->d_prow = (const int32_t*)(W->d_tables + o_pr);
        W->d_fin = (const int32_t*)(W->d_tables + o_f);
        W->d_fin_off = (const int32_t*)(W->d_tables + o_fo);
        W->nblk = (B + 63) / 64;
        const size_t nwords = (size_t)cfg->max_substeps * W->W;
        if (hipMalloc((void**)&W->d_mask, nwords * 4) != hipSuccess ||
            hipMalloc((void**)&W->d_blk, (size_t)W->nblk * 2 * nwords * 4) != hipSuccess ||
            hipMalloc((void**)&W->d_viol, 4) != hipSuccess ||
            hipHostMalloc((void**)&W->h_viol, 4, hipHostMallocDefault) != hipSuccess)
            return cleanup(fail(VMAS_E_NOMEM, "hipMalloc broadphase scratch"));
        if (W->global_scratch) {
            if (hipMalloc((void**)&W->d_scratch, (size_t)W->nblk * W->lds_state_floats * 4) != hipSuccess)
                return cleanup(fail(VMAS_E_NOMEM, "hipMalloc state scratch"));
        }
        // allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU); harmless if refused
        (void)hipFuncSetAttribute((const void*)k_step<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipGetLastError();
    }
    *out_world = W;
    return VMAS_OK;
}

int32_t vmas_world_destroy(VmasWorld* W) {
    if (!W) return VMAS_OK;
    if (W->cfg.device >= 0) {
        use_device(W->cfg.device);
        vmas::chain_free_drain();
        if (W->d_tables) (void)hipFree(W->d_tables);
        if (W->d_mask) (void)hipFree(W->d_mask);
        if (W->d_blk) (void)hipFree(W->d_blk);
        if (W->d_viol) (void)hipFree(W->d_viol);
        if (W->h_viol) (void)hipHostFree(W->h_viol);
        if (W->d_scratch) (void)hipFree(W->d_scratch);
        for (auto& ev : W->ev_pending) { (void)hipEventDestroy(ev.first); (void)hipEventDestroy(ev.second); }
        for (auto& ev : W->ev_free) { (void)hipEventDestroy(ev.first); (void)hipEventDestroy(ev.second); }
    }
    delete W;
    return VMAS_OK;
}

int32_t vmas_world_step(VmasWorld* W, const VmasStepIO* io, void* stream_, int32_t* iterations) {
    if (!W || !io) return fail(VMAS_E_INVALID, "null argument");
    const VmasWorldConfig& cfg = W->cfg;
    if (io->substeps <= 0 || io->substeps > cfg.max_substeps)
        return fail(VMAS_E_INVALID, "substeps %d outside [1, %d]", io->substeps, cfg.max_substeps);
    if (cfg.n_entities == 0) return VMAS_OK;
    if (cfg.device < 0) return host_step(*W, *io, iterations);

    hipStream_t stream = (hipStream_t)stream_;
    if (int32_t rc = use_device(cfg.device)) return rc;
    // upload the per-call pointer tables in one slot
    const int E = cfg.n_entities, A = cfg.n_agents, J = cfg.n_joints;
    const size_t be = sizeof(VmasEntityIO) * E, ba = sizeof(VmasAgentIO) * A, bj = sizeof(VmasJointIO) * J;
    const size_t oa = align_up(be, 16), oj = align_up(oa + ba, 16), tot = std::max<size_t>(oj + bj, 16);
    char buf[kSlot];
    if (tot > kSlot) return fail(VMAS_E_INVALID, "too many entities for one pointer table");
    memcpy(buf, io->entities, be);
    if (A) memcpy(buf + oa, io->agents, ba);
    if (J) memcpy(buf + oj, io->joints, bj);
    const void* dtab = nullptr;
    if (int32_t rc = ring_upload(cfg.device, buf, tot, stream, &dtab)) return rc;

    StepK k{};
    k.ed = W->d_ed; k.pd = W->d_pd; k.jd = W->d_jd; k.dyn = W->d_dyn; k.trig = W->d_trig;
    k.contrib = W->d_contrib; k.contrib_off = W->d_contrib_off;
    k.sched = W->d_sched; k.sched_off = W->d_sched_off;
    k.prow = W->d_prow; k.fin = W->d_fin; k.fin_off = W->d_fin_off;
    k.eio = (const VmasEntityIO*)dtab;
    k.aio = (const VmasAgentIO*)((const char*)dtab + oa);
    k.jio = (const VmasJointIO*)((const char*)dtab + oj);
    k.out_pos = io->out_pos; k.out_vel = io->out_vel; k.out_rot = io->out_rot;
    k.out_ang = io->out_ang_vel; k.out_force = io->out_force; k.out_torque = io->out_torque;
    k.out_fd = io->out_fdict; k.out_td = io->out_tdict;
    k.mask = W->d_mask;
    const bool batch_bp = io->broadphase == VMAS_BROADPHASE_BATCH;
    k.blk = batch_bp ? W->d_blk : nullptr;
    k.scratch = W->global_scratch ? W->d_scratch : nullptr;
    k.scratch_floats = W->lds_state_floats;
    k.B = cfg.batch; k.E = E; k.A = A; k.P = cfg.n_pairs; k.W = W->W; k.S = io->substeps;
    k.n_dyn = (int)W->dyn.size(); k.n_trig = W->n_trig; k.rs_rows = W->rs_rows; k.n_chunks = W->n_chunks;
    k.sdt = io->sub_dt;
    k.wk = WorldK{cfg.contact_margin, cfg.collision_force, cfg.joint_force, cfg.torque_constraint_force};
    k.gx = cfg.gravity_x; k.gy = cfg.gravity_y; k.has_g = cfg.has_world_gravity;
    k.xs = cfg.x_semidim; k.ys = cfg.y_semidim; k.has_xs = cfg.has_x_semidim; k.has_ys = cfg.has_y_semidim;

    const size_t flags_bytes = align_up((size_t)2 * io->substeps * W->W * 4, 16);
    const size_t lds = flags_bytes + (W->global_scratch ? 0 : W->lds_state_floats * 4);
    const size_t nwords = (size_t)io->substeps * W->W;
    HIP_TRY(vmas_aux::fill_u32_async(W->d_mask, 0xFFFFFFFFu, nwords, stream));
    const int max_it = batch_bp ? io->substeps + 2 : 1;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(stream, &cap));
    const bool timed = W->timing && cap == hipStreamCaptureStatusNone;  // (no events inside a graph)
    for (int it = 0; it < max_it; ++it) {
        std::pair<hipEvent_t, hipEvent_t> ev{};
        if (timed) {
            if (W->ev_free.empty()) {
                HIP_TRY(hipEventCreate(&ev.first));
                HIP_TRY(hipEventCreate(&ev.second));
            } else {
                ev = W->ev_free.back();
                W->ev_free.pop_back();
            }
            HIP_TRY(hipEventRecord(ev.first, stream));
        }
        if (W->global_scratch)
            hipLaunchKernelGGL(k_step<true>, dim3(W->nblk), dim3(W->nw * 64), lds, stream, k);
        else
            hipLaunchKernelGGL(k_step<false>, dim3(W->nblk), dim3(W->nw * 64), lds, stream, k);
        HIP_TRY(hipGetLastError());
        if (timed) {
            HIP_TRY(hipEventRecord(ev.second, stream));
            W->ev_pending.push_back(ev);
        }
        if (iterations) *iterations = it + 1;
        if (!batch_bp) return VMAS_OK;
        hipLaunchKernelGGL(k_flags_reduce, dim3(1), dim3(1024), 0, stream, (const uint32_t*)W->d_blk,
                           W->nblk, io->substeps, W->W, W->d_mask, W->d_viol);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(W->h_viol, W->d_viol, 4, hipMemcpyDeviceToHost, stream));
        vmas_aux::note_host_wait();
        HIP_TRY(hipStreamSynchronize(stream));
        if (*W->h_viol == 0u) return VMAS_OK;
    }
    return fail(VMAS_E_NOCONVERGE, "broadphase fixed point did not converge");
}

int32_t vmas_world_set_timing(VmasWorld* W, int32_t enable) {
    if (!W) return fail(VMAS_E_INVALID, "null world");
    W->timing = enable != 0 && W->cfg.device >= 0;
    return VMAS_OK;
}

int32_t vmas_world_get_timing(VmasWorld* W, int32_t reset, double* total_ms, int64_t* launches) {
    if (!W) return fail(VMAS_E_INVALID, "null world");
    if (W->cfg.device >= 0) {
        if (int32_t rc = use_device(W->cfg.device)) return rc;
        for (auto& ev : W->ev_pending) {
            float ms = 0.f;
            HIP_TRY(hipEventSynchronize(ev.second));
            HIP_TRY(hipEventElapsedTime(&ms, ev.first, ev.second));
            W->timed_ms += ms;
            W->timed_launches += 1;
            W->ev_free.push_back(ev);
        }
        W->ev_pending.clear();
    }
    if (total_ms) *total_ms = W->timed_ms;
    if (launches) *launches = W->timed_launches;
    if (reset) {
        W->timed_ms = 0.0;
        W->timed_launches = 0;
    }
    return VMAS_OK;
}

int32_t vmas_cast_rays(int32_t device, int32_t batch, int32_t n_rays, const float* origin,
                       int32_t origin_s0, int32_t origin_s1, const float* angles, int32_t ang_s0,
                       int32_t ang_s1, const float* rot_offset, int32_t rot_s0,
                       const VmasRayTarget* targets, int32_t n_targets, float max_range,
                       float* out, void* stream_) {
    if (batch <= 0 || n_rays <= 0) return VMAS_OK;
    if (!origin || !angles || !out || (n_targets > 0 && !targets)) return fail(VMAS_E_INVALID, "null argument");
    RayK k{};
    k.nt = n_targets; k.B = batch; k.R = n_rays; k.origin = origin; k.o_s0 = origin_s0; k.o_s1 = origin_s1;
    k.ang = angles; k.a_s0 = ang_s0; k.a_s1 = ang_s1; k.rot = rot_offset; k.r_s0 = rot_s0;
    k.max_range = max_range; k.out = out;
    if (device < 0) {
        const long n = (long)batch * n_rays;
        Pool& pool = Pool::get();
        const int nch = (int)std::min<long>(n, pool.size() * 4);
        const long per = (n + nch - 1) / nch;
        pool.run(nch, [&](int c) {
            for (long idx = c * per; idx < std::min(n, (c + 1) * per); ++idx) {
                const int b = (int)(idx / n_rays), r = (int)(idx % n_rays);
                const V2 o = mk(origin[(long)b * origin_s0], origin[(long)b * origin_s0 + origin_s1]);
                float a = angles[(long)b * ang_s0 + (long)r * ang_s1];
                if (rot_offset) a = a + rot_offset[(long)b * rot_s0];
                out[idx] = cast_one(targets, n_targets, o, a, b, max_range);
            }
        });
        return VMAS_OK;
    }
    hipStream_t stream = (hipStream_t)stream_;
    if (int32_t rc = use_device(device)) return rc;
    const void* dt = nullptr;
    if (n_targets > 0) {
        if (int32_t rc = ring_upload(device, targets, sizeof(VmasRayTarget) * n_targets, stream, &dt)) return rc;
    }
    k.tg = (const VmasRayTarget*)dt;
    const long n = (long)batch * n_rays;
    hipLaunchKernelGGL(k_cast_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, k);
    HIP_TRY(hipGetLastError());
    return VMAS_OK;
}

int32_t vmas_check_actions(int32_t device, int32_t batch, const VmasActionRef* refs, int32_t n_refs,
                           uint8_t* flags, void* stream_) {
    if (n_refs <= 0) return VMAS_OK;
    if (!refs || !flags || n_refs > 1024) return fail(VMAS_E_INVALID, "bad action refs");
    if (device < 0) {
        for (int i = 0; i < n_refs; ++i) {
            const VmasActionRef& r = refs[i];
            bool nan_seen = false, oor = false;
            for (int b = 0; b < batch; ++b)
                for (int c = 0; c < r.n_cols; ++c) {
                    const float x = r.u[(long)b * r.s0 + (long)c * r.s1];
                    nan_seen |= (x != x);
                    if (c < r.n_phys && !r.clamp) oor |= (fabsf(x) > r.u_range[c]);
                }
            flags[2 * i] = nan_seen;
            flags[2 * i + 1] = oor;
        }
        return VMAS_OK;
    }
    hipStream_t stream = (hipStream_t)stream_;
    if (int32_t rc = use_device(device)) return rc;
    CheckScratch* cs = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_check_mu);
        for (CheckScratch* x : g_checks)
            if (x->device == device) cs = x;
        if (!cs) {
            cs = new CheckScratch();
            cs->device = device;
            HIP_TRY(hipMalloc((void**)&cs->d_flags, 2048 * 4));
            HIP_TRY(hipHostMalloc((void**)&cs->h_flags, 2048 * 4, hipHostMallocDefault));
            g_checks.push_back(cs);
        }
    }
    const void* dref = nullptr;
    if (int32_t rc = ring_upload(device, refs, sizeof(VmasActionRef) * n_refs, stream, &dref)) return rc;
    HIP_TRY(vmas_aux::fill_u32_async(cs->d_flags, 0u, 2 * (size_t)n_refs, stream));
    const long per = (long)batch * 2;
    const unsigned gx = (unsigned)std::max(1L, std::min(64L, (per + 4095) / 4096));
    hipLaunchKernelGGL(k_check_actions, dim3(gx, n_refs), dim3(256), 0, stream, (const VmasActionRef*)dref,
                       batch, cs->d_flags);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(cs->h_flags, cs->d_flags, 8 * n_refs, hipMemcpyDeviceToHost, stream));
    vmas_aux::note_host_wait();
    HIP_TRY(hipStreamSynchronize(stream));
    for (int i = 0; i < 2 * n_refs; ++i) flags[i] = cs->h_flags[i] != 0u;
    return VMAS_OK;
}

int32_t vmas_distance(int32_t device, int32_t batch, int32_t kind, const VmasShapeRef* a,
                      const VmasShapeRef* b, const float* test_point, int32_t tp_s0,
                      int32_t tp_s1, void* out, void* stream_) {
    if (batch <= 0) return VMAS_OK;
    if (!a || !out || (kind == VMAS_DIST_POINT && !test_point) || (kind != VMAS_DIST_POINT && !b))
        return fail(VMAS_E_INVALID, "null argument");
    VmasShapeRef bb{};
    if (b) bb = *b;
    if (device < 0) {
        Pool& pool = Pool::get();
        const int nch = std::min(batch, pool.size() * 4);
        const int per = (batch + nch - 1) / nch;
        pool.run(nch, [&](int c) {
            for (int i = c * per; i < std::min(batch, (c + 1) * per); ++i)
                store_query(out, kind, i, distance_query(kind, *a, bb, test_point, tp_s0, tp_s1, i));
        });
        return VMAS_OK;
    }
    hipStream_t stream = (hipStream_t)stream_;
    if (int32_t rc = use_device(device)) return rc;
    hipLaunchKernelGGL(k_distance, dim3((batch + 255) / 256), dim3(256), 0, stream, batch, kind, *a,
                       bb, test_point, tp_s0, tp_s1, out);
    HIP_TRY(hipGetLastError());
    return VMAS_OK;
}

}  // extern "C"
