// vmas_spawn.hip -- rejection-sampling resolver for ScenarioUtils.find_random_pos_for_entity
// (reference vmas/simulator/utils.py:272-319), gfx950 kernel + host backend + C ABI.
//
// The reference loop draws a full [B,1,2] proposal per try (x then y, torch uniform_), checks
// every env's current position against the occupied positions with torch.cdist, replaces the
// overlapping envs' positions with the new proposal, and stops at the first try where no env
// overlaps -- one host sync and ~10 kernels per try.  Per env, the accepted position is therefore
// the FIRST candidate that overlaps nothing (a non-overlapping position never changes again), and
// the number of tries the loop consumes is 1 if every env accepts candidate 0, else
// max_env(first accepted index) + 2.  The host side draws the candidates with the same torch
// calls (so the random numbers are the reference's), this kernel resolves a whole batch of tries
// at once, and the host rewinds the generator to exactly the reference's consumption.
//
// Distance: torch.cdist (p = 2) computes sqrt(fl(fl(d0^2) + fl(d1^2))) with d = a - b on both the
// CUDA/HIP kernel (per-dim squares, then a shuffle-reduction add) and the CPU kernel; the
// comparison `dist < min_dist` runs in fp32.  Compiled with -ffp-contract=off like the engine.
#include <hip/hip_runtime.h>

#include <rocrand/rocrand_philox4x32_10.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <string>

#include "vmas_aux.hpp"
#include "vmas_mi355x.h"

namespace vmas_aux {

namespace {
thread_local std::string g_aux_err;
}

int32_t fail(int32_t code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_aux_err = buf;
    return code;
}

const char* last_error() { return g_aux_err.c_str(); }

std::atomic<uint32_t> g_host_waits{0};
void note_host_wait() { g_host_waits.fetch_add(1u, std::memory_order_relaxed); }

int32_t wait_host_word(const uint32_t* word, uint32_t seq, hipStream_t stream) {
    note_host_wait();
    for (uint64_t i = 1;; ++i) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return VMAS_OK;
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {  // the stream drained: the store must be visible by now
                if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return VMAS_OK;
                return fail(VMAS_E_HIP, "kernel finished without publishing its result word");
            }
            if (q != hipErrorNotReady) return fail(VMAS_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

int32_t wait_host_word64(const uint64_t* word, uint32_t seq, uint64_t* value, hipStream_t stream) {
    note_host_wait();
    for (uint64_t i = 1;; ++i) {
        uint64_t v = __atomic_load_n(word, __ATOMIC_ACQUIRE);
        if ((uint32_t)(v >> 32) == seq) {
            *value = v;
            return VMAS_OK;
        }
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {
                v = __atomic_load_n(word, __ATOMIC_ACQUIRE);
                if ((uint32_t)(v >> 32) == seq) {
                    *value = v;
                    return VMAS_OK;
                }
                return fail(VMAS_E_HIP, "kernel finished without publishing its result word");
            }
            if (q != hipErrorNotReady) return fail(VMAS_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

}  // namespace vmas_aux

namespace {

std::mutex g_aux_mu;

struct SpawnArgs {
    int B, n_occ, occ_s0, occ_s1, occ_s2;
    const float* occ;
    const float* cand;  // [n_tries][2][B]: candidate k of env b = (cand[k*2B + b], cand[k*2B + B + b])
    int first_try, n_tries;
    float min_dist;
    float* pos;         // [B][2]
    int32_t* resolved;  // [B], -1 = not yet
};

__host__ __device__ inline bool overlaps(const SpawnArgs& a, int b, float x, float y) {
    bool hit = false;
    for (int j = 0; j < a.n_occ; ++j) {
        const float* o = a.occ + (long)b * a.occ_s0 + (long)j * a.occ_s1;
        const float d0 = o[0] - x, d1 = o[a.occ_s2] - y;
        const float dist = sqrtf(d0 * d0 + d1 * d1);
        hit = hit || (dist < a.min_dist);
    }
    return hit;
}

// resolve env b over this batch's candidates; returns its accepted index or -1
__host__ __device__ inline int resolve_env(const SpawnArgs& a, int b) {
    int r = a.resolved[b];
    if (r >= 0) return r;
    for (int k = 0; k < a.n_tries; ++k) {
        const float x = a.cand[(long)k * 2 * a.B + b], y = a.cand[(long)k * 2 * a.B + a.B + b];
        if (!overlaps(a, b, x, y)) {
            a.pos[2 * (long)b] = x;
            a.pos[2 * (long)b + 1] = y;
            a.resolved[b] = a.first_try + k;
            return a.first_try + k;
        }
    }
    return -1;
}

// out[0] = max accepted index over envs, out[1] = number of unresolved envs
__global__ void __launch_bounds__(256) k_spawn_resolve(SpawnArgs a, int32_t* out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int r = 0, unresolved = 0;
    if (b < a.B) {
        r = resolve_env(a, b);
        unresolved = r < 0;
    }
    // wave-level max / count, then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        r = max(r, __shfl_xor(r, off));
        unresolved += __shfl_xor(unresolved, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], r);
        if (unresolved) atomicAdd(&out[1], unresolved);
    }
}

// ---- the respawn loop of several entities, tries drawn on the device (vmas_spawn_targets) --------
constexpr int kUniformThreads = 256;  // PyTorch's distribution kernel block (vmas_actions.hip)

struct DrawGrid {
    long long step;  // threads of torch's uniform_ grid on B elements
    unsigned long long inc;
};

// Element b of torch's uniform_(lo, hi) on B floats at generator offset `off`: thread b % step of
// the distribution kernel, 4 numbers per grid-stride round (k_uniform_columns, which is probed bit
// for bit against torch: `mode` bit 0 fused (0, 1] mapping, bit 1 fused affine transform).
__device__ __forceinline__ float uniform_at(unsigned long long seed, unsigned long long off, const DrawGrid& g, int b,
                                            float lo, float hi, int mode) {
    const long long t = b % g.step, q = b / g.step;
    rocrand_state_philox4x32_10 st;
    rocrand_init(seed, (unsigned long long)t, off, &st);
    uint4 v = rocrand4(&st);
    for (long long r = 0; r < q / 4; ++r) v = rocrand4(&st);
    const int k = (int)(q % 4);
    const unsigned int u = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
    const float inv = 2.3283064e-10f;  // ROCRAND_2POW32_INV
    const float unit = (mode & 1) ? __builtin_fmaf((float)u, inv, inv) : inv + (float)u * inv;
    const float range = hi - lo;
    const float val = (mode & 2) ? __builtin_fmaf(unit, range, lo) : unit * range + lo;
    return val == hi ? lo : val;  // (0, 1] -> [lo, hi)
}

__device__ __forceinline__ bool near(float ox, float oy, float x, float y, float min_dist) {
    const float d0 = ox - x, d1 = oy - y;  // torch.cdist: sqrt(fl(fl(d0^2) + fl(d1^2)))
    return sqrtf(d0 * d0 + d1 * d1) < min_dist;
}

// Target i of the respawn loop: one thread per env.  The generator offset of its first try
// follows from the earlier targets' max accepted tries (stream order: their kernels completed).
__global__ void __launch_bounds__(64) k_spawn_target(VmasSpawnTargetsIO io, DrawGrid g, int i) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= io.batch) return;
    const unsigned long long per_try = 2ull * g.inc;
    unsigned long long off = io.offset;
    for (int j = 0; j < i; ++j) {
        const int m = io.max_accepted[j];
        off += (unsigned long long)(m == 0 ? 1 : m + 2) * per_try;
    }
    // occupied: the agents, then every other target (earlier ones already moved)
    float occ[2 * (32 + VMAS_SPAWN_MAX_TARGETS)];
    int n = 0;
    for (int a = 0; a < io.n_agents; ++a) {
        const float* p = io.agents + (long)b * io.ag_s0 + (long)a * io.ag_s1;
        occ[n++] = p[0];
        occ[n++] = p[io.ag_s2];
    }
    for (int j = 0; j < io.n_targets; ++j) {
        if (j == i) continue;
        const float* p = io.pos[j] + (long)b * io.pos_s0[j];
        occ[n++] = p[0];
        occ[n++] = p[io.pos_s1[j]];
    }
    float x = 0.f, y = 0.f;
    int k = 0;
    for (; k < VMAS_SPAWN_MAX_TRIES; ++k) {
        const unsigned long long o = off + (unsigned long long)k * per_try;
        x = uniform_at(io.seed, o, g, b, io.x_lo, io.x_hi, io.mode);
        y = uniform_at(io.seed, o + g.inc, g, b, io.y_lo, io.y_hi, io.mode);
        bool hit = false;
        for (int m = 0; m < n; m += 2) hit = hit || near(occ[m], occ[m + 1], x, y, io.min_dist);
        if (!hit) break;
    }
    if (k == VMAS_SPAWN_MAX_TRIES) {  // counted in the extra word after the per-target maxima
        atomicAdd(&io.max_accepted[io.n_targets], 1);
        return;
    }
    if (k > 0) atomicMax(&io.max_accepted[i], k);
    if (io.covered[(long)b * io.cov_s0 + (long)i * io.cov_s1]) {
        float* p = io.pos[i] + (long)b * io.pos_s0[i];
        p[0] = x;
        p[io.pos_s1[i]] = y;
    }
}

struct DevScratch {
    int32_t* d_out = nullptr;
    int32_t* h_out = nullptr;
};
DevScratch g_scratch[64];

}  // namespace

extern "C" {

const char* vmas_aux_last_error(void) { return vmas_aux::last_error(); }

int32_t vmas_host_waits(void) { return (int32_t)vmas_aux::g_host_waits.load(std::memory_order_relaxed); }

int32_t vmas_spawn_resolve(int32_t device, int32_t batch, const float* occupied, int32_t n_occ,
                           int32_t occ_s0, int32_t occ_s1, int32_t occ_s2, const float* candidates,
                           int32_t first_try, int32_t n_tries, float min_dist, float* pos,
                           int32_t* resolved, int32_t* max_accepted, int32_t* n_unresolved,
                           void* stream) {
    std::lock_guard<std::mutex> lk(g_aux_mu);
    if (batch <= 0 || n_occ < 0 || n_tries <= 0 || first_try < 0 || !candidates || !pos || !resolved ||
        !max_accepted || !n_unresolved || (n_occ > 0 && !occupied))
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_resolve: bad argument");
    SpawnArgs a{batch, n_occ, occ_s0, occ_s1, occ_s2, occupied, candidates, first_try, n_tries, min_dist,
                pos, resolved};
    if (device < 0) {
        int mx = 0, un = 0;
        for (int b = 0; b < batch; ++b) {
            const int r = resolve_env(a, b);
            if (r < 0) ++un;
            else mx = r > mx ? r : mx;
        }
        *max_accepted = mx;
        *n_unresolved = un;
        return VMAS_OK;
    }
    if (device >= 64) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_resolve: device %d", device);
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    DevScratch& s = g_scratch[device];
    if (!s.d_out) {
        VMAS_AUX_HIP(hipMalloc((void**)&s.d_out, 2 * sizeof(int32_t)));
        VMAS_AUX_HIP(hipHostMalloc((void**)&s.h_out, 2 * sizeof(int32_t), hipHostMallocDefault));
    }
    hipStream_t st = (hipStream_t)stream;
    VMAS_AUX_HIP(hipMemsetAsync(s.d_out, 0, 2 * sizeof(int32_t), st));
    hipLaunchKernelGGL(k_spawn_resolve, dim3((batch + 255) / 256), dim3(256), 0, st, a, s.d_out);
    VMAS_AUX_HIP(hipGetLastError());
    VMAS_AUX_HIP(hipMemcpyAsync(s.h_out, s.d_out, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    vmas_aux::note_host_wait();
    VMAS_AUX_HIP(hipStreamSynchronize(st));
    *max_accepted = s.h_out[0];
    *n_unresolved = s.h_out[1];
    return VMAS_OK;
}

int32_t vmas_spawn_targets(int32_t device, const VmasSpawnTargetsIO* io, uint64_t* increment, void* stream) {
    if (!io || !increment || device < 0 || device >= 64 || io->batch <= 0 || io->n_agents < 0 || io->n_agents > 32 ||
        io->n_targets < 1 || io->n_targets > VMAS_SPAWN_MAX_TARGETS || !io->covered || !io->max_accepted ||
        (io->n_agents > 0 && !io->agents) || io->mode < 0 || io->mode > 3)
        return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_targets: bad arguments");
    for (int i = 0; i < io->n_targets; ++i)
        if (!io->pos[i]) return vmas_aux::fail(VMAS_E_INVALID, "vmas_spawn_targets: null target %d", i);
    int cur = -1;
    VMAS_AUX_HIP(hipGetDevice(&cur));
    if (cur != device) VMAS_AUX_HIP(hipSetDevice(device));
    static int max_blocks[64] = {0};
    if (!max_blocks[device]) {
        hipDeviceProp_t prop;
        VMAS_AUX_HIP(hipGetDeviceProperties(&prop, device));
        max_blocks[device] = prop.multiProcessorCount * (prop.maxThreadsPerMultiProcessor / kUniformThreads);
        if (max_blocks[device] <= 0) return vmas_aux::fail(VMAS_E_HIP, "vmas_spawn_targets: device properties");
    }
    // torch's distribution-kernel grid and per-call philox increment on B elements (as
    // vmas_uniform_columns)
    const long long B = io->batch;
    const long long gx = std::min<long long>((B + kUniformThreads - 1) / kUniformThreads, max_blocks[device]);
    DrawGrid g{kUniformThreads * gx, (unsigned long long)((B - 1) / (kUniformThreads * gx * 4) + 1) * 4};
    hipStream_t st = (hipStream_t)stream;
    VMAS_AUX_HIP(hipMemsetAsync(io->max_accepted, 0, sizeof(int32_t) * (io->n_targets + 1), st));
    for (int i = 0; i < io->n_targets; ++i) {
        hipLaunchKernelGGL(k_spawn_target, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, st, *io, g, i);
        VMAS_AUX_HIP(hipGetLastError());
    }
    *increment = g.inc;
    return VMAS_OK;
}

}  // extern "C"
