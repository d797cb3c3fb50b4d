// vmas_host.cpp -- the host half of a graph-mode step in C++ (a torch extension, _vmas_host):
// the per-step work between two replays that runs no simulation code but, written in Python,
// took more host time than the GPU took for the whole step ("Graph mode: host path"):
//
//   * OutputAlloc: the fresh output tensors of a replayed step (the reference returns new tensors
//     every step, environment.py:394-412).  Per (dtype, shape) group one allocation [n, *shape]
//     split into its n tensors, the address of every member written into the post-replay copy
//     table (VmasCopySpan rows, simulator/environment/_graph.py _post_table), then ONE
//     vmas_copy_spans launch for the outputs, the carried state and the backups.
//     Direct outputs (simulator/environment/_graph.py DirectOutputs): categories a fused program
//     wrote straight into this step's fresh buffer are handed out as views of it, and the next
//     step's buffer is allocated here, its offset from the captured buffer going out in the same
//     launch (a VMAS_COPY_STORE64 row).
//   * UniformDraw: Environment.get_random_actions for continuous actions on a GPU (environment.py:
//     524-606): one [A, B, n] allocation split per agent, the column table's output addresses, one
//     vmas_uniform_columns launch at the device generator's (seed, offset) and the offset advanced
//     exactly as the reference's per-column uniform_ calls advance it.
//
// Nothing here decides anything the Python layer does not: the plans are built there (once per
// capture / table) and these objects only replay them.  The C ABI entry points are called through
// function pointers handed over from the ctypes binding (_native.py), so the extension shares the
// one loaded libvmas_mi355x.so and its state.
#include <torch/extension.h>

#include <ATen/hip/HIPGeneratorImpl.h>
#include <c10/hip/HIPStream.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "vmas_mi355x.h"

namespace py = pybind11;

namespace {

using CopySpansFn = int32_t (*)(int32_t, const VmasCopySpan*, int32_t, void*);
using UniformColumnsSnapFn = int32_t (*)(int32_t, int64_t, const VmasUniformColumn*, int32_t, uint64_t, uint64_t,
                                         int32_t, int64_t, uint64_t*, void*);
using CopySpansDrawFn = int32_t (*)(int32_t, const VmasCopySpan*, int32_t, int64_t, const VmasUniformColumn*, int32_t,
                                    uint64_t, uint64_t, const uint64_t*, int32_t, int64_t, uint64_t*, void*);
using LastErrorFn = const char* (*)(void);
using ChainLaunchFn = int32_t (*)(const void*, void*);
using ChainTailFn = int32_t (*)(const void*, int32_t, const VmasCopySpan*, int32_t, int64_t, const VmasUniformColumn*,
                                int32_t, uint64_t, uint64_t, const uint64_t*, int32_t, int64_t, uint64_t*, void*);

void* current_stream(int device) {
    return (void*)c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
}

// A tensor over `base`'s storage with its own dtype, sizes, strides and (storage) offset: what
// as_strided / select return, without a dispatcher round trip and autograd's view bookkeeping
// (~0.4 us each, tens per step: post_draw's profile).  The step's outputs are fresh
// non-differentiable tensors, as the reference's are, not views of anything a caller holds.
// VMAS_HOST_RAW_VIEWS=0: as_strided / select (an A/B knob).
bool raw_views() {
    static const bool on = !(getenv("VMAS_HOST_RAW_VIEWS") && getenv("VMAS_HOST_RAW_VIEWS")[0] == '0');
    return on;
}

at::Tensor storage_view(const at::Tensor& base, at::ScalarType dtype, at::IntArrayRef sizes, at::IntArrayRef strides,
                        int64_t offset) {
    if (!raw_views() || base.requires_grad()) return base.view(dtype).as_strided(sizes, strides, offset);
    auto impl = c10::make_intrusive<c10::TensorImpl>(c10::Storage(base.storage()), base.key_set(),
                                                     caffe2::TypeMeta::fromScalarType(dtype));
    impl->set_sizes_and_strides(sizes, strides, offset);
    return at::Tensor(std::move(impl));
}

// One (dtype, shape) group of a step's outputs: `n` tensors of `shape`, allocated as [n, *shape];
// members `contig[k]` get table row r0 + (their rank among the contiguous members).
struct Group {
    std::vector<int64_t> shape;  // [n, *shape]
    at::ScalarType dtype;
    int64_t n = 0;
    int64_t r0 = 0;
    std::vector<int64_t> row_members;  // member index of each table row r0, r0 + 1, ...
    int64_t member_bytes = 0;
    // one allocation per step (OutputAlloc::one_): this group's byte offset in it, a member's sizes
    // and (contiguous) strides
    int64_t off = 0;
    std::vector<int64_t> msizes, mstrides;
};

// One directly written category: the captured buffer's address, the buffer the next replay writes
// (box[0], a Python list shared with the graph: a rebuilt table's OutputAlloc takes over where this
// one left off) and the one after it (pending, allocated by alloc(), current after the launch:
// commit()), its members as (sizes, strides, element offset) of the category's dtype, its row.
struct Region {
    at::ScalarType dtype;
    int64_t nbytes = 0, row = 0;
    uintptr_t base = 0;
    std::vector<std::vector<int64_t>> sizes, strides;
    std::vector<int64_t> offsets;
    py::list box;
    at::Tensor pending;
    int64_t off = 0;  // (one allocation per step: the next buffer's byte offset in it)
};

class OutputAlloc {
public:
    // groups: [(sample tensor of the group's dtype, shape tuple, n, r0, [member index per row])]
    // table: the copy table (numpy, VmasCopySpan rows), kept alive here
    // regions: [(captured buffer, [buffer the next replay writes], sample tensor of the dtype, row,
    //            [(sizes, strides, element offset) per member])]
    OutputAlloc(int device, py::list groups, py::object table, int64_t table_addr, int64_t copy_fn,
                int64_t last_error_fn, py::list regions)
        : device_(device), table_(std::move(table)), tbl_((VmasCopySpan*)table_addr),
          copy_((CopySpansFn)copy_fn), last_error_((LastErrorFn)last_error_fn) {
        for (py::handle h : regions) {
            py::tuple t = h.cast<py::tuple>();
            Region r;
            at::Tensor buf = t[0].cast<at::Tensor>();
            r.base = (uintptr_t)buf.data_ptr();
            r.nbytes = buf.numel();
            r.box = t[1].cast<py::list>();
            r.dtype = t[2].cast<at::Tensor>().scalar_type();
            r.row = t[3].cast<int64_t>();
            for (py::handle m : t[4].cast<py::list>()) {
                py::tuple mt = m.cast<py::tuple>();
                r.sizes.push_back(mt[0].cast<std::vector<int64_t>>());
                r.strides.push_back(mt[1].cast<std::vector<int64_t>>());
                r.offsets.push_back(mt[2].cast<int64_t>());
            }
            regions_.push_back(std::move(r));
        }
        for (py::handle g : groups) {
            py::tuple t = g.cast<py::tuple>();
            Group gr;
            gr.dtype = t[0].cast<at::Tensor>().scalar_type();
            std::vector<int64_t> shape = t[1].cast<std::vector<int64_t>>();
            gr.n = t[2].cast<int64_t>();
            gr.r0 = t[3].cast<int64_t>();
            gr.row_members = t[4].cast<std::vector<int64_t>>();
            int64_t numel = 1;
            for (int64_t s : shape) numel *= s;
            gr.member_bytes = numel * (int64_t)c10::elementSize(gr.dtype);
            gr.shape.push_back(gr.n);
            gr.shape.insert(gr.shape.end(), shape.begin(), shape.end());
            gr.msizes = shape;
            gr.mstrides.assign(shape.size(), 1);
            for (int64_t d = (int64_t)shape.size() - 2; d >= 0; --d) gr.mstrides[d] = gr.mstrides[d + 1] * shape[d + 1];
            groups_.push_back(std::move(gr));
        }
        opts_ = at::TensorOptions().device(at::Device(at::kCUDA, (c10::DeviceIndex)device));
        // the step's fresh outputs in ONE allocation and the next direct buffers in another (two
        // caching-allocator calls per step instead of one per group and region; kept apart so that
        // a caller holding only the next step's observations does not keep this step's state and
        // info outputs alive); VMAS_HOST_ONE_ALLOC=0: one allocation each
        static const bool one = !(getenv("VMAS_HOST_ONE_ALLOC") && getenv("VMAS_HOST_ONE_ALLOC")[0] == '0');
        one_ = one;
        constexpr int64_t kAlign = 256;
        for (Group& g : groups_) {
            g.off = total_;
            total_ += (g.n * g.member_bytes + kAlign - 1) / kAlign * kAlign;
        }
        for (Region& r : regions_) {
            r.off = rtotal_;
            rtotal_ += (r.nbytes + kAlign - 1) / kAlign * kAlign;
        }
    }

    // Fresh tensors of every group (in group order, members in order), their addresses written
    // into the table's output rows; then the direct categories' members (views of the buffer the
    // replay wrote), the next buffers allocated and their offsets written into the store rows.
    std::vector<at::Tensor> alloc() {
        std::vector<at::Tensor> out;
        out.reserve(count());
        if (one_ && total_ + rtotal_ > 0) {
            at::Tensor big = at::empty({total_}, opts_.dtype(at::kByte));
            const uintptr_t b0 = (uintptr_t)big.data_ptr();
            at::Tensor rbig = rtotal_ > 0 ? at::empty({rtotal_}, opts_.dtype(at::kByte)) : at::Tensor();
            const uintptr_t r0 = rtotal_ > 0 ? (uintptr_t)rbig.data_ptr() : 0;
            for (const Group& g : groups_) {
                for (size_t r = 0; r < g.row_members.size(); ++r)
                    tbl_[g.r0 + (int64_t)r].dst = (void*)(b0 + (uintptr_t)(g.off + g.row_members[r] * g.member_bytes));
                const int64_t es = (int64_t)c10::elementSize(g.dtype), e0 = g.off / es, en = g.member_bytes / es;
                for (int64_t k = 0; k < g.n; ++k) out.push_back(storage_view(big, g.dtype, g.msizes, g.mstrides, e0 + k * en));
            }
            for (Region& r : regions_) {
                at::Tensor box = r.box[0].cast<at::Tensor>();  // (a byte tensor: its offset in bytes)
                const int64_t es = (int64_t)c10::elementSize(r.dtype), so = box.storage_offset() / es;
                for (size_t m = 0; m < r.offsets.size(); ++m)
                    out.push_back(storage_view(box, r.dtype, r.sizes[m], r.strides[m], so + r.offsets[m]));
                r.pending = rbig.narrow(0, r.off, r.nbytes);
                tbl_[r.row].src = (const void*)(r0 + (uintptr_t)r.off - r.base);
            }
            return out;
        }
        for (const Group& g : groups_) {
            at::Tensor buf = at::empty(g.shape, opts_.dtype(g.dtype));
            const uintptr_t base = (uintptr_t)buf.data_ptr();
            for (size_t r = 0; r < g.row_members.size(); ++r)
                tbl_[g.r0 + (int64_t)r].dst = (void*)(base + (uintptr_t)(g.row_members[r] * g.member_bytes));
            for (int64_t k = 0; k < g.n; ++k) out.push_back(buf.select(0, k));
        }
        for (Region& r : regions_) {
            at::Tensor typed = r.box[0].cast<at::Tensor>().view(r.dtype);
            const int64_t so = typed.storage_offset();
            for (size_t m = 0; m < r.offsets.size(); ++m)
                out.push_back(typed.as_strided(r.sizes[m], r.strides[m], so + r.offsets[m]));
            r.pending = at::empty({r.nbytes}, opts_.dtype(at::kByte));
            tbl_[r.row].src = (const void*)((uintptr_t)r.pending.data_ptr() - r.base);
        }
        return out;
    }

    // after the launch that stored the pending buffers' offsets: they are what the next replay writes
    void commit() {
        for (Region& r : regions_)
            if (r.pending.defined()) {
                r.box[0] = py::cast(r.pending);
                r.pending = at::Tensor();
            }
    }

    // One vmas_copy_spans launch of table rows [lo, hi) on the current stream.
    void launch(int64_t lo, int64_t hi) {
        if (hi <= lo) return;
        const int32_t rc = copy_(device_, tbl_ + lo, (int32_t)(hi - lo), current_stream(device_));
        if (rc != VMAS_OK) throw std::runtime_error(std::string("vmas_copy_spans failed: ") + last_error_());
    }

    // The replay's kernel chain (vmas_graph_chain_launch at chain_fn; 0: already launched) on the
    // current stream: a replay and its post-replay launch in one call from Python.
    void launch_chain(int64_t chain, int64_t chain_fn) {
        if (!chain) return;
        const int32_t rc = ((ChainLaunchFn)chain_fn)((const void*)chain, current_stream(device_));
        if (rc != VMAS_OK) throw std::runtime_error(std::string("vmas_graph_chain_launch failed: ") + last_error_());
    }

    // alloc() then the launches: rows [0, mid) and [mid, hi) as two launches when mid > 0 (outputs
    // that lie in a carry destination are copied before the carry), else [0, hi) as one.
    std::vector<at::Tensor> post(int64_t mid, int64_t hi, int64_t chain, int64_t chain_fn) {
        launch_chain(chain, chain_fn);
        std::vector<at::Tensor> out = alloc();
        if (mid > 0) {
            launch(0, mid);
            launch(mid, hi);
        } else {
            launch(0, hi);
        }
        commit();
        return out;
    }

    int64_t count() const {
        int64_t n = 0;
        for (const Group& g : groups_) n += g.n;
        for (const Region& r : regions_) n += (int64_t)r.offsets.size();
        return n;
    }

    VmasCopySpan* table() const { return tbl_; }
    const char* last_error() const { return last_error_(); }

private:
    int device_;
    py::object table_;
    VmasCopySpan* tbl_;
    CopySpansFn copy_;
    LastErrorFn last_error_;
    std::vector<Group> groups_;
    std::vector<Region> regions_;
    at::TensorOptions opts_;
    bool one_ = true;
    int64_t total_ = 0;
    int64_t rtotal_ = 0;  // (the direct regions' allocation)
};

class UniformDraw {
public:
    // n_agents tensors [B, width] of one [n_agents, B, width] allocation; column k's output is
    // out_offs[k] bytes into it (its `out` field in the column table at cols_addr)
    UniformDraw(int device, int64_t batch, int64_t n_agents, int64_t width, py::object cols, int64_t cols_addr,
                int64_t n_cols, std::vector<int64_t> out_offs, int mode, int64_t uniform_fn, int64_t last_error_fn)
        : device_(device), batch_(batch), n_agents_(n_agents), width_(width), cols_obj_(std::move(cols)),
          cols_((VmasUniformColumn*)cols_addr), n_cols_(n_cols), out_offs_(std::move(out_offs)), mode_(mode),
          uniform_((UniformColumnsSnapFn)uniform_fn), last_error_((LastErrorFn)last_error_fn) {
        if ((int64_t)out_offs_.size() != n_cols_) throw std::invalid_argument("UniformDraw: one offset per column");
        opts_ = at::TensorOptions().device(at::Device(at::kCUDA, (c10::DeviceIndex)device)).dtype(at::kFloat);
    }

    // snap_numel > 0: the pre-applied columns' previous values (the buffer of snap_numel floats at
    // snap_base that agents' actions view) are first copied into a fresh buffer, returned second
    // (vmas_uniform_columns_snap)
    std::pair<std::vector<at::Tensor>, c10::optional<at::Tensor>> draw(int64_t snap_base, int64_t snap_numel) {
        at::Tensor buf = at::empty({n_agents_, batch_, width_}, opts_);
        const uintptr_t base = (uintptr_t)buf.data_ptr();
        for (int64_t k = 0; k < n_cols_; ++k) cols_[k].out = (float*)(base + (uintptr_t)out_offs_[k]);
        c10::optional<at::Tensor> snap;
        int64_t delta = 0;
        if (snap_numel > 0) {
            snap = at::empty({snap_numel}, opts_);
            delta = (int64_t)((uintptr_t)snap->data_ptr() - (uintptr_t)snap_base);
        }
        at::Generator gen = at::cuda::detail::getDefaultCUDAGenerator((c10::DeviceIndex)device_);
        {
            // (the generator's own lock, as torch's distribution kernels take it)
            std::lock_guard<std::mutex> lock(gen.mutex());
            auto* impl = gen.get<at::CUDAGeneratorImpl>();
            const uint64_t off = impl->get_offset();
            uint64_t inc = 0;
            const int32_t rc = uniform_(device_, batch_, cols_, (int32_t)n_cols_, impl->current_seed(), off, mode_,
                                        delta, &inc, current_stream(device_));
            if (rc != VMAS_OK)
                throw std::runtime_error(std::string("vmas_uniform_columns failed: ") + last_error_());
            impl->set_offset(off + inc);
        }
        return {agents(buf), std::move(snap)};
    }

    // The draw's buffers and column table without the launch (a speculative draw merged into the
    // post-replay launch, OutputAlloc.post_draw): (per-agent tensors, snapshot, snap delta)
    std::tuple<std::vector<at::Tensor>, c10::optional<at::Tensor>, int64_t> prepare(int64_t snap_base,
                                                                                   int64_t snap_numel) {
        at::Tensor buf = at::empty({n_agents_, batch_, width_}, opts_);
        const uintptr_t base = (uintptr_t)buf.data_ptr();
        for (int64_t k = 0; k < n_cols_; ++k) cols_[k].out = (float*)(base + (uintptr_t)out_offs_[k]);
        c10::optional<at::Tensor> snap;
        int64_t delta = 0;
        if (snap_numel > 0) {
            snap = at::empty({snap_numel}, opts_);
            delta = (int64_t)((uintptr_t)snap->data_ptr() - (uintptr_t)snap_base);
        }
        return {agents(buf), std::move(snap), delta};
    }

    // the [A, B, n] buffer's per-agent [B, n] tensors
    std::vector<at::Tensor> agents(const at::Tensor& buf) const {
        std::vector<at::Tensor> out;
        out.reserve(n_agents_);
        const std::vector<int64_t> sizes{batch_, width_}, strides{width_, 1};
        for (int64_t a = 0; a < n_agents_; ++a) out.push_back(storage_view(buf, at::kFloat, sizes, strides, a * batch_ * width_));
        return out;
    }

    int device() const { return device_; }
    int64_t batch() const { return batch_; }
    const VmasUniformColumn* cols() const { return cols_; }
    int64_t n_cols() const { return n_cols_; }
    int mode() const { return mode_; }

private:
    int device_;
    int64_t batch_, n_agents_, width_;
    py::object cols_obj_;
    VmasUniformColumn* cols_;
    int64_t n_cols_;
    std::vector<int64_t> out_offs_;
    int mode_;
    UniformColumnsSnapFn uniform_;
    LastErrorFn last_error_;
    at::TensorOptions opts_;
};

// OutputAlloc.post with the next step's random actions drawn in the same launch (speculatively:
// the generator is NOT advanced here; the host hands the draw out and advances it by `increment`
// only if get_random_actions is called next at the same generator state).  Returns (outputs,
// drawn per-agent tensors, snapshot, seed, offset, increment).  off_dev (a device address, 0:
// none): the draw's generator offset is read there when the launch runs (a spawn launch earlier on
// the stream leaves it); the returned offset is then None.
// VMAS_HOST_TIMING=1 (a diagnostic): post_draw's phases timed on the host, means to stderr at exit
struct HostTiming {
    bool on = getenv("VMAS_HOST_TIMING") && getenv("VMAS_HOST_TIMING")[0] == '1';
    double ns[5] = {0, 0, 0, 0, 0};
    long calls = 0;
    ~HostTiming() {
        if (on && calls)
            fprintf(stderr, "[post_draw] %ld calls, us per call: alloc %.2f prepare %.2f launch %.2f commit %.2f tuple %.2f\n",
                    calls, ns[0] / calls / 1e3, ns[1] / calls / 1e3, ns[2] / calls / 1e3, ns[3] / calls / 1e3,
                    ns[4] / calls / 1e3);
    }
};
HostTiming g_timing;
int64_t g_tail_launches = 0;  // (post_draw calls whose launch ran the tail: tests, diagnostics)
inline double now_ns() {
    return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// chain / chain_fn: the replay's kernel chain, launched first (OutputAlloc.launch_chain; 0: none).
// tail_fn (vmas_graph_chain_launch_tail; 0: none) with wb (the chain's write-back variant): the chain's
// one fused launch also runs these copies and the draw as its tail (csrc/vmas_tail.hpp) -- the
// outputs and the draw's buffers are then prepared before that launch is queued; a chain that does
// not admit the tail falls back to the two launches.
py::tuple post_draw(OutputAlloc& oa, UniformDraw& d, int64_t mid, int64_t hi, int64_t snap_base, int64_t snap_numel,
                    int64_t copy_draw_fn, int64_t off_dev, int64_t chain, int64_t chain_fn, int64_t tail_fn,
                    int64_t wb) {
    const bool tail = tail_fn && chain && mid == 0;
    if (!tail) oa.launch_chain(chain, chain_fn);
    const bool tm = g_timing.on;
    double t0 = tm ? now_ns() : 0.0, t1 = 0.0;
    std::vector<at::Tensor> outs = oa.alloc();
    if (tm) g_timing.ns[0] += (t1 = now_ns()) - t0;
    auto [acts, snap, delta] = d.prepare(snap_base, snap_numel);
    if (tm) g_timing.ns[1] += (t0 = now_ns()) - t1;
    if (mid > 0) oa.launch(0, mid);
    const int64_t lo = mid > 0 ? mid : 0;
    at::Generator gen = at::cuda::detail::getDefaultCUDAGenerator((c10::DeviceIndex)d.device());
    uint64_t seed = 0, off = 0, inc = 0;
    {
        std::lock_guard<std::mutex> lock(gen.mutex());
        auto* impl = gen.get<at::CUDAGeneratorImpl>();
        seed = impl->current_seed();
        off = off_dev ? 0 : impl->get_offset();
    }
    int32_t rc = 0;
    if (tail) {
        rc = ((ChainTailFn)tail_fn)((const void*)chain, (int32_t)wb, oa.table() + lo, (int32_t)(hi - lo), d.batch(),
                                    d.cols(), (int32_t)d.n_cols(), seed, off, (const uint64_t*)off_dev, d.mode(), delta,
                                    &inc, current_stream(d.device()));
        if (rc < 0) throw std::runtime_error(std::string("vmas_graph_chain_launch_tail failed: ") + oa.last_error());
        if (rc == 0) oa.launch_chain(chain, chain_fn);
    }
    if (rc != 1) {
        rc = ((CopySpansDrawFn)copy_draw_fn)(d.device(), oa.table() + lo, (int32_t)(hi - lo), d.batch(), d.cols(),
                                             (int32_t)d.n_cols(), seed, off, (const uint64_t*)off_dev, d.mode(), delta,
                                             &inc, current_stream(d.device()));
        if (rc != VMAS_OK) throw std::runtime_error(std::string("vmas_copy_spans_draw failed: ") + oa.last_error());
    }
    g_tail_launches += tail && rc == 1 ? 1 : 0;
    if (tm) g_timing.ns[2] += (t1 = now_ns()) - t0;
    oa.commit();
    if (tm) g_timing.ns[3] += (t0 = now_ns()) - t1;
    py::tuple res = py::make_tuple(outs, acts, snap, seed, off_dev ? py::object(py::none()) : py::object(py::int_(off)), inc);
    if (tm) {
        g_timing.ns[4] += now_ns() - t0;
        ++g_timing.calls;
    }
    return res;
}

// (tensor._version of each, as a tuple: the version snapshots of the post-replay bookkeeping)
py::tuple versions(const std::vector<at::Tensor>& ts) {
    py::tuple out(ts.size());
    for (size_t i = 0; i < ts.size(); ++i) out[i] = py::int_((int64_t)ts[i]._version());
    return out;
}

}  // namespace

PYBIND11_MODULE(_vmas_host, m) {
    m.doc() = "Host path of a graph-mode step in C++ (csrc/vmas_host.cpp)";
    m.attr("ABI_VERSION") = VMAS_ABI_VERSION;
    py::class_<OutputAlloc>(m, "OutputAlloc")
        .def(py::init<int, py::list, py::object, int64_t, int64_t, int64_t, py::list>())
        .def("alloc", &OutputAlloc::alloc)
        .def("commit", &OutputAlloc::commit)
        .def("launch", &OutputAlloc::launch)
        .def("post", &OutputAlloc::post, py::arg("mid"), py::arg("hi"), py::arg("chain") = 0, py::arg("chain_fn") = 0)
        .def("count", &OutputAlloc::count);
    py::class_<UniformDraw>(m, "UniformDraw")
        .def(py::init<int, int64_t, int64_t, int64_t, py::object, int64_t, int64_t, std::vector<int64_t>, int, int64_t,
                      int64_t>())
        .def("draw", &UniformDraw::draw);
    m.def("post_draw", &post_draw, py::arg("oa"), py::arg("d"), py::arg("mid"), py::arg("hi"), py::arg("snap_base"),
          py::arg("snap_numel"), py::arg("copy_draw_fn"), py::arg("off_dev"), py::arg("chain") = 0,
          py::arg("chain_fn") = 0, py::arg("tail_fn") = 0, py::arg("wb") = 0);
    m.def("tail_launches", []() { return g_tail_launches; });
    m.def("versions", &versions);
}
