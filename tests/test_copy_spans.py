"""vmas_copy_spans (csrc/vmas_copy.hip), graph mode's post-replay launch: byte copies of every
alignment class in one launch, more spans than one launch takes (VMAS_COPY_MAX_SPANS), and
increment spans (src NULL: +1.0f on each float of dst, the folded `steps += 1`)."""
import pytest
import torch

from vectorizedmultiagentsimulator_amd import _native as N


def test_copy_span_limit_fits_the_kernel_arguments():
    assert N.VMAS_COPY_MAX_SPANS * N.COPY_SPAN_DTYPE.itemsize + 8 <= 4096


@pytest.mark.gpu
def test_copy_spans_match_torch_copies_gpu(gpu_device):
    g = torch.Generator(device="cpu").manual_seed(0)
    n = N.VMAS_COPY_MAX_SPANS + 37  # two launches
    srcs, dsts, spans = [], [], []
    for i in range(n):
        nbytes = int(torch.randint(1, 70000, (1,), generator=g))
        off = int(torch.randint(0, 4, (1,), generator=g)) if i % 3 == 0 else 0  # unaligned spans too
        src = torch.randint(0, 256, (nbytes + off,), dtype=torch.uint8, generator=g).to(gpu_device)
        dst = torch.zeros(nbytes + off, dtype=torch.uint8, device=gpu_device)
        srcs.append((src, off, nbytes))
        dsts.append(dst)
        spans.append((src.data_ptr() + off, dst.data_ptr() + off, nbytes))
    steps = torch.arange(1000, dtype=torch.float32, device=gpu_device) * 0.5
    spans.append((0, steps.data_ptr(), steps.numel() * 4))  # increment span
    N.copy_raw(0, spans, N.stream_ptr(0))
    torch.cuda.synchronize()
    for (src, off, nbytes), dst in zip(srcs, dsts):
        assert torch.equal(dst[off:off + nbytes], src[off:off + nbytes])
        assert not dst[:off].any()
    assert torch.equal(steps, torch.arange(1000, dtype=torch.float32, device=gpu_device) * 0.5 + 1.0)


@pytest.mark.gpu
def test_increment_span_needs_aligned_floats_gpu(gpu_device):
    t = torch.zeros(8, dtype=torch.float32, device=gpu_device)
    with pytest.raises(N.NativeLibraryError):
        N.copy_raw(0, [(0, t.data_ptr(), 6)], N.stream_ptr(0))  # not a whole number of floats
    with pytest.raises(N.NativeLibraryError):
        N.copy_raw(0, [(0, t.data_ptr() + 2, 8)], N.stream_ptr(0))  # not 4-byte aligned


@pytest.mark.gpu
@pytest.mark.parametrize("numel", [1000, 32768])
def test_copy_spans_draw_matches_copies_and_the_standalone_draw_gpu(gpu_device, numel):
    """vmas_copy_spans_draw (the post-replay launch with the next step's draw, on its packed 1-D
    grid: each item's own share of workgroups): copies of every alignment class and size, an
    increment span, a store span, and uniform columns equal to vmas_uniform_columns' draw at the
    same generator state -- also at an offset read from the device (offset_dev)."""
    import ctypes

    import numpy as np

    lib = N.load_library()
    g = torch.Generator(device="cpu").manual_seed(1)
    srcs, dsts, spans = [], [], []
    for i in range(60):
        nbytes = int(torch.randint(1, 300000 if i % 7 == 0 else 5000, (1,), generator=g))
        off = int(torch.randint(0, 4, (1,), generator=g)) if i % 3 == 0 else 0
        src = torch.randint(0, 256, (nbytes + off,), dtype=torch.uint8, generator=g).to(gpu_device)
        dst = torch.zeros(nbytes + off, dtype=torch.uint8, device=gpu_device)
        srcs.append((src, off, nbytes))
        dsts.append(dst)
        spans.append((src.data_ptr() + off, dst.data_ptr() + off, nbytes))
    steps = torch.arange(3000, dtype=torch.float32, device=gpu_device)
    spans.append((0, steps.data_ptr(), steps.numel() * 4))  # increment span
    word = torch.zeros(1, dtype=torch.int64, device=gpu_device)
    spans.append((0x123456789A, word.data_ptr(), N.VMAS_COPY_STORE64))  # store span
    tbl = np.zeros(len(spans), dtype=N.COPY_SPAN_DTYPE)
    for k, s in enumerate(spans):
        tbl[k] = s

    def columns(n_cols, out):
        cols = np.zeros(n_cols, dtype=N.UNIFORM_COLUMN_DTYPE)
        for k in range(n_cols):
            cols[k]["out"], cols[k]["stride"] = out[k].data_ptr(), 1
            cols[k]["from_"], cols[k]["to"] = -1.0 - 0.25 * k, 1.0 + 0.5 * k
        return cols

    n_cols, seed, offset, mode = 6, 1234, 40, 0
    got = torch.full((n_cols, numel), float("nan"), device=gpu_device)
    want = torch.full((n_cols, numel), float("nan"), device=gpu_device)
    inc, inc2 = ctypes.c_uint64(0), ctypes.c_uint64(0)
    cg, cw = columns(n_cols, got), columns(n_cols, want)
    off_dev = torch.tensor([offset], dtype=torch.int64, device=gpu_device)
    for dev_off in (False, True):
        rc = lib.vmas_copy_spans_draw(0, tbl.ctypes.data, len(spans), numel, cg.ctypes.data, n_cols, seed,
                                      0 if dev_off else offset, off_dev.data_ptr() if dev_off else None, mode, 0,
                                      ctypes.byref(inc), N.stream_ptr(0))
        assert rc == 0, lib.vmas_aux_last_error()
        assert lib.vmas_uniform_columns(0, numel, cw.ctypes.data, n_cols, seed, offset, mode, ctypes.byref(inc2),
                                        N.stream_ptr(0)) == 0
        torch.cuda.synchronize()
        assert inc.value == inc2.value
        assert torch.equal(got, want), (dev_off, (got - want).abs().max().item())
    for (src, off, nbytes), dst in zip(srcs, dsts):
        assert torch.equal(dst[off:off + nbytes], src[off:off + nbytes])
        assert not dst[:off].any()
    assert torch.equal(steps, torch.arange(3000, dtype=torch.float32, device=gpu_device) + 2.0)  # (two launches)
    assert int(word.item()) == 0x123456789A


@pytest.mark.gpu
@pytest.mark.parametrize("numel", [1000, 65536, 3_000_000])
def test_tail_draw_matches_the_standalone_draw_gpu(gpu_device, numel):
    """The post-replay tail's draw (csrc/vmas_tail.hpp: any thread computes any element from its
    philox subsequence, round and offset residue) equals vmas_uniform_columns -- itself held to
    torch's uniform_ -- bit for bit, in every mode, at every offset residue (offset % 4: rocrand's
    interleave into the next block) and over several rounds (3 M elements: q >= 4)."""
    import ctypes

    import numpy as np

    lib = N.load_library()
    n_cols = 3

    def columns(out):
        cols = np.zeros(n_cols, dtype=N.UNIFORM_COLUMN_DTYPE)
        for k in range(n_cols):
            cols[k]["out"], cols[k]["stride"] = out[k].data_ptr(), 1
            cols[k]["from_"], cols[k]["to"] = -1.0 - 0.25 * k, 1.0 + 0.5 * k
        return cols

    got = torch.full((n_cols, numel), float("nan"), device=gpu_device)
    want = torch.full((n_cols, numel), float("nan"), device=gpu_device)
    cg, cw = columns(got), columns(want)
    for mode in range(4):
        for offset in (0, 1, 2, 3, 4, 40, 4097):
            inc, inc2 = ctypes.c_uint64(0), ctypes.c_uint64(0)
            assert lib.vmas_test_tail_draw(0, cg.ctypes.data, n_cols, numel, 987654321, offset, mode, ctypes.byref(inc),
                                           N.stream_ptr(0)) == 0, lib.vmas_last_error()
            assert lib.vmas_uniform_columns(0, numel, cw.ctypes.data, n_cols, 987654321, offset, mode, ctypes.byref(inc2),
                                            N.stream_ptr(0)) == 0, lib.vmas_aux_last_error()
            torch.cuda.synchronize()
            assert inc.value == inc2.value
            assert torch.equal(got, want), (mode, offset, (got - want).abs().max().item())
