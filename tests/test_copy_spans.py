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
