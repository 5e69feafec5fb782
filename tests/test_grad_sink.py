"""GradSink / _ChanSplit bookkeeping on CPU tensors (the HIP GEMMs that fill the sink on the GPU are
covered by the -m gpu gradient tests): a slice claimed twice gets no buffer, the split's backward
returns the buffer only when every slice gradient is its untouched channel range, and otherwise
assembles the gradients itself."""
import torch

from turtlevsr_amd.train import _split
from turtlevsr_amd.train_ops import GradSink

CL = torch.channels_last


def test_claim_once_per_slice_and_dtype():
    x = torch.randn(2, 12, 4, 5).contiguous(memory_format=CL)
    s = GradSink(x)
    a = s.claim(0, 8, x.dtype)
    assert a is not None and a.shape == (2, 8, 4, 5) and a.stride() == (240, 1, 60, 12)
    assert s.claim(0, 8, x.dtype) is None                 # a second consumer of the same slice
    assert s.claim(8, 4, torch.bfloat16) is None           # another dtype than the buffer's
    b = s.claim(8, 4, x.dtype)
    assert b is not None and b.data_ptr() == s.buf.data_ptr() + 8 * 4


def test_split_backward_returns_sink_buffer_when_slices_are_filled_in_place():
    x = torch.randn(2, 12, 4, 5).contiguous(memory_format=CL).requires_grad_()
    sink = GradSink(x)

    class Fill(torch.autograd.Function):          # a consumer writing its input gradient into the sink
        @staticmethod
        def forward(ctx, t, off, val):
            ctx.off, ctx.val, ctx.n = off, val, t.shape[1]
            return t.sum()

        @staticmethod
        def backward(ctx, g):
            dst = sink.claim(ctx.off, ctx.n, torch.float32)
            dst.fill_(ctx.val)
            return dst, None, None

    qk, v = _split(x, 8, 4, sink=sink)
    (Fill.apply(qk, 0, 2.0) + Fill.apply(v, 8, 3.0)).backward()
    assert torch.equal(x.grad[:, :8], torch.full((2, 8, 4, 5), 2.0))
    assert torch.equal(x.grad[:, 8:], torch.full((2, 4, 4, 5), 3.0))
    assert sink.buf is None                                # reset for the next backward


def test_split_backward_falls_back_when_a_slice_gradient_is_not_the_sink():
    x = torch.randn(2, 12, 4, 5).contiguous(memory_format=CL).requires_grad_()
    sink = GradSink(x)
    qk, v = _split(x, 8, 4, sink=sink)
    w = torch.randn(2, 4, 4, 5)
    (2.0 * qk.sum() + (v * w).sum()).backward()            # ATen consumers: no claims
    assert x.grad.is_contiguous(memory_format=CL)
    assert torch.equal(x.grad[:, :8], torch.full((2, 8, 4, 5), 2.0))
    assert torch.equal(x.grad[:, 8:], w)
