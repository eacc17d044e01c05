"""Descriptor uploads vs. pending fills on a non-blocking stream (the round-2/3 conv-round fault).

cgl_linear_prepare and cgl_gan_create upload their GEMM descriptors with synchronous copies on the
legacy null stream.  A torch stream (torch.cuda.Stream()) is non-blocking: the null stream does not
wait for it.  When the descriptor buffer was zero-filled by torch.zeros on such a stream, and that
stream was still busy, the fill could land AFTER the upload and zero the descriptors; the next GEMM
then dereferenced null operand pointers.  bench.py builds the conv round inside
``with torch.cuda.stream(side)``, and under the serialising rocprofv3 counter pass the zero-fill of
PreparedLinear's descriptor (G's nn.Linear(100, 8192)) was delayed past its upload: the illegal
address of profiles/r03_conv_fault.md.  Both uploads now drain the device first.

Here the side stream is kept busy with matmuls before the buffers are created, and the uploaded bytes
are checked BEFORE anything is launched from them (a lost upload fails the test, it cannot fault)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _busy(n=6):
    a = torch.randn(4096, 4096, device="cuda")
    for _ in range(n):
        a = torch.tanh(a @ a * 1e-3)
    return a


def test_prepared_linear_descriptor_survives_side_stream_fill():
    from cglgan import conv_ops as O
    s = torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(3)
    with torch.cuda.stream(s):
        _busy()
        x = torch.randn(64, 100, device="cuda", generator=g)
        w = torch.randn(256, 100, device="cuda", generator=g) * 0.1
        b = torch.randn(256, device="cuda", generator=g)
        y = torch.zeros(64, 256, device="cuda")
        lin = O.PreparedLinear(0, x, w, b, y, None, 64, 256, 100)
    torch.cuda.synchronize()
    assert int(lin.desc.count_nonzero()) > 0, "descriptor zeroed by the side-stream fill after its upload"
    with torch.cuda.stream(s):
        lin()
    torch.cuda.synchronize()
    ref = x.double() @ w.double().t() + b.double()
    assert torch.allclose(y.double(), ref, rtol=1e-5, atol=1e-4)


def test_gan_step_descriptors_survive_side_stream_fill():
    from cglgan import GanStep, specs
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        _busy()
        st = GanStep(specs.mnist_generator(), specs.mnist_discriminator(), batch=64, gen_z=True, seed=5)
    torch.cuda.synchronize()
    # the GEMM descriptor table (cgl_gan_tensor 5): a fill landing after the upload leaves it all zero
    assert int(st.internal(5).view(torch.int32).count_nonzero()) > 0, "GanStep descriptors zeroed by the fill"
