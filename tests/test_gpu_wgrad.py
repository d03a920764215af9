"""swarm_wgrad (include/swarmtrain.h): the weight and bias gradients of a linear layer over R rows
in one launch, against float64 products of the same operands (tolerance: fp32 accumulation over
<= 4,096 rows, |error| <= 2e-5 * sum |terms|), and the autograd paths that route through it
(poca_networks._RowsWgradLinear, the LSTM's dW_hh from the hidden sequence read in place)
against the library's own gradients of the same forward."""

import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(dy, x):
    d, xx = dy.double(), x.double()
    return d.t() @ xx, d.abs().t() @ xx.abs()


def _close(got, ref, mag, rel=2e-5):
    err = (got.double() - ref).abs()
    bound = rel * mag + 1e-30
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("R,out_f,ins", [(2048, 256, (64,)), (2048, 256, (128,)), (2047, 144, (64,)),
                                         (1999, 65, (1, 24)), (4095, 20, (128, 64)), (3, 7, (5,)), (0, 16, (16,))])
def test_wgrad_matches_float64(gpu_device, R, out_f, ins):
    from SwarmACB_isaac.agents import poca_networks as PN

    g = torch.Generator(device=gpu_device).manual_seed(R + out_f)
    dy = torch.randn(R, out_f, device=gpu_device, generator=g)
    xs = [torch.randn(R, n, device=gpu_device, generator=g) for n in ins]
    dws, db = PN.wgrad(dy, [PN._wgrad_src(x) for x in xs], True)
    torch.cuda.synchronize(gpu_device)
    for x, dw in zip(xs, dws):
        ref, mag = _ref(dy, x)
        _close(dw, ref, mag)
    _close(db, dy.double().sum(0), dy.double().abs().sum(0))


def test_wgrad_strided_rows_and_no_bias(gpu_device):
    from SwarmACB_isaac.agents import poca_networks as PN

    g = torch.Generator(device=gpu_device).manual_seed(5)
    big = torch.randn(1024, 300, device=gpu_device, generator=g)
    dy = big[:, 10:138]                       # row stride 300
    x = torch.randn(1024, 200, device=gpu_device, generator=g)[:, 50:114]
    dws, db = PN.wgrad(dy, [PN._wgrad_src(x)], False)
    assert db is None
    ref, mag = _ref(dy, x)
    _close(dws[0], ref, mag)


@pytest.mark.parametrize("with_keep", [False, True])
def test_wgrad_lstm_previous_hidden_state(gpu_device, with_keep):
    """mode 1: row n T + t of the B operand is h0[n] (t = 0) or h[n][t-1] * keep[n][t-1]."""
    from SwarmACB_isaac.agents import poca_networks as PN

    n, T, U = 16, 128, 64
    g = torch.Generator(device=gpu_device).manual_seed(11)
    h = torch.randn(n, T, U, device=gpu_device, generator=g)
    h0 = torch.randn(n, U, device=gpu_device, generator=g)
    keep = (torch.rand(n, T, device=gpu_device, generator=g) > 0.1).float() if with_keep else None
    dxg = torch.randn(n * T, 4 * U, device=gpu_device, generator=g)
    dws, _ = PN.wgrad(dxg, [PN._wgrad_src(h.reshape(n * T, U), 1, h0, keep, T)], False)
    prev = h[:, :-1] if keep is None else h[:, :-1] * keep[:, :-1, None]
    h_prev = torch.cat([h0.unsqueeze(1), prev], dim=1).reshape(n * T, U)
    ref, mag = _ref(dxg, h_prev)
    _close(dws[0], ref, mag)


def test_rows_wgrad_linear_matches_library_autograd(gpu_device):
    """_RowsWgradLinear: forward bitwise = addmm (F.linear), gradients = the library's within fp32."""
    from SwarmACB_isaac.agents import poca_networks as PN

    g = torch.Generator(device=gpu_device).manual_seed(2)
    x = torch.randn(2048, 128, device=gpu_device, generator=g, requires_grad=True)
    h = torch.randn(2048, 64, device=gpu_device, generator=g, requires_grad=True)
    w = torch.randn(256, 128, device=gpu_device, generator=g, requires_grad=True)
    w2 = torch.randn(256, 64, device=gpu_device, generator=g, requires_grad=True)
    b = torch.randn(256, device=gpu_device, generator=g, requires_grad=True)
    up = torch.randn(2048, 256, device=gpu_device, generator=g)
    y = PN._RowsWgradLinear.apply(x, w, b, h, w2)
    y_ref = torch.addmm(torch.nn.functional.linear(x, w, b), h, w2.t())
    assert torch.equal(y, y_ref)
    grads = torch.autograd.grad((y * up).sum(), [x, w, b, h, w2])
    grads_ref = torch.autograd.grad((y_ref * up).sum(), [x, w, b, h, w2])
    for a, r in zip(grads, grads_ref):
        assert torch.allclose(a, r, rtol=1e-4, atol=1e-3), float((a - r).abs().max())


def test_wgrad_rejects_bad_arguments(gpu_device):
    from SwarmACB_isaac import _native

    lib = _native.load()
    st = C.c_void_p(torch.cuda.current_stream(gpu_device).cuda_stream)
    dy = torch.zeros(8, 4, device=gpu_device)
    dw = torch.zeros(4, 4, device=gpu_device)
    x = torch.zeros(8, 4, device=gpu_device)
    src = _native.WgradSrc(4, 1, 4, x.data_ptr(), dw.data_ptr(), None, None, 3, 0)   # mode 1 without h0, 8 % 3
    arr = (_native.WgradSrc * 1)(src)
    assert lib.swarm_wgrad(8, 4, C.c_void_p(dy.data_ptr()), 4, 1, C.cast(arr, C.c_void_p), None, st) != 0
    assert lib.swarm_wgrad(8, 4, C.c_void_p(dy.data_ptr()), 4, 3, C.cast(arr, C.c_void_p), None, st) != 0
