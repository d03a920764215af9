"""The LayerNorm and split-row gradient kernels of the critic's training path (swarm_row_norm_* /
swarm_set_pool_*, include/swarmtrain.h) against torch's layer_norm / add / mean in fp32
(the reference's formulation, poca_networks.py:417-491), forward and every gradient.

Tolerance: the statistics are summed in another order (two-pass per row vs torch's
Welford, set means in another order): 2e-6 relative to each tensor's scale forward,
1e-5 backward.
"""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, what):
    scale = max(1.0, float(ref.abs().max()))
    err = float((got - ref).abs().max())
    assert err <= rtol * scale, f"{what}: max err {err:.3g} (scale {scale:.3g})"
    return err / scale


@pytest.mark.parametrize("rows,D", [(1, 128), (37, 128), (81920, 128), (1000, 256), (9, 256)])
def test_row_norm_matches_torch(rows, D, gpu_device):
    from SwarmACB_isaac.agents.poca_networks import _RowNorm

    g = torch.Generator(device=gpu_device).manual_seed(rows + D)
    x = torch.randn(rows, D, device=gpu_device, generator=g) * 3.0 + 0.5
    a = x.clone().requires_grad_(True)
    b = x.clone().requires_grad_(True)
    got = _RowNorm.apply(a)
    ref = F.layer_norm(b, (D,), eps=1e-5)
    e_f = _close(got.detach(), ref.detach(), 2e-6, "xhat")
    dy = torch.randn(rows, D, device=gpu_device, generator=g)
    got.backward(dy)
    ref.backward(dy)
    e_b = _close(a.grad, b.grad, 1e-5, "dx")
    print(f"[row_norm] rows={rows} D={D}: fwd {e_f:.3g}, bwd {e_b:.3g}")


@pytest.mark.parametrize("S,n,D", [(1, 1, 128), (5, 20, 128), (4096, 20, 128), (33, 7, 256), (6, 21, 128)])
def test_set_pool_matches_torch(S, n, D, gpu_device):
    from SwarmACB_isaac.agents.poca_networks import _SetPool

    g = torch.Generator(device=gpu_device).manual_seed(S * 31 + n)
    a0 = torch.randn(S * n, D, device=gpu_device, generator=g)
    x0 = torch.randn(S * n, D, device=gpu_device, generator=g)
    a1, x1 = a0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
    a2, x2 = a0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
    got = _SetPool.apply(a1, x1, S, n)
    ref = F.layer_norm(a2 + x2, (D,), eps=1e-5).view(S, n, D).mean(dim=1)
    e_f = _close(got.detach(), ref.detach(), 2e-6, "pooled")
    dp = torch.randn(S, D, device=gpu_device, generator=g)
    got.backward(dp)
    ref.backward(dp)
    e_b = max(_close(a1.grad, a2.grad, 1e-5, "da"), _close(x1.grad, x2.grad, 1e-5, "dx"))
    print(f"[set_pool] S={S} n={n} D={D}: fwd {e_f:.3g}, bwd {e_b:.3g}")


@pytest.mark.parametrize("heads,n", [(4, 20), (2, 20), (1, 9)])
def test_residual_self_attention_fused_norms(heads, n, gpu_device):
    """The whole module with the fused norms against FUSED_NORMS = False (torch's norms, the
    same attention core): outputs and every parameter / input gradient."""
    from SwarmACB_isaac.agents import poca_networks as pn

    torch.manual_seed(heads * 7 + n)
    m = pn.ResidualSelfAttention(128, heads).to(gpu_device)
    g = torch.Generator(device=gpu_device).manual_seed(5)
    inp = torch.randn(512, n, 128, device=gpu_device, generator=g)
    dp = torch.randn(512, 128, device=gpu_device, generator=g)
    outs = []
    for fused in (True, False):
        pn.FUSED_NORMS = fused
        try:
            m.zero_grad()
            x = inp.clone().requires_grad_(True)
            y = m(x)
            y.backward(dp)
            outs.append((y.detach(), x.grad.clone(), [p.grad.clone() for p in m.parameters()]))
        finally:
            pn.FUSED_NORMS = True
    (y1, gx1, gp1), (y0, gx0, gp0) = outs
    _close(y1, y0, 2e-6, "pooled")
    _close(gx1, gx0, 2e-5, "d inp")
    for k, (p1, p0) in enumerate(zip(gp1, gp0)):
        _close(p1, p0, 2e-5, f"d param {k}")


def test_norm_kernels_refuse_bad_arguments(gpu_device):
    from SwarmACB_isaac import _native

    lib = _native.load()
    x = torch.zeros(4, 128, device=gpu_device)
    r = torch.zeros(4, device=gpu_device)
    assert lib.swarm_row_norm_forward(4, 96, x.data_ptr(), x.data_ptr(), r.data_ptr(), None) != 0
    assert lib.swarm_set_pool_forward(2, 0, 128, x.data_ptr(), x.data_ptr(), x.data_ptr(), r.data_ptr(),
                                      x.data_ptr(), None) != 0
    assert lib.swarm_row_norm_backward(4, 128, x.data_ptr() + 4, x.data_ptr(), r.data_ptr(), x.data_ptr(),
                                       None) != 0


@pytest.mark.parametrize("rows,fin,fout,bias", [(40960, 5, 128, True), (81920, 128, 384, True),
                                                 (9000, 11, 128, True), (16384, 128, 128, False)])
def test_splitk_linear_gradients(rows, fin, fout, bias, gpu_device):
    """_SplitKLinear's weight / bias gradients through swarm_splitk_colsum / _finish against
    torch's linear backward (fp32 sums in another order: 2e-5 of scale)."""
    from SwarmACB_isaac.agents.poca_networks import _SplitKLinear

    g = torch.Generator(device=gpu_device).manual_seed(rows + fout)
    x = torch.randn(rows, fin, device=gpu_device, generator=g)
    w0 = torch.randn(fout, fin, device=gpu_device, generator=g) * 0.1
    b0 = torch.randn(fout, device=gpu_device, generator=g) if bias else None
    dy = torch.randn(rows, fout, device=gpu_device, generator=g)
    w1, w2 = w0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
    b1 = b0.clone().requires_grad_(True) if bias else None
    b2 = b0.clone().requires_grad_(True) if bias else None
    _SplitKLinear.apply(x, w1, b1).backward(dy)
    F.linear(x, w2, b2).backward(dy)
    _close(w1.grad, w2.grad, 2e-5, "dW")
    if bias:
        _close(b1.grad, b2.grad, 2e-5, "db")
