"""The training-time attention core on the matrix cores (swarm_rsa_attn_forward /
_backward, include/swarmtrain.h) against the reference's PyTorch formulation of
ResidualSelfAttention (poca_networks.py:417-491) in fp32, forward and every gradient.

Tolerance: fp32 sums in another order (MFMA tiles vs torch's bmm): 1e-5 relative to
each tensor's scale for the outputs, 2e-5 for the gradients.
"""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_core(qkv, mask, S, N, H):
    D = qkv.shape[1] // 3
    d = D // H
    q, k, v = (qkv[:, i * D:(i + 1) * D].reshape(S, N, H, d).transpose(1, 2) for i in range(3))
    logits = (q @ k.transpose(-2, -1)) / math.sqrt(D)
    if mask is not None:
        logits = logits + mask.view(S, 1, 1, N) * -1e6
    return (logits.softmax(dim=-1) @ v).transpose(1, 2).reshape(S * N, D)


def _close(got, ref, rtol, what):
    scale = max(1.0, float(ref.abs().max()))
    err = float((got - ref).abs().max())
    assert err <= rtol * scale, f"{what}: max err {err:.3g} (scale {scale:.3g})"
    return err / scale


@pytest.mark.parametrize("S,N,H,masked", [(37, 20, 4, False), (64, 20, 2, True), (5, 7, 1, False), (9, 32, 4, True),
                                          (2048, 20, 4, False), (11, 1, 4, False), (13, 19, 2, True)])
def test_attention_core_matches_torch(S, N, H, masked, gpu_device):
    from SwarmACB_isaac.agents.poca_networks import _AttnCore

    g = torch.Generator(device=gpu_device).manual_seed(S * 100 + N)
    D = 128
    qkv = torch.randn(S * N, 3 * D, device=gpu_device, generator=g)
    mask = None
    if masked:
        mask = (torch.rand(S, N, device=gpu_device, generator=g) < 0.3).float()
        mask[:, 0] = 0.0                      # every set keeps at least one entity
    a = qkv.clone().requires_grad_(True)
    b = qkv.clone().requires_grad_(True)
    got = _AttnCore.apply(a, mask, S, N, H)
    ref = _torch_core(b, mask, S, N, H)
    e_fwd = _close(got.detach(), ref.detach(), 1e-5, "att")
    dout = torch.randn(S * N, D, device=gpu_device, generator=g)
    got.backward(dout)
    ref.backward(dout)
    e_bwd = 0.0
    for name, sl in (("dq", slice(0, D)), ("dk", slice(D, 2 * D)), ("dv", slice(2 * D, 3 * D))):
        e_bwd = max(e_bwd, _close(a.grad[:, sl], b.grad[:, sl], 2e-5, name))
    print(f"[attn] S={S} N={N} H={H} masked={masked}: fwd {e_fwd:.3g}, bwd {e_bwd:.3g} (relative)")


@pytest.mark.parametrize("heads", [1, 2, 4])
def test_residual_self_attention_module_native_vs_torch(heads, gpu_device):
    """The whole module (norms, projections, fc_out, pooling) with the native core equals the
    reference path, outputs and parameter gradients."""
    from SwarmACB_isaac.agents import poca_networks as PN

    torch.manual_seed(heads)
    m = PN.ResidualSelfAttention(128, heads).to(gpu_device)
    x = torch.randn(300, 20, 128, device=gpu_device)
    outs, grads = [], []
    for native in (True, False):
        PN.FUSED_ATTENTION = native
        try:
            m.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_(True)
            y = m(xi)
            (y * torch.linspace(-1, 1, y.numel(), device=gpu_device).view_as(y)).sum().backward()
            outs.append(y.detach())
            grads.append([xi.grad] + [p.grad.clone() for p in m.parameters()])
        finally:
            PN.FUSED_ATTENTION = True
    _close(outs[0], outs[1], 1e-5, "pooled")
    for i, (ga, gb) in enumerate(zip(grads[0], grads[1])):
        _close(ga, gb, 2e-5, f"grad {i}")
