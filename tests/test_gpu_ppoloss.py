"""The PPO trust-region loss kernels (swarm_ppo_value_loss* / swarm_ppo_policy_loss*,
include/swarmtrain.h) against the reference's torch formulation (ML-Agents
trust_region_value_loss / trust_region_policy_loss, poca_trainer.py:144-191, and the
log-ratio-bounded policy loss of learned_option_critic_trainer.py:45-72), forward and gradient.

The rows include the kinks: values equal to the old values (max tie), |v - old| exactly eps
(clamp boundary), log-ratios of exactly 0 (min tie) and beyond +-20 (stable clamp). Tolerance:
the masked sums run in another order (1e-6 of scale forward); gradients are elementwise with the
same subgradient choices as torch (1e-6 of scale).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, what):
    scale = max(1.0, float(ref.abs().max()))
    err = float((got - ref).abs().max())
    assert err <= rtol * scale, f"{what}: max err {err:.3g} (scale {scale:.3g})"


def _run(fn, fused, *args, **kw):
    from SwarmACB_isaac.agents import _trainer

    old = _trainer.FUSED_LOSSES
    _trainer.FUSED_LOSSES = fused
    try:
        return fn(*args, **kw)
    finally:
        _trainer.FUSED_LOSSES = old


def _mask(kind, M, g, dev):
    if kind is None:
        return None
    m = torch.rand(M, device=dev, generator=g) < 0.7
    return m if kind == "bool" else m.float()


@pytest.mark.parametrize("mask_kind", [None, "bool", "float"])
@pytest.mark.parametrize("with_denom", [False, True])
@pytest.mark.parametrize("M", [2048, 37])
def test_value_loss(mask_kind, with_denom, M, gpu_device):
    from SwarmACB_isaac.agents._trainer import trust_region_value_loss

    g = torch.Generator(device=gpu_device).manual_seed(M + (7 if with_denom else 0))
    eps = 0.2
    v0 = torch.randn(M, device=gpu_device, generator=g)
    old = v0 + torch.randn(M, device=gpu_device, generator=g) * 0.3
    old[:M // 8] = v0[:M // 8]                     # tie of the two squared errors
    old[M // 8:M // 4] = v0[M // 8:M // 4] - eps   # on the clamp boundary (up to rounding)
    ret = torch.randn(M, device=gpu_device, generator=g)
    mask = _mask(mask_kind, M, g, gpu_device)
    denom = torch.tensor(float(M) * 0.5, device=gpu_device) if with_denom else None
    out = []
    for fused in (True, False):
        v = v0.clone().requires_grad_(True)
        loss = _run(trust_region_value_loss, fused, v, old, ret, eps, mask, denom)
        loss.backward(torch.tensor(1.7, device=gpu_device))
        out.append((loss.detach(), v.grad.clone()))
    _close(out[0][0], out[1][0], 1e-6, "value loss")
    _close(out[0][1], out[1][1], 1e-6, "d values")


@pytest.mark.parametrize("stable", [False, True])
@pytest.mark.parametrize("A,adv_per_elem", [(1, False), (2, False), (2, True)])
@pytest.mark.parametrize("mask_kind,with_denom", [(None, False), ("bool", False), ("bool", True), ("float", False)])
def test_policy_loss(stable, A, adv_per_elem, mask_kind, with_denom, gpu_device):
    from SwarmACB_isaac.agents._trainer import trust_region_policy_loss
    from SwarmACB_isaac.agents.learned_option_critic_trainer import stable_trust_region_policy_loss

    fn = stable_trust_region_policy_loss if stable else trust_region_policy_loss
    M = 2048
    g = torch.Generator(device=gpu_device).manual_seed(A * 10 + int(stable))
    lp0 = torch.randn(M, A, device=gpu_device, generator=g) * 0.3
    old = lp0 + torch.randn(M, A, device=gpu_device, generator=g) * 0.2
    old[:M // 8] = lp0[:M // 8]                    # ratio exactly 1: a tie of the min
    old[M // 8:M // 8 + 16] = lp0[M // 8:M // 8 + 16] - 25.0   # beyond the stable bound
    adv = torch.randn(M, A if adv_per_elem else 1, device=gpu_device, generator=g)
    mask = _mask(mask_kind, M, g, gpu_device)
    denom = torch.tensor(float(M * A) * 0.6, device=gpu_device) if with_denom else None
    out = []
    for fused in (True, False):
        lp = lp0.clone().requires_grad_(True)
        loss = _run(fn, fused, adv, lp, old, 0.2, mask, denom)
        loss.backward(torch.tensor(0.9, device=gpu_device))
        out.append((loss.detach(), lp.grad.clone()))
    if not stable:
        # the unbounded ratio overflows to inf in both paths for the -25 rows; compare the rest
        keep = torch.ones(M, dtype=torch.bool, device=gpu_device)
        keep[M // 8:M // 8 + 16] = False
        assert torch.isfinite(out[0][0]) == torch.isfinite(out[1][0])
        _close(out[0][1][keep], out[1][1][keep], 1e-6, "d log_probs")
        if torch.isfinite(out[1][0]):
            _close(out[0][0], out[1][0], 1e-6, "policy loss")
        return
    _close(out[0][0], out[1][0], 1e-6, "policy loss")
    _close(out[0][1], out[1][1], 1e-6, "d log_probs")


def test_loss_kernels_refuse_bad_arguments(gpu_device):
    from SwarmACB_isaac import _native

    lib = _native.load()
    x = torch.zeros(8, device=gpu_device)
    m = torch.zeros(8, dtype=torch.uint8, device=gpu_device)
    p = x.data_ptr()
    assert lib.swarm_ppo_value_loss(0, p, p, p, None, None, 0.2, None, p, p, None) != 0
    assert lib.swarm_ppo_value_loss(8, p, p, p, p, m.data_ptr(), 0.2, None, p, p, None) != 0
    assert lib.swarm_ppo_policy_loss(4, 2, 3, p, p, p, None, None, 0.8, 1.2, 0, None, p, p, None) != 0


@pytest.mark.parametrize("K,mask_kind,with_denom", [(6, "bool", False), (6, "bool", True), (6, None, False),
                                                    (18, "bool", False), (1, "bool", False)])
def test_categorical_terms(K, mask_kind, with_denom, gpu_device):
    """log_prob and the masked mean entropy of Categorical(logits) (swarm_categorical_terms*) against
    torch.distributions.Categorical, forward and the logits' gradient (both outputs weighted)."""
    from SwarmACB_isaac.agents._trainer import categorical_terms

    M = 2048
    g = torch.Generator(device=gpu_device).manual_seed(K * 3 + int(with_denom))
    z0 = torch.randn(M, K, device=gpu_device, generator=g) * 2.0
    z0[:8] = 0.0                                     # uniform rows
    acts = torch.randint(0, K, (M,), device=gpu_device, generator=g)
    mask = _mask(mask_kind, M, g, gpu_device)
    denom = torch.tensor(1500.0, device=gpu_device) if with_denom else None
    glp = torch.randn(M, device=gpu_device, generator=g)
    out = []
    for fused in (True, False):
        z = z0.clone().requires_grad_(True)
        lp, ent = _run(categorical_terms, fused, z, acts, mask, denom)
        (lp * glp).sum().backward(retain_graph=True)
        (ent * 0.37).backward()
        out.append((lp.detach(), ent.detach(), z.grad.clone()))
    _close(out[0][0], out[1][0], 1e-6, "log_prob")
    _close(out[0][1], out[1][1], 1e-6, "mean entropy")
    _close(out[0][2], out[1][2], 2e-6, "d logits")


def test_categorical_terms_flag_out_of_range_actions(gpu_device):
    """An action outside [0, K) (e.g. a -1 option sentinel), even on a masked-out row, is not a
    silent NaN: the kernel flags it and check_categorical_actions raises (torch's gather raises
    on such an index too); valid actions leave the flag clear."""
    from SwarmACB_isaac.agents._trainer import categorical_terms, check_categorical_actions

    M, K = 256, 6
    z = torch.randn(M, K, device=gpu_device)
    acts = torch.randint(0, K, (M,), device=gpu_device)
    mask = torch.ones(M, dtype=torch.bool, device=gpu_device)
    categorical_terms(z, acts, mask)
    check_categorical_actions(gpu_device)                     # clean
    acts[17] = -1
    mask[17] = False
    categorical_terms(z, acts, mask)
    with pytest.raises(IndexError):
        check_categorical_actions(gpu_device)
    check_categorical_actions(gpu_device)                     # the check reset the flag
