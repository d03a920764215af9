"""The critic's training-time entity sets (swarm_entity_sets_forward / _backward,
include/swarmtrain.h) against POCACritic's module path (the reference's encoders and set
assembly, poca_networks.py:597-820): the stacked sets of the value / joint / focal baseline passes
and the encoders' parameter gradients. Tolerance: the small-K products run in another order than the
library GEMM (1e-6 of scale forward, 1e-5 for the gradients summed over 80 k rows)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, what):
    scale = max(1.0, float(ref.abs().max()))
    err = float((got - ref).abs().max())
    assert err <= rtol * scale, f"{what}: max err {err:.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("passes,S,A", [(("value", "baseline"), 5, 6), (("value", "joint", "baseline"), 5, 6),
                                        (("value",), 5, 1), (("baseline",), 11, 2), (("joint", "baseline"), 5, 6)])
def test_entity_sets_match_module_path(passes, S, A, gpu_device):
    from SwarmACB_isaac.agents import poca_networks as pn

    torch.manual_seed(len(passes) * 7 + S)
    critic = pn.POCACritic(S, A, num_agents=20, h_size=128, num_heads=4).to(gpu_device)
    g = torch.Generator(device=gpu_device).manual_seed(3)
    B, N = 2048, 20
    states = torch.randn(B, N, S, device=gpu_device, generator=g)
    actions = torch.nn.functional.one_hot(torch.randint(0, A, (B, N), device=gpu_device, generator=g), A).float()
    focal = torch.randint(0, N, (B,), device=gpu_device, generator=g)
    d_out = torch.randn(len(passes) * B, N, 128, device=gpu_device, generator=g)
    res = []
    prev = pn.FUSED_ENTITIES
    for fused in (True, False):
        pn.FUSED_ENTITIES = fused
        try:
            critic.zero_grad()
            if fused:
                ents = critic._fused_entity_sets(states, actions, focal, passes)
                assert ents is not None
            else:
                sets = []
                for p in passes:
                    if p == "value":
                        sets.append(critic.obs_entity_enc(states))
                    elif p == "joint":
                        sets.append(critic.obs_act_entity_enc(torch.cat([states, actions], dim=-1)))
                    else:
                        sets.append(critic._focal_entities(states, actions, focal))
                ents = torch.cat(sets, dim=0)
            ents.backward(d_out)
            grads = [None if p.grad is None else p.grad.clone()
                     for p in list(critic.obs_entity_enc.parameters()) + list(critic.obs_act_entity_enc.parameters())]
            res.append((ents.detach(), grads))
        finally:
            pn.FUSED_ENTITIES = prev
    _close(res[0][0], res[1][0], 1e-6, "entity sets")
    for k, (a, b) in enumerate(zip(res[0][1], res[1][1])):
        if b is None:
            assert a is None or float(a.abs().max()) == 0.0, f"param {k}: gradient where the module path has none"
            continue
        _close(a, b, 1e-5, f"d param {k}")
