#!/usr/bin/env python3
"""Golden vectors for the reference's OC2 architecture audit
(scripts/validate_oc2_architecture.py:55-427), made by running the REFERENCE's
own ``learned_option_critic_networks`` module with the audit's constructions.

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. Recorded as data:

* ``main``: the audit's 6-option actor (seed 7, hidden 128, option hidden 64 x 2
  layers, option memory 64, :58-74), the (3, 5, 24) observation drawn after it
  and the seven outputs of ``forward_sequence`` (attentions and packed state
  incl.); the weights are not stored: seeded construction must reproduce them;
* ``legacy``: the version-2 checkpoint of :146-177 (tanh-squashed actor, values as
  selector logits, initial_log_std -0.7) with its state_dict and the outputs of
  ``LearnedOptionActor.from_checkpoint(legacy_checkpoint)`` on a second
  observation (:178-188);
* ``two``: the OC2-2 ablation actor (:387-413, seed 21) and its outputs;
* ``init``: the default-constructed actor's (seed 22) mean termination
  probability on a zero observation (:306-316, 0.27);
* the epsilon-soft option probabilities / V_Omega of :258-285 and :414-421;
* ``termination_objective`` gradient of a useful and of an inferior option
  (:317-342: continuation / switch signs), and the values of both.

Usage: python tests/golden/audit/make_oc2_audit_golden.py
"""

from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
AGENTS = "/root/reference/source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct/agents"


def load_networks():
    """The audit's own loader (:16-38): poca_networks + learned_option_critic_networks as a namespace package."""
    pkg_name = "oc2_audit_ref"
    pkg = types.ModuleType(pkg_name)
    pkg.__path__ = [AGENTS]
    sys.modules[pkg_name] = pkg
    mods = {}
    for m in ("poca_networks", "learned_option_critic_networks"):
        spec = importlib.util.spec_from_file_location(f"{pkg_name}.{m}", os.path.join(AGENTS, m + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[f"{pkg_name}.{m}"] = mod
        spec.loader.exec_module(mod)
        mods[m] = mod
    return mods["learned_option_critic_networks"]


def put_state(out, prefix, module):
    names = list(module.state_dict())
    out[f"{prefix}/names"] = np.array(names)
    for k, v in module.state_dict().items():
        out[f"{prefix}/sd/{k}"] = v.detach().numpy().copy()


def put_outputs(out, prefix, outputs):
    for i in range(6):
        out[f"{prefix}/out{i}"] = outputs[i].detach().numpy().copy()
    out[f"{prefix}/state_h"] = outputs[6][0].detach().numpy().copy()
    out[f"{prefix}/state_c"] = outputs[6][1].detach().numpy().copy()


def main():
    net = load_networks()
    out = {}
    torch.manual_seed(7)
    main_kw = dict(obs_dim=24, act_dim=2, num_options=6, hidden=128, num_layers=1, memory_size=128, option_hidden=64,
                   option_num_layers=2, option_memory_size=64, initial_termination_probability=0.27,
                   initial_log_std=0.0, min_log_std=-2.5, max_log_std=0.0, squash_actions=False)
    actor = net.LearnedOptionActor(**main_kw)
    obs = torch.randn(3, 5, 24)
    with torch.no_grad():
        outputs = actor.forward_sequence(obs)
    out["main/obs"] = obs.numpy().copy()
    put_outputs(out, "main", outputs)
    out["version"] = np.int64(net.LEARNED_OPTION_CRITIC_VERSION)

    legacy_actor = net.LearnedOptionActor(obs_dim=24, act_dim=2, num_options=6, hidden=128, num_layers=1,
                                          memory_size=128, option_hidden=64, option_num_layers=2,
                                          option_memory_size=64, initial_log_std=-0.7, separate_selector=False,
                                          epsilon_greedy_selector=False, squash_actions=True)
    legacy_meta = {"learned_option_critic_version": 2, "obs_dim": 24, "discrete": False, "num_actions": 2,
                   "act_dim": 2, "num_options": 6, "hidden_dim": 128, "num_layers": 1, "memory_size": 128,
                   "option_hidden_dim": 64, "option_num_layers": 2, "option_memory_size": 64,
                   "initial_termination_probability": 0.27, "initial_log_std": -0.7, "min_log_std": -2.5,
                   "max_log_std": 0.0, "option_selector_temperature": 1.0, "option_value_temperature": 1.0,
                   "action_distribution": "tanh_squashed_normal", "action_transform": "identity_normalized"}
    ckpt = dict(legacy_meta, actor=legacy_actor.state_dict())
    loaded = net.LearnedOptionActor.from_checkpoint(ckpt, "cpu")
    legacy_obs = torch.randn(3, 5, 24)
    with torch.no_grad():
        legacy_out = loaded.forward_sequence(legacy_obs)
    assert torch.equal(legacy_out[0], legacy_out[1])
    put_state(out, "legacy", legacy_actor)
    out["legacy/obs"] = legacy_obs.numpy().copy()
    put_outputs(out, "legacy", legacy_out)
    for k, v in legacy_meta.items():
        out[f"legacy/meta/{k}"] = np.asarray(v)
    # the squashed distribution of the legacy actor: mean and log-prob of fixed wheel commands
    sel = torch.arange(3).view(3, 1).expand(3, 5) % 6
    with torch.no_grad():
        d = loaded.selected_action_dist(legacy_out[3], legacy_out[4], sel)
        wheels = torch.tanh(torch.randn(3, 5, 2)) * 0.9
        out["legacy/wheels"] = wheels.numpy().copy()
        out["legacy/logp"] = d.log_prob(wheels).numpy().copy()

    two_kw = dict(obs_dim=24, act_dim=2, num_options=2, hidden=128, num_layers=1, memory_size=128, option_hidden=128,
                  option_num_layers=1, option_memory_size=128, initial_termination_probability=0.27,
                  initial_log_std=0.0, squash_actions=False)
    torch.manual_seed(21)
    two = net.LearnedOptionActor(**two_kw)
    with torch.no_grad():
        two_out = two.forward_sequence(obs)
    put_outputs(out, "two", two_out)
    out["two/eps_probs"] = two.option_dist(torch.tensor([[2.0, -1.0]]), epsilon=0.2).probs.numpy().copy()

    torch.manual_seed(22)
    init_actor = net.LearnedOptionActor(24, 2, 6, initial_termination_probability=0.27, initial_log_std=0.0)
    with torch.no_grad():
        out["init/mean_beta"] = np.float64(torch.sigmoid(init_actor.forward_sequence(torch.zeros(2, 1, 24))[2]).mean())

    scores = torch.tensor([[3.0, 2.0, 1.0, 0.0, -1.0, -2.0]])
    cf = torch.tensor([[12.0, 6.0, 3.0, 0.0, -3.0, -6.0]])
    out["eps/scores"] = scores.numpy().copy()
    out["eps/counterfactual"] = cf.numpy().copy()
    out["eps/probs_02"] = actor.option_dist(scores, epsilon=0.2).probs.detach().numpy().copy()
    out["eps/probs_1"] = actor.option_dist(scores, epsilon=1.0).probs.detach().numpy().copy()
    out["eps/value_02"] = actor.option_state_value(scores, cf, epsilon=0.2).detach().numpy().copy()

    for tag, adv in (("good", 1.0), ("bad", -1.0)):
        logit = torch.tensor(0.0, requires_grad=True)
        loss = net.termination_objective(logit.sigmoid(), torch.tensor(adv), 0.0, torch.tensor(1.0))
        loss.backward()
        out[f"term/{tag}_loss"] = np.float64(loss.detach())
        out[f"term/{tag}_grad"] = np.float64(logit.grad)
    path = os.path.join(HERE, "oc2_audit.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({len(out)} arrays)")


if __name__ == "__main__":
    main()
