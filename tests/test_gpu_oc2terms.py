"""The OC2 update's termination, option-selection and attention terms on one kernel each way
(csrc/swarm_oc2terms.hip) against the torch formulation of the same terms
(LearnedOptionCriticTrainer._compute_sequence_losses, LOT:956-997, 1050-1093, 1282-1322):
forward values and the logits' / attentions' gradients, with local and given denominators,
degenerate rows (zero-norm attention vectors, unchanged consecutive attentions, saturated
logits, epsilon 0 and 1). The trainers' teacher-forced OC2 tests run the fused path too."""

import math

import pytest
import torch
import torch.nn.functional as F
from torch.distributions import Bernoulli, Categorical

pytestmark = pytest.mark.gpu


def _close(a, b, tol, what):
    a, b = a.detach().double(), b.detach().double()
    scale = max(1.0, float(b.abs().max()))
    err = float((a - b).abs().max())
    assert err <= tol * scale, f"{what}: max err {err:.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("with_denom", [False, True])
def test_termination_terms(with_denom, gpu_device):
    from SwarmACB_isaac.agents import learned_option_critic_trainer as LT

    g = torch.Generator(device=gpu_device).manual_seed(3 + with_denom)
    B, L = 16, 128
    z0 = torch.randn(B, L, device=gpu_device, generator=g) * 3
    z0[0, :4] = torch.tensor([40.0, -40.0, 0.0, 1e-3])           # saturated and neutral logits
    adv = torch.randn(B, L, device=gpu_device, generator=g)
    loss_mask = torch.rand(B, L, device=gpu_device, generator=g) > 0.2
    dones = (torch.rand(B, L, device=gpu_device, generator=g) > 0.9).float()
    term_mask = (1.0 - dones) * loss_mask
    denom = torch.tensor(1500.0, device=gpu_device) if with_denom else None
    pen, prior_p = 0.01, 0.27
    coef = torch.tensor([0.7, -0.3, 1.3], device=gpu_device)
    outs = []
    for fused in (True, False):
        z = z0.clone().requires_grad_(True)
        n = denom if denom is not None else term_mask.sum().clamp_min(1.0)
        if fused:
            t = LT.fused_termination_terms(z, adv, pen, prior_p, term_mask, denom)
            assert t is not None
        else:
            beta = torch.sigmoid(z)
            t = ((beta * (adv + pen) * term_mask).sum() / n,
                 (F.binary_cross_entropy_with_logits(z, torch.full_like(z, prior_p), reduction="none")
                  * term_mask).sum() / n,
                 (Bernoulli(validate_args=False, logits=z).entropy() * term_mask).sum() / n,
                 (beta * term_mask).sum() / n, (adv * term_mask).sum() / n, ((adv + pen) * term_mask).sum() / n,
                 ((beta < 1e-3).float() * term_mask).sum() / n, ((beta > 1 - 1e-3).float() * term_mask).sum() / n)
        (coef[0] * t[0] + coef[1] * t[1] + coef[2] * t[2]).backward()
        outs.append((torch.stack([x.detach() for x in t]), z.grad.clone()))
    _close(outs[0][0], outs[1][0], 2e-6, "termination terms")
    _close(outs[0][1], outs[1][1], 2e-6, "d logits")


@pytest.mark.parametrize("eps", [0.0, 0.1, 1.0])
def test_option_terms(eps, gpu_device):
    from SwarmACB_isaac.agents import learned_option_critic_trainer as LT

    g = torch.Generator(device=gpu_device).manual_seed(int(eps * 10))
    B, L, O = 16, 128, 6
    q = torch.randn(B, L, O, device=gpu_device, generator=g)
    q[0, 0] = 1.0                                                  # a tie: argmax takes the first
    options = torch.randint(0, O, (B, L), device=gpu_device, generator=g)
    loss_mask = torch.rand(B, L, device=gpu_device, generator=g) > 0.3
    boundary = (torch.rand(B, L, device=gpu_device, generator=g) > 0.6) & loss_mask

    class Actor:
        epsilon_greedy_selector = True

    got = LT.fused_option_terms(Actor(), q, options, loss_mask, boundary, eps, None)
    probs = torch.full_like(q, eps / O)
    greedy = q.argmax(dim=-1, keepdim=True)
    probs.scatter_add_(-1, greedy, torch.full_like(greedy, 1.0 - eps, dtype=probs.dtype))
    dist = Categorical(validate_args=False, probs=probs)
    n_b = boundary.sum().clamp_min(1)
    sel_w = loss_mask.unsqueeze(-1).float()
    marginal = ((dist.probs * sel_w).sum(dim=(0, 1)) / sel_w.sum().clamp_min(1.0)).clamp_min(1e-8)
    ent = -(marginal * marginal.log()).sum()
    ref = torch.stack([dist.log_prob(options).sum(), (dist.entropy() * boundary).sum() / n_b, ent,
                       (marginal * (marginal.log() + torch.log(torch.tensor(float(O), device=gpu_device)))).sum(),
                       ent.exp()])
    _close(torch.stack(got), ref, 2e-6, "option terms")


@pytest.mark.parametrize("with_denom", [False, True])
def test_attention_terms(with_denom, gpu_device):
    from SwarmACB_isaac.agents import learned_option_critic_trainer as LT
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer

    g = torch.Generator(device=gpu_device).manual_seed(7 + with_denom)
    B, L, O, D = 16, 128, 6, 24
    a0 = torch.sigmoid(torch.randn(B, L, O, D, device=gpu_device, generator=g) * 2)
    a0[0, 3, 2] = 0.0                                                # a zero-norm option vector
    a0[1, 5] = a0[1, 4]                                              # unchanged step (abs' kink)
    loss_mask = torch.rand(B, L, device=gpu_device, generator=g) > 0.2
    dones = (torch.rand(B, L, device=gpu_device, generator=g) > 0.9).float()
    d_rows = torch.tensor(1700.0, device=gpu_device) if with_denom else None
    d_pairs = torch.tensor(1400.0, device=gpu_device) if with_denom else None
    outs = []
    for fused in (True, False):
        a = a0.clone().requires_grad_(True)
        if fused:
            t = LT.fused_attention_terms(a, loss_mask, dones, d_rows, d_pairs)
            assert t is not None
        else:
            t = LearnedOptionCriticTrainer._attention_losses(a, loss_mask, dones, d_rows, d_pairs)
        (0.9 * t[0] - 1.7 * t[1]).backward()
        outs.append((torch.stack([x.detach() for x in t]), a.grad.clone()))
    _close(outs[0][0], outs[1][0], 2e-6, "attention terms")
    _close(outs[0][1], outs[1][1], 2e-6, "d attentions")


@pytest.mark.parametrize("squash,with_denom", [(False, False), (True, False), (True, True)])
def test_action_terms(squash, with_denom, gpu_device):
    """Intra-option wheel terms: the option's Normal / tanh-squashed Normal log-probs of the current
    and the frozen actor, approx KL, behaviour error and entropy, and the gradients of
    (PPO-style weights on the new log-probs + an entropy coefficient) w.r.t. means and stds."""
    from SwarmACB_isaac.agents import learned_option_critic_trainer as LT
    from SwarmACB_isaac.agents.learned_option_critic_networks import LearnedOptionActor, SquashedNormal
    from torch.distributions import Normal

    g = torch.Generator(device=gpu_device).manual_seed(11 + squash + 2 * with_denom)
    B, L, O, A = 16, 128, 6, 2
    means0 = torch.randn(B, L, O, A, device=gpu_device, generator=g) * 0.5
    stds0 = torch.rand(B, L, O, A, device=gpu_device, generator=g) * 0.5 + 0.1
    r_means = means0 + 0.05 * torch.randn(B, L, O, A, device=gpu_device, generator=g)
    r_stds = stds0 * (1 + 0.05 * torch.rand(B, L, O, A, device=gpu_device, generator=g))
    options = torch.randint(0, O, (B, L), device=gpu_device, generator=g)
    actions = torch.tanh(torch.randn(B, L, A, device=gpu_device, generator=g)) if squash else \
        torch.randn(B, L, A, device=gpu_device, generator=g)
    if squash:
        actions[0, 0] = torch.tensor([1.0, -1.0])                       # clamped to +-(1 - 1e-6)
    old_lp = torch.randn(B, L, A, device=gpu_device, generator=g)
    loss_mask = torch.rand(B, L, device=gpu_device, generator=g) > 0.25
    d_mask = torch.tensor(1700.0, device=gpu_device) if with_denom else None
    w_lp = torch.randn(B, L, A, device=gpu_device, generator=g)
    actor = LearnedOptionActor(24, A, O, hidden=16, option_hidden=16, option_memory_size=8, memory_size=16,
                               squash_actions=squash).to(gpu_device)
    outs = []
    for fused in (True, False):
        mu = means0.clone().requires_grad_(True)
        sd = stds0.clone().requires_grad_(True)
        if fused:
            lp, lp_r, kl, beh, ent = LT.fused_action_terms(actor, mu, sd, r_means, r_stds, options, actions, old_lp,
                                                           loss_mask, d_mask)
        else:
            dist_cls = SquashedNormal if squash else Normal
            m_ = actor._gather_options(mu, options)
            s_ = actor._gather_options(sd, options)
            dist = dist_cls(m_, s_, validate_args=False)
            lp = dist.log_prob(actions)
            lp_r = dist_cls(actor._gather_options(r_means, options), actor._gather_options(r_stds, options),
                            validate_args=False).log_prob(actions)
            lr = (lp - lp_r).clamp(-20.0, 20.0)
            kw = loss_mask.unsqueeze(-1).expand_as(lr).float()
            n_kl = d_mask * A if d_mask is not None else kw.sum().clamp_min(1.0)
            n_m = d_mask if d_mask is not None else loss_mask.sum().clamp_min(1)
            kl = ((lr.exp() - 1.0 - lr) * kw).sum() / n_kl
            beh = ((lp_r - old_lp).abs() * kw).sum() / n_kl
            ent = (dist.entropy().mean(dim=-1) * loss_mask).sum() / n_m
        ((lp * w_lp).sum() - 0.37 * ent).backward()
        outs.append((lp.detach(), lp_r.detach(), torch.stack([kl.detach(), beh.detach(), ent.detach()]),
                     mu.grad.clone(), sd.grad.clone()))
    for k, what in enumerate(("log_prob", "ref log_prob", "kl / behaviour / entropy", "d means", "d stds")):
        _close(outs[0][k], outs[1][k], 3e-6, what)


def test_input_checks_flag_what_torch_distributions_reject(gpu_device):
    """An option outside [0, O) (Categorical.log_prob raises) and a non-positive / non-finite std
    (Normal's validation raises) are flagged by the fused kernels and raised by the once-per-update
    check; clean inputs leave the flag clear."""
    from SwarmACB_isaac.agents import learned_option_critic_trainer as LT
    from SwarmACB_isaac.agents._trainer import check_policy_inputs
    from SwarmACB_isaac.agents.learned_option_critic_networks import LearnedOptionActor

    check_policy_inputs(gpu_device)
    g = torch.Generator(device=gpu_device).manual_seed(5)
    B, L, O, A = 4, 16, 6, 2
    q = torch.randn(B, L, O, device=gpu_device, generator=g)
    options = torch.randint(0, O, (B, L), device=gpu_device, generator=g)
    mask = torch.ones(B, L, dtype=torch.bool, device=gpu_device)

    class Actor:
        epsilon_greedy_selector = True

    LT.fused_option_terms(Actor(), q, options, mask, mask, 0.1, None)
    check_policy_inputs(gpu_device)                                   # clean
    bad = options.clone()
    bad[1, 3] = -1                                                    # the 'fresh option' sentinel
    LT.fused_option_terms(Actor(), q, bad, mask, mask, 0.1, None)
    with pytest.raises(ValueError):                                   # Categorical's support check
        check_policy_inputs(gpu_device)
    check_policy_inputs(gpu_device)                                   # the check reset the flag

    actor = LearnedOptionActor(24, A, O, hidden=16, option_hidden=16, option_memory_size=8, memory_size=16,
                               squash_actions=True).to(gpu_device)
    means = torch.randn(B, L, O, A, device=gpu_device, generator=g) * 0.5
    stds = torch.rand(B, L, O, A, device=gpu_device, generator=g) * 0.5 + 0.1
    actions = torch.tanh(torch.randn(B, L, A, device=gpu_device, generator=g))
    old_lp = torch.randn(B, L, A, device=gpu_device, generator=g)
    LT.fused_action_terms(actor, means, stds, means, stds, options, actions, old_lp, mask, None)
    check_policy_inputs(gpu_device)
    for v in (0.0, float("nan")):
        s2 = stds.clone()
        s2[2, 5, options[2, 5]] = v                                      # the selected option's std
        LT.fused_action_terms(actor, means, s2, means, stds, options, actions, old_lp, mask, None)
        with pytest.raises(ValueError):
            check_policy_inputs(gpu_device)
    # torch's constraints pass +inf scales and +-inf locs (the loss then goes non-finite and the
    # trainer's own FloatingPointError fires): no input flag for them
    s2, m2 = stds.clone(), means.clone()
    s2[2, 5, options[2, 5]] = float("inf")
    m2[1, 1, options[1, 1]] = float("-inf")
    LT.fused_action_terms(actor, m2, s2, means, stds, options, actions, old_lp, mask, None)
    check_policy_inputs(gpu_device)


def test_attention_terms_concurrent_streams(gpu_device):
    """Two attention / option forwards in flight on two streams at once each reduce through their
    own workspace (the partials were a single library buffer before): both equal their
    one-at-a-time results bit for bit."""
    from SwarmACB_isaac.agents import learned_option_critic_trainer as LT

    g = torch.Generator(device=gpu_device).manual_seed(9)
    B, L, O, D = 32, 128, 6, 24
    xs = [torch.sigmoid(torch.randn(B, L, O, D, device=gpu_device, generator=g)) for _ in range(2)]
    mask = torch.rand(B, L, device=gpu_device, generator=g) > 0.2
    dones = (torch.rand(B, L, device=gpu_device, generator=g) > 0.9).float()
    alone = [torch.stack(LT.fused_attention_terms(x, mask, dones, None, None)) for x in xs]
    torch.cuda.synchronize(gpu_device)
    streams = [torch.cuda.Stream(gpu_device) for _ in xs]
    outs = [None, None]
    for _ in range(20):
        for k, (x, s) in enumerate(zip(xs, streams)):
            s.wait_stream(torch.cuda.current_stream(gpu_device))
            with torch.cuda.stream(s):
                outs[k] = torch.stack(LT.fused_attention_terms(x, mask, dones, None, None))
        torch.cuda.synchronize(gpu_device)
        for k in range(2):
            assert torch.equal(outs[k], alone[k])


def test_input_flag_is_one_per_device(gpu_device):
    """'cuda' and 'cuda:<current>' name the same input-check flag: a trainer built with
    device='cuda' reads the flag the kernels set through tensors on cuda:0."""
    from SwarmACB_isaac.agents._trainer import _bad_action_flag, _flag_key, check_policy_inputs

    with torch.cuda.device(gpu_device):
        assert _flag_key("cuda") == _flag_key(gpu_device) == f"cuda:{torch.cuda.current_device()}"
        assert _bad_action_flag("cuda") is _bad_action_flag(gpu_device)
        _bad_action_flag(gpu_device).fill_(4)
        with pytest.raises(ValueError):
            check_policy_inputs("cuda")
        check_policy_inputs(gpu_device)                                   # cleared by the first check
