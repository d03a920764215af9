"""GPU parity of the fused critic attention (swarm_rsa_pool, include/swarmcritic.h)
as used by the drop-in POCACritic under torch.no_grad() on the GPU.

Against (1) the reference modules' own outputs (tests/golden/critic/
poca_networks.npz, fp32 within 1e-5) and (2) at the C3 size (8192 envs x 20
e-pucks, cyclamen critic with LSTM memory) against the same module's PyTorch
path on the same GPU, plus size-independent properties (agent permutation
equivariance of the baselines)."""

import numpy as np
import pytest
import torch

import networks_io as IO
from SwarmACB_isaac.agents import poca_networks as PN

pytestmark = pytest.mark.gpu

G = IO.load()
TOL = dict(rtol=1e-5, atol=1e-5)


@pytest.fixture
def fused_calls(monkeypatch):
    calls = []
    orig = PN._fused_rsa

    def spy(attn, rows, mode, n):
        calls.append(mode)
        return orig(attn, rows, mode, n)

    monkeypatch.setattr(PN, "_fused_rsa", spy)
    return calls


def close(got, key):
    np.testing.assert_allclose(got.detach().cpu().numpy(), G[key], err_msg=key, **TOL)


@pytest.mark.parametrize("prefix", IO.CRITICS)
def test_fused_critic_matches_reference(gpu_device, fused_calls, prefix):
    c = IO.critic(G, prefix, gpu_device)
    s, a = IO.t(G, prefix + "states", gpu_device), IO.t(G, prefix + "actions", gpu_device)
    with torch.no_grad():
        close(PN._fused_rsa(c.self_attn, c.obs_entity_enc(s), 0, 20), prefix + "pool_critic")
        rows = torch.cat([c.obs_entity_enc(s), c.obs_act_entity_enc(torch.cat([s, a], -1))], 1)
        close(PN._fused_rsa(c.self_attn, rows, 1, 20), prefix + "pool_baselines")
        close(c.critic_pass(s), prefix + "critic_pass")
        close(c.joint_action_pass(s, a), prefix + "joint_action_pass")
        close(c.all_baselines(s, a), prefix + "all_baselines")
        close(c.baseline(s[:, 3], torch.cat([s[:, :3], s[:, 4:]], 1), torch.cat([a[:, :3], a[:, 4:]], 1)),
              prefix + "baseline3")
        if c.lstm is not None:
            mc = (IO.t(G, prefix + "mem_critic_h", gpu_device), IO.t(G, prefix + "mem_critic_c", gpu_device))
            mb = (IO.t(G, prefix + "mem_base_h", gpu_device), IO.t(G, prefix + "mem_base_c", gpu_device))
            v, (vh, vc) = c.critic_pass(s, mc, return_memory=True)
            close(v, prefix + "critic_pass_mem"), close(vh, prefix + "critic_pass_mem_h")
            b, (bh, bc) = c.all_baselines(s, a, mb, return_memory=True)
            close(b, prefix + "all_baselines_mem"), close(bh, prefix + "all_baselines_mem_h")
            close(bc, prefix + "all_baselines_mem_c")
    assert 1 in fused_calls and 0 in fused_calls  # both kernel modes ran


def test_autograd_uses_pytorch_path(gpu_device, fused_calls):
    c = IO.critic(G, "cyc_", gpu_device).train()   # MIOpen's LSTM backward needs training mode
    s, a = IO.t(G, "cyc_states", gpu_device), IO.t(G, "cyc_actions", gpu_device)
    out = c.all_baselines(s, a)
    out.sum().backward()
    assert fused_calls == [] and c.self_attn.fc_out.weight.grad is not None
    close(out, "cyc_all_baselines")


@pytest.mark.parametrize("heads", [4, 2, 1])
def test_fused_matches_torch_path_at_c3_size(gpu_device, heads):
    """Foraging cyclamen C3: 8192 envs x 20 agents, one-hot module actions,
    recurrent critic (memory 128)."""
    torch.manual_seed(heads)
    E, N = 8192, 20
    c = PN.POCACritic(5, 6, N, 128, heads, 1, memory_size=128).to(gpu_device).eval()
    with torch.no_grad():
        for p in c.parameters():
            p.add_(torch.randn_like(p) * 0.05)
        s = torch.randn(E, N, 5, device=gpu_device)
        a = torch.nn.functional.one_hot(torch.randint(0, 6, (E, N), device=gpu_device), 6).float()
        mem = (torch.randn(1, E * N, 64, device=gpu_device), torch.randn(1, E * N, 64, device=gpu_device))
        fused, (fh, fc) = c.all_baselines(s, a, mem, return_memory=True)
        v_fused = c.critic_pass(s)
        c.use_fused = False
        ref, (rh, rc) = c.all_baselines(s, a, mem, return_memory=True)
        v_ref = c.critic_pass(s)
    torch.testing.assert_close(fused, ref, **TOL)
    torch.testing.assert_close(fh, rh, **TOL)
    torch.testing.assert_close(v_fused, v_ref, **TOL)


def test_baselines_are_permutation_equivariant(gpu_device):
    """Relabelling the agents permutes the baselines (the critic is permutation
    invariant over the other agents; PN:822-882)."""
    torch.manual_seed(1)
    c = IO.critic(G, "ff_", gpu_device)
    s = torch.randn(512, 20, 5, device=gpu_device)
    a = torch.randn(512, 20, 2, device=gpu_device)
    perm = torch.randperm(20, device=gpu_device)
    with torch.no_grad():
        b = c.all_baselines(s, a)
        bp = c.all_baselines(s[:, perm], a[:, perm])
    torch.testing.assert_close(bp, b[:, perm], **TOL)


def test_rejects_unsupported_shapes(gpu_device):
    from SwarmACB_isaac import _native
    import ctypes as C

    lib = _native.load()
    z = torch.zeros(4, device=gpu_device)
    p = C.c_void_p(z.data_ptr())
    assert lib.swarm_rsa_pool(0, 1, 21, 4, 128, p, p, p, p, p, None) == -1   # N > 20
    assert lib.swarm_rsa_pool(0, 1, 20, 8, 128, p, p, p, p, p, None) == -1   # 8 heads
    assert lib.swarm_rsa_pool(0, 1, 20, 4, 256, p, p, p, p, p, None) == -1   # hidden 256
    assert lib.swarm_rsa_pool(4, 1, 20, 4, 128, p, p, p, p, p, None) == -1   # mode


@pytest.mark.parametrize("B,N,heads", [(1, 20, 4), (7, 20, 2), (5, 13, 4), (9, 3, 1), (2, 1, 4)])
def test_single_sets_odd_env_counts(gpu_device, B, N, heads):
    """SINGLE mode stages two envs per iteration: odd env counts (a last iteration
    with one env), runtime set sizes and N = 1 against the module's PyTorch path."""
    torch.manual_seed(B * 100 + N)
    c = PN.POCACritic(5, 2, N, 128, heads, 1).to(gpu_device).eval()
    s = torch.randn(B, N, 5, device=gpu_device)
    a = torch.randn(B, N, 2, device=gpu_device)
    with torch.no_grad():
        v, q = c.critic_pass(s), c.joint_action_pass(s, a)
        bl = c.all_baselines(s, a) if N > 1 else None
        c.use_fused = False
        torch.testing.assert_close(v, c.critic_pass(s), **TOL)
        torch.testing.assert_close(q, c.joint_action_pass(s, a), **TOL)
        if bl is not None:
            torch.testing.assert_close(bl, c.all_baselines(s, a), **TOL)


@pytest.mark.parametrize("rows", [1, 7, 8, 163841])
def test_embedding_norm_matches_layer_norm(gpu_device, rows):
    from SwarmACB_isaac import _native
    import ctypes as C

    torch.manual_seed(rows)
    x = torch.randn(rows, 128, device=gpu_device) * 3.0 + 0.5
    out = torch.full_like(x, float("nan"))
    lib = _native.load()
    rc = lib.swarm_rsa_embedding_norm(rows, 128, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), None)
    assert rc == 0
    torch.cuda.synchronize()
    torch.testing.assert_close(out, torch.nn.functional.layer_norm(x, (128,)), **TOL)
    assert lib.swarm_rsa_embedding_norm(rows, 64, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), None) == -1


@pytest.mark.parametrize("n,inp,units", [(163840, 128, 64), (8192, 128, 64), (5, 7, 3), (1, 128, 64)])
def test_fused_lstm_step_matches_torch(gpu_device, n, inp, units):
    """One LSTM step through swarm_lstm_cell (GEMMs + fused cell) against nn.LSTM
    (MIOpen) on the same GPU; the actor at C3 is 8192 envs x 20 agents."""
    torch.manual_seed(n)
    lstm = PN._mlagents_lstm(inp, 2 * units)[0].to(gpu_device)
    with torch.no_grad():
        for p in lstm.parameters():
            p.add_(torch.randn_like(p) * 0.1)
        x = torch.randn(n, 1, inp, device=gpu_device)
        h = torch.randn(1, n, units, device=gpu_device)
        c = torch.randn(1, n, units, device=gpu_device) * 2
        out, (h1, c1) = PN._lstm(lstm, x, (h, c))
        ref, (rh, rc) = lstm(x, (h, c))
    torch.testing.assert_close(out, ref, **TOL)
    torch.testing.assert_close(h1, rh, **TOL)
    torch.testing.assert_close(c1, rc, **TOL)


def test_option_critic_counterfactuals_fused(gpu_device, fused_calls):
    """The OC targets (PN:674-820) through the fused kernel against the reference
    modules' outputs (tests/golden/critic)."""
    c = IO.critic(G, "cyc_", gpu_device)
    s, a = IO.t(G, "cyc_states", gpu_device), IO.t(G, "cyc_actions", gpu_device)
    ids, focal = IO.t(G, "cyc_action_ids", gpu_device), IO.t(G, "cyc_focal_ids", gpu_device)
    mf = (IO.t(G, "cyc_mem_focal_h", gpu_device), IO.t(G, "cyc_mem_focal_c", gpu_device))
    with torch.no_grad():
        close(c.all_discrete_counterfactual_values(s, ids, 6), "cyc_all_cf")
        close(c.focal_discrete_counterfactual_values(s, ids, focal, 6), "cyc_focal_cf")
        close(c.focal_baselines(s, a, focal), "cyc_focal_baselines")
        close(c.focal_discrete_counterfactual_values(s, ids, focal, 6, memory=mf), "cyc_focal_cf_mem")
        close(c.focal_baselines(s, a, focal, mf), "cyc_focal_baselines_mem")
    assert fused_calls and set(fused_calls) == {0}


def test_focal_counterfactuals_at_c4_size(gpu_device):
    """DirGate cyclamen OC (C4): 2048 envs per GPU, 6 options; fused vs PyTorch path."""
    torch.manual_seed(4)
    E, N, A = 2048, 20, 6
    c = PN.POCACritic(5, A, N, 128, 4, 1, memory_size=128).to(gpu_device).eval()
    with torch.no_grad():
        for p in c.parameters():
            p.add_(torch.randn_like(p) * 0.05)
        s = torch.randn(E, N, 5, device=gpu_device)
        ids = torch.randint(0, A, (E, N), device=gpu_device)
        focal = torch.randint(0, N, (E,), device=gpu_device)
        mem = (torch.randn(1, E, 64, device=gpu_device), torch.randn(1, E, 64, device=gpu_device))
        fused = c.focal_discrete_counterfactual_values(s, ids, focal, A, memory=mem)
        c.use_fused = False
        ref = c.focal_discrete_counterfactual_values(s, ids, focal, A, memory=mem)
    torch.testing.assert_close(fused, ref, **TOL)


@pytest.mark.parametrize("B,N,A,heads", [(12288, 20, 6, 4), (33, 20, 20, 4), (17, 13, 6, 2), (9, 5, 3, 1),
                                         (4, 1, 2, 4)])
def test_focal_shared_sets_match_torch_path(gpu_device, B, N, A, heads):
    """swarm_rsa_pool_focal (the N joint rows and the A alternative rows of a row embedded
    once, logits shared by its A sets) against the module's PyTorch path, which embeds and
    attends the B * A sets separately: C5's 12,288 termination-advantage rows, the largest
    row block (N + A = 40), runtime set sizes, N = 1."""
    torch.manual_seed(B + N + A)
    c = PN.POCACritic(5, A, N, 128, heads, 1, memory_size=128).to(gpu_device).eval()
    with torch.no_grad():
        for p in c.parameters():
            p.add_(torch.randn_like(p) * 0.05)
        s = torch.randn(B, N, 5, device=gpu_device)
        ids = torch.randint(0, A, (B, N), device=gpu_device)
        focal = torch.randint(0, N, (B,), device=gpu_device)
        mem = (torch.randn(1, B, 64, device=gpu_device), torch.randn(1, B, 64, device=gpu_device))
        shared = c.focal_discrete_counterfactual_values(s, ids, focal, A, memory=mem)
        c.use_fused = False
        ref = c.focal_discrete_counterfactual_values(s, ids, focal, A, memory=mem)
    torch.testing.assert_close(shared, ref, **TOL)


def test_focal_rejects_oversized_row_blocks(gpu_device):
    from SwarmACB_isaac import _native
    import ctypes as C

    lib = _native.load()
    z = torch.zeros(4, device=gpu_device)
    p = C.c_void_p(z.data_ptr())
    assert lib.swarm_rsa_pool_focal(1, 20, 21, 4, 128, p, p, p, p, p, p, None) == -1   # N + A > 40
    assert lib.swarm_rsa_pool_focal(1, 20, 0, 4, 128, p, p, p, p, p, p, None) == -1    # A = 0
    assert lib.swarm_rsa_pool_focal(1, 20, 6, 4, 128, p, p, p, p, None, p, None) == -1  # no focal ids


@pytest.mark.parametrize("memory", [False, True])
def test_value_and_baselines_shares_rows(gpu_device, fused_calls, memory):
    """The rollout's pair of critic calls on one projection pass (SINGLE_OF_PAIRS +
    BASELINES) equals critic_pass and all_baselines called separately."""
    torch.manual_seed(7)
    E, N = 1027, 20
    c = PN.POCACritic(5, 6, N, 128, 4, 1, memory_size=128 if memory else 0).to(gpu_device).eval()
    with torch.no_grad():
        for p in c.parameters():
            p.add_(torch.randn_like(p) * 0.05)
        s = torch.randn(E, N, 5, device=gpu_device)
        a = torch.nn.functional.one_hot(torch.randint(0, 6, (E, N), device=gpu_device), 6).float()
        mc = mb = None
        if memory:
            mc = (torch.randn(1, E, 64, device=gpu_device), torch.randn(1, E, 64, device=gpu_device))
            mb = (torch.randn(1, E * N, 64, device=gpu_device), torch.randn(1, E * N, 64, device=gpu_device))
        (v, vm), (b, bm) = c.value_and_baselines(s, a, mc, mb)
        assert fused_calls == [(2, 1)]  # one shared projection pass, both kernel modes
        rv, rvm = c.critic_pass(s, mc, return_memory=True)
        rb, rbm = c.all_baselines(s, a, mb, return_memory=True)
    torch.testing.assert_close(v, rv, **TOL)
    torch.testing.assert_close(b, rb, **TOL)
    if memory:
        torch.testing.assert_close(vm[0], rvm[0], **TOL)
        torch.testing.assert_close(bm[1], rbm[1], **TOL)


@pytest.mark.parametrize("N", [20, 7])
def test_decision_passes_value_joint_baselines_share_rows(gpu_device, fused_calls, N):
    """The option-critic decision's three critic calls on one projection pass
    (SINGLE_OF_PAIRS + ACTIONS_OF_PAIRS + BASELINES) equal critic_pass,
    joint_action_pass and all_baselines called separately, memories included."""
    torch.manual_seed(11)
    E = 515
    c = PN.POCACritic(5, 6, N, 128, 4, 2, memory_size=128).to(gpu_device).eval()
    with torch.no_grad():
        for p in c.parameters():
            p.add_(torch.randn_like(p) * 0.05)
        s = torch.randn(E, N, 5, device=gpu_device)
        a = torch.nn.functional.one_hot(torch.randint(0, 6, (E, N), device=gpu_device), 6).float()
        mem = lambda n: (torch.randn(1, n, 64, device=gpu_device), torch.randn(1, n, 64, device=gpu_device))  # noqa
        mv, mj, mb = mem(E), mem(E), mem(E * N)
        (v, vm), (j, jm), (b, bm) = c.decision_passes(s, a, value=True, joint=True, baselines=True,
                                                      value_memory=mv, joint_memory=mj, baseline_memory=mb)
        assert fused_calls == [(2, 3, 1)]
        _, (j2, jm2), _ = c.decision_passes(s, a, value=False, joint=True, baselines=False, joint_memory=mj)
        rv, rvm = c.critic_pass(s, mv, return_memory=True)
        rj, rjm = c.joint_action_pass(s, a, mj, return_memory=True)
        rb, rbm = c.all_baselines(s, a, mb, return_memory=True)
    for got, ref in ((v, rv), (j, rj), (j2, rj), (b, rb), (vm[0], rvm[0]), (jm[1], rjm[1]), (jm2[0], rjm[0]),
                     (bm[0], rbm[0])):
        torch.testing.assert_close(got, ref, **TOL)
