"""Stacked parameter storage (poca_networks.StackedLinears) and the OC2 actor's two-stream forward,
on the CPU: the head / q|k|v Parameters alias one storage without changing the module's
Parameters, state_dict keys or results (bitwise against the concatenated weights), survive a
deepcopy, .to() and load_state_dict, and the merged-row stages of two streams match the stages
run one stream at a time."""

import copy

import torch

from SwarmACB_isaac.agents import learned_option_critic_networks as LON
from SwarmACB_isaac.agents import poca_networks as PN


def _actor(seed=0):
    torch.manual_seed(seed)
    return LON.LearnedOptionActor(24, 2, 6, option_hidden=64, option_memory_size=32)


def test_heads_alias_one_storage_and_keep_state_dict_keys():
    a = _actor()
    st = a.__dict__["_stacked"]
    assert st.intact()
    plain = {k for k, _ in a.named_parameters()}
    assert set(a.state_dict().keys()) >= plain
    # every head Parameter is a slice of the stacked storage
    w = st.W
    assert a.option_value_heads[0].weight.data_ptr() == w.data_ptr()
    assert a.action_heads[5].weight.untyped_storage().data_ptr() == w.untyped_storage().data_ptr()


def test_stacked_forward_and_grads_equal_concatenation():
    a = _actor(1)
    x = torch.randn(3, 7, 24)
    out = a.forward_sequence(x)
    loss = out[1].square().sum() + out[3].sum() + out[2].sum()
    g = torch.autograd.grad(loss, list(a.parameters()), allow_unused=True)
    # the same module through the concatenating path
    b = copy.deepcopy(a)
    b.__dict__["_stacked"] = None
    out_b = b.forward_sequence(x)
    for u, v in zip(out[:6], out_b[:6]):
        assert torch.equal(u, v)
    loss_b = out_b[1].square().sum() + out_b[3].sum() + out_b[2].sum()
    g_b = torch.autograd.grad(loss_b, list(b.parameters()), allow_unused=True)
    for u, v in zip(g, g_b):
        assert (u is None and v is None) or torch.equal(u, v)


def test_deepcopy_to_and_load_state_dict_restack():
    a = _actor(2)
    b = copy.deepcopy(a)
    assert not b.__dict__["_stacked"].intact()          # a deepcopy gives the Parameters own storages
    x = torch.randn(2, 5, 24)
    assert torch.equal(b.forward_sequence(x)[1], a.forward_sequence(x)[1])   # detected and re-stacked
    assert b.__dict__["_stacked"].intact()
    c = _actor(3).to(torch.float32)
    assert c.__dict__["_stacked"].intact()              # .to() re-stacks
    c.load_state_dict(a.state_dict())
    assert c.__dict__["_stacked"].intact()              # load_state_dict copies in place
    assert torch.equal(c.__dict__["_stacked"].W, a.__dict__["_stacked"].W)


def test_optimizer_steps_update_the_stacked_storage():
    a = _actor(4)
    opt = torch.optim.Adam(a.parameters(), lr=1e-2)
    x = torch.randn(2, 4, 24)
    before = a.__dict__["_stacked"].W.clone()
    a.forward_sequence(x)[1].sum().backward()
    opt.step()
    st = a.__dict__["_stacked"]
    assert st.intact() and not torch.equal(st.W, before)
    assert torch.equal(st.W[0], a.option_value_heads[0].weight.detach()[0])


def test_rsa_qkv_stacked_equals_concatenation():
    torch.manual_seed(5)
    rsa = PN.ResidualSelfAttention(128, 4)
    w, b = rsa.qkv_params(True)
    assert torch.equal(w, torch.cat([rsa.fc_q.weight, rsa.fc_k.weight, rsa.fc_v.weight]))
    assert torch.equal(b, torch.cat([rsa.fc_q.bias, rsa.fc_k.bias, rsa.fc_v.bias]))
    w.sum().backward()
    assert torch.equal(rsa.fc_k.weight.grad, torch.ones_like(rsa.fc_k.weight))


def test_two_stream_stages_match_one_stream_at_a_time():
    a = _actor(6)
    B, L = 3, 6
    obs = torch.randn(B, L, 24)
    nxt = torch.randn(B * L, 1, 24)
    s0 = tuple(torch.randn(1, B, a.hidden_size) * 0.3 for _ in range(2))
    s1 = tuple(torch.randn(1, B * L, a.hidden_size) * 0.3 for _ in range(2))
    (ai, ac), (ni, nc) = a.manager_stages([(obs, s0), (nxt, s1)])
    outs = PN.lstm_sequences([ai, ni])
    (ai, ac), (ni, nc) = a.option_stages([ac, nc], [outs[0], outs[1]])
    opt = PN.lstm_sequences([ai, ni])
    seq_out, next_out = a.head_stages([ac, nc], [opt[0], opt[1]], with_state=(True, False))
    ref_seq = a.forward_sequence(obs, s0)
    ref_next = a.forward_sequence(nxt, s1)
    for u, v in zip(seq_out[:6], ref_seq[:6]):
        assert torch.allclose(u, v, rtol=1e-5, atol=1e-6)
    for u, v in zip(next_out[:6], ref_next[:6]):
        assert torch.allclose(u, v, rtol=1e-5, atol=1e-6)
    assert next_out[6] is None and seq_out[6] is not None
