"""The whole-sequence LSTM kernels (swarm_lstm_seq_forward / _backward,
include/swarmtrain.h) against torch's LSTM on the same GPU: the hidden sequence,
the final state and every gradient (input, W_ih, W_hh, both biases, initial
state), unmasked (one nn.LSTM call over the sequence) and masked (the trainers'
per-step loop that zeroes the carried state after episode ends)."""

import pytest
import torch

from SwarmACB_isaac.agents import poca_networks as PN

pytestmark = pytest.mark.gpu

TOL = dict(rtol=2e-5, atol=2e-6)


def _case(n, T, inp, units, masked, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    lstm, _ = PN._mlagents_lstm(inp, 2 * units)
    with torch.no_grad():
        for p in lstm.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 0.1)
    lstm = lstm.to(dev)
    x = (torch.randn(n, T, inp, generator=g)).to(dev)
    h0 = (torch.randn(1, n, units, generator=g) * 0.5).to(dev)
    c0 = (torch.randn(1, n, units, generator=g) * 0.5).to(dev)
    keep = (torch.rand(n, T, generator=g) > 0.2).float().to(dev) if masked else None
    wout = torch.randn(n, T, units, generator=g).to(dev)
    return lstm, x, h0, c0, keep, wout


def _run(fused, lstm, x, h0, c0, keep, wout):
    PN.FUSED_LSTM = fused
    try:
        xs, hs, cs = (t.clone().requires_grad_(True) for t in (x, h0, c0))
        lstm.zero_grad()
        out, (hn, cn) = PN.lstm_sequence(lstm, xs, (hs, cs), keep)
        loss = (out * wout).sum() + (hn ** 2).sum() + (cn * 0.3).sum()
        loss.backward()
        grads = [xs.grad, hs.grad, cs.grad] + [p.grad.clone() for p in lstm.parameters()]
        return [out.detach(), hn.detach(), cn.detach()], grads
    finally:
        PN.FUSED_LSTM = True


@pytest.mark.parametrize("n,T,inp,units,masked", [(16, 128, 128, 64, True), (16, 128, 128, 64, False),
                                                  (96, 128, 128, 64, False), (5, 7, 16, 8, True),
                                                  (12288, 1, 128, 32, False), (2048, 1, 64, 64, True),
                                                  (511, 1, 64, 64, False), (3, 2, 4, 1, True)])
def test_lstm_sequence_matches_torch(gpu_device, n, T, inp, units, masked):
    case = _case(n, T, inp, units, masked, gpu_device)
    outs_k, grads_k = _run(True, *case)
    outs_t, grads_t = _run(False, *case)
    for a, b in zip(outs_k, outs_t):
        torch.testing.assert_close(a, b, **TOL)
    names = ["x", "h0", "c0", "w_ih", "w_hh", "b_ih", "b_hh"]
    for name, a, b in zip(names, grads_k, grads_t):
        scale = max(1.0, float(b.abs().max()))
        torch.testing.assert_close(a / scale, b / scale, rtol=1e-4, atol=1e-5, msg=name)


def test_lstm_sequence_rejects_wide_units(gpu_device):
    """> 64 units take torch's LSTM (the kernels keep a gate row of W_hh in registers)."""
    from SwarmACB_isaac import _native

    lib = _native.load()
    assert lib.swarm_lstm_seq_forward(1, 1, 65, *([None] * 9)) == -1
    case = _case(4, 3, 8, 96, True, gpu_device)
    outs_k, _ = _run(True, *case)
    outs_t, _ = _run(False, *case)
    torch.testing.assert_close(outs_k[0], outs_t[0])


def test_lstm_sequences_batch_equals_single_launches(gpu_device):
    """lstm_sequences: three independent recurrences (different sequence counts, with and
    without the keep mask) in one swarm_lstm_seq_*_batch launch each way give bit for bit
    the outputs and gradients of one launch per recurrence."""
    cases = [_case(16, 128, 128, 64, True, gpu_device, seed=1), _case(40, 128, 128, 64, False, gpu_device, seed=2),
             _case(7, 128, 64, 64, True, gpu_device, seed=3)]

    def run(batched):
        for lstm, *_ in cases:
            lstm.zero_grad()
        ins = [[t.clone().requires_grad_(True) for t in (x, h0, c0)] for _, x, h0, c0, _, _ in cases]
        items = [(c[0], i[0], (i[1], i[2]), c[4]) for c, i in zip(cases, ins)]
        res = PN.lstm_sequences(items) if batched else [PN.lstm_sequence(*it) for it in items]
        loss = sum((out * c[5]).sum() + (hn ** 2).sum() + (cn * 0.3).sum() for (out, (hn, cn)), c in zip(res, cases))
        loss.backward()
        outs = [t.detach() for out, (hn, cn) in res for t in (out, hn, cn)]
        grads = [t.grad for i in ins for t in i] + [p.grad.clone() for c in cases for p in c[0].parameters()]
        return outs, grads

    outs_b, grads_b = run(True)
    outs_s, grads_s = run(False)
    for a, b in zip(outs_b + grads_b, outs_s + grads_s):
        assert torch.equal(a, b)


def test_lstm_batch_rejects_bad_counts(gpu_device):
    from SwarmACB_isaac import _native

    lib = _native.load()
    assert lib.swarm_lstm_seq_forward_batch(0, 8, 64, None, None) == -1
    assert lib.swarm_lstm_seq_forward_batch(_native.LSTM_MAX_BATCH + 1, 8, 64, None, None) == -1
    assert lib.swarm_lstm_seq_backward_batch(1, 8, 65, None, None) == -1


@pytest.mark.parametrize("n,inp,units", [(2048, 128, 64), (12288, 512, 32), (513, 24, 64)])
def test_lstm_single_step_fused_cell_matches_torch(gpu_device, n, inp, units):
    """_lstm_single_step with the fused cell (swarm_lstm_cell / _backward) against nn.LSTM for one
    step: h1, c1 and every gradient (x, h0, c0, W_ih, W_hh, both biases), with c1 unused (its
    gradient unmaterialised) and used."""
    lstm, x, h0, c0, _, _ = _case(n, 1, inp, units, False, gpu_device, seed=n)
    params = list(lstm.parameters())
    for use_c in (False, True):
        xs, hs, cs = (t.clone().requires_grad_(True) for t in (x, h0, c0))
        out, (h1, c1) = PN._lstm_single_step(lstm, xs, (hs, cs))
        loss = (out.square()).sum() + ((c1 * 0.5).sum() if use_c else 0.0)
        g = torch.autograd.grad(loss, [xs, hs, cs] + params)
        xr, hr, cr = (t.clone().requires_grad_(True) for t in (x, h0, c0))
        out_r, (h1_r, c1_r) = lstm(xr, (hr, cr))
        loss_r = (out_r.square()).sum() + ((c1_r * 0.5).sum() if use_c else 0.0)
        g_r = torch.autograd.grad(loss_r, [xr, hr, cr] + params)
        # the gate GEMMs differ from MIOpen's in their reduction order over inp + units terms (up to
        # 544 at the option LSTM's shape): fp32 tolerance of that depth
        assert torch.allclose(out, out_r, rtol=1e-4, atol=1e-5) and torch.allclose(c1, c1_r, rtol=1e-4, atol=1e-5)
        for a, b in zip(g, g_r):
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-4), float((a - b).abs().max())
