"""The one-step LSTM path of lstm_sequences (poca_networks._lstm_single_step: the OC2 update's
next-state actor pass over >= SINGLE_STEP_ROWS rows) against torch's nn.LSTM on the CPU: the
output, the final state and every gradient. The GPU runs are in test_gpu_lstm_seq.py."""

import torch

from SwarmACB_isaac.agents import poca_networks as PN


def test_single_step_matches_nn_lstm():
    g = torch.Generator().manual_seed(5)
    lstm, _ = PN._mlagents_lstm(24, 2 * 16)
    with torch.no_grad():
        for p in lstm.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 0.1)
    n = 37
    x = torch.randn(n, 1, 24, generator=g)
    h0, c0 = torch.randn(1, n, 16, generator=g) * 0.5, torch.randn(1, n, 16, generator=g) * 0.5
    w = torch.randn(n, 1, 16, generator=g)

    def run(fn):
        lstm.zero_grad()
        ins = [t.clone().requires_grad_(True) for t in (x, h0, c0)]
        out, (hn, cn) = fn(ins)
        ((out * w).sum() + (hn ** 2).sum() + (cn * 0.3).sum()).backward()
        return [out.detach(), hn.detach(), cn.detach()] + [t.grad for t in ins] + [p.grad.clone() for p in lstm.parameters()]

    a = run(lambda i: PN._lstm_single_step(lstm, i[0], (i[1], i[2])))
    b = run(lambda i: lstm(i[0], (i[1], i[2])))
    for u, v in zip(a, b):
        torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)
