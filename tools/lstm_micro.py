#!/usr/bin/env python3
"""Event-timed swarm_lstm_seq_forward / _backward per call over sequence counts n and
lengths T (units 64, with the per-step keep mask as the trainers pass it), to see the
per-recurrence-step latency and whether it depends on n."""

import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "swarmacb-isaaclab_amd"))

from SwarmACB_isaac import _native  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    lib = _native.load()
    dev = torch.device("cuda")
    U = 64
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
    for T in (128, 64):
        for n in (16, 48, 96, 256, 512):
            xg = torch.randn(n, T, 4 * U, device=dev) * 0.3
            w = torch.randn(4 * U, U, device=dev) * 0.1
            h0, c0 = torch.zeros(n, U, device=dev), torch.zeros(n, U, device=dev)
            keep = (torch.rand(n, T, device=dev) > 0.01).float()
            h_out, c_out, act = torch.empty(n, T, U, device=dev), torch.empty(n, T, U, device=dev), torch.empty_like(xg)
            dh = torch.randn(n, T, U, device=dev)
            dxg, dh0, dc0 = torch.empty_like(xg), torch.empty_like(h0), torch.empty_like(c0)
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

            def fwd():
                lib.swarm_lstm_seq_forward(n, T, U, p(xg), p(w), p(h0), p(c0), p(keep), p(h_out), p(c_out), p(act), st)

            def bwd():
                lib.swarm_lstm_seq_backward(n, T, U, p(w), p(c0), p(keep), p(c_out), p(act), p(dh), None, None,
                                            p(dxg), p(dh0), p(dc0), st)

            f, b = timed(fwd), timed(bwd)
            print(json.dumps({"T": T, "n": n, "fwd_us": f, "bwd_us": b, "fwd_ns_per_step": f * 1e3 / T,
                              "bwd_ns_per_step": b * 1e3 / T}), flush=True)


if __name__ == "__main__":
    main()
