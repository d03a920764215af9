#!/usr/bin/env python3
"""A/B of two builds of the LSTM sequence kernels (swarm_lstm_seq_forward / _backward): the same
inputs through both libraries, outputs compared BITWISE, then event-timed per call.

    python tools/lstm_ab.py build/variants7/lib_lstm0.so build/variants7/lib_lstmpk.so
"""

import ctypes as C
import json
import sys

import torch


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


def run(lib, n, T, U, seed):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(seed)
    xg = torch.randn(n, T, 4 * U, device=dev, generator=g) * 0.5
    w = torch.randn(4 * U, U, device=dev, generator=g) * 0.2
    h0 = torch.randn(n, U, device=dev, generator=g) * 0.3
    c0 = torch.randn(n, U, device=dev, generator=g) * 0.3
    keep = (torch.rand(n, T, device=dev, generator=g) > 0.05).float()
    dh = torch.randn(n, T, U, device=dev, generator=g)
    dhn = torch.randn(n, U, device=dev, generator=g)
    dcn = torch.randn(n, U, device=dev, generator=g)
    h_out, c_out, act = torch.empty(n, T, U, device=dev), torch.empty(n, T, U, device=dev), torch.empty_like(xg)
    dxg, dh0, dc0 = torch.empty_like(xg), torch.empty_like(h0), torch.empty_like(c0)
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def fwd():
        rc = lib.swarm_lstm_seq_forward(n, T, U, p(xg), p(w), p(h0), p(c0), p(keep), p(h_out), p(c_out), p(act), st)
        assert rc == 0, rc

    def bwd():
        rc = lib.swarm_lstm_seq_backward(n, T, U, p(w), p(c0), p(keep), p(c_out), p(act), p(dh), p(dhn), p(dcn),
                                         p(dxg), p(dh0), p(dc0), st)
        assert rc == 0, rc

    fwd()
    bwd()
    torch.cuda.synchronize()
    outs = [t.clone() for t in (h_out, c_out, act, dxg, dh0, dc0)]
    return outs, timed(fwd), timed(bwd)


def main():
    libs = [C.CDLL(x) for x in sys.argv[1:3]]
    ok = True
    for (n, T, U) in ((16, 128, 64), (96, 128, 64), (192, 128, 64), (512, 128, 64), (64, 128, 32), (40, 37, 48),
                      (8, 5, 16), (3000, 1, 64)):
        res = [run(lib, n, T, U, 1234) for lib in libs]
        same = all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(res[0][0], res[1][0]))
        ok &= same
        print(json.dumps({"n": n, "T": T, "U": U, "bitwise_equal": same,
                          "fwd_us": [round(r[1], 2) for r in res], "bwd_us": [round(r[2], 2) for r in res]}),
              flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
