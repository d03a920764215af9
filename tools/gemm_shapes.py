#!/usr/bin/env python3
"""Weight-gradient GEMM shapes of the critic's entity rows (dW = dy^T x over R rows):
one library GEMM vs the row-chunked batched GEMM + chunk sum of
poca_networks._SplitKLinear, per chunk size. Event-timed on the current stream."""

import json
import os

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


def split(dy, x, L):
    R = x.shape[0]
    c = R // L
    m = c * L
    dw = torch.bmm(dy[:m].view(c, L, -1).transpose(1, 2), x[:m].view(c, L, -1)).sum(0)
    if m < R:
        dw.addmm_(dy[m:].t(), x[m:])
    return dw


def main():
    dev = torch.device("cuda")
    out = []
    for R in (40960, 81920, 122880):
        for M, K in ((384, 128), (128, 128), (128, 5), (128, 10)):
            dy = torch.randn(R, M, device=dev)
            x = torch.randn(R, K, device=dev)
            ref = dy.t().mm(x)
            row = {"R": R, "M": M, "K": K, "mm_us": timed(lambda: dy.t().mm(x))}
            for L in (256, 512, 1024, 2048, 4096):
                got = split(dy, x, L)
                err = float((got - ref).abs().max() / ref.abs().max())
                row[f"split{L}_us"] = timed(lambda: split(dy, x, L))
                row[f"split{L}_err"] = err
            row["flops"] = 2.0 * R * M * K
            print(json.dumps(row), flush=True)
            out.append(row)


if __name__ == "__main__" and not os.environ.get("GEMM_BIAS"):
    main()


def bias_grads():
    """db = column sums of dy over R rows: the chunked reduction _SplitKLinear uses vs
    alternatives."""
    dev = torch.device("cuda")
    for R, M in ((40960, 384), (81920, 384), (81920, 128), (122880, 128)):
        dy = torch.randn(R, M, device=dev)
        L = 1024
        c = R // L
        ones = torch.ones(c, 1, L, device=dev)
        row = {"R": R, "M": M,
               "chunked_us": timed(lambda: dy.view(c, L, M).sum(dim=1).sum(dim=0)),
               "plain_us": timed(lambda: dy.sum(dim=0)),
               "bmm_ones_us": timed(lambda: torch.bmm(ones, dy.view(c, L, M)).sum(dim=0)),
               "mv_us": timed(lambda: dy.t().mv(torch.ones(R, device=dev)))}
        print(json.dumps(row), flush=True)


if __name__ == "__main__" and os.environ.get("GEMM_BIAS"):
    bias_grads()
