"""Per-wave timing of the production step kernel (diagnostic build only).

Build a variant with -DSWARM_WAVE_TIMING=1 (tools/variants.sh build), then on the GPU box:
    SWARMSTEP_LIB=build/variants/lib_wt.so python3 tools/wave_timing.py
It runs the bench workload (C2: Homing dandelion, 4096 envs x 20 e-pucks, 5 substeps per
launch), reads each wave's start / end clocks and hardware slot after single launches, and
prints how the kernel's span splits into wave lifetimes: whether the launch is bound by the
average wave (throughput) or by its slowest arenas (tail), and what the slow arenas hold.
"""

from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "swarmacb-isaaclab_amd"))

from SwarmACB_isaac.engine import SwarmEngine  # noqa: E402


PHASES = ["act_int", "solve", "resolve", "reward", "publish", "prox", "rab", "combine", "finish",
          "push_pub", "push_cand", "push_pairs", "push_xchg"]   # swarm_step_impl.h WtPhase


def pct(a, qs=(0, 10, 50, 90, 99, 100)):
    return {f"p{q}": float(np.percentile(a, q)) for q in qs}


def pair_counts(x, y, r):
    d2 = (x[:, :, None] - x[:, None, :]) ** 2 + (y[:, :, None] - y[:, None, :]) ** 2
    n = x.shape[1]
    m = (d2 < r * r) & ~np.eye(n, dtype=bool)[None]
    return m.sum(axis=(1, 2)) // 2


def main():
    E, N, dp = int(os.environ.get("WT_ENVS", "4096")), 20, 5
    dev = torch.device("cuda:0")
    eng = SwarmEngine("homing", "isaac", E, N, 24, False, 1200, 1, 0, 1, dev)
    read = eng.lib.swarm_debug_wave_log
    read.restype = C.c_int
    read.argtypes = [C.c_void_p, C.c_size_t]
    out = eng.reset()
    g = torch.Generator(device=dev).manual_seed(1000)
    acts = (torch.randn(400, E, N, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()
    for d in range(300):
        eng.step(acts[d], dp, out=out)
    torch.cuda.synchronize(dev)
    buf = np.zeros((E, 7, 4), np.uint32)
    rows = []
    prev_life = prev_pred = None
    prev_simd_end = prev_simd_key = None
    for d in range(300, 310):
        st = eng.dump_state()
        eng.step(acts[d], dp, out=out)
        torch.cuda.synchronize(dev)
        assert read(buf.ctypes.data, buf.nbytes) == 0
        life = buf[:, 0, 1].astype(np.int64)                  # shader clocks
        w0 = buf[:, 1, 0].astype(np.int64)
        w1 = buf[:, 1, 1].astype(np.int64)
        w1 = np.where(w1 < w0, w1 + (1 << 32), w1)
        t0 = w0.min()
        span = (w1.max() - t0) * 10.0                         # ns (100 MHz wall clock)
        life_ns = (w1 - w0) * 10.0
        clk = life / np.maximum(life_ns, 1) * 1e3             # MHz per wave
        hw, xcc = buf[:, 0, 2], buf[:, 0, 3] & 0xF
        simd = (xcc.astype(np.int64) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)
        _, inv, cnt = np.unique(simd, return_inverse=True, return_counts=True)
        simd_end = np.zeros(cnt.size)
        np.maximum.at(simd_end, inv, (w1 - t0) * 10.0)
        x, y = st["pos"][..., 0], st["pos"][..., 1]
        contacts = pair_counts(x, y, 0.0705)
        rab = pair_counts(x, y, 0.60)
        slow = np.argsort(life_ns)[-max(1, E // 100):]
        rows.append({
            "launch": d, "span_us": span / 1e3, "life_us": pct(life_ns / 1e3),
            "mean_life_over_span": float(life_ns.mean() / span),
            "start_us": pct((w0 - t0) * 10.0 / 1e3), "end_us": pct((w1 - t0) * 10.0 / 1e3),
            "clock_mhz": pct(clk, (50,)), "waves_per_simd": pct(cnt, (0, 50, 100)),
            "simd_end_us": pct(simd_end / 1e3, (0, 50, 100)),
            "corr_life_contact_pairs": float(np.corrcoef(life_ns, contacts)[0, 1]),
            "corr_life_rab_pairs": float(np.corrcoef(life_ns, rab)[0, 1]),
            "contact_pairs_mean_all_vs_slowest1pct": [float(contacts.mean()), float(contacts[slow].mean())],
            "rab_pairs_mean_all_vs_slowest1pct": [float(rab.mean()), float(rab[slow].mean())],
        })
        # wave-max loop trips per launch: push calls, contact pair terms, kept RAB terms,
        # near wall segments, proximity discs
        work = {"push": buf[:, 1, 2], "pair": buf[:, 1, 3], "rab": buf[:, 2, 0], "seg": buf[:, 2, 1],
                "disc": buf[:, 2, 2]}
        for k, v in work.items():
            v = v.astype(np.float64)
            rows[-1][f"{k}_mean_all_vs_slowest1pct"] = [float(v.mean()), float(v[slow].mean())]
            rows[-1][f"corr_life_{k}"] = float(np.corrcoef(life_ns, v)[0, 1]) if v.std() > 0 else None
        # shader clocks per phase (the push phases are inside "solve"/"resolve"), as a
        # fraction of the wave's life; mean over all waves and over the slowest 1 %
        ph = buf[:, 3:7, :].reshape(E, 16)[:, :len(PHASES)].astype(np.float64)
        lf = np.maximum(life.astype(np.float64), 1.0)
        rows[-1]["phase_frac_mean"] = {k: float((ph[:, i] / lf).mean()) for i, k in enumerate(PHASES)}
        rows[-1]["phase_frac_slowest1pct"] = {k: float((ph[slow, i] / lf[slow]).mean()) for i, k in enumerate(PHASES)}
        rows[-1]["phase_kclk_mean"] = {k: float(ph[:, i].mean() / 1e3) for i, k in enumerate(PHASES)}
        rows[-1]["life_kclk_mean"] = float(life.mean() / 1e3)
        pushes = np.maximum(buf[:, 1, 2].astype(np.float64), 1.0)
        rows[-1]["clk_per_push"] = {k: float((ph[:, PHASES.index(k)] / pushes).mean())
                                    for k in ("push_pub", "push_cand", "push_pairs", "push_xchg")}
        A = np.stack([np.ones(E)] + [w.astype(np.float64) for w in work.values()], 1)
        coef, *_ = np.linalg.lstsq(A, life_ns / 1e3, rcond=None)
        pred = A @ coef
        rows[-1]["fit_us"] = dict(zip(["const"] + list(work), map(float, coef)))
        rows[-1]["fit_r2"] = float(1 - ((life_ns / 1e3 - pred) ** 2).sum() / ((life_ns / 1e3 - life_ns.mean() / 1e3) ** 2).sum())
        # schedule view: which SIMD each block landed on, in what start order, and how far a
        # SIMD's end follows the work of the four arenas it holds
        start = w0 - t0
        order = np.argsort(start, kind="stable")
        rank = np.zeros(E, np.int64)
        for s_ in range(cnt.size):
            blk = np.nonzero(inv == s_)[0]
            rank[blk[np.argsort(start[blk], kind="stable")]] = np.arange(blk.size)
        first = np.arange(E) < cnt.size
        rows[-1]["sched"] = {
            "simds": int(cnt.size),
            "distinct_simds_of_first_blocks": int(np.unique(inv[first]).size),
            "rank_of_block_quarters": [np.bincount(rank[q * E // 4:(q + 1) * E // 4], minlength=4).tolist()
                                       for q in range(4)],
            "start_order_vs_block_corr": float(np.corrcoef(order, np.arange(E))[0, 1]),
            "corr_simd_end_sum_life": float(np.corrcoef(simd_end, np.bincount(inv, life_ns))[0, 1]),
            "corr_simd_end_max_life": float(np.corrcoef(simd_end, np.maximum.reduceat(
                life_ns[np.argsort(inv, kind="stable")], np.r_[0, np.cumsum(cnt)[:-1]]))[0, 1]),
        }
        simd_key = np.unique(simd)
        rows[-1]["sched"]["slowest_simd"] = int(simd_key[int(np.argmax(simd_end))])
        rows[-1]["sched"]["simd_end_by_xcc_us"] = [round(float(simd_end[(simd_key >> 16) == x].mean() / 1e3), 2)
                                                   for x in range(8)]
        if prev_simd_end is not None and prev_simd_key.size == simd_key.size and (prev_simd_key == simd_key).all():
            rows[-1]["sched"]["corr_simd_end_prev_launch"] = float(np.corrcoef(simd_end, prev_simd_end)[0, 1])
        prev_simd_end, prev_simd_key = simd_end.copy(), simd_key
        if prev_life is not None:
            rows[-1]["sched"]["corr_life_prev_launch"] = float(np.corrcoef(life_ns, prev_life)[0, 1])
            rows[-1]["sched"]["corr_pred_prev_launch"] = float(np.corrcoef(pred, prev_pred)[0, 1])
        prev_life, prev_pred = life_ns.copy(), pred.copy()
        print(json.dumps(rows[-1]), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
