#!/usr/bin/env python3
"""Benchmark: agent-steps/s of SwarmACB-Homing-v0 (dandelion) on MI355X.

Workload (BASELINE.json configs[1]): SwarmACB-Homing-v0,
dandelion variant (24-D obs, continuous wheels), 20 e-pucks x 4096 envs per
GPU, Isaac-profile step semantics, in-kernel Philox packet loss. Actions are
the ML-Agents initial policy N(0,1) -> clamp(-3,3)/3 per wheel, drawn once per
decision (decision period 5) and held for the 5 env.steps of the decision,
which run as ONE fused kernel launch (every substep still integrates, resolves
contacts, computes rewards/time-outs/auto-reset and writes the 24-D
observation). All actions are generated in HBM before the timed region.

One "step" = one env.step (physics update) of all envs on all GPUs; an
agent-step = one robot advanced by one such step (the reference's own SPS
counts agent-decisions = agent-steps / 5). Multi-GPU: one process per GPU
(torchrun), envs sharded by global index (weak scaling), no collective in the
data path; value = all agent-steps / max-over-ranks time.
"""

from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "swarmacb-isaaclab_amd")
for _p in (ROOT, PKG_DIR):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

METRIC = "agent-steps/sec (20 e-pucks × num_envs) SwarmACB-Homing-v0 at 1/2/4/8 MI355X"
ALGO_BYTES_PER_AGENT_STEP = 129.0   # read x,y,yaw+action 20 B, write x,y,yaw+obs 108 B, ~1 B counters
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9   # MI355X_MICROARCH.md: 256 CUs, 4 SIMD32 each, 2.4 GHz max clock
N_AGENTS = 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1200, help="timed env.steps (physics updates)")
    ap.add_argument("--warmup", type=int, default=50, help="untimed env.steps")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--decision-period", type=int, default=5)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL, one GPU per rank) or gloo")
    ap.add_argument("--layout", type=int, default=0,
                    help="kernel work layout (4 = 4 waves share 3 arenas, 103 = 3 lanes per robot; 0 = library default)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU-baseline sample budget per leg (0 = skip)")
    ap.add_argument("--prewarm", type=float, default=1.0,
                    help="seconds of untimed step launches on the timed engine before the warm-up "
                         "(steady clocks, arenas past the post-spawn contact burst; steps/warmup unchanged)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: the timed decisions are captured once as a HIP graph and replayed inside the "
                         "timed region; 0: eager launches")
    ap.add_argument("--gate", type=int, default=1,
                    help="1: the timed launches are enqueued behind a stream gate released after the enqueue "
                         "(swarm_gate_wait); 0: launched as they are enqueued")
    ap.add_argument("--rollout", action="store_true",
                    help="instead of the step: the rollout-buffer kernels at C3 (tools/bench_rollout.py)")
    ap.add_argument("--critic", action="store_true",
                    help="instead of the step: the fused critic attention at C3 (tools/bench_critic.py)")
    ap.add_argument("--collect", action="store_true",
                    help="instead of the step: the whole C3 rollout decision loop (tools/bench_collect.py)")
    ap.add_argument("--train", action="store_true",
                    help="instead of the step: the C3/C4/C5 trainers' rollout + update (tools/bench_train.py)")
    args, rest = ap.parse_known_args()
    args.rest = rest
    return args


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_worker(args):
    """One process of the CPU baseline: its own oracle instance stepping `E` envs for `budget_s`."""
    E, budget_s, seed = args
    import numpy as np

    from oracle import oracle as O

    env = O.OracleEnv("homing", "isaac", E, N_AGENTS, 24, False, 1200)
    O.seed(seed)
    env.reset_all()
    rng = np.random.default_rng(seed)
    steps, t0 = 0, time.perf_counter()
    while True:
        a = (np.clip(rng.normal(size=(E, N_AGENTS, 2)), -3, 3) / 3).astype(np.float32)
        for _ in range(5):
            env.step(a)
            steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            return E * N_AGENTS * steps, el


CPU_SAMPLE_ENVS = (1, 64, 1024, 4096)   # the reference's CPU step at E = 1 / 64 / 1024 / 4096


def _cpu_share() -> tuple[int, int]:
    """(worker processes, CPUs in the affinity set). The GPU box's job share is the pool's
    OMP_NUM_THREADS (16 per GPU there): its affinity set lists every CPU of the host
    (256), but a pool larger than the share oversubscribes the job's quota, so the
    all-cores leg runs one process per CPU of the share."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return max(1, min(aff, share)), aff


def cpu_baseline(budget_s: float, envs: int) -> dict | None:
    """Reference-equivalent CPU step (the C restatement in oracle/) on bounded samples at
    E = 1, 64, 1024, 4096 envs: 1 thread, then one process per CPU of the job's share, each
    stepping its own slice of the E envs. `value` is the all-cores rate at the bench's E."""
    if budget_s <= 0:
        return None
    import multiprocessing as mp

    from oracle import oracle as O

    O.build()
    cores, aff = _cpu_share()
    sizes = sorted(set(CPU_SAMPLE_ENVS) | {envs})
    per_leg = max(0.5, budget_s / (2 * len(sizes)))
    table, value, one_at_e = [], None, None
    with mp.get_context("fork").Pool(cores) as pool:
        for E in sizes:
            n1, el1 = _oracle_worker((E, per_leg, 0))
            procs = max(1, min(cores, E))
            res = pool.map(_oracle_worker, [(E // procs + (1 if k < E % procs else 0), per_leg, 1 + k)
                                            for k in range(procs)])
            allv = sum(n / el for n, el in res)
            table.append({"envs": E, "one_thread": n1 / el1, "all_cores": allv, "processes": procs})
            if E == envs:
                value, one_at_e = allv, n1 / el1
    return {"value": value, "unit": "agent-steps/s", "cores": cores, "kind": "port", "one_thread": one_at_e,
            "by_envs": table, "cpu_model": _cpu_model(), "host_cpus_visible": os.cpu_count(),
            "affinity_cpus": aff,
            "sample": f"oracle/swarm_oracle.c (C restatement of the reference step, pinned by tests/golden) "
                      f"Homing dandelion isaac profile, policy N(0,1)->clamp/3 per 5-step decision, "
                      f"E in {list(sizes)} envs x 20 e-pucks, {per_leg:.1f} s per leg: 1 thread, then "
                      f"{cores} processes (the job's CPU share; the affinity set lists {aff}) each stepping "
                      f"E / {cores} envs; value = all-cores rate at E = {envs}"}


def load_pmc(envs: int, sub: int) -> dict:
    """Per-launch HBM bytes and VALU instruction count of the step kernel from the
    committed rocprofv3 PMC record (profiles/pmc_traffic.json, tools/pmc.sh), if it
    was taken on this workload."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    if d.get("envs") != envs or d.get("substeps") != sub:
        return {}
    return d


def prewarm(seconds: float, eng, E: int, dp: int, dev, out) -> float:
    """Untimed launches of the same workload (same step, same action distribution) on the
    timed engine itself for `seconds`, right before the warm-up decisions: the clocks are
    up and the arenas are past the contact burst that follows a spawn when the timed
    region starts, however few launches it has."""
    if seconds <= 0:
        return 0.0
    g = torch.Generator(device=dev).manual_seed(12345)
    acts = (torch.randn(8, E, N_AGENTS, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            eng.step(acts[i % 8], dp, out=out)
            i += 1
        torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


def main():
    args = parse()
    if args.rollout or args.critic or args.collect or args.train:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        sys.argv = [sys.argv[0]] + args.rest
        if args.train:
            import bench_train

            bench_train.main()
        elif args.collect:
            import bench_collect

            bench_collect.main()
        elif args.rollout:
            import bench_rollout

            bench_rollout.main()
        else:
            import bench_critic

            bench_critic.main()
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; (rank % visible devices) only matters when rehearsing
    # several ranks on one device (with --dist-backend gloo: RCCL refuses that)
    local = local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    from SwarmACB_isaac import _native
    from SwarmACB_isaac.engine import SwarmEngine
    from SwarmACB_isaac.shard import EnvShard, max_over_ranks

    E, dp = args.envs, args.decision_period
    shard = EnvShard.weak(E, rank, world)     # weak scaling: E envs per GPU, keyed by global env id
    eng = SwarmEngine("homing", "isaac", E, N_AGENTS, 24, False, 1200, 1, shard.env_offset, args.seed, dev,
                      layout=args.layout or None)
    obs, rew, tr = eng.reset()
    out = (obs, rew, tr)

    n_warm = max(1, math.ceil(args.warmup / dp))
    n_dec = max(1, args.steps // dp)
    steps = n_dec * dp
    # synthetic policy actions for every decision, resident in HBM before timing
    g = torch.Generator(device=dev).manual_seed(args.seed * 1000 + rank)
    acts = (torch.randn(n_warm + n_dec, E, N_AGENTS, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()

    prewarm_s = prewarm(args.prewarm, eng, E, dp, dev, out)
    for d in range(n_warm):
        eng.step(acts[d], dp, out=out)
    torch.cuda.synchronize(dev)

    # HIP events bracket the whole timed region (not every launch: each event is a packet of
    # its own in the stream, and a pair per decision added ~5 us of GPU-side gap per launch);
    # the per-launch average includes the gaps between back-to-back launches, so it is an
    # upper bound on the kernel's own duration.
    # --gate 1 (default): the timed region is enqueued behind a stream gate (swarm_gate_wait: a
    # one-wave kernel that waits for a host-coherent flag) and released after the enqueue, so
    # the launches run back to back from the release on and the events see only the GPU's own
    # work; with few timed launches (the driver's 4) eager events otherwise also counted the
    # host's launch latency after the first event (BENCH_r03: 68.3 vs 59.5 us rocprofv3). The
    # wall clock starts at the release and stops after the synchronize: exactly the K steps.
    # --graph 1: the timed decisions are captured once as a HIP graph and replayed behind the
    # gate (the timing events stay outside the capture: ROCm refuses external events in one).
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph = None
    if args.graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for d in range(n_dec):
                eng.step(acts[n_warm + d], dp, out=out)
    gate = None
    if args.gate:
        gate = C.c_void_p()
        _native.check(eng.lib.swarm_gate_alloc(C.byref(gate)), "swarm_gate_alloc")
        flag = C.c_uint32.from_address(gate.value)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if gate is not None:
        flag.value = 0
        _native.check(eng.lib.swarm_gate_wait(gate, 10_000_000, C.c_void_p(stream.cuda_stream)), "swarm_gate_wait")
    ev0.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for d in range(n_dec):
            eng.step(acts[n_warm + d], dp, out=out)
    ev1.record(stream)
    t0 = time.perf_counter()
    if gate is not None:
        flag.value = 1
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if gate is not None:
        _native.check(eng.lib.swarm_gate_free(gate), "swarm_gate_free")
    avg_kernel_s = ev0.elapsed_time(ev1) / n_dec / 1e3
    elapsed = max_over_ranks(elapsed, dev)
    total_agent_steps = world * E * N_AGENTS * steps
    value = total_agent_steps / elapsed

    if rank == 0:
        bytes_per_launch = ALGO_BYTES_PER_AGENT_STEP * E * N_AGENTS * dp
        achieved = bytes_per_launch / avg_kernel_s / 1e9
        pmc = load_pmc(E, dp)
        traffic = pmc.get("hbm_bytes_per_launch")
        valu = None
        if pmc.get("valu_insts_per_launch"):
            # VALU issue roof: 256 CUs x 4 SIMD32 x 32 lanes/clk x 2.4 GHz (a wave64 VALU op = 64 lane-ops)
            lane_ops = pmc["valu_insts_per_launch"] * 64.0
            peak = VALU_PEAK_LANE_OPS
            valu = {"achieved": lane_ops / avg_kernel_s / 1e12, "peak": peak / 1e12, "unit": "T lane-ops/s",
                    "frac": lane_ops / avg_kernel_s / peak,
                    "valu_insts_per_launch": pmc["valu_insts_per_launch"],
                    "valu_insts_source": "profiles/pmc_traffic.json (SQ_INSTS_VALU pass); not measured in this process"}
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": n_warm * dp,
            "prewarm_s": prewarm_s,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (Homing spawn + in-kernel Philox packet loss; actions N(0,1)->clamp(-3,3)/3 per decision)",
            "config": {
                "workload": "SwarmACB-Homing-v0 dandelion, Isaac-profile env.step, 20 e-pucks x "
                            f"{E} envs per GPU, decision period {dp} fused per launch",
                "num_envs_per_gpu": E,
                "num_agents": N_AGENTS,
                "global_envs": world * E,
                "decision_period": dp,
                "layout": args.layout or "default",
                "timed_launches": ("one HIP graph of the timed decisions, replayed once" if graph is not None
                                   else "eager launches") + (", enqueued behind a stream gate released after the "
                                                             "enqueue" if gate is not None else ""),
                "parallelism": f"env-sharded x{world}",
                "agent_decisions_per_s": value / dp,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": "profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes of "
                                  "this workload, tools/pmc.sh); not measured in this process" if traffic else None,
                "traffic_per_agent_step": (traffic / (E * N_AGENTS * dp)) if traffic else None,
                "valu": valu,
                "kernel": "step_kernel<HOMING,ISAAC,continuous,N=20,W>",
                "kernel_avg_us": avg_kernel_s * 1e6,
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "cpu_baseline": cpu_baseline(args.cpu_seconds if world == 1 else 0.0, E),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
