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
import hashlib
import json
import math
import os
import socket
import subprocess
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
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (step bench default 4096; passed on to "
                                                            "--collect / --rollout / --critic / --train when given)")
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
    ap.add_argument("--groups", type=int, default=2,
                    help="env groups per GPU: each decision is K launches over contiguous env ranges on K "
                         "streams with no cross-stream ordering (swarm_step_streams): every range's decisions "
                         "form an independent chain, as in the pipelined collector")
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


def lib_sha256(path: str) -> str | None:
    """sha256 of the step library file (the PMC record is tied to the exact build it measured)."""
    try:
        h = hashlib.sha256()
        with open(path, "rb") as f:
            for blk in iter(lambda: f.read(1 << 20), b""):
                h.update(blk)
        return h.hexdigest()
    except OSError:
        return None


def load_pmc(envs: int, sub: int, lib_path: str | None, path: str | None = None,
             groups: int = 1) -> tuple[dict, str | None]:
    """Per-launch HBM bytes and VALU instruction count of the step kernel from the
    committed rocprofv3 PMC record (profiles/pmc_traffic.json, tools/pmc.sh).

    Returns (record, None) only if the record was taken on this workload AND on the very
    library this process loaded (its `lib_sha256` stamp equals the loaded file's sha256);
    otherwise ({}, reason): after any rebuild of the kernels a stale record must not feed the
    bench line, so `traffic` and the VALU figures are then null with the reason stated."""
    path = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return {}, f"no PMC record ({type(e).__name__})"
    if d.get("envs") != envs or d.get("substeps") != sub or d.get("groups", 1) != groups:
        return {}, (f"PMC record taken at envs={d.get('envs')} substeps={d.get('substeps')} "
                    f"groups={d.get('groups', 1)}, not {envs} / {sub} / {groups}")
    want = d.get("lib_sha256")
    have = lib_sha256(lib_path) if lib_path else None
    if not want:
        return {}, "PMC record carries no lib_sha256 stamp"
    if have != want:
        return {}, f"PMC record measured libswarmstep.so sha256 {want[:12]}..., this process loaded {str(have)[:12]}..."
    return d, None


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_plan(gpus: int, env: dict) -> tuple[str, str]:
    """What this process must do for `--gpus N` (no GPU is touched here).

    ("run", "")      : run as one rank (WORLD_SIZE agrees with --gpus, or a single GPU);
    ("spawn", "")    : --gpus N > 1 and no launcher environment: start N rank processes;
    ("refuse", why)  : WORLD_SIZE is set and differs from --gpus (a silent 1-GPU number is
                       the failure this prevents: the line must measure the GPUs it names)."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: need at least 1"
    ws = env.get("WORLD_SIZE")
    if ws is not None and ws != "":
        if int(ws) != gpus:
            return "refuse", f"WORLD_SIZE={ws} but --gpus {gpus}: launch {gpus} ranks or pass --gpus {ws}"
        return "run", ""
    if gpus == 1:
        return "run", ""
    return "spawn", ""


def spawn_ranks(gpus: int, argv: list[str], poll_s: float = 0.2, script: str | None = None) -> int:
    """Start `gpus` fresh rank processes of this script (one per GPU, RANK = LOCAL_RANK = r,
    WORLD_SIZE = gpus, MASTER_ADDR 127.0.0.1 and a free port) BEFORE this process touches any
    GPU, wait for them and return the worst exit status. Rank 0 prints the line. If a rank
    fails, the others (which would wait in a collective forever) are terminated."""
    port = _free_port()
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(poll_s)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or (code if code > 0 else 128 - code)
                for q in live:
                    q.terminate()
    for p in procs:
        p.wait()
    return rc


def prewarm(seconds: float, eng, E: int, dp: int, dev, out, streams=None) -> float:
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
            eng.step(acts[i % 8], dp, out=out, streams=streams)
            i += 1
        torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


def ranks_table(rank: int, dev, dist) -> list[dict]:
    """Every rank's (rank, device index, PCI domain:bus:device) from the live process group, so
    the line shows which physical GPUs ran (one entry per rank)."""
    p = torch.cuda.get_device_properties(dev)
    mine = [rank, dev.index, int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)]
    if dist is None:
        rows = [mine]
    else:
        t = torch.tensor(mine, dtype=torch.int64, device=dev)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        rows = [o.tolist() for o in out]
    return [{"rank": r, "device": d, "pci": f"{a:04x}:{b:02x}:{c:02x}"} for r, d, a, b, c in rows]


def gpu_count(ranks_seen: list[dict]) -> tuple[int, int]:
    """(n_gpus, ranks_per_device) of the live process group: n_gpus counts DISTINCT physical
    devices (PCI addresses), so ranks rehearsed on one card (gloo) can never print a multi-GPU
    line; ranks_per_device is the largest number of ranks that shared one device."""
    per: dict[str, int] = {}
    for r in ranks_seen:
        per[r["pci"]] = per.get(r["pci"], 0) + 1
    return len(per), max(per.values()) if per else 0


def valu_roofline(pmc: dict, pmc_why: str | None, avg_kernel_s: float, hbm_achieved: float, traffic, E: int,
                  dp: int, bytes_per_launch: float, lib_sha: str | None, layout: int = 103, groups: int = 1) -> dict:
    """The step kernel's roofline line: the binding roof is VALU issue
    (~80 op/B against a ~20 op/B ridge), so `bound` is "valu" with the measured SQ_INSTS_VALU
    x 64 lane-ops / kernel time against 256 CUs x 4 SIMD32 x 32 lanes x 2.4 GHz; HBM
    (algorithmic bytes / kernel time, and the PMC traffic) is the secondary roof. The VALU
    count and the traffic come from the PMC record only when it was taken on the loaded
    library (load_pmc); otherwise they are null and `pmc_status` says why."""
    valu_insts = pmc.get("valu_insts_per_decision", pmc.get("valu_insts_per_launch"))
    lane_ops = valu_insts * 64.0 if valu_insts else None
    achieved = lane_ops / avg_kernel_s / 1e12 if lane_ops else None
    return {
        "bound": "valu",
        "achieved": achieved,
        "peak": VALU_PEAK_LANE_OPS / 1e12,
        "unit": "T lane-ops/s",
        "frac": (lane_ops / avg_kernel_s / VALU_PEAK_LANE_OPS) if lane_ops else None,
        "traffic": traffic,
        "valu_insts_per_decision": valu_insts,
        "valu_busy": pmc.get("valu_busy"),
        "sq_wait_any_frac": pmc.get("sq_wait_any_frac"),
        "pmc_status": "ok" if pmc_why is None else pmc_why,
        "pmc_source": "profiles/pmc_traffic.json (rocprofv3 --pmc passes of this workload, tools/pmc.sh), "
                      "stamped with the sha256 of the libswarmstep.so it measured",
        "lib_sha256": lib_sha,
        "kernel": ("step_kernel_pipe<HOMING> (layout 203)" if layout == 203
                   else f"step_kernel<HOMING,ISAAC,continuous,N=20,layout {layout}>"),
        "layout": layout,
        "groups": groups,
        # per decision: the timed region / decisions. With groups > 1 a decision is K launches over
        # env ranges whose chains overlap, so one launch lives longer than this (rocprofv3's
        # per-launch average); the decision's algorithmic bytes / VALU work over the decision's
        # share of the region is the chip-level rate
        "kernel_avg_us": avg_kernel_s * 1e6,
        "secondary": {
            "bound": "hbm",
            "achieved": hbm_achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": hbm_achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_per_agent_step": (traffic / (E * N_AGENTS * dp)) if traffic else None,
            "algorithmic_bytes_per_launch": bytes_per_launch,
        },
    }


def main():
    args = parse()
    if args.rollout or args.critic or args.collect or args.train:
        if args.gpus != 1 and os.environ.get("WORLD_SIZE") is None:
            print("bench.py: --rollout/--critic/--collect/--train are single-GPU measurements; "
                  "pass --gpus 1 (or launch ranks yourself)", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        sys.argv = [sys.argv[0]] + args.rest
        if args.collect and args.groups != 1:
            sys.argv += ["--groups", str(args.groups)]   # the pipelined collector's env groups
        if args.envs is not None:
            sys.argv += ["--envs", str(args.envs)]
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
    # --gpus N decides the world: spawn N ranks here (before any torch.cuda call), run as one
    # rank of a launcher that agrees, or refuse a mismatch
    plan, why = rank_plan(args.gpus, os.environ)
    if plan == "refuse":
        print(f"bench.py: {why}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > 1 and local >= ndev:
        print(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {ndev} GPUs are visible "
              f"(RCCL needs one GPU per rank)", file=sys.stderr, flush=True)
        sys.exit(2)
    # (rank % visible devices) only matters when rehearsing several ranks on one device
    # (--dist-backend gloo: RCCL refuses that)
    local = local % max(1, ndev)
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

    E, dp = args.envs or 4096, args.decision_period
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

    # --groups K: K caller streams; each decision's K range launches go to them with no join, so
    # every range's decisions form an independent chain (the pipelined collector's schedule)
    streams = [torch.cuda.Stream(dev) for _ in range(args.groups)] if args.groups > 1 else None
    torch.cuda.synchronize(dev)
    prewarm_s = prewarm(args.prewarm, eng, E, dp, dev, out, streams)
    for d in range(n_warm):
        eng.step(acts[d], dp, out=out, streams=streams)
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
    graph = None
    if args.graph and streams is not None:
        print("bench.py: --graph with --groups > 1 is not supported", file=sys.stderr, flush=True)
        sys.exit(2)
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
    # the streams the timed launches run on: the current stream, or the K group streams, each of
    # which gets its own gate and start / end events (no cross-stream event inside the region:
    # a fork / join between queues adds signalling latency the short driver run would count)
    run_streams = streams if streams is not None else [stream]
    starts = [torch.cuda.Event(enable_timing=True) for _ in run_streams]
    ends = [torch.cuda.Event(enable_timing=True) for _ in run_streams]
    if gate is not None:
        flag.value = 0
        C.c_uint32.from_address(gate.value + 4).value = 0
        for st_k in run_streams:
            _native.check(eng.lib.swarm_gate_wait(gate, 10_000_000, C.c_void_p(st_k.cuda_stream)), "swarm_gate_wait")
    for st_k, ev in zip(run_streams, starts):
        ev.record(st_k)
    if graph is not None:
        graph.replay()
    else:
        for d in range(n_dec):
            eng.step(acts[n_warm + d], dp, out=out, streams=streams)
    for st_k, ev in zip(run_streams, ends):
        ev.record(st_k)
    t0 = time.perf_counter()
    if gate is not None:
        flag.value = 1
    # the wall clock stops when the host sees every stream's end event complete (a spin on the
    # events: a blocking device synchronize adds a wake-up latency of up to ~80 us, measured on
    # the driver's 4-decision region, profiles/r06/groups/)
    while not all(e.query() for e in ends):
        pass
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    gate_timed_out = False
    if gate is not None:
        # word 1 of the gate buffer: set by gate_kernel when it released on its timeout instead
        # of the host's flag (the host enqueue blocked; the timed launches then started before
        # t0 and the wall clock would miss them)
        gate_timed_out = C.c_uint32.from_address(gate.value + 4).value != 0
        _native.check(eng.lib.swarm_gate_free(gate), "swarm_gate_free")
    # GPU region: earliest start to latest end over the streams (events are device timestamps)
    first = starts[0]
    region_s = (max(first.elapsed_time(e) for e in ends) - min(first.elapsed_time(e) for e in starts)) / 1e3
    avg_kernel_s = region_s / n_dec
    # per stream: its back-to-back launches' region / decisions = the average duration of one of its
    # launches (what rocprofv3 --stats reports per launch; with groups > 1 the streams' launches
    # overlap, so this exceeds the per-decision share avg_kernel_s of the region)
    stream_launch_us = [s_.elapsed_time(e_) * 1e3 / n_dec for s_, e_ in zip(starts, ends)]
    if gate_timed_out or elapsed < 0.98 * region_s:
        print(f"bench.py: rank {rank}: invalid timed region (gate timed out: {gate_timed_out}; wall "
              f"{elapsed * 1e3:.3f} ms vs GPU events {region_s * 1e3:.3f} ms): rerun with fewer --steps",
              file=sys.stderr, flush=True)
        sys.exit(3)
    elapsed = max_over_ranks(elapsed, dev)
    ranks_seen = ranks_table(rank, dev, dist)
    world_live = dist.get_world_size() if dist is not None else 1
    n_gpus, ranks_per_device = gpu_count(ranks_seen)
    total_agent_steps = world_live * E * N_AGENTS * steps
    value = total_agent_steps / elapsed

    if rank == 0:
        bytes_per_launch = ALGO_BYTES_PER_AGENT_STEP * E * N_AGENTS * dp
        achieved = bytes_per_launch / avg_kernel_s / 1e9
        lib_path = getattr(eng.lib, "_name", None)
        pmc, pmc_why = load_pmc(E, dp, lib_path, groups=args.groups)
        # per decision (= per launch when groups = 1): a decision is `groups` launches
        traffic = pmc.get("hbm_bytes_per_decision", pmc.get("hbm_bytes_per_launch"))
        roofline = valu_roofline(pmc, pmc_why, avg_kernel_s, achieved, traffic, E, dp, bytes_per_launch,
                                 lib_sha256(lib_path) if lib_path else None, eng.split_layout(args.groups), args.groups)
        roofline["launch_avg_us_per_stream"] = stream_launch_us
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": n_gpus,
            "ranks": world_live,
            "ranks_per_device": ranks_per_device,
            "ranks_seen": ranks_seen,
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
                "layout": eng.split_layout(args.groups),
                "groups": args.groups,
                "timed_launches": ("one HIP graph of the timed decisions, replayed once" if graph is not None
                                   else "eager launches" if streams is None
                                   else f"eager launches, each decision as {args.groups} env-range launches on "
                                        f"{args.groups} streams without a per-decision join (swarm_step_streams)") + (", enqueued behind a stream gate released after the "
                                                             "enqueue" if gate is not None else ""),
                "parallelism": f"env-sharded x{world}",
                "agent_decisions_per_s": value / dp,
            },
            "roofline": roofline,
            "cpu_baseline": cpu_baseline(args.cpu_seconds if world_live == 1 else 0.0, E),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
