"""PPO optimizer steps replayed from a HIP graph.

A trainer's optimizer step (forward of every network over one minibatch, the
loss, backward and Adam) is a few hundred small kernels whose launch cost on
the host exceeds their GPU time at the ML-Agents minibatch sizes. `GraphedStep`
runs the first steps of a trainer eagerly (they warm up the allocator, the
library handles and the optimizer state, and they ARE training steps), then
captures the step once with torch.cuda.graph over static copies of the
minibatch tensors and replays it for every later minibatch of the same
structure. A minibatch of another structure (the last, ragged one of an epoch)
runs eagerly. The step function must not synchronise with the host; its
Python-side constants (clip epsilon, entropy beta, learning rate) are part of
the capture, so `GraphedStep.key` holds them and a new key recaptures.

The optimizers are switched to `capturable=True` (their step counters live on
the device); the same kernels then run eagerly and in the graph, so a graphed
update equals the eager one (tests/test_gpu_graph_step.py).
"""

from __future__ import annotations

import gc
import os
import traceback
import warnings

import torch

# SWARM_GRAPHS=0 forces eager steps
ENABLED = os.environ.get("SWARM_GRAPHS", "1") != "0"
# Multi-rank steps on the RCCL ("nccl") backend are captured too (SWARM_GRAPHS_DIST=0 keeps
# them eager): the flat-gradient all-reduce and the loss-denominator all-reduces go into the
# graph (RCCL collectives are stream-ordered and capturable; gloo's host round trips are not).
# On by default since round 4: on MI355X a world-1 RCCL group running every collective of the
# multi-rank update eagerly, then captured and replayed, gives the eager update bit for bit
# (tests/test_gpu_rccl_graph.py; two ranks need two GPUs, which one process never gets here).
# Every rank reports whether its steps were graphed (Trainer.step_path). Whether a capture
# succeeded is agreed on by all ranks before the first replay (one MIN all-reduce of a flag,
# outside the graph): if any rank could not capture, every rank drops its graph and runs its
# steps eagerly, so no rank replays a captured collective that another rank issues eagerly.
DIST_ENABLED = os.environ.get("SWARM_GRAPHS_DIST", "1") != "0"


def make_capturable(optimizers, device: torch.device):
    """capturable=True for every param group; existing step counters move to the device."""
    for opt in optimizers:
        for pg in opt.param_groups:
            pg["capturable"] = True
        for st in opt.state.values():
            s = st.get("step")
            if isinstance(s, torch.Tensor) and s.device != device:
                st["step"] = s.to(device=device, dtype=torch.float32)


def all_ranks_agree(ok: bool) -> bool:
    """True iff `ok` holds on every rank of the default process group (one MIN all-reduce of a
    flag, issued eagerly on the current stream); `ok` itself without a multi-rank group."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() < 2:
        return ok
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


class GraphedStep:
    """fn(batch: dict[str, Tensor]) -> Tensor (detached per-step outputs)."""

    def __init__(self, fn, warmup: int = 2):
        self.fn = fn
        self.warmup = warmup
        self.eager_done = 0
        self.graph = None
        self.sig = None
        self.key = None
        self.static = None
        self.out = None
        self.replays = 0
        self.failed = False

    @staticmethod
    def signature(batch: dict):
        return tuple((k, tuple(v.shape), v.dtype, v.device) for k, v in sorted(batch.items()))

    def reset(self, key=None):
        """Drop the captured graph (new constants); later steps recapture without warmup."""
        self.graph = None
        self.static = None
        self.out = None
        self.key = key

    def __call__(self, batch: dict, key=None) -> torch.Tensor:
        if key != self.key:
            self.reset(key)
        sig = self.signature(batch)
        if self.graph is not None and sig == self.sig:
            if hasattr(batch, "gather_into") and batch.keys() == self.static.keys():
                batch.gather_into(self.static)   # one gather launch into the static inputs
            else:
                for k, v in batch.items():
                    self.static[k].copy_(v)
            self.graph.replay()
            self.replays += 1
            return self.out
        if self.eager_done < self.warmup or (self.graph is not None and sig != self.sig):
            # warm-up (side stream, as torch.cuda.graph requires) or a minibatch of another shape
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.fn(batch)
            torch.cuda.current_stream().wait_stream(s)
            self.eager_done += 1
            return out
        if self.failed:
            return self.fn(batch)
        # capture this structure, then replay it for this minibatch. Capture records and
        # does not execute, so a step that cannot be captured (an op that synchronises)
        # leaves the parameters untouched: it then runs eagerly, as do all later steps.
        self.static = {k: v.clone() for k, v in batch.items()}
        self.sig = sig
        self.graph = torch.cuda.CUDAGraph()
        ok = True
        # no cyclic garbage collection inside the capture: an unreachable CUDAGraph of an earlier
        # runner destroyed while a stream is capturing aborts the process (torch.cuda.graph collects
        # once before it begins)
        gc_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(self.graph):
                self.out = self.fn(self.static)
        except RuntimeError as e:   # torch.AcceleratorError derives from RuntimeError
            where = "".join(traceback.format_exception(e)[-8:-1])
            warnings.warn(f"optimizer step not capturable, running eagerly: {e}\n{where}")
            ok = False
        finally:
            if gc_on:
                gc.enable()
        # every rank takes the same path (captured collectives replayed on one rank and eager
        # ones on another would pair up wrongly and hang)
        if not all_ranks_agree(ok):
            if ok:
                warnings.warn("another rank could not capture its optimizer step: running eagerly like it")
            self.failed = True
            self.reset(self.key)
            torch.cuda.synchronize()
            return self.fn(batch)
        self.graph.replay()
        self.replays += 1
        return self.out
