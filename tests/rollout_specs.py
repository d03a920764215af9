"""Shared helpers of the rollout-buffer tests: the golden fixture and the batch
field lists of the product buffers (the fixture pins both)."""

from __future__ import annotations

import os

import numpy as np

from SwarmACB_isaac.agents import learned_option_critic_buffer as LOB
from SwarmACB_isaac.agents import option_critic_buffer as OCB
from SwarmACB_isaac.agents import poca_buffer as PB
from SwarmACB_isaac.agents._rollout import batch_starts

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rollout", "rollout_buffers.npz")

_META = ("ids", "mask")


def load_golden():
    return np.load(GOLDEN)


def _data(spec):
    return [s for s in spec if s[2] not in _META]


SEQ_SPECS = {
    "poca_": _data(PB.SEQ_SPEC + PB.SEQ_SPEC_CRITIC_MEMORY),
    "oc_": _data(OCB.SEQ_SPEC),
    "loc_": _data(LOB.SEQ_SPEC),
}
FULL_SEQ_SPECS = {"poca_": PB.SEQ_SPEC + PB.SEQ_SPEC_CRITIC_MEMORY, "oc_": OCB.SEQ_SPEC, "loc_": LOB.SEQ_SPEC}
FLAT_SPEC = _data(PB.FLAT_SPEC)
BUFFER_CLASSES = {"poca_": PB.POCARolloutBuffer, "oc_": OCB.FixedOptionRolloutBuffer,
                  "loc_": LOB.LearnedOptionRolloutBuffer}
ADV_SETS = {"poca_": [("baselines", "advantages")], "poca2_": [("baselines", "advantages")],
            "oc_": [("baselines", "advantages")], "long_": [("baselines", "advantages")],
            "loc_": [("action_baselines", "action_advantages"), ("option_baselines", "option_advantages")]}


def golden_arrays(g, prefix):
    """attr -> array[:T] of one recorded buffer (inputs plus the reference's
    returns / advantages)."""
    out = {k[len(prefix) + 3:]: g[k] for k in g.files if k.startswith(prefix + "in_")}
    for k in ("returns", "advantages", "action_advantages", "option_advantages"):
        if prefix + k in g.files:
            out[k] = g[prefix + k]
    return out


def batch_slices(n, per_batch):
    return [(a, min(a + per_batch, n)) for a in batch_starts(n, per_batch)]
