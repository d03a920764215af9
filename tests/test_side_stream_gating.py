"""When an optimizer step runs its critic branch on a side stream: CUDA, one process
(a gradient all-reduce keeps one collective order on one stream), and the environment switches
SWARM_CRITIC_STREAM (every trainer) / SWARM_OC2_CRITIC_STREAM (OC2 alone) over each class's
default (POCA off, fixed-option OC on, OC2 on). CPU only: torch.cuda.Stream is stubbed, so no
stream is created; the GPU graph tests run the branches themselves."""

import pytest
import torch


class _Comm:
    def __init__(self, active):
        self.active = active


def _probe(cls, device="cuda", active=False):
    o = cls.__new__(cls)           # no __init__: only the attributes the gate reads
    o.device = torch.device(device)
    o.comm = _Comm(active)
    o.critic_comm = _Comm(active)
    return o


def _gate(o):
    fn = getattr(o, "_critic_side_stream", None) or o._side_stream
    return fn()


@pytest.fixture
def classes(monkeypatch):
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.option_critic_trainer import FixedOptionCriticTrainer
    from SwarmACB_isaac.agents.poca_trainer import POCATrainer

    monkeypatch.setattr(torch.cuda, "Stream", lambda dev: ("side", dev))
    for k in ("SWARM_CRITIC_STREAM", "SWARM_OC2_CRITIC_STREAM"):
        monkeypatch.delenv(k, raising=False)
    return {"poca": POCATrainer, "oc": FixedOptionCriticTrainer, "oc2": LearnedOptionCriticTrainer}


def test_class_defaults(classes):
    assert _gate(_probe(classes["poca"])) is None
    assert _gate(_probe(classes["oc"])) == ("side", torch.device("cuda"))
    assert _gate(_probe(classes["oc2"])) == ("side", torch.device("cuda"))


def test_one_stream_per_trainer(classes):
    o = _probe(classes["oc"])
    assert _gate(o) is _gate(o)


@pytest.mark.parametrize("kind", ["poca", "oc", "oc2"])
def test_never_on_cpu_or_with_a_collective(classes, monkeypatch, kind):
    monkeypatch.setenv("SWARM_CRITIC_STREAM", "1")
    assert _gate(_probe(classes[kind], device="cpu")) is None
    assert _gate(_probe(classes[kind], active=True)) is None
    assert _gate(_probe(classes[kind])) is not None


def test_environment_overrides(classes, monkeypatch):
    monkeypatch.setenv("SWARM_CRITIC_STREAM", "0")
    for kind in ("poca", "oc", "oc2"):
        assert _gate(_probe(classes[kind])) is None, kind
    monkeypatch.setenv("SWARM_OC2_CRITIC_STREAM", "1")       # OC2's own switch wins for OC2
    assert _gate(_probe(classes["oc2"])) is not None
    assert _gate(_probe(classes["oc"])) is None
    monkeypatch.setenv("SWARM_CRITIC_STREAM", "1")
    monkeypatch.setenv("SWARM_OC2_CRITIC_STREAM", "0")
    assert _gate(_probe(classes["oc2"])) is None
    assert _gate(_probe(classes["poca"])) is not None
