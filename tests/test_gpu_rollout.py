"""GPU parity of the rollout-buffer kernels (swarm_rollout.hip via the C ABI in
include/swarmrollout.h, driven through the drop-in buffer classes).

Bit-exact against (1) the reference's own outputs recorded in
tests/golden/rollout/rollout_buffers.npz and (2) the numpy oracle at the BASELINE
configs' sizes (C3: T=240 decisions x 8192 envs x 20 agents)."""

import numpy as np
import pytest
import torch

from oracle import rollout_oracle as RO
import rollout_specs as S
from SwarmACB_isaac.agents import _base
from SwarmACB_isaac.agents import _rollout as R
from SwarmACB_isaac.agents import LearnedOptionRolloutBuffer, POCARolloutBuffer

pytestmark = pytest.mark.gpu

GOLD = S.load_golden()


def _buffer_from_golden(prefix, dev, extra_rows=2):
    T, E, N, L, MB = (int(v) for v in GOLD[f"{prefix}meta"])
    arrays = S.golden_arrays(GOLD, prefix)
    gamma, lam = GOLD[f"{prefix}gamma_lam"]
    cls = S.BUFFER_CLASSES["poca_" if prefix.startswith("poca") else prefix]
    if cls is POCARolloutBuffer:
        buf = cls(T + extra_rows, E, N, obs_dim=4, act_dim=2, state_dim=5, memory_size=3, critic_memory_size=2,
                  gamma=gamma, lam=lam, device=dev)
    elif cls is LearnedOptionRolloutBuffer:
        buf = cls(T + extra_rows, E, N, obs_dim=4, state_dim=5, act_dim=2, memory_size=3, critic_memory_size=2,
                  gamma=gamma, lam=lam, device=dev)
    else:
        buf = cls(T + extra_rows, E, N, obs_dim=4, state_dim=5, memory_size=3, critic_memory_size=2, gamma=gamma,
                  lam=lam, device=dev)
    for name, v in arrays.items():
        if name in ("returns", "advantages", "action_advantages", "option_advantages"):
            continue
        getattr(buf, name)[:T] = torch.as_tensor(v).to(dev)
    buf.ptr = T
    return buf, (T, E, N, L, MB)


@pytest.mark.parametrize("prefix", ["poca_", "poca2_", "oc_", "loc_"])
def test_returns_and_advantages_match_reference(gpu_device, prefix):
    buf, (T, E, N, L, MB) = _buffer_from_golden(prefix, gpu_device)
    buf.compute_returns_and_advantages(torch.as_tensor(GOLD[f"{prefix}last_team_value"]).to(gpu_device))
    np.testing.assert_array_equal(buf.returns[:T].cpu().numpy(), GOLD[f"{prefix}returns"])
    for _b, adv in S.ADV_SETS[prefix]:
        np.testing.assert_array_equal(getattr(buf, adv)[:T].cpu().numpy(), GOLD[f"{prefix}{adv}"])


def test_long_horizon_scan_matches_reference(gpu_device):
    g = {k[len("long_in_"):]: torch.as_tensor(GOLD[k]).to(gpu_device) for k in GOLD.files if k.startswith("long_in_")}
    T, E, N = g["baselines"].shape
    buf = POCARolloutBuffer(T, E, N, obs_dim=4, act_dim=1, device=gpu_device)
    for k, v in g.items():
        getattr(buf, k).copy_(v)
    buf.ptr = T
    buf.compute_returns_and_advantages(torch.as_tensor(GOLD["long_last_team_value"]).to(gpu_device))
    np.testing.assert_array_equal(buf.returns.cpu().numpy(), GOLD["long_returns"])
    np.testing.assert_array_equal(buf.advantages.cpu().numpy(), GOLD["long_advantages"])


def _fixed_perm(monkeypatch, perm, dev):
    calls = []

    def fake(n, device=None, **kw):
        calls.append(n)
        assert n == len(perm), (n, len(perm))
        return torch.as_tensor(perm, dtype=torch.int64).to(dev)

    monkeypatch.setattr(_base.torch, "randperm", fake)
    return calls


@pytest.mark.parametrize("prefix", ["poca_", "oc_", "loc_"])
@pytest.mark.parametrize("budget", [256 << 20, 1])  # one launch for all batches / one launch per batch
def test_sequence_batches_match_reference(gpu_device, monkeypatch, prefix, budget):
    buf, (T, E, N, L, MB) = _buffer_from_golden(prefix, gpu_device)
    for _b, adv in S.ADV_SETS[prefix]:
        getattr(buf, adv)[:T] = torch.as_tensor(GOLD[f"{prefix}{adv}"]).to(gpu_device)
    buf.returns[:T] = torch.as_tensor(GOLD[f"{prefix}returns"]).to(gpu_device)
    calls = _fixed_perm(monkeypatch, GOLD[f"{prefix}seq_perm"], gpu_device)
    orig = R.windowed
    monkeypatch.setattr(_base.R, "windowed", lambda *a, **kw: orig(*a, **{**kw, "budget_bytes": budget}))
    got = list(buf.get_sequence_batches(L, MB))
    assert calls == [len(GOLD[f"{prefix}seq_perm"])]
    assert len(got) == int(GOLD[f"{prefix}seq_n_batches"])
    for k, b in enumerate(got):
        keys = {kk[len(f"{prefix}seq_b{k}_"):] for kk in GOLD.files if kk.startswith(f"{prefix}seq_b{k}_")}
        assert set(b) == keys
        for key in keys:
            ref = GOLD[f"{prefix}seq_b{k}_{key}"]
            val = b[key].cpu().numpy()
            assert val.dtype == ref.dtype and val.shape == ref.shape, (key, val.dtype, ref.dtype, val.shape)
            np.testing.assert_array_equal(val, ref, err_msg=f"batch {k} {key}")


def test_flat_batches_match_reference(gpu_device, monkeypatch):
    buf, (T, E, N, L, MB) = _buffer_from_golden("poca_", gpu_device)
    buf.advantages[:T] = torch.as_tensor(GOLD["poca_advantages"]).to(gpu_device)
    buf.returns[:T] = torch.as_tensor(GOLD["poca_returns"]).to(gpu_device)
    _fixed_perm(monkeypatch, GOLD["poca_flat_perm"], gpu_device)
    got = list(buf.get_batches(MB))
    assert len(got) == int(GOLD["poca_flat_n_batches"])
    for k, b in enumerate(got):
        keys = {kk[len(f"poca_flat_b{k}_"):] for kk in GOLD.files if kk.startswith(f"poca_flat_b{k}_")}
        assert set(b) == keys
        for key in keys:
            np.testing.assert_array_equal(b[key].cpu().numpy(), GOLD[f"poca_flat_b{k}_{key}"], err_msg=key)


def _random_rollout(T, E, N, seed, p_done=0.01):
    g = np.random.default_rng(seed)
    d = (g.random((T, E)) < p_done).astype(np.float32)
    d[-1, : E // 4] = 1.0  # synchronous episode end on a quarter of the envs
    to = d * (g.random((T, E)) < 0.7)
    return dict(rewards=np.round(g.normal(size=(T, E)) * 3).astype(np.float32), dones=d,
                timeouts=to.astype(np.float32), timeout_values=g.normal(size=(T, E)).astype(np.float32),
                team_values=g.normal(size=(T, E)).astype(np.float32),
                baselines=g.normal(size=(T, E, N)).astype(np.float32)), g.normal(size=E).astype(np.float32)


@pytest.mark.parametrize("T,E", [(240, 8192), (1, 4096), (1001, 64)])
def test_scan_full_size_matches_oracle(gpu_device, T, E):
    """C3 (Foraging cyclamen, 8192 envs x 20, 240 decisions per episode); T=1; the
    config's time_horizon 1000 + buffer-target rows."""
    N = 20
    data, last = _random_rollout(T, E, N, seed=T * 7 + E)
    buf = POCARolloutBuffer(T, E, N, obs_dim=4, act_dim=1, device=gpu_device)
    for k, v in data.items():
        getattr(buf, k).copy_(torch.as_tensor(v))
    buf.ptr = T
    buf.compute_returns_and_advantages(torch.as_tensor(last).to(gpu_device))
    ref = RO.lambda_returns(data["rewards"], data["dones"], data["timeouts"], data["timeout_values"],
                            data["team_values"], last, 0.99, 0.95)
    np.testing.assert_array_equal(buf.returns.cpu().numpy(), ref)
    np.testing.assert_array_equal(buf.advantages.cpu().numpy(), RO.advantages(ref, data["baselines"]))


@pytest.mark.parametrize("T,E,N,L", [(240, 1024, 20, 128), (37, 300, 7, 5), (5, 3, 2, 8), (240, 8192, 20, 128)])
def test_chunk_table_matches_oracle(gpu_device, T, E, N, L):
    data, _ = _random_rollout(T, E, N, seed=E + L, p_done=0.05)
    Lc = max(1, min(L, T))
    chunks, n = R.sequence_chunks(torch.as_tensor(data["dones"]).to(gpu_device), N, Lc)
    got = chunks.cpu().numpy()
    if E * N <= 1024 * 20:
        ref, _ = RO.sequence_chunks(data["dones"], N, L)
        np.testing.assert_array_equal(got, ref)
    else:  # full C3 size: size-independent properties of the table
        assert n == len(got) and (got[:, 3] - got[:, 2] >= 1).all() and (got[:, 3] - got[:, 2] <= Lc).all()
        assert (np.diff(got[:, 0]) >= 0).all()  # env-major
        assert (got[:, 1] == np.tile(np.arange(N), n // N)).all()  # agent fastest
        per_env = np.bincount(got[::N, 0], weights=got[::N, 3] - got[::N, 2], minlength=E)
        assert (per_env == T).all()  # windows tile every env's rollout exactly


def test_gather_full_size_matches_oracle_rows(gpu_device):
    """C3-sized recurrent POCA buffer (T=240 decisions, E=8192 envs, N=20, window
    128, minibatch 2048): the first three sequence batches checked row by row
    against the oracle (on host copies of just the envs those rows touch)."""
    T, E, N, L = 240, 8192, 20, 128
    buf = POCARolloutBuffer(T, E, N, obs_dim=4, act_dim=1, memory_size=8, critic_memory_size=8, device=gpu_device)
    gen = torch.Generator(device=gpu_device).manual_seed(3)
    for name in ("obs", "critic_states", "actions", "log_probs", "advantages", "returns", "team_values",
                 "baselines", "memory_h", "memory_c", "critic_memory_h", "critic_memory_c", "baseline_memory_h",
                 "baseline_memory_c"):
        t = getattr(buf, name)
        t.copy_(torch.randn(t.shape, generator=gen, device=gpu_device))
    d = torch.zeros(T, E, device=gpu_device)
    d[119, ::3] = 1
    d[T - 1] = 1
    buf.dones.copy_(d)
    buf.ptr = T
    torch.manual_seed(0)
    it = buf.get_sequence_batches(L, 2048)
    batches = [next(it) for _ in range(3)]
    torch.manual_seed(0)
    chunks, n = R.sequence_chunks(buf.dones, N, L)
    perm = torch.randperm(n, device=gpu_device)
    per = 2048 // L
    sel = chunks[perm[: 3 * per]].cpu().numpy()
    envs = np.unique(sel[:, 0])
    local = sel.copy()
    local[:, 0] = np.searchsorted(envs, sel[:, 0])
    idx = torch.as_tensor(envs, device=gpu_device)
    spec = S._data(S.FULL_SEQ_SPECS["poca_"])
    arrays = {attr: getattr(buf, attr).index_select(1, idx).cpu().numpy() for _k, attr, _kind in spec}
    for k, b in enumerate(batches):
        ref = RO.gather_sequences(local, np.arange(k * per, (k + 1) * per), L, spec, arrays)
        for key, v in ref.items():
            np.testing.assert_array_equal(b[key].cpu().numpy(), v, err_msg=f"batch {k} {key}")


def test_edge_cases(gpu_device):
    buf = POCARolloutBuffer(3, 2, 2, obs_dim=4, act_dim=2, memory_size=2, device=gpu_device)
    assert list(buf.get_sequence_batches(4, 8)) == []  # empty buffer
    buf.compute_returns_and_advantages(torch.zeros(2, device=gpu_device))  # T = 0: no-op
    z = lambda *s: torch.zeros(*s, device=gpu_device)
    for _ in range(3):
        buf.add(z(2, 2, 4), z(2, 2, 5), z(2, 2, 2), z(2, 2, 2), z(2), z(2), z(2), z(2), z(2), z(2, 2),
                memory_h=z(2, 2, 2), memory_c=z(2, 2, 2))
    with pytest.raises(RuntimeError, match="full"):
        buf.add(z(2, 2, 4), z(2, 2, 5), z(2, 2, 2), z(2, 2, 2), z(2), z(2), z(2), z(2), z(2), z(2, 2),
                memory_h=z(2, 2, 2), memory_c=z(2, 2, 2))
    # fewer chunks than one minibatch: a single short batch (poca_buffer.py:270)
    got = list(buf.get_sequence_batches(4, 1000))
    assert len(got) == 1 and got[0]["obs"].shape == (4, 3, 4)
    fresh = POCARolloutBuffer(3, 2, 2, obs_dim=4, act_dim=2, memory_size=2, device=gpu_device)
    with pytest.raises(ValueError):
        fresh.add(z(2, 2, 4), z(2, 2, 5), z(2, 2, 2), z(2, 2, 2), z(2), z(2), z(2), z(2), z(2), z(2, 2))
    cpu = POCARolloutBuffer(2, 2, 2, obs_dim=4, act_dim=2, device="cpu")
    cpu.ptr = 2
    with pytest.raises(RuntimeError, match="GPU"):
        cpu.compute_returns_and_advantages(torch.zeros(2))


@pytest.mark.parametrize("cls", ["poca", "oc2"])
def test_chunk_start_storage_batches_equal_plain_layout(cls, gpu_device):
    """A buffer keeping its recurrent memories only at chunk-start rows (_base.RolloutStorage,
    chunk_length / episode_decisions) yields the same sequence minibatches, field for field and
    bit for bit, as the plain (T, E, ...) layout fed the same rollout (rows written in order,
    episode ends inside and across the 16-row windows)."""
    from SwarmACB_isaac.agents.learned_option_critic_buffer import LearnedOptionRolloutBuffer

    T, E, N, L = 70, 6, 3, 16
    if cls == "poca":
        mk = lambda **kw: POCARolloutBuffer(T, E, N, obs_dim=4, act_dim=1, memory_size=8, critic_memory_size=8,  # noqa: E731
                                            device=gpu_device, **kw)
    else:
        mk = lambda **kw: LearnedOptionRolloutBuffer(T, E, N, obs_dim=24, state_dim=5, act_dim=2, memory_size=12,  # noqa: E731
                                                     critic_memory_size=8, gamma=0.99, lam=0.95, device=gpu_device,
                                                     **kw)
    plain, compact = mk(), mk(chunk_length=L, episode_decisions=25)
    assert compact.compact_starts and not plain.compact_starts
    gen = torch.Generator(device=gpu_device).manual_seed(5)
    d = torch.zeros(T, E, device=gpu_device)
    d[10, 0] = d[24, 1] = d[25, 1] = d[3, 2] = d[40, 2] = d[0, 3] = d[T - 1] = 1
    for t in range(T):
        for name in plain.START_FIELDS:
            v = torch.randn(getattr(plain, name).shape[1:], generator=gen, device=gpu_device)
            plain.put_start(name, t, v)
            compact.put_start(name, t, v)
        plain.dones[t] = compact.dones[t] = d[t]
    for b in (plain, compact):
        b.ptr = T
    for name in ("obs", "critic_states", "actions", "advantages", "returns", "team_values"):
        src = getattr(plain, name, None)
        if src is not None:
            v = torch.randn(src.shape, generator=gen, device=gpu_device)
            src.copy_(v)
            getattr(compact, name).copy_(v)
    torch.manual_seed(11)
    a = list(plain.get_sequence_batches(L, 5 * L))
    torch.manual_seed(11)
    b = list(compact.get_sequence_batches(L, 5 * L))
    assert len(a) == len(b) > 1
    for k, (x, y) in enumerate(zip(a, b)):
        assert set(x) == set(y)
        for key in x:
            torch.testing.assert_close(x[key], y[key], rtol=0, atol=0, msg=f"batch {k} {key}")
