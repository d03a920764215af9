"""The CPU oracle reproduces the reference on every golden vector (teacher forced).

This pins the oracle before it is trusted as the checker of the HIP path.
Fixtures come from tests/golden/make_golden.py (reference run in the build
container): scripts/manual_control.py (standalone) and the stub-run Isaac
mission envs (isaac), every mission, continuous and discrete variants,
crowded layouts, wall corners and episode ends with auto-reset.
"""

import numpy as np
import pytest

import parity
from oracle import oracle as O


@pytest.mark.parametrize("name", parity.fixture_ids())
def test_oracle_matches_reference(name):
    fx = parity.load(name)
    T = fx["obs"].shape[0]
    failures, stats = [], {}
    for t in range(T):
        base, spread = parity.envelope(fx, t)
        errs = parity.compare(base, parity.reference_after(fx, t), spread, stats=stats)
        failures += [f"step {t}: {e}" for e in errs]
    parity.record_stats(f"oracle_vs_reference/{name}", stats)
    assert not failures, "\n".join(failures[:10])


def test_fixture_chain_is_consistent():
    """after_t == before_{t+1}: fixtures are consecutive reference steps."""
    for name in parity.fixture_ids():
        fx = parity.load(name)
        for t in range(fx["obs"].shape[0] - 1):
            np.testing.assert_array_equal(fx["after_pos"][t], fx["before_pos"][t + 1], err_msg=name)


def test_oracle_free_run_tracks_reference():
    """Chained (not teacher-forced) oracle steps stay with the reference over a 24-frame window."""
    for name in ("standalone_homing_m1_mid", "standalone_dgt_m4_mid", "standalone_xor_m2_mid"):
        fx = parity.load(name)
        env, _ = O.fixture_env(fx)
        before, _ = O.fixture_step_inputs(fx, 0)
        env.load(before)
        for t in range(fx["obs"].shape[0]):
            _, kw = O.fixture_step_inputs(fx, t)
            obs, rew, _ = env.step(**kw)
            np.testing.assert_allclose(env.s["pos"], fx["after_pos"][t], atol=1e-4, err_msg=f"{name} t={t}")
            np.testing.assert_array_equal(rew, fx["reward"][t])


def test_mt19937_stream_matches_torch():
    torch = pytest.importorskip("torch")
    O.seed(2024)
    got = O.rng_uniform(1000)
    torch.manual_seed(2024)
    np.testing.assert_array_equal(got, torch.rand(1000).numpy())


def test_fixture_coverage():
    """The fixture set exercises what the reference tests leave unpinned."""
    names = parity.fixture_ids()
    for mission in ("dgt", "xor", "homing", "foraging", "sheltering"):
        assert any(n.startswith(f"standalone_{mission}") for n in names)
        for variant in ("dandelion", "cyclamen", "daisy"):
            assert f"isaac_{mission}_{variant}_mid" in names
    resets = rewards = turns = 0
    for n in names:
        fx = parity.load(n)
        resets += int(fx["truncated"].sum() if "truncated" in fx.files else fx["reset"].sum())
        rewards += int(np.abs(fx["reward"]).sum() > 0)
        turns += int(fx["turn_present"].sum())
    assert resets > 20 and rewards > 20 and turns > 100
