"""The rollout-buffer oracle (oracle/rollout_oracle.py) against the reference's
own outputs (tests/golden/rollout/rollout_buffers.npz, made by make_rollout_golden.py
from poca_buffer.py / option_critic_buffer.py / learned_option_critic_buffer.py).
CPU only; bit-exact."""

import numpy as np
import pytest

from oracle import rollout_oracle as RO
import rollout_specs as S

GOLD = S.load_golden()


def _inputs(prefix):
    g = GOLD
    return [g[f"{prefix}in_{k}"] for k in ("rewards", "dones", "timeouts", "timeout_values", "team_values")] + [
        g[f"{prefix}last_team_value"]]


@pytest.mark.parametrize("prefix", ["poca_", "poca2_", "oc_", "loc_", "long_"])
def test_lambda_returns_bit_exact(prefix):
    gamma, lam = GOLD[f"{prefix}gamma_lam"]
    ret = RO.lambda_returns(*_inputs(prefix), gamma, lam)
    np.testing.assert_array_equal(ret, GOLD[f"{prefix}returns"])


@pytest.mark.parametrize("prefix,sets", [
    ("poca_", [("baselines", "advantages")]), ("poca2_", [("baselines", "advantages")]),
    ("oc_", [("baselines", "advantages")]), ("long_", [("baselines", "advantages")]),
    ("loc_", [("action_baselines", "action_advantages"), ("option_baselines", "option_advantages")])])
def test_advantages_bit_exact(prefix, sets):
    for bl, adv in sets:
        got = RO.advantages(GOLD[f"{prefix}returns"], GOLD[f"{prefix}in_{bl}"])
        np.testing.assert_array_equal(got, GOLD[f"{prefix}{adv}"])


@pytest.mark.parametrize("prefix", ["poca_", "oc_", "loc_"])
def test_sequence_batches_match_reference(prefix):
    T, E, N, L, MB = (int(v) for v in GOLD[f"{prefix}meta"])
    chunks, Lc = RO.sequence_chunks(GOLD[f"{prefix}in_dones"], N, L)
    perm = GOLD[f"{prefix}seq_perm"]
    assert len(perm) == len(chunks)
    arrays = S.golden_arrays(GOLD, prefix)
    spec = S.SEQ_SPECS[prefix]
    batches = S.batch_slices(len(chunks), max(1, MB // Lc))
    assert len(batches) == int(GOLD[f"{prefix}seq_n_batches"])
    for k, (a, b) in enumerate(batches):
        got = RO.gather_sequences(chunks, perm[a:b], Lc, spec, arrays)
        keys = {kk[len(f"{prefix}seq_b{k}_"):] for kk in GOLD.files if kk.startswith(f"{prefix}seq_b{k}_")}
        assert keys == set(got), keys ^ set(got)
        for key in keys:
            np.testing.assert_array_equal(got[key], GOLD[f"{prefix}seq_b{k}_{key}"], err_msg=f"batch {k} {key}")


def test_flat_batches_match_reference():
    T, E, N, L, MB = (int(v) for v in GOLD["poca_meta"])
    perm = GOLD["poca_flat_perm"]
    arrays = S.golden_arrays(GOLD, "poca_")
    usable = len(perm) if len(perm) < MB else len(perm) - len(perm) % MB
    starts = list(range(0, usable, MB))
    assert len(starts) == int(GOLD["poca_flat_n_batches"])
    for k, a in enumerate(starts):
        got = RO.gather_flat(perm[a:a + MB], N, S.FLAT_SPEC, arrays)
        for key, v in got.items():
            np.testing.assert_array_equal(v, GOLD[f"poca_flat_b{k}_{key}"], err_msg=f"batch {k} {key}")
