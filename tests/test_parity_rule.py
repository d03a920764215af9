"""The fp32 parity rule itself (tests/parity.py): the ill-conditioned-element rule accepts a
value only near an outcome the oracle's own arithmetic reaches one ulp away, never a value
inside the jump between two such outcomes."""

import numpy as np

import parity as P


def _spread(base, outs, key="obs"):
    spread = {}
    b = {key: np.asarray(base, np.float32)}
    for o in outs:
        P.accumulate_spread(spread, {key: np.asarray(o, np.float32)}, b)
    return spread


def test_discontinuity_accepts_only_reached_outcomes():
    # a tangent IR ray: the oracle reads 0.0, one perturbed run reads 0.3937 (spread > cap)
    base = [0.0, 0.25]
    outs = [[0.0, 0.25], [0.3937, 0.25], [0.0, 0.25 + 1e-7]]
    sp = _spread(base, outs)
    ref = np.array(base, np.float32)
    for got, ok in (([0.3937, 0.25], True), ([0.0, 0.25], True), ([0.393695, 0.25], True),
                    ([0.2, 0.25], False), ([0.39, 0.25], False)):
        v_ok, _plain, hull = P.float_verdict("obs", np.array(got, np.float32), ref, sp)
        assert bool(v_ok[0]) is ok, (got, v_ok)
        assert bool(v_ok[1])
        assert bool(hull[0]) is (ok and got[0] != 0.0)


def test_well_conditioned_elements_keep_the_plain_bar():
    sp = _spread([0.5], [[0.5], [0.5]])
    ref = np.array([0.5], np.float32)
    assert P.float_verdict("obs", np.array([0.5 + 9e-6], np.float32), ref, sp)[0].all()
    assert not P.float_verdict("obs", np.array([0.5 + 2e-5], np.float32), ref, sp)[0].any()


def test_outcomes_follow_env_subsets():
    sp = _spread(np.zeros((4, 2)), [np.eye(4, 2), np.zeros((4, 2))])
    sub = P._take_envs(sp, np.array([0, 2]), {})
    assert len(sub["obs@outs"]) == 2 and sub["obs@outs"][0].shape == (2, 2)
    np.testing.assert_array_equal(sub["obs@outs"][0], np.eye(4, 2)[[0, 2]])


def test_perturbation_set_is_frozen():
    # the envelope's definition: changing it needs a new record, not a silent edit
    assert P.PERTURBATIONS == ("yaw+", "yaw-", "pos+", "pos-", "lm+", "lm-", "sin+", "sin-", "cos+", "cos-",
                               "sc+-", "sc-+")


def test_hull_examples_name_the_perturbation_that_reproduces_them():
    base = np.zeros(2)
    outs = [np.zeros(2)] * len(P.PERTURBATIONS)
    outs[5] = np.array([0.3937, 0.0])                      # "lm-" reaches the far side of the jump
    sp = _spread(base, outs)
    stats = {}
    errs = P.compare({"obs": np.array([0.3937, 0.0], np.float32)}, {"obs": np.zeros(2, np.float32)}, sp,
                     stats=stats)
    assert not errs and stats["hull_elements"] == 1
    ex, = stats["hull_examples"]
    assert ex["got_reproduced_by"] == ["lm-"] and ex["ref_reproduced_by"][0] == "plain"
