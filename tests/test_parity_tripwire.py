"""The parity tripwire (tests/parity.py tripwire) on the CPU: it fails a GPU test group whose
envelope grows past the committed record (tests/parity_bounds.json) and a run whose hull-rule
count passes the recorded maximum."""

import json

import pytest

import parity

BOUNDS = {"hull_elements_max": 5,
          "envelope_max_delta": {"gpu_philox": {"cache": 7.6e-4, "obs": 5.7e-5}, "gpu_vs_reference": {"obs": 3e-5}}}


def test_within_record_passes():
    seen = {}
    parity.tripwire("gpu_philox/c2", {"hull_elements": 3, "envelope_max_delta": {"cache": 7.0e-4}}, BOUNDS, seen)
    parity.tripwire("gpu_philox/c5", {"hull_elements": 2, "envelope_max_delta": {"obs": 5.7e-5}}, BOUNDS, seen)
    parity.tripwire("oracle_vs_reference/x", {"hull_elements": 50, "envelope_max_delta": {"obs": 1.0}}, BOUNDS,
                    seen)   # CPU oracle group: not the GPU record's business
    assert seen["hull_elements"] == 5


def test_hull_count_past_record_fails():
    seen = {}
    parity.tripwire("gpu_philox/a", {"hull_elements": 5}, BOUNDS, seen)
    with pytest.raises(AssertionError, match="hull-rule"):
        parity.tripwire("gpu_philox/b", {"hull_elements": 1}, BOUNDS, seen)


def test_envelope_delta_past_record_fails():
    with pytest.raises(AssertionError, match="exceeds the recorded"):
        parity.tripwire("gpu_philox/a", {"envelope_max_delta": {"cache": 8e-4}}, BOUNDS, {})
    with pytest.raises(AssertionError, match="exceeds the recorded"):   # a key the record never saw
        parity.tripwire("gpu_vs_reference/a", {"envelope_max_delta": {"cache": 1e-6}}, BOUNDS, {})


def test_committed_bounds_are_well_formed():
    with open(parity.BOUNDS_PATH) as f:
        b = json.load(f)
    assert b["hull_elements_max"] <= 5
    for group, keys in b["envelope_max_delta"].items():
        assert group.startswith("gpu_")
        assert all(0.0 <= v < 1e-3 for v in keys.values())
