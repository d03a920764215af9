"""The step kernel decides contact (DG:1009-1046, ov = min_dist - sqrt(s) > 0) and range-and-bearing
range (ES:300-330, sqrt(s) < range) from the squared distance s alone: s < sqrt_lim(R)
(swarm_geom_build.h), the smallest float whose correctly rounded sqrt reaches R. That is the same
decision as the reference's float32 sqrt test for every float s, because a correctly rounded sqrt is
monotone. Checked here in float32 over a window of ulps around each threshold and on random s."""

import numpy as np

f32 = np.float32


def sqrt_lim(R):
    """Restatement of swarm_geom_build.h sqrt_lim (float32 search down, then up)."""
    R = f32(R)
    s = f32(R * R)
    while s > 0 and np.sqrt(s) >= R:
        s = np.nextafter(s, f32(0))
    while np.sqrt(s) < R:
        s = np.nextafter(s, f32(np.inf))
    return s


def test_squared_threshold_is_the_sqrt_decision():
    rng = np.random.default_rng(3)
    for R in (0.07, 0.0700001, 0.1, 0.5, 1.0, 0.035 * 2, 0.3):
        lim = sqrt_lim(R)
        bits = lim.view(np.int32) + np.arange(-4096, 4097, dtype=np.int32)
        s = bits.view(np.float32)
        np.testing.assert_array_equal(np.sqrt(s) < f32(R), s < lim)
        s = (rng.uniform(0, 2 * R * R, 200_000)).astype(f32)
        np.testing.assert_array_equal(np.sqrt(s) < f32(R), s < lim)
        # the kernel adds the reference's 1e-8 before the sqrt: the threshold applies to that sum
        s = (rng.uniform(0, 2 * R * R, 200_000)).astype(f32)
        t = (s + f32(1e-8)).astype(f32)
        np.testing.assert_array_equal(f32(R) - np.sqrt(t) > 0, t < lim)


def add_lim(c, L):
    """Restatement of swarm_geom_build.h add_lim: the smallest float32 s >= 0 with fl(s + c) >= L."""
    c, L = f32(c), f32(L)
    s = f32(L - c)
    while s > 0 and f32(s + c) >= L:
        s = np.nextafter(s, f32(0))
    while f32(s + c) < L:
        s = np.nextafter(s, f32(np.inf))
    return s


def test_pre_add_threshold_is_the_same_decision():
    """The candidate masks compare s = |d|^2 itself with x_pre_lim = add_lim(1e-8, x_s_lim) instead of
    adding the reference's 1e-8 first (DG:1088 dist = sqrt(dx^2 + dy^2 + 1e-8), ES:411): the same
    decision for every float32 s, as float addition is monotone."""
    rng = np.random.default_rng(5)
    for R in (0.07, 0.6):
        lim = sqrt_lim(R)
        pre = add_lim(1e-8, lim)
        bits = pre.view(np.int32) + np.arange(-8192, 8193, dtype=np.int32)
        s = bits.view(np.float32)
        np.testing.assert_array_equal((s + f32(1e-8)).astype(f32) < lim, s < pre)
        s = rng.uniform(0, 2 * R * R, 500_000).astype(f32)
        np.testing.assert_array_equal((s + f32(1e-8)).astype(f32) < lim, s < pre)
        # and end to end against the reference's sqrt decision
        np.testing.assert_array_equal(f32(R) - np.sqrt((s + f32(1e-8)).astype(f32)) > 0, s < pre)
