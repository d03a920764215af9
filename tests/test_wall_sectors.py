"""The step kernel's nearest-faces wall pushes (SWARM_WALL_NEAR, swarm_step_impl.h walls_dg_near)
evaluate only the 3 faces that wall_sector3 (swarm_geom_build.h) lists for the 15-degree sector of
a position's direction, found from an octant-folded angle estimate in float32. Every face the
reference's walls_dg loop (DG:1048-1078) pushes from - signed distance below the clearance - must
be among them, for positions inside the arena, on the walls and past them. Restated here in numpy
(float32 where the kernel computes in float32); no GPU needed."""

import numpy as np

f32 = np.float32


def arena_faces():
    """Face midpoints and inward normals of the dodecagon (swarm_geom_build.h, DG:615-628, 858-868)."""
    n = 12
    R = np.sqrt(2 * 4.91 / (n * np.sin(2 * np.pi / n)))
    a = 2 * np.pi * np.arange(n) / n + np.pi / n
    vx, vy = R * np.cos(a), R * np.sin(a)
    mx, my = 0.5 * (vx + np.roll(vx, -1)), 0.5 * (vy + np.roll(vy, -1))
    nrm = np.sqrt(mx * mx + my * my) + 1e-12
    return mx.astype(f32), my.astype(f32), (-mx / nrm).astype(f32), (-my / nrm).astype(f32)


def sector_table(px, py):
    """wall_sector3: the 3 faces whose midpoint directions are nearest each sector centre."""
    out = []
    for s in range(24):
        c = np.deg2rad(15.0 * s + 7.5)
        d = np.abs((np.arctan2(py.astype(np.float64), px.astype(np.float64)) - c + np.pi) % (2 * np.pi) - np.pi)
        out.append(sorted(np.lexsort((np.arange(12), d))[:3].tolist()))
    return out


def kernel_sector(x, y):
    """wall_faces(): octant-folded angle estimate (t * 45 degrees), float32."""
    ax, ay = np.abs(x), np.abs(y)
    mn, mx = np.minimum(ax, ay), np.maximum(ax, ay)
    t = np.where(mx > 0, mn / np.where(mx > 0, mx, f32(1)), f32(0)).astype(f32)
    a = (t * f32(45.0)).astype(f32)
    a = np.where(ay > ax, f32(90.0) - a, a)
    a = np.where(x < 0, f32(180.0) - a, a)
    a = np.where(y < 0, f32(360.0) - a, a)
    return np.clip((a * f32(1.0 / 15.0)).astype(np.int32), 0, 23)


def test_pushing_faces_are_among_the_sector_candidates():
    px, py, nx, ny = arena_faces()
    table = np.array(sector_table(px, py))
    clear = f32(0.035 + 0.5 * 0.01 + 1e-4)
    rng = np.random.default_rng(0)
    M = 2_000_000
    ang = rng.uniform(0, 2 * np.pi, M)
    apo = float(np.min(-(px * nx + py * ny)))
    # radii from 0.2 m inside the apothem to past the corners
    r = rng.uniform(apo - 0.2, apo / np.cos(np.pi / 12) + 0.1, M)
    x, y = (r * np.cos(ang)).astype(f32), (r * np.sin(ang)).astype(f32)
    sd = (x[:, None] - px[None]) * nx[None] + (y[:, None] - py[None]) * ny[None]   # (M, 12), float32
    pushing = sd < clear
    cand = np.zeros((M, 12), bool)
    rows = table[kernel_sector(x, y)]
    for k in range(3):
        cand[np.arange(M), rows[:, k]] = True
    missed = pushing & ~cand
    assert not missed.any(), f"{int(missed.any(1).sum())} positions push from a face outside their sector's 3"
    assert pushing.any(1).mean() > 0.3     # the sample does exercise the walls
    assert (pushing.sum(1) == 2).any()     # ... and the corners (two faces at once)


def test_sector_table_lists_three_distinct_faces_ascending():
    px, py, _, _ = arena_faces()
    for row in sector_table(px, py):
        assert len(set(row)) == 3 and row == sorted(row)
