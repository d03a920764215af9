"""The oracle's restatement of the production kernel's Philox draws (CPU only).

Philox4x32-10 is checked against the Random123 known-answer vectors
(kat_vectors: philox4x32_10); the draw layout (which block / bits each
packet-loss, turn and spawn uniform comes from) is the kernel's own design
(swarm_step_impl.h rng4 / ChunkRng / u01_of5 / u01_of7 / draw_turn /
spawn_isaac / spawn_mc), restated here independently in numpy and compared
with oracle/or_philox_draws. The GPU side is test_gpu_philox.py.
"""

import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox_py(c, k):
    c, k0, k1 = list(c), k[0], k[1]
    for _ in range(10):
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF,
             p0 & 0xFFFFFFFF]
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return c


@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_known_answers(ctr, key, expect):
    assert tuple(philox_py(ctr, key)) == expect
    a = (C.c_uint32 * 4)(*ctr)
    O.lib().or_philox4x32(a, C.c_uint32(key[0]), C.c_uint32(key[1]))
    assert tuple(a) == expect


def _rng4(seed, genv, robot, block, purpose, tick):
    return philox_py((genv, robot | (block << 8) | (purpose << 24), tick & 0xFFFFFFFF, tick >> 32),
                     (seed & 0xFFFFFFFF, seed >> 32))


@pytest.mark.parametrize("parts", [3, 1, 4])
def test_draw_layout_matches_numpy_restatement(parts):
    seed, off, E, N, tick = (1 << 40) + 77, 5, 2, 20, (1 << 33) + 9
    d = O.philox_draws(seed, off, E, N, tick, parts=parts, spawn_k=3)
    Cc = -(-N // parts)
    for e in range(E):
        for i in range(N):
            for j in range(N):
                p, jj = j // Cc, j % Cc
                if Cc in (6, 7):
                    r = _rng4(seed, off + e, i, 16 * p, 1, tick)
                    bits = (r[0] | r[1] << 32 | r[2] << 64 | r[3] << 96) >> (18 * jj) & 0x3FFFF
                    u = np.float32(bits) * np.float32(1.0 / 262144.0)
                else:
                    r = _rng4(seed, off + e, i, 16 * p + jj // 5, 1, tick)
                    w = jj % 5
                    v = r[w] >> 8 if w < 4 else (r[0] & 255) | (r[1] & 255) << 8 | (r[2] & 255) << 16
                    u = np.float32(v) * np.float32(1.0 / 16777216.0)
                assert d["rab_u_obs"][e, i, j] == u
            for slot in range(3):
                assert d["turns"][slot, e, i] == 1 + (_rng4(seed, off + e, i, 0, 3 + slot, tick)[0] & 3)
            for k in range(3):
                r = _rng4(seed, off + e, i, k >> 1, 8, tick)
                pair = (r[2], r[3]) if k & 1 else (r[0], r[1])
                for c in range(2):
                    assert d["spawn_u"][k, e, i, c] == np.float32(pair[c] >> 8) * np.float32(2.0 ** -24)
            assert d["spawn_yaw_u"][e, i] == np.float32(_rng4(seed, off + e, i, 0, 9, tick)[0] >> 8) * np.float32(2.0 ** -24)


def test_packet_loss_uniforms_are_uniform():
    d = O.philox_draws(3, 0, 512, 20, 11)
    u = d["rab_u_obs"].ravel()
    assert abs(u.mean() - 0.5) < 0.003 and abs((u >= 0.85).mean() - 0.15) < 0.003
    assert u.min() >= 0.0 and u.max() < 1.0
