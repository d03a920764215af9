"""Layout 203 (the continuous-action Isaac step as a two-wave pipeline per arena: a physics wave
and an observation wave, swarm_step_impl.h step_kernel_pipe) against layout 103 (one wave per
arena): the same arithmetic distributed over two waves, so every output and every state word must
be bitwise equal, for every mission, across episode time-outs (auto-reset and the all-env
re-solve of DG:1262) and fused decisions of 1 and 5 substeps."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

MISSIONS = ["homing", "xor", "dgt", "foraging", "sheltering"]


def _run(mission, layout, E, steps, dp, seed, gpu_device):
    from SwarmACB_isaac.engine import SwarmEngine

    eng = SwarmEngine(mission, "isaac", E, 20, 24, False, 1200, 1, 0, seed, gpu_device, layout=layout)
    out = eng.reset()
    lens = np.full(E, 0, np.int32)
    lens[: E // 3] = 1200 - 7          # a third of the envs time out inside the run
    eng.episode_length.copy_(torch.as_tensor(lens).to(gpu_device))
    eng.sync_episode_lengths()
    g = torch.Generator(device=gpu_device).manual_seed(seed + 7)
    rows = []
    for k in range(steps):
        a = (torch.randn(E, 20, 2, device=gpu_device, generator=g).clamp_(-3, 3) / 3).contiguous()
        obs, rew, tr = eng.step(a, dp, out=out)
        torch.cuda.synchronize(gpu_device)
        rows.append((obs.cpu().numpy().copy(), rew.cpu().numpy().copy(), tr.cpu().numpy().copy()))
    st = eng.dump_state()
    crit = eng.terminal_critic.cpu().numpy().copy()
    eng.close()
    return rows, st, crit


@pytest.mark.parametrize("mission", MISSIONS)
@pytest.mark.parametrize("dp", [1, 5])
def test_pipe_layout_bitwise_equals_layout_103(mission, dp, gpu_device):
    E, steps = 96, 12 if dp == 5 else 24
    a_rows, a_st, a_crit = _run(mission, 103, E, steps, dp, 11, gpu_device)
    b_rows, b_st, b_crit = _run(mission, 203, E, steps, dp, 11, gpu_device)
    for k, (ra, rb) in enumerate(zip(a_rows, b_rows)):
        for name, x, y in zip(("obs", "reward", "trunc"), ra, rb):
            np.testing.assert_array_equal(x.view(np.uint8), y.view(np.uint8), err_msg=f"{mission} step {k} {name}")
    for key in a_st:
        np.testing.assert_array_equal(np.asarray(a_st[key]).view(np.uint8), np.asarray(b_st[key]).view(np.uint8),
                                      err_msg=f"{mission} state {key}")
    np.testing.assert_array_equal(a_crit.view(np.uint8), b_crit.view(np.uint8), err_msg=f"{mission} terminal critic")
    assert any(r[2].any() for r in a_rows), "no time-out exercised"
