"""Learned-option Option-Critic (OC2, C5) on the MI355X vs the reference's own
trainer (tests/golden/trainer/oc2_*.npz from make_oc2_golden.py).

* collect: the OC2 decision loop (option_collector.LearnedOptionCollector:
  option-LSTM rows through the LSTM-cell kernel, the critics through the fused
  attention kernel at hidden 128 with the option critic's Q and baselines on one
  projection, one decision-record launch) replays the reference's env script
  and its option / termination / wheel draws; every buffer row, the wheel
  commands the env received, the end-of-rollout memories and options and the
  completed-episode log are compared (discrete fields exactly, floats within
  rtol 1e-4 + 1e-5 of each tensor's scale).
* update: teacher-forced per optimizer step on the GPU (device buffers + HIP
  gathers under the recorded permutations), with torch's fused Adam (the
  reference's choice on a GPU) and with the plain one; the KL early stop and
  the adaptive actor learning rate must take the reference's decisions.
* end to end: train() on the HIP XOR env (cyclamen with continuous wheels and
  24-D observations), one update, metrics with the reference's tags,
  checkpoint round trip.
"""

import numpy as np
import pytest
import torch

import oc2_fixtures as O2
import oc_fixtures as OF
import trainer_fixtures as TFX

pytestmark = pytest.mark.gpu

EXACT = {"options", "option_masks", "dones", "timeouts", "rewards", "termination_options", "termination_valid"}


@pytest.mark.parametrize("name", ["oc2_update", "oc2_collect_h128"])
def test_oc2_collect_matches_reference(name, gpu_device):
    tr, fx, _, _ = O2.make_oc2_trainer(name, gpu_device)
    col, dev = tr.collector, torch.device(gpu_device)
    draws = {tag: [torch.as_tensor(fx[f"sample_{tag}/{i}"]).to(dev) for i in range(int(fx[f"n_{tag}"]))]
             for tag in ("option", "term", "action")}
    col.sample_options = lambda d: draws["option"].pop(0)
    col.sample_termination = lambda d: draws["term"].pop(0)
    col.sample_actions = lambda d: draws["action"].pop(0)
    env = tr.env
    R, dp = int(fx["meta"][3]), int(fx["meta"][4])
    tr.collect_rollout(env.reset()[0], rollout_steps=R)
    torch.cuda.synchronize()
    T = int(fx["ptr"])
    assert tr.buffer.ptr == T and tr.global_step == int(fx["global_step"])
    ref_actions = fx["env_actions"][::dp]     # the wheel command is held for dp substeps
    TFX._close(torch.stack(env.actions), ref_actions, 1e-6, 1e-7, "env wheel commands")
    worst = {}
    for key in fx.files:
        if key.startswith("buf/"):
            attr = key[4:]
            got = tr.buffer.rows(attr, T)
            if attr in tr.buffer.START_FIELDS:     # chunk-start storage holds those rows only
                m = tr.buffer.start_row_mask(T).cpu().numpy()
                fx_v = np.where(m.reshape(m.shape + (1,) * (fx[key].ndim - 2)), fx[key], 0)
                worst[attr] = TFX._close(got, fx_v, 1e-4, 1e-5, f"buffer {attr}")
                continue
            if attr in EXACT:
                np.testing.assert_array_equal(got.cpu().numpy(), fx[key], err_msg=attr)
            else:
                worst[attr] = TFX._close(got, fx[key], 1e-4, 1e-5, f"buffer {attr}")
        elif key.startswith("state/"):
            attr = key[6:]
            got = getattr(tr, attr)
            if attr == "current_options":
                np.testing.assert_array_equal(got.cpu().numpy(), fx[key])
            else:
                worst[attr] = TFX._close(got, fx[key], 1e-4, 1e-5, f"end state {attr}")
    r, ln, g = tr.collector.recorder.drain()
    np.testing.assert_allclose(r, fx["completed_returns"], rtol=1e-6)
    np.testing.assert_allclose(ln, fx["completed_lengths"])
    np.testing.assert_allclose(g, fx["completed_group_rewards"], rtol=1e-6)
    print(f"[oc2 collect] {name}: worst relative error {max(worst.values()):.3g} ({max(worst, key=worst.get)})")


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", O2.UPDATE_CASES)
def test_oc2_update_on_gpu_matches_reference(name, fused, gpu_device):
    tr, tf, metrics, fx = O2.run_teacher_forced_oc2(name, gpu_device, fused_optimizer=fused)
    assert tr.fused_optimizer_active == fused
    O2.check_metrics(metrics, fx)
    assert tr.actor_lr_scale == pytest.approx(float(fx["actor_lr_scale_after"]), rel=1e-12)
    print(f"[oc2 update] {name} fused={fused}: {len(tf.seen)} optimizer steps, max grad err "
          f"{tf.max_grad_err:.3g}, max param err {tf.max_param_err:.3g}")


def test_oc2_trainer_end_to_end_on_swarm_env(gpu_device, tmp_path):
    """train() on the HIP env (XOR, cyclamen + continuous wheels / 24-D obs, 64 envs): one
    update, metrics with the reference's tags, checkpoint round trip, finite parameters."""
    from SwarmACB_isaac.agents.config import LearnedOptionCriticConfig, make_env_cfg
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.metrics import read_scalars
    from SwarmACB_isaac.registry import make

    env = make("SwarmACB-XOR-v0", make_env_cfg("SwarmACB-XOR-v0", "cyclamen", {"num_envs": 64},
                                               "learned_option_critic"), device=gpu_device)
    cfg = LearnedOptionCriticConfig(horizon=12, mini_batch_size=512, num_epochs=1, sequence_length=8,
                                    option_hidden_dim=128, buffer_size_hint=64 * 20 * 10,
                                    total_timesteps=64 * 20 * 12, summary_freq=1, checkpoint_interval=10 ** 9,
                                    log_dir=str(tmp_path / "runs"), checkpoint_dir=str(tmp_path / "ckpt"),
                                    lr_schedule="linear", matmul_precision="highest")
    torch.manual_seed(0)
    tr = LearnedOptionCriticTrainer(env, cfg)
    assert tr.obs_dim == 24 and tr.act_dim == 2
    tr.train()
    assert tr.update_count == 1 and tr.global_step == 64 * 20 * 12
    tags = {r["tag"] for r in read_scalars(str(tmp_path / "runs"))}
    for t in ("Losses/Intra-Option Policy Loss", "Losses/Termination Loss", "Update/Max Policy KL",
              "Performance/Rollout SPS", "Policy/Option Usage/0", "Extra/SPS"):
        assert t in tags, t
    assert all(torch.isfinite(p).all() for p in tr.params)
    ck = torch.load(tmp_path / "ckpt" / "option_critic_2_final.pt", weights_only=True)
    assert ck["global_step"] == tr.global_step and ck["trainer_type"] == "learned_option_critic"
    tr2 = LearnedOptionCriticTrainer(env, cfg)
    tr2.load_checkpoint(tmp_path / "ckpt" / "option_critic_2_final.pt")
    for a, b in zip(tr.params, tr2.params):
        assert torch.equal(a, b)
    env.close()
