"""Fixed-option Option-Critic (C4) on the MI355X vs the reference's own trainer
(tests/golden/trainer/oc_*.npz from make_oc_golden.py).

* collect: the decision loop (option_collector.py: manager LSTM cell kernel,
  fused critic kernel at hidden 128, one decision-record launch per decision)
  replays the reference's env script and option / termination draws; every
  buffer row the reference wrote, the options the env received, the trainer's
  end-of-rollout memories and options and the completed-episode log are
  compared (discrete fields exactly, floats within rtol 1e-4 + 1e-5 of each
  tensor's scale: fp32 GEMM / reduction order on the GPU).
* update: teacher-forced per optimizer step on the GPU (device buffers and
  HIP gathers under the recorded permutations; and host-gathered batches).
* end to end: train() on the HIP DirGate cyclamen env, one update, metrics
  with the reference's tags, checkpoint round trip.
"""

import numpy as np
import pytest
import torch

import oc_fixtures as OF
import trainer_fixtures as TFX

pytestmark = pytest.mark.gpu

EXACT = {"options", "option_masks", "dones", "timeouts", "rewards"}


@pytest.mark.parametrize("name", sorted(OF.OC_CASES))
def test_oc_collect_matches_reference(name, gpu_device):
    tr, fx, _, _ = OF.make_oc_trainer(name, gpu_device)
    env = tr.env
    OF.ReplayDraws(tr.collector, fx)
    obs_dict = env.reset()[0]
    R = int(fx["meta"][3])
    tr.collect_rollout(obs_dict, rollout_steps=R)
    torch.cuda.synchronize()
    T = int(fx["ptr"])
    assert tr.buffer.ptr == T and tr.global_step == int(fx["global_step"])
    dp = int(fx["meta"][4])
    ref_actions = fx["env_actions"][::dp].reshape(R, *fx["env_actions"].shape[1:3])   # held for dp substeps
    np.testing.assert_array_equal(torch.stack(env.actions).cpu().numpy(), ref_actions)
    worst = {}
    for key in OF.load(name).files:
        if not key.startswith("buf/"):
            continue
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
    for k in OF.load(name).files:
        if k.startswith("state/"):
            attr = k[6:]
            got = getattr(tr, attr)
            if attr == "current_options":
                np.testing.assert_array_equal(got.cpu().numpy(), fx[k])
            else:
                worst[attr] = TFX._close(got, fx[k], 1e-4, 1e-5, f"end state {attr}")
    r, ln, g = tr.collector.recorder.drain()
    np.testing.assert_allclose(r, fx["completed_returns"], rtol=1e-6)
    np.testing.assert_allclose(ln, fx["completed_lengths"])
    np.testing.assert_allclose(g, fx["completed_group_rewards"], rtol=1e-6)
    print(f"[oc collect] {name}: worst relative error {max(worst.values()):.3g} ({max(worst, key=worst.get)})")


@pytest.mark.parametrize("name", OF.UPDATE_CASES)
def test_oc_update_on_gpu_matches_reference(name, gpu_device):
    tf, metrics, fx = OF.run_teacher_forced_oc(name, gpu_device)
    ref = dict(zip([str(k) for k in fx["metrics_keys"]], fx["metrics_values"]))
    for k in ("lr", "eps", "beta"):
        assert metrics[k] == pytest.approx(ref[k], rel=1e-12)
    for k in ("policy_loss", "value_loss", "joint_option_value_loss", "baseline_loss", "termination_loss",
              "option_entropy", "termination_entropy", "mean_beta", "mean_option_advantage", "switch_rate"):
        assert metrics[k] == pytest.approx(ref[k], rel=1e-4, abs=1e-5), k
    np.testing.assert_allclose(metrics["option_usage"], fx["metrics_option_usage"], rtol=1e-6)
    print(f"[oc update] {tf.steps} optimizer steps, max grad err {tf.max_grad_err:.3g}, "
          f"max param err {tf.max_param_err:.3g}")


@pytest.mark.parametrize("name", OF.UPDATE_CASES)
def test_oc_update_on_gpu_with_host_batches(name, gpu_device):
    tf, _, _ = OF.run_teacher_forced_oc(name, gpu_device, batches="oracle")
    assert tf.steps > 0


def test_oc_trainer_end_to_end_on_swarm_env(gpu_device, tmp_path):
    """train() on the HIP env (DirGate cyclamen, 64 envs): one update, metrics with the
    reference's tags, checkpoint round trip, finite parameters."""
    from SwarmACB_isaac.agents.config import FixedOptionCriticConfig, make_env_cfg
    from SwarmACB_isaac.agents.metrics import read_scalars
    from SwarmACB_isaac.agents.option_critic_trainer import FixedOptionCriticTrainer
    from SwarmACB_isaac.registry import make

    env = make("SwarmACB-DirectionalGate-v0",
               make_env_cfg("SwarmACB-DirectionalGate-v0", "cyclamen", {"num_envs": 64}, "option_critic"),
               device=gpu_device)
    cfg = FixedOptionCriticConfig(horizon=12, mini_batch_size=256, num_epochs=1, sequence_length=8,
                                  buffer_size_hint=64 * 20 * 10, total_timesteps=64 * 20 * 12, summary_freq=1,
                                  checkpoint_interval=10 ** 9, log_dir=str(tmp_path / "runs"),
                                  checkpoint_dir=str(tmp_path / "ckpt"), lr_schedule="linear")
    torch.manual_seed(0)
    tr = FixedOptionCriticTrainer(env, cfg)
    tr.train()
    assert tr.update_count == 1 and tr.global_step == 64 * 20 * 12
    tags = {r["tag"] for r in read_scalars(str(tmp_path / "runs"))}
    for t in ("Losses/Policy Loss", "Losses/OptionCritic/Termination Loss", "Policy/Switch Rate",
              "Policy/Option Usage/0", "Extra/SPS"):
        assert t in tags, t
    assert all(torch.isfinite(p).all() for p in tr.params)
    assert int(tr.current_options.min()) >= 0
    ck = torch.load(tmp_path / "ckpt" / "option_critic_final.pt", weights_only=True)
    assert ck["global_step"] == tr.global_step and ck["trainer_type"] == "option_critic"
    tr2 = FixedOptionCriticTrainer(env, cfg)
    tr2.load_checkpoint(tmp_path / "ckpt" / "option_critic_final.pt")
    for a, b in zip(tr.params, tr2.params):
        assert torch.equal(a, b)
    env.close()
