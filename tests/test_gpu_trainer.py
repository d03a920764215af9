"""POCA update on the MI355X vs the reference's own update() (tests/golden/trainer).

`trainer.update()` runs end to end on the GPU: advantage normalisation, the
buffers' HIP minibatch gathers (under the reference's recorded permutations),
the actor / critic losses through autograd, Adam. Teacher-forced per optimizer
step (trainer_fixtures.TeacherForcing): losses and every gradient are checked
against the reference's (rtol 1e-4 + 1e-5 of each tensor's scale: fp32
reduction order of GPU library kernels), then the reference's gradients are
loaded and the post-Adam parameters must match within 1e-6.
"""

import pytest
import torch

import trainer_fixtures as TF

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(TF.CASES))
def test_poca_update_on_gpu_matches_reference(name, gpu_device):
    tf, metrics, fx = TF.run_teacher_forced(name, gpu_device)
    keys = [str(k) for k in fx["metrics_keys"]]
    ref = dict(zip(keys, fx["metrics_values"]))
    for k in ("lr", "eps", "beta"):
        assert metrics[k] == pytest.approx(ref[k], rel=1e-12)
    for k in ("policy_loss", "value_loss", "baseline_loss", "entropy"):
        assert metrics[k] == pytest.approx(ref[k], rel=1e-4, abs=1e-5)
    print(f"[trainer] {name}: {tf.steps} optimizer steps, max grad err {tf.max_grad_err:.3g}, "
          f"max param err {tf.max_param_err:.3g} (relative to tensor scale)")


@pytest.mark.parametrize("name", sorted(TF.CASES))
def test_poca_update_on_gpu_with_host_batches(name, gpu_device):
    """Same with the minibatches gathered on the host (isolates the loss / autograd path)."""
    tf, _, _ = TF.run_teacher_forced(name, gpu_device, batches="oracle")
    assert tf.steps > 0


def test_poca_trainer_end_to_end_on_swarm_env(gpu_device, tmp_path):
    """train() on the HIP env (Foraging cyclamen, recurrent, 64 envs): one update is
    triggered, metrics land in the JSONL writer with the reference's tags, the
    checkpoint round-trips, and every parameter stays finite."""
    from SwarmACB_isaac.agents.config import POCAConfig, make_env_cfg
    from SwarmACB_isaac.agents.metrics import read_scalars
    from SwarmACB_isaac.agents.poca_trainer import POCATrainer
    from SwarmACB_isaac.registry import make

    env = make("SwarmACB-Foraging-v0", make_env_cfg("SwarmACB-Foraging-v0", "cyclamen", {"num_envs": 64}),
               device=gpu_device)
    cfg = POCAConfig(horizon=12, mini_batch_size=256, num_epochs=1, hidden_dim=128, num_layers=1, recurrent=True,
                     memory_size=128, sequence_length=8, critic_hidden_dim=128, critic_num_layers=1,
                     critic_num_heads=4, buffer_size_hint=64 * 20 * 10, total_timesteps=64 * 20 * 12,
                     summary_freq=1, checkpoint_interval=10 ** 9, log_dir=str(tmp_path / "runs"),
                     checkpoint_dir=str(tmp_path / "ckpt"), lr_schedule="linear")
    torch.manual_seed(0)
    tr = POCATrainer(env, cfg)
    tr.train()
    assert tr.update_count == 1 and tr.global_step == 64 * 20 * 12
    tags = {r["tag"] for r in read_scalars(str(tmp_path / "runs"))}
    for t in ("Losses/Policy Loss", "Losses/Value Loss", "Losses/POCA/Baseline Loss", "Policy/Entropy",
              "Policy/Learning Rate", "Extra/SPS", "Extra/Mean Rollout Reward"):
        assert t in tags, t
    assert all(torch.isfinite(p).all() for p in tr.params)
    ck = torch.load(tmp_path / "ckpt" / "poca_final.pt", weights_only=True)
    assert ck["global_step"] == tr.global_step and ck["recurrent"] and ck["memory_size"] == 128
    tr2 = POCATrainer(env, cfg)
    tr2.load_checkpoint(tmp_path / "ckpt" / "poca_final.pt")
    for a, b in zip(tr.params, tr2.params):
        assert torch.equal(a, b)
    env.close()
