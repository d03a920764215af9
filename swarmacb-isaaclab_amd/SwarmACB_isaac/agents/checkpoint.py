"""POCA checkpoint format and headless playback.

* `poca_checkpoint` / `save_poca_checkpoint` write the dict of
  PT:1056-1083 (`POCATrainer.save_checkpoint`), key for key, so a checkpoint
  written here loads in the reference's `play.py` (and, when it carries the
  optimizer state, resumes in its trainer) and vice versa.
* `load_poca_checkpoint` follows PT:1085-1106: the paper-parity version must
  match and the actor / critic (/ optimizer) state dicts must load strictly.
  Files are read with `torch.load(weights_only=True)`: a checkpoint holds
  tensors, numbers, strings and optimizer state only.
* `actor_from_checkpoint` rebuilds the policy the way play.py:379-436 does for
  POCA checkpoints (Actor / DiscreteActor / RecurrentDiscreteActor from the
  stored architecture keys). Option-critic checkpoints name networks this build
  does not carry (FixedOptionManager, LearnedOptionActor) and are refused.
* `evaluate` is play.py:537-705's evaluation loop for those actors: one policy
  call per decision, the action held for `decision_period` env steps, rewards
  of an env counted until it finishes inside the decision, done envs' actions
  zeroed for the rest of the decision, LSTM memories of done envs cleared, and
  the decision cut short once every env has finished. Completed episode
  returns are listed in the order play.py appends them.
"""

from __future__ import annotations

import torch

from .config import PAPER_PARITY_VERSION
from .poca_networks import Actor, DiscreteActor, POCACritic, RecurrentDiscreteActor, checkpoint_memory_size

OPTION_TRAINERS = ("option_critic", "learned_option_critic")


def poca_checkpoint(actor, critic: POCACritic, optimizer=None, *, obs_dim: int, global_step: int = 0,
                    update_count: int = 0,
                    seed: int = 0, hidden_dim: int = 256, num_layers: int = 2, memory_size: int = 0,
                    sequence_length: int = 0, critic_hidden_dim: int = 256, critic_num_layers: int = 2,
                    critic_num_heads: int = 4, decision_period: int = 5, state_dim: int = 5,
                    act_dim: int | None = None) -> dict:
    """The checkpoint dict of PT:1057-1083 for these modules. A checkpoint without an
    optimizer state loads in play.py only: the reference's load_checkpoint
    (PT:1085-1106) hands the empty dict to ``optimizer.load_state_dict``."""
    recurrent = isinstance(actor, RecurrentDiscreteActor)
    if recurrent:
        # ML-Agents total memory (h and c) = 2 x LSTM units (poca_networks.py:85-113)
        total = 2 * int(actor.hidden_size)
        if memory_size in (0, None):
            memory_size = total
        elif int(memory_size) != total:
            raise ValueError(f"memory_size {memory_size} disagrees with the recurrent actor's {total}")
    discrete = isinstance(actor, (DiscreteActor, RecurrentDiscreteActor))
    return {
        "paper_parity_version": PAPER_PARITY_VERSION,
        "actor": actor.state_dict(),
        "critic": critic.state_dict(),
        "optimizer": optimizer.state_dict() if optimizer is not None else {},
        "global_step": int(global_step),
        "update_count": int(update_count),
        "seed": int(seed),
        "hidden_dim": int(hidden_dim),
        "num_layers": int(num_layers),
        "recurrent": recurrent,
        "memory_size": int(memory_size),
        "memory_size_semantics": "mlagents_total",
        "lstm_hidden_size": actor.hidden_size if recurrent else 0,
        "sequence_length": int(sequence_length),
        "critic_hidden_dim": int(critic_hidden_dim),
        "critic_num_layers": int(critic_num_layers),
        "critic_num_heads": int(critic_num_heads),
        "decision_period": int(decision_period),
        "discrete": discrete,
        "num_actions": int(actor.num_actions) if discrete else 0,
        "act_dim": int(act_dim if act_dim is not None else (1 if discrete else actor.mu_head.out_features)),
        "state_dim": int(state_dim),
        "obs_dim": int(obs_dim),
    }


def save_poca_checkpoint(path, actor, critic, optimizer=None, **meta) -> None:
    torch.save(poca_checkpoint(actor, critic, optimizer, **meta), path)


def read_checkpoint(path_or_dict, map_location="cpu") -> dict:
    if isinstance(path_or_dict, dict):
        return path_or_dict
    return torch.load(path_or_dict, map_location=map_location, weights_only=True)


def load_poca_checkpoint(path_or_dict, actor, critic, optimizer=None, map_location="cpu") -> tuple[int, int]:
    """PT:1085-1106: refuse other parity versions, load strictly; returns
    (global_step, update_count)."""
    ckpt = read_checkpoint(path_or_dict, map_location)
    version = int(ckpt.get("paper_parity_version", 0))
    if version != PAPER_PARITY_VERSION:
        raise RuntimeError(
            f"Refusing to resume a parity-v{version} checkpoint with the parity-v{PAPER_PARITY_VERSION} "
            "trainer. Its critic architecture or training semantics may differ.")
    try:
        actor.load_state_dict(ckpt["actor"])
        critic.load_state_dict(ckpt["critic"])
        if optimizer is not None:
            optimizer.load_state_dict(ckpt["optimizer"])
    except RuntimeError as exc:
        raise RuntimeError("Checkpoint architecture does not match the paper-parity trainer.") from exc
    return int(ckpt["global_step"]), int(ckpt["update_count"])


def actor_from_checkpoint(path_or_dict, obs_dim: int, device="cpu"):
    """play.py:379-436 for POCA checkpoints: (actor in eval mode, info dict)."""
    ckpt = read_checkpoint(path_or_dict)
    trainer_type = ckpt.get("trainer_type", "poca")
    if trainer_type in OPTION_TRAINERS:
        raise NotImplementedError(f"{trainer_type} checkpoints need the option-critic networks, "
                                  "which this build does not carry (DESIGN.md §9)")
    discrete = bool(ckpt.get("discrete", False))
    hidden_dim = int(ckpt.get("hidden_dim", 256))
    num_layers = int(ckpt.get("num_layers", 2))
    num_actions = int(ckpt.get("num_actions", 6))
    recurrent = bool(ckpt.get("recurrent", False))
    memory_size = checkpoint_memory_size(ckpt)
    act_dim = int(ckpt.get("act_dim", 2))
    if recurrent and not discrete:
        raise ValueError("Recurrent playback is only implemented for discrete actors")
    if discrete and recurrent:
        actor = RecurrentDiscreteActor(obs_dim, num_actions, hidden_dim, num_layers, memory_size)
    elif discrete:
        actor = DiscreteActor(obs_dim, num_actions, hidden_dim, num_layers)
    else:
        actor = Actor(obs_dim, act_dim, hidden_dim, num_layers)
    actor = actor.to(device)
    actor.load_state_dict(ckpt["actor"])
    actor.eval()
    info = {"trainer_type": trainer_type, "discrete": discrete, "recurrent": recurrent, "act_dim": act_dim,
            "num_actions": num_actions, "hidden_dim": hidden_dim, "num_layers": num_layers,
            "memory_size": memory_size, "decision_period": int(ckpt.get("decision_period", 5))}
    return actor, info


@torch.no_grad()
def evaluate(env, actor, num_episodes: int, decision_period: int, deterministic: bool = False) -> list[float]:
    """play.py:537-705 (POCA actors): returns the completed episodes' rewards."""
    agents = env.possible_agents
    E, N = env.num_envs, len(agents)
    dev = env.device
    discrete = isinstance(actor, (DiscreteActor, RecurrentDiscreteActor))
    recurrent = isinstance(actor, RecurrentDiscreteActor)
    mem_h = mem_c = None
    if recurrent:
        mem_h, mem_c = actor.initial_state(E * N, dev)
    obs_dict, _ = env.reset()
    ep_reward = torch.zeros(E, device=dev)
    episode_rewards: list[float] = []
    count = 0
    while count < num_episodes:
        flat_obs = torch.stack([obs_dict[a] for a in agents], dim=1).reshape(E * N, -1)
        if recurrent:
            logits, nxt = actor.step(flat_obs, (mem_h, mem_c))
            mem_h, mem_c = nxt[0], nxt[1]
            flat_act = logits.argmax(dim=-1) if deterministic else torch.distributions.Categorical(
                logits=logits).sample()
            all_actions = flat_act.view(E, N, 1)
        else:
            if deterministic:
                flat_act = actor(flat_obs).argmax(dim=-1) if discrete else actor(flat_obs)[0]
            else:
                flat_act = actor.get_dist(flat_obs).sample()
            all_actions = (flat_act.view(E, N, 1) if discrete
                           else flat_act.clamp(-3, 3).div_(3).view(E, N, -1))
        action_dict = {a: all_actions[:, i] for i, a in enumerate(agents)}
        active = torch.ones(E, dtype=torch.bool, device=dev)
        for _ in range(decision_period):
            obs_dict, rew, term, trunc, _ = env.step(action_dict)
            ep_reward += rew[agents[0]] * active.float()
            done = term[agents[0]] | trunc[agents[0]]
            newly = active & done
            if newly.any():
                for ei in newly.nonzero(as_tuple=False).flatten().tolist():
                    episode_rewards.append(ep_reward[ei].item())
                    ep_reward[ei] = 0.0
                    if recurrent:
                        mem_h[:, ei * N:(ei + 1) * N, :] = 0.0
                        mem_c[:, ei * N:(ei + 1) * N, :] = 0.0
                    count += 1
                    if count >= num_episodes:
                        break
                for a in agents:
                    action_dict[a][newly] = 0
                active = active & ~done
                if count >= num_episodes or not active.any():
                    break
    return episode_rewards
