"""POCA checkpoint format and headless playback.

* `poca_checkpoint` / `save_poca_checkpoint` write the dict of
  PT:1056-1083 (`POCATrainer.save_checkpoint`), key for key, so a checkpoint
  written here loads in the reference's `play.py` (and, when it carries the
  optimizer state, resumes in its trainer) and vice versa.
* `load_poca_checkpoint` follows PT:1085-1106: the paper-parity version must
  match and the actor / critic (/ optimizer) state dicts must load strictly.
  Files are read with `torch.load(weights_only=True)`: a checkpoint holds
  tensors, numbers, strings and optimizer state only.
* `actor_from_checkpoint` rebuilds the policy the way play.py:379-436 does:
  Actor / DiscreteActor / RecurrentDiscreteActor for POCA checkpoints from the
  stored architecture keys, the FixedOptionManager of an ``option_critic``
  checkpoint, the LearnedOptionActor of a ``learned_option_critic`` one
  (``LearnedOptionActor.from_checkpoint``).
* `PlaybackPolicy` is the per-decision action choice of play.py:528-671 for
  all five kinds (Gaussian, categorical, recurrent categorical, fixed-option
  call-and-return, learned-option call-and-return with its wheel policy and
  the checkpoint's action transform), stochastic or deterministic.
* `evaluate` is play.py:537-705's evaluation loop: one policy call per
  decision, the action held for `decision_period` env steps, rewards of an env
  counted until it finishes inside the decision, done envs' actions zeroed for
  the rest of the decision, LSTM memories (and current options) of done envs
  cleared, and the decision cut short once every env has finished. Completed
  episode returns are listed in the order play.py appends them.
"""

from __future__ import annotations

import torch

from .config import PAPER_PARITY_VERSION
from .learned_option_critic_networks import LearnedOptionActor
from .option_critic_networks import FixedOptionManager
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
    """play.py:379-436: (network in eval mode, info dict) for every trainer's checkpoint."""
    ckpt = read_checkpoint(path_or_dict)
    trainer_type = ckpt.get("trainer_type", "poca")
    discrete = bool(ckpt.get("discrete", False))
    hidden_dim = int(ckpt.get("hidden_dim", 256))
    num_layers = int(ckpt.get("num_layers", 2))
    num_actions = int(ckpt.get("num_actions", 6))
    num_options = int(ckpt.get("num_options", num_actions))
    recurrent = bool(ckpt.get("recurrent", False))
    memory_size = checkpoint_memory_size(ckpt)
    act_dim = int(ckpt.get("act_dim", 2))
    if trainer_type not in OPTION_TRAINERS and recurrent and not discrete:
        raise ValueError("Recurrent playback is only implemented for discrete actors")
    if trainer_type == "learned_option_critic":
        actor = LearnedOptionActor.from_checkpoint(ckpt, device)
        if actor.obs_dim != obs_dim:
            raise RuntimeError(f"OC2 checkpoint expects obs_dim={actor.obs_dim}, but the environment produced "
                               f"obs_dim={obs_dim}.")
    elif trainer_type == "option_critic":
        actor = FixedOptionManager(obs_dim, num_options, hidden_dim, num_layers, memory_size).to(device)
        actor.load_state_dict(ckpt["manager"])
    else:
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
            "num_actions": num_actions, "num_options": num_options, "hidden_dim": hidden_dim,
            "num_layers": num_layers, "memory_size": memory_size,
            "decision_period": int(ckpt.get("decision_period", 5)),
            "option_epsilon": float(ckpt.get("current_option_epsilon", ckpt.get("option_epsilon_final", 0.1))),
            "action_transform": ckpt.get("action_transform", "identity_normalized")}
    return actor, info


class PlaybackPolicy:
    """The action choice of one decision for every checkpoint kind (play.py:528-671)."""

    def __init__(self, net, num_envs: int, num_agents: int, device, deterministic: bool = False,
                 option_epsilon: float = 0.1, action_transform: str = "identity_normalized"):
        self.net, self.E, self.N, self.device = net, int(num_envs), int(num_agents), device
        self.deterministic = bool(deterministic)
        self.option_epsilon, self.action_transform = float(option_epsilon), action_transform
        if isinstance(net, LearnedOptionActor):
            self.kind = "learned_option_critic"
        elif isinstance(net, FixedOptionManager):
            self.kind = "option_critic"
        elif isinstance(net, RecurrentDiscreteActor):
            self.kind = "recurrent"
        elif isinstance(net, DiscreteActor):
            self.kind = "discrete"
        else:
            self.kind = "continuous"
        self.memory = None
        if self.kind in ("learned_option_critic", "option_critic", "recurrent"):
            self.memory = net.initial_state(self.E * self.N, device)
        self.current_options = (torch.full((self.E, self.N), -1, dtype=torch.long, device=device)
                                if self.kind in OPTION_TRAINERS else None)

    def _switch(self, proposed, beta_logits):
        """Call-and-return: keep the option unless it terminates (or none is set)."""
        if self.deterministic:
            terminate = (beta_logits > 0.0).view(self.E, self.N)
        else:
            terminate = torch.distributions.Bernoulli(validate_args=False, logits=beta_logits).sample().bool().view(self.E, self.N)
        self.current_options = torch.where(terminate | (self.current_options < 0), proposed.view(self.E, self.N),
                                           self.current_options)

    @torch.no_grad()
    def act(self, flat_obs: torch.Tensor) -> torch.Tensor:
        """(E*N, obs) -> the (E, N, k) action tensor the env receives."""
        E, N, net, det = self.E, self.N, self.net, self.deterministic
        if self.kind == "learned_option_critic":
            _s, values, term, means, stds, _a, nm = net.step(flat_obs, self.memory)
            self.memory = (nm[0], nm[1])
            proposed = values.argmax(dim=-1) if det else net.option_dist(values, epsilon=self.option_epsilon).sample()
            self._switch(proposed, net.selected_termination_logits(term, self.current_options.clamp(min=0)
                                                                   .reshape(-1)))
            dist = net.selected_action_dist(means, stds, self.current_options.reshape(-1))
            raw = dist.mean if det else dist.sample()
            if self.action_transform == "clip_minus3_3_divide3":
                raw = raw.clamp(-3.0, 3.0) / 3.0
            elif self.action_transform != "identity_normalized":
                raise RuntimeError(f"Unsupported learned Option-Critic action transform {self.action_transform!r}.")
            return raw.view(E, N, -1)
        if self.kind == "option_critic":
            logits, term, nm = net.step(flat_obs, self.memory)
            self.memory = (nm[0], nm[1])
            proposed = logits.argmax(dim=-1) if det else torch.distributions.Categorical(validate_args=False, logits=logits).sample()
            self._switch(proposed, term.gather(-1, self.current_options.clamp(min=0).reshape(-1, 1)).squeeze(-1))
            return self.current_options.unsqueeze(-1)
        if self.kind == "recurrent":
            logits, nm = net.step(flat_obs, self.memory)
            self.memory = (nm[0], nm[1])
            act = logits.argmax(dim=-1) if det else torch.distributions.Categorical(validate_args=False, logits=logits).sample()
            return act.view(E, N, 1)
        if self.kind == "discrete":
            act = net(flat_obs).argmax(dim=-1) if det else net.get_dist(flat_obs).sample()
            return act.view(E, N, 1)
        act = net(flat_obs)[0] if det else net.get_dist(flat_obs).sample()
        return act.clamp(-3, 3).div_(3).view(E, N, -1)      # ML-Agents preprocessing

    def reset_env(self, ei: int):
        """A finished env: its options back to -1 and its robots' memories cleared."""
        if self.current_options is not None:
            self.current_options[ei] = -1
        if self.memory is not None:
            self.memory[0][:, ei * self.N:(ei + 1) * self.N, :] = 0.0
            self.memory[1][:, ei * self.N:(ei + 1) * self.N, :] = 0.0


@torch.no_grad()
def evaluate(env, actor, num_episodes: int, decision_period: int, deterministic: bool = False,
             **policy_kw) -> list[float]:
    """play.py:537-705: returns the completed episodes' rewards. `actor` is a network
    from actor_from_checkpoint (policy_kw: option_epsilon / action_transform) or a
    PlaybackPolicy."""
    agents = env.possible_agents
    E, N = env.num_envs, len(agents)
    dev = env.device
    policy = actor if isinstance(actor, PlaybackPolicy) else PlaybackPolicy(actor, E, N, dev, deterministic,
                                                                            **policy_kw)
    obs_dict, _ = env.reset()
    ep_reward = torch.zeros(E, device=dev)
    episode_rewards: list[float] = []
    count = 0
    while count < num_episodes:
        flat_obs = torch.stack([obs_dict[a] for a in agents], dim=1).reshape(E * N, -1)
        all_actions = policy.act(flat_obs)
        # views, as in play.py:640-641: for the fixed-option kind all_actions IS a view of
        # the current options, so zeroing a finished env's actions below (play.py:703)
        # also turns its freshly reset option (-1, play.py:689) into option 0 — the
        # reference's effective semantics, reproduced rather than "fixed"
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
                    policy.reset_env(ei)
                    count += 1
                    if count >= num_episodes:
                        break
                for a in agents:
                    action_dict[a][newly] = 0
                active = active & ~done
                if count >= num_episodes or not active.any():
                    break
    return episode_rewards
