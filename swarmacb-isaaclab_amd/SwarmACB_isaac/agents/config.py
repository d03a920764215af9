"""ML-Agents-style YAML configs (drop-in for agents/config_loader.py,
network_config.py and the three trainer config dataclasses).

``load_config(path)`` returns what the reference's returns
(config_loader.py:30-186): ``(run_name, variant, cfg, env_overrides)`` with
``cfg`` one of ``POCAConfig`` (poca_trainer.py:44-110),
``FixedOptionCriticConfig`` (option_critic_trainer.py:34-96) or
``LearnedOptionCriticConfig`` (learned_option_critic_trainer.py:75-167), same
fields, defaults and resolution rules, so the reference's 40 ``configs/*.yaml``
load unchanged. ``make_env_cfg`` applies the result to this package's env cfg
the way scripts/train.py:165-185 does.
"""

from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Any, Mapping

import yaml

PAPER_PARITY_VERSION = 5


@dataclass
class POCAConfig:
    """poca_trainer.py:44-110."""

    horizon: int = 1000
    num_epochs: int = 3
    mini_batch_size: int = 2048
    clip_eps: float = 0.2
    beta: float = 0.005
    gamma: float = 0.99
    lam: float = 0.95
    lr: float = 3e-4
    adam_eps: float = 1e-8
    lr_schedule: str = "constant"
    eps_schedule: str = "constant"
    beta_schedule: str = "constant"
    total_timesteps: int = 120_000_000
    checkpoint_interval: int = 120_000
    summary_freq: int = 120_000
    keep_checkpoints: int = 5
    checkpoint_dir: str = "checkpoints/poca"
    seed: int = 0
    decision_period: int = 5
    reward_strength: float = 1.0
    hidden_dim: int = 512
    num_layers: int = 2
    critic_hidden_dim: int = 128
    critic_num_layers: int = 2
    critic_num_heads: int = 4
    recurrent: bool = False
    memory_size: int = 128
    sequence_length: int = 128
    log_dir: str = "runs/poca"
    buffer_size_hint: int = 0

    @property
    def log_interval(self) -> int:
        return 10

    @property
    def save_interval(self) -> int:
        return 50


@dataclass
class FixedOptionCriticConfig:
    """option_critic_trainer.py:34-96."""

    trainer_type: str = "option_critic"
    horizon: int = 1000
    num_epochs: int = 3
    mini_batch_size: int = 2048
    clip_eps: float = 0.2
    beta: float = 0.005
    value_coef: float = 0.5
    option_value_coef: float = 0.5
    baseline_coef: float = 0.25
    termination_coef: float = 0.1
    termination_entropy_coef: float = 0.001
    termination_penalty: float = 0.01
    gamma: float = 0.99
    lam: float = 0.95
    lr: float = 3e-4
    adam_eps: float = 1e-8
    lr_schedule: str = "constant"
    eps_schedule: str = "constant"
    beta_schedule: str = "constant"
    total_timesteps: int = 120_000_000
    checkpoint_interval: int = 120_000
    summary_freq: int = 120_000
    keep_checkpoints: int = 5
    checkpoint_dir: str = "checkpoints/option_critic"
    seed: int = 0
    decision_period: int = 5
    reward_strength: float = 1.0
    hidden_dim: int = 128
    num_layers: int = 1
    critic_hidden_dim: int = 128
    critic_num_layers: int = 2
    critic_num_heads: int = 4
    recurrent: bool = True
    memory_size: int = 128
    sequence_length: int = 128
    num_options: int = 6
    log_dir: str = "runs/option_critic"
    buffer_size_hint: int = 0


@dataclass
class LearnedOptionCriticConfig:
    """learned_option_critic_trainer.py:75-167."""

    trainer_type: str = "learned_option_critic"
    horizon: int = 1000
    num_epochs: int = 3
    mini_batch_size: int = 4096
    clip_eps: float = 0.2
    beta: float = 0.001
    intra_option_coef: float = 1.0
    selector_coef: float = 0.0
    local_option_value_coef: float = 0.5
    option_entropy_coef: float = 0.0
    option_balance_coef: float = 0.0
    option_balance_final_coef: float = 0.0
    value_coef: float = 0.5
    action_baseline_coef: float = 0.25
    option_value_coef: float = 0.5
    option_baseline_coef: float = 0.25
    termination_coef: float = 1.0
    termination_entropy_coef: float = 0.0
    termination_penalty: float = 0.0
    termination_prior_probability: float = 0.05
    termination_prior_coef: float = 0.0
    termination_prior_final_coef: float = 0.0
    attention_diversity_coef: float = 0.002
    attention_temporal_coef: float = 0.001
    gamma: float = 0.99
    lam: float = 0.95
    lr: float = 3e-4
    actor_lr: float = 3e-4
    adam_eps: float = 1e-8
    lr_schedule: str = "constant"
    eps_schedule: str = "constant"
    beta_schedule: str = "constant"
    option_epsilon_start: float = 1.0
    option_epsilon_final: float = 0.1
    option_epsilon_schedule: str = "linear"
    option_epsilon_decay_fraction: float = 0.1
    max_grad_norm: float = 10.0
    actor_max_grad_norm: float = 1.0
    target_kl: float = 0.01
    adaptive_actor_lr: bool = False
    actor_lr_scale_min: float = 0.05
    actor_lr_decay_factor: float = 1.5
    actor_lr_recovery_factor: float = 1.05
    fused_optimizer: bool = True
    matmul_precision: str = "high"
    total_timesteps: int = 120_000_000
    checkpoint_interval: int = 120_000
    summary_freq: int = 120_000
    keep_checkpoints: int = 5
    checkpoint_dir: str = "checkpoints/learned_option_critic"
    seed: int = 0
    decision_period: int = 5
    reward_strength: float = 1.0
    hidden_dim: int = 128
    num_layers: int = 1
    critic_hidden_dim: int = 128
    critic_num_layers: int = 1
    critic_num_heads: int = 4
    recurrent: bool = True
    memory_size: int = 128
    sequence_length: int = 128
    num_options: int = 6
    option_hidden_dim: int = 512
    option_num_layers: int = 2
    option_memory_size: int = 64
    initial_termination_probability: float = 0.27
    initial_log_std: float = 0.0
    min_log_std: float = -2.5
    max_log_std: float = 0.0
    option_selector_temperature: float = 1.0
    log_dir: str = "runs/learned_option_critic"
    buffer_size_hint: int = 0


# trainer_type spellings (config_loader.py:69-84) -> (config class, canonical name)
_TRAINERS = {}
for _names, _cls, _canon in (
        (("learned_option_critic", "option_critic_2", "learned_oc", "oc2"), LearnedOptionCriticConfig,
         "learned_option_critic"),
        (("option_critic", "fixed_option_critic", "fixed_oc", "oc"), FixedOptionCriticConfig, "option_critic"),
        (("poca",), POCAConfig, "poca")):
    for _n in _names:
        _TRAINERS[_n] = (_cls, _canon)

# YAML hyperparameter key -> cfg attribute, applied only where the cfg has it (config_loader.py:93-139)
_OPTIONAL_HYPERS = {k: k for k in (
    "termination_penalty", "termination_coef", "termination_entropy_coef", "value_coef", "option_value_coef",
    "baseline_coef", "intra_option_coef", "selector_coef", "local_option_value_coef", "option_entropy_coef",
    "option_balance_coef", "option_balance_final_coef", "action_baseline_coef", "option_baseline_coef",
    "attention_diversity_coef", "attention_temporal_coef", "initial_termination_probability",
    "termination_prior_probability", "termination_prior_coef", "termination_prior_final_coef", "initial_log_std",
    "min_log_std", "max_log_std", "max_grad_norm", "actor_max_grad_norm", "target_kl", "adaptive_actor_lr",
    "actor_lr_scale_min", "actor_lr_decay_factor", "actor_lr_recovery_factor", "fused_optimizer",
    "matmul_precision", "option_selector_temperature", "option_epsilon_start", "option_epsilon_final",
    "option_epsilon_decay_fraction")}
_OPTIONAL_HYPERS.update({"actor_learning_rate": "actor_lr", "option_value_temperature": "option_selector_temperature"})

# always-present hyperparameters: YAML key -> cfg attribute
_HYPERS = {"batch_size": "mini_batch_size", "learning_rate": "lr", "beta": "beta", "epsilon": "clip_eps",
           "lambd": "lam", "num_epoch": "num_epochs"}


def apply_network_settings(cfg: Any, network: Mapping[str, Any], critic: Mapping[str, Any], variant: str,
                           block: Mapping[str, Any]) -> Any:
    """network_config.py:14-59: the critic inherits the actor's NetworkSettings
    unless critic_settings overrides a field; cyclamen is always recurrent."""
    cfg.hidden_dim = network.get("hidden_units", cfg.hidden_dim)
    cfg.num_layers = network.get("num_layers", cfg.num_layers)
    cfg.critic_hidden_dim = critic.get("hidden_units", cfg.hidden_dim)
    cfg.critic_num_layers = critic.get("num_layers", cfg.num_layers)
    cfg.critic_num_heads = critic.get("num_heads", cfg.critic_num_heads)
    if hasattr(cfg, "num_options"):
        cfg.num_options = network.get("num_options", block.get("num_options", cfg.num_options))
    if hasattr(cfg, "option_hidden_dim"):
        cfg.option_hidden_dim = network.get("option_hidden_units", cfg.option_hidden_dim)
        cfg.option_num_layers = network.get("option_num_layers", cfg.option_num_layers)
    memory = network.get("memory", {})
    cfg.recurrent = bool(memory) or variant == "cyclamen"
    if cfg.recurrent:
        cfg.memory_size = memory.get("memory_size", cfg.memory_size)
        cfg.sequence_length = memory.get("sequence_length", cfg.sequence_length)
        if hasattr(cfg, "option_memory_size"):
            cfg.option_memory_size = memory.get("option_memory_size", cfg.option_memory_size)
    return cfg


def config_from_document(doc: Mapping[str, Any]) -> tuple[str, str, Any, dict[str, Any]]:
    """load_config on an already parsed YAML document."""
    behaviors = doc.get("behaviors", doc)
    if not behaviors:
        raise ValueError("Config must have a top-level 'behaviors' key.")
    run_name = next(iter(behaviors))
    block = behaviors[run_name]
    variant = block.get("variant", "dandelion")
    trainer_type = block.get("trainer_type", "poca").lower()
    hypers = block.get("hyperparameters", {})
    network = block.get("network_settings", {})
    environment = block.get("environment", {})
    task_id = block.get("task", environment.get("task", None))
    if trainer_type not in _TRAINERS:
        raise ValueError(f"Unsupported trainer_type: {trainer_type}")
    cls, canon = _TRAINERS[trainer_type]
    cfg = cls()
    cfg.trainer_type = canon
    for key, attr in _HYPERS.items():
        setattr(cfg, attr, hypers.get(key, getattr(cfg, attr)))
    for key, attr in _OPTIONAL_HYPERS.items():
        if hasattr(cfg, attr):
            setattr(cfg, attr, hypers.get(key, getattr(cfg, attr)))
    cfg.lr_schedule = hypers.get("learning_rate_schedule", "constant")
    cfg.eps_schedule = hypers.get("epsilon_schedule", "constant")
    cfg.beta_schedule = hypers.get("beta_schedule", "constant")
    if hasattr(cfg, "option_epsilon_schedule"):
        cfg.option_epsilon_schedule = hypers.get("option_epsilon_schedule", cfg.option_epsilon_schedule)
    apply_network_settings(cfg, network, block.get("critic_settings", {}), variant, block)
    extrinsic = block.get("reward_signals", {}).get("extrinsic", {})
    cfg.gamma = extrinsic.get("gamma", cfg.gamma)
    cfg.reward_strength = extrinsic.get("strength", 1.0)
    cfg.total_timesteps = block.get("max_steps", cfg.total_timesteps)
    cfg.horizon = block.get("time_horizon", cfg.horizon)
    cfg.summary_freq = block.get("summary_freq", 120000)
    cfg.checkpoint_interval = block.get("checkpoint_interval", 120000)
    cfg.keep_checkpoints = block.get("keep_checkpoints", 5)
    cfg.buffer_size_hint = hypers.get("buffer_size", 0)
    cfg.decision_period = environment.get("decision_period", cfg.decision_period)
    cfg.log_dir = f"runs/{run_name}"
    cfg.checkpoint_dir = f"checkpoints/{run_name}"
    env_overrides: dict[str, Any] = {}
    if task_id is not None:
        env_overrides["task"] = task_id
    env_overrides.update({k: v for k, v in environment.items() if k not in ("task", "decision_period")})
    return run_name, variant, cfg, env_overrides


def load_config(path: str | Path) -> tuple[str, str, Any, dict[str, Any]]:
    """config_loader.py:30-186."""
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(f"Config file not found: {path}")
    with open(path, "r", encoding="utf-8") as f:
        return config_from_document(yaml.safe_load(f))


def make_env_cfg(task_id: str, variant: str, env_overrides: Mapping[str, Any], trainer_type: str = "poca",
                 seed: int = 0):
    """The env cfg scripts/train.py:165-185 builds before gym.make: registry cfg
    class, seed, variant, continuous primitive actions for learned OC, overrides."""
    from ..registry import cfg_class

    env_cfg = cfg_class(task_id)()
    env_cfg.seed = seed
    env_cfg.update_variant(variant)
    if trainer_type == "learned_option_critic":
        env_cfg.use_continuous_actions(full_observations=True)
    ignored = []
    for key, value in env_overrides.items():
        if key == "task":
            continue
        if key == "num_envs":
            env_cfg.scene.num_envs = value
        elif hasattr(env_cfg, key):
            setattr(env_cfg, key, value)
        else:
            ignored.append(key)
    for key in ignored:
        print(f"[Train] Warning: ignored unknown environment override {key!r}")
    return env_cfg


_TRAINER_LABELS = {"learned_option_critic": "Learned Option-Critic (Phase 2)",
                   "option_critic": "Fixed Option-Critic (Phase 1)", "poca": "POCA"}


def config_summary(run_name: str, variant: str, cfg: Any, env_ov: Mapping[str, Any]) -> list[tuple[str, str]]:
    """(section, "label : value") rows of the console summary (config_loader.py:193-322)."""
    rows: list[tuple[str, str]] = []
    tt = getattr(cfg, "trainer_type", "poca")

    def add(sec, label, value):
        rows.append((sec, f"{label:20s}: {value}"))

    add("Run", "Run name", run_name)
    add("Run", "CASA variant", variant)
    add("Run", "Trainer", _TRAINER_LABELS.get(tt, tt))
    h = "Hyperparameters"
    add(h, "batch_size", cfg.mini_batch_size)
    add(h, "learning_rate", f"{cfg.lr}  (schedule: {cfg.lr_schedule})")
    add(h, "beta", f"{cfg.beta}  (schedule: {cfg.beta_schedule})")
    add(h, "epsilon", f"{cfg.clip_eps}  (schedule: {cfg.eps_schedule})")
    for label, attr in (("lambd", "lam"), ("num_epoch", "num_epochs"), ("gamma", "gamma"),
                        ("termination_penalty", "termination_penalty"), ("termination_coef", "termination_coef"),
                        ("termination_entropy", "termination_entropy_coef"), ("value_coef", "value_coef"),
                        ("option_value_coef", "option_value_coef"), ("baseline_coef", "baseline_coef"),
                        ("intra_option_coef", "intra_option_coef"), ("selector_coef", "selector_coef"),
                        ("local_option_value", "local_option_value_coef"),
                        ("action_baseline", "action_baseline_coef"), ("option_baseline", "option_baseline_coef"),
                        ("option_entropy", "option_entropy_coef"),
                        ("attention_diversity", "attention_diversity_coef"),
                        ("attention_temporal", "attention_temporal_coef"),
                        ("initial_termination", "initial_termination_probability"),
                        ("actor_learning_rate", "actor_lr"), ("actor_max_grad_norm", "actor_max_grad_norm"),
                        ("target_kl", "target_kl"), ("adaptive_actor_lr", "adaptive_actor_lr"),
                        ("fused_optimizer", "fused_optimizer"), ("matmul_precision", "matmul_precision")):
        if hasattr(cfg, attr):
            add(h, label, getattr(cfg, attr))
    if hasattr(cfg, "option_balance_coef"):
        add(h, "option_balance", f"{cfg.option_balance_coef} -> {cfg.option_balance_final_coef}")
        add(h, "option_exploration", f"epsilon={cfg.option_epsilon_start} -> {cfg.option_epsilon_final} "
                                     f"({cfg.option_epsilon_schedule}, first "
                                     f"{100.0 * cfg.option_epsilon_decay_fraction:g}% of training)")
    n = "Network"
    add(n, "hidden_units", cfg.hidden_dim)
    add(n, "num_layers", cfg.num_layers)
    add(n, "critic_hidden", cfg.critic_hidden_dim)
    add(n, "critic_layers", cfg.critic_num_layers)
    add(n, "critic_heads", cfg.critic_num_heads)
    if hasattr(cfg, "option_hidden_dim"):
        add(n, "option_hidden", cfg.option_hidden_dim)
        add(n, "option_layers", cfg.option_num_layers)
    if hasattr(cfg, "num_options"):
        add(n, "learned_options" if tt == "learned_option_critic" else "fixed_options", cfg.num_options)
    if cfg.recurrent:
        add(n, "memory_size", f"{cfg.memory_size} ({cfg.memory_size // 2} LSTM units)")
        if hasattr(cfg, "option_memory_size"):
            add(n, "option_memory", f"{cfg.option_memory_size} ({cfg.option_memory_size // 2} LSTM units/option)")
        add(n, "sequence_length", cfg.sequence_length)
    t = "Training"
    add(t, "seed", cfg.seed)
    add(t, "max_steps", f"{cfg.total_timesteps:,}")
    if cfg.buffer_size_hint:
        add(t, "buffer_size", f"{cfg.buffer_size_hint:,} (ML-Agents reference target)")
    add(t, "time_horizon", cfg.horizon)
    add(t, "decision_period", cfg.decision_period)
    add(t, "checkpoint_interval", f"{cfg.checkpoint_interval:,}")
    add(t, "summary_freq", f"{cfg.summary_freq:,}")
    if cfg.reward_strength != 1.0:
        add(t, "reward_strength", cfg.reward_strength)
    for k, v in env_ov.items():
        add("Environment overrides", k, v)
    return rows


def print_config(run_name: str, variant: str, cfg: Any, env_ov: Mapping[str, Any]) -> None:
    """Console summary of a resolved config (config_loader.py:193-322)."""
    sep = "-" * 60
    print(f"\n{sep}\n  SwarmACB Training Config\n{sep}")
    section = None
    for sec, line in config_summary(run_name, variant, cfg, env_ov):
        if sec != section and sec != "Run":
            if section == "Run":
                print(sep)
            print(f"  {sec}")
        section = sec
        print(f"    {line}" if sec != "Run" else f"  {line}")
    print(f"{sep}\n")
