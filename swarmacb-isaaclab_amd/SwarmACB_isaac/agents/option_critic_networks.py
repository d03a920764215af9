"""Fixed-option manager of the phase-1 Option-Critic (drop-in for
agents/option_critic_networks.py:FixedOptionManager, lines 20-111).

The six ACB behaviour modules are the options; the shared per-robot network
only selects an option (pi_O) and decides when to terminate it (beta_o). Module
tree, parameter names and initialisation order follow the reference so its
checkpoints load unchanged and a seeded construction draws the same weights.
The LSTM goes through ``poca_networks._lstm``: at rollout time (one step, no
autograd, on the GPU) the cell update is the swarm_lstm_cell HIP kernel.
"""

from __future__ import annotations

import torch
import torch.nn as nn
from torch.distributions import Bernoulli, Categorical

from .poca_networks import LinearEncoder, _linear_layer, _lstm, _mlagents_lstm


class FixedOptionManager(nn.Module):
    """Shared recurrent option selector + per-option termination heads
    (option_critic_networks.py:20-111)."""

    def __init__(self, obs_dim: int, num_options: int, hidden: int = 128, num_layers: int = 1,
                 memory_size: int = 128):
        super().__init__()
        self.obs_dim, self.num_options, self.memory_size = obs_dim, num_options, memory_size
        self.encoder = LinearEncoder(obs_dim, num_layers, hidden, kernel_init="kaiming_normal")
        self.lstm, self.hidden_size = _mlagents_lstm(hidden, memory_size)
        # ML-Agents categorical gain for the selector, a wider 0.2 for the Bernoulli heads (OCN:51-65)
        self.option_head = _linear_layer(self.hidden_size, num_options, kernel_init="kaiming_normal",
                                         kernel_gain=0.1)
        self.termination_head = _linear_layer(self.hidden_size, num_options, kernel_init="kaiming_normal",
                                              kernel_gain=0.2)
        nn.init.constant_(self.termination_head.bias, -1.0)   # options persist at the start (OCN:66-67)

    def initial_state(self, batch_size: int, device):
        z = torch.zeros(1, batch_size, self.hidden_size, device=device)
        return z, z.clone()

    def forward_sequence(self, obs_seq: torch.Tensor, state=None, keep: torch.Tensor | None = None):
        """(B, T, obs) -> selector logits (B, T, O), termination logits (B, T, O), memory.
        keep (B, T): the memory is multiplied by keep[:, t] after step t."""
        out, nxt = _lstm(*self.sequence_lstm_item(obs_seq, state, keep))
        return self.option_head(out), self.termination_head(out), nxt

    def sequence_lstm_item(self, obs_seq: torch.Tensor, state=None, keep: torch.Tensor | None = None):
        """forward_sequence up to its LSTM: (lstm, encoded sequence, state, keep) for
        poca_networks.lstm_sequences; the heads then take the LSTM output."""
        B, T = obs_seq.shape[:2]
        enc = self.encoder(obs_seq.reshape(B * T, self.obs_dim)).view(B, T, -1)
        return self.lstm, enc, state if state is not None else self.initial_state(B, obs_seq.device), keep

    def step(self, obs: torch.Tensor, state=None):
        opt, term, nxt = self.forward_sequence(obs.unsqueeze(1), state)
        return opt[:, 0], term[:, 0], nxt

    def get_option_dist(self, option_logits: torch.Tensor) -> Categorical:
        return Categorical(validate_args=False, logits=option_logits)

    def get_termination_dist(self, termination_logits: torch.Tensor, options: torch.Tensor) -> Bernoulli:
        return Bernoulli(validate_args=False, logits=termination_logits.gather(-1, options.long().unsqueeze(-1)).squeeze(-1))
