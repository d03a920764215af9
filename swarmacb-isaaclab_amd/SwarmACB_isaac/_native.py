"""ctypes binding of libswarmstep.so (the C ABI declared in include/swarmstep.h).

The product path has no fallback: if the HIP library is missing or fails to
load, importing the engine raises immediately.
"""

from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SWARMSTEP_LIB", os.path.join(HERE, "libswarmstep.so"))

ABI_VERSION = 2
MAX_AGENTS = 64
MAX_SUBSTEPS = 64

MISSIONS = {"dgt": 0, "xor": 1, "homing": 2, "foraging": 3, "sheltering": 4}
PROFILES = {"isaac": 0, "standalone": 1}


class SwarmParams(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("mission", C.c_int32), ("profile", C.c_int32),
        ("num_envs", C.c_int32), ("num_agents", C.c_int32), ("obs_dim", C.c_int32),
        ("discrete_actions", C.c_int32), ("max_episode_length", C.c_int32), ("decimation", C.c_int32),
        ("layout", C.c_int32), ("env_offset", C.c_int64), ("seed", C.c_uint64),
    ]


class SwarmState(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "pos_x", "pos_y", "yaw", "fsm", "wheel_l", "wheel_r", "sensor_cache", "ground_prev", "flags",
        "episode_length", "episode_reward", "completed_reward", "terminal_critic")]


class SwarmOutputs(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("reward", C.c_void_p), ("truncated", C.c_void_p)]


class SwarmReplay(C.Structure):
    _fields_ = [
        ("rab_uniform", C.c_void_p), ("rab_uniform_dispatch", C.c_void_p), ("turn_steps", C.c_void_p),
        ("spawn_uniform", C.c_void_p), ("spawn_draws", C.c_int32), ("reserved0", C.c_int32),
        ("spawn_yaw_uniform", C.c_void_p),
    ]


# Every symbol include/swarmstep.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = [
    "swarm_abi_version", "swarm_strerror", "swarm_last_hip_error", "swarm_create", "swarm_destroy",
    "swarm_reset", "swarm_step", "swarm_critic_state", "swarm_sync_episode_lengths", "swarm_tick",
    "swarm_last_timeouts", "swarm_set_step_groups", "swarm_step_streams", "swarm_layout",
    "swarm_critic_state_range",
    "swarm_gate_alloc", "swarm_gate_free", "swarm_gate_wait",
    "swarm_fsm_pack",
]

# Every symbol include/swarmrollout.h declares (rollout-buffer kernels, same library).
ROLLOUT_EXPORTS = ["swarm_lambda_returns", "swarm_sequence_chunk_offsets", "swarm_sequence_chunk_fill", "swarm_gather",
                   "swarm_decision_record"]

GATHER_MAX_FIELDS = 48
GATHER_KINDS = {"focal": 0, "group": 1, "focal_first": 2, "group_first": 3}


class GatherField(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("row_words", C.c_int32), ("kind", C.c_int32)]


# Every symbol include/swarmcritic.h declares (fused critic attention, same library).
CRITIC_EXPORTS = ["swarm_rsa_pool", "swarm_rsa_pool_focal", "swarm_rsa_embedding_norm", "swarm_lstm_cell",
                  "swarm_lstm_cell_backward"]
TRAIN_EXPORTS = ["swarm_lstm_seq_forward", "swarm_lstm_seq_backward", "swarm_rsa_attn_forward",
                 "swarm_rsa_attn_backward", "swarm_tensor_list_copy", "swarm_lstm_seq_forward_batch",
                 "swarm_lstm_seq_backward_batch", "swarm_row_norm_forward", "swarm_row_norm_backward",
                 "swarm_set_pool_forward", "swarm_set_pool_backward", "swarm_splitk_colsum",
                 "swarm_splitk_finish", "swarm_ppo_value_loss", "swarm_ppo_value_loss_backward",
                 "swarm_ppo_policy_loss", "swarm_ppo_policy_loss_backward", "swarm_categorical_terms",
                 "swarm_categorical_terms_backward", "swarm_oc2_termination_terms",
                 "swarm_oc2_termination_terms_backward", "swarm_oc2_option_terms", "swarm_oc2_attention_terms",
                 "swarm_oc2_attention_terms_backward", "swarm_oc2_action_terms", "swarm_oc2_action_terms_backward",
                 "swarm_wgrad"]
NORM_WIDTHS = (128, 256)   # row widths of swarm_row_norm_* / swarm_set_pool_*
LSTM_MAX_BATCH = 6     # SWARM_LSTM_MAX_BATCH (include/swarmtrain.h)
OC2_PARTIALS_FLOATS = 2048 * 24   # SWARM_OC2_PARTIALS_FLOATS (include/swarmtrain.h)


class LstmSeqFwd(C.Structure):
    _fields_ = [("n", C.c_int64)] + [(f, C.c_void_p) for f in ("xg", "w_hh", "h0", "c0", "keep", "h_out", "c_out",
                                                                  "act")]


class WgradSrc(C.Structure):
    """swarm_wgrad_src_t (include/swarmtrain.h)."""
    _fields_ = [("in_f", C.c_int32), ("mode", C.c_int32), ("ld", C.c_int64), ("x", C.c_void_p), ("dw", C.c_void_p),
                ("h0", C.c_void_p), ("keep", C.c_void_p), ("T", C.c_int32), ("pad", C.c_int32)]


class LstmSeqBwd(C.Structure):
    _fields_ = [("n", C.c_int64)] + [(f, C.c_void_p) for f in ("w_hh", "c0", "keep", "c_out", "act", "dh_out", "dh_n",
                                                                  "dc_n", "dxg", "dh0", "dc0")]
ATTN_MAX_ENTITIES = 32
ATTN_HEAD_DIMS = (32, 64, 128)
LSTM_SEQ_MAX_UNITS = 64
RSA_SINGLE, RSA_BASELINES, RSA_SINGLE_OF_PAIRS, RSA_ACTIONS_OF_PAIRS, RSA_FOCAL = 0, 1, 2, 3, 4
RSA_MAX_ROWS = 40   # N + alternatives of swarm_rsa_pool_focal

RECORD_MAX_MEMORIES = 12


class MemorySlab(C.Structure):
    _fields_ = [("data", C.c_void_p), ("rows_per_env", C.c_int32), ("width", C.c_int32)]


class DecisionRecord(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("rewards", "dones", "timeouts", "timeout_values", "episode_reward",
                                          "episode_steps", "log_returns", "log_lengths", "log_group_rewards",
                                          "log_count")] + [
        ("log_capacity", C.c_int32), ("n_memories", C.c_int32), ("memories", MemorySlab * RECORD_MAX_MEMORIES),
        ("options", C.c_void_p), ("options_per_env", C.c_int32), ("reserved", C.c_int32)]


_lib = None


def load() -> C.CDLL:
    """Load libswarmstep.so (raises if the HIP extension has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libswarmstep.so not found at {LIB_PATH}; build it with "
            "`make -C swarmacb-isaaclab_amd/csrc` or __graft_entry__.build()")
    lib = C.CDLL(LIB_PATH)
    lib.swarm_abi_version.restype = C.c_int32
    lib.swarm_strerror.restype = C.c_char_p
    lib.swarm_strerror.argtypes = [C.c_int32]
    lib.swarm_last_hip_error.restype = C.c_int32
    lib.swarm_create.restype = C.c_int32
    lib.swarm_create.argtypes = [C.POINTER(SwarmParams), C.POINTER(C.c_void_p)]
    lib.swarm_destroy.restype = C.c_int32
    lib.swarm_destroy.argtypes = [C.c_void_p]
    lib.swarm_reset.restype = C.c_int32
    lib.swarm_reset.argtypes = [C.c_void_p, C.POINTER(SwarmState), C.c_void_p, C.POINTER(SwarmOutputs),
                                C.POINTER(SwarmReplay), C.c_void_p]
    lib.swarm_step.restype = C.c_int32
    lib.swarm_step.argtypes = [C.c_void_p, C.POINTER(SwarmState), C.c_void_p, C.c_void_p,
                               C.POINTER(SwarmOutputs), C.c_int32, C.POINTER(SwarmReplay), C.c_void_p]
    lib.swarm_critic_state.restype = C.c_int32
    lib.swarm_critic_state.argtypes = [C.c_void_p, C.POINTER(SwarmState), C.c_void_p, C.c_void_p]
    lib.swarm_sync_episode_lengths.restype = C.c_int32
    lib.swarm_sync_episode_lengths.argtypes = [C.c_void_p, C.c_void_p]
    lib.swarm_tick.restype = C.c_int64
    lib.swarm_tick.argtypes = [C.c_void_p]
    lib.swarm_last_timeouts.restype = C.c_int64
    lib.swarm_last_timeouts.argtypes = [C.c_void_p]
    lib.swarm_set_step_groups.restype = C.c_int32
    lib.swarm_set_step_groups.argtypes = [C.c_void_p, C.c_int32]
    lib.swarm_step_streams.restype = C.c_int32
    lib.swarm_step_streams.argtypes = [C.c_void_p, C.POINTER(SwarmState), C.c_void_p, C.c_void_p,
                                       C.POINTER(SwarmOutputs), C.c_int32, C.POINTER(SwarmReplay),
                                       C.POINTER(C.c_void_p), C.c_int32]
    lib.swarm_critic_state_range.restype = C.c_int32
    lib.swarm_critic_state_range.argtypes = [C.c_void_p, C.POINTER(SwarmState), C.c_int32, C.c_int32, C.c_void_p,
                                             C.c_void_p]
    lib.swarm_layout.restype = C.c_int32
    lib.swarm_layout.argtypes = [C.c_void_p, C.c_int32]
    lib.swarm_fsm_pack.restype = C.c_uint32
    lib.swarm_fsm_pack.argtypes = [C.c_int32, C.c_int32, C.c_float] * 3
    i32, i64, vp = C.c_int32, C.c_int64, C.c_void_p
    lib.swarm_lambda_returns.restype = i32
    lib.swarm_lambda_returns.argtypes = [i32, i32, i32, C.c_double, C.c_double, vp, vp, vp, vp, vp, vp, i32,
                                         C.POINTER(vp), vp, C.POINTER(vp), vp]
    lib.swarm_sequence_chunk_offsets.restype = i32
    lib.swarm_sequence_chunk_offsets.argtypes = [i32, i32, i32, i32, vp, vp, vp]
    lib.swarm_sequence_chunk_fill.restype = i32
    lib.swarm_sequence_chunk_fill.argtypes = [i32, i32, i32, i32, vp, vp, vp, vp]
    lib.swarm_gather.restype = i32
    lib.swarm_gather.argtypes = [i32, C.POINTER(GatherField), i32, vp, vp, i32, i32, i32, i32, i32, i64, vp, vp, vp]
    lib.swarm_decision_record.restype = i32
    lib.swarm_decision_record.argtypes = [i32, i32, C.c_double, vp, vp, vp, vp, C.POINTER(DecisionRecord), vp]
    lib.swarm_rsa_pool.restype = i32
    lib.swarm_rsa_pool.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]
    lib.swarm_rsa_pool_focal.restype = i32
    lib.swarm_rsa_pool_focal.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]
    lib.swarm_rsa_embedding_norm.restype = i32
    lib.swarm_rsa_embedding_norm.argtypes = [C.c_int64, i32, vp, vp, vp]
    lib.swarm_lstm_cell.restype = i32
    lib.swarm_lstm_cell.argtypes = [C.c_int64, i32, vp, vp, vp, vp, vp]
    lib.swarm_lstm_cell_backward.restype = i32
    lib.swarm_lstm_cell_backward.argtypes = [C.c_int64, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.swarm_lstm_seq_forward.restype = i32
    lib.swarm_lstm_seq_forward.argtypes = [C.c_int64, i32, i32] + [vp] * 9
    lib.swarm_lstm_seq_backward.restype = i32
    lib.swarm_lstm_seq_backward.argtypes = [C.c_int64, i32, i32] + [vp] * 12
    lib.swarm_lstm_seq_forward_batch.restype = i32
    lib.swarm_lstm_seq_forward_batch.argtypes = [i32, i32, i32, vp, vp]
    lib.swarm_lstm_seq_backward_batch.restype = i32
    lib.swarm_lstm_seq_backward_batch.argtypes = [i32, i32, i32, vp, vp]
    lib.swarm_rsa_attn_forward.restype = i32
    lib.swarm_rsa_attn_forward.argtypes = [C.c_int64, i32, i32, i32, vp, vp, vp, vp]
    lib.swarm_rsa_attn_backward.restype = i32
    lib.swarm_rsa_attn_backward.argtypes = [C.c_int64, i32, i32, i32, vp, vp, vp, vp, vp]
    lib.swarm_gate_alloc.restype = i32
    lib.swarm_gate_alloc.argtypes = [vp]
    lib.swarm_gate_free.restype = i32
    lib.swarm_gate_free.argtypes = [vp]
    lib.swarm_gate_wait.restype = i32
    lib.swarm_gate_wait.argtypes = [vp, C.c_int64, vp]
    lib.swarm_tensor_list_copy.restype = i32
    lib.swarm_tensor_list_copy.argtypes = [i32, vp, vp, vp, C.c_int64, vp, vp]
    lib.swarm_row_norm_forward.restype = i32
    lib.swarm_row_norm_forward.argtypes = [i64, i32, vp, vp, vp, vp]
    lib.swarm_row_norm_backward.restype = i32
    lib.swarm_row_norm_backward.argtypes = [i64, i32, vp, vp, vp, vp, vp]
    lib.swarm_set_pool_forward.restype = i32
    lib.swarm_set_pool_forward.argtypes = [i64, i32, i32, vp, vp, vp, vp, vp, vp]
    lib.swarm_set_pool_backward.restype = i32
    lib.swarm_set_pool_backward.argtypes = [i64, i32, i32, vp, vp, vp, vp, vp]
    lib.swarm_splitk_colsum.restype = i32
    lib.swarm_splitk_colsum.argtypes = [i64, i32, i32, vp, vp, vp]
    lib.swarm_splitk_finish.restype = i32
    lib.swarm_splitk_finish.argtypes = [i32, i64, vp, vp, i32, i32, vp, vp, vp]
    lib.swarm_wgrad.restype = i32
    lib.swarm_wgrad.argtypes = [i64, i32, vp, i64, i32, vp, vp, vp]
    f32 = C.c_float
    lib.swarm_ppo_value_loss.restype = i32
    lib.swarm_ppo_value_loss.argtypes = [i64, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp]
    lib.swarm_ppo_value_loss_backward.restype = i32
    lib.swarm_ppo_value_loss_backward.argtypes = [i64, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp]
    lib.swarm_ppo_policy_loss.restype = i32
    lib.swarm_ppo_policy_loss.argtypes = [i64, i32, i32, vp, vp, vp, vp, vp, f32, f32, i32, vp, vp, vp, vp]
    lib.swarm_ppo_policy_loss_backward.restype = i32
    lib.swarm_ppo_policy_loss_backward.argtypes = [i64, i32, i32, vp, vp, vp, vp, vp, f32, f32, i32, vp, vp, vp, vp]
    lib.swarm_categorical_terms.restype = i32
    lib.swarm_categorical_terms.argtypes = [i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.swarm_oc2_termination_terms.restype = i32
    lib.swarm_oc2_termination_terms.argtypes = [i64, vp, vp, vp, vp, C.c_float, C.c_float, vp, vp, vp]
    lib.swarm_oc2_termination_terms_backward.restype = i32
    lib.swarm_oc2_termination_terms_backward.argtypes = [i64, vp, vp, vp, vp, C.c_float, C.c_float, vp, vp, vp]
    lib.swarm_oc2_option_terms.restype = i32
    lib.swarm_oc2_option_terms.argtypes = [i64, i32, vp, vp, vp, vp, vp, C.c_float, C.c_float, C.c_float, vp, vp, vp,
                                           vp]
    lib.swarm_oc2_action_terms.restype = i32
    lib.swarm_oc2_action_terms.argtypes = [i64, i32, i32] + [vp] * 13
    lib.swarm_oc2_action_terms_backward.restype = i32
    lib.swarm_oc2_action_terms_backward.argtypes = [i64, i32, i32] + [vp] * 10
    lib.swarm_oc2_attention_terms.restype = i32
    lib.swarm_oc2_attention_terms.argtypes = [i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.swarm_oc2_attention_terms_backward.restype = i32
    lib.swarm_oc2_attention_terms_backward.argtypes = [i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]
    lib.swarm_categorical_terms_backward.restype = i32
    lib.swarm_categorical_terms_backward.argtypes = [i64, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    if lib.swarm_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libswarmstep ABI {lib.swarm_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        lib = load()
        msg = lib.swarm_strerror(rc).decode()
        raise RuntimeError(f"{what} failed: {msg} (status {rc}, hip error {lib.swarm_last_hip_error()})")
