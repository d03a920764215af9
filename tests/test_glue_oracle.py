"""Decision-loop glue oracle (oracle/rollout_oracle.DecisionGlue) against the
reference's own collect_rollout (tests/golden/rollout/decision_glue.npz, made by
make_glue_golden.py from poca_trainer.py:441-649 with a scripted env). CPU, bit-exact."""

import os

import numpy as np

from oracle import rollout_oracle as RO

GLUE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rollout", "decision_glue.npz")


def test_glue_oracle_matches_reference():
    g = np.load(GLUE)
    E, N, dp, R = (int(v) for v in g["meta"])
    glue = RO.DecisionGlue(E)
    for d in range(R):
        row = glue.record(g["reward_sum"][d], g["truncated"][d], g["group_reward"][d], g["timeout_value_raw"][d],
                          dp, float(g["reward_strength"]))
        for k, v in row.items():
            np.testing.assert_array_equal(v, g[f"out_{k}"][d], err_msg=f"decision {d} {k}")
    np.testing.assert_array_equal(np.asarray(glue.returns, np.float32), g["out_completed_returns"])
    np.testing.assert_array_equal(np.asarray(glue.lengths, np.float32), g["out_completed_lengths"])
    np.testing.assert_array_equal(np.asarray(glue.group, np.float32), g["out_completed_group_rewards"])
    np.testing.assert_array_equal(glue.acc, g["out_episode_reward_acc"])
    np.testing.assert_array_equal(glue.steps, g["out_episode_step_count"])
