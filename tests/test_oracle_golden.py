"""The C oracle (oracle/wab_oracle.c) reproduces the reference's golden vectors bit for bit.

The fixtures were produced by the unmodified reference (wab_env.py) under the keyed RNG
(tests/golden/make_golden.py); this pins the oracle before it is used as the checker.
"""
import pytest

import golden_replay as gr
from backends import OracleBackend


@pytest.mark.parametrize("name", gr.SETS)
def test_oracle_matches_reference_golden(name):
    steps = gr.replay(name, OracleBackend)
    assert steps > 0


def test_oracle_padded_stride_matches_golden():
    # C3 layout: 31x31 viewport stored in 32-byte rows (padding must be zero)
    assert gr.replay("wide31", OracleBackend, plane_stride=32, max_steps=40) > 0


def test_golden_sets_cover_the_dynamics():
    """The fixtures exercise every branch of step(): eat, kill, starve, finish, resets."""
    import numpy as np

    seen = {"killed": 0, "starved": 0, "finished": 0, "ate": 0, "multi_wolf": 0}
    for name in gr.SETS:
        g = gr.load(name)
        st = g["scalars"][..., 2]
        done = g["done"]
        seen["killed"] += int(((st == 2) & done).sum())
        seen["starved"] += int(((st == 1) & done).sum())
        seen["finished"] += int(((st == 0) & done).sum())
        eat = g["meta"]["options"]["reward_for_eating"]
        r = g["reward"]
        seen["ate"] += int((np.isclose(r, eat) | np.isclose(r, eat - 1) | np.isclose(r, eat + 1)).sum())
        seen["multi_wolf"] += int((g["n_wolves"] >= 2).sum())
    assert all(v > 0 for v in seen.values()), seen


class _OracleRollout(OracleBackend):
    """A multi-step oracle backend for gr.replay_rollout (the harness the GPU rollout replay
    uses), stepping the oracle once per row of the segment."""

    def rollout(self, actions):
        import numpy as np

        out = [self.step(a)[:6] for a in actions]
        return tuple(np.stack([o[k] for o in out]) for k in range(6))


@pytest.mark.parametrize("name", ["default", "continue", "wolfy"])
def test_rollout_replay_harness_on_oracle(name):
    assert gr.replay_rollout(name, _OracleRollout) > 0
