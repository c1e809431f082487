"""Host logic of BatchedWolvesAndBushesEnv that needs no device: how the device counters turn
into exceptions (hand-off timeouts must not pass silently; deferred action errors
must carry the data the raising call read)."""
import pytest

from wab_gym_amd import _lib
from wab_gym_amd.env import BatchedWolvesAndBushesEnv


def _host_env(validate):
    env = object.__new__(BatchedWolvesAndBushesEnv)  # no handle: only the counter logic
    env.validate_actions = "sync" if validate is True else validate
    env._bad_seen = env._handoff_seen = 0
    env.n_actions = 5
    return env


def _c(bad=0, hand=0):
    return {"wolf_overflow": 0, "eaten_overflow": 0, "bad_actions": bad, "steps": 0, "resets": 0,
            "ego_missing": 0, "handoff_timeouts": hand}


def test_handoff_timeout_raises_once_with_result():
    env = _host_env(False)  # even with action validation off
    env._raise_pending(_c(), "r0")
    with pytest.raises(_lib.WabError) as ei:
        env._raise_pending(_c(hand=3), "r1")
    assert ei.value.result == "r1" and "3 LDS hand-off" in str(ei.value)
    env._raise_pending(_c(hand=3), "r2")  # reported once
    with pytest.raises(_lib.WabError):
        env._raise_pending(_c(hand=4), "r3")


def test_deferred_bad_actions_raise_once():
    env = _host_env("deferred")
    with pytest.raises(IndexError) as ei:
        env._raise_pending(_c(bad=128), {"x": 1})
    assert ei.value.result == {"x": 1}
    env._raise_pending(_c(bad=128), None)
    off = _host_env(False)
    off._raise_pending(_c(bad=128), None)  # validation off: counted, never raised

