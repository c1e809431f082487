"""bench.py's timed window has a floor whatever --steps asks: at least
MIN_TIMED_LAUNCHES launches of the line's kernel in the captured graph, replayed until at least
MIN_TIMED_SECONDS are timed.  CPU-only: the sizing functions, and the argument checks of the
closed-loop C5 mode."""
import os
import subprocess
import sys

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_window_steps_floor():
    # the driver's `--steps 20` on 64-step launches: 32 launches, not one
    assert bench.window_steps(20, 64) == 32 * 64
    assert bench.window_steps(2000, 64) == 32 * 64        # 31 whole launches -> the floor
    assert bench.window_steps(5000, 64) == 78 * 64        # above the floor: whole launches
    assert bench.window_steps(20, 1) == 32                # per-step launches
    assert bench.window_steps(3000, 1) == 3000
    assert bench.window_steps(1, 64, min_launches=1) == 64  # at least one launch
    # the bench line's env-steps at B = 65536 are then >= 32 x 64 x 65536
    assert bench.window_steps(20, 64) * bench.window_replays(10.0) * 65536 >= 32 * 64 * 65536


def test_window_replays_reach_min_seconds():
    assert bench.MIN_TIMED_SECONDS >= 0.2 and bench.MIN_TIMED_LAUNCHES >= 32
    for g in (0.0004, 0.013, 0.2, 0.9):
        r = bench.window_replays(g)
        assert r >= 1 and r * g >= min(bench.MIN_TIMED_SECONDS, g * r)
        assert r * g >= bench.MIN_TIMED_SECONDS or r == 1 and g >= bench.MIN_TIMED_SECONDS
        assert (r - 1) * g < bench.MIN_TIMED_SECONDS  # no more replays than needed
    assert bench.window_replays(0.0) >= 1 and bench.window_replays(1e-9) <= 10000


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + list(args),
                          capture_output=True, text=True, timeout=600, env=env)


def test_policy_mode_argument_checks():
    r = _run("--policy", "mlp", "--no-cpu")  # the default config has no features
    assert r.returncode != 0 and "--config c5" in r.stderr
    r = _run("--config", "c5", "--policy", "mlp", "--rollout", "64", "--no-cpu")
    assert r.returncode != 0 and "one launch per step" in r.stderr


def test_bench_line_is_strict_json():
    # a surface the run did not measure (NaN) is null in the printed line, never a bare NaN
    import json

    line = {"a": float("nan"), "b": [1.0, float("inf")], "c": {"d": float("-inf"), "e": 2}, "f": (3.0,)}
    out = json.loads(json.dumps(bench.finite(line), allow_nan=False))
    assert out == {"a": None, "b": [1.0, None], "c": {"d": None, "e": 2}, "f": [3.0]}
