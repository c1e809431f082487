"""The C-ABI without Python: examples/c_api_demo (a C++ host program linked to libwab_hip.so,
no interpreter in the process) builds wab_config with bush_thresholds = NULL, so wab_create
computes the bush table in C (wab_bush_thresholds).  Its run must equal the Python host's
run of the same actions, step for step (the default options' C and numpy tables are equal,
tests/test_capi.py)."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(REPO, "examples", "bin", "c_api_demo")


@pytest.mark.gpu
def test_c_caller_equals_python_host(tmp_path):
    import torch

    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    if not os.path.exists(DEMO):
        pytest.fail("examples/bin/c_api_demo not built (__graft_entry__.build())")
    B, T, seed = 4096, 120, 0x5EED
    out = tmp_path / "demo.bin"
    r = subprocess.run([DEMO, str(B), str(T), str(seed), str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, np.uint8)
    o = 0
    acts = raw[o:o + T * B].view(np.int8).reshape(T, B); o += T * B
    rew = raw[o:o + 4 * T * B].view(np.float32).reshape(T, B); o += 4 * T * B
    done = raw[o:o + T * B].reshape(T, B); o += T * B
    planes = raw[o:o + B * 363].reshape(B, 3, 11, 11); o += B * 363
    scal = raw[o:o + 3 * B].reshape(3, B); o += 3 * B
    assert o == raw.size
    assert done.any() and (acts >= 0).all() and (acts < 5).all()

    env = BatchedWolvesAndBushesEnv(num_envs=B, seed=seed, device="cuda:0")
    env.reset()
    for t in range(T):
        _, rw, dn, _ = env.step(torch.as_tensor(acts[t], device="cuda:0"))
        assert np.array_equal(rw.cpu().numpy().view(np.uint32), rew[t].view(np.uint32)), t
        assert np.array_equal(dn.cpu().numpy().astype(np.uint8), done[t]), t
    assert np.array_equal(env._obs["planes"].cpu().numpy(), planes)
    assert np.array_equal(env._obs["scalars"].cpu().numpy(), scal)


@pytest.mark.gpu
def test_c_torus_caller_equals_python_host(tmp_path):
    """examples/c_api_torus_demo (include/wab_torus.h only): World_tests.py's two known-answer
    tests through the HIP kernel (checked inside the program), then B worlds created and reset
    at caller-chosen positions (wab2_create_at, wab2_reset_at), T wab2_step turns and a T-turn
    wab2_rollout; the Python host given the same positions and actions must see the same records,
    rewards, dones and resets, turn for turn."""
    import torch

    from wab_gym_amd.torus import BatchedWABEnvironment2

    demo = os.path.join(REPO, "examples", "bin", "c_api_torus_demo")
    if not os.path.exists(demo):
        pytest.fail("examples/bin/c_api_torus_demo not built (__graft_entry__.build())")
    B, T, N, R = 256, 32, 25, 96
    out = tmp_path / "torus.bin"
    r = subprocess.run([demo, str(B), str(T), "0x5EED", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("as World_tests.py expects") == 2, r.stdout
    raw = np.fromfile(out, np.uint8)
    o = 0

    def take(n, dt):
        nonlocal o
        a = raw[o:o + n * np.dtype(dt).itemsize].view(dt)
        o += n * np.dtype(dt).itemsize
        return a

    cpos = take(B * N * 2, np.int32).reshape(B, N, 2)
    rpos = take(B * N * 2, np.int32).reshape(B, N, 2)
    acts = take(2 * T * B * N, np.int8).reshape(2 * T, B, N)
    recs = take(2 * T * B * N * R, np.uint8).reshape(2 * T, B, N, R)
    rew = take(2 * T * B * N, np.float32).reshape(2 * T, B, N)
    done = take(2 * T * B * N, np.uint8).reshape(2 * T, B, N)
    wr = take(2 * T * B, np.uint8).reshape(2 * T, B)
    assert o == raw.size
    assert (cpos < 0).any() and (rpos[..., 0] == 32).any() and (rpos < 0).any()

    env = BatchedWABEnvironment2(32, 32, None, 1, 8, 16, num_worlds=B, device="cuda:0", spawn_positions=cpos)
    env.reset_environment(positions=rpos)
    for t in range(T):
        obs, rw, dn, info = env.step(torch.as_tensor(acts[t]))
        assert np.array_equal(obs.cpu().numpy(), recs[t]), t
        assert np.array_equal(rw.cpu().numpy().view(np.uint32), rew[t].view(np.uint32)), t
        assert np.array_equal(dn.cpu().numpy().astype(np.uint8), done[t]), t
        assert np.array_equal(info["world_reset"].cpu().numpy().astype(np.uint8), wr[t]), t
    obs, rw, dn, w = env.rollout(torch.as_tensor(acts[T:]))
    assert np.array_equal(obs.cpu().numpy(), recs[T:])
    assert np.array_equal(rw.cpu().numpy().view(np.uint32), rew[T:].view(np.uint32))
    assert np.array_equal(dn.cpu().numpy(), done[T:]) and np.array_equal(w.cpu().numpy(), wr[T:])
