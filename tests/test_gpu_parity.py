"""GPU parity: the HIP product path (C-ABI via ctypes) against the reference's golden vectors
and against the pinned C oracle, bit for bit (integer/byte outputs; reward as f32 of the
reference's double; the hidden food double compared by its bit pattern)."""
import numpy as np
import pytest

import golden_replay as gr
from backends import SEED, GpuBackend

pytestmark = pytest.mark.gpu


def _env(opts=None, n=4096, base=0, **kw):
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    return BatchedWolvesAndBushesEnv(opts, num_envs=n, seed=SEED, device="cuda:0", env_id_base=base, **kw)


def _device_counters(env):
    """env.counters() without the host-side launch tallies (which differ by design between a
    rollout handle and a step-loop handle)."""
    return {k: v for k, v in env.counters().items() if k not in ("rollout_launches", "rollout_step_calls")}


def _oracle(opts=None, n=4096, base=0, autoreset=True, stride=0):
    from oracle.oracle import OracleBatch

    return OracleBatch(opts, n, SEED, base, autoreset, stride)


# ------------------------------------------------------------------ golden vectors
@pytest.mark.parametrize("name", gr.SETS)
def test_gpu_matches_reference_golden(name):
    assert gr.replay(name, GpuBackend) > 0


@pytest.mark.parametrize("name", gr.SETS)
def test_gpu_rollout_matches_reference_golden(name):
    """Every golden set through env.rollout (wab_rollout: the multi-step launches bench.py
    times), in consecutive rollouts of 1, 7 and 64 steps with the state carried across them.
    Each group is padded to a multiple of 16 envs so that its plane slices are 16-byte aligned:
    the backend asserts that every rollout ran as the ONE launch bench.py times."""
    from backends import GpuPaddedRolloutBackend

    assert gr.replay_rollout(name, GpuPaddedRolloutBackend) > 0


def test_gpu_rollout_golden_misaligned_falls_back_per_step():
    """The golden groups as they are (40 and 1 envs of 363-byte planes: misaligned step slices)
    take wab_rollout's per-step path through the handle's scratch planes; same results."""
    from backends import GpuRolloutBackend

    seen = []

    class Tally(GpuRolloutBackend):
        def rollout(self, actions):
            before = self.env.counters()
            out = super().rollout(actions)
            c = self.env.counters()
            seen.append((c["rollout_launches"] - before["rollout_launches"],
                         c["rollout_step_calls"] - before["rollout_step_calls"]))
            return out

    assert gr.replay_rollout("default", Tally) > 0
    assert seen and all(x == (0, 1) for x in seen), seen


def test_gpu_rollout_golden_wide_kernel_and_8_slots():
    """The wide kernel's rollout build (31x31 in 32-byte rows, C3's layout) and the small one
    with 8 wolf rows (the headline's handle) on the golden sets."""
    from backends import GpuRolloutBackend

    class Slots8(GpuRolloutBackend):
        wolf_slots = 8

    assert gr.replay_rollout("wide31", GpuRolloutBackend, plane_stride=32) > 0
    assert gr.replay_rollout("wolfy", GpuRolloutBackend, plane_stride=16, segments=(64, 5)) > 0  # 16-byte rows: wide kernel
    assert gr.replay_rollout("default", Slots8) > 0


def test_gpu_golden_8_slots_and_padded_stride():
    class Slots8(GpuBackend):
        wolf_slots = 8

    assert gr.replay("default", Slots8) > 0
    assert gr.replay("wide31", Slots8, plane_stride=32) > 0


# ------------------------------------------------------------------ lockstep vs oracle
def _lockstep(opts, n, T, autoreset=True, stride=0, threads=16, seed_actions=0, base=0,
              check_terminal=True, wolf_slots=0, return_terminal=True):
    """The HIP step against the oracle, bit for bit, every step.  return_terminal=False runs
    the kernels' default auto-reset path (the one bench.py, rollout and step_features use:
    in the small kernel W3 builds the new episodes after W1's hand-off) instead of the
    terminal-obs path (W0 builds them after one more barrier)."""
    import torch

    env = _env(opts, n, base, autoreset=autoreset, return_terminal=return_terminal, plane_stride=stride,
               wolf_slots=wolf_slots)
    orc = _oracle(opts, n, base, autoreset, stride)
    obs = env.reset()
    op, of, orl, ost = orc.reset()
    assert np.array_equal(env._obs["planes"].cpu().numpy(), op)
    assert np.array_equal(obs[3].cpu().numpy(), of)
    rng = np.random.RandomState(seed_actions)
    for t in range(T):
        a = rng.randint(env.n_actions, size=n)
        obs, rew, done, info = env.step(torch.as_tensor(a))
        op, of, orl, ost, orew, odone = orc.step(a, nthreads=threads)
        d = odone.astype(bool)
        assert np.array_equal(done.cpu().numpy(), d), t
        assert np.array_equal(rew.cpu().numpy(), orew), t
        assert np.array_equal(obs[3].cpu().numpy(), of), t
        assert np.array_equal(obs[4].cpu().numpy(), orl), t
        assert np.array_equal(obs[5].cpu().numpy(), ost), t
        gp = env._obs["planes"].cpu().numpy()
        if not np.array_equal(gp, op):
            bad = np.nonzero((gp != op).reshape(n, -1).any(1))[0]
            raise AssertionError("planes differ at t=%d envs %s" % (t, bad[:10]))
        if autoreset and check_terminal and return_terminal and d.any():
            tp = env._term["planes"].cpu().numpy()
            assert np.array_equal(tp[d], orc.t_planes[d]), t
            ts = env._term["scalars"].cpu().numpy()
            assert np.array_equal(ts[0][d], orc.t_food_turns[d]), t
            assert np.array_equal(ts[2][d], orc.t_status[d]), t
    gs, os_ = env.state(), orc.state()
    for k in ("x", "y", "turn", "n_wolves", "episode"):
        assert np.array_equal(gs[k], os_[k]), k
    assert np.array_equal(gs["food"].view(np.uint64), os_["food"].view(np.uint64))
    c = env.counters()
    assert c["wolf_overflow"] == 0 and c["eaten_overflow"] == 0 and c["bad_actions"] == 0
    assert c["handoff_timeouts"] == 0 and c["steps"] == n * T
    return env, orc


def test_c2_batch4096_default_lockstep():
    env, _ = _lockstep(None, 4096, 160)
    assert env.counters()["resets"] > 4096  # every env finished at least one episode


@pytest.mark.parametrize("return_terminal", [False, True])
def test_c3_batch65536_wide31_padded_lockstep(return_terminal):
    """C3 at full size as the bench runs it (8 wolves per env in registers, 32 wolf rows: the
    rare 9th+ in HBM), past the turn-40 starvation (the first mass auto-reset) to
    desynchronised second episodes."""
    _lockstep({"width": 31, "height": 31}, 65536, 100, stride=32, wolf_slots=32,
              return_terminal=return_terminal, seed_actions=3)


@pytest.mark.parametrize("opts,stride,slots,autoreset", [
    ({"width": 31, "height": 31}, 32, 16, True),
    ({"width": 31, "height": 31, "chance_wolf_on_square": 0.01, "wolf_chance_to_despawn": 0.2,
      "wolf_spawn_margin": 2}, 32, 32, True),
    ({"width": 17, "height": 13, "lookout_only": False}, 16, 8, True),
    ({"width": 25, "height": 29, "starting_food": None, "starting_role": None}, 32, 16, True),
    ({"width": 31, "height": 15, "wolves_can_move": False, "god_mode": True}, 16, 8, True),
    ({"width": 13, "height": 11, "turns_to_fill_food": 4, "max_turns": 60, "bush_power": 60}, 16, 8, True),
    ({"width": 31, "height": 31}, 32, 16, False),
])
@pytest.mark.parametrize("return_terminal", [True, False])
def test_wide_kernel_lockstep(opts, stride, slots, autoreset, return_terminal):
    """The wide-view kernel (width <= 31, height <= 32, rows of 16 or 32 bytes) against the oracle."""
    env, _ = _lockstep(opts, 1000, 120, autoreset=autoreset, stride=stride, wolf_slots=slots, base=5,
                       return_terminal=return_terminal)
    assert env.step_kernel == "wide"


@pytest.mark.parametrize("width,height,kernel", [(31, 31, "wide"), (33, 31, "block"), (31, 33, "block")])
def test_wide_kernel_width_limit(width, height, kernel):
    """The wide kernel takes width <= 31 and height <= 32 (wab_capi.hip wide_view; sizes are
    odd, wab_env.py:147-148, so 31 is the largest): 33 either way in 32- or 48-byte rows steps
    on the block kernel, still equal to the oracle."""
    env, _ = _lockstep({"width": width, "height": height}, 200, 40, stride=32 if height <= 32 else 48,
                       wolf_slots=16)
    assert env.step_kernel == kernel


def test_wide_kernel_reset_mask():
    import torch

    opts = {"width": 31, "height": 31}
    env = _env(opts, 300, plane_stride=32, wolf_slots=16)
    orc = _oracle(opts, 300, stride=32)
    env.reset()
    orc.reset()
    rng = np.random.RandomState(9)
    for t in range(30):
        a = rng.randint(5, size=300)
        env.step(torch.as_tensor(a))
        orc.step(a)
        if t % 10 == 9:
            mask = (rng.random_sample(300) < 0.3).astype(np.uint8)
            env.reset(torch.as_tensor(mask))
            orc.reset(mask)
        assert np.array_equal(env._obs["planes"].cpu().numpy(), orc.planes), t
    assert np.array_equal(env.state()["episode"], orc.state()["episode"])


@pytest.mark.parametrize("return_terminal", [False, True])
def test_headline_batch65536_default_lockstep(return_terminal):
    """The headline configuration at full size for 200 steps (> 2 x max_turns): the turn-40
    mass starvation, the turn-80 cap and the desynchronised later episodes, on both auto-reset
    paths of the small kernel (return_terminal=False is the bench's)."""
    env, _ = _lockstep(None, 65536, 200, return_terminal=return_terminal, seed_actions=11)
    assert env.step_kernel == "small"
    assert env.counters()["resets"] > 3 * 65536


def test_c4_eight_shards_of_65536_match_oracle():
    """C4 (BASELINE configs[3]) on one GPU: eight 65536-env handles with env_id_base =
    r * 65536, stepped in turn, against the oracle over all 524288 global env ids, bit for bit,
    for 100 steps; zero overflow on every shard.  (On 8 GPUs each rank runs exactly one of
    these handles: bench.py's shards.)"""
    import torch

    R, B, T = 8, 65536, 100
    shards = [_env(None, B, r * B, validate_actions=False) for r in range(R)]
    orc = _oracle(None, R * B)
    op, of, _, _ = orc.reset()
    for r, e in enumerate(shards):
        e.reset()
        assert np.array_equal(e._obs["planes"].cpu().numpy(), op[r * B:(r + 1) * B]), r
    rng = np.random.RandomState(2024)
    for t in range(T):
        a = rng.randint(5, size=R * B).astype(np.int8)
        ad = torch.as_tensor(a, device="cuda:0")
        for r, e in enumerate(shards):
            e.step(ad[r * B:(r + 1) * B])
        op, of, orl, ost, orew, odone = orc.step(a, nthreads=16)
        for r, e in enumerate(shards):
            sl = slice(r * B, (r + 1) * B)
            assert np.array_equal(e._obs["planes"].cpu().numpy(), op[sl]), (t, r)
            assert np.array_equal(e._obs["scalars"].cpu().numpy(), np.stack([of[sl], orl[sl], ost[sl]])), (t, r)
            assert np.array_equal(e.reward.cpu().numpy(), orew[sl]), (t, r)
            assert np.array_equal(e.done.cpu().numpy(), odone[sl]), (t, r)
    os_ = orc.state()
    for r, e in enumerate(shards):
        gs = e.state()
        sl = slice(r * B, (r + 1) * B)
        for k in ("x", "y", "turn", "n_wolves", "episode"):
            assert np.array_equal(gs[k], os_[k][sl]), (r, k)
        assert np.array_equal(gs["food"].view(np.uint64), os_["food"][sl].view(np.uint64)), r
        c = e.counters()
        assert c["wolf_overflow"] == 0 and c["eaten_overflow"] == 0 and c["handoff_timeouts"] == 0, (r, c)
        assert c["steps"] == B * T


def test_no_autoreset_keeps_stepping_like_reference():
    _lockstep(None, 2048, 140, autoreset=False)


@pytest.mark.parametrize("return_terminal", [True, False])
def test_option_variants_lockstep(return_terminal):
    for opts in ({"lookout_only": False}, {"restrict_view": True, "lookout_only": False},
                 {"wolves": False}, {"wolves_can_move": False, "god_mode": True},
                 {"starting_food": None, "starting_role": None}, {"width": 9, "height": 13},
                 {"width": 1, "height": 3}, {"width": 45, "height": 45}, {"wolf_spawn_margin": 2},
                 {"width": 9, "height": 9}):
        _lockstep(opts, 640, 90, base=77, wolf_slots=32,  # 45x45 exceeds 8 live wolves
                  return_terminal=return_terminal)


@pytest.mark.parametrize("return_terminal", [True, False])
def test_partial_batch_and_large_env_ids(return_terminal):
    _lockstep(None, 1000, 60, base=2**40 + 5, return_terminal=return_terminal)  # 15 full blocks + a 40-env tail


# ------------------------------------------------------------------ surface behaviour
def test_reset_mask_only_touches_masked_envs():
    import torch

    env = _env(None, 256)
    orc = _oracle(None, 256)
    env.reset()
    orc.reset()
    a = np.random.RandomState(3).randint(5, size=256)
    env.step(torch.as_tensor(a))
    orc.step(a)
    mask = np.zeros(256, np.uint8)
    mask[::3] = 1
    env.reset(torch.as_tensor(mask))
    op, of, _, _ = orc.reset(mask)
    assert np.array_equal(env._obs["planes"].cpu().numpy(), op)
    assert np.array_equal(env._obs["scalars"][0].cpu().numpy(), of)
    assert np.array_equal(env.state()["episode"], orc.state()["episode"])


def test_bad_action_raises_and_counts():
    """validate_actions=True (the default, "sync"): an out-of-range action raises IndexError
    from step() itself, host or device.  "deferred": step() does not synchronise; the kernel
    applies the actions as no-ops and counts them, and the next synchronising call (counters,
    state, check, reset) raises once, with what it read attached as err.result."""
    import torch

    env = _env(None, 128)
    env.reset()
    with pytest.raises(IndexError):
        env.step(torch.full((128,), 5, device="cuda:0"))   # device actions: immediate
    with pytest.raises(IndexError):
        env.step(np.full(128, 5))                          # host actions: before the copy
    with pytest.raises(IndexError):
        env.rollout(torch.full((2, 128), 5, device="cuda:0"))
    env.validate_actions = "deferred"
    env.step(torch.full((128,), 5, device="cuda:0"))  # asynchronous
    with pytest.raises(IndexError) as ei:
        env.counters()
    assert ei.value.result["bad_actions"] == 128
    env.check()  # reported once
    env.step(torch.full((128,), 2, device="cuda:0"))
    env.step(torch.full((128,), -3, device="cuda:0", dtype=torch.int8))
    with pytest.raises(IndexError) as ei:
        env.state()
    assert ei.value.result["turn"].shape == (128,)
    env.step(torch.full((128,), 7, device="cuda:0"))
    with pytest.raises(IndexError):
        env.reset()
    env.reset()
    env.validate_actions = False
    env.step(torch.full((128,), -1))
    env.step(torch.full((128,), 261))  # int64 261 must not narrow to the valid action 5
    env.step(np.full(128, 256))        # nor 256 to 0
    c = env.counters()
    assert c["bad_actions"] == 128 * 6
    assert c["steps"] == 128 * 7 and c["handoff_timeouts"] == 0


def test_input_shape_checks():
    import torch

    from wab_gym_amd.wrappers import PragmaticObsWrapper

    env = _env(None, 256, validate_actions=False)
    env.reset()
    with pytest.raises(ValueError):
        env.rollout(torch.zeros((4, 255), dtype=torch.int8, device="cuda:0"))
    w = PragmaticObsWrapper(env)
    with pytest.raises(ValueError):
        env.step_features(torch.zeros(256, dtype=torch.int8, device="cuda:0"),
                          torch.zeros((255, w.feature_dim), device="cuda:0"))
    with pytest.raises(ValueError):
        w.observation(out=torch.zeros((256, w.feature_dim), dtype=torch.float64, device="cuda:0"))


def test_shard_invariance():
    """Two shards [0, B/2) + [B/2, B) produce exactly what one handle over [0, B) does."""
    import torch

    B, T = 8192, 50
    one = _env(None, B)
    lo, hi = _env(None, B // 2, 0), _env(None, B // 2, B // 2)
    for e in (one, lo, hi):
        e.reset()
    rng = np.random.RandomState(9)
    for _ in range(T):
        a = torch.as_tensor(rng.randint(5, size=B))
        one.step(a)
        lo.step(a[: B // 2])
        hi.step(a[B // 2:])
        both = torch.cat([lo._obs["planes"], hi._obs["planes"]])
        assert torch.equal(one._obs["planes"], both)
        assert torch.equal(one.reward, torch.cat([lo.reward, hi.reward]))


def test_rollout_equals_step_loop():
    import torch

    B, T = 2048, 30
    a = torch.as_tensor(np.random.RandomState(4).randint(5, size=(T, B)))
    e1, e2 = _env(None, B), _env(None, B)
    e1.reset()
    e2.reset()
    planes, scal, rew, done = e1.rollout(a)
    for t in range(T):
        obs, r, d, _ = e2.step(a[t])
        assert torch.equal(planes[t], e2._obs["planes"])
        assert torch.equal(rew[t], r) and torch.equal(done[t].bool(), d)
        assert torch.equal(scal[t], e2._obs["scalars"])


@pytest.mark.parametrize("opts,kw", [
    (None, {}),
    ({"width": 9, "height": 9}, {"wolf_slots": 32}),                 # runtime geometry (G = 0)
    ({"restrict_view": True, "lookout_only": False}, {"wolf_slots": 16}),
    (None, {"autoreset": False}),
    ({"starting_food": None, "starting_role": None}, {}),
    # berries on every tile, two per bush: the ostrich eats nearly every turn and empties tiles
    # (long eaten logs: entries >= 4 in HBM; emptied tiles scrolling back into view)
    ({"bush_power": 1, "max_berries_per_bush": 2, "max_turns": 120}, {"eaten_capacity": 40}),
    ({"bush_power": 1, "max_berries_per_bush": 3}, {"eaten_capacity": 3}),  # log overflow
])
def test_rollout_variants_equal_step_loop(opts, kw):
    """wab_rollout == T wab_step calls, bit for bit, over two consecutive rollouts (state carried
    across calls), a partial last group included; final hidden state and counters equal too."""
    import torch

    B, T = 1008, 60  # 15 full groups + 48 envs; B * 363 obs bytes keeps every step 16-byte aligned
    rs = np.random.RandomState(9)
    e1, e2 = _env(opts, B, validate_actions=False, **kw), _env(opts, B, validate_actions=False, **kw)
    assert e1.step_kernel == "small"
    e1.reset()
    e2.reset()
    for seg in range(2):
        a = torch.as_tensor(rs.randint(e1.n_actions, size=(T, B)))
        planes, scal, rew, done = e1.rollout(a)
        for t in range(T):
            obs, r, d, _ = e2.step(a[t])
            assert torch.equal(planes[t], e2._obs["planes"]), (seg, t)
            assert torch.equal(scal[t], e2._obs["scalars"]), (seg, t)
            assert torch.equal(rew[t], r) and torch.equal(done[t].bool(), d), (seg, t)
    s1, s2 = e1.state(), e2.state()
    for k in s1:
        assert np.array_equal(np.asarray(s1[k]), np.asarray(s2[k])), k
    assert _device_counters(e1) == _device_counters(e2)


def test_full_size_properties():
    """B = 65536 over 200 steps: invariants that hold regardless of the trajectory."""
    import torch

    env = _env(None, 65536, validate_actions=False)
    obs = env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    total_done = 0
    for _ in range(200):
        a = torch.randint(0, 5, (65536,), device="cuda:0", generator=g)
        obs, rew, done, _ = env.step(a)
        assert bool((obs[2][:, 5, 5] == 1).all())            # the ostrich is always centred
        assert int(obs[2].sum()) == 65536                      # ... and alone on its grid
        assert int(obs[3].max()) <= 40
        assert bool(((obs[0] <= 1) & (obs[1] <= 1)).all())
        total_done += int(done.sum())
    c = env.counters()
    assert c["resets"] == total_done + 65536  # + the initial reset of every env
    assert c["wolf_overflow"] == 0 and c["eaten_overflow"] == 0
    # mean episode length of a random policy ~41 steps
    assert 30 < 65536 * 200 / max(total_done, 1) < 55


# ------------------------------------------------------------------ config 5 (actor_critic.py)
def test_featurizer_matches_reference_golden():
    """Device PragmaticObsWrapper + flatten == reference wrapper on 1503 grids (incl. KATs)."""
    import torch

    from wab_gym_amd.wrappers import PragmaticObsWrapper

    z = np.load(gr.GOLDEN_DIR + "/pragmatic.npz")
    n = len(z["features"])
    env = _env(None, n)
    wrap = PragmaticObsWrapper(env)
    assert wrap.feature_dim == int(z["flatdim"]) == 449
    planes = torch.as_tensor(z["planes"]).cuda()
    scal = torch.as_tensor(np.ascontiguousarray(z["scalars"].T)).cuda()
    f = wrap.observation({"planes": planes, "scalars": scal}, view_mask=torch.as_tensor(z["view_mask"]))
    assert np.array_equal(f.cpu().numpy(), z["features"])


def test_featurizer_small_kernel_golden_subsets():
    """Views of <= 128 cells without a caller-given mask use wab_featurize_small_kernel: the
    golden grids whose mask is all zero (no restrict_view) or the role's restrict_view mask."""
    import torch

    from wab_gym_amd.options import view_masks
    from wab_gym_amd.wrappers import PragmaticObsWrapper

    z = np.load(gr.GOLDEN_DIR + "/pragmatic.npz")
    vm, sc = z["view_mask"], z["scalars"]
    for opts in (None, {"restrict_view": True, "lookout_only": False}):
        if opts is None:
            sel = np.nonzero(vm.reshape(len(vm), -1).sum(1) == 0)[0]
        else:
            table = view_masks(dict(opts))
            sel = np.nonzero([np.array_equal(vm[i], table[sc[i, 1]]) for i in range(len(vm))])[0]
        assert len(sel) > 400
        env = _env(opts, len(sel))
        wrap = PragmaticObsWrapper(env)
        planes = torch.as_tensor(z["planes"][sel]).cuda()
        scal = torch.as_tensor(np.ascontiguousarray(sc[sel].T)).cuda()
        f = wrap.observation({"planes": planes, "scalars": scal})
        assert np.array_equal(f.cpu().numpy(), z["features"][sel])


@pytest.mark.parametrize("wh", [(11, 11), (9, 9), (7, 13), (13, 9), (5, 5)])
def test_featurizer_small_kernel_random_planes(wh):
    """Random planes at densities from sparse to full (ties at every distance) against the
    oracle, for both wrappers, including a partial last block."""
    import torch

    from oracle import oracle as orc
    from wab_gym_amd.wrappers import PragmaticObsWrapper, SuperBasicObservationWrapper

    W, H = wh
    n = 64 * 37 + 23
    rng = np.random.default_rng(W * 100 + H)
    dens = rng.choice([0.0, 0.01, 0.05, 0.2, 0.5, 0.9, 1.0], size=(n, 1, 1, 1))
    planes = (rng.random((n, 3, W, H)) < dens).astype(np.uint8)
    sc = np.stack([rng.integers(0, 41, n), rng.integers(0, 2, n), rng.integers(0, 3, n)]).astype(np.uint8)
    env = _env({"width": W, "height": H}, n)
    obs = {"planes": torch.as_tensor(planes).cuda(), "scalars": torch.as_tensor(sc).cuda()}
    f = PragmaticObsWrapper(env).observation(obs)
    want = orc.featurize(planes, sc[0], sc[1], sc[2], np.zeros((n, 11, 11), np.uint8), W, H)
    assert np.array_equal(f.cpu().numpy(), want)
    f = SuperBasicObservationWrapper(env).observation(obs)
    assert np.array_equal(f.cpu().numpy(), orc.featurize_superbasic(planes, sc[0], sc[1], sc[2], W, H))


def test_featurizer_on_env_obs_matches_oracle():
    import torch

    from oracle import oracle as orc
    from wab_gym_amd.options import view_masks
    from wab_gym_amd.wrappers import PragmaticObsWrapper

    for opts in (None, {"restrict_view": True, "lookout_only": False}, {"width": 31, "height": 31}):
        env = _env(opts, 3000, validate_actions=False)
        wrap = PragmaticObsWrapper(env)
        wrap.reset()
        g = torch.Generator(device="cuda:0")
        g.manual_seed(1)
        vm_table = view_masks(env.game_options)
        for _ in range(30):
            f, r, d, _ = wrap.step(torch.randint(0, env.n_actions, (3000,), device="cuda:0", generator=g))
            planes = env._obs["planes"].cpu().numpy()
            sc = env._obs["scalars"].cpu().numpy()
            want = orc.featurize(planes, sc[0], sc[1], sc[2], vm_table[sc[1]], env.W, env.H,
                                 env.game_options["turns_to_empty_food"])
            assert np.array_equal(f.cpu().numpy(), want)


@pytest.mark.parametrize("opts,kw", [
    (None, {}),                                                   # 11x11: G = 11 kernel, 8 slots
    (None, {"wolf_slots": 32, "autoreset": False}),               # stepping past done
    ({"restrict_view": True, "lookout_only": False}, {"wolf_slots": 16}),
    ({"width": 9, "height": 9, "starting_food": None, "starting_role": None}, {}),  # G = 0
    ({"wolf_spawn_margin": 2}, {}),                               # 104-tile ring, G = 0
    ({"width": 9, "height": 13}, {}),                             # not fusable: step + featurize
    ({"width": 31, "height": 31}, {"plane_stride": 32}),          # wide kernel: step + featurize
])
def test_step_features_matches_step_then_featurize(opts, kw):
    """wab_step_features (one kernel where the small kernel steps the handle, obs planes not
    stored) == wab_step followed by wab_featurize, bit for bit, over 100 steps of a batch with a
    partial last group; reward, done and the obs scalars too."""
    import torch

    from wab_gym_amd.wrappers import PragmaticObsWrapper

    n = 1000
    ea = _env(opts, n, validate_actions=False, **kw)
    eb = _env(opts, n, validate_actions=False, **kw)
    wa, wb = PragmaticObsWrapper(ea), PragmaticObsWrapper(eb)
    fa = torch.full((n, wa.feature_dim), 7.0, device="cuda:0")
    assert torch.equal(wa.reset(), wb.reset())
    g = torch.Generator(device="cuda:0")
    g.manual_seed(3)
    for t in range(100):
        a = torch.randint(0, ea.n_actions, (n,), device="cuda:0", generator=g)
        f, ra, da = ea.step_features(a, fa, store_planes=False)
        _, rb, db, _ = eb.step(a)
        fb = wb.observation()
        assert torch.equal(f, fb), t
        assert torch.equal(ra, rb) and torch.equal(da, db), t
        assert torch.equal(ea._obs["scalars"], eb._obs["scalars"]), t
    ca, cb = ea.counters(), eb.counters()
    assert ca == cb


def test_step_features_full_size_c5():
    """C5 at its full size (B = 65536): the fused launch (planes not stored) == wab_step +
    wab_featurize on a twin env for 40 steps; every row one-hot per group (each Discrete block
    of the flattened 11-tuple holds exactly one 1)."""
    import torch

    from wab_gym_amd.wrappers import PragmaticObsWrapper

    B = 65536
    ea, eb = _env(None, B, validate_actions=False), _env(None, B, validate_actions=False)
    wa, wb = PragmaticObsWrapper(ea), PragmaticObsWrapper(eb)
    wa.reset()
    wb.reset()
    fa = torch.empty((B, wa.feature_dim), device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    md = 11
    sizes = [md + 1] * 8 + [11] * 4 + [md + 1] * 8 + [11] * 4 + [2, 41, 2, 3]
    for t in range(40):
        a = torch.randint(0, 5, (B,), device="cuda:0", generator=g)
        ea.step_features(a, fa, store_planes=False)
        eb.step(a)
        assert torch.equal(fa, wb.observation()), t
    o = 0
    for n in sizes:  # the last step's rows
        assert bool((fa[:, o:o + n].sum(1) == 1).all()), o
        o += n
    assert bool((fa[:, o:] == 0).all())  # view mask: zeros without restrict_view
    assert _device_counters(ea) == _device_counters(eb)


def test_step_features_argument_errors():
    import ctypes

    import torch

    from wab_gym_amd import _lib

    env = _env(None, 256)
    env.reset()
    L = _lib.load()
    F = int(L.wab_feature_dim(env._h))
    feats = torch.zeros(256 * F + 8, device="cuda:0")
    a = torch.zeros(256, dtype=torch.int8, device="cuda:0")
    o = env._obs["struct"]
    s = env._stream()
    args = lambda f, obs=o: (env._h, a.data_ptr(), ctypes.addressof(obs), env.reward.data_ptr(),  # noqa: E731
                             env.done.data_ptr(), f, s)
    assert L.wab_step_features(*args(feats.data_ptr() + 4)) == -1  # features not 16-byte aligned
    assert b"aligned" in L.wab_last_error()
    assert L.wab_step_features(*args(None)) == -1
    bad = _lib.WabObs(o.planes, None, o.role, o.status)
    assert L.wab_step_features(*args(feats.data_ptr(), bad)) == -1
    assert L.wab_step_features(*args(feats.data_ptr())) == 0
    torch.cuda.synchronize()
    fresh = _env(None, 256)  # no reset yet
    assert L.wab_step_features(fresh._h, a.data_ptr(), ctypes.addressof(fresh._obs["struct"]),
                               fresh.reward.data_ptr(), fresh.done.data_ptr(), feats.data_ptr(), s) == -4


def test_step_features_keeps_planes_when_asked():
    import torch

    from wab_gym_amd.wrappers import PragmaticObsWrapper

    ea, eb = _env(None, 640), _env(None, 640)
    wa = PragmaticObsWrapper(ea)
    wa.reset()
    eb.reset()
    for t in range(30):
        a = torch.full((640,), t % 5, device="cuda:0", dtype=torch.int8)
        wa.step(a)  # fused, planes stored
        eb.step(a)
        assert torch.equal(ea._obs["planes"], eb._obs["planes"]), t


def test_superbasic_matches_reference_golden_and_oracle():
    """Device SuperBasicObservationWrapper + flatten == the reference wrapper's golden vectors,
    and == the oracle on live env observations (31x31 included)."""
    import torch

    from oracle import oracle as orc
    from wab_gym_amd.wrappers import SuperBasicObservationWrapper

    z = np.load(gr.GOLDEN_DIR + "/superbasic.npz")
    n = len(z["features"])
    env = _env(None, n)
    wrap = SuperBasicObservationWrapper(env)
    assert wrap.feature_dim == int(z["flatdim"]) == 90
    planes = torch.as_tensor(z["planes"]).cuda()
    scal = torch.as_tensor(np.ascontiguousarray(z["scalars"].T)).cuda()
    f = wrap.observation({"planes": planes, "scalars": scal})
    assert np.array_equal(f.cpu().numpy(), z["features"])
    for opts in (None, {"width": 31, "height": 31}):
        env = _env(opts, 2000, validate_actions=False)
        wrap = SuperBasicObservationWrapper(env)
        wrap.reset()
        g = torch.Generator(device="cuda:0")
        g.manual_seed(2)
        for _ in range(20):
            f, r, d, _ = wrap.step(torch.randint(0, env.n_actions, (2000,), device="cuda:0", generator=g))
            planes = env._obs["planes"].cpu().numpy()
            sc = env._obs["scalars"].cpu().numpy()
            want = orc.featurize_superbasic(planes, sc[0], sc[1], sc[2], env.W, env.H,
                                            env.game_options["turns_to_empty_food"])
            assert np.array_equal(f.cpu().numpy(), want)


def test_render_matches_reference_frames_and_oracle():
    """f3: device render == the reference's rgb_array frames, with the draw_health text (its
    default) at scales 2, 32 and 1 and without it, and == the oracle on live observations
    (31x31, restrict_view, killed envs)."""
    import torch

    from oracle import oracle as orc

    z = np.load(gr.GOLDEN_DIR + "/render.npz")
    names = bytes(z["set_names"]).decode().split(",")
    scale = int(z["scale"])
    for si, name in enumerate(names):
        sel = z["set"] == si
        n = int(sel.sum())
        opts = {"restrict": {"restrict_view": True, "lookout_only": False},
                "longfood": {"turns_to_empty_food": 150}}.get(name)
        env = _env(opts, n)
        env.reset()
        env._obs["planes"].copy_(torch.as_tensor(z["planes"][sel]))
        env._obs["scalars"].copy_(torch.as_tensor(np.ascontiguousarray(z["scalars"][sel].T)))
        img = env.render(scale=scale, draw_health=False)
        assert np.array_equal(img.cpu().numpy(), z["images"][sel]), name
        img = env.render(scale=scale)  # draw_health=True, the reference's default
        assert np.array_equal(img.cpu().numpy(), z["images_health"][sel]), name
        big = np.nonzero(sel[z["big_idx"]])[0]
        bi = z["big_idx"][big]
        obs = {"planes": torch.as_tensor(z["planes"][bi]).cuda(),
               "scalars": torch.as_tensor(np.ascontiguousarray(z["scalars"][bi].T)).cuda()}
        env_b = _env(opts, len(bi))
        for s2, key in ((32, "images_health32"), (1, "images_health1")):
            img = env_b.render(scale=s2, obs=obs)
            assert np.array_equal(img.cpu().numpy(), z[key][big]), (name, s2)
    for opts in (None, {"width": 31, "height": 31}, {"restrict_view": True, "lookout_only": False},
                 {"chance_wolf_on_square": 0.05}):
        env = _env(opts, 300, validate_actions=False)
        env.reset()
        g = torch.Generator(device="cuda:0")
        g.manual_seed(3)
        for _ in range(15):
            env.step(torch.randint(0, env.n_actions, (300,), device="cuda:0", generator=g))
        for scale in (1, 3):
            for dh in (False, True):
                img = env.render(scale=scale, draw_health=dh).cpu().numpy()
                sc = env._obs["scalars"].cpu().numpy()
                want = orc.render(env._obs["planes"].cpu().numpy(), sc[1], sc[2], env.W, env.H,
                                  env.game_options["restrict_view"], scale, food_turns=sc[0], draw_health=dh)
                assert np.array_equal(img, want)


def test_discounted_returns_match_oracle():
    import torch

    from oracle import oracle as orc
    from wab_gym_amd.wrappers import discounted_returns, normalize_episode_returns

    rng = np.random.RandomState(0)
    T, B = 80, 5000
    reward = rng.choice([0.0, 0.1, -1.0, 1.0, -0.9, 1.1], size=(T, B)).astype(np.float32)
    done = (rng.random_sample((T, B)) < 0.03).astype(np.uint8)
    boot = rng.standard_normal(B).astype(np.float32)
    got = discounted_returns(torch.as_tensor(reward).cuda(), torch.as_tensor(done).cuda(), 0.99,
                             torch.as_tensor(boot).cuda())
    assert np.array_equal(got.cpu().numpy(), orc.discounted_returns(reward, done, 0.99, boot))
    # per-episode normalisation vs torch's own (R - mean) / (std + eps) on each segment
    norm = normalize_episode_returns(got, torch.as_tensor(done).cuda()).cpu()
    g = got.cpu()
    for b in range(0, B, 97):
        start = 0
        for t in range(T):
            if done[t, b] or t == T - 1:
                seg = g[start:t + 1, b]
                if seg.numel() > 1:
                    want = (seg - seg.mean()) / (seg.std() + np.finfo(np.float32).eps)
                    assert torch.allclose(norm[start:t + 1, b], want, rtol=1e-5, atol=1e-5)  # fp32 tolerance
                start = t + 1


def test_discounted_returns_exact_match_reference_finish_episode():
    """a14 on device, pinned by the reference's own finish_episode (tests/golden/returns.npz):
    the episodes laid out in 61 columns at different offsets, the device's exact-reward scan
    equals float32 of the reference's double returns bit for bit; per-episode normalisation
    matches the reference's float32 values within fp32 tolerance (rtol 1e-5, atol 1e-5: a
    different summation order of mean/std)."""
    import torch

    from wab_gym_amd.wrappers import discounted_returns, normalize_episode_returns

    z = np.load(gr.GOLDEN_DIR + "/returns.npz")
    n = len(z["done"])
    cols = 61
    # column c starts at the beginning of episode 29c (mod the episode count) and wraps around
    starts = np.concatenate([[0], np.nonzero(z["done"])[0][:-1] + 1])
    idx = (starts[(29 * np.arange(cols)) % len(starts)][None, :] + np.arange(n)[:, None]) % n
    rew = torch.as_tensor(z["rewards32"][idx]).cuda()
    done = torch.as_tensor(z["done"][idx]).cuda()
    env = _env(None, cols)
    got = discounted_returns(rew, done, float(z["gamma"]), env=env).cpu().numpy()
    want = z["returns64"].astype(np.float32)[idx]
    assert np.array_equal(got, want)
    plain = discounted_returns(rew, done, float(z["gamma"])).cpu().numpy()
    assert (plain != want).any()
    norm = normalize_episode_returns(torch.as_tensor(got).cuda(), done).cpu().numpy()
    # (a column's last, wrapped-around segment is cut short: compare whole episodes only)
    for c in range(cols):
        last_done = np.nonzero(z["done"][idx[:, c]])[0][-1]
        np.testing.assert_allclose(norm[:last_done + 1, c], z["normalised32"][idx[:last_done + 1, c]],
                                   rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------ config 5: fused rollout
def _step_features_loop(env, a, F, store_planes):
    """T step_features() calls of `env` (the unfused-launch reference of rollout_features)."""
    import torch

    T, B = a.shape
    feats = torch.empty((T, B, F), device="cuda:0")
    rew = torch.empty((T, B), device="cuda:0")
    done = torch.empty((T, B), dtype=torch.uint8, device="cuda:0")
    scal, planes = [], []
    for t in range(T):
        _, r, d = env.step_features(a[t], feats[t], store_planes=store_planes)
        rew[t] = r
        done[t] = d.to(torch.uint8)
        scal.append(env._obs["scalars"].clone())
        if store_planes:
            planes.append(env._obs["planes"].clone())
    return feats, rew, done, torch.stack(scal), (torch.stack(planes) if store_planes else None)


@pytest.mark.parametrize("opts,kw,T,planes", [
    (None, {}, 40, False),                                            # G = 11, 8 slots
    (None, {}, 33, True),                                             # planes stored too
    ({"width": 9, "height": 9, "starting_food": None, "starting_role": None}, {"wolf_slots": 16}, 40, False),
    ({"restrict_view": True, "lookout_only": False}, {"wolf_slots": 32}, 40, False),
    (None, {"autoreset": False}, 90, False),                          # stepping past done
    (None, {}, 130, False),                                           # T > 128: returns by the scan kernel
    ({"width": 9, "height": 13}, {}, 20, False),                      # not fusable: step_features loop
])
def test_rollout_features_equals_step_features_loop(opts, kw, T, planes):
    """wab_rollout_features (one launch: T fused steps + the segment's returns) == T
    wab_step_features calls + wab_discounted_returns_exact, bit for bit, over two consecutive
    rollouts (state carried across calls; the second with a bootstrap), a partial last group
    included; final hidden state and counters equal too."""
    import torch

    from wab_gym_amd.wrappers import discounted_returns

    B = 1008  # 15 full groups + 48 envs; B * 449 (B * 363) a multiple of 4 (16): aligned steps
    e1, e2 = _env(opts, B, validate_actions=False, **kw), _env(opts, B, validate_actions=False, **kw)
    e1.reset()
    e2.reset()
    rs = np.random.RandomState(11)
    for seg in range(2):
        a = torch.as_tensor(rs.randint(e1.n_actions, size=(T, B)))
        bs = None if seg == 0 else torch.as_tensor(rs.standard_normal(B).astype(np.float32), device="cuda:0")
        r = e1.rollout_features(a, gamma=0.97, bootstrap=bs, store_planes=planes)
        F = r["features"].shape[2]
        feats, rew, done, scal, pl = _step_features_loop(e2, a.cuda(), F, planes)
        for t in range(T):
            assert torch.equal(r["features"][t], feats[t]), (seg, t)
            assert torch.equal(r["scalars"][t], scal[t]), (seg, t)
        assert torch.equal(r["reward"], rew) and torch.equal(r["done"], done), seg
        if planes:
            assert torch.equal(r["planes"], pl), seg
        want = discounted_returns(rew, done, gamma=0.97, bootstrap=bs, env=e2)
        assert torch.equal(r["returns"], want), seg
    s1, s2 = e1.state(), e2.state()
    for k in s1:
        assert np.array_equal(np.asarray(s1[k]), np.asarray(s2[k])), k
    assert _device_counters(e1) == _device_counters(e2)


def test_rollout_features_full_size_c5():
    """C5 at full size (B = 65536, T = 64 = bench.py's C5_SEGMENT): the single rollout launch ==
    64 fused step launches + the exact returns scan, bit for bit, twice in a row; the returns
    equal the reference's recursion run in float64 on the host for a sample of envs.  (The
    same launches against the oracle: tests/test_gpu_bench_parity.py.)"""
    import torch

    from wab_gym_amd.wrappers import discounted_returns

    B, T = 65536, 64
    e1, e2 = _env(None, B, validate_actions=False), _env(None, B, validate_actions=False)
    e1.reset()
    e2.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(21)
    for seg in range(2):
        a = torch.randint(0, 5, (T, B), device="cuda:0", generator=g).to(torch.int8)
        r = e1.rollout_features(a)
        feats, rew, done, scal, _ = _step_features_loop(e2, a, 449, False)
        assert torch.equal(r["features"], feats), seg
        assert torch.equal(r["reward"], rew) and torch.equal(r["done"], done), seg
        assert torch.equal(r["scalars"], scal), seg
        assert torch.equal(r["returns"], discounted_returns(rew, done, gamma=0.99, env=e2)), seg
        del feats
    # finish_episode's loop (actor_critic.py:139-143) on the float64 rewards of 64 envs
    opts = e1.game_options
    rt = rew.double().cpu().numpy()
    dn = done.cpu().numpy()
    exact = {np.float32(v): v for v in (opts["reward_per_turn"], opts["reward_for_finishing"],
                                        opts["reward_for_starving"], opts["reward_for_being_killed"])}
    for x in list(exact.values()):
        exact[np.float32(0.0 + opts["reward_for_eating"] + x)] = 0.0 + opts["reward_for_eating"] + x
    ret = r["returns"].cpu().numpy()
    for b in range(0, B, B // 64):
        R = 0.0
        for t in range(T - 1, -1, -1):
            if dn[t, b]:
                R = 0.0
            R = exact.get(np.float32(rt[t, b]), float(rt[t, b])) + 0.99 * R
            assert np.float32(R) == ret[t, b], (b, t)
    assert _device_counters(e1) == _device_counters(e2)


# ------------------------------------------------------------------ the wide kernel's rollout build
@pytest.mark.parametrize("opts,stride,slots,autoreset", [
    ({"width": 31, "height": 31}, 32, 8, True),
    ({"width": 31, "height": 31}, 32, 32, True),
    ({"width": 31, "height": 31, "chance_wolf_on_square": 0.01, "wolf_chance_to_despawn": 0.2,
      "wolf_spawn_margin": 2}, 32, 32, True),                          # HBM wolf rows every step
    ({"width": 31, "height": 31, "chance_wolf_on_square": 0.01, "wolf_chance_to_despawn": 0.2,
      "wolf_spawn_margin": 2}, 32, 16, True),                          # ... and the cap
    ({"width": 17, "height": 13, "lookout_only": False}, 16, 8, True),
    ({"width": 25, "height": 29, "starting_food": None, "starting_role": None}, 32, 16, True),
    ({"width": 31, "height": 15, "wolves_can_move": False, "god_mode": True}, 16, 8, True),
    ({"width": 13, "height": 11, "turns_to_fill_food": 4, "max_turns": 60, "bush_power": 60}, 16, 8, True),
    ({"width": 31, "height": 31}, 32, 16, False),                     # stepping past done
    # eats nearly every turn, two berries per bush: eaten logs past the entries the wide rollout keeps on chip (kWideRollLog)
    ({"width": 31, "height": 31, "bush_power": 1, "max_berries_per_bush": 2, "max_turns": 120}, 32, 16, True),
    ({"width": 25, "height": 25, "bush_power": 1, "max_berries_per_bush": 3}, 32, 8, True),
])
def test_wide_rollout_equals_step_loop(opts, stride, slots, autoreset):
    """wab_rollout on the wide kernel (one launch of T steps, state carried on chip) == T wab_step
    calls, bit for bit, over two consecutive rollouts, a partial last group included; final hidden
    state and counters equal too."""
    import torch

    B, T = 1000, 45
    rs = np.random.RandomState(13)
    kw = dict(validate_actions=False, plane_stride=stride, wolf_slots=slots, autoreset=autoreset)
    if opts.get("bush_power") == 1:
        kw["eaten_capacity"] = 40 if opts.get("max_turns") else 3  # (3: the log overflows)
    e1, e2 = _env(opts, B, **kw), _env(opts, B, **kw)
    assert e1.step_kernel == "wide"
    e1.reset()
    e2.reset()
    for seg in range(2):
        a = torch.as_tensor(rs.randint(e1.n_actions, size=(T, B)))
        planes, scal, rew, done = e1.rollout(a)
        for t in range(T):
            obs, r, d, _ = e2.step(a[t])
            assert torch.equal(planes[t], e2._obs["planes"]), (seg, t)
            assert torch.equal(scal[t], e2._obs["scalars"]), (seg, t)
            assert torch.equal(rew[t], r) and torch.equal(done[t].bool(), d), (seg, t)
    s1, s2 = e1.state(), e2.state()
    for k in s1:
        assert np.array_equal(np.asarray(s1[k]), np.asarray(s2[k])), k
    assert _device_counters(e1) == _device_counters(e2)


@pytest.mark.parametrize("wide", [False, True])
def test_rollout_tiny_batch(wide):
    """A batch smaller than one 64-env group (16 envs), both rollout builds."""
    import torch

    opts = {"width": 31, "height": 31} if wide else None
    kw = dict(validate_actions=False, plane_stride=32) if wide else dict(validate_actions=False)
    e1, e2 = _env(opts, 16, **kw), _env(opts, 16, **kw)
    e1.reset()
    e2.reset()
    a = torch.as_tensor(np.random.RandomState(5).randint(5, size=(50, 16)))
    planes, scal, rew, done = e1.rollout(a)
    for t in range(50):
        e2.step(a[t])
        assert torch.equal(planes[t], e2._obs["planes"]), t
        assert torch.equal(rew[t], e2.reward), t
    assert _device_counters(e1) == _device_counters(e2)


def test_wide_rollout_full_size_c3():
    """C3 at full size (B = 65536, 31x31 in 32x32 planes, 8 register wolves + HBM rows to 32):
    two 64-step rollout launches (bench.py's T) == 128 wab_step launches, bit for bit, past the
    turn-40 and turn-80 mass resets.  (The same launches against the oracle:
    tests/test_gpu_bench_parity.py.)"""
    import torch

    B, T = 65536, 64
    kw = dict(validate_actions=False, plane_stride=32, wolf_slots=32)
    opts = {"width": 31, "height": 31}
    e1, e2 = _env(opts, B, **kw), _env(opts, B, **kw)
    e1.reset()
    e2.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(17)
    for seg in range(2):
        a = torch.randint(0, 5, (T, B), device="cuda:0", generator=g).to(torch.int8)
        planes, scal, rew, done = e1.rollout(a)
        for t in range(T):
            e2.step(a[t])
            assert torch.equal(planes[t], e2._obs["planes"]), (seg, t)
            assert torch.equal(rew[t], e2.reward) and torch.equal(done[t].bool(), e2.done.bool()), (seg, t)
            assert torch.equal(scal[t], e2._obs["scalars"]), (seg, t)
        del planes
    assert _device_counters(e1) == _device_counters(e2)


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("T", [1, 2, 3])
def test_rollout_short_segments(wide, T):
    """Rollouts of 1, 2 and 3 steps (the first step is also the last; one carried step) chained
    five times, both rollout builds, == the step loop; C5's fused rollout too on the small view."""
    import torch

    from wab_gym_amd.wrappers import discounted_returns

    opts = {"width": 31, "height": 31} if wide else None
    kw = dict(validate_actions=False, plane_stride=32) if wide else dict(validate_actions=False)
    B = 192
    e1, e2 = _env(opts, B, **kw), _env(opts, B, **kw)
    e1.reset()
    e2.reset()
    rs = np.random.RandomState(T)
    for seg in range(5):
        a = torch.as_tensor(rs.randint(5, size=(T, B)))
        planes, scal, rew, done = e1.rollout(a)
        for t in range(T):
            e2.step(a[t])
            assert torch.equal(planes[t], e2._obs["planes"]), (seg, t)
            assert torch.equal(rew[t], e2.reward) and torch.equal(done[t].bool(), e2.done.bool()), (seg, t)
    assert _device_counters(e1) == _device_counters(e2)
    if not wide:
        e3, e4 = _env(None, B, **kw), _env(None, B, **kw)
        e3.reset()
        e4.reset()
        for seg in range(5):
            a = torch.as_tensor(rs.randint(5, size=(T, B))).cuda()
            r = e3.rollout_features(a)
            feats, rw, dn, _, _ = _step_features_loop(e4, a, 449, False)
            assert torch.equal(r["features"], feats) and torch.equal(r["reward"], rw), seg
            assert torch.equal(r["returns"], discounted_returns(rw, dn, gamma=0.99, env=e4)), seg


def test_env_buffers_after_rollouts():
    """After env.rollout the env's obs, reward and done are the last step's (as after T step()
    calls); after rollout_features without planes the scalars/reward/done are, and the env's
    own planes are reported stale (observation()/render() of them raise) until the next step;
    PragmaticObsWrapper.rollout leaves the wrapper's features at the last step's."""
    import torch

    from wab_gym_amd.wrappers import PragmaticObsWrapper

    B, T = 640, 12
    e1, e2 = _env(None, B, validate_actions=False), _env(None, B, validate_actions=False)
    e1.reset()
    e2.reset()
    a = torch.as_tensor(np.random.RandomState(1).randint(5, size=(T, B)))
    planes, scal, rew, done = e1.rollout(a)
    for t in range(T):
        e2.step(a[t])
    e1._require_planes()  # (the env's own planes are copied from planes[T-1] when first needed)
    assert torch.equal(e1._obs["planes"], e2._obs["planes"]) and torch.equal(e1._obs["planes"], planes[-1])
    assert torch.equal(e1._obs["scalars"], e2._obs["scalars"])
    assert torch.equal(e1.reward, e2.reward) and torch.equal(e1.done, e2.done)
    w1, w2 = PragmaticObsWrapper(e1), PragmaticObsWrapper(e2)
    assert torch.equal(w1.observation(), w2.observation())
    f, r, d, ret = w1.rollout(a)
    for t in range(T):
        w2.step(a[t])
    assert torch.equal(w1.features, f[-1]) and torch.equal(w1.features, w2.features)
    assert torch.equal(e1.reward, e2.reward) and torch.equal(e1._obs["scalars"], e2._obs["scalars"])
    with pytest.raises(RuntimeError):
        w1.observation()
    with pytest.raises(RuntimeError):
        e1.render(scale=1)
    e1.step(a[0])
    e2.step(a[0])
    assert torch.equal(w1.observation(), w2.observation())


def test_rollout_features_ambiguous_rewards_fail_before_stepping():
    """Options whose step rewards collide in float32 (r_x and r_eat + r_x) cannot give exact
    returns from the scan kernel: a rollout_features call that would need it (T > 128) fails
    before any step runs (the env's counters do not move); T <= 128 fuses the returns from the
    reward codes and works; returns=False always works."""
    import torch

    from wab_gym_amd.options import default_game_options

    o = dict(default_game_options)
    o["reward_for_eating"] = 1e-12
    o["reward_per_turn"] = 0.3
    env = _env(o, 256, validate_actions=False)
    env.reset()
    a = torch.zeros((130, 256), dtype=torch.int8, device="cuda:0")
    steps0 = env.counters()["steps"]
    with pytest.raises(ValueError):
        env.rollout_features(a)
    assert env.counters()["steps"] == steps0
    r = env.rollout_features(a[:64])
    assert r["returns"] is not None
    r = env.rollout_features(a, returns=False)
    assert r["returns"] is None and env.counters()["steps"] == steps0 + 194 * 256


def test_wide_step_into_alternating_buffers():
    """The wide view's wab_step runs the per-step kernel (WAB_OBS_SAME_BUFFER, the default) or a
    one-step launch of its rollout build (wab_set_obs_placement(WAB_OBS_FRESH_BUFFER)): steps
    alternating between two obs buffers, under either placement and switching placement every
    20 steps, match the oracle bit for bit."""
    import ctypes

    import torch

    from wab_gym_amd import _lib

    opts = {"width": 31, "height": 31}
    n = 1024
    env = _env(opts, n, plane_stride=32, wolf_slots=32, validate_actions=False)
    orc = _oracle(opts, n, stride=32)
    env.reset()
    orc.reset()
    assert env.step_kernel == "wide"
    bufs = [env._alloc_obs() for _ in range(2)]
    L = _lib.load()
    assert L.wab_set_obs_placement(env._h, 7) == -1
    rng = np.random.RandomState(21)
    for t in range(120):
        if t % 20 == 0:
            _lib.check(L.wab_set_obs_placement(env._h, (t // 20) % 2), "wab_set_obs_placement")
        a = rng.randint(5, size=n)
        o = bufs[t % 2] if t < 80 else bufs[0]
        ad = torch.as_tensor(a.astype(np.int8), device="cuda:0")
        _lib.check(L.wab_step(env._h, ad.data_ptr(), ctypes.addressof(o["struct"]), env.reward.data_ptr(),
                              env.done.data_ptr(), None, env._stream()), "wab_step")
        op, of, orl, ost, orew, odone = orc.step(a, nthreads=16)
        assert np.array_equal(o["planes"].cpu().numpy(), op), t
        assert np.array_equal(o["scalars"].cpu().numpy(), np.stack([of, orl, ost])), t
        assert np.array_equal(env.reward.cpu().numpy(), orew), t
        assert np.array_equal(env.done.cpu().numpy(), odone), t
    c = env.counters()
    assert c["wolf_overflow"] == 0 and c["handoff_timeouts"] == 0 and c["steps"] == 120 * n


def test_env_step_into_obs_ring_fresh_placement():
    """BatchedWolvesAndBushesEnv(obs_placement="fresh") + step(actions, obs=slot): a closed
    loop's ring of observation buffers on the wide view (the one-step rollout build) and on the
    default view, against the oracle; every slot keeps its step's observation."""
    import torch

    for opts, stride, slots in (({"width": 31, "height": 31}, 32, 32), (None, 0, 8)):
        n = 512
        env = _env(opts, n, plane_stride=stride, wolf_slots=slots, obs_placement="fresh")
        orc = _oracle(opts, n, stride=stride)
        env.reset()
        orc.reset()
        ring = [env.alloc_obs() for _ in range(3)]
        kept = []
        rng = np.random.RandomState(5)
        for t in range(40):
            a = rng.randint(5, size=n)
            obs, rew, done, _ = env.step(torch.as_tensor(a), obs=ring[t % 3])
            op, of, orl, ost, orew, odone = orc.step(a, nthreads=16)
            assert obs[0].data_ptr() == ring[t % 3]["planes"].data_ptr()
            assert np.array_equal(ring[t % 3]["planes"].cpu().numpy(), op), t
            assert np.array_equal(obs[3].cpu().numpy(), of), t
            assert np.array_equal(rew.cpu().numpy(), orew), t
            kept.append(op.copy())  # (the oracle returns its own buffer)
            if t >= 2:  # the slot written two steps ago still holds its step
                assert np.array_equal(ring[(t - 2) % 3]["planes"].cpu().numpy(), kept[t - 2]), t
        with pytest.raises(RuntimeError):
            env.render(scale=1)  # the env's own buffer was not written
        with pytest.raises(ValueError):
            env.step(torch.zeros(n, dtype=torch.int8), obs={"planes": ring[0]["planes"][:, :, :, :1],
                                                           "scalars": ring[0]["scalars"]})
        env.close()


def test_rollout_updates_obs_views_eagerly():
    """After env.rollout(T), the obs tuple an earlier step() returned shows step T-1 in planes and
    scalars alike (planes[T-1] copied into the env's buffer on the launch's stream)."""
    import torch

    env = _env(None, 256)
    env.reset()
    obs, _, _, _ = env.step(torch.zeros(256, dtype=torch.int8))
    planes, scal, rew, done = env.rollout(torch.randint(0, 5, (9, 256), device="cuda:0"))
    for k in range(3):
        assert torch.equal(obs[k], planes[8, :, k, :, :env.H])
    assert torch.equal(obs[3], scal[8, 0]) and torch.equal(obs[5], scal[8, 2])
