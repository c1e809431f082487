"""The kernels bench.py times, against the C oracle, at the bench's own configuration.

Every line of bench.py is a chain of 64-step rollout launches at B = 65536: `wab_rollout` on
the small kernel (default 11x11, the headline), `wab_rollout` on the wide kernel (C3: 31x31 in
32x32 planes, 32 wolf rows) and `wab_rollout_features` (C5: features + the segment's returns).
Here the same launches run back to back (state carried across them, past the turn-40 mass
starvation and the turn-80 cap) and every step of every launch is compared with
`OracleBatch.step` (oracle/wab_oracle.c, pinned to the reference's golden vectors by
tests/test_oracle_golden.py): obs planes, scalars, reward, done; after each launch the hidden
state (food double by bit pattern, position, turn, wolf count, episode).  C5's features are
compared with the oracle's PragmaticObsWrapper + flatten of the oracle's own planes, and the
returns with the oracle's float64 recursion of finish_episode (actor_critic.py:139-143) over the
exact double rewards.  Reference semantics: wab_env.py:250-342, actor_critic.py:185-200.
"""
import numpy as np
import pytest

from backends import SEED

pytestmark = pytest.mark.gpu

B = 65536
T = 64  # bench.py DEFAULT_ROLLOUT / C5_SEGMENT
THREADS = 16  # the GPU box's CPU share


def _pair(opts, stride=0, slots=0):
    from oracle.oracle import OracleBatch
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    env = BatchedWolvesAndBushesEnv(opts, num_envs=B, seed=SEED, device="cuda:0", autoreset=True,
                                    validate_actions=False, plane_stride=stride, wolf_slots=slots)
    orc = OracleBatch(opts, B, SEED, 0, True, stride)
    env.reset()
    orc.reset()
    return env, orc


def _actions(seed, n_actions):
    """One launch's [T, B] int8 actions, drawn on the device as bench.py draws them."""
    import torch

    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    return torch.randint(0, n_actions, (T, B), device="cuda:0", generator=g).to(torch.int8)


def _same(got, want_np, what):
    """Device tensor == host array, compared on the device (the arrays are tens of MB)."""
    import torch

    want = torch.from_numpy(np.ascontiguousarray(want_np)).to(got.device)
    if not torch.equal(got, want):
        bad = (got != want).reshape(got.shape[0], -1).any(1).nonzero()[:8, 0].tolist()
        raise AssertionError("%s differs for envs %s" % (what, bad))


def _state_equal(env, orc, what):
    gs, os_ = env.state(), orc.state()
    for k in ("x", "y", "turn", "n_wolves", "episode"):
        assert np.array_equal(gs[k], os_[k]), (what, k)
    assert np.array_equal(gs["food"].view(np.uint64), os_["food"].view(np.uint64)), what


def _counters_clean(env, steps):
    c = env.counters()
    assert c["wolf_overflow"] == 0 and c["eaten_overflow"] == 0, c
    assert c["handoff_timeouts"] == 0 and c["bad_actions"] == 0, c
    assert c["steps"] == steps, c
    return c


def _rollout_vs_oracle(opts, stride, slots, launches, kernel):
    env, orc = _pair(opts, stride, slots)
    assert env.step_kernel == kernel
    for k in range(launches):
        a = _actions(100 + k, env.n_actions)
        planes, scal, rew, done = env.rollout(a)
        ah = a.cpu().numpy()
        for t in range(T):
            op, of, orl, ost, orew, odone = orc.step(ah[t], nthreads=THREADS)
            what = "launch %d step %d" % (k, t)
            _same(planes[t], op, what + " planes")
            _same(scal[t], np.stack([of, orl, ost]), what + " scalars")
            _same(rew[t], orew, what + " reward")
            _same(done[t], odone, what + " done")
        del planes
        _state_equal(env, orc, "after launch %d" % k)
    return _counters_clean(env, launches * T * B)


def test_headline_rollout_bench_config_vs_oracle():
    """The headline line's kernel (wab_step_small rollout build, T = 64, B = 65536, all 1024
    workgroups resident: 4 per CU), four launches = 256 steps, every step vs the oracle."""
    c = _rollout_vs_oracle(None, 0, 8, 4, "small")
    assert c["resets"] > 4 * B  # the initial reset + at least three episodes per env


def test_wide_rollout_bench_config_vs_oracle():
    """C3's line (wab_rollout_wide<8>: 31x31 in 32x32 planes, 8 register wolves + 32 HBM rows,
    T = 64, B = 65536), three launches = 192 steps, every step vs the oracle."""
    c = _rollout_vs_oracle({"width": 31, "height": 31}, 32, 32, 3, "wide")
    assert c["resets"] > 2 * B


def test_rollout_features_bench_config_vs_oracle():
    """C5's line (wab_rollout_features: T = 64, B = 65536, planes rendered on chip and not
    stored, R_T = 0 as bench.py runs it), four launches: features vs the oracle's
    PragmaticObsWrapper + flatten of the oracle's obs, reward/done/scalars vs the oracle step,
    returns vs the oracle's float64 finish_episode recursion over the exact double rewards."""
    from oracle import oracle as O
    from test_featurizer_oracle import step_reward_values

    env, orc = _pair(None)
    vm = np.zeros((B, 11, 11), np.uint8)
    exact = step_reward_values()
    for k in range(4):
        a = _actions(200 + k, env.n_actions)
        r = env.rollout_features(a, gamma=0.99)
        assert r["planes"] is None
        ah = a.cpu().numpy()
        rew = np.zeros((T, B), np.float32)
        done = np.zeros((T, B), np.uint8)
        for t in range(T):
            op, of, orl, ost, orew, odone = orc.step(ah[t], nthreads=THREADS)
            what = "launch %d step %d" % (k, t)
            _same(r["features"][t], O.featurize(op, of, orl, ost, vm, 11, 11), what + " features")
            _same(r["scalars"][t], np.stack([of, orl, ost]), what + " scalars")
            _same(r["reward"][t], orew, what + " reward")
            _same(r["done"][t], odone, what + " done")
            rew[t], done[t] = orew, odone
        want = O.discounted_returns(rew, done, 0.99, None, exact_values=exact)
        _same(r["returns"], want, "launch %d returns" % k)
        _state_equal(env, orc, "after launch %d" % k)
    c = _counters_clean(env, 4 * T * B)
    assert c["resets"] > 4 * B


def _shards_equal_one_handle(opts, stride, slots, launch, keys, seed0):
    """bench.py's --stream-shards 2: the batch as two handles of B / 2 envs (ids 0.. and B/2..),
    each shard's launches on its own HIP stream, running concurrently.  Every output of every
    launch (launch(env, actions) -> dict of [T, ..., B-slice ...] tensors, the env axis at
    keys[name]), and the final hidden state, equal one handle of B envs stepped with the same
    actions (which the tests above pin to the oracle)."""
    import torch

    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    S, Bs = 2, B // 2
    mk = lambda n, base: BatchedWolvesAndBushesEnv(opts, num_envs=n, seed=SEED, device="cuda:0",  # noqa: E731
                                                   env_id_base=base, autoreset=True, validate_actions=False,
                                                   plane_stride=stride, wolf_slots=slots)
    one = mk(B, 0)
    shards = [mk(Bs, k * Bs) for k in range(S)]
    for e in [one] + shards:
        e.reset()
    streams = [torch.cuda.Stream() for _ in range(S)]
    for k in range(3):  # three launches: past the turn-80 cap of the first episodes
        a = _actions(seed0 + k, one.n_actions)
        a_sh = [a[:, j * Bs:(j + 1) * Bs].contiguous() for j in range(S)]
        cur = torch.cuda.current_stream()
        outs = []
        for j, (e, st) in enumerate(zip(shards, streams)):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                outs.append(launch(e, a_sh[j]))
        want = launch(one, a)
        for st in streams:
            cur.wait_stream(st)
        torch.cuda.synchronize()
        for j, got in enumerate(outs):
            for name, axis in keys.items():
                w = want[name].narrow(axis, j * Bs, Bs)
                assert torch.equal(got[name], w), (k, j, name)
        del outs, want
    so = one.state()
    for j, e in enumerate(shards):
        ss = e.state()
        for key in ss:
            assert np.array_equal(ss[key], so[key][j * Bs:(j + 1) * Bs]), (j, key)


def _rollout_dict(e, a):
    planes, scal, rew, done = e.rollout(a)
    return {"planes": planes, "scalars": scal, "reward": rew, "done": done}


def test_headline_stream_shards_equal_one_handle():
    """The headline line as bench.py runs it: two shards of wab_rollout (small kernel)."""
    _shards_equal_one_handle(None, 0, 8, _rollout_dict, {"planes": 1, "scalars": 2, "reward": 1, "done": 1}, 900)


def test_wide_stream_shards_equal_one_handle():
    """C3's line as bench.py runs it: two shards of wab_rollout on the wide kernel."""
    _shards_equal_one_handle({"width": 31, "height": 31}, 32, 32, _rollout_dict,
                             {"planes": 1, "scalars": 2, "reward": 1, "done": 1}, 910)


def test_features_stream_shards_equal_one_handle():
    """C5's line as bench.py runs it: two shards of wab_rollout_features (features, scalars,
    reward, done and the segment's returns)."""
    _shards_equal_one_handle(None, 0, 8, lambda e, a: e.rollout_features(a, gamma=0.99),
                             {"features": 1, "scalars": 2, "reward": 1, "done": 1, "returns": 1}, 920)
