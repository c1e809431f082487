"""The HIP torus world (wab_torus.hip via include/wab_torus.h) against the golden vectors of the
real Environment 2.0 reference and against the C oracle, bit for bit.

Sizes: every golden world replayed turn by turn and as one rollout launch; lockstep against the
oracle at B = 4096 and at the bench's configuration (B = 65536, 32x32, 1/8/16, 64-turn rollout
launches); ragged batches, misaligned action slices, masked resets, no autoreset."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ["torus_c3", "torus_multi", "torus_tiny", "torus_continue", "torus_placed"]


def load_set(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    return d, json.loads(d["meta"].tobytes())


def make_env(meta, world_id, batch=1, **kw):
    from wab_gym_amd.torus import BatchedWABEnvironment2

    return BatchedWABEnvironment2(meta["width"], meta["height"], meta["options"], meta["num_ostriches"],
                                  meta["num_wolves"], meta["num_bushes"], num_worlds=batch, seed=meta["seed"],
                                  device="cuda:0", world_id_base=world_id,
                                  autoreset=meta["protocol"] == "autoreset", **kw)


def oracle(meta, base, batch, autoreset=None):
    from oracle.torus_oracle import OracleTorus

    ar = meta["protocol"] == "autoreset" if autoreset is None else autoreset
    return OracleTorus(meta["width"], meta["height"], meta["num_ostriches"], meta["num_wolves"],
                       meta["num_bushes"], meta["options"], batch=batch, seed=meta["seed"],
                       world_id_base=base, autoreset=ar)


def placed_schedule(d, meta, e):
    """A placed set's explicit positions of world index e: (create [N, 2] or None, {turn:
    reset positions [N, 2]}; turn 0 is the first reset)."""
    turns = meta.get("placed_resets") or []
    if not turns:
        return None, {}
    return d["create_pos"][e], {t: d["reset_pos"][k, e] for k, t in enumerate(turns)}


def check_state(env, d, t, e, where):
    s = env.state()
    NO = env.num_ostriches
    assert np.array_equal(s["df_xy"][0], d["df_xy"][t, e]), where + " frame X/Y"
    assert np.array_equal(s["obj_xy"][0], d["obj_xy"][t, e]), where + " object x/y"
    assert np.array_equal(s["food"][0], d["food"][t, e]), where + " food"
    assert np.array_equal(s["visible"][0].astype(bool), d["visible"][t, e]), where + " Visible"
    assert np.array_equal(s["status"][0, :NO], d["status"][t, e, :NO]), where + " status"


@pytest.mark.parametrize("name", SETS)
def test_torus_steps_match_reference_golden(name):
    import torch

    d, meta = load_set(name)
    for e, g in enumerate(meta["world_ids"]):
        create, resets = placed_schedule(d, meta, e)
        env = make_env(meta, g, spawn_positions=create)
        s = env.state()
        assert np.array_equal(s["df_xy"][0], d["create_df_xy"][e]), "create_* positions"
        env.reset_environment(positions=resets.get(0))
        assert np.array_equal(env.state()["obj_xy"][0], d["reset0_obj_xy"][e]), "reset positions"
        for t in range(meta["T"]):
            if t > 0 and t in resets:
                env.reset_environment(positions=resets[t])
            obs, rew, done, info = env.step(torch.as_tensor(d["actions"][t, e][None]))
            where = "%s world %d turn %d" % (name, g, t)
            o = obs[0].cpu().numpy()
            bad = np.nonzero((o != d["records"][t, e]).any(axis=1))[0]
            assert len(bad) == 0, "%s: records of entities %s differ" % (where, bad.tolist())
            assert np.array_equal(rew[0].cpu().numpy(), d["reward"][t, e].astype(np.float32)), where
            assert np.array_equal(done[0].cpu().numpy(), d["done"][t, e]), where
            assert bool(info["world_reset"][0]) == bool(d["world_reset"][t, e]), where
            if t % 10 == 9 or t == meta["T"] - 1:
                check_state(env, d, t, e, where)


@pytest.mark.parametrize("name", SETS)
def test_torus_rollout_matches_reference_golden(name):
    """Every golden world's whole run as ONE rollout launch (state on chip between turns)."""
    import torch

    d, meta = load_set(name)
    T = meta["T"]
    for e, g in enumerate(meta["world_ids"]):
        create, resets = placed_schedule(d, meta, e)
        env = make_env(meta, g, spawn_positions=create)
        env.reset_environment(positions=resets.get(0))
        # one launch per stretch between explicit resets (one launch for the sets without)
        cuts = [0] + sorted(t for t in resets if t > 0) + [T]
        parts = []
        for t0, t1 in zip(cuts[:-1], cuts[1:]):
            if t0 > 0:
                env.reset_environment(positions=resets[t0])
            parts.append(env.rollout(torch.as_tensor(d["actions"][t0:t1, e][:, None])))
        obs, rew, done, wr = (torch.cat([p[k] for p in parts]) for k in range(4))
        o = obs[:, 0].cpu().numpy()
        bad = np.argwhere((o != d["records"][:, e]).any(axis=2))
        assert len(bad) == 0, "%s world %d: (turn, entity) %s differ" % (name, g, bad[:5].tolist())
        assert np.array_equal(rew[:, 0].cpu().numpy(), d["reward"][:, e].astype(np.float32))
        assert np.array_equal(done[:, 0].cpu().numpy().astype(bool), d["done"][:, e])
        assert np.array_equal(wr[:, 0].cpu().numpy().astype(bool), d["world_reset"][:, e])
        check_state(env, d, T - 1, e, "%s world %d after the rollout" % (name, g))


def _lockstep(meta, B, T, rollout_T=0, base=0, seed_actions=7, check_every=1):
    import torch

    env = make_env(meta, base, batch=B)
    orc = oracle(meta, base, B)
    env.reset_environment()
    orc.reset()
    rng = np.random.RandomState(seed_actions)
    N = env.N
    hi = np.array([6] * meta["num_ostriches"] + [5] * meta["num_wolves"] + [1] * meta["num_bushes"])
    t = 0
    while t < T:
        n = rollout_T or 1
        acts = (rng.randint(0, 1 << 30, size=(n, B, N)) % hi).astype(np.int8)
        if rollout_T:
            obs, rew, done, wr = env.rollout(torch.as_tensor(acts))  # (device; one turn at a time to host)
        for k in range(n):
            r_o, rw_o, d_o, wr_o = orc.step(acts[k], nthreads=16)
            if rollout_T:
                g = (obs[k].cpu().numpy(), rew[k].cpu().numpy(), done[k].cpu().numpy(), wr[k].cpu().numpy())
            else:
                ob, rw, dn, info = env.step(torch.as_tensor(acts[k]))
                g = (ob.cpu().numpy(), rw.cpu().numpy(), dn.cpu().numpy(), info["world_reset"].cpu().numpy())
            where = "B=%d turn %d" % (B, t + k)
            if (t + k) % check_every == 0 or t + k == T - 1:
                bad = np.argwhere((g[0] != r_o).any(axis=2))
                assert len(bad) == 0, "%s: (world, entity) %s differ" % (where, bad[:5].tolist())
            assert np.array_equal(g[1], rw_o), where
            assert np.array_equal(g[2].astype(np.uint8), d_o), where
            assert np.array_equal(g[3].astype(np.uint8), wr_o), where
        t += n
    s, so = env.state(), orc.state()
    for key in so:
        assert np.array_equal(s[key], so[key]), key
    c = env.counters()
    assert c["turns"] == B * T
    return env


def test_torus_lockstep_b4096_vs_oracle():
    _, meta = load_set("torus_c3")
    _lockstep(meta, 4096, 120)


def test_torus_rollout_bench_config_vs_oracle():
    """The bench's workload: B = 65536 worlds, 32x32, 1 ostrich / 8 wolves / 16 bushes, 64-turn
    rollout launches, every turn's records against the oracle."""
    _, meta = load_set("torus_c3")
    env = _lockstep(meta, 65536, 128, rollout_T=64, check_every=1)
    assert env.counters()["resets"] > 1000


def test_torus_lockstep_multi_ostrich_ragged_batch():
    """3 ostriches (the Visible-label quirk), a batch that is not a multiple of 64 and whose
    [B, N] action slices are not 4-byte aligned (the kernel's per-byte action path)."""
    _, meta = load_set("torus_multi")
    _lockstep(meta, 1001, 90)
    _lockstep(meta, 77, 70, rollout_T=35, base=123)


def test_torus_rollout_misaligned_actions():
    """N = 9: the [B, N] action slice of every turn is not 4-byte aligned (B * N odd), so each
    workgroup reads the next turn's actions per byte instead of with scalar loads."""
    _, meta = load_set("torus_continue")
    _lockstep(meta, 301, 60, rollout_T=30, base=9)


def test_torus_tiny_worlds_lockstep():
    _, meta = load_set("torus_tiny")
    _lockstep(meta, 640, 100, rollout_T=25)


def test_torus_masked_reset_and_no_autoreset():
    import torch

    _, meta = load_set("torus_continue")
    B = 300
    env = make_env(meta, 5, batch=B)
    orc = oracle(meta, 5, B)
    rng = np.random.RandomState(3)
    for t in range(60):
        if t % 20 == 10:
            mask = (rng.random_sample(B) < 0.3).astype(np.uint8)
            env.reset_environment(torch.as_tensor(mask))
            orc.reset(mask)
        acts = rng.randint(-128, 128, size=(B, env.N)).astype(np.int8)
        ob, rw, dn, info = env.step(torch.as_tensor(acts))
        r_o, rw_o, d_o, wr_o = orc.step(acts, nthreads=8)
        assert np.array_equal(ob.cpu().numpy(), r_o), t
        assert np.array_equal(rw.cpu().numpy(), rw_o), t
        assert not info["world_reset"].any()
    s, so = env.state(), orc.state()
    for key in so:
        assert np.array_equal(s[key], so[key]), key


def test_torus_shard_invariance():
    """Results depend on the world id only: worlds [64, 128) of a 192-world batch equal a
    64-world batch based at 64."""
    import torch

    _, meta = load_set("torus_c3")
    a = make_env(meta, 0, batch=192)
    b = make_env(meta, 64, batch=64)
    a.reset_environment()
    b.reset_environment()
    rng = np.random.RandomState(11)
    acts = rng.randint(0, 5, size=(40, 192, a.N)).astype(np.int8)
    oa = a.rollout(torch.as_tensor(acts))[0].cpu().numpy()
    ob = b.rollout(torch.as_tensor(acts[:, 64:128].copy()))[0].cpu().numpy()
    assert np.array_equal(oa[:, 64:128], ob)


def test_torus_decoded_obs_matches_reference_frame():
    """frame() decodes a record into the reference's rows and internal obs (golden)."""
    import torch

    from wab_gym_amd.torus import decode_record

    d, meta = load_set("torus_multi")
    env = make_env(meta, meta["world_ids"][0])
    env.reset_environment()
    obs, _, _, _ = env.step(torch.as_tensor(d["actions"][0, 0][None]))
    for i in range(env.N):
        rows, internal = env.frame(obs[0, i])
        assert [rows, internal] == decode_record(d["records"][0, 0, i], env.types, env.num_bushes)
        assert internal[:2] == [int(v) for v in d["reset0_obj_xy"][0, i]]


@pytest.mark.parametrize("name", ["torus_multi", "torus_tiny"])
def test_torus_per_entity_calls_match_reference_golden(name):
    """get_obs(i) then take_action(i, a) for every entity, the reference's own loop
    (Env2Tests.py:40-88), in every world at once: the golden records, rewards, dones and resets."""
    import torch

    d, meta = load_set(name)
    ids = meta["world_ids"]
    T = min(meta["T"], 60)
    envs = [make_env(meta, g) for g in ids]
    for env in envs:
        env.reset_environment()
    N = envs[0].N
    for t in range(T):
        for i in range(N):
            for e, env in enumerate(envs):
                rec = env.get_obs(i)[0].cpu().numpy()
                assert np.array_equal(rec, d["records"][t, e, i]), "%s world %d turn %d entity %d" % (name, ids[e], t, i)
                r, dn, info = env.take_action(i, torch.as_tensor(d["actions"][t, e, i:i + 1]))
                assert float(r[0]) == d["reward"][t, e, i] and bool(dn[0]) == d["done"][t, e, i]
                if i == N - 1:
                    assert bool(info["world_reset"][0]) == bool(d["world_reset"][t, e])
    for e, env in enumerate(envs):
        check_state(env, d, T - 1, e, "%s world %d after %d turns of per-entity calls" % (name, ids[e], T))


def test_torus_per_entity_order_is_enforced():
    import torch

    _, meta = load_set("torus_c3")
    env = make_env(meta, 0, batch=128)
    env.reset_environment()
    a = torch.zeros(128, dtype=torch.int8)
    with pytest.raises(ValueError):
        env.take_action(1, a)  # entity 0 acts first
    env.get_obs(3)  # not acted yet: allowed
    env.take_action(0, a)
    with pytest.raises(ValueError):
        env.get_obs(0)  # acted this turn
    with pytest.raises(ValueError):
        env.step(torch.zeros((128, env.N), dtype=torch.int8))  # a turn is half done
    env.reset_environment()  # restarts the turn
    env.step(torch.zeros((128, env.N), dtype=torch.int8))


def test_torus_per_entity_equals_turn_launch_at_scale():
    """N get_obs + take_action launches per turn == one wab2_step launch, at B = 65536."""
    import torch

    _, meta = load_set("torus_c3")
    B = 65536
    a_env = make_env(meta, 0, batch=B)
    b_env = make_env(meta, 0, batch=B)
    a_env.reset_environment()
    b_env.reset_environment()
    rng = np.random.RandomState(5)
    hi = np.array([6] + [5] * 8 + [1] * 16)
    for t in range(12):
        acts = torch.as_tensor((rng.randint(0, 1 << 20, size=(B, 25)) % hi).astype(np.int8), device="cuda:0")
        obs, rew, done, info = a_env.step(acts)
        for i in range(25):
            rec = b_env.get_obs(i)
            assert torch.equal(rec, obs[:, i]), (t, i)
            r, dn, inf = b_env.take_action(i, acts[:, i].contiguous())
            assert torch.equal(r, rew[:, i]) and torch.equal(dn, done[:, i]), (t, i)
        assert torch.equal(inf["world_reset"], info["world_reset"]), t
    sa, sb = a_env.state(), b_env.state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k


def test_torus_rejects_bad_options():
    from wab_gym_amd.torus import BatchedWABEnvironment2

    for kw in ({"num_ostriches": 9}, {"num_wolves": 30}, {"world_width": 128},
               {"game_options": {"starting_role": 2}}, {"game_options": {"food_per_bush": 300}},
               {"game_options": {"lookout_view_radius": 4.5}}):
        with pytest.raises(ValueError):
            BatchedWABEnvironment2(num_worlds=64, device="cuda:0", **kw)


def _kat_env(W, H, counts, radius, positions):
    from wab_gym_amd.torus import BatchedWABEnvironment2

    opts = {"lookout_view_radius": radius, "gatherer_view_radius": radius}
    return BatchedWABEnvironment2(W, H, opts, *counts, num_worlds=3, device="cuda:0",
                                  spawn_positions=np.array(positions, np.int32))


def test_torus_world_tests_no_wrap_kat_on_gpu():
    """`Environment 2.0/World_tests.py:5-45` through the HIP kernel: a 20x20 world with the
    test's six entities at the test's positions (wab2_create_at; ids in this surface's
    ostrich, wolves, bushes order), the ostrich at (10, 10) looking with radius 8 sees all six at
    the test's deltas, bushes with their 20 food."""
    # ostrich (10, 10); wolves (5, 5), (15, 15); bushes (10, 5), (10, 10), (15, 10)
    env = _kat_env(20, 20, (1, 2, 3), 8, [(10, 10), (5, 5), (15, 15), (10, 5), (10, 10), (15, 10)])
    rec = env.get_obs(0)
    for b in range(3):
        rows, internal = env.frame(rec[b])
        got = sorted((typ, dx, dy, tuple(extra)) for _, dx, dy, typ, extra in rows)
        want = sorted([("Wolf", -5, -5, ()), ("Bush", 0, -5, (20,)), ("Ostrich", 0, 0, ()),
                       ("Bush", 0, 0, (20,)), ("Bush", 5, 0, (20,)), ("Wolf", 5, 5, ())])
        assert got == want, (b, rows)
        assert internal[:2] == [10, 10]


def test_torus_world_tests_wrap_kat_on_gpu():
    """`World_tests.py:49-88` through the HIP kernel: the other ostrich (id 0 here) takes action 0
    from (15, 15) to (15, 16) (wab2_take_action), then the ostrich at (19, 10) looking with
    radius 10 (id 1) sees the wolf at x = 5 through the wrap (Delta_X 6) and the rows the
    reference computes: the test's five plus the moved ostrich at (-4, 6) (World.py returns six
    rows where the test asserts five: tests/test_torus_oracle.py)."""
    import torch

    # ostriches (15, 15) [the mover], (19, 10) [the observer]; wolves (5, 5), (15, 15);
    # bushes (10, 10), (15, 10)
    env = _kat_env(20, 20, (2, 2, 2), 10, [(15, 15), (19, 10), (5, 5), (15, 15), (10, 10), (15, 10)])
    env.take_action(0, torch.zeros(3, dtype=torch.int8))
    rec = env.get_obs(1)
    for b in range(3):
        rows, internal = env.frame(rec[b])
        got = sorted((typ, dx, dy, tuple(extra)) for _, dx, dy, typ, extra in rows)
        want = sorted([("Wolf", 6, -5, ()), ("Ostrich", 0, 0, ()), ("Bush", -9, 0, (20,)),
                       ("Bush", -4, 0, (20,)), ("Wolf", -4, 5, ()), ("Ostrich", -4, 6, ())])
        assert got == want, (b, rows)
    assert env.state()["obj_xy"][0, 0].tolist() == [15, 16]


def test_torus_explicit_positions_lockstep_vs_oracle():
    """wab2_create_at / wab2_reset_at (explicit positions, a quarter of them negative = the
    keyed random draw, reset positions on the far edges x = W, y = H too) at B = 4096, 1/8/16, against
    the oracle given the same positions: full and masked resets, 60 turns, every record."""
    import torch

    from oracle.torus_oracle import OracleTorus
    from wab_gym_amd.torus import BatchedWABEnvironment2

    B, W, H, N = 4096, 32, 32, 25
    rng = np.random.RandomState(11)
    create = np.stack([rng.randint(W, size=(B, N)), rng.randint(H, size=(B, N))], -1).astype(np.int32)
    create[rng.random_sample((B, N)) < 0.25] = -1
    env = BatchedWABEnvironment2(W, H, None, 1, 8, 16, num_worlds=B, device="cuda:0", spawn_positions=create)
    orc = OracleTorus(W, H, 1, 8, 16, batch=B, spawn_positions=create)
    assert np.array_equal(env.state()["df_xy"], orc.state()["df_xy"])
    hi = np.array([6] + [5] * 8 + [1] * 16)
    for t in range(60):
        if t % 20 == 0:
            pos = np.stack([rng.randint(W + 1, size=(B, N)), rng.randint(H + 1, size=(B, N))], -1)
            pos[rng.random_sample((B, N)) < 0.25] = (-1, 5)
            mask = None if t == 0 else (rng.random_sample(B) < 0.5).astype(np.uint8)
            env.reset_environment(mask=mask, positions=pos.astype(np.int32))
            orc.reset(mask=mask, positions=pos.astype(np.int32))
            s_g, s_o = env.state(), orc.state()
            for k in ("obj_xy", "df_xy", "food", "episode"):
                assert np.array_equal(s_g[k], s_o[k]), (t, k)
        a = (rng.randint(0, 1 << 20, size=(B, N)) % hi).astype(np.int8)
        obs, rew, done, info = env.step(torch.as_tensor(a))
        r_o, rw_o, d_o, wr_o = orc.step(a, nthreads=8)
        assert np.array_equal(obs.cpu().numpy(), r_o), t
        assert np.array_equal(rew.cpu().numpy(), rw_o), t
        assert np.array_equal(info["world_reset"].cpu().numpy(), wr_o.astype(bool)), t
    with pytest.raises(Exception):
        BatchedWABEnvironment2(W, H, None, 1, 8, 16, num_worlds=2, device="cuda:0",
                               spawn_positions=np.full((N, 2), W, np.int32))  # x = W is not a tile
    with pytest.raises(Exception):
        env.reset_environment(positions=np.full((N, 2), W + 1, np.int64))  # past randint(0, W)
