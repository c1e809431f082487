"""Monitor-style episode statistics (wab_gym_amd.monitor): episode returns and lengths equal the
sums gym's stats recorder would form from the reference's own double rewards (golden vectors),
bit for bit, although the device hands out float32 rewards."""
import json

import numpy as np
import pytest

import golden_replay as gr
from backends import SEED

AUTORESET_SETS = [n for n in gr.SETS if n != "continue"]


def reference_episodes(g):
    """gym 0.17 StatsRecorder over each golden env: rewards summed as Python numbers from the
    int 0 in step order, one episode per done; (step, env) order."""
    reward, done = g["reward"], g["done"]
    T, n = reward.shape
    acc = [0] * n
    steps = [0] * n
    out = []
    for t in range(T):
        for e in range(n):
            acc[e] += float(reward[t, e])
            steps[e] += 1
            if done[t, e]:
                out.append((float(acc[e]), steps[e], e))
                acc[e], steps[e] = 0, 0
    return out


def _opts(g):
    from wab_gym_amd.options import default_game_options

    o = dict(default_game_options)
    o.update(g["meta"]["options"])
    return o


@pytest.mark.parametrize("name", AUTORESET_SETS)
def test_episode_sums_match_reference_doubles(name):
    from wab_gym_amd.monitor import EpisodeStats

    g = gr.load(name)
    T, n = g["reward"].shape
    st = EpisodeStats(_opts(g), n, "cpu", flush_every=7)
    for t in range(T):
        st.update(g["reward"][t].astype(np.float32), g["done"][t])
    st.flush()
    want = reference_episodes(g)
    assert len(want) > 0
    got = list(zip(st.episode_rewards, st.episode_lengths, st.episode_envs))
    assert got == want  # float == float: bit for bit


def test_reward_table_covers_every_golden_reward():
    from wab_gym_amd.monitor import reward_table

    for name in AUTORESET_SETS + ["continue"]:
        g = gr.load(name)
        doubles = {d for _, d in reward_table(_opts(g))}
        assert set(np.unique(g["reward"]).tolist()) <= doubles, name


def test_reward_table_rejects_ambiguous_rewards():
    from wab_gym_amd.monitor import reward_table
    from wab_gym_amd.options import default_game_options

    o = dict(default_game_options)
    o["reward_for_eating"] = 1e-12  # r_x and r_eat + r_x round to the same float32
    o["reward_per_turn"] = 0.3
    with pytest.raises(ValueError):
        reward_table(o)


class _GoldenEnv:
    """a stand-in env that replays a golden set's rewards and dones (CPU)"""

    def __init__(self, g):
        import torch

        from wab_gym_amd.spaces import DummySpec

        self.g, self.t = g, 0
        self.game_options = _opts(g)
        self.num_envs = g["reward"].shape[1]
        self.device = torch.device("cpu")
        self.spec = DummySpec(id="WolvesAndBushes-v0", max_episode_steps=80, reward_threshold=80)
        self._torch = torch

    def reset(self, mask=None):
        return None

    def step(self, actions):
        t, self.t = self.t, self.t + 1
        return (None, self._torch.as_tensor(self.g["reward"][t].astype(np.float32)),
                self._torch.as_tensor(self.g["done"][t]), {})

    def close(self):
        pass


def test_monitor_writes_gym_stats_files(tmp_path):
    from wab_gym_amd.monitor import EpisodeMonitor

    g = gr.load("default")
    env = EpisodeMonitor(_GoldenEnv(g), directory=str(tmp_path), force=True, flush_every=16)
    env.reset()
    for _ in range(g["reward"].shape[0]):
        env.step(None)
    path = env.close()
    d = json.load(open(path))
    assert set(d) == {"initial_reset_timestamp", "timestamps", "episode_lengths", "episode_rewards",
                      "episode_types"}
    want = reference_episodes(g)
    assert d["episode_rewards"] == [w[0] for w in want]
    assert d["episode_lengths"] == [w[1] for w in want]
    assert len(d["timestamps"]) == len(want) and set(d["episode_types"]) == {"t"}
    man = [p for p in tmp_path.iterdir() if p.name.endswith(".manifest.json")]
    assert len(man) == 1 and json.load(open(man[0]))["stats"] == tmp_path.joinpath(path).name
    assert env.get_total_steps() == g["reward"].size


@pytest.mark.gpu
def test_monitor_over_device_env_matches_reference_episodes():
    """The device env replaying the golden actions, through EpisodeMonitor: the episodes gym's
    Monitor records from the reference's double rewards."""
    import torch

    from wab_gym_amd.env import BatchedWolvesAndBushesEnv
    from wab_gym_amd.monitor import EpisodeMonitor

    for name in ("default", "neither6", "restrict"):
        g = gr.load(name)
        for e0, base, n in gr.groups(g["meta"]["env_ids"]):  # runs of consecutive env ids
            sl = slice(e0, e0 + n)
            env = EpisodeMonitor(BatchedWolvesAndBushesEnv(g["meta"]["options"], num_envs=n, seed=SEED,
                                                           device="cuda:0", env_id_base=base, wolf_slots=32),
                                 flush_every=9)
            env.reset()
            for t in range(g["reward"].shape[0]):
                env.step(torch.as_tensor(g["actions"][t, sl], device="cuda:0"))
            got = list(zip(env.get_episode_rewards(), env.get_episode_lengths(), env.stats.episode_envs))
            assert got == reference_episodes({"reward": g["reward"][:, sl], "done": g["done"][:, sl]}), (name, base)


class _FrameEnv:
    """a CPU stand-in with scripted dones whose render() frames name the step they show
    (value t after step t, 100 + t for the terminal observation of step t)"""

    metadata = {"video.frames_per_second": 12}

    def __init__(self, done, return_terminal=True):
        import torch

        self._torch = torch
        self.done = np.asarray(done, dtype=bool)  # [T, B]
        self.num_envs = self.done.shape[1]
        from wab_gym_amd.options import default_game_options

        self.game_options = dict(default_game_options)
        self.device = torch.device("cpu")
        self.t = 0
        self._rt = return_terminal

    @property
    def terminal_observation(self):
        return "term" if self._rt else None

    def reset(self, mask=None):
        return None

    def step(self, actions):
        self.t += 1
        t = self._torch
        return None, t.zeros(self.num_envs, dtype=t.float32), t.as_tensor(self.done[self.t - 1]), {}

    def render(self, scale=32, obs=None, envs=None):
        v = self.t if obs is None else 100 + self.t
        assert envs == (0, 1) and scale == 2
        return self._torch.full((1, 3, 5, 3), v, dtype=self._torch.uint8)

    def close(self):
        pass


def _gym_video_frames(done0, schedule, return_terminal=True):
    """gym 0.17 Monitor's recorded frames per episode id for one env, restated: a recorder per
    reset (frame of the start), a frame after every step (the terminal observation's on the
    done step), a new recorder when an episode ends (the env resets itself)."""
    out, ep, frames = {}, 0, [0]
    for t, d in enumerate(done0, start=1):
        if d:
            if return_terminal:
                frames.append(100 + t)
            if schedule(ep):
                out[ep] = frames
            ep, frames = ep + 1, [t]
        else:
            frames.append(t)
    if schedule(ep):
        out[ep] = frames
    return out


def _read_gif(path):
    from PIL import Image, ImageSequence

    with Image.open(path) as im:
        return [int(np.asarray(f.convert("RGB"))[0, 0, 0]) for f in ImageSequence.Iterator(im)]


@pytest.mark.parametrize("pattern", ["every_step", "mixed", "no_terminal"])
def test_monitor_video_schedule_and_frames(tmp_path, pattern):
    from wab_gym_amd.monitor import EpisodeMonitor, capped_cubic_video_schedule

    assert [k for k in range(2001) if capped_cubic_video_schedule(k)] == [k ** 3 for k in range(10)] + [1000, 2000]
    rng = np.random.default_rng(3)
    T, B = 90, 3
    if pattern == "every_step":  # 90 one-step episodes of env 0: 0, 1, 8, 27, 64 recorded
        done = np.ones((T, B), dtype=bool)
    else:
        done = rng.random((T, B)) < 0.3
    rt = pattern != "no_terminal"
    env = EpisodeMonitor(_FrameEnv(done, return_terminal=rt), directory=str(tmp_path), force=True, flush_every=4,
                         video_scale=2)
    env.reset()
    for _ in range(T):
        env.step(None)
    env.close()
    want = _gym_video_frames(done[:, 0], capped_cubic_video_schedule, rt)
    got = {}
    for v, m in env.videos:
        meta = json.load(open(m))
        got[meta["episode_id"]] = _read_gif(v)
        assert meta["frames"] == len(got[meta["episode_id"]]) and meta["content_type"] == "image/gif"
    assert got == want
    man = [p for p in tmp_path.iterdir() if p.name.endswith(".manifest.json")]
    assert len(json.load(open(man[0]))["videos"]) == len(want)


def test_monitor_video_off(tmp_path):
    from wab_gym_amd.monitor import EpisodeMonitor

    env = EpisodeMonitor(_FrameEnv(np.ones((5, 2), dtype=bool)), directory=str(tmp_path), video_callable=False,
                         video_scale=2)
    env.reset()
    for _ in range(5):
        env.step(None)
    env.close()
    assert env.videos == [] and not [p for p in tmp_path.iterdir() if p.name.endswith(".gif")]


@pytest.mark.gpu
def test_monitor_video_over_device_env(tmp_path):
    """EpisodeMonitor's GIFs over the device env: each frame equals render() of env 0 at that
    point (the terminal frame: of the step's own observation), per gym's schedule."""
    import torch
    from PIL import Image, ImageSequence

    from wab_gym_amd.env import BatchedWolvesAndBushesEnv
    from wab_gym_amd.monitor import EpisodeMonitor

    B, T, scale = 64, 300, 4
    opts = {"max_turns": 20}
    acts = torch.randint(0, 5, (T, B), generator=torch.Generator().manual_seed(5)).to("cuda:0")
    ref = BatchedWolvesAndBushesEnv(opts, num_envs=B, seed=SEED, device="cuda:0", return_terminal=True)
    ref.reset()
    full = ref.render(scale=scale)
    one = ref.render(scale=scale, envs=(0, 1))
    assert torch.equal(full[:1], one) and torch.equal(full[5:7], ref.render(scale=scale, envs=(5, 2)))
    with pytest.raises(ValueError):
        ref.render(scale=scale, envs=(B - 1, 2))
    frames, dones = [one[0].cpu().numpy()], []
    for t in range(T):
        _, _, d, _ = ref.step(acts[t])
        dones.append(bool(d[0]))
        frames.append((ref.render(scale=scale, envs=(0, 1))[0].cpu().numpy(),
                       ref.render(scale=scale, obs=ref.terminal_observation, envs=(0, 1))[0].cpu().numpy()))
    env = EpisodeMonitor(BatchedWolvesAndBushesEnv(opts, num_envs=B, seed=SEED, device="cuda:0", return_terminal=True),
                         directory=str(tmp_path), flush_every=4, video_scale=scale)
    env.reset()
    for t in range(T):
        env.step(acts[t])
    env.close()
    want, ep, cur = {}, 0, [frames[0]]
    for t, d in enumerate(dones, start=1):
        if d:
            cur.append(frames[t][1])
            want[ep], ep, cur = cur, ep + 1, [frames[t][0]]
        else:
            cur.append(frames[t][0])
    assert sum(dones) >= 9  # episodes 0, 1 and 8 closed
    got = {}
    for v, m in env.videos:
        meta = json.load(open(m))
        fr = []
        with Image.open(v) as im:  # (PIL merges identical consecutive frames, adding their durations)
            for f in ImageSequence.Iterator(im):
                fr += [np.asarray(f.convert("RGB"))] * int(round(f.info["duration"] / (1000 / 12)))
        assert len(fr) == meta["frames"]
        got[meta["episode_id"]] = fr
    assert sorted(got) == [k for k in (0, 1, 8, 27, 64) if k < ep or k == ep]
    for k, fr in got.items():
        exp = want.get(k, cur)
        assert len(fr) == len(exp) and all(np.array_equal(a, b) for a, b in zip(fr, exp)), k
