"""Monitor-style episode statistics for a batched env.

The reference wraps its env in gym 0.17's `gym.wrappers.Monitor` (actor_critic.py:46,
wab_env.py:1013), whose stats recorder sums each episode's rewards as Python floats in step
order (starting from the int 0) and counts its steps, and on close writes
`openaigym.episode_batch.<infix>.stats.json` with `initial_reset_timestamp`, `timestamps`,
`episode_lengths`, `episode_rewards` and `episode_types`.  gym is not installed here, so the
file layout is a restatement of gym 0.17's stats recorder (parity unpinned); the episode sums
themselves are pinned bit for bit against sums of the reference's own double rewards in the
golden vectors (tests/test_monitor.py).

Videos follow gym 0.17's Monitor for one env of the batch (`video_env`, default 0): episode
k of that env is recorded when `video_callable(k)` (default: gym's capped cubic schedule, k
in 0, 1, 8, 27, ... 729, then every 1000th), one frame after its reset and one after every
step, the terminal observation included (when the env was made with return_terminal=True;
the autoreset env's obs on a done step is already the next episode's).  Frames come from
`env.render(envs=(video_env, 1))` on device.  There is no ffmpeg or imageio in this image, so
a video is an animated GIF (PIL) at the env's `video.frames_per_second` instead of gym's
mp4, with gym's `<base>.meta.json` beside it.  The monitor reads that env's done flag on the
host (one synchronisation per step) only while the env's current or a soon-starting episode
is scheduled; otherwise episodes are counted on device and read at the stats flushes.

The device reward is the reference's double reward rounded to float32 (include/wab.h).  Each
step's double is recovered exactly from the few values a step can produce, `r_x` or
`r_eat + r_x` for r_x in (per turn, finishing, starving, killed) (wab_env.py:299-340), then
summed in float64 on device.  Finished episodes are gathered every `flush_every` steps (one
host synchronisation), so the per-step path stays asynchronous.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

_REWARD_KEYS = ("reward_per_turn", "reward_for_finishing", "reward_for_starving", "reward_for_being_killed")


def reward_table(game_options):
    """[(float32 value, exact double)] of every reward a step can return (wab_env.py:299-340):
    `0 + r_x` without an eat, `0 + r_eat + r_x` with one."""
    r_eat = game_options["reward_for_eating"]
    pairs = {}
    for k in _REWARD_KEYS:
        rx = game_options[k]
        for d in (0 + rx, 0 + r_eat + rx):
            d = float(d)
            f = float(np.float32(d))
            if f in pairs and pairs[f] != d:
                raise ValueError("rewards %r and %r round to the same float32: the double sum is "
                                 "not recoverable from the device reward" % (pairs[f], d))
            pairs[f] = d
    return sorted(pairs.items())


class EpisodeStats:
    """Per-env episode return (float64) and length on device; finished episodes are gathered
    into host lists in (step, env) order by flush()."""

    def __init__(self, game_options, num_envs, device, flush_every=32):
        import torch

        self._torch = torch
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.flush_every = int(flush_every)
        tab = reward_table(game_options)
        self._f32 = torch.tensor([f for f, _ in tab], dtype=torch.float32, device=self.device)
        self._f64 = torch.tensor([d for _, d in tab], dtype=torch.float64, device=self.device)
        B, K = self.num_envs, self.flush_every
        self.ret = torch.zeros(B, dtype=torch.float64, device=self.device)
        self.length = torch.zeros(B, dtype=torch.int64, device=self.device)
        self._buf_ret = torch.zeros((K, B), dtype=torch.float64, device=self.device)
        self._buf_len = torch.zeros((K, B), dtype=torch.int64, device=self.device)
        self._times = []
        self.episode_rewards, self.episode_lengths, self.episode_envs = [], [], []
        self.timestamps, self.episode_types = [], []
        self.total_steps = 0

    def restart(self, mask=None):
        """Start new episodes (all envs, or those with mask[i]); unfinished ones are dropped."""
        if mask is None:
            self.ret.zero_()
            self.length.zero_()
        else:
            m = self._torch.as_tensor(mask, device=self.device).bool()
            self.ret.masked_fill_(m, 0.0)
            self.length.masked_fill_(m, 0)

    def decode(self, reward):
        """float32 device rewards -> the reference's doubles."""
        r = reward.to(self._torch.float32)
        hit = r.unsqueeze(1) == self._f32.unsqueeze(0)  # [B, n_values]
        exact = (hit.to(self._torch.float64) * self._f64.unsqueeze(0)).sum(1)
        return self._torch.where(hit.any(1), exact, r.to(self._torch.float64))

    def update(self, reward, done):
        """One step of every env: add the step's reward, count it, close the done episodes."""
        t = self._torch
        d = t.as_tensor(done, device=self.device).bool()
        self.ret += self.decode(t.as_tensor(reward, device=self.device))
        self.length += 1
        k = len(self._times)
        self._buf_ret[k].copy_(self.ret)
        self._buf_len[k].copy_(t.where(d, self.length, t.zeros_like(self.length)))
        self._times.append(time.time())
        self.ret.masked_fill_(d, 0.0)
        self.length.masked_fill_(d, 0)
        self.total_steps += self.num_envs
        if len(self._times) == self.flush_every:
            self.flush()

    def flush(self):
        """Gather the episodes finished since the last flush (synchronises)."""
        k = len(self._times)
        if k == 0:
            return
        lens = self._buf_len[:k].cpu().numpy()
        rets = self._buf_ret[:k].cpu().numpy()
        steps, envs = np.nonzero(lens)
        self.episode_rewards.extend(float(x) for x in rets[steps, envs])
        self.episode_lengths.extend(int(x) for x in lens[steps, envs])
        self.episode_envs.extend(int(x) for x in envs)
        self.timestamps.extend(self._times[s] for s in steps)
        self.episode_types.extend("t" for _ in steps)
        self._times = []


def capped_cubic_video_schedule(episode_id):
    """gym 0.17 monitor.capped_cubic_video_schedule: episodes 0, 1, 8, 27, ..., 729, then
    every 1000th."""
    if episode_id < 1000:
        return int(round(episode_id ** (1.0 / 3))) ** 3 == episode_id
    return episode_id % 1000 == 0


class GifRecorder:
    """gym's VideoRecorder for rgb_array frames, as an animated GIF (no ffmpeg here):
    `<base>.gif` and `<base>.meta.json`; an episode closed with no frames writes only the
    metadata, marked empty."""

    def __init__(self, base_path, metadata, fps, enabled=True):
        self.path = base_path + ".gif"
        self.metadata_path = base_path + ".meta.json"
        self.metadata = dict(metadata)
        self.fps = fps
        self.enabled = enabled
        self.frames = []

    def capture_frame(self, frame):
        if self.enabled:
            self.frames.append(np.asarray(frame, dtype=np.uint8))

    @property
    def functional(self):
        return self.enabled and bool(self.frames)

    def close(self):
        if not self.enabled:
            return
        if self.frames:
            from PIL import Image

            ims = [Image.fromarray(f) for f in self.frames]
            ims[0].save(self.path, save_all=True, append_images=ims[1:], duration=int(round(1000.0 / self.fps)),
                        loop=0)
            import PIL

            self.metadata.update(content_type="image/gif", encoder_version={"backend": "PIL", "version": PIL.__version__},
                                 frames=len(self.frames))
        else:
            self.metadata["empty"] = True
        with open(self.metadata_path, "w") as f:
            json.dump(self.metadata, f)


class EpisodeMonitor:
    """`gym.wrappers.Monitor(env, directory, video_callable, force)` for a batched env: episode
    statistics of every env, video of env `video_env`'s scheduled episodes (module
    docstring).  video_callable=False records none.  Attributes of the wrapped env pass
    through."""

    def __init__(self, env, directory=None, force=False, flush_every=32, monitor_id=0, video_callable=None,
                 video_env=0, video_scale=32):
        self.env = env
        self.stats = EpisodeStats(env.game_options, env.num_envs, env.device, flush_every)
        self.directory = directory
        self.initial_reset_timestamp = None
        self._infix = "%d.%d" % (monitor_id, os.getpid())
        self.video_callable = capped_cubic_video_schedule if video_callable is None else video_callable
        self.video_env = int(video_env)
        self.video_scale = int(video_scale)
        self._video_on = (directory is not None and self.video_callable is not False
                          and hasattr(env, "render") and 0 <= self.video_env < env.num_envs)
        self.episode_id = 0  # episodes of video_env started (gym's Monitor.episode_id)
        self.videos = []
        self._rec = None
        self._ep_dev = None  # video_env's episode ends since the last count (device, unarmed)
        self._unsynced = 0
        if directory is not None:
            os.makedirs(directory, exist_ok=True)
            if force:
                for f in os.listdir(directory):
                    if f.startswith("openaigym."):
                        os.remove(os.path.join(directory, f))

    def __getattr__(self, name):
        return getattr(self.env, name)

    def reset(self, mask=None):
        obs = self.env.reset(mask)
        if self.initial_reset_timestamp is None:
            self.initial_reset_timestamp = time.time()
        self.stats.restart(mask)
        if self._video_on and (mask is None or bool(np.asarray(self._host(mask))[self.video_env])):
            self._sync_episode_count()
            self._new_episode()
        return obs

    def step(self, actions):
        obs, reward, done, info = self.env.step(actions)
        if self._video_on:
            self._video_step(done)
        self.stats.update(reward, done)
        return obs, reward, done, info

    # ------------------------------------------------------------------ video
    def _host(self, x):
        return x.cpu().numpy() if hasattr(x, "cpu") else x

    def _frame(self, obs=None):
        img = self.env.render(scale=self.video_scale, obs=obs, envs=(self.video_env, 1))
        return self._host(img[0])

    def _armed(self):
        """True when video_env's done flag must be read every step: its current episode is
        being recorded, or one of the next flush_every + 1 may be (an episode lasts >= 1 step,
        and the device count is read every flush_every unarmed steps)."""
        if self._rec is not None and self._rec.enabled:
            return True
        return any(self.video_callable(self.episode_id + k) for k in range(self.stats.flush_every + 1))

    def _sync_episode_count(self):
        """Fold the device-counted episode ends (unarmed steps) into episode_id."""
        if self._ep_dev is not None:
            n = int(self._ep_dev.item())
            self._ep_dev = None
            self._unsynced = 0
            for _ in range(n):  # (each ended episode started the next one, unrecorded)
                self._close_recorder()
                self.episode_id += 1

    def _new_episode(self):
        """gym's reset_video_recorder + episode_id bump: a recorder for the episode that
        starts now, its first frame captured."""
        self._close_recorder()
        base = os.path.join(self.directory, "openaigym.video.%s.video%06d" % (self._infix, self.episode_id))
        fps = getattr(self.env, "metadata", {}).get("video.frames_per_second", 30)
        self._rec = GifRecorder(base, {"episode_id": self.episode_id}, fps,
                                enabled=bool(self.video_callable(self.episode_id)))
        if self._rec.enabled:
            self._rec.capture_frame(self._frame())
        self.episode_id += 1

    def _close_recorder(self):
        if self._rec is not None:
            self._rec.close()
            if self._rec.functional:
                self.videos.append((self._rec.path, self._rec.metadata_path))
            self._rec = None

    def _video_step(self, done):
        t = self.stats._torch
        d_e = t.as_tensor(done, device=self.stats.device)[self.video_env]
        if not self._armed():
            if self._ep_dev is None:
                self._ep_dev = t.zeros((), dtype=t.int64, device=self.stats.device)
            self._ep_dev += d_e.to(t.int64)
            self._unsynced += 1
            if self._unsynced == self.stats.flush_every:  # (with the stats' own flush, normally)
                self._sync_episode_count()
            return
        self._sync_episode_count()
        if bool(d_e):
            if self._rec is not None and self._rec.enabled:
                term = getattr(self.env, "terminal_observation", None)
                if term is not None:
                    self._rec.capture_frame(self._frame(obs=term))
            self._new_episode()  # (the autoreset obs is the new episode's first)
        elif self._rec is not None and self._rec.enabled:
            self._rec.capture_frame(self._frame())

    def get_episode_rewards(self):
        self.stats.flush()
        return list(self.stats.episode_rewards)

    def get_episode_lengths(self):
        self.stats.flush()
        return list(self.stats.episode_lengths)

    def get_total_steps(self):
        return self.stats.total_steps

    def write_stats(self):
        """The stats file of gym 0.17's stats recorder (+ a manifest naming it)."""
        self.stats.flush()
        if self.directory is None:
            return None
        s = self.stats
        path = os.path.join(self.directory, "openaigym.episode_batch.%s.stats.json" % self._infix)
        with open(path, "w") as f:
            json.dump({"initial_reset_timestamp": self.initial_reset_timestamp,
                       "timestamps": s.timestamps, "episode_lengths": s.episode_lengths,
                       "episode_rewards": s.episode_rewards, "episode_types": s.episode_types}, f)
        spec = getattr(self.env, "spec", None)
        with open(os.path.join(self.directory, "openaigym.manifest.%s.manifest.json" % self._infix), "w") as f:
            json.dump({"stats": os.path.basename(path),
                       "videos": [(os.path.basename(v), os.path.basename(m)) for v, m in self.videos],
                       "env_info": {"env_id": getattr(spec, "id", None), "gym_version": "0.17.2 (restated)"}}, f)
        return path

    def close(self):
        self._close_recorder()
        path = self.write_stats()
        self.env.close()
        return path
