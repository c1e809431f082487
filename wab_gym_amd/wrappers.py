"""Batched observation wrappers and the actor-critic return scan (config 5).

`PragmaticObsWrapper` mirrors the reference wrapper (wab_env.py:670-824) for a batched env:
`observation(obs)` turns the batched 7-tuple into the wrapper's 11-tuple already flattened
the way actor_critic.py feeds the policy (`gym.spaces.flatten`, actor_critic.py:188), i.e. a
float32 tensor [B, 449] computed on device by one HIP kernel (wab_featurize).
`SuperBasicObservationWrapper` (wab_env.py:900-927) does the same for its 4-tuple
(nearest bush, food, role, status): float32 [B, 90] (wab_featurize_superbasic).
"""
from __future__ import annotations

import ctypes
import warnings

from . import _lib
from .spaces import Box, Discrete, Tuple


class PragmaticObsWrapper:
    def __init__(self, env):
        self.env = env
        lib = _lib.load()
        F = lib.wab_feature_dim(env._h)
        if F < 0:
            raise ValueError("PragmaticObsWrapper cannot index a %dx%d viewport (wab_env.py:742)"
                             % (env.W, env.H))
        self.feature_dim = int(F)
        opts = env.game_options
        self.max_distance = opts["width"] // 2 + opts["height"] // 2 + 1  # wab_env.py:709
        md = self.max_distance
        self.single_observation_space = Tuple((                          # wab_env.py:710-724
            Tuple([Discrete(md + 1)] * 4), Tuple([Discrete(md + 1)] * 4), Tuple([Discrete(11)] * 4),
            Tuple([Discrete(md + 1)] * 4), Tuple([Discrete(md + 1)] * 4), Tuple([Discrete(11)] * 4),
            Discrete(2), Discrete(opts["turns_to_empty_food"] + 1), Discrete(2), Discrete(3),
            Box(0, 1, (121,))))
        self.observation_space = Box(0.0, 1.0, (env.num_envs, self.feature_dim), dtype="float32")
        self.action_space = env.action_space
        self.spec = env.spec
        t = env._torch
        self.features = t.zeros((env.num_envs, self.feature_dim), dtype=t.float32, device=env.device)

    def __getattr__(self, name):
        return getattr(self.env, name)

    def observation(self, obs=None, view_mask=None, out=None):
        """Features of the env's current observation buffer (or of `obs`, a dict with
        planes [B,3,W,S] and scalars [3,B] u8 tensors).  Returns float32 [B, F] (a view
        of `out` or of a wrapper-owned buffer overwritten by the next call)."""
        env = self.env
        t = env._torch
        if obs is None:
            env._require_planes()
            st = env._obs["struct"]
            keep = None
        else:
            st, keep = env._obs_struct(obs)
        vm = None
        if view_mask is not None:
            vm = t.as_tensor(view_mask, device=env.device).to(t.uint8).contiguous()
        dst = self.features if out is None else out
        env._check_features(dst, self.feature_dim)
        _lib.check(_lib.load().wab_featurize(env._h, ctypes.addressof(st),
                                             None if vm is None else vm.data_ptr(), dst.data_ptr(),
                                             env._stream()), "wab_featurize")
        del keep
        return dst

    def reset(self, mask=None):
        self.env.reset(mask)
        return self.observation()

    def rollout(self, actions, gamma=0.99, bootstrap=None):
        """T steps of this wrapper with the actions [T, B] and the discounted returns of the
        segment (actor_critic.py:139-143, 185-200): (features [T,B,F], reward [T,B], done [T,B],
        returns [T,B]), one kernel launch where the fused path applies (env.rollout_features)."""
        if type(self) is not PragmaticObsWrapper:
            raise NotImplementedError("rollout() fuses PragmaticObsWrapper only")
        r = self.env.rollout_features(actions, gamma=gamma, bootstrap=bootstrap)
        if r["features"].shape[0] > 0:
            self.features.copy_(r["features"][-1])  # as after T step() calls
        return r["features"], r["reward"], r["done"].view(self.env._torch.bool), r["returns"]

    def step(self, actions):
        if self.env._term is None and type(self) is PragmaticObsWrapper:
            # one kernel: the step and the features of its obs (wab_step_features)
            f, reward, done = self.env.step_features(actions, self.features)
            return f, reward, done, {}
        _, reward, done, info = self.env.step(actions)
        if "terminal_obs" in info:
            t = self.env._term
            info["terminal_features"] = self.observation(
                {"planes": t["planes"], "scalars": t["scalars"]},
                out=self.env._torch.empty_like(self.features))
        return self.observation(), reward, done, info


class SuperBasicObservationWrapper(PragmaticObsWrapper):
    """SuperBasicObservationWrapper (wab_env.py:900-927): (nearest bush, food, role, status),
    flattened by gym's rules (nearest bush 4 x Discrete(max_distance), :906)."""

    def __init__(self, env):
        self.env = env
        lib = _lib.load()
        self.feature_dim = int(lib.wab_superbasic_dim(env._h))
        opts = env.game_options
        self.max_distance = opts["width"] // 2 + opts["height"] // 2 + 1  # wab_env.py:903
        md = self.max_distance
        self.single_observation_space = Tuple((                          # wab_env.py:904-911
            Tuple([Discrete(md)] * 4), Discrete(opts["turns_to_empty_food"] + 1), Discrete(2), Discrete(3)))
        self.observation_space = Box(0.0, 1.0, (env.num_envs, self.feature_dim), dtype="float32")
        self.action_space = env.action_space
        self.spec = env.spec
        t = env._torch
        self.features = t.zeros((env.num_envs, self.feature_dim), dtype=t.float32, device=env.device)

    def observation(self, obs=None, view_mask=None, out=None):
        """Features of the env's current observation buffer (or of `obs`, as in
        PragmaticObsWrapper.observation; the view mask is not part of this wrapper)."""
        env = self.env
        if obs is None:
            env._require_planes()
            st = env._obs["struct"]
            keep = None
        else:
            st, keep = env._obs_struct(obs)
        dst = self.features if out is None else out
        env._check_features(dst, self.feature_dim)
        _lib.check(_lib.load().wab_featurize_superbasic(env._h, ctypes.addressof(st), dst.data_ptr(),
                                                        env._stream()), "wab_featurize_superbasic")
        del keep
        return dst


def discounted_returns(reward, done, gamma=0.99, bootstrap=None, out=None, env=None):
    """R_t = r_t + gamma * R_{t+1}, restarted after each done (actor_critic.py:139-143),
    over [T, B] device tensors; one HIP kernel, double accumulation, float32 out.  With `env`
    (the env whose steps returned `reward`) each float32 reward is first mapped back to the
    exact double the reference's step() returns, so the result is float32 of finish_episode's
    own double returns bit for bit (wab_discounted_returns_exact)."""
    import torch

    r = reward.to(torch.float32).contiguous()
    d = done.to(torch.uint8).contiguous()
    T, B = r.shape
    if d.shape != (T, B):
        raise ValueError("done must have the shape of reward [T, B]")
    o = torch.empty_like(r) if out is None else out
    if o.shape != (T, B) or o.dtype != torch.float32 or not o.is_contiguous():
        raise ValueError("out must be a contiguous float32 tensor of shape [T, B]")
    bs = None if bootstrap is None else bootstrap.to(torch.float32).contiguous()
    stream = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
    L = _lib.load()
    args = (r.data_ptr(), d.data_ptr(), T, B, float(gamma), None if bs is None else bs.data_ptr(), o.data_ptr(),
            stream)
    if env is not None:
        if r.device != env.device:
            raise ValueError("reward is on %s, the env on %s" % (r.device, env.device))
        try:
            _lib.check(L.wab_discounted_returns_exact(env._h, *args), "wab_discounted_returns_exact")
            return o
        except ValueError as e:
            if "round to the same" not in str(e):
                raise
            # two of the options' rewards are one float32: the doubles are not recoverable
            warnings.warn("discounted_returns(env=...): %s; using the float32 rewards" % e)
    _lib.check(L.wab_discounted_returns(*args), "wab_discounted_returns")
    return o


def normalize_episode_returns(returns, done, eps=1.1920928955078125e-07):
    """(R - mean) / (std + eps) per episode segment of every env, as finish_episode does per
    episode (actor_critic.py:145-146; torch.std is unbiased; eps = float32 machine eps).
    Segments still open at the end of the rollout are normalised as they stand.  Two-pass
    segment statistics with scatter_add (trainer-side plumbing, not the env hot path)."""
    import torch

    T, B = returns.shape
    d = done.to(torch.int64)
    seg = torch.cumsum(d, 0) - d                           # dones strictly before t
    key = (torch.arange(B, device=returns.device).unsqueeze(0) * (T + 1) + seg).flatten()
    x = returns.to(torch.float64).flatten()
    n = torch.zeros(B * (T + 1), dtype=torch.float64, device=returns.device)
    cnt = n.clone().scatter_add_(0, key, torch.ones_like(x))
    mean = n.clone().scatter_add_(0, key, x) / cnt.clamp(min=1)
    dev = x - mean[key]
    var = n.clone().scatter_add_(0, key, dev * dev) / (cnt - 1)
    std = torch.sqrt(var)[key]
    return ((x - mean[key]) / (std + eps)).to(returns.dtype).reshape(T, B)
