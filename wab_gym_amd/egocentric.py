"""Egocentric env variants, batched: `WolvesAndBushesEnvEgoCentric` and
`WolvesAndBushesEnvEgocentricJustBushes` (wab_env.py:930-979).

Same dynamics as `BatchedWolvesAndBushesEnv`; the observation is replaced by the bush
proximities of `_get_bush_proximities` (wab_env.py:652-667), computed on device by
`wab_egocentric` (include/wab.h): for the squares reached by up, right, down, left, stay,
clip(max_distance - d, 0, max_distance) with d the taxicab distance to the nearest food>0
bush among all tiles seen this episode; max_distance when there is none.

    EgoCentric obs:   (proximity [B,5] u8, food_turns [B] u8, role [B] u8, status [B] u8)
    JustBushes obs:    proximity [B,5] u8

The proximities depend on the whole episode's path, so every reset and step goes through
this class (no fused `rollout`).  With `autoreset=True` a done env is reset after its
terminal proximities are taken: `info["terminal_obs"]` (when `return_terminal=True`) holds
the step's own observation and the returned obs the new episode's first one, as for the
base env.  The `_get_wolf_proximities` result that the reference computes and discards
(:939) is not computed.
"""
from __future__ import annotations

from . import _lib
from .env import BatchedWolvesAndBushesEnv
from .spaces import Box, Discrete, Tuple


class BatchedWolvesAndBushesEnvEgoCentric(BatchedWolvesAndBushesEnv):
    def __init__(self, game_options=None, num_envs=4096, seed=0x5EED, device="cuda", env_id_base=0,
                 autoreset=True, return_terminal=False, **kw):
        # the handle never resets by itself: the terminal proximities need the terminal state
        super().__init__(game_options, num_envs=num_envs, seed=seed, device=device,
                         env_id_base=env_id_base, autoreset=False, return_terminal=False, **kw)
        self.autoreset = bool(autoreset)
        self.return_terminal = bool(return_terminal)
        t = self._torch
        o = self.game_options
        self.max_distance = o["width"] // 2 + o["height"] // 2 + 1  # wab_env.py:933-935
        if self.max_distance > 31:
            raise ValueError("egocentric observation needs width//2 + height//2 <= 30")
        B, md = self.num_envs, self.max_distance
        self.proximity = t.zeros((B, 5), dtype=t.uint8, device=self.device)
        self._set_spaces(o, B, md)

    def _set_spaces(self, o, B, md):
        self.single_observation_space = Tuple((                   # wab_env.py:936-948
            Tuple([Discrete(md + 1)] * 5), Discrete(o["turns_to_empty_food"] + 1), Discrete(2),
            Discrete(3)))
        self.observation_space = Tuple((
            Box(0, md, (B, 5)), Box(0, o["turns_to_empty_food"], (B,)), Box(0, 1, (B,)), Box(0, 2, (B,))))

    def _observe(self, mask=None):
        m = None if mask is None else mask.data_ptr()
        _lib.check(_lib.load().wab_egocentric(self._h, m, self.proximity.data_ptr(), self._stream()),
                   "wab_egocentric")

    def _ego_obs(self, prox=None, scal=None):
        prox = self.proximity if prox is None else prox
        scal = self._obs["scalars"] if scal is None else scal
        return (prox, scal[0], scal[1], scal[2])

    def reset(self, mask=None):
        super().reset(mask)
        self._observe(None if mask is None else self._reset_mask_keepalive)
        return self._ego_obs()

    def step(self, actions):
        _, reward, done, _ = super().step(actions)
        self._observe()
        info = {}
        if self.autoreset:
            if self.return_terminal:
                info["terminal_obs"] = self._ego_obs(self.proximity.clone(), self._obs["scalars"].clone())
            BatchedWolvesAndBushesEnv.reset(self, self.done)
            self._observe(self._reset_mask_keepalive)
        return self._ego_obs(), reward, done, info

    def rollout(self, actions):
        raise NotImplementedError("the egocentric observation is computed per step; use step()")


class BatchedWolvesAndBushesEnvEgocentricJustBushes(BatchedWolvesAndBushesEnvEgoCentric):
    """Observation = the 5 bush proximities only; action_space Discrete(5) (wab_env.py:963-964)."""

    def _set_spaces(self, o, B, md):
        self.single_observation_space = Tuple([Discrete(md + 1)] * 5)  # wab_env.py:959-961
        self.observation_space = Box(0, md, (B, 5))
        self.action_space = Discrete(5)

    def _ego_obs(self, prox=None, scal=None):
        return self.proximity if prox is None else prox


__all__ = ["BatchedWolvesAndBushesEnvEgoCentric", "BatchedWolvesAndBushesEnvEgocentricJustBushes"]
