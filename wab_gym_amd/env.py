"""BatchedWolvesAndBushesEnv — the reference's gym surface with a leading batch dimension.

Mirrors `WolvesAndBushesEnv` (wab_env.py:103-342): same constructor options
(`game_options`, validated like wab_env.py:147-148), `reset()`, `step(actions)` ->
`(obs, reward, done, info)`, `action_space`, `observation_space`, `spec`.  Every call
advances `num_envs` independent envs at once through one fused HIP kernel (C-ABI in
include/wab.h).  Buffers are PyTorch-ROCm tensors on the env's device.

Observation: the reference's 7-tuple (wab_env.py:374-385) batched:
    (wolf_grid [B,W,H] u8, bush_grid [B,W,H] u8, ostrich_grid [B,W,H] u8,
     food_turns [B] u8, role [B] u8, alive_starved_killed [B] u8, view_mask [B,11,11] u8)
The grids are views into an env-owned buffer that the next call overwrites (clone to keep).

Differences from the reference, by design (documented in DESIGN.md):
  * random draws are keyed by (seed, env id, episode, what is drawn) instead of numpy's
    global MT19937 stream, so batches are reproducible and shard-invariant;
  * with `autoreset=True` (default) an env whose step returns done=True is reset inside
    the same call; `obs` then holds the new episode's first observation and
    `info["terminal_obs"]` (if `return_terminal=True`) the step's own observation;
  * an action outside [0, n_actions) raises IndexError from the call that received it
    (the reference raises for a >= n via `.iloc` and silently wraps negatives,
    wab_env.py:253).  Host actions are checked before their copy; device actions with one
    synchronising reduction per call (validate_actions=True, the default, = "sync").
    validate_actions="deferred" (opt-in, for throughput) skips that synchronisation: the
    kernel applies out-of-range actions as no-ops and counts them, and the IndexError comes
    from the next synchronising call -- counters(), state(), check() -- or the next reset();
    the data that call read is attached to the exception (`err.result`).
  * the kernel's LDS hand-off between its waves is bounded (wab_device.h lds_await); a
    timed-out hand-off means results computed from unpublished data, so a non-zero
    `handoff_timeouts` count raises WabError from counters(), state() and check().
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .options import default_game_options, make_config, n_actions, view_masks
from .spaces import Box, Discrete, DummySpec, Tuple


class BatchedWolvesAndBushesEnv:
    metadata = {"render.modes": ["rgb_array"], "video.frames_per_second": 12}

    def __init__(self, game_options=None, num_envs=4096, seed=0x5EED, device="cuda",
                 env_id_base=0, autoreset=True, return_terminal=False, plane_stride=0,
                 wolf_slots=0, eaten_capacity=0, validate_actions=True, obs_placement="same"):
        import torch

        self._torch = torch
        lib = _lib.load()
        opts = dict(default_game_options if game_options is None else game_options)
        for k, v in default_game_options.items():
            opts.setdefault(k, v)
        self.game_options = opts
        self.cfg, self._keep = make_config(opts, autoreset=autoreset, plane_stride=plane_stride,
                                           eaten_capacity=eaten_capacity, wolf_slots=wolf_slots)
        self.num_envs = int(num_envs)
        self.base_seed = int(seed)
        self.env_id_base = int(env_id_base)
        self.autoreset = bool(autoreset)
        self.return_terminal = bool(return_terminal)
        if validate_actions not in (True, False, "sync", "deferred"):
            raise ValueError("validate_actions must be True/'sync', 'deferred' or False")
        self.validate_actions = "sync" if validate_actions is True else validate_actions
        self._bad_seen = 0  # bad_actions already reported (deferred validation)
        self._handoff_seen = 0  # handoff_timeouts already reported
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("BatchedWolvesAndBushesEnv runs on a HIP device (device='cuda[:i]')")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.W, self.H = self.cfg.width, self.cfg.height
        self.S = plane_stride or self.H
        h = ctypes.c_void_p()
        _lib.check(lib.wab_create(ctypes.addressof(self.cfg), self.num_envs, self.base_seed,
                                  self.env_id_base, dev.index, ctypes.byref(h)), "wab_create")
        self._h = h
        # which per-step build the wide (C3) kernel runs (wab_set_obs_placement, include/wab.h):
        # "same" = every step into one buffer (the env's own: the per-step kernel), "fresh" = a
        # closed loop stepping into a ring of buffers (step(actions, obs=...)): whole-line stores
        if obs_placement not in ("same", "fresh"):
            raise ValueError("obs_placement must be 'same' or 'fresh'")
        self.obs_placement = obs_placement
        _lib.check(lib.wab_set_obs_placement(h, _lib.OBS_FRESH_BUFFER if obs_placement == "fresh"
                                             else _lib.OBS_SAME_BUFFER), "wab_set_obs_placement")
        B = self.num_envs
        u8 = dict(dtype=torch.uint8, device=dev)
        self._obs = self._alloc_obs()
        self._term = self._alloc_obs() if self.return_terminal else None
        self.reward = torch.zeros(B, dtype=torch.float32, device=dev)
        self.done = torch.zeros(B, **u8)
        self._actions = torch.zeros(B, dtype=torch.int8, device=dev)
        self._masks = torch.as_tensor(view_masks(opts), device=dev)
        self._zero_mask = torch.zeros((11, 11), **u8)
        self._reset_once = False
        self._planes_valid = True  # False while the obs planes buffer is stale (planes not stored)
        self.n_actions = n_actions(opts)
        self.action_space = Discrete(self.n_actions)  # wab_env.py:188-191
        W, H = self.W, self.H
        self.single_observation_space = Tuple((        # wab_env.py:193-229
            Box(0, 1, (W, H)), Box(0, 1, (W, H)), Box(0, 1, (W, H)),
            Discrete(opts["turns_to_empty_food"] + 1), Discrete(2), Discrete(3)))
        self.observation_space = Tuple((
            Box(0, 1, (B, W, H)), Box(0, 1, (B, W, H)), Box(0, 1, (B, W, H)),
            Box(0, opts["turns_to_empty_food"], (B,)), Box(0, 1, (B,)), Box(0, 2, (B,))))
        self.spec = DummySpec(id="WolvesAndBushes-v0", max_episode_steps=opts["max_turns"],
                              reward_threshold=80)  # wab_env.py:140-146

    # ------------------------------------------------------------------ buffers
    def alloc_obs(self):
        """A new observation buffer (dict of planes [B,3,W,S] and scalars [3,B] u8) for
        step(actions, obs=...), e.g. the slots of a closed loop's ring of observations."""
        o = self._alloc_obs()
        return {"planes": o["planes"], "scalars": o["scalars"]}

    def _alloc_obs(self):
        t = self._torch
        B = self.num_envs
        planes = t.zeros((B, 3, self.W, self.S), dtype=t.uint8, device=self.device)
        scal = t.zeros((3, B), dtype=t.uint8, device=self.device)
        st = _lib.WabObs(planes.data_ptr(), scal[0].data_ptr(), scal[1].data_ptr(), scal[2].data_ptr())
        return {"planes": planes, "scalars": scal, "struct": st}

    def _obs_struct(self, obs):
        """WabObs over a caller's observation dict (planes [B,3,W,S] and scalars [3,B] u8 on
        this env's device), checked before any pointer reaches a kernel: a wrong dtype,
        device or batch would be an out-of-bounds device read.  Returns (struct, keepalive)."""
        t = self._torch
        planes, scal = obs["planes"], obs["scalars"]
        want = (self.num_envs, 3, self.W, self.S)
        for name, x, shape in (("planes", planes, want), ("scalars", scal, (3, self.num_envs))):
            if (not isinstance(x, t.Tensor) or x.dtype != t.uint8 or x.device != self.device
                    or tuple(x.shape) != shape):
                raise ValueError("obs['%s'] must be a uint8 tensor of shape %s on %s"
                                 % (name, shape, self.device))
        planes, scal = planes.contiguous(), scal.contiguous()
        st = _lib.WabObs(planes.data_ptr(), scal[0].data_ptr(), scal[1].data_ptr(), scal[2].data_ptr())
        return st, (planes, scal)

    def _obs_tuple(self, o):
        planes, scal = o["planes"], o["scalars"]
        H = self.H
        grids = [planes[:, k, :, :H] for k in range(3)]
        if self.game_options["restrict_view"]:
            vm = self._masks[scal[1].long()]
        else:
            vm = self._zero_mask.expand(self.num_envs, 11, 11)
        return (grids[0], grids[1], grids[2], scal[0], scal[1], scal[2], vm)

    def _stream(self):
        return ctypes.c_void_p(self._torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ gym surface
    def reset(self, mask=None):
        """Reset all envs (mask=None) or those with mask[i] true; returns the batched obs."""
        t = self._torch
        m = None
        if self.validate_actions == "deferred" and self._reset_once and mask is None:
            # a deferred out-of-range action must not disappear behind the new episodes (this
            # reads the device counters: a synchronisation, on full resets only; a masked reset
            # leaves the check to the next counters()/state()/check())
            self._raise_pending(self._read_counters(), None)
        if mask is not None:
            if not self._reset_once:
                raise RuntimeError("the first reset must cover every env (mask=None)")
            m = t.as_tensor(mask, device=self.device).to(t.uint8).contiguous()
            if m.shape != (self.num_envs,):
                raise ValueError("mask must have shape [num_envs]")
        _lib.check(_lib.load().wab_reset(self._h, None if m is None else m.data_ptr(),
                                         ctypes.addressof(self._obs["struct"]), self._stream()),
                   "wab_reset")
        self._reset_mask_keepalive = m
        self._reset_once = True
        if m is None:
            self._planes_valid = True
        return self._obs_tuple(self._obs)

    def _step_actions(self, actions):
        t = self._torch
        if not self._reset_once:
            raise RuntimeError("call reset() before step()")
        if not isinstance(actions, t.Tensor):
            # host actions: checked on the host before the copy (no device synchronisation)
            import numpy as np

            h = np.asarray(actions)
            if h.shape != (self.num_envs,):
                raise ValueError("actions must have shape [num_envs]")
            if self.validate_actions and h.size and (h.min() < 0 or h.max() >= self.n_actions):
                raise IndexError("action out of range [0, %d)" % self.n_actions)
            if h.dtype != np.int8:  # out-of-range values stay out of range in int8
                h = np.clip(h, -1, 127)
            a = t.as_tensor(h.astype(np.int8, copy=False), device=self.device)
        else:
            a = actions.to(self.device)
            if a.shape != (self.num_envs,):
                raise ValueError("actions must have shape [num_envs]")
            # device actions: "sync" (the default) checks here with one blocking reduction
            # per step; "deferred" lets the kernel count them (applied as no-ops) and raises
            # at the next synchronising call
            self._sync_action_check(a)
        if a.dtype != t.int8:
            # narrowing must not wrap an out-of-range value into a valid one (256 -> 0)
            self._actions.copy_(a.clamp(-1, 127) if not a.is_floating_point() else a.clamp(-1.0, 127.0))
            a = self._actions
        else:
            a = a.contiguous()
        return a

    def _check_features(self, features, F):
        t = self._torch
        if (not isinstance(features, t.Tensor) or features.dtype != t.float32 or features.device != self.device
                or tuple(features.shape) != (self.num_envs, F) or not features.is_contiguous()):
            raise ValueError("features must be a contiguous float32 tensor of shape (%d, %d) on %s"
                             % (self.num_envs, F, self.device))

    def _sync_action_check(self, a):
        if self.validate_actions == "sync" and a.numel() and bool(((a < 0) | (a >= self.n_actions)).any()):
            raise IndexError("action out of range [0, %d)" % self.n_actions)

    def _raise_pending(self, c, result):
        """Raise what the device counters report since the last check: a WabError for
        timed-out LDS hand-offs (the step then computed from unpublished data), an IndexError
        for out-of-range device actions stepped under validate_actions="deferred" (applied as
        no-ops).  `result` (the data the calling method read) rides on the exception."""
        hand = c["handoff_timeouts"] - self._handoff_seen
        self._handoff_seen = c["handoff_timeouts"]
        bad = c["bad_actions"] - self._bad_seen
        self._bad_seen = c["bad_actions"]
        err = None
        if hand > 0:
            err = _lib.WabError("%d LDS hand-off(s) timed out in the step kernel since the last check: "
                                "the affected steps are not reference results" % hand)
        elif self.validate_actions and bad > 0:
            err = IndexError("%d action(s) out of range [0, %d) were stepped since the last check "
                             "(applied as no-ops)" % (bad, self.n_actions))
        if err is not None:
            err.result = result
            raise err

    def _read_counters(self):
        c = _lib.WabCounters()
        _lib.check(_lib.load().wab_get_counters(self._h, ctypes.addressof(c), self._stream()),
                   "wab_get_counters")
        return {k: int(getattr(c, k)) for k, _ in _lib.WabCounters._fields_}

    def check(self):
        """Synchronise; raise for timed-out hand-offs and deferred out-of-range actions."""
        self.counters()

    @property
    def terminal_observation(self):
        """The last step's own observation buffer (dict of planes and scalars, for render(obs=)),
        or None unless the env was made with return_terminal=True."""
        return self._term

    def step(self, actions, obs=None):
        """Advance every env one step (wab_env.py:250-342).  The returned obs, reward and done
        are views of the env's buffers, overwritten by the next step (clone to keep them).
        obs=<dict from alloc_obs()> writes the observation into that buffer instead (a closed
        loop keeping several steps' observations: construct with obs_placement="fresh"); the
        returned obs are views of it, and the env's own buffer is not updated (render() and the
        wrappers then need obs= too, until the next step()/reset() into the env's own)."""
        a = self._step_actions(actions)
        term = ctypes.addressof(self._term["struct"]) if self._term is not None else None
        if obs is None:
            st, keep, o = self._obs["struct"], None, self._obs
        else:
            if not (obs["planes"].is_contiguous() and obs["scalars"].is_contiguous()):
                raise ValueError("obs= buffers must be contiguous (the step writes them in place)")
            st, keep = self._obs_struct(obs)
            o = {"planes": keep[0], "scalars": keep[1]}
        _lib.check(_lib.load().wab_step(self._h, a.data_ptr(), ctypes.addressof(st),
                                        self.reward.data_ptr(), self.done.data_ptr(), term,
                                        self._stream()), "wab_step")
        self._planes_valid = obs is None
        info = {}
        if self._term is not None:
            info["terminal_obs"] = self._obs_tuple(self._term)
        return self._obs_tuple(o), self.reward, self.done.view(self._torch.bool), info

    def step_features(self, actions, features, store_planes=True):
        """step() fused with the PragmaticObsWrapper featurizer (wab_step_features): writes the
        features [B, F] float32 of the returned obs into `features`; reward, done and the obs
        scalars as step() does.  store_planes=False leaves the obs planes unwritten (the policy
        of actor_critic.py never sees them)."""
        a = self._step_actions(actions)
        self._check_features(features, int(_lib.load().wab_feature_dim(self._h)))
        o = self._obs["struct"]
        st = o if store_planes else _lib.WabObs(None, o.food_turns, o.role, o.status)
        _lib.check(_lib.load().wab_step_features(self._h, a.data_ptr(), ctypes.addressof(st),
                                                 self.reward.data_ptr(), self.done.data_ptr(),
                                                 features.data_ptr(), self._stream()),
                   "wab_step_features")
        self._planes_valid = bool(store_planes)
        return features, self.reward, self.done.view(self._torch.bool)

    def rollout(self, actions):
        """T fused steps: actions [T, B] -> (planes [T,B,3,W,S], scalars [T,3,B], reward [T,B],
        done [T,B]).  Equivalent to T step() calls without terminal observations: the env's
        scalars, reward and done show the last step afterwards, and so do its own obs planes
        (planes[T-1] is copied into them on the same stream, right after the launch, so every obs
        tuple reset()/step() returned is consistent).  terminal_observation is not updated (it
        keeps the last step()'s)."""
        t = self._torch
        a = t.as_tensor(actions, device=self.device)
        if a.dim() != 2 or a.shape[1] != self.num_envs:
            raise ValueError("actions must have shape [T, num_envs]")
        self._sync_action_check(a)
        if a.dtype != t.int8:
            a = a.clamp(-1, 127)
        a = a.to(t.int8).contiguous()
        T = a.shape[0]
        planes = t.empty((T, self.num_envs, 3, self.W, self.S), dtype=t.uint8, device=self.device)
        scal = t.empty((3, T, self.num_envs), dtype=t.uint8, device=self.device)
        rew = t.empty((T, self.num_envs), dtype=t.float32, device=self.device)
        done = t.empty((T, self.num_envs), dtype=t.uint8, device=self.device)
        o = _lib.WabObs(planes.data_ptr(), scal[0].data_ptr(), scal[1].data_ptr(), scal[2].data_ptr())
        _lib.check(_lib.load().wab_rollout(self._h, a.data_ptr(), T, ctypes.addressof(o),
                                           rew.data_ptr(), done.data_ptr(), self._stream()),
                   "wab_rollout")
        if T > 0:  # the env's buffers show the last step, as after T step() calls
            self._sync_last_step(scal[:, T - 1], rew[T - 1], done[T - 1])
            self._obs["planes"].copy_(planes[T - 1])
        return planes, scal.permute(1, 0, 2), rew, done

    def _sync_last_step(self, scal, rew, done):
        self._obs["scalars"].copy_(scal)
        self.reward.copy_(rew)
        self.done.copy_(done)
        self._planes_valid = True

    def rollout_features(self, actions, gamma=0.99, bootstrap=None, returns=True, store_planes=False,
                         features=None):
        """T steps of PragmaticObsWrapper(env).step with the actions [T, B] (the loop of
        actor_critic.main, actor_critic.py:185-200) and finish_episode's discounted returns of
        the segment (actor_critic.py:139-143; R after the last step = bootstrap [B] or 0), one
        launch where the fused small-view kernel applies (wab_rollout_features).  Returns a dict:
        features [T,B,F] f32, scalars [T,3,B], reward [T,B], done [T,B], returns [T,B] f32 (or
        None), planes [T,B,3,W,S] (or None unless store_planes).  Bit for bit T step_features()
        calls followed by discounted_returns(env=self)."""
        t = self._torch
        a = t.as_tensor(actions, device=self.device)
        if a.dim() != 2 or a.shape[1] != self.num_envs:
            raise ValueError("actions must have shape [T, num_envs]")
        self._sync_action_check(a)
        if a.dtype != t.int8:
            a = a.clamp(-1, 127)
        a = a.to(t.int8).contiguous()
        T, B = a.shape
        L = _lib.load()
        F = int(L.wab_feature_dim(self._h))
        if F < 0:
            raise ValueError("PragmaticObsWrapper cannot index this viewport")
        if features is None:
            features = t.empty((T, B, F), dtype=t.float32, device=self.device)
        elif (features.dtype != t.float32 or tuple(features.shape) != (T, B, F) or not features.is_contiguous()
              or features.device != self.device):
            raise ValueError("features must be a contiguous float32 tensor of shape (%d, %d, %d) on %s"
                             % (T, B, F, self.device))
        planes = (t.empty((T, B, 3, self.W, self.S), dtype=t.uint8, device=self.device) if store_planes
                  else None)
        scal = t.empty((3, T, B), dtype=t.uint8, device=self.device)
        rew = t.empty((T, B), dtype=t.float32, device=self.device)
        done = t.empty((T, B), dtype=t.uint8, device=self.device)
        ret = t.empty((T, B), dtype=t.float32, device=self.device) if returns else None
        bs = None
        if bootstrap is not None:
            bs = t.as_tensor(bootstrap, device=self.device).to(t.float32).contiguous()
            if bs.shape != (B,):
                raise ValueError("bootstrap must have shape [num_envs]")
        o = _lib.WabObs(None if planes is None else planes.data_ptr(), scal[0].data_ptr(), scal[1].data_ptr(),
                        scal[2].data_ptr())
        _lib.check(L.wab_rollout_features(self._h, a.data_ptr(), T, ctypes.addressof(o), rew.data_ptr(),
                                          done.data_ptr(), features.data_ptr(), float(gamma),
                                          None if bs is None else bs.data_ptr(),
                                          None if ret is None else ret.data_ptr(), self._stream()),
                   "wab_rollout_features")
        if T > 0:
            # the env's scalars, reward and done show the last step; its planes too when they
            # were stored -- otherwise they were never written (rendered on chip only) and the
            # env's obs planes are stale until the next step()/reset() (observation() and
            # render() of the env's own buffer then raise)
            self._sync_last_step(scal[:, T - 1], rew[T - 1], done[T - 1])
            if planes is not None:
                self._obs["planes"].copy_(planes[T - 1])
            else:
                self._planes_valid = False
        return {"features": features, "scalars": scal.permute(1, 0, 2), "reward": rew, "done": done,
                "returns": ret, "planes": planes}

    def render(self, mode="rgb_array", scale=32, draw_health=True, out=None, obs=None, envs=None):
        """render (wab_env.py:468-502) of every env's current observation (or of `obs`, a
        dict of planes [B,3,W,S] and scalars [3,B] u8 tensors) on device: u8 [B, W*scale,
        H*scale, 3].  draw_health (the reference's default) draws the turns-until-starve
        count in blue at (0, 0) with PIL's default font's digit glyphs (tools/make_glyphs.py;
        parity with the reference's pinned Pillow 7.2 font is unpinned).  envs=(first, count)
        renders only those envs: [count, W*scale, H*scale, 3]."""
        if mode != "rgb_array":
            raise NotImplementedError("only mode='rgb_array' (wab_env.py:104 metadata)")
        t = self._torch
        first, count = (0, self.num_envs) if envs is None else (int(envs[0]), int(envs[1]))
        if first < 0 or count < 0 or first + count > self.num_envs:
            raise ValueError("envs=(first, count) must lie in [0, %d)" % self.num_envs)
        shape = (count, self.W * scale, self.H * scale, 3)
        img = t.empty(shape, dtype=t.uint8, device=self.device) if out is None else out
        if tuple(img.shape) != shape or img.dtype != t.uint8 or not img.is_contiguous() or img.device != self.device:
            raise ValueError("out must be a contiguous uint8 tensor of shape %s on %s" % (shape, self.device))
        keep = None
        if obs is None:
            self._require_planes()
            st = self._obs["struct"]
        else:
            st, keep = self._obs_struct(obs)
        _lib.check(_lib.load().wab_render_envs(self._h, ctypes.addressof(st), first, count, int(scale),
                                               int(bool(draw_health)), img.data_ptr(), self._stream()),
                   "wab_render_envs")
        del keep
        return img

    def _require_planes(self):
        if not self._planes_valid:
            raise RuntimeError("the env's obs planes were not stored by the last call "
                               "(step_features/rollout_features with store_planes=False); pass obs= "
                               "or step()/reset() first")

    @property
    def step_kernel(self):
        """Which fused step kernel this handle launches: "small", "wide" or "block"."""
        return _lib.load().wab_step_kernel(self._h).decode()

    def counters(self):
        """The handle's cumulative counters (wab_counters).  Raises (counters attached as
        `err.result`) for hand-off timeouts and deferred out-of-range actions since the last
        check."""
        out = self._read_counters()
        self._raise_pending(out, out)
        return out

    def state(self):
        """Hidden per-env state (host numpy): food f64, x, y, turn, n_wolves, episode."""
        B = self.num_envs
        food = np.zeros(B, np.float64)
        x, y, turn, nw = (np.zeros(B, np.int32) for _ in range(4))
        ep = np.zeros(B, np.uint32)
        P = lambda a: a.ctypes.data  # noqa: E731
        _lib.check(_lib.load().wab_get_state(self._h, P(food), P(x), P(y), P(turn), P(nw), P(ep),
                                             self._stream()), "wab_get_state")
        out = dict(food=food, x=x, y=y, turn=turn, n_wolves=nw, episode=ep)
        self._raise_pending(self._read_counters(), out)
        return out

    def seed(self, seed=None):
        """No-op like gym 0.17's Env.seed in the reference (wab_env.py:1014); draws are keyed
        by the constructor's `seed`."""
        return [self.base_seed]

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().wab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
