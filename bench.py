"""Benchmark: batched Wolves-and-Bushes env-steps/s on MI355X (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config default|wide31|c5|torus]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one fused pass over all B envs of a rank: move, wolves, bushes, kill/eat/starve,
reward/done, auto-reset and the full observation render, with the inputs (actions,
pre-generated [W+K, B] int8 on device from torch.randint) resident in HBM.  The line times
64-step rollout launches (`wab_rollout`; C5 `wab_rollout_features` with the features and the
segment's returns), the steps' outputs into [64, B] buffers; the per-step launch (`wab_step`,
the gym `env.step` surface) is timed beside it (`rollout.per_step_launch`; `--rollout 0`
makes it the line).  Each rank
owns env ids [rank*B, (rank+1)*B) — independent shards, no collective on the data path
(weak scaling).  Timing: barrier + synchronize on both sides of exactly K steps, max over
ranks; value = N*B*K / that time.  Rank 0 prints one JSON line.

Steady state: whatever --warmup asks, at least 2 * max_turns steps run untimed after the
reset, so the timed window holds the auto-reset mix of the workload (random policy: ~2.4 % of
the envs finish an episode each step) rather than the first turns of the first episode.
N > 1: the barrier and the timing MAX go over a CPU (gloo) process group; RCCL is never
initialised (the shards exchange nothing).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "env-steps/sec (whole node) at batch=65536; obs bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (game options, plane_stride, wolf slots, description)
    "default": ({}, 0, 8, "batch=65536 envs x default options (11x11 viewport), random policy, autoreset"),
    # "8 wolves" (SURVEY.md A.5): the wide kernel keeps 8 wolves per env in registers; the
    # handle's 32 wolf rows let the rare 9th+ (ring spawns mid-episode: 14 in a 2000-step window
    # at 8 rows) live in HBM instead of being dropped
    "wide31": ({"width": 31, "height": 31}, 32, 32,
               "batch=65536 envs x 31x31 viewport in 32x32 planes (C3), random policy, autoreset"),
    # C5: T-step wab_rollout_features launches (the step fused with the PragmaticObsWrapper
    # features into a [T, B, 449] rollout buffer, reward/done into [T, B], the segment's
    # discounted returns at the launch's end); --rollout 0: one wab_step_features launch per step
    # and the returns scan (wab_discounted_returns_exact) every T steps (--c5-unfused: wab_step
    # then wab_featurize per step)
    "c5": ({}, 0, 8, "batch=65536 envs x default options, actor-critic rollout (C5): step + "
                     "PragmaticObsWrapper features + discounted returns of each %d-step segment "
                     "(episodes crossing a segment end are cut there, R_T = 0), random policy"),
}
# steps per rollout launch of every config's line, and C5's return segment (actor_critic.py
# collects one episode per update, <= max_turns = 80 steps).  Measured at B = 65536 on the
# default config: T = 16 6.55, 32 6.35, 64 6.20, 128 6.11-6.17 us per step (fewer launch
# boundaries: each costs the launch gap, step 0's state loads and the last step's tail)
C5_SEGMENT = 64
DEFAULT_ROLLOUT = 64
# the timed window's floor, whatever --steps asks: at least this many launches of the line's
# kernel in the captured graph, and graph replays until at least this many seconds are timed
# (a one-launch window, 0.4 ms, is at the mercy of one launch's jitter)
MIN_TIMED_LAUNCHES = 32
MIN_TIMED_SECONDS = 0.2


def window_steps(requested, steps_per_launch, min_launches=MIN_TIMED_LAUNCHES):
    """Steps captured in the timed graph: the requested count in whole launches (at least one),
    raised to `min_launches` launches."""
    per = max(1, int(steps_per_launch))
    k = max(per, int(requested) // per * per)
    return max(k, min_launches * per)


def window_replays(graph_seconds, min_seconds=MIN_TIMED_SECONDS, cap=10000):
    """Replays of the captured graph that make the timed window at least `min_seconds`, given
    one replay's measured duration."""
    import math

    if graph_seconds <= 0:
        return cap
    return max(1, min(cap, int(math.ceil(min_seconds / graph_seconds))))


def committed_traffic(config, batch):
    """HBM bytes per launch from the PMC summary committed under profiles/ for this
    workload (tools/profile.sh + tools/summarize_profile.py), or None."""
    path = os.path.join(REPO, "profiles", "traffic_%s_b%d.json" % (config, batch))
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    return d.get("hbm_bytes_per_launch", {}).get("total_corrected"), os.path.relpath(path, REPO)


def alg_bytes_per_env_step(W, H):
    """1 B action + 3*W*H u8 obs + 8 B scalars/reward/done + 2*36 B state."""
    return 3 * W * H + 81


def alg_bytes_per_env_step_rollout(W, H, T):
    """A T-step rollout launch: per env-step the action, obs, scalars, reward and done
    (3*W*H + 9 B); the 2*36 B of minimal state once per launch (read by the first step,
    written by the last), i.e. 72 / T per env-step."""
    return 3 * W * H + 9 + 72.0 / T


def c5_rollout_alg_bytes(F, T):
    """A T-step wab_rollout_features launch per env-step: action, obs scalars, reward, done
    (9 B), the F float32 features, the float32 return, and 72 / T of state (the planes are
    rendered on chip and not stored)."""
    return 9 + 4 * F + 4 + 72.0 / T


def featurize_alg_bytes(W, H, F):
    """wab_featurize per env: reads the 3*W*H obs bytes and 3 scalar bytes, writes F float32."""
    return 3 * W * H + 3 + 4 * F


# wab_discounted_returns per env-step: reads reward f32 + done u8, writes the f32 return
RETURNS_ALG_BYTES = 9

# The Environment 2.0 torus world (include/wab_torus.h): BASELINE config 3's
# literal reading.  A step is one turn of a world: every entity's get_obs() then take_action()
# (WAB_Environment2.py:120-134), in id order.
TORUS = {"width": 32, "height": 32, "counts": (1, 8, 16),
         "desc": "batch=65536 worlds x Environment 2.0 torus 32x32, 1 ostrich / 8 wolves / 16 bushes "
                 "(BASELINE config 3 read literally), uniform random actions (ostrich 0..5, wolf 0..4, "
                 "bush 0), autoreset (every ostrich done or 80 turns)"}


def torus_state_bytes(NO, NW, NB):
    """Per-world state of the torus kernel: own x, y i32 and frame X|Y u16 per entity, food f64
    per ostrich and wolf, food u8 per bush, the ostrich state byte, turn and episode."""
    N = NO + NW + NB
    return 10 * N + 8 * (NO + NW) + NB + NO + 8


def torus_alg_bytes(NO, NW, NB, T):
    """Per world-turn of a T-turn wab2_rollout launch: the N actions, N records of
    24 + 2N + NB bytes (padding to 16 not counted), reward f32 and done u8 per entity, the
    world_reset byte, and 2 x state / T."""
    N = NO + NW + NB
    return N + N * (24 + 2 * N + NB) + 5 * N + 1 + 2.0 * torus_state_bytes(NO, NW, NB) / T


def torus_actions(T, B, NO, NW, NB, dev, gen):
    """Uniform random actions [T, B, N] int8 on device: ostrich 0..5, wolf 0..4 (Env2Tests.py:27-36
    draws randint(0, 5) / randint(0, 4)), bush 0."""
    import torch

    N = NO + NW + NB
    hi = torch.tensor([6] * NO + [5] * NW + [1] * NB, dtype=torch.int32, device=dev)
    out = torch.empty((T, B, N), dtype=torch.int8, device=dev)
    for t0 in range(0, T, 16):
        t1 = min(T, t0 + 16)
        r = torch.randint(0, 1 << 30, (t1 - t0, B, N), device=dev, generator=gen, dtype=torch.int32)
        out[t0:t1] = (r % hi).to(torch.int8)
    return out


def finite(x):
    """The line with every non-finite float (a surface the run did not measure) as null, so
    it is strict JSON."""
    if isinstance(x, float) and not math.isfinite(x):
        return None
    if isinstance(x, dict):
        return {k: finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [finite(v) for v in x]
    return x


class ClockSampler:
    """The device's shader clock while a timed window runs, sampled every ~5 ms by a host thread
    from sysfs (hwmon freq1_input, else the current level of pp_dpm_sclk): the DVFS evidence
    beside each line (`sclk_mhz`: median, min, max, samples; None where sysfs has no clock)."""

    def __init__(self, pci):
        import glob

        base = "/sys/bus/pci/devices/%s.0" % pci
        self.hwmon = sorted(glob.glob(base + "/hwmon/hwmon*/freq1_input"))
        self.dpm = base + "/pp_dpm_sclk"
        self.last = None

    def read(self):
        try:
            if self.hwmon:
                return int(open(self.hwmon[0]).read()) / 1e6
            for ln in open(self.dpm):
                if ln.rstrip().endswith("*"):
                    return float(ln.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz"))
        except (OSError, ValueError, IndexError):
            return None
        return None

    def __enter__(self):
        import threading

        self.samples, self.stop = [], threading.Event()

        def loop():
            while not self.stop.wait(0.005):
                v = self.read()
                if v is not None:
                    self.samples.append(v)
        self.th = threading.Thread(target=loop, daemon=True)
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()
        v = sorted(self.samples)
        self.last = None if not v else {"median": v[len(v) // 2], "min": v[0], "max": v[-1], "samples": len(v)}
        return False


CLOCK = None  # a ClockSampler of the bench's device (main), read by time_launches


def time_launches(launch, n, dev, stream, mode="graph", min_seconds=MIN_TIMED_SECONDS, shards=1):
    """Average duration of one of `n` back-to-back launches (launch(i, hip_stream), or with
    shards > 1 launch(i, hip_stream, k) for every shard k, shard k's chain on its own stream
    forked from the launch stream and joined back after the n launches), captured in a graph as
    the timed region is, replayed until at least `min_seconds` are timed; HIP events on the
    launch stream.  Returns (ms per launch of the whole batch, launches timed)."""
    import torch

    subs = [torch.cuda.Stream(dev) for _ in range(shards - 1)]

    def launches(st):
        if shards == 1:
            sc = ctypes.c_void_p(st.cuda_stream)
            for i in range(n):
                launch(i, sc)
            return
        for sub in subs:
            sub.wait_stream(st)
        scs = [ctypes.c_void_p(x.cuda_stream) for x in [st] + subs]
        for i in range(n):
            for k in range(shards):
                launch(i, scs[k], k)
        for sub in subs:
            st.wait_stream(sub)
    g = None
    if mode == "graph":
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                launches(torch.cuda.current_stream(dev))
        stream.wait_stream(side)

    def once():
        if g is not None:
            g.replay()
        else:
            launches(stream)
    once()  # warm
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    once()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    reps = window_replays(e0.elapsed_time(e1) * 1e-3, min_seconds)
    import contextlib

    with CLOCK if CLOCK is not None else contextlib.nullcontext():
        e0.record(stream)
        for _ in range(reps):
            once()
        e1.record(stream)
        torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / (reps * n), reps * n


def torus_cpu_baseline(seconds, threads):
    """oracle/wab_torus_oracle.c (the scalar restatement of World.py's turn) on this host's
    cores, a bounded sample of the same workload."""
    import numpy as np

    from oracle.torus_oracle import OracleTorus

    NO, NW, NB = TORUS["counts"]
    Bc = 2048
    orc = OracleTorus(TORUS["width"], TORUS["height"], NO, NW, NB, batch=Bc)
    orc.reset()
    rng = np.random.RandomState(0)
    hi = np.array([6] * NO + [5] * NW + [1] * NB)
    acts = [(rng.randint(0, 1 << 30, size=(Bc, NO + NW + NB)) % hi).astype(np.int8) for _ in range(32)]
    orc.step(acts[0], nthreads=threads)
    n, t0 = 0, time.perf_counter()
    while True:
        orc.step(acts[n % 32], nthreads=threads)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(Bc * n / el, 1), "unit": "env-steps/s (world-turns)", "cores": threads, "kind": "port",
            "sample": "oracle/wab_torus_oracle.c turn, %d worlds x %d turns (%.1f s) of the same workload%s"
                      % (Bc, n, el, ", OpenMP over worlds" if threads > 1 else ", 1 thread")}


def roofline_entry(alg, us_per_step, B, traffic_key=None, kernel=None, steps_per_launch=1):
    """The roofline object of a `configs` entry: algorithmic bytes per env-step x B over the
    measured time per step, against the HBM peak; traffic from the committed PMC summary."""
    achieved = alg * B / (us_per_step * 1e-6) / 1e9
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "alg_bytes_per_env_step": round(alg, 3),
           "alg_bytes_per_launch": round(alg * B * steps_per_launch), "kernel": kernel}
    traffic, src = committed_traffic(traffic_key, B) if traffic_key else (None, None)
    out["traffic"] = None if traffic is None else round(traffic)
    out["traffic_unit"] = "bytes/launch (PMC 2*FETCH_SIZE + WRITE_SIZE, committed profile)"
    out["traffic_source"] = src
    return out


def extra_configs(args, dev, B):
    """The other BASELINE configs and surfaces, timed beside the headline on the same GPU (rank 0
    of a 1-GPU run): C3's wide rollout and its per-step launch into a 32-slot obs ring, C5's
    wab_rollout_features, the default per-step launch into a ring, and the Environment 2.0
    torus world.  Each: reset, >= 2 x max_turns untimed steps, then >= 32 launches and >= 0.2 s
    timed (time_launches)."""
    import torch

    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv
    from wab_gym_amd.torus import BatchedWABEnvironment2

    L = _lib.load()
    stream = torch.cuda.current_stream(dev)
    T = DEFAULT_ROLLOUT
    out = {}
    gen = torch.Generator(device=dev)
    gen.manual_seed(4321)
    NL = MIN_TIMED_LAUNCHES

    def entry(us, alg, key, kernel, spl, n, api):
        return {"api": api, "us_per_step": round(us, 3), "env_steps_per_s": round(B / (us * 1e-6), 1),
                "launches_timed": n, "steps_per_launch": spl,
                "roofline": roofline_entry(alg, us, B, key, kernel, spl),
                "sclk_mhz": CLOCK.last if CLOCK is not None else None}

    # the rollout entries as the main line runs them: the batch as S shards of Bs envs, each
    # shard's launches on its own stream (--stream-shards)
    S = args.stream_shards if args.stream_shards >= 1 and B % (64 * args.stream_shards) == 0 else 1
    Bs = B // S

    def shards_of(env, opts, stride, slots, acts):
        envs = [env] if S == 1 else [
            BatchedWolvesAndBushesEnv(opts, num_envs=Bs, seed=0x5EED, device=dev, env_id_base=k * Bs, autoreset=True,
                                      validate_actions=False, plane_stride=stride, wolf_slots=slots)
            for k in range(S)]
        if S > 1:
            for e in envs:
                e.reset()
        return envs, acts.view(-1, S, Bs).permute(1, 0, 2).contiguous()

    for cfg in ("wide31", "c5", "default"):
        opts, stride, slots, _ = CONFIGS[cfg]
        env = BatchedWolvesAndBushesEnv(opts, num_envs=B, seed=0x5EED, device=dev, autoreset=True,
                                        validate_actions=False, plane_stride=stride, wolf_slots=slots)
        h, W = env._h, 2 * int(env.game_options["max_turns"])
        W = -(-W // T) * T
        acts = torch.randint(0, env.n_actions, (W + NL * T, B), device=dev, generator=gen).to(torch.int8)
        a0 = acts.data_ptr()
        env.reset()
        if cfg == "c5":
            F = int(L.wab_feature_dim(h))
            envs, sacts = shards_of(env, opts, stride, slots, acts)
            bufs = []
            for k in range(S):
                sc = torch.empty((3, T, Bs), dtype=torch.uint8, device=dev)
                bufs.append((_lib.WabObs(None, sc[0].data_ptr(), sc[1].data_ptr(), sc[2].data_ptr()),
                             torch.empty((T, Bs), dtype=torch.float32, device=dev),
                             torch.empty((T, Bs), dtype=torch.uint8, device=dev),
                             torch.empty((T, Bs, F), dtype=torch.float32, device=dev),
                             torch.empty((T, Bs), dtype=torch.float32, device=dev), sc))

            def roll(t, s, k=0):
                rseq, rd, dn, feats, ret, _ = bufs[k]
                _lib.check(L.wab_rollout_features(envs[k]._h, sacts[k].data_ptr() + t * Bs, T, ctypes.addressof(rseq),
                                                  rd.data_ptr(), dn.data_ptr(), feats.data_ptr(), 0.99, None,
                                                  ret.data_ptr(), s), "wab_rollout_features")
            for t in range(0, W, T):
                for k in range(S):
                    roll(t, ctypes.c_void_p(stream.cuda_stream), k)
            ms, n = time_launches(lambda i, s, k=0: roll(W + i * T, s, k), NL, dev, stream, args.mode, shards=S)
            out["c5_rollout"] = entry(ms * 1e3 / T, c5_rollout_alg_bytes(F, T),
                                      "c5_rollout%d" % T + ("_s%d" % S if S > 1 else ""),
                                      "wab_step_small + features + returns, rollout build (wab_rollout_features)",
                                      T, n, "wab_rollout_features, %d steps per launch (C5: actor_critic.py:185-200)%s"
                                      % (T, ", the batch as %d shards of %d envs on %d streams" % (S, Bs, S)
                                         if S > 1 else ""))
            out["c5_rollout"]["stream_shards"] = S
            del bufs, envs
        else:
            pl = torch.empty((T, B, 3, env.W, env.S), dtype=torch.uint8, device=dev)
            sc = torch.empty((3, T, B), dtype=torch.uint8, device=dev)
            rd = torch.empty((T, B), dtype=torch.float32, device=dev)
            dn = torch.empty((T, B), dtype=torch.uint8, device=dev)
            seq = _lib.WabObs(pl.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), sc[2].data_ptr())

            def roll(t, s):
                _lib.check(L.wab_rollout(h, a0 + t * B, T, ctypes.addressof(seq), rd.data_ptr(), dn.data_ptr(), s),
                           "wab_rollout")
            for t in range(0, W, T):
                roll(t, ctypes.c_void_p(stream.cuda_stream))
            kname = "wab_step_%s" % L.wab_step_kernel(h).decode()
            if cfg == "wide31":
                del pl
                envs, sacts = shards_of(env, opts, stride, slots, acts)
                bufs = []
                for k in range(S):
                    pk = torch.empty((T, Bs, 3, env.W, env.S), dtype=torch.uint8, device=dev)
                    sk = torch.empty((3, T, Bs), dtype=torch.uint8, device=dev)
                    bufs.append((_lib.WabObs(pk.data_ptr(), sk[0].data_ptr(), sk[1].data_ptr(), sk[2].data_ptr()),
                                 torch.empty((T, Bs), dtype=torch.float32, device=dev),
                                 torch.empty((T, Bs), dtype=torch.uint8, device=dev), pk, sk))

                def sroll(t, s, k=0):
                    o, rdk, dnk, _, _ = bufs[k]
                    _lib.check(L.wab_rollout(envs[k]._h, sacts[k].data_ptr() + t * Bs, T, ctypes.addressof(o),
                                             rdk.data_ptr(), dnk.data_ptr(), s), "wab_rollout")
                if S > 1:
                    for t in range(0, W, T):
                        for k in range(S):
                            sroll(t, ctypes.c_void_p(stream.cuda_stream), k)
                ms, n = time_launches(lambda i, s, k=0: sroll(W + i * T, s, k), NL, dev, stream, args.mode, shards=S)
                out["wide31_rollout"] = entry(ms * 1e3 / T, alg_bytes_per_env_step_rollout(env.W, env.H, T),
                                              "wide31_rollout%d" % T + ("_s%d" % S if S > 1 else ""),
                                              kname + ", rollout build", T, n,
                                              "wab_rollout, %d steps per launch (C3: 31x31 in 32x32 planes)%s"
                                              % (T, ", the batch as %d shards of %d envs on %d streams" % (S, Bs, S)
                                                 if S > 1 else ""))
                out["wide31_rollout"]["stream_shards"] = S
                del bufs, envs
                pl = None
            # the per-step surface: one wab_step launch per step, step t's obs into slot t % 32
            # of a ring of [B] buffers (so they reach HBM as a closed loop's would)
            del pl
            NR = 32
            rp = torch.empty((NR, B, 3, env.W, env.S), dtype=torch.uint8, device=dev)
            rs = torch.empty((3, NR, B), dtype=torch.uint8, device=dev)
            rr = torch.empty((NR, B), dtype=torch.float32, device=dev)
            rdn = torch.empty((NR, B), dtype=torch.uint8, device=dev)
            slots_ = [_lib.WabObs(rp[i].data_ptr(), rs[0, i].data_ptr(), rs[1, i].data_ptr(), rs[2, i].data_ptr())
                      for i in range(NR)]
            _lib.check(L.wab_set_obs_placement(h, _lib.OBS_FRESH_BUFFER), "wab_set_obs_placement")
            ms, n = time_launches(lambda i, s: _lib.check(L.wab_step(h, a0 + (W + i % (NL * T)) * B,
                                                                     ctypes.addressof(slots_[i % NR]),
                                                                     rr[i % NR].data_ptr(), rdn[i % NR].data_ptr(),
                                                                     None, s), "wab_step"),
                                  256, dev, stream, args.mode)
            out["%s_per_step_ring" % cfg] = entry(
                ms * 1e3, alg_bytes_per_env_step(env.W, env.H), "%s_ring%d" % (cfg, NR), kname, 1, n,
                "wab_step (the raw C-ABI per-step launch), step t's obs into slot t %% %d of a ring of [B] "
                "buffers" % NR)
            del rp
        del env, acts
        torch.cuda.empty_cache()
    # the Environment 2.0 torus world
    NO, NW, NB = TORUS["counts"]
    tenv = BatchedWABEnvironment2(TORUS["width"], TORUS["height"], None, NO, NW, NB, num_worlds=B, seed=0x5EED,
                                  device=dev)
    N, R, h = tenv.N, tenv.R, tenv._h
    W = -(-2 * int(tenv.game_options["max_turns"]) // T) * T
    acts = torus_actions(W + NL * T, B, NO, NW, NB, dev, gen)
    ob = torch.empty((T, B, N, R), dtype=torch.uint8, device=dev)
    rw = torch.empty((T, B, N), dtype=torch.float32, device=dev)
    dn = torch.empty((T, B, N), dtype=torch.uint8, device=dev)
    wr = torch.empty((T, B), dtype=torch.uint8, device=dev)

    def troll(t, s):
        _lib.check2(L.wab2_rollout(h, acts.data_ptr() + t * B * N, T, ob.data_ptr(), rw.data_ptr(), dn.data_ptr(),
                                   wr.data_ptr(), s), "wab2_rollout")
    tenv.reset_environment()
    for t in range(0, W, T):
        troll(t, ctypes.c_void_p(stream.cuda_stream))
    ms, n = time_launches(lambda i, s: troll(W + i * T, s), NL, dev, stream, args.mode)
    e = entry(ms * 1e3 / T, torus_alg_bytes(NO, NW, NB, T), "torus_rollout%d" % T,
              "wab_torus_kernel (%d turns per launch)" % T, T, n,
              "wab2_rollout, %d turns per launch (Environment 2.0 torus 32x32, 1/8/16)" % T)
    e["entity_actions_per_s"] = round(e["env_steps_per_s"] * N, 1)
    out["torus_rollout"] = e
    del tenv, ob, acts
    torch.cuda.empty_cache()
    return out


def run_torus(args, dev, rank, world):
    """bench.py --config torus: T-turn wab2_rollout launches of B worlds per rank."""
    import torch
    import torch.distributed as dist

    from wab_gym_amd.shard import all_gather_objects, env_id_base, max_over_ranks
    from wab_gym_amd.torus import BatchedWABEnvironment2

    NO, NW, NB = TORUS["counts"]
    B, T = args.batch, (args.rollout if args.rollout > 0 else DEFAULT_ROLLOUT)
    env = BatchedWABEnvironment2(TORUS["width"], TORUS["height"], None, NO, NW, NB, num_worlds=B,
                                 seed=0x5EED, device=dev, world_id_base=env_id_base(rank, B))
    N, R = env.N, env.R
    W = max(args.warmup, 2 * int(env.game_options["max_turns"]))
    W = -(-W // T) * T
    K = window_steps(args.steps, T)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    actions = torus_actions(W + K, B, NO, NW, NB, dev, gen)
    obs = torch.empty((T, B, N, R), dtype=torch.uint8, device=dev)
    rew = torch.empty((T, B, N), dtype=torch.float32, device=dev)
    done = torch.empty((T, B, N), dtype=torch.uint8, device=dev)
    wr = torch.empty((T, B), dtype=torch.uint8, device=dev)
    from wab_gym_amd import _lib
    L, h = _lib.load(), env._h
    a0, o0, r0, d0, w0 = actions.data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(), wr.data_ptr()

    def run(t0, n, stream):
        s = ctypes.c_void_p(stream.cuda_stream)
        for t in range(t0, t0 + n, T):
            _lib.check2(L.wab2_rollout(h, a0 + t * B * N, T, o0, r0, d0, w0, s), "wab2_rollout")

    stream = torch.cuda.current_stream(dev)
    env.reset_environment()
    run(0, W, stream)
    torch.cuda.synchronize(dev)
    graph = None
    if args.mode == "graph":
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                run(W, K, torch.cuda.current_stream(dev))
        stream.wait_stream(side)
        torch.cuda.synchronize(dev)
        env.reset_environment()  # the capture did not execute the turns: rewind
        run(0, W, stream)
        torch.cuda.synchronize(dev)

    def replay_once():
        if graph is not None:
            graph.replay()
        else:
            run(W, K, stream)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record(stream)
    replay_once()
    c1.record(stream)
    torch.cuda.synchronize(dev)
    reps = window_replays(c0.elapsed_time(c1) * 1e-3)
    if world > 1:
        reps = int(max_over_ranks(reps))
    cb = env.counters()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_wall = time.perf_counter()
    with CLOCK:
        ev0.record(stream)
        for _ in range(reps):
            replay_once()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t_wall
    line_sclk = CLOCK.last
    stream_ms = ev0.elapsed_time(ev1)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(stream_ms * 1e-3)
    ca = env.counters()
    steps = K * reps
    kern_ms = stream_ms / steps  # per turn (launch / T)
    alg = torus_alg_bytes(NO, NW, NB, T)
    # the per-step surface beside it: one wab2_step launch per turn, records into a 32-slot ring
    NR = 32
    ps_ms = float("nan")
    if not args.no_diag:
        ring = torch.empty((NR, B, N, R), dtype=torch.uint8, device=dev)
        ring_rd = torch.empty((NR, B, N), dtype=torch.float32, device=dev)
        ring_dn = torch.empty((NR, B, N), dtype=torch.uint8, device=dev)
        ps_ms, ps_n = time_launches(
            lambda i, s: _lib.check2(L.wab2_step(h, a0 + (W + i) * B * N, ring[i % NR].data_ptr(),
                                                 ring_rd[i % NR].data_ptr(), ring_dn[i % NR].data_ptr(), None, s),
                                     "wab2_step"), min(K, 256), dev, stream, args.mode)
        del ring
    ps_alg = torus_alg_bytes(NO, NW, NB, 1)
    achieved = alg * B / (kern_ms * 1e-3) / 1e9
    per_rank = all_gather_objects({"rank": rank, "device": str(dev), "pci": pci_id(dev),
                                   "env_steps_per_s": round(B * steps / (stream_ms * 1e-3), 1),
                                   "stream_ms": round(stream_ms, 3), "achieved_GBs": round(achieved, 1)})
    if rank == 0:
        traffic, traffic_src = committed_traffic("torus_rollout%d" % T, B)
        line = {
            "metric": METRIC, "value": round(world * B * steps / elapsed, 1), "unit": "env-steps/s",
            "n_gpus": world, "steps": steps, "steps_requested": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / steps, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: uniform random actions (torch.randint on device), keyed-RNG worlds",
            "config": {"workload": TORUS["desc"] + "; %d-turn wab2_rollout launches (records, reward, done "
                                                   "of every turn into [%d, B] buffers)" % (T, T),
                       "batch_per_gpu": B, "global_batch": B * world, "world": [TORUS["width"], TORUS["height"]],
                       "entities": {"ostriches": NO, "wolves": NW, "bushes": NB}, "record_bytes": R,
                       "launch": args.mode, "parallelism": "independent world shards x%d (no collective)" % world},
            "entity_actions_per_s": round(world * B * steps * N / elapsed, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_unit": "bytes/launch (PMC 2*FETCH_SIZE + WRITE_SIZE)", "traffic_source": traffic_src,
                         "alg_bytes_per_launch": round(alg * B * T), "kernel": "wab_torus_kernel (%d turns per launch)" % T,
                         "kernel_us": round(kern_ms * T * 1e3, 3), "alg_bytes_per_env_step": round(alg, 3)},
            "per_step_launch": {"api": "wab2_step, records into a %d-slot ring of [B, N, R] buffers" % NR,
                                "us_per_step": round(ps_ms * 1e3, 3),
                                "env_steps_per_s": round(B / (ps_ms * 1e-3), 1),
                                "alg_bytes_per_env_step": round(ps_alg, 3),
                                "frac": round(ps_alg * B / (ps_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "timed_window": {"turns": ca["turns"] - cb["turns"], "resets": ca["resets"] - cb["resets"],
                             "graph_steps": K, "graph_replays": reps, "launches": steps // T,
                             "stream_ms": round(stream_ms, 3), "wall_ms": round(wall * 1e3, 3),
                             "floor": {"min_launches": MIN_TIMED_LAUNCHES, "min_seconds": MIN_TIMED_SECONDS}},
            "warmup_effective": W,
            "devices": sorted({r["pci"] for r in per_rank}),
            "sclk_mhz": line_sclk,
        }
        if world > 1:
            line["per_rank"] = per_rank
        if world == 1 and not args.no_cpu:
            cores = host_cores()
            line["cpu_baseline"] = torus_cpu_baseline(args.cpu_seconds, cores["used"])
            line["cpu_baseline"]["host"] = cores
        print(json.dumps(finite(line), allow_nan=False), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_cores():
    """The host's CPU count (nproc), the cores this process may run on (affinity), the
    cgroup CPU quota, and the thread count the baseline uses: every core available to the
    process, capped by the box's CPU share (OMP_NUM_THREADS, which the GPU box sets to its
    per-GPU share)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    used = aff if quota is None else max(1, min(aff, int(quota)))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if share > 0:
        used = min(used, share)
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "omp_num_threads": share or None,
            "used": used}


def committed_pmc(config, batch):
    """VALU figures of the committed PMC summary of this workload's step kernel (SQ counters,
    tools/profile.sh), or None."""
    path = os.path.join(REPO, "profiles", "traffic_%s_b%d.json" % (config, batch))
    if not os.path.exists(path):
        return None
    return json.load(open(path)).get("valu")


def cpu_baseline(opts, stride, seconds, threads, with_features=False):
    """The C oracle (scalar port of the reference step) timed on this host's cores; for C5 each
    step is followed by the oracle's PragmaticObsWrapper featurizer (one thread)."""
    import numpy as np

    from oracle import oracle as O

    Bc = 4096
    orc = O.OracleBatch(opts, Bc, 0x5EED, 0, True, stride)
    orc.reset()
    rng = np.random.RandomState(0)
    acts = [rng.randint(orc.n_actions, size=Bc).astype(np.int8) for _ in range(64)]
    vm = np.zeros((Bc, 11, 11), np.uint8)

    def one(a):
        orc.step(a, nthreads=threads)
        if with_features:
            O.featurize(orc.planes, orc.food_turns, orc.role, orc.status, vm, orc.W, orc.H)

    one(acts[0])
    n, t0 = 0, time.perf_counter()
    while True:
        one(acts[n % 64])
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    what = "step + featurize (1 thread)" if with_features else "step"
    return {"value": round(Bc * n / el, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "oracle/wab_oracle.c %s, %d envs x %d steps (%.1f s) of the same workload, "
                      "OpenMP over envs" % (what, Bc, n, el) if threads > 1 else
                      "oracle/wab_oracle.c %s, %d envs x %d steps (%.1f s), 1 thread" % (what, Bc, n, el)}


def config_cpu_baselines(line, threads, seconds):
    """Each `configs` entry's own CPU baseline (the C oracle on this host's cores, a bounded
    sample of that entry's workload, outside every timed region): C3 at 31x31 in 32-byte rows,
    C5's step + featurizer, the torus world; the default per-step ring is the headline's own
    workload (its `cpu_baseline`)."""
    cfgs = line["configs"]
    wopts, wstride = CONFIGS["wide31"][0], CONFIGS["wide31"][1]
    if "wide31_rollout" in cfgs or "wide31_per_step_ring" in cfgs:
        wb = cpu_baseline(wopts, wstride, seconds, threads)
        for k in ("wide31_rollout", "wide31_per_step_ring"):
            if k in cfgs:
                cfgs[k]["cpu_baseline"] = wb
    if "c5_rollout" in cfgs:
        cfgs["c5_rollout"]["cpu_baseline"] = cpu_baseline(CONFIGS["c5"][0], CONFIGS["c5"][1], seconds, threads, True)
    if "default_per_step_ring" in cfgs:
        cfgs["default_per_step_ring"]["cpu_baseline"] = dict(line["cpu_baseline"], same_as="cpu_baseline")
    if "torus_rollout" in cfgs:
        cfgs["torus_rollout"]["cpu_baseline"] = torus_cpu_baseline(seconds, threads)


def make_policy(F, n_actions, dev, seed=0):
    """actor_critic.py's Policy (actor_critic.py:54-97: 449 -> 128 -> 150 -> 128, leaky_relu,
    clamp(-4, 4), softmax action head and a value head) in stock torch, fp32, random init, and
    select_action's sampling (:108-125): the features plus U(0, 1)/100 noise, a Categorical draw
    by inverse CDF over the probabilities (torch.rand only, so the whole step captures in a
    graph).  act(features [B, F], out [B] int8) writes the sampled actions."""
    import torch
    import torch.nn.functional as Fn

    torch.manual_seed(seed)

    class Policy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.affine1 = torch.nn.Linear(F, 128)
            self.affine2 = torch.nn.Linear(128, 150)
            self.affine3 = torch.nn.Linear(150, 128)
            self.action_head = torch.nn.Linear(128, n_actions)
            self.value_head = torch.nn.Linear(128, 1)

        def forward(self, x):
            x = Fn.leaky_relu(self.affine1(x))
            x = Fn.leaky_relu(self.affine2(x))
            x = Fn.leaky_relu(self.affine3(x))
            x = torch.clamp(x, -4, 4)
            return Fn.softmax(self.action_head(x), dim=-1), self.value_head(x)

        @torch.no_grad()
        def act(self, feats, out):
            probs, value = self(feats + torch.rand_like(feats) / 100)
            u = torch.rand((feats.shape[0], 1), device=feats.device)
            a = (probs.cumsum(-1) < u).sum(-1).clamp_(max=n_actions - 1)
            out.copy_(a)
            self.last_value = value
            return out

    return Policy().to(dev).eval()


def probe_device_count():
    """GPUs visible to a fresh process, counted in a child so this (launcher) process never
    touches the GPU runtime before it starts the ranks."""
    import subprocess

    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        raise SystemExit("bench.py: could not count GPUs: %s" % r.stderr[-2000:])


def self_launch(args):
    """`bench.py --gpus N` run without a torch.distributed launcher (WORLD_SIZE unset): start N
    fresh rank processes of this script, one per GPU (RANK = LOCAL_RANK = r), wait for all,
    print rank 0's JSON line and return the first failing child's exit code.  Nothing here
    touches the GPU: the device count comes from a child process."""
    from wab_gym_amd.shard import launch_ranks

    n = args.gpus
    ndev = probe_device_count()
    if n > ndev and not args.share_gpu:
        raise SystemExit("bench.py: --gpus %d but %d GPU(s) visible; pass --share-gpu to run "
                         "%d ranks on the visible GPU(s) (a rehearsal, not a scaling figure)" % (n, ndev, n))
    rc, out, codes = launch_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], n)
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    for ln in out.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if rc != 0:
        print("bench.py: rank exit codes %s" % codes, file=sys.stderr)
        return rc if rc > 0 else 1
    if not lines:
        print("bench.py: rank 0 printed no JSON line", file=sys.stderr)
        return 1
    print(lines[-1], flush=True)
    return 0


def pci_id(dev):
    """domain:bus:device of a torch device (tells ranks on distinct GPUs from shared ones)."""
    import torch

    p = torch.cuda.get_device_properties(dev)
    return "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--share-gpu", action="store_true",
                    help="allow --gpus N above the visible GPU count: ranks then share GPUs "
                         "(rank r on GPU r mod count); a rehearsal of the N-rank path")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--config", default="default", choices=sorted(CONFIGS) + ["torus"])
    ap.add_argument("--mode", default="graph", choices=["graph", "launch"])
    ap.add_argument("--rollout", type=int, default=-1,
                    help="T > 0: wab_rollout (c5: wab_rollout_features) segments of T steps (one "
                         "launch each; obs or features, reward, done into a [T, B] rollout buffer) "
                         "instead of one launch per step; 0: per-step launches; default: %d (the "
                         "small and wide kernels' multi-step builds)" % DEFAULT_ROLLOUT)
    ap.add_argument("--obs-ring", type=int, default=0,
                    help="per-step launches: N > 0 writes step t's obs, reward and done into slot t %% N of "
                         "[N, B] buffers (the stores then reach HBM, as a rollout's do) instead of one "
                         "[B] buffer rewritten every step (which a 256 MB Infinity Cache can absorb)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stream-shards", type=int, default=2,
                    help="rollout lines: the batch as this many independent shards (handles of B / S envs, "
                         "contiguous env ids), each shard's launches on its own HIP stream, so that one "
                         "shard's launch tail overlaps the other's next launch (1: one handle)")
    ap.add_argument("--no-extra", action="store_true",
                    help="default config: skip the other configs' lines (configs key) timed beside it")
    ap.add_argument("--no-diag", action="store_true",
                    help="skip the diagnostic launches beside the line (per-step launches, single-launch "
                         "timings): for profiling the line's kernel alone")
    ap.add_argument("--wolf-slots", type=int, default=0, choices=[0, 8, 16, 32],
                    help="override the config's wolf rows per env (0: the config's own; the wide "
                         "kernel keeps 8 of them in registers)")
    ap.add_argument("--policy", default="random", choices=["random", "mlp"],
                    help="c5 only.  random: actions drawn up front (the line's open-loop rollout); "
                         "mlp: closed loop, each step's actions sampled from actor_critic.py's "
                         "Policy (449-128-150-128-{5,1}, stock torch, fp32, random init) on the "
                         "previous step's features, then one wab_step_features launch; graph-captured")
    ap.add_argument("--c5-unfused", action="store_true",
                    help="C5 as wab_step + wab_featurize (obs planes stored) instead of wab_step_features")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.policy == "mlp" and args.config != "c5":
        raise SystemExit("bench.py: --policy mlp needs --config c5 (the policy reads the features)")
    if args.rollout < 0:
        args.rollout = DEFAULT_ROLLOUT if not (args.c5_unfused or args.policy == "mlp") else 0
    if args.policy == "mlp" and args.rollout > 0:
        raise SystemExit("bench.py: --policy mlp picks each step's action from that step's features: "
                         "one launch per step (--rollout 0)")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args))

    import torch
    import torch.distributed as dist

    from wab_gym_amd.shard import all_gather_objects, device_for_rank, env_id_base, max_over_ranks, rank_info

    rank, world, local = rank_info()
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d; the line reports WORLD_SIZE" % (args.gpus, world),
              file=sys.stderr)
    ndev = torch.cuda.device_count()
    # LOCAL_RANK r -> GPU r; ranks share a GPU only when asked (--share-gpu: the 1-GPU rehearsal)
    local = device_for_rank(local, ndev, args.share_gpu)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    global CLOCK
    CLOCK = ClockSampler(pci_id(dev))
    if world > 1:
        dist.init_process_group("gloo")  # CPU only: barrier + timing MAX; no RCCL

    if args.config == "torus":
        return run_torus(args, dev, rank, world)

    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    opts, stride, slots, desc = CONFIGS[args.config]
    slots = args.wolf_slots or slots
    c5 = args.config == "c5"
    c5_roll = c5 and args.rollout > 0
    if c5_roll:
        args.rollout = C5_SEGMENT if args.rollout <= 0 else args.rollout
    rollout = args.rollout > 0 and not c5
    T_roll = args.rollout
    B, K, W = args.batch, args.steps, args.warmup
    S = args.stream_shards if (rollout or (c5_roll and args.policy != "mlp")) else 1
    if S < 1 or B % (64 * S):
        S = 1  # (whole 64-env groups per shard)
    env = BatchedWolvesAndBushesEnv(opts, num_envs=B, seed=0x5EED, device=dev,
                                    env_id_base=env_id_base(rank, B),
                                    autoreset=True, validate_actions=False, plane_stride=stride,
                                    wolf_slots=slots)
    # steady state: at least two full episodes' worth of untimed steps after the reset
    W = max(W, 2 * int(env.game_options["max_turns"]))
    if c5:
        seg = T_roll if c5_roll else C5_SEGMENT
        desc = desc % seg
        per_launch_steps = seg if c5_roll else 1
        W = max(seg, -(-W // seg) * seg)
        if args.policy == "mlp":
            # closed loop: ~16 graph nodes per step (the policy's kernels and the env launch), so
            # the captured graph holds 2-4 segments and replays make up the timed window
            K = min(window_steps(K, seg, 2), 4 * seg)
        else:
            K = window_steps(K, seg, MIN_TIMED_LAUNCHES if c5_roll else MIN_TIMED_LAUNCHES * seg)
    elif rollout:
        per_launch_steps = args.rollout
        W = -(-W // args.rollout) * args.rollout
        K = window_steps(K, args.rollout)
    else:
        per_launch_steps = 1
        K = window_steps(K, 1)
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    actions = torch.randint(0, env.n_actions, (W + K, B), device=dev, generator=gen).to(torch.int8)
    L = _lib.load()
    h = env._h
    obs_addr = ctypes.addressof(env._obs["struct"])
    a0 = actions.data_ptr()
    rew, done = env.reward.data_ptr(), env.done.data_ptr()
    # a sharded rollout line: the B envs as S handles of Bs envs (ids contiguous, so the union is
    # the one-handle batch bit for bit), shard k's launches in order on its own stream
    Bs = B // S
    shard_envs = [env] if S == 1 else [
        BatchedWolvesAndBushesEnv(opts, num_envs=Bs, seed=0x5EED, device=dev,
                                  env_id_base=env_id_base(rank, B) + k * Bs, autoreset=True,
                                  validate_actions=False, plane_stride=stride, wolf_slots=slots)
        for k in range(S)]
    if S > 1:
        for e in shard_envs:
            e.reset()
    # each shard's actions [W + K][Bs] contiguous (the same random draws, shard-major)
    shard_actions = actions.view(W + K, S, Bs).permute(1, 0, 2).contiguous() if S > 1 else None
    shard_streams = [torch.cuda.Stream(dev) for _ in range(S - 1)]

    def shard_chains(t0, n, T, stream, launch):
        """launch(k, t, hip_stream) for every T-step launch t in [t0, t0 + n) of every shard k,
        shard 0 on `stream`, the others on their own streams forked from it and joined back"""
        subs = [stream] + shard_streams
        for st in shard_streams:
            st.wait_stream(stream)
        for t in range(t0, t0 + n, T):
            for k, st in enumerate(subs):
                launch(k, t, ctypes.c_void_p(st.cuda_stream))
        for st in shard_streams:
            stream.wait_stream(st)
    if c5:
        T = T_roll if c5_roll else C5_SEGMENT
        F = int(L.wab_feature_dim(h))
        feats = torch.zeros((T, B, F), dtype=torch.float32, device=dev)
        seg_rew = torch.zeros((T, B), dtype=torch.float32, device=dev)
        seg_done = torch.zeros((T, B), dtype=torch.uint8, device=dev)
        seg_ret = torch.empty((T, B), dtype=torch.float32, device=dev)
        f0, r0, d0, ret0 = feats.data_ptr(), seg_rew.data_ptr(), seg_done.data_ptr(), seg_ret.data_ptr()
        fused = not args.c5_unfused
        # the wrapped env of actor_critic.py returns features only: the fused call renders the
        # obs planes on chip for the featurizer and does not store them
        o = env._obs["struct"]
        fobs = _lib.WabObs(None, o.food_turns, o.role, o.status)
        fobs_addr = ctypes.addressof(fobs)
        seg_scal = torch.empty((3, T, B), dtype=torch.uint8, device=dev)
        rseq = _lib.WabObs(None, seg_scal[0].data_ptr(), seg_scal[1].data_ptr(), seg_scal[2].data_ptr())
        rseq_addr = ctypes.addressof(rseq)

        def c5_step(t, i, s):
            if fused:
                return L.wab_step_features(h, a0 + t * B, fobs_addr, r0 + 4 * i * B, d0 + i * B,
                                           f0 + 4 * i * B * F, s)
            rc = L.wab_step(h, a0 + t * B, obs_addr, r0 + 4 * i * B, d0 + i * B, None, s)
            return rc or L.wab_featurize(h, obs_addr, None, f0 + 4 * i * B * F, s)

        policy = None
        if args.policy == "mlp":
            policy = make_policy(F, env.n_actions, dev)
        c5_shard = []  # per shard: scalars WabObs, reward, done, features, returns (+ keepalive)
        if c5_roll and S > 1:
            for k in range(S):
                sc_k = torch.empty((3, T, Bs), dtype=torch.uint8, device=dev)
                c5_shard.append((_lib.WabObs(None, sc_k[0].data_ptr(), sc_k[1].data_ptr(), sc_k[2].data_ptr()),
                                 torch.empty((T, Bs), dtype=torch.float32, device=dev),
                                 torch.empty((T, Bs), dtype=torch.uint8, device=dev),
                                 torch.empty((T, Bs, F), dtype=torch.float32, device=dev),
                                 torch.empty((T, Bs), dtype=torch.float32, device=dev), sc_k))

        def run(t0, n, stream):
            s = ctypes.c_void_p(stream.cuda_stream)
            if policy is not None:  # closed loop: each step's action from the policy on the last features
                for t in range(t0, t0 + n):
                    i = t % T
                    prev = feats[(i - 1) % T]
                    policy.act(prev, actions[t])
                    _lib.check(c5_step(t, i, s), "c5 step")
                    if i == T - 1:
                        _lib.check(L.wab_discounted_returns_exact(h, r0, d0, T, B, 0.99, None, ret0, s),
                                   "wab_discounted_returns_exact")
                return
            if c5_roll and S > 1:  # the shards' segments on their streams
                shard_chains(t0, n, T, stream, lambda k, t, sk: _lib.check(L.wab_rollout_features(
                    shard_envs[k]._h, shard_actions[k].data_ptr() + t * Bs, T, ctypes.addressof(c5_shard[k][0]),
                    c5_shard[k][1].data_ptr(), c5_shard[k][2].data_ptr(), c5_shard[k][3].data_ptr(), 0.99, None,
                    c5_shard[k][4].data_ptr(), sk), "wab_rollout_features"))
                return
            if c5_roll:  # one launch per segment: T fused steps and the segment's returns
                for t in range(t0, t0 + n, T):
                    _lib.check(L.wab_rollout_features(h, a0 + t * B, T, rseq_addr, r0, d0, f0, 0.99, None, ret0, s),
                               "wab_rollout_features")
                return
            for t in range(t0, t0 + n):
                i = t % T
                _lib.check(c5_step(t, i, s), "c5 step")
                if i == T - 1:
                    _lib.check(L.wab_discounted_returns_exact(h, r0, d0, T, B, 0.99, None, ret0, s),
                               "wab_discounted_returns_exact")
    elif rollout:
        T = args.rollout
        if S == 1:
            shard_actions = actions.view(1, W + K, B)
        shard_bufs = []
        for k, e in enumerate(shard_envs):
            pl = torch.empty((T, Bs, 3, env.W, env.S), dtype=torch.uint8, device=dev)
            sc = torch.empty((3, T, Bs), dtype=torch.uint8, device=dev)
            rw = torch.empty((T, Bs), dtype=torch.float32, device=dev)
            dn = torch.empty((T, Bs), dtype=torch.uint8, device=dev)
            o = _lib.WabObs(pl.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), sc[2].data_ptr())
            shard_bufs.append((e._h, shard_actions[k].data_ptr(), o, pl, sc, rw, dn))

        def run(t0, n, stream):
            def launch(k, t, sk):
                hk, ak, o, pl, sc, rw, dn = shard_bufs[k]
                _lib.check(L.wab_rollout(hk, ak + t * Bs, T, ctypes.addressof(o), rw.data_ptr(), dn.data_ptr(), sk),
                           "wab_rollout")
            shard_chains(t0, n, T, stream, launch)
    elif args.obs_ring > 0:
        N = args.obs_ring
        ring_planes = torch.empty((N, B, 3, env.W, env.S), dtype=torch.uint8, device=dev)
        ring_scal = torch.empty((3, N, B), dtype=torch.uint8, device=dev)
        ring_rew = torch.empty((N, B), dtype=torch.float32, device=dev)
        ring_done = torch.empty((N, B), dtype=torch.uint8, device=dev)
        ring_slots = [_lib.WabObs(ring_planes[i].data_ptr(), ring_scal[0, i].data_ptr(), ring_scal[1, i].data_ptr(),
                             ring_scal[2, i].data_ptr()) for i in range(N)]
        slot_addr = [ctypes.addressof(o) for o in ring_slots]
        _lib.check(L.wab_set_obs_placement(h, _lib.OBS_FRESH_BUFFER), "wab_set_obs_placement")

        def run(t0, n, stream):
            s = ctypes.c_void_p(stream.cuda_stream)
            for t in range(t0, t0 + n):
                i = t % N
                rc = L.wab_step(h, a0 + t * B, slot_addr[i], ring_rew[i].data_ptr(), ring_done[i].data_ptr(), None, s)
                if rc:
                    _lib.check(rc, "wab_step")
    else:
        def run(t0, n, stream):
            s = ctypes.c_void_p(stream.cuda_stream)
            for t in range(t0, t0 + n):
                rc = L.wab_step(h, a0 + t * B, obs_addr, rew, done, None, s)
                if rc:
                    _lib.check(rc, "wab_step")

    stream = torch.cuda.current_stream(dev)
    run(0, W, stream)
    torch.cuda.synchronize(dev)
    print("bench.py: %d warm-up steps done" % W, file=sys.stderr, flush=True)
    graph = None
    if args.mode == "graph":
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                run(W, K, torch.cuda.current_stream(dev))
        stream.wait_stream(side)
        torch.cuda.synchronize(dev)
        print("bench.py: %d steps captured" % K, file=sys.stderr, flush=True)
        # the capture itself did not execute the steps; rewind state by a fresh reset
        env.reset()
        if S > 1:
            for e in shard_envs:
                e.reset()
        run(0, W, stream)
        torch.cuda.synchronize(dev)

    def replay_once():
        if graph is not None:
            graph.replay()
        else:
            run(W, K, stream)

    # calibration (untimed): one replay of the window's K steps sizes the replay count
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record(stream)
    replay_once()
    c1.record(stream)
    torch.cuda.synchronize(dev)
    reps = window_replays(c0.elapsed_time(c1) * 1e-3)
    if world > 1:  # every rank times the same number of steps
        reps = int(max_over_ranks(reps))

    timed_envs = shard_envs if (rollout or c5_roll) else [env]

    def workload_counters():
        out = {}
        for e in timed_envs:
            for k_, v in e.counters().items():
                out[k_] = out.get(k_, 0) + v
        return out
    c_before = workload_counters()  # (synchronises; outside the timed region)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    with CLOCK:  # (a host thread reading sysfs: nothing on the device's path)
        ev0.record(stream)
        for _ in range(reps):
            replay_once()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
    wall_rank = time.perf_counter() - t0
    line_sclk = CLOCK.last
    # each rank's time is its own launch stream's, from the HIP events around the window; the
    # MAX over ranks is taken afterwards (no barrier inside the window)
    stream_ms = ev0.elapsed_time(ev1)
    elapsed_rank = stream_ms * 1e-3
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed_rank)
    K_req, K = K, K * reps  # steps in the graph; steps timed
    c_after = workload_counters()
    window = {"env_steps": c_after["steps"] - c_before["steps"],
              "resets": c_after["resets"] - c_before["resets"],
              "graph_steps": K_req, "graph_replays": reps,
              "launches": K // per_launch_steps,
              "stream_ms": round(stream_ms, 3), "wall_ms": round(wall_rank * 1e3, 3)}
    window["resets_per_env_step"] = round(window["resets"] / max(1, window["env_steps"]), 5)
    window["floor"] = {"min_launches": MIN_TIMED_LAUNCHES, "min_seconds": MIN_TIMED_SECONDS}

    # kernel duration: the HIP events around the timed region on the launch stream give the
    # average per launch (back-to-back graph launches: kernel time plus the launch gap, the
    # figure rocprofv3's average agrees with); events bracketing single launches (below, not
    # timed above) add their own overhead and are reported as a diagnostic only
    kern_ms = stream_ms / K
    n_k = min(K_req, 200) if not args.no_diag else 0  # (the actions buffer holds W + K_req steps)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_k)]
    s = ctypes.c_void_p(stream.cuda_stream)
    for i in range(n_k):
        evs[i][0].record(stream)
        L.wab_step(h, a0 + (W + i) * B, obs_addr, rew, done, None, s)
        evs[i][1].record(stream)
    torch.cuda.synchronize(dev)
    single_ms = sorted(a.elapsed_time(b) for a, b in evs)[n_k // 2] if n_k else float("nan")
    kernel_name = "wab_step_%s (fused step)" % L.wab_step_kernel(h).decode()
    alg = alg_bytes_per_env_step(env.W, env.H)
    c5_line = None
    roll_line = None

    # a kernel's average launch from n back-to-back launches of it alone, captured in a graph
    # (as the timed region is) so that host launch cost does not pace a short kernel; HIP
    # events on the launch stream around one replay
    def per_launch(fn, n, required=False):
        if args.no_diag and not required:
            return float("nan")

        def launches(st):
            sc = ctypes.c_void_p(st.cuda_stream)
            for i in range(n):
                _lib.check(fn(i, sc), "kernel timing")
        if args.mode == "graph":
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(dev)
            side.wait_stream(stream)
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    launches(torch.cuda.current_stream(dev))
            stream.wait_stream(side)
            g.replay()  # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if args.mode == "graph":
            g.replay()
        else:
            launches(stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    if rollout:
        # the gym surface's per-step launches (wab_step, obs into the same buffer each step),
        # measured beside the rollout line; a rollout launch moves the state once per T steps
        # (loaded by its first step, stored by its last), so its algorithmic bytes per env-step
        # are the obs, action, scalars, reward and done plus 2 * 36 / T of state
        # into a 32-slot ring of [B] obs buffers (step t into slot t % 32, so the stores reach
        # HBM as the rollout's do) and, as a diagnostic, into one [B] buffer rewritten every step
        # (which the 256 MB Infinity Cache can hold)
        NR = 32
        ring_planes = torch.empty((NR, B, 3, env.W, env.S), dtype=torch.uint8, device=dev)
        ring_scal = torch.empty((3, NR, B), dtype=torch.uint8, device=dev)
        ring_rd = torch.empty((NR, B, 5), dtype=torch.uint8, device=dev)  # reward f32 + done u8
        ring_obs = [_lib.WabObs(ring_planes[i].data_ptr(), ring_scal[0, i].data_ptr(), ring_scal[1, i].data_ptr(),
                                ring_scal[2, i].data_ptr()) for i in range(NR)]
        ring_addr = [ctypes.addressof(o) for o in ring_obs]
        rr = torch.empty((NR, B), dtype=torch.float32, device=dev)
        n_ps = min(K_req, 512)
        _lib.check(L.wab_set_obs_placement(h, _lib.OBS_FRESH_BUFFER), "wab_set_obs_placement")
        ps_ms = per_launch(lambda i, s: L.wab_step(h, a0 + (W + i) * B, ring_addr[i % NR], rr[i % NR].data_ptr(),
                                                   ring_rd[i % NR].data_ptr(), None, s), n_ps)
        _lib.check(L.wab_set_obs_placement(h, _lib.OBS_SAME_BUFFER), "wab_set_obs_placement")
        psc_ms = per_launch(lambda i, s: L.wab_step(h, a0 + (W + i) * B, obs_addr, rew, done, None, s), n_ps)
        del ring_planes
        # the same rollout as ONE handle of B envs on one stream (the S = 1 line), for comparison
        one_ms = float("nan")
        if S > 1 and not args.no_diag:
            seq_planes = torch.empty((T, B, 3, env.W, env.S), dtype=torch.uint8, device=dev)
            seq_scal = torch.empty((3, T, B), dtype=torch.uint8, device=dev)
            seq_rd = torch.empty((T, B, 5), dtype=torch.uint8, device=dev)
            seq = _lib.WabObs(seq_planes.data_ptr(), seq_scal[0].data_ptr(), seq_scal[1].data_ptr(),
                              seq_scal[2].data_ptr())
            n_one = max(1, min(K_req // T, MIN_TIMED_LAUNCHES))
            one_ms = per_launch(lambda i, s: L.wab_rollout(h, a0 + (W + (i * T) % K_req) * B, T, ctypes.addressof(seq),
                                                           seq_rd.data_ptr(), seq_rd.data_ptr() + 4 * T * B, s),
                                n_one) / T
            del seq_planes
        roll_line = {"steps_per_launch": T_roll, "launch_us": round(kern_ms * T_roll * 1e3, 3),
                     "stream_shards": S, "envs_per_launch": B // S,
                     "one_handle_us_per_step": None if one_ms != one_ms else round(one_ms * 1e3, 3),
                     "per_step_launch": {"api": "wab_step (the raw C-ABI per-step launch), step t's obs into "
                                                "slot t %% %d of a ring of [B] buffers" % NR,
                                         "us_per_step": round(ps_ms * 1e3, 3),
                                         "env_steps_per_s": round(B / (ps_ms * 1e-3), 1),
                                         "alg_bytes_per_env_step": alg,
                                         "frac": round(alg * B / (ps_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                         # BatchedWolvesAndBushesEnv.step's own pattern: every step
                                         # into the env's one [B] obs buffer (Infinity-Cache resident)
                                         "env_step_one_buffer_us_per_step": round(psc_ms * 1e3, 3)}}
        alg = alg_bytes_per_env_step_rollout(env.W, env.H, T_roll)
        kernel_name = "wab_step_%s, rollout build (%d steps per launch)" % (L.wab_step_kernel(h).decode(), T_roll)
    if c5:
        n_k = min(K_req, 512)
        ret_ms = per_launch(lambda i, s: L.wab_discounted_returns_exact(h, r0, d0, T, B, 0.99, None, ret0, s), 64)
        if fused:
            sf_ms = per_launch(lambda i, s: L.wab_step_features(h, a0 + (W + i) * B, fobs_addr, rew, done,
                                                                f0 + 4 * (i % T) * B * F, s), n_k,
                               required=not c5_roll)
            # per env-step: the step's bytes without the planes (never stored), the F floats
            sf_alg = alg - 3 * env.W * env.H + 4 * F
            c5_line = {"segment": T, "feature_dim": F, "fused": True,
                       "api": ("wab_rollout_features (%d steps + returns per launch)" % T if c5_roll else
                               "wab_step_features per step + wab_discounted_returns_exact per segment"),
                       "step_features_us": round(sf_ms * 1e3, 3),
                       "returns_us_per_segment": round(ret_ms * 1e3, 3),
                       "returns_frac": round(RETURNS_ALG_BYTES * T * B / (ret_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                       "alg_bytes_per_env_step": sf_alg + RETURNS_ALG_BYTES}
            if not c5_roll and policy is None:
                # the per-step line: the fused launch's bytes + the scan's, over the timed step
                c5_line["achieved_GBs_whole_step"] = round((sf_alg + RETURNS_ALG_BYTES) * B / (kern_ms * 1e-3) / 1e9, 1)
            kernel_name = "wab_step_%s + PragmaticObsWrapper features (wab_step_features)" % L.wab_step_kernel(h).decode()
            if c5_roll:
                # the line's kernel is the rollout launch itself (kern_ms: per step from the
                # timed region); the per-step fused launch is a diagnostic beside it
                c5_line["rollout_launch_us"] = round(kern_ms * T * 1e3, 3)
                c5_line["stream_shards"] = S
                c5_line["per_step_launch_frac"] = round(sf_alg * B / (sf_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                alg = c5_rollout_alg_bytes(F, T)
                kernel_name = ("wab_step_%s + PragmaticObsWrapper features + returns, rollout build (%d steps "
                               "per launch, wab_rollout_features)" % (L.wab_step_kernel(h).decode(), T))
            else:
                if policy is not None:
                    # closed loop: the timed step is the policy forward + sample + the fused env
                    # launch (+ the scan every T steps); the env's share from its own launches
                    def policy_only(i, s):
                        policy.act(feats[i % T], actions[W + i])
                        return 0
                    pol_ms = per_launch(policy_only, n_k)
                    step_total = kern_ms
                    c5_line["policy"] = {
                        "model": "actor_critic.py Policy 449-128-150-128-{%d,1}, fp32 stock torch, "
                                 "random init; Categorical sample by inverse CDF" % env.n_actions,
                        "us_per_step": round(step_total * 1e3, 3),
                        "policy_us": round(pol_ms * 1e3, 3),
                        "env_us": round(sf_ms * 1e3 + ret_ms * 1e3 / T, 3),
                        "env_share": round((sf_ms + ret_ms / T) / step_total, 4)}
                alg, kern_ms = sf_alg, sf_ms
        step_ms = per_launch(lambda i, s: L.wab_step(h, a0 + (W + i) * B, obs_addr, rew, done, None, s), n_k)
        feat_ms = per_launch(lambda i, s: L.wab_featurize(h, obs_addr, None, f0 + 4 * (i % T) * B * F, s), n_k)
        feat_alg = featurize_alg_bytes(env.W, env.H, F)
        if fused:
            c5_line["unfused_step_us"] = round(step_ms * 1e3, 3)
            c5_line["unfused_featurize_us"] = round(feat_ms * 1e3, 3)
        else:
            c5_line = {"segment": T, "feature_dim": F, "fused": False, "step_us": round(step_ms * 1e3, 3),
                       "featurize_us": round(feat_ms * 1e3, 3), "returns_us_per_segment": round(ret_ms * 1e3, 3),
                       "alg_bytes_per_env_step": alg + feat_alg + RETURNS_ALG_BYTES,
                       "achieved_GBs_whole_step": round((alg + feat_alg + RETURNS_ALG_BYTES) * B / (kern_ms * 1e-3) / 1e9, 1)}
            if feat_ms > step_ms:  # the dominant kernel carries the roofline object
                fk = ("wab_featurize_small_kernel" if env.W * env.H <= 128 and env.S == env.H
                      else "wab_featurize_kernel")
                kernel_name, alg, kern_ms = fk + " (PragmaticObsWrapper + flatten)", feat_alg, feat_ms
            else:
                kern_ms = step_ms
    counters = workload_counters() if (rollout or c5_roll) else env.counters()
    achieved_rank = alg * B / (kern_ms * 1e-3) / 1e9
    per_rank = all_gather_objects({
        "rank": rank, "device": str(dev), "pci": pci_id(dev), "env_steps_per_s": round(B * K / elapsed_rank, 1),
        "ms_per_step": round(elapsed_rank * 1e3 / K, 5), "stream_ms": round(stream_ms, 3),
        "wall_ms": round(wall_rank * 1e3, 3), "kernel_us": round(kern_ms * 1e3, 3),
        "achieved_GBs": round(achieved_rank, 1), "frac": round(achieved_rank / HBM_PEAK_GBS, 4),
        "timed_window": window, "overflow": counters["wolf_overflow"] + counters["eaten_overflow"],
        "handoff_timeouts": counters["handoff_timeouts"]})

    if rank == 0:
        Wv, Hv = env.W, env.H
        achieved = achieved_rank
        value = world * B * K / elapsed
        # the committed PMC traffic is of the default launch of each config (C5: the fused one)
        tkey = args.config + ("_rollout%d" % T_roll if rollout or c5_roll else
                              "_ring%d" % args.obs_ring if args.obs_ring else "") + ("_s%d" % S if S > 1 else "")
        traffic, traffic_src = committed_traffic(tkey, B) if not args.c5_unfused else (None, None)
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "steps_requested": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / K, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: uniform random actions (torch.randint on device), keyed-RNG worlds",
            "config": {"workload": desc + ("; %d-step wab_rollout launches (obs, reward, done of every "
                                           "step into a [%d, B] rollout buffer)%s" % (
                                               T_roll, T_roll,
                                               ", the batch as %d shards of %d envs, each on its own HIP stream"
                                               % (S, B // S) if S > 1 else "")
                                           if rollout else
                                           "; %d-step wab_rollout_features launches (features, reward, done, "
                                           "returns into [%d, B] rollout buffers)%s" % (
                                               T_roll, T_roll,
                                               ", the batch as %d shards of %d envs, each on its own HIP stream"
                                               % (S, B // S) if S > 1 else "")
                                           if c5_roll else
                                           "; one step launch per step, obs into a %d-slot ring" % args.obs_ring
                                           if args.obs_ring > 0 else "; one step launch per step"),
                       "batch_per_gpu": B, "global_batch": B * world,
                       "viewport": [Wv, Hv], "plane_stride": env.S, "wolf_slots": slots, "launch": args.mode,
                       "stream_shards": S,
                       "parallelism": "independent env shards x%d (no collective)" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_unit": "bytes/launch (PMC 2*FETCH_SIZE + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "alg_bytes_per_launch": round(alg * (B // S) * (T_roll if rollout or c5_roll else 1)),
                         "kernel": kernel_name,
                         "kernel_us": round(kern_ms * 1e3 * (T_roll if rollout or c5_roll else 1), 3),
                         "alg_bytes_per_env_step": round(alg, 3)},
            "stream_us_per_step": round(stream_ms * 1e3 / K, 3),
            "warmup_requested": args.warmup,
            "warmup_effective": W,
            "timed_window": window,
            "overflow": {"wolf": counters["wolf_overflow"], "wolf_at_reset": counters["wolf_overflow_reset"],
                         "eaten": counters["eaten_overflow"],
                         "handoff_timeouts": counters["handoff_timeouts"]},
        }
        valu = committed_pmc(tkey, B) if not args.c5_unfused else None
        if valu:
            line["roofline"]["valu"] = valu
        line["devices"] = sorted({r["pci"] for r in per_rank})
        if world > 1:
            line["per_rank"] = per_rank
            if len(line["devices"]) < world:
                line["shared_gpus"] = True  # a rehearsal: ranks share a GPU, not a scaling figure
        if c5:
            line["c5"] = c5_line
        if rollout:
            roll_line["per_step_launch"]["single_launch_median_us"] = round(single_ms * 1e3, 3)
            line["rollout"] = roll_line
        else:
            line["roofline"]["kernel_us_single_launch_median"] = round(single_ms * 1e3, 3)
        line["sclk_mhz"] = line_sclk
        if world == 1 and args.config == "default" and rollout and not args.no_extra:
            # C3, C5, the per-step surfaces and the torus world beside the headline (their own
            # roofline each; the headline fields above are the default config's alone)
            line["configs"] = extra_configs(args, dev, B)
        if world == 1 and not args.no_cpu:
            cores = host_cores()
            line["cpu_baseline"] = cpu_baseline(opts, stride, args.cpu_seconds, cores["used"], c5)
            line["cpu_baseline"]["host"] = cores
            line["cpu_baseline_1t"] = cpu_baseline(opts, stride, args.cpu_seconds / 2, 1, c5)
            if "configs" in line:
                config_cpu_baselines(line, cores["used"], min(args.cpu_seconds, 5.0))
        print(json.dumps(finite(line), allow_nan=False), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
