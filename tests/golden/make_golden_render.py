"""Golden vectors for the batched renderer: the reference `WolvesAndBushesEnv.render`
(wab_env.py:468-502) with `draw_health=False`, on states reached by the reference itself.

Container-only (imports /root/reference through ref_harness).  For a few option sets, each
env takes random actions; after every step (and reset) we record the observation (planes,
role, status) and the reference's rgb_array at scale 2.  `draw_health=True` overlays the
food count with PIL's default font, whose glyphs depend on the Pillow version (the pinned
7.x font is not the one in this container): that overlay is out of scope and not recorded.

Usage: python tests/golden/make_golden_render.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as rh  # noqa: E402

SEED = 0x5EED
SCALE = 2
SETS = {
    # name: (options override, env ids, steps)
    "default": ({}, list(range(2000, 2006)), 60),
    "restrict": ({"restrict_view": True, "lookout_only": False}, list(range(2100, 2106)), 60),
    "wolfy": ({"chance_wolf_on_square": 0.03, "wolf_chance_to_despawn": 0.2, "wolf_spawn_margin": 2},
              list(range(2200, 2206)), 60),
}


def main():
    wab_env = rh.load_reference()
    planes_all, scal_all, img_all, set_ids = [], [], [], []
    for si, (name, (opts, env_ids, T)) in enumerate(SETS.items()):
        full = dict(wab_env.default_game_options)
        full.update(opts)
        rng = np.random.RandomState(17 + si)
        for g in env_ids:
            env = rh.make_env(SEED, g, full)
            obs = env.reset()
            n_actions = env.action_space.n
            for t in range(T + 1):
                planes, f, r, s = rh.obs_arrays(obs)
                img = env.render(mode="rgb_array", scale=SCALE, draw_health=False)
                planes_all.append(planes.astype(np.uint8))
                scal_all.append((f, r, s))
                img_all.append(np.asarray(img, dtype=np.uint8))
                set_ids.append(si)
                if t == T:
                    break
                obs, _, done, _ = env.step(int(rng.randint(n_actions)))
                if done:
                    planes, f, r, s = rh.obs_arrays(obs)  # the terminal state, rendered too
                    img = env.render(mode="rgb_array", scale=SCALE, draw_health=False)
                    planes_all.append(planes.astype(np.uint8))
                    scal_all.append((f, r, s))
                    img_all.append(np.asarray(img, dtype=np.uint8))
                    set_ids.append(si)
                    obs = env.reset()
    out = {
        "planes": np.stack(planes_all),
        "scalars": np.asarray(scal_all, dtype=np.uint8),
        "images": np.stack(img_all),
        "set": np.asarray(set_ids, dtype=np.uint8),
        "scale": np.int64(SCALE),
        "set_names": np.frombuffer(",".join(SETS).encode(), dtype=np.uint8),
    }
    np.savez_compressed(os.path.join(HERE, "render.npz"), **out)
    st = out["scalars"][:, 2]
    print("render.npz: %d frames (%d killed, %d starved), image %s" % (
        len(img_all), int((st == 2).sum()), int((st == 1).sum()), out["images"].shape[1:]))


if __name__ == "__main__":
    main()
