"""Golden vectors for the batched renderer: the reference `WolvesAndBushesEnv.render`
(wab_env.py:468-502), on states reached by the reference itself.

Container-only (imports /root/reference through ref_harness).  For a few option sets, each
env takes random actions; after every step (and reset) we record the observation (planes,
scalars) and the reference's rgb_array at scale 2, both without (`images`) and with
(`images_health`) the `draw_health=True` food-count text, its default.  Every BIG_EVERY-th
frame is also rendered with the text at scale 32 (the reference's default) and scale 1
(where the text covers several cells and is clipped).  The text uses PIL's default font:
this container's Pillow 12.2 (FreeType), not the pinned 7.2's bitmap font, so font parity
with the pinned reference is unpinned; the frames pin the device renderer against the
reference's own drawing code under this Pillow.

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
BIG_EVERY = 12
SETS = {
    # name: (options override, env ids, steps)
    "default": ({}, list(range(2000, 2006)), 60),
    "restrict": ({"restrict_view": True, "lookout_only": False}, list(range(2100, 2106)), 60),
    "wolfy": ({"chance_wolf_on_square": 0.03, "wolf_chance_to_despawn": 0.2, "wolf_spawn_margin": 2},
              list(range(2200, 2206)), 60),
    # three-digit food counts (turns_to_empty_food >= 100)
    "longfood": ({"turns_to_empty_food": 150, "max_turns": 200}, list(range(2300, 2303)), 60),
}


def main():
    wab_env = rh.load_reference()
    planes_all, scal_all, img_all, set_ids = [], [], [], []
    health_all, big_idx, health32, health1 = [], [], [], []

    def record(env, obs, si):
        planes, f, r, s = rh.obs_arrays(obs)
        planes_all.append(planes.astype(np.uint8))
        scal_all.append((f, r, s))
        img_all.append(np.asarray(env.render(mode="rgb_array", scale=SCALE, draw_health=False), dtype=np.uint8))
        health_all.append(np.asarray(env.render(mode="rgb_array", scale=SCALE, draw_health=True), dtype=np.uint8))
        if len(img_all) % BIG_EVERY == 1:
            big_idx.append(len(img_all) - 1)
            health32.append(np.asarray(env.render(mode="rgb_array"), dtype=np.uint8))  # scale 32, text: defaults
            health1.append(np.asarray(env.render(mode="rgb_array", scale=1, draw_health=True), dtype=np.uint8))
        set_ids.append(si)

    for si, (name, (opts, env_ids, T)) in enumerate(SETS.items()):
        full = dict(wab_env.default_game_options)
        full.update(opts)
        rng = np.random.RandomState(17 + si)
        for g in env_ids:
            env = rh.make_env(SEED, g, full)
            obs = env.reset()
            n_actions = env.action_space.n
            for t in range(T + 1):
                record(env, obs, si)
                if t == T:
                    break
                obs, _, done, _ = env.step(int(rng.randint(n_actions)))
                if done:
                    record(env, obs, si)  # the terminal state, rendered too
                    obs = env.reset()
    out = {
        "planes": np.stack(planes_all),
        "scalars": np.asarray(scal_all, dtype=np.uint8),
        "images": np.stack(img_all),
        "images_health": np.stack(health_all),
        "big_idx": np.asarray(big_idx, dtype=np.int64),
        "images_health32": np.stack(health32),
        "images_health1": np.stack(health1),
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
