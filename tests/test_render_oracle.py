"""f3: the oracle's restatement of WolvesAndBushesEnv.render (wab_env.py:468-502,
draw_health=False) against frames rendered by the reference itself (tests/golden/render.npz,
made by tests/golden/make_golden_render.py)."""
import os

import numpy as np

from oracle import oracle as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "render.npz")


def test_oracle_render_matches_reference_frames():
    z = np.load(GOLDEN)
    names = bytes(z["set_names"]).decode().split(",")
    scale = int(z["scale"])
    for si, name in enumerate(names):
        sel = z["set"] == si
        planes, sc = z["planes"][sel], z["scalars"][sel]
        img = orc.render(planes, sc[:, 1], sc[:, 2], 11, 11, restrict_view=(name == "restrict"), scale=scale)
        assert np.array_equal(img, z["images"][sel]), name
    # the frames cover the killed (127 background) and masked (restrict_view) branches
    assert (z["scalars"][:, 2] == 2).sum() > 10
    assert (z["images"] == 127).any() and (z["images"] == 0).all(axis=-1).any()
