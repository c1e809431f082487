"""f3: the oracle's restatement of WolvesAndBushesEnv.render (wab_env.py:468-502, with and
without the draw_health text) against frames rendered by the reference itself
(tests/golden/render.npz, made by tests/golden/make_golden_render.py), and the baked digit
glyphs (wab_glyphs.h) against PIL's own text drawing."""
import os
import re

import numpy as np

from oracle import oracle as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "render.npz")


def _opts(name):
    return {"restrict": {"restrict_view": True, "lookout_only": False},
            "longfood": {"turns_to_empty_food": 150}}.get(name, {})


def test_oracle_render_matches_reference_frames():
    z = np.load(GOLDEN)
    names = bytes(z["set_names"]).decode().split(",")
    scale = int(z["scale"])
    for si, name in enumerate(names):
        sel = z["set"] == si
        planes, sc = z["planes"][sel], z["scalars"][sel]
        rv = name == "restrict"
        img = orc.render(planes, sc[:, 1], sc[:, 2], 11, 11, restrict_view=rv, scale=scale)
        assert np.array_equal(img, z["images"][sel]), name
        img = orc.render(planes, sc[:, 1], sc[:, 2], 11, 11, restrict_view=rv, scale=scale, food_turns=sc[:, 0],
                         draw_health=True)
        assert np.array_equal(img, z["images_health"][sel]), name
        big = np.nonzero(sel[z["big_idx"]])[0]
        bi = z["big_idx"][big]
        for s2, key in ((32, "images_health32"), (1, "images_health1")):
            img = orc.render(z["planes"][bi], z["scalars"][bi, 1], z["scalars"][bi, 2], 11, 11, restrict_view=rv,
                             scale=s2, food_turns=z["scalars"][bi, 0], draw_health=True)
            assert np.array_equal(img, z[key][big]), (name, s2)
    # three-digit counts are covered
    assert z["scalars"][:, 0].max() >= 100
    # the frames cover the killed (127 background) and masked (restrict_view) branches
    assert (z["scalars"][:, 2] == 2).sum() > 10
    assert (z["images"] == 127).any() and (z["images"] == 0).all(axis=-1).any()


def test_glyph_table_matches_pil():
    """wab_glyphs.h is what tools/make_glyphs.py derives from this image's PIL, and every
    count 0..255 renders as its digits side by side (the kernels' composition rule)."""
    import importlib.util

    import pytest

    pytest.importorskip("PIL")
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("make_glyphs", os.path.join(here, "tools", "make_glyphs.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    r0, g = mg.glyph_table()
    mg.check(r0, g)
    text = open(os.path.join(here, "wab_gym_amd", "csrc", "wab_glyphs.h")).read()
    data = re.sub(r"/\*.*?\*/", " ", text.split("#define WAB_GLYPH_DATA")[1]).replace("\\", " ")
    vals = [int(v) for v in data.replace(",", " ").split()]
    assert "#define WAB_GLYPH_ROW0 %d " % r0 in text and "#define WAB_GLYPH_ROWS %d\n" % g.shape[1] in text
    assert vals == [int(v) for v in g.reshape(-1)]
