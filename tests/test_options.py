"""Host-side option handling mirrors the reference's constructor (wab_env.py:106-229)."""
import numpy as np
import pytest

from wab_gym_amd.options import default_game_options, make_config, n_actions, view_masks


def test_defaults_match_reference_dict():
    assert default_game_options["width"] == 11 and default_game_options["height"] == 11
    assert default_game_options["max_turns"] == 80
    assert default_game_options["chance_wolf_on_square"] == 0.001
    assert len(default_game_options) == 23  # wab_env.py:11-39


@pytest.mark.parametrize("w,h", [(10, 11), (11, 12), (4, 4)])
def test_even_viewport_rejected_like_reference(w, h):
    with pytest.raises(ValueError, match="odd"):
        make_config({"width": w, "height": h})


def test_action_tables():
    assert n_actions(default_game_options) == 5
    assert n_actions(dict(default_game_options, lookout_only=False)) == 6
    assert n_actions(dict(default_game_options, lookout_only=False, gatherer_only=True)) == 5


def test_none_options_map_to_random_flags():
    c, _ = make_config({"starting_food": None, "starting_role": None})
    assert c.starting_food_random == 1 and c.starting_role_random == 1


def test_view_masks():
    assert not view_masks(default_game_options).any()
    m = view_masks(dict(default_game_options, restrict_view=True))
    assert m.shape == (2, 11, 11) and m[0].sum() == 24 and m[1].sum() == 100
    assert np.array_equal(m[0], m[0][::-1]) and np.array_equal(m[1], m[1].T)
