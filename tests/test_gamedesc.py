"""galvanise_zero_amd/defs/gamedesc.py against the reference's own game descriptions
(tests/golden/gamedesc.json, written by tests/golden/make_gamedesc_golden.py from the reference's
ggpzero.defs.gamedesc, gamedesc.py:142-239, 309-318): board channels, control channels and
coordinates -- the planes geometry and control values of SURVEY 8 row A5 -- field for field."""
import json
import os

import attr
import pytest

from galvanise_zero_amd.defs import gamedesc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gamedesc.json")
with open(GOLDEN) as _f:
    REF = json.load(_f)


@pytest.mark.parametrize("game", sorted(REF))
def test_gamedesc_matches_reference(game):
    mine = attr.asdict(getattr(gamedesc.Games(), game)())
    assert mine == REF[game]


def test_planes_geometry_from_gamedesc():
    """Channel counts and board shape implied by the descriptions (num_previous_states = 1):
    C = channels_per_state * 2 + controls."""
    expect = {"breakthrough": (5, 8, 8), "breakthroughSmall": (5, 6, 6), "reversi": (5, 8, 8),
              "hexLG13": (5, 13, 13), "amazons_10x10": (12, 10, 10)}
    for game, (c, h, w) in expect.items():
        d = REF[game]
        per_state = 0
        for bc in d["board_channels"]:
            n = 1
            for bt in bc["board_terms"]:
                n *= len(bt["terms"])
            per_state += n
        assert per_state * 2 + len(d["control_channels"]) == c, game
        assert (len(d["y_cords"]), len(d["x_cords"])) == (h, w), game
