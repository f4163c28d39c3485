"""Config defaults pinned by the reference itself: tests/golden/configs.json is written by
tests/golden/make_config_golden.py from the reference's ggpzero.defs.confs / templates
(confs.py:9-151, templates.py:21-129).  Every default the engine reads must match, and the native
config structs (gz_selfplay_config via _native.make_selfplay_config) must carry them."""
import json
import os

import attr
import pytest

from galvanise_zero_amd import _native
from galvanise_zero_amd.defs import confs, templates

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "configs.json")))


def _cmp(mine, ref, path=""):
    """Every field of the reference record exists here with the same value (extra local fields
    are allowed only where documented as build extensions)."""
    for k, v in ref.items():
        assert k in mine, path + k
        if isinstance(v, dict):
            _cmp(mine[k], v, path + k + ".")
        else:
            assert mine[k] == v, (path + k, mine[k], v)


@pytest.mark.parametrize("name", ["PUCTEvaluatorConfig", "PUCTPlayerConfig", "SelfPlayConfig", "NNModelConfig"])
def test_conf_defaults(name):
    _cmp(attr.asdict(getattr(confs, name)()), GOLDEN["confs"][name])


def test_templates():
    _cmp(attr.asdict(templates.base_puct_config()), GOLDEN["base_puct_config"])
    _cmp(attr.asdict(templates.selfplay_config_template()), GOLDEN["selfplay_config_template"])


class _T(object):
    def __init__(self, rows, cols, ch, pol):
        self.role_count, self.num_rows, self.num_cols, self.num_channels = len(pol), rows, cols, ch
        self.policy_dist_count = pol


GAMES = {"breakthroughSmall": (6, 6, 5, [81, 81]), "breakthrough": (8, 8, 5, [155, 155]),
         "reversi": (8, 8, 5, [65, 65]), "hexLG13": (13, 13, 5, [170, 171]),
         "amazons_10x10": (10, 10, 12, [3041, 3041])}


def test_nn_model_config_templates():
    for key, ref in GOLDEN["nn_model_config_template"].items():
        game, hint, features = key.split("/")
        c = templates.nn_model_config_template(game, hint, _T(*GAMES[game]), bool(int(features)))
        _cmp(attr.asdict(c), ref, key + ":")


def test_native_selfplay_config_carries_template():
    """The C struct the engine runs on (gz_selfplay_config) holds the template's values."""
    ref = GOLDEN["selfplay_config_template"]
    c = _native.make_selfplay_config(templates.selfplay_config_template())
    for k, v in ref.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                if hasattr(getattr(c, k), kk) and not isinstance(vv, str):
                    assert getattr(getattr(c, k), kk) == pytest.approx(float(vv), rel=1e-6), (k, kk)
            assert getattr(c, k).choose == {"choose_top_visits": 0, "choose_temperature": 1}[v["choose"]]
        elif hasattr(c, k) and not isinstance(v, str):
            assert getattr(c, k) == pytest.approx(float(v), rel=1e-6), k
