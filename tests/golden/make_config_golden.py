"""Generates tests/golden/configs.json from the REFERENCE's own config modules.

Run in the build container (the reference is not on the GPU box):
    PYTHONPATH=/root/reference/src python tests/golden/make_config_golden.py

Regenerating executes the reference's module code (third-party, untrusted): run it only in an
isolated sandbox such as this container.  The committed configs.json is the pin; no test imports
the reference.

It imports ggpzero.defs.confs / templates (py3-importable) and records every default the
self-play hot path reads: the attrs defaults of PUCTEvaluatorConfig, PUCTPlayerConfig,
SelfPlayConfig, NNModelConfig (confs.py:9-151), templates.base_puct_config() and
selfplay_config_template() (templates.py:73-129), and nn_model_config_template() for every size
hint and both feature settings (templates.py:21-71) over a transformer-shaped record of each
BASELINE game (the reference function only reads role_count, num_rows/cols/channels and
policy_dist_count from it).
"""
import json
import os
import sys

import attr

from ggpzero.defs import confs, templates

HERE = os.path.dirname(os.path.abspath(__file__))

# (game, num_rows, num_cols, num_channels, policy_dist_count) of the BASELINE configs
GAMES = [("breakthroughSmall", 6, 6, 5, [81, 81]), ("breakthrough", 8, 8, 5, [155, 155]),
         ("reversi", 8, 8, 5, [65, 65]), ("hexLG13", 13, 13, 5, [170, 171]),
         ("amazons_10x10", 10, 10, 12, [3041, 3041])]


class _Transformer(object):
    def __init__(self, rows, cols, channels, policy):
        self.role_count, self.num_rows, self.num_cols = len(policy), rows, cols
        self.num_channels, self.policy_dist_count = channels, list(policy)


def main():
    out = {"confs": {name: attr.asdict(getattr(confs, name)())
                     for name in ("PUCTEvaluatorConfig", "PUCTPlayerConfig", "SelfPlayConfig", "NNModelConfig")},
           "base_puct_config": attr.asdict(templates.base_puct_config()),
           "selfplay_config_template": attr.asdict(templates.selfplay_config_template()),
           "nn_model_config_template": {}}
    for game, rows, cols, ch, pol in GAMES:
        for hint in ("small", "medium", "large"):
            for features in (False, True):
                c = templates.nn_model_config_template(game, hint, _Transformer(rows, cols, ch, pol), features)
                out["nn_model_config_template"]["%s/%s/%d" % (game, hint, features)] = attr.asdict(c)
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote configs.json", file=sys.stderr)


if __name__ == "__main__":
    main()
