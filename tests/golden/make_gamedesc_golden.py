"""Generates tests/golden/gamedesc.json from the REFERENCE's own ggpzero.defs.gamedesc.

Run in the build container only (the reference is not on the GPU box):
    PYTHONPATH=/root/reference/src python tests/golden/make_gamedesc_golden.py

Regenerating executes the reference's module code (third-party, untrusted): run it only in an
isolated sandbox such as this container.  The committed gamedesc.json is the pin; tests never
import the reference.

Records attr.asdict(Games().<game>()) (gamedesc.py:142-239, 309-318) for the five BASELINE games
and bt_7: the board channels (base term, coordinate term indices, piece terms), the control
channels (the GDL bases and the value each flood-fills) and the coordinate lists whose lengths are
the planes' H and W (bases.py:104-121).  These decide the planes geometry and control values of
SURVEY 8 row A5.
"""
import json
import os

import attr

from ggpzero.defs import gamedesc

HERE = os.path.dirname(os.path.abspath(__file__))
GAMES = ["breakthrough", "breakthroughSmall", "reversi", "hexLG13", "amazons_10x10", "bt_7"]


def main():
    g = gamedesc.Games()
    out = {name: attr.asdict(getattr(g, name)()) for name in GAMES}
    with open(os.path.join(HERE, "gamedesc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", len(out), "game descriptions")


if __name__ == "__main__":
    main()
