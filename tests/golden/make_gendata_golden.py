"""Generates tests/golden/gendata_ref.json: a GenerationSamples document serialised by the
reference's own attrutil (src/ggpzero/util/attrutil.py:143-151) from the reference's own datadesc
records (src/ggpzero/defs/datadesc.py:7-52), with states encoded as util/state.py:7-12 does
(base64.encodestring == base64.encodebytes of np.packbits).  Run in the build container (the
reference is mounted there, not on the GPU box):  python tests/golden/make_gendata_golden.py"""
import base64
import json
import os
import sys

import numpy as np

sys.path.insert(0, "/root/reference/src")
from ggpzero.defs import datadesc            # noqa: E402  (reference, py3-importable)
from ggpzero.util import attrutil            # noqa: E402


def enc(bits):
    return base64.encodebytes(np.packbits(np.array(bits)).tobytes()).decode("ascii")


def main():
    rng = np.random.default_rng(4242)
    samples, bits = [], []
    for i in range(3):
        state = [int(b) for b in rng.integers(0, 2, size=130)]   # breakthrough: 130 bases
        prev = [int(b) for b in rng.integers(0, 2, size=130)]
        pol = [[[int(m), round(float(p), 5)] for m, p in zip(rng.choice(155, 5, replace=False),
                                                               rng.dirichlet(np.ones(5)))], []]
        samples.append(datadesc.Sample(state=enc(state), prev_states=[enc(prev)], policies=pol,
                                       final_score=[1.0, 0.0] if i % 2 else [0.0, 1.0], depth=7 + i,
                                       game_length=40 + i, match_identifier="m_%d" % i,
                                       has_resigned=bool(i == 2), resign_false_positive=False,
                                       starting_sample_depth=3, resultant_puct_score=[0.61, 0.39],
                                       resultant_puct_visits=800))
        bits.append([state, prev])
    gen = datadesc.GenerationSamples(game="breakthrough", date_created="2025/10/15 12:00",
                                     with_generation="x6_1", num_samples=3, samples=samples)
    doc = attrutil.attr_to_json(gen, pretty=False)
    out = {"json": doc, "bits": bits}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gendata_ref.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path, len(doc))


if __name__ == "__main__":
    main()
