"""Generates tests/golden/keras_v1_descs.json: the NetDesc the importer reads from every v1 model
file of the reference (data/<game>/models/*.json) and the NotSupported reason for the others,
plus each v1 file's per-layer Keras weight shapes.  Run in the build container (the reference is
mounted there, not on the GPU box):  python tests/golden/make_keras_golden.py"""
import dataclasses
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from galvanise_zero_amd.nn import keras_model as K  # noqa: E402


def main():
    out = {}
    for f in sorted(glob.glob("/root/reference/data/*/models/*.json")):
        key = f.split("/data/")[1]
        try:
            d = K.desc_from_keras_json(f)
            out[key] = {"desc": dataclasses.asdict(d),
                        "layers": {n: [list(s) for s in shapes] for n, shapes in K.keras_layer_shapes(f).items()}}
        except K.NotSupported as e:
            out[key] = {"not_supported": str(e)}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "keras_v1_descs.json")
    with open(path, "w") as fo:
        json.dump(out, fo, indent=1, sort_keys=True)
    print("wrote", path, len(out))


if __name__ == "__main__":
    main()
