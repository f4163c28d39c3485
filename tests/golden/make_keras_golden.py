"""Generates tests/golden/keras_descs.json from every model file of the reference
(data/<game>/models/*.json): the NetDesc the importer reads (or the NotSupported reason), each
supported file's per-layer Keras weight shapes, and its layer graph (class, name, the config keys a
Keras-JSON reader needs, inbound layers) so the import and forward tests run where the reference is
not mounted.  Run in the build container:  python tests/golden/make_keras_golden.py"""
import dataclasses
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from galvanise_zero_amd.nn import keras_model as K  # noqa: E402

CONFIG_KEYS = ("batch_input_shape", "data_format", "filters", "kernel_size", "use_bias", "units", "activation",
               "epsilon", "target_shape", "dims", "axis", "alpha", "padding", "rate")


def skeleton(path):
    with open(path) as f:
        doc = json.load(f)
    layers = []
    for l in doc["config"]["layers"]:
        nodes = l.get("inbound_nodes") or []
        layers.append({"class_name": l["class_name"], "name": l["name"],
                       "config": {k: l["config"][k] for k in CONFIG_KEYS if k in l["config"]},
                       "inbound_nodes": [[[n[0], 0, 0, {}] for n in nodes[0]]] if nodes else []})
    return {"class_name": doc["class_name"], "config": {"layers": layers}}


def main():
    out = {}
    for f in sorted(glob.glob("/root/reference/data/*/models/*.json")):
        key = f.split("/data/")[1]
        try:
            d = K.desc_from_keras_json(f)
            out[key] = {"desc": dataclasses.asdict(d),
                        "layers": {n: [list(s) for s in shapes] for n, shapes in K.keras_layer_shapes(f).items()},
                        "graph": skeleton(f)}
        except K.NotSupported as e:
            out[key] = {"not_supported": str(e)}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "keras_descs.json")
    with open(path, "w") as fo:
        json.dump(out, fo, indent=None, sort_keys=True, separators=(",", ":"))
    print("wrote", path, len(out))


if __name__ == "__main__":
    main()
