"""Sample emission format: base64 state encoding (util/state.py:7-39), attrutil JSON
class tags (util/attrutil.py:34-156) and the gendata_<game>_<step>.json.gz writer
(distributed/server.py:293-330), checked against a document the reference's own attrutil wrote
(tests/golden/gendata_ref.json, made by tests/golden/make_gendata_golden.py)."""
import gzip
import json
import os

import numpy as np
import pytest

from galvanise_zero_amd import gendata
from galvanise_zero_amd.defs import datadesc
from galvanise_zero_amd.util import attrutil
from galvanise_zero_amd.util.state import decode_state, encode_state, state_from_words

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "gendata_ref.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_encode_state_matches_reference_strings(golden):
    gen = attrutil.json_to_attr(golden["json"])
    assert isinstance(gen, datadesc.GenerationSamples)
    for s, (bits, prev) in zip(gen.samples, golden["bits"]):
        assert isinstance(s, datadesc.Sample)
        assert encode_state(bits) == s.state
        assert encode_state(prev) == s.prev_states[0]
        padded = tuple(bits) + (0,) * (-len(bits) % 8)
        assert decode_state(s.state) == padded


def test_reference_document_roundtrips_identically(golden):
    """Our writer re-emits the reference writer's document exactly (the reference's reader,
    attrutil.py:100-133, is Python-2 only: it mutates a dict while iterating d.keys())."""
    gen = attrutil.json_to_attr(golden["json"])
    assert json.loads(attrutil.attr_to_json(gen)) == json.loads(golden["json"])


def test_gendata_file_roundtrip(tmp_path, golden):
    bits = golden["bits"]
    samples = [datadesc.Sample(state=b[0], prev_states=[b[1]], policies=[[(1, 0.123456789), (5, 0.876543211)], []],
                               final_score=[1.0, 0.0], depth=i, game_length=30, match_identifier="g_%d" % i,
                               resultant_puct_score=[0.5, 0.5], resultant_puct_visits=800)
               for i, b in enumerate(bits)]
    path, gen = gendata.save_sample_data(str(tmp_path), 7, "breakthrough", "x6_7", samples, num_samples_to_train=2)
    assert os.path.basename(path) == "gendata_breakthrough_7.json.gz"
    raw = json.loads(gzip.open(path).read())
    assert raw["obj__clz__"] == ["ggpzero.defs.datadesc", "GenerationSamples"]
    assert raw["obj"]["samples__clzlist__"] == ["ggpzero.defs.datadesc", "Sample"]
    back = gendata.load_sample_data(path)
    assert back.num_samples == 2 and len(back.samples) == 2
    assert back.samples[0].state == encode_state(bits[0][0])
    assert back.samples[0].policies[0][0] == [1, 0.12346]          # server.py:316 '%.5f'


def test_state_from_engine_words():
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 2, size=130)
    words = np.zeros(3, dtype=np.uint64)
    for i, b in enumerate(bits):
        if b:
            words[i // 64] |= np.uint64(1) << np.uint64(i % 64)
    assert state_from_words(words, 130) == tuple(int(b) for b in bits)


def test_engine_samples_to_gendata(tmp_path):
    """Samples fetched from the native supervisor (CPU oracle forward) go through the worker's
    encoding and the server's writer, and decode back to the engine's own state bits."""
    from puct_harness import Setup, run_native_supervisor
    from galvanise_zero_amd.defs import templates
    setup = Setup("breakthroughSmall")
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 16
    _, samples, _, keep = run_native_supervisor(setup, conf, 4, 1500, seed=5)
    assert len(samples) > 0
    recs = [datadesc.Sample(**s) for s in samples]
    raw_states = [list(r.state) for r in recs]
    path, _ = gendata.save_sample_data(str(tmp_path), 0, "breakthroughSmall", "b1_0", recs)
    back = gendata.load_sample_data(path)
    assert back.num_samples == len(samples)
    for s, bits in zip(back.samples, raw_states):
        dec = decode_state(s.state)
        assert list(dec[:len(bits)]) == [int(b) for b in bits]
        assert s.match_identifier and len(s.policies) == 2
