"""Sample emission in the reference's wire / on-disk format.

* :func:`encode_samples` - what the worker does to each fetched sample before sending it
  (``distributed/worker.py:162-167``): states and previous states become base64 strings.
* :func:`save_sample_data` - the server's ``gendata_<game>_<step>.json.gz`` writer
  (``distributed/server.py:293-320``): a ``GenerationSamples`` record, at most
  ``num_samples_to_train`` samples, floats written to 5 decimals, gzip.
* :func:`load_sample_data` - the reader the server and the trainer's data cache use
  (``server.py:324-330``, ``nn/datacache.py:684``).

The files carry the reference's class tags (``ggpzero.defs.datadesc``), so the reference trainer
reads them unchanged.
"""
import datetime
import gzip
import os

from .defs import datadesc
from .util import attrutil
from .util.state import encode_state


def get_date_string():
    return datetime.datetime.now().strftime("%Y/%m/%d %H:%M")


def gendata_filename(game, step):
    """server.py:293-298."""
    return "gendata_%s_%s.json.gz" % (game, step)


def encode_samples(samples):
    """worker.py:162-167: fetched Sample records -> wire form (in place, returned for chaining)."""
    out = []
    for s in samples:
        if isinstance(s, dict):
            s = datadesc.Sample(**s)
        if not isinstance(s.state, str):
            s.state = encode_state(list(s.state))
            s.prev_states = [encode_state(list(p)) for p in s.prev_states]
        out.append(s)
    return out


def make_generation_samples(game, with_generation, samples, num_samples_to_train=None, date_created=None):
    """server.py:305-313."""
    gen = datadesc.GenerationSamples()
    gen.game = game
    gen.date_created = date_created or get_date_string()
    gen.with_generation = with_generation
    n = len(samples) if num_samples_to_train is None else min(len(samples), num_samples_to_train)
    gen.num_samples = n
    gen.samples = encode_samples(samples[:n])
    return gen


def save_sample_data(directory, step, game, with_generation, samples, num_samples_to_train=None,
                     date_created=None):
    """server.py:300-320: write gendata_<game>_<step>.json.gz; returns (path, GenerationSamples)."""
    gen = make_generation_samples(game, with_generation, samples, num_samples_to_train, date_created)
    path = os.path.join(directory, gendata_filename(game, step))
    with gzip.open(path, "wb") as f:
        f.write(attrutil.attr_to_json(gen, float_fmt="%.5f").encode("utf-8"))
    return path, gen


def load_sample_data(path):
    """server.py:324-330 / datacache.py:684."""
    with gzip.open(path, "rb") as f:
        return attrutil.json_to_attr(f.read().decode("utf-8"))
