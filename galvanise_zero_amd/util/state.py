"""Wire encoding of base states in samples (reference src/ggpzero/util/state.py:7-39).

A state is the tuple of base bits (0/1, propnet base order).  ``encode_state`` packs the bits
MSB-first into bytes (numpy ``packbits``) and base64-encodes them with the MIME line breaks of
Python 2's ``base64.encodestring`` (= ``base64.encodebytes``: a newline after every 76 characters
and at the end), so the strings are byte-identical to the ones the reference worker puts on the
wire (``worker.py:162-167``) and into ``gendata_*.json.gz``.  ``decode_state`` returns the bits
padded to a multiple of 8, as the reference's does (state.py:24-27).
"""
import base64

import numpy as np


def encode_state(s):
    """state.py:7-12."""
    assert isinstance(s, (list, tuple))
    a = np.asarray(s, dtype=np.uint8)
    return base64.encodebytes(np.packbits(a).tobytes()).decode("ascii")


def decode_state(s):
    """state.py:15-28: tuples/lists pass through; strings decode to a bit tuple (length rounded
    up to a multiple of 8)."""
    if isinstance(s, tuple):
        return s
    if isinstance(s, list):
        return tuple(s)
    if isinstance(s, str):
        s = s.encode("ascii")
    aa = np.frombuffer(base64.decodebytes(s), dtype=np.uint8)
    return tuple(int(b) for b in np.unpackbits(aa))


def fast_decode_state(s):
    """state.py:31-39 (``buf_to_tuple_reverse_bytes``): same bits as decode_state."""
    return decode_state(s)


def state_from_words(words, num_bases):
    """Native engine state (uint64 words, bit i of the state in word i//64, bit i%64) -> bit tuple."""
    w = np.asarray(words, dtype=np.uint64)
    bits = np.unpackbits(w.view(np.uint8), bitorder="little")
    return tuple(int(b) for b in bits[:num_bases])
