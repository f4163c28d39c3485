"""JSON (de)serialisation of attrs records with class tags (reference src/ggpzero/util/attrutil.py).

The reference tags every nested attrs object with ``"<key>__clz__": [module, class]`` and every list
of attrs objects with ``"<key>__clzlist__"`` (attrutil.py:34-91), wrapped as ``{"obj": ...}``
(attrutil.py:94-97), and only rebuilds registered classes (attrutil.py:16-31).  The module written
into the tags here is the reference's (``ggpzero.defs.datadesc`` ...), not this package's, so a file
written by :func:`attr_to_json` loads with the reference's ``json_to_attr`` and vice versa.
"""
import json

import attr

# wire name (reference module, class) <-> local class
_by_wire = {}
_by_class = {}


class SerialiseException(Exception):
    pass


def register_attrs(wire_module):
    """Class decorator: register an attrs class under the reference's module name."""
    def deco(clz):
        key = (wire_module, clz.__name__)
        _by_wire[key] = clz
        _by_class[clz] = key
        return clz
    return deco


def _get_clz(mod, name):
    # attrutil.py:21-31 (legacy names from ggpzero.defs.confs)
    if mod == "ggpzero.defs.confs" and name == "Generation":
        mod, name = "ggpzero.defs.datadesc", "GenerationSamples"
    if mod == "ggpzero.defs.confs" and name == "Sample":
        mod = "ggpzero.defs.datadesc"
    try:
        return _by_wire[(mod, name)]
    except KeyError:
        raise SerialiseException("Attempt to create an unregistered class: %s / %s" % (mod, name))


def _wire(obj):
    try:
        return list(_by_class[obj.__class__])
    except KeyError:
        raise SerialiseException("Attempt to serialise unregistered class: %s" % obj.__class__.__name__)


def _to_plain(obj):
    """attrs object -> dict with __clz__/__clzlist__ tags (attrutil.py:58-91)."""
    out = {}
    for a in attr.fields(obj.__class__):
        k, v = a.name, getattr(obj, a.name)
        if isinstance(v, (list, tuple)) and any(attr.has(i) for i in v):
            if sum(issubclass(type(i), type(v[0])) for i in v) != len(v):
                raise SerialiseException("Bad list %s" % (v,))
            out[k + "__clzlist__"] = _wire(v[0])
            out[k] = [_to_plain(i) for i in v]
        elif attr.has(v):
            out[k + "__clz__"] = _wire(v)
            out[k] = _to_plain(v)
        elif isinstance(v, tuple):
            out[k] = list(v)
        else:
            out[k] = v
    return out


def _from_plain(d):
    """attrutil.py:100-133."""
    for k in list(d.keys()):
        if k.endswith("__clz__"):
            clz = _get_clz(*d.pop(k))
            name = k[:-len("__clz__")]
            d[name] = clz(**_from_plain(d[name]))
        elif k.endswith("__clzlist__"):
            clz = _get_clz(*d.pop(k))
            name = k[:-len("__clzlist__")]
            d[name] = [clz(**_from_plain(i)) for i in d[name]]
    return d


def _round_floats(o, fmt):
    """server.py:316 sets json FLOAT_REPR to '%.5f' before writing sample files; Python 3's encoder
    has no such hook, so floats are rounded through the format instead (same values on reading)."""
    if isinstance(o, float):
        return o if (o != o or o in (float("inf"), float("-inf"))) else float(fmt % o)
    if isinstance(o, dict):
        return {k: _round_floats(v, fmt) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_round_floats(v, fmt) for v in o]
    return o


def attr_to_json(obj, float_fmt=None, **kwds):
    """attrutil.py:143-151 (pretty=True -> sorted keys, indent 4)."""
    assert attr.has(obj)
    if kwds.pop("pretty", False):
        kwds.update(sort_keys=True, separators=(",", ": "), indent=4)
    doc = {"obj__clz__": _wire(obj), "obj": _to_plain(obj)}
    if float_fmt is not None:
        doc = _round_floats(doc, float_fmt)
    return json.dumps(doc, **kwds)


def json_to_attr(buf, **kwds):
    """attrutil.py:154-156."""
    d = _from_plain(json.loads(buf, **kwds))
    assert "obj" in d and len(d) == 1
    return d["obj"]


def clone(obj):
    return json_to_attr(attr_to_json(obj))
