"""The drop-in boundary: both C-ABI libraries load on a host without a GPU and export every function
their header declares (include/gzero_engine.h -> libgz_engine.so, include/gzero_nn.h ->
libgz_nn.so).  No compute calls are made."""
import ctypes
import os
import re
import subprocess

import pytest

from galvanise_zero_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAIRS = [("gzero_engine.h", "libgz_engine.so"), ("gzero_nn.h", "libgz_nn.so")]


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set()
    for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(gz_\w+)\s*\(", text, flags=re.M):
        names.add(m.group(1))
    return names


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.mark.parametrize("header,lib", PAIRS)
def test_library_exports_every_declared_function(header, lib):
    path = _native.lib_path(lib)
    assert os.path.exists(path), "build the libraries first (__graft_entry__.build())"
    names = declared(header)
    assert len(names) > 10
    missing = sorted(names - exported(path))
    assert not missing, missing


@pytest.mark.parametrize("header,lib", PAIRS)
def test_library_loads_and_resolves(header, lib):
    so = ctypes.CDLL(_native.lib_path(lib))
    for name in declared(header):
        assert getattr(so, name) is not None


@pytest.mark.parametrize("hw,precision,ok", [((21, 21), "bf16", False), ((19, 19), "bf16x3", True), ((19, 19), "bf16", True),
                                              ((13, 13), "bf16x3", True)])
def test_net_geometry_check(hw, precision, ok):
    """gz_net_create checks the board against the compiled kernels before any HIP call (so this runs
    without a GPU): boards up to 19 x 19 (23 position tiles) are accepted -- the reference's hex19
    net among them --, larger ones are refused with a clear error instead of failing at launch."""
    import json
    from galvanise_zero_amd.nn.desc import NetDesc
    with open(os.path.join(ROOT, "tests", "golden", "keras_descs.json")) as f:
        base = json.load(f)["hex19/models/h2_477.json"]["desc"]
    desc = NetDesc(**dict(base, input_columns=hw[0], input_rows=hw[1]))
    lib = _native.nn_lib()
    cdesc = _native.make_net_desc(desc, _native.PRECISIONS[precision])
    # geometry is checked first; past it gz_net_create needs a device, which this host lacks
    h = lib.gz_net_create(ctypes.byref(cdesc), 0)
    err = lib.gz_nn_last_error().decode()
    if h:
        lib.gz_net_destroy(h)
    if ok:
        assert "unsupported network geometry" not in err, err
    else:
        assert not h and "unsupported network geometry F=80 H=21 W=21" in err, err


def test_precision_names():
    """The split mode is named for what it computes: "bf16x3" (alias "split"),
    three bf16 MFMAs per product -- fp32-class, not IEEE fp32; the pre-round-6 name "fp32" still
    selects it, with a DeprecationWarning.  Both map to the same gz_net_desc.precision."""
    import warnings
    assert _native.PRECISIONS["bf16x3"] == _native.PRECISIONS["split"] == _native.PRECISIONS["fp32"] \
        == _native.GZ_PRECISION_SPLIT != _native.PRECISIONS["bf16"]
    assert _native.canonical_precision("bf16x3") == _native.canonical_precision("split") == "bf16x3"
    assert _native.canonical_precision("bf16") == "bf16"
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert _native.canonical_precision("fp32") == "bf16x3"
    assert any(issubclass(x.category, DeprecationWarning) and "bf16x3" in str(x.message) for x in w)
    with pytest.raises(ValueError):
        _native.canonical_precision("fp16")
