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
