"""lookup_transpositions (reference PuctConfig option, evaluator.cpp:144-163, 216-239; off in the
reference's self-play templates, confs.py:73) under AddressSanitizer.

A transposed node gets a second parent; when its first parent's subtree is released the surviving
node must drop its mirror entry and parent pointer into the freed node (evaluator.cpp detachEdge).
Without that, the next backup through the node writes into freed memory (ASan: heap-use-after-free
in PuctNode::syncParent).  CPU only: the engine sources and tests/native/transposition_check.cpp are
compiled with -fsanitize=address and driven by a synthetic network."""
import glob
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def asan_binary(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("asan") / "transposition_check")
    srcs = [os.path.join(ROOT, "tests", "native", "transposition_check.cpp")] + \
        sorted(glob.glob(os.path.join(ROOT, "galvanise_zero_amd", "csrc", "engine", "*.cpp")))
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", "-pthread",
           "-fsanitize=address", "-fno-omit-frame-pointer", "-o", out] + srcs
    subprocess.check_call(cmd)
    return out


@pytest.mark.parametrize("game,polls", [("breakthrough", 4000), ("breakthroughSmall", 3000)])
def test_transpositions_no_use_after_free(asan_binary, game, polls):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([asan_binary, game, "16", str(polls), "64"], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    st = json.loads(r.stdout.strip().splitlines()[-1])
    print(game, st)
    assert st["transpositions"] > 0 and st["games_completed"] > 0, st
