"""The engine's deferred RNG jump (rng.h Rng::discard) against single steps, compiled on the host."""
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rng_discard_equals_single_steps():
    src = os.path.join(ROOT, "tests", "native", "rng_jump_check.cpp")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "rng_jump_check")
        subprocess.check_call(["g++", "-O2", "-std=c++17", src, "-o", exe])
        out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "0 mismatches" in out.stdout
