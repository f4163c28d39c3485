"""The bench configuration of the native runner with every engine fast path cross-checked.

The steady state the bench measures is dominated by NN-free root-spin playouts (spinBuild /
spinRun), sort-free selections, root-latch RNG draws and deferred RNG jumps,
which the oracle-replay tests reach only at low evals/move.  Here the runner plays the bench's
configuration (800 evals/move, aged past completed games) for two minutes in a child process with
GZ_VERIFY_FASTPATH=1, which re-runs the reference's literal path (evaluator.cpp:341-517, 744-886)
beside every fast-path decision and aborts on the first difference; every register-resident spin
run (spinRunRegs) is replayed from the same state through the per-playout verified loop and the two
end states compared.
Reference: src/cpp/puct/evaluator.cpp:341-517, 744-886; src/cpp/selfplay.cpp:292-337.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_runner_bench_config_fastpaths_verified(hip_device):
    env = dict(os.environ, GZ_VERIFY_FASTPATH="1")
    script = os.path.join(ROOT, "tests", "native", "runner_verify.py")
    # 6 engine threads x 2 pools x 64 games: games complete within the window (aged play)
    r = subprocess.run([sys.executable, script, "130", "6", "2", "64"], capture_output=True, text=True, env=env,
                       timeout=360)
    print(r.stderr[-2000:])
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    st = json.loads(r.stdout.strip().splitlines()[-1])
    print(st)
    # games complete in the window (aged play reaches endgames and their root spins; verification makes
    # every spin playout several times slower, so the population turns over only partly: 237 of 768
    # slots on MI355X, profiles/r03i_tests.log)
    assert st["games_completed"] >= 150, st
    assert st["tree_playouts"] - st["rows"] > 10 * st["rows"], st   # NN-free (spin) playouts ran, verified
    assert st["large_launches"] > 0, st
