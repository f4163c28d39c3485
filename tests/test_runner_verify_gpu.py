"""The bench configuration of the native runner, aged to the bench's regime, then every engine fast
path cross-checked.

The steady state the bench measures (three completed games per slot) is dominated by NN-free
root-spin playouts (spinBuild / spinRun / spinRunRegs), sort-free selections, root-latch RNG draws
and deferred RNG jumps, which the oracle-replay tests reach only at low
evals/move.  Here, in a child process, the runner plays the bench's configuration (800 evals/move)
UNVERIFIED until three games per slot have completed, then switches the engine's run-time
verification on (gz_engine_set_verify_fastpath): every fast-path decision is re-made by the
reference's literal path (evaluator.cpp:341-517, 744-886) and every register spin run is replayed
through the per-playout verified loop from the same state; the first difference aborts the child.
Reference: src/cpp/puct/evaluator.cpp:341-517, 744-886; src/cpp/selfplay.cpp:292-337.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# config -> (runner_verify.py arguments, minimum NN-free playouts per leaf in the verified window).
# cfg2: the headline's window (three games per slot, 800 evals/move, bench's weights).  cfg3-5: the
# bench's own slot layout (2 pools x 256 games per engine thread) and evals/move (reversi 800,
# hexLG13 / amazons 1600) on each config's bench weights, aged by time as the bench ages them (the
# bench: 3 games per slot or 400 s; hexLG13 and amazons complete no game inside it), then verified.
CASES = {
    2: (["--age-games", "3", "--age-seconds", "200", "--verify-seconds", "75"], 300),
    3: (["--config", "3", "--batch", "256", "--age-games", "3", "--age-seconds", "120", "--verify-seconds", "45"], 20),
    4: (["--config", "4", "--batch", "256", "--age-games", "3", "--age-seconds", "100", "--verify-seconds", "45"], -0.01),
    5: (["--config", "5", "--batch", "256", "--age-games", "3", "--age-seconds", "100", "--verify-seconds", "45"], -0.01),
}
# (hexLG13 / amazons in the bench's regime are a few moves into their games: no playout is NN-free
# yet -- no terminal node is in reach --, so what runs verified there is the sort-free selection, the
# top-visits / convergence shortcuts and the root-latch draws; the spin paths are verified in cfg2 / cfg3
# and, for these games, through the oracle replays of complete games, tests/test_runner_deep_gpu.py.
# Rows counted at launch run slightly ahead of completed playouts, hence the small negative floor.)


@pytest.mark.timeout(420)
@pytest.mark.parametrize("config", sorted(CASES), ids=["cfg%d" % c for c in sorted(CASES)])
def test_runner_aged_fastpaths_verified(config, hip_device):
    args, nn_free_min = CASES[config]
    env = dict(os.environ)
    env.pop("GZ_VERIFY_FASTPATH", None)
    script = os.path.join(ROOT, "tests", "native", "runner_verify.py")
    r = subprocess.run([sys.executable, script] + args, capture_output=True, text=True, env=env, timeout=400)
    print(r.stderr[-3000:])
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    st = json.loads(r.stdout.strip().splitlines()[-1])
    print(st)
    if config == 2:
        assert st["games_per_slot_before"] >= 3.0, st             # the bench's window age
        assert st["window_games_completed"] > 0, st
    else:
        assert st["aging_s"] >= 90 or st["games_per_slot_before"] >= 3.0, st
    assert st["window_verified_decisions"] > 1e6, st              # the window ran verified
    assert st["window_nn_free_playouts_per_leaf"] >= nn_free_min, st
    assert st["stop_s"] < 5.0, st                                 # bounded stop (gz_pool_cancel)
