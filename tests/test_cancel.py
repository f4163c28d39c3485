"""Bounded teardown of a game pool (gz_pool_cancel).

The reference's playoutMain keeps selecting finalised wins until enough NN evaluations accumulate
(evaluator.cpp:744-886): a pool's poll can sit inside one game's NN-free spin for seconds to
minutes, and the reference only ever tears its workers down with the process (supervisor.cpp:36).
gz_pool_cancel, callable from another thread, makes the poll in progress return at the game's next
playout; the runner's stop and the Supervisor's workers use it.  Here a breakthrough pool with the
reference's spin behaviour (no spin yield, fast path off so spins are slow) is cancelled from the
main thread while one poll has been inside the engine for over 0.3 s."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_pool_cancel_bounds_a_spinning_poll():
    env = dict(os.environ, GZ_SPIN_FAST="0")
    env.pop("GZ_VERIFY_FASTPATH", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "native", "cancel_check.py"),
                        "breakthrough", "4", "800", "0.3", "150"], capture_output=True, text=True, env=env,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    st = json.loads(r.stdout.strip().splitlines()[-1])
    print(st)
    assert st["long_poll_s"] >= 0.3, st                  # a poll was inside a long NN-free spin
    assert st["tree_playouts"] > 20 * st["evaluations"], st
    assert not st["alive"] and st["cancel_to_return_s"] < 1.0, st
    assert st["rows_after_cancel"] == [0, 0, 0], st       # every later poll returns at once, empty
    assert st["destroy_s"] < 1.0, st
