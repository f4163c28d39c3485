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


@pytest.mark.timeout(300)
def test_supervisor_cancel_ends_poll_loop():
    """cppinterface.Supervisor.cancel() (gz_supervisor_cancel) from another thread ends a
    poll_loop() whose worker pools are busy -- the reference's Supervisor has no such call (its
    workers end with the process) -- and the supervisor tears down promptly afterwards."""
    import threading
    import time
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests", "native"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from galvanise_zero_amd import cppinterface
    from galvanise_zero_amd.defs import templates
    from puct_harness import Setup
    from spin_check import fake_forward
    setup = Setup("breakthrough")

    class Model(object):
        def predict_on_batch(self, x):
            return fake_forward(setup.desc, np.asarray(x, dtype=np.float32))

    class NN(object):
        gdl_bases_transformer = setup.transformer

        def get_model(self):
            return Model()

    conf = templates.selfplay_config_template()
    conf.evals_per_move = 400
    sup = cppinterface.Supervisor(setup.sm, NN(), batch_size=8, seed=2, per_pool_unique_states=True)
    sup.start_self_play(conf, 2)
    done = {}

    def loop():
        sup.poll_loop()
        done["t"] = time.time()

    th = threading.Thread(target=loop, daemon=True)
    th.start()
    time.sleep(5.0)
    assert th.is_alive()                          # self-play runs forever until cancelled
    t0 = time.time()
    sup.cancel()
    th.join(timeout=30)
    assert not th.is_alive() and done["t"] - t0 < 2.0, done
    assert sup.poll() is None                     # every later poll returns at once, empty
    st = sup.stats()
    assert st["evaluations"] > 0, st
    t1 = time.time()
    del sup
    assert time.time() - t1 < 2.0
