"""A bounded runner stop.

The reference's playoutMain keeps selecting finalised wins until enough NN evaluations accumulate
(evaluator.cpp:744-886), so a game near its end can spin for minutes without an evaluation; the
reference only tears its workers down with the process (supervisor.cpp:36).  The runner hosts live
generation rolls and reconfiguration, so gz_runner_stop cancels every pool (gz_pool_cancel): an
engine thread inside a spinning game's poll returns at the game's next playout.  Here 16 slots of
hexLG13 (BASELINE cfg4's game and evals/move, one game per engine thread, the reference's
never-yielding loop: spin yield 0) run on a small net until their games reach end-of-game spins,
then the runner is stopped mid-run: the stop must return within 2 s, and the samples fetched before
it stay as they were (the stop only abandons the games in progress).
"""
import json
import time

import pytest

from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS, NetDesc
from galvanise_zero_amd.nn.weights import random_weights, to_blob

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_runner_stop_bounded_mid_spin(hip_device):
    import bench
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    sm, transformer, big = bench.setup_game(4)
    desc = NetDesc(big.input_channels, big.input_columns, big.input_rows, 64, 2, list(big.policy_dist_count))
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(to_blob(random_weights(desc, 7921)))
    r = SelfPlayRunner(net, sm, transformer, bench.selfplay_conf("template", BASELINE_CONFIGS[4]["evals"]),
                       device=hip_device, num_threads=16, pools_per_thread=1, batch_size=1, seed=77,
                       keep_samples=True, spin_yield_playouts=0)
    r.start()
    t0 = time.time()
    windows = []
    prev = r.stats()
    while time.time() - t0 < 150:
        time.sleep(5)
        st = r.stats()
        d_rows = st["rows"] - prev["rows"]
        d_tp = st["tree_playouts"] - prev["tree_playouts"]
        windows.append((d_rows, d_tp, st["games_completed"]))
        print("t %.0fs rows %d tree playouts %d games %d" % (time.time() - t0, d_rows, d_tp, st["games_completed"]),
              flush=True)
        prev = st
        # stop once games have completed and the last window was spin-dominated (NN-free playouts
        # far above evaluations: some engine threads are inside end-of-game spins)
        if st["games_completed"] >= 4 and d_tp > 50 * max(1, d_rows) and time.time() - t0 > 30:
            break
    before = r.fetch_samples()
    snapshot = json.dumps(before, sort_keys=True)
    ts = time.time()
    r.stop()
    stop_s = time.time() - ts
    after = r.fetch_samples()
    r.close()
    print("stop %.3f s; samples before %d, after %d; last window %s" % (stop_s, len(before), len(after), windows[-1]))
    assert windows[-1][1] > 50 * max(1, windows[-1][0]), windows   # the run was spinning when stopped
    assert stop_s < 2.0, stop_s
    assert json.dumps(before, sort_keys=True) == snapshot and len(before) > 0
    for s in after:
        assert set(s) == set(before[0]), s
