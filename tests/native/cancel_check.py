"""Subprocess body of tests/test_cancel.py: one breakthrough self-play pool (cheap synthetic network,
tests/native/spin_check.py) is polled on a thread while the main thread watches the poll durations;
once a poll has been inside the engine for --long seconds (an NN-free root spin: the reference's
playoutMain selects finalised wins until enough evaluations accumulate) the main thread cancels the
pool (gz_pool_cancel) and times how long the poll takes to return.  Prints one JSON line."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "native"))


def main(game, games, evals, long_s, budget_s):
    from galvanise_zero_amd.defs import templates
    from galvanise_zero_amd.runner import GamePool
    from puct_harness import Setup
    from spin_check import fake_forward
    setup = Setup(game)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    pool = GamePool(setup.sm, setup.transformer, conf, games, identifier="c", seed=3, game_index_base=0)
    state = {"t0": None, "polls": 0, "rows_after_cancel": [], "samples": 0}
    cancelled = threading.Event()

    def run():
        n = 0
        while True:
            state["t0"] = time.time()
            n = pool.poll(n)
            state["t0"] = None
            state["polls"] += 1
            state["samples"] += len(pool.fetch_samples())
            if cancelled.is_set():
                state["rows_after_cancel"].append(n)
                if len(state["rows_after_cancel"]) >= 3:
                    return
                continue
            outs = fake_forward(setup.desc, pool.planes[:n])
            for dst, src in zip(pool.policies + [pool.values], outs):
                dst[:n] = src

    th = threading.Thread(target=run, daemon=True)
    th.start()
    start = time.time()
    longest = 0.0
    while time.time() - start < budget_s:
        t0 = state["t0"]
        if t0 is not None:
            longest = max(longest, time.time() - t0)
            if longest >= long_s:
                break
        time.sleep(0.01)
    tc = time.time()
    pool.cancel()
    cancelled.set()
    th.join(timeout=60)
    joined = time.time() - tc
    st = pool.stats()
    t1 = time.time()
    pool.close()
    print(json.dumps({"long_poll_s": longest, "cancel_to_return_s": joined, "alive": th.is_alive(),
                      "rows_after_cancel": state["rows_after_cancel"], "polls": state["polls"],
                      "destroy_s": time.time() - t1, "evaluations": st["evaluations"],
                      "tree_playouts": st["tree_playouts"], "samples": state["samples"]}))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), float(sys.argv[5]))
