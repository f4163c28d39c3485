"""Subprocess body of tests/test_runner_verify_gpu.py: the native runner in a bench configuration
(--config 2: the headline cfg2 6x128 bf16x3 net; 3 / 4 / 5: reversi 10x128, hexLG13 12x256 and
amazons 20x256 on their bench weights, each at its own evals/move: 800 / 1600 / 1600), template
self-play, spin yield 1000, launch batching 1024 rows / 3 ms, exact-round composition) is AGED
unverified until --age-games completed games per slot or --age-seconds (the bench ages 3 games per
slot or 400 s), then the engine's run-time verification is switched on (gz_engine_set_verify_fastpath):
from there every sort-free selection, spin playout (root-latch draws included), register spin run and
convergence shortcut is re-run through the reference's literal path, and any difference aborts the
process.  A heartbeat every 10 s goes to stderr (and gpurun_out/runner_verify.log when present); the
last stdout line is one JSON document with the aging and the verified window's counters."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--age-games", type=float, default=3.0)
    ap.add_argument("--age-seconds", type=float, default=150.0)
    ap.add_argument("--verify-seconds", type=float, default=60.0)
    ap.add_argument("--threads", type=int, default=14)
    ap.add_argument("--pools", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--evals", type=int, default=0, help="evals/move (0: the config's)")
    a = ap.parse_args()
    import bench
    from galvanise_zero_amd import _native
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.weights import random_weights, to_blob
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    from galvanise_zero_amd.runner import SelfPlayRunner
    assert not _native.set_verify_fastpath(False), "aging runs unverified (unset GZ_VERIFY_FASTPATH)"
    sm, transformer, desc = bench.setup_game(a.config)
    evals = a.evals or BASELINE_CONFIGS[a.config]["evals"]
    net = HipNet(desc, 0, "bf16x3")
    net.set_weights(to_blob(random_weights(desc, 7921)))
    r = SelfPlayRunner(net, sm, transformer, bench.selfplay_conf("template", evals), device=0, num_threads=a.threads,
                       pools_per_thread=a.pools, batch_size=a.batch, seed=20251015, spin_yield_playouts=1000,
                       min_launch_rows=1024, max_launch_wait_us=3000)
    slots = a.threads * a.pools * a.batch
    log = os.path.join(ROOT, "gpurun_out", "runner_verify.log") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else None

    def beat(tag, t0):
        st = r.stats()
        line = "[verify cfg%d %s] %.0fs rows %d games %d (%.2f per slot) tree_playouts %d verified %d" % (
            a.config, tag, time.time() - t0, st["rows"], st["games_completed"], st["games_completed"] / slots,
            st["tree_playouts"], _native.verified_decisions())
        print(line, file=sys.stderr, flush=True)
        if log:
            with open(log, "a") as f:
                f.write(line + "\n")
        return st

    t0 = time.time()
    r.start()
    st = r.stats()
    while st["games_completed"] < a.age_games * slots and time.time() - t0 < a.age_seconds:
        time.sleep(2)
        st = r.stats() if int(time.time() - t0) % 10 >= 2 else beat("aging", t0)
    aged = r.stats()
    aged_s = time.time() - t0
    v0 = _native.verified_decisions()
    _native.set_verify_fastpath(True)
    t1 = time.time()
    while time.time() - t1 < a.verify_seconds:
        time.sleep(10)
        beat("verified", t0)
    win = r.stats()
    v1 = _native.verified_decisions()
    _native.set_verify_fastpath(False)
    ts = time.time()
    r.stop()
    stop_s = time.time() - ts
    r.close()
    rows = win["rows"] - aged["rows"]
    tp = win["tree_playouts"] - aged["tree_playouts"]
    out = {"config": a.config, "evals_per_move": evals, "slots": slots, "aging_s": aged_s, "games_per_slot_before": aged["games_completed"] / slots,
           "aging_nn_free_playouts_per_leaf": (aged["tree_playouts"] - aged["rows"]) / max(1, aged["rows"]),
           "window_s": time.time() - t1, "window_rows": rows, "window_tree_playouts": tp,
           "window_nn_free_playouts_per_leaf": (tp - rows) / max(1, rows),
           "window_games_completed": win["games_completed"] - aged["games_completed"],
           "window_verified_decisions": v1 - v0,
           "stop_s": stop_s}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
