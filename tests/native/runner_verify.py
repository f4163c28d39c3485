"""Subprocess body of tests/test_runner_verify_gpu.py: the native runner in the bench's
configuration (cfg2 6x128 bf16x3 net on the bench's weights, template self-play at 800 evals/move,
spin yield 1000, launch batching 1024 rows / 3 ms, exact-round composition) with
GZ_VERIFY_FASTPATH=1 in the environment (read once per process by the engine): every sort-free
selection, spin playout and convergence shortcut is re-run through the reference's literal path and
any difference aborts the process.  Plays for the given seconds, printing a heartbeat every 10 s
(to stderr and, when present, gpurun_out/runner_verify.log), then one JSON line of runner counters."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(seconds, threads, pools, batch):
    assert os.environ.get("GZ_VERIFY_FASTPATH") == "1"
    import bench
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.weights import random_weights, to_blob
    from galvanise_zero_amd.runner import SelfPlayRunner
    sm, transformer, desc = bench.setup_game(2)
    net = HipNet(desc, 0, "fp32")
    net.set_weights(to_blob(random_weights(desc, 7921)))
    r = SelfPlayRunner(net, sm, transformer, bench.selfplay_conf("template", 800), device=0, num_threads=threads,
                       pools_per_thread=pools, batch_size=batch, seed=20251015, spin_yield_playouts=1000,
                       min_launch_rows=1024, max_launch_wait_us=3000)
    log = os.path.join(ROOT, "gpurun_out", "runner_verify.log") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else None
    t0 = time.time()
    r.start()
    while time.time() - t0 < seconds:
        time.sleep(10)
        st = r.stats()
        line = "[verify] %.0fs rows %d games %d tree_playouts %d" % (time.time() - t0, st["rows"], st["games_completed"],
                                                                  st["tree_playouts"])
        print(line, file=sys.stderr, flush=True)
        if log:
            with open(log, "a") as f:
                f.write(line + "\n")
    r.stop()
    st = r.stats()
    r.close()
    st["seconds"] = time.time() - t0
    print(json.dumps(st), flush=True)


if __name__ == "__main__":
    main(float(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
