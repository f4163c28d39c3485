"""Host-only self-play probe for any BASELINE config (no GPU): the drop-in cppinterface.Supervisor with
C++ worker threads runs the config's template self-play while the poll loop answers every batch with a
synthetic network -- per row a softmax over random logits (scaled by --logit-scale: large scales give the
saturated policies of the bench's random deep nets) and a random value head.  Prints the engine's rate,
NN-free playouts per leaf and, with GZ_SPIN_STATS=1 in the environment, the engine's spin / exit
counters at exit.  Diagnostics only (the search's cost structure per game), not a parity tool.

  GZ_SPIN_STATS=1 python tools/host_probe.py --config 3 --seconds 120 --workers 7 --batch 64
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--workers", type=int, default=7)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--evals", type=int, default=0, help="evals/move (0: the config's)")
    ap.add_argument("--logit-scale", type=float, default=3.0)
    ap.add_argument("--report", type=float, default=10)
    a = ap.parse_args()
    if os.environ.get("GZ_SPROF_LIB"):   # host sampling profiler (tools/sprof), as bench.py loads it
        import ctypes
        ctypes.CDLL(os.environ["GZ_SPROF_LIB"])
    import bench
    from galvanise_zero_amd import cppinterface
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS

    sm, transformer, desc = bench.setup_game(a.config)
    evals = a.evals or BASELINE_CONFIGS[a.config]["evals"]
    rng = np.random.default_rng(1)
    sizes = list(transformer.policy_dist_count)
    nv = transformer.num_rewards

    class Model(object):
        def predict_on_batch(self, X):
            n = X.shape[0]
            out = []
            for p in sizes:
                z = rng.standard_normal((n, p), dtype=np.float32) * a.logit_scale
                z = np.exp(z - z.max(axis=1, keepdims=True))
                out.append(z / z.sum(axis=1, keepdims=True))
            v = rng.random((n, nv), dtype=np.float32)
            out.append(v / v.sum(axis=1, keepdims=True))
            return out

    class NN(object):
        gdl_bases_transformer = transformer
        model = Model()

        def get_model(self):
            return self.model

    sup = cppinterface.Supervisor(sm, NN(), batch_size=a.batch, seed=1, per_pool_unique_states=True)
    sup.start_self_play(bench.selfplay_conf("template", evals), a.workers)
    t0 = time.time()
    last = t0
    prev = sup.stats()
    # a poll can block for minutes while every pool spins: a timer cancels the supervisor at the end
    import threading
    timer = threading.Timer(a.seconds, sup.cancel)
    timer.start()
    while time.time() - t0 < a.seconds:
        if sup.poll(do_stats=True) is None:
            break
        if time.time() - last >= a.report:
            st = sup.stats()
            rows = st["evaluations"] - prev["evaluations"]
            tp = st["tree_playouts"] - prev["tree_playouts"]
            el = time.time() - last
            print("%5.0fs %8.0f leaf-evals/s  NN-free/leaf %7.1f  games %d  samples %d" % (
                time.time() - t0, rows / el, (tp - rows) / max(1, rows), st["games_completed"], st["samples"]),
                flush=True)
            prev, last = st, time.time()
    st = sup.stats()
    el = time.time() - t0
    print("total: %.0f leaf-evals/s, %.2f M tree playouts/s, NN-free/leaf %.1f, games %d" % (
        st["evaluations"] / el, st["tree_playouts"] / el / 1e6,
        (st["tree_playouts"] - st["evaluations"]) / max(1, st["evaluations"]), st["games_completed"]), flush=True)
    timer.cancel()
    sup.cancel()
    t = time.time()
    del sup   # bounded teardown: the workers' pools are cancelled (gz_pool_cancel)
    print("teardown %.2f s" % (time.time() - t), flush=True)

if __name__ == "__main__":
    main()
