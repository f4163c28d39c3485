"""Self-play throughput over time from the initial position (the approach to steady state): per
interval leaf-evals/s, games/s, GPU busy and launch size of the native runner on one GPU.
Usage: python tools/steady_curve.py [--seconds S] [--interval I] [--pools P] [--threads T]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_gb():
    try:
        with open("/proc/self/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return int(line.split()[1]) / 1e6
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--interval", type=float, default=10)
    ap.add_argument("--pools", type=int, default=2)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--spin-yield", type=int, default=1000)
    ap.add_argument("--out", default="")
    ap.add_argument("--roll-seconds", type=float, default=0,
                    help="clear the unique-states filters every S seconds, as the reference worker does "
                         "at each new generation (worker.py:160); 0 = never")
    args = ap.parse_args()
    import bench
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    from galvanise_zero_amd.nn.weights import random_weights, to_blob
    from galvanise_zero_amd.runner import SelfPlayRunner
    sm, t, desc = bench.setup_game(args.config)
    # the bench's network: bf16x3 split where compiled, the bench's weights
    net = HipNet(desc, 0, "fp32")
    net.set_weights(to_blob(random_weights(desc, 7921)))
    threads = args.threads or max(1, bench.cpu_share())   # as bench.py (cgroup quota aware)
    conf = bench.selfplay_conf("template", BASELINE_CONFIGS[args.config]["evals"])
    r = SelfPlayRunner(net, sm, t, conf, device=0, num_threads=threads, pools_per_thread=args.pools,
                       batch_size=args.batch, seed=20251015, spin_yield_playouts=args.spin_yield,
                       min_launch_rows=1024, max_launch_wait_us=3000)
    games = threads * args.pools * args.batch
    r.start()
    t0 = time.time()
    prev, tp = r.stats(), t0
    rows_log = []
    next_roll = args.roll_seconds if args.roll_seconds > 0 else float("inf")
    rolls = 0
    while time.time() - t0 < args.seconds:
        time.sleep(args.interval)
        if time.time() - t0 >= next_roll:
            r.clear_unique_states()
            rolls += 1
            next_roll += args.roll_seconds
        st, now = r.stats(), time.time()
        dt = now - tp
        d = {k: st[k] - prev[k] for k in st}
        row = {"t": round(now - t0, 1), "evals_per_s": d["rows"] / dt, "games_per_s": d["games_completed"] / dt,
               "games_total": st["games_completed"], "games_per_slot": st["games_completed"] / games,
               "gpu_busy": d["kernel_ms"] / 1e3 / dt,
               "rows_per_launch": d["rows"] / max(1, d["kernel_launches"]),
               "nn_free_playouts_per_leaf": (d["tree_playouts"] - d["rows"]) / max(1, d["rows"]),
               "engine_idle": d["engine_idle_ms"] / 1e3 / dt / threads,
               "samples_per_s": d["samples"] / dt, "dupes_per_s": d["dupes"] / dt, "rolls": rolls,
               "rss_gb": rss_gb(),
               "evals_per_game_cum": st["completed_game_evals"] / max(1, st["games_completed"])}
        # per-ordinal game costs (gz_ordinal_stats): completed games and the games in progress, by
        # the game's ordinal within its slot -- the first-game cohort (ordinal 1, one per slot)
        # completes over the run, and its costs bound the stationary per-game cost
        o = r.ordinal_stats()
        row["ordinals"] = {k: o[k] for k in ("games", "evals", "tree_playouts", "engine_s", "inflight_games_ord",
                                             "inflight_engine_s_ord", "inflight_evals_ord")}
        row["engine_s_in_games"] = sum(o["engine_s"]) + o["inflight_engine_s"]
        row["thread_s"] = threads * (now - t0)
        rows_log.append(row)
        print(json.dumps(row), flush=True)
        prev, tp = st, now
    r.stop()
    r.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"threads": threads, "pools_per_thread": args.pools, "games": games, "curve": rows_log}, f)


if __name__ == "__main__":
    main()
