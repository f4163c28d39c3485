"""Summarise a tools/steady_curve.py run (its --out JSON): per logged interval the rate, the
population's age and the stationary estimates of DESIGN.md section 6 -- threads x f x evals per
engine-second of (a) the completed games (cheap-biased: an upper estimate) and (b) the first-game
cohort so far (every slot's first game, completed or in progress), f = the share of the engine
threads' time spent inside game coroutines.

Usage: python tools/curve_report.py CURVE.json [--every N]
"""
import argparse
import json


def estimates(row, threads):
    o = row["ordinals"]
    f = row["engine_s_in_games"] / row["thread_s"] if row["thread_s"] > 0 else 0.0
    ev, es = sum(o["evals"]), sum(o["engine_s"])
    c_e = o["evals"][0] + o["inflight_evals_ord"][0]
    c_s = o["engine_s"][0] + o["inflight_engine_s_ord"][0]
    upper = threads * f * ev / es if es > 0 else None
    cohort = threads * f * c_e / c_s if c_s > 0 else None
    return f, upper, cohort


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("curve")
    ap.add_argument("--every", type=int, default=1)
    args = ap.parse_args()
    d = json.load(open(args.curve))
    threads, games = d["threads"], d["games"]
    print("threads %d, game slots %d" % (threads, games))
    print("%7s %12s %9s %8s %10s %6s %14s %14s %10s" % ("t (s)", "leaf-evals/s", "games/s", "gpu", "games/slot",
                                                          "f", "est. completed", "est. cohort", "1st done"))
    for i, row in enumerate(d["curve"]):
        if i % args.every and i != len(d["curve"]) - 1:
            continue
        f, up, co = estimates(row, threads)
        done = row["ordinals"]["games"][0] / games
        print("%7.0f %12.0f %9.1f %8.2f %10.2f %6.2f %14s %14s %9.1f%%" % (
            row["t"], row["evals_per_s"], row["games_per_s"], row["gpu_busy"], row["games_per_slot"], f,
            "%.0f" % up if up else "-", "%.0f" % co if co else "-", 100 * done))


if __name__ == "__main__":
    main()
