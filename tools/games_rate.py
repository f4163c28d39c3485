"""games/s for the BASELINE configs whose games do not complete inside the bench's window (hexLG13,
amazons: SURVEY 8d metric 2), by renewal: every poll advances each game of a pool by one evaluation,
so a slot completes games at (rate / slots) / E[evals per game], i.e. games/s = rate / E[evals per
game].  E[evals per game] comes from a few-slot run of the same config (tools/gpu_r05k.sh len4 /
len5: 64 slots, ~9 minutes) in which every slot's first game completes -- one independent game per
slot from the initial position, so their mean is unbiased (the completed games of a run that ends
before its slow games do are the cheap part of a heavy-tailed distribution).  `rate` is the config's
bench rate (leaf-evals/s at the bench's 16 threads x 2 pools x 256 games).
Usage: python tools/games_rate.py <few-slot bench log> <bench log or leaf-evals/s> [label]"""
import json
import sys


def last_json(path):
    return json.loads([line for line in open(path) if line.startswith("{")][-1])


def main(len_log, bench, label=""):
    d = last_json(len_log)
    c = d["per_game_cost"]["first_game_cohort"]
    slots, done, running = c["slots"], c["completed"], c["in_progress"]
    evals = c["evals_completed"] + c["evals_in_progress"]
    mean_e = evals / slots
    try:
        rate = float(bench)
        src = "given"
    except ValueError:
        b = last_json(bench)
        rate, src = b["value"], bench
    by_ord = d["per_game_cost"]["by_ordinal"]
    first = by_ord[0] if by_ord else {}
    out = {"config": label or d["config"]["workload"], "few_slot_run": {"slots": slots, "first_games_completed": done,
                                                                        "first_games_in_progress": running,
                                                                        "run_s": d["per_game_cost"]["stationary_estimate"]["run_s"],
                                                                        "moves_per_game": first.get("moves_per_game"),
                                                                        "engine_ms_per_game": first.get("engine_ms_per_game")},
           "evals_per_game": mean_e, "bench_rate_leaf_evals_per_s": rate, "bench_rate_source": src,
           "games_per_sec": rate / mean_e,
           "kind": "renewal estimate (every slot's first game completed)" if running == 0 else
                   "upper bound (%d of %d first games still in progress, counted at their evaluations so far)"
                   % (running, slots)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
