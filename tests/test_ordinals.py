"""Per-game cost by the game's ordinal within its slot (gz_ordinal_stats) and the run-time
verification switch (gz_engine_set_verify_fastpath), on the CPU through the engine C-ABI.

The steady-state question: does a slot's k-th game cost more than its first
(state carried from one game to the next), or does the population only fill up with expensive games?
The counters answer it on the GPU box; here they are checked for consistency, and the engine is
replayed against the oracle over three and more games per slot (reference selfplay.cpp:292-337,
evaluator.cpp:971-1004: a game starts from reset(), carrying only the slot's RNG streams)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.runner import GamePool
from puct_harness import Setup, run_native_supervisor, run_oracle_supervisor, sample_key

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def small():
    return Setup("breakthroughSmall")


def _uniform(pool, n):
    for p in pool.policies:
        p[:n] = 1.0 / p.shape[1]
    pool.values[:n] = 0.5


def test_ordinal_stats_consistent(small):
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 8
    conf.run_to_end_evals = 4
    games = 4
    pool = GamePool(small.sm, small.transformer, conf, games, identifier="o", seed=5)
    n = 0
    for _ in range(20000):
        n = pool.poll(n)
        _uniform(pool, n)
        st = pool.stats()
        if st["games_completed"] >= 4 * games:
            break
    st, o = pool.stats(), pool.ordinal_stats()
    pool.close()
    assert st["games_completed"] >= 4 * games
    assert sum(o["games"]) == st["games_completed"]
    assert sum(o["evals"]) == st["completed_game_evals"]
    assert sum(o["cost_hist"]) == st["games_completed"]
    # every slot plays its games in order: ordinal k+1 never completes more often than ordinal k
    assert all(a >= b for a, b in zip(o["games"][:-2], o["games"][1:-1]))
    assert o["games"][0] == games and o["games"][2] > 0
    for k in range(3):
        assert o["moves"][k] > 0 and o["tree_playouts"][k] >= o["evals"][k] > 0 and o["engine_s"][k] > 0
    assert o["inflight_games"] == games and o["inflight_engine_s"] >= 0


def test_three_games_per_slot_bit_exact(small):
    """Native supervisor vs the oracle, planes compared at every poll, until every slot has
    completed at least three games: no state carried between a slot's games diverges.  Games are
    capped at 12 moves (abort_max_length) so the pure-Python oracle replays four games per slot in
    seconds; full-length games are replayed by test_puct_parity.py."""
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 8
    conf.run_to_end_evals = 4
    conf.abort_max_length = 12
    polls = 1400
    nlog, nsamples, nstats, _ = run_native_supervisor(small, conf, 4, polls, seed=7)
    olog, osamples, man = run_oracle_supervisor(small, conf, 4, polls, seed=7, native_log=nlog)
    assert len(nlog) == len(olog) == polls
    assert [sample_key(small, s, True) for s in nsamples] == [sample_key(small, s, False) for s in osamples]
    started = [sp.match_count for sp in man.self_plays]
    assert min(started) >= 4, started            # >= 3 completed games per slot, the 4th under way
    assert nstats["games_completed"] == sum(started) - len(started)


_VERIFY_CHILD = r"""
import json, sys
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/tests")
from galvanise_zero_amd import _native
from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.runner import GamePool
from puct_harness import Setup
small = Setup("breakthroughSmall")
conf = templates.selfplay_config_template()
conf.evals_per_move = 16
pool = GamePool(small.sm, small.transformer, conf, 4, identifier="v", seed=9)
def run(polls, n):
    for _ in range(polls):
        n = pool.poll(n)
        for p in pool.policies:
            p[:n] = 1.0 / p.shape[1]
        pool.values[:n] = 0.5
    return n
n = run(1500, 0)
before = _native.verified_decisions()
assert not _native.set_verify_fastpath(True)
n = run(1500, n)
during = _native.verified_decisions() - before
assert _native.set_verify_fastpath(False)
n = run(200, n)
after = _native.verified_decisions() - before - during
print(json.dumps({"before": before, "during": during, "after": after,
                  "games": pool.stats()["games_completed"]}))
"""


def test_verify_switch_on_live_pool():
    """Verification switched on mid-run re-checks decisions (a mismatch would abort the child),
    and switched off again stops re-checking."""
    env = dict(os.environ)
    env.pop("GZ_VERIFY_FASTPATH", None)
    out = subprocess.run([sys.executable, "-c", _VERIFY_CHILD % {"root": ROOT}], capture_output=True, text=True,
                         env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["before"] == 0 and r["during"] > 1000 and r["after"] == 0, r


def test_bench_per_game_cost_stationary_estimate():
    """bench.py's per-game cost summary: by-ordinal rows, first-game cohort and the stationary
    estimates (threads x in-game share x evals per engine-second) from a synthetic counter set."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    K = 8
    o = {"games": [10, 4] + [0] * (K - 2), "evals": [1000.0, 400.0] + [0.0] * (K - 2),
         "tree_playouts": [5000.0, 2000.0] + [0.0] * (K - 2), "moves": [100.0, 40.0] + [0.0] * (K - 2),
         "spin_epochs": [3.0, 1.0] + [0.0] * (K - 2), "engine_s": [2.0, 1.0] + [0.0] * (K - 2),
         "cost_hist": [0] * 32, "inflight_games": 6, "inflight_engine_s": 5.0, "inflight_evals": 300.0,
         "inflight_games_ord": [2, 4] + [0] * (K - 2), "inflight_engine_s_ord": [3.0, 2.0] + [0.0] * (K - 2),
         "inflight_evals_ord": [100.0, 200.0] + [0.0] * (K - 2)}
    r = bench.per_game_cost(o, threads=2, slots=12, run_s=5.0)
    assert [row["ordinal"] for row in r["by_ordinal"]] == [1, 2]
    assert r["by_ordinal"][0]["evals_per_game"] == 100.0
    st = r["stationary_estimate"]
    f = (3.0 + 5.0) / (2 * 5.0)
    assert st["in_game_thread_share"] == pytest.approx(f)
    assert st["from_completed_games_leaf_evals_per_s"] == pytest.approx(2 * f * 1400.0 / 3.0)
    assert st["from_first_game_cohort_leaf_evals_per_s"] == pytest.approx(2 * f * 1100.0 / 5.0)
    assert r["first_game_cohort"]["mean_engine_ms_per_game_lower_bound"] == pytest.approx(1e3 * 5.0 / 12)
