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
