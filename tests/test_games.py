"""Native state machines (libgz_engine.so via C-ABI) against the oracle restatement of the GDL
rule sheets (oracle/games_ref.py) on random playouts; action counts pinned by the reference model
files' policy sizes (tests/golden/arch.json)."""
import json
import os

import numpy as np
import pytest

from galvanise_zero_amd.sm import get_sm
from oracle import games_ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


ALL_GAMES = ["breakthrough", "breakthroughSmall", "reversi", "hexLG13", "amazons_10x10"]
# playouts per game: the pure-Python oracles of the larger games are slow
PLAYOUTS = {"breakthrough": 60, "breakthroughSmall": 60, "reversi": 30, "hexLG13": 12, "amazons_10x10": 6}


@pytest.mark.parametrize("game", ALL_GAMES)
def test_policy_sizes_match_reference_models(game):
    arch = json.load(open(os.path.join(GOLDEN, "arch.json")))
    sm = get_sm(game)
    assert [sm.action_count(r) for r in range(sm.role_count)] == arch[game]["policy_units"]


@pytest.mark.parametrize("game", ALL_GAMES)
def test_random_playouts_match_oracle(game):
    sm = get_sm(game)
    ref = games_ref.make(game)
    assert sm.num_bases == ref.num_bases
    for i in range(sm.num_bases):
        assert sm.base_name(i) == ref.base_name(i)
    rng = np.random.default_rng(123)
    games = 0
    for g in range(PLAYOUTS[game]):
        words = sm.get_initial_state()
        s = ref.initial_state
        assert games_ref.words_to_state(words) == s
        for depth in range(1000):
            sm.update_bases(words)
            assert sm.is_terminal() == ref.is_terminal(s)
            if sm.is_terminal():
                assert [sm.get_goal_value(r) for r in range(2)] == [ref.goal(s, r) for r in range(2)]
                games += 1
                break
            legals = [sm.get_legal_state(r) for r in range(2)]
            assert legals == [ref.legal(s, r) for r in range(2)]
            for r in range(2):
                for a in legals[r]:
                    assert sm.legal_to_move(r, a) == ref.legal_to_move(r, a)
            joint = [int(rng.choice(legals[r])) for r in range(2)]
            words = sm.next_state(joint)
            s = ref.next_state(s, joint)
            assert games_ref.words_to_state(words) == s
    assert games == PLAYOUTS[game]


def test_breakthrough_initial_moves():
    sm = get_sm("breakthrough")
    sm.update_bases(sm.get_initial_state())
    assert len(sm.get_legal_state(0)) == 22 and sm.get_legal_state(1) == [0]
