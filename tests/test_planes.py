"""State -> planes: native transformer (C-ABI) and the product geometry (nn/bases.py) against the
oracle restatement of gdltransformer.cpp / bases.py (oracle/planes_ref.py)."""
import numpy as np
import pytest

from galvanise_zero_amd import cppinterface
from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.bases import GdlBasesTransformer
from galvanise_zero_amd.sm import get_sm
from oracle import games_ref, planes_ref


@pytest.mark.parametrize("game,prev", [("breakthrough", 1), ("breakthroughSmall", 1), ("breakthrough", 0),
                                       ("reversi", 1), ("hexLG13", 1), ("amazons_10x10", 1), ("amazons_10x10", 0)])
def test_planes_match_oracle(game, prev):
    sm = get_sm(game)
    t = GdlBasesTransformer(sm, templates.default_generation_desc(game, num_previous_states=prev))
    ct = cppinterface.create_c_transformer(t)
    ref = planes_ref.Planes(game, [sm.base_name(i) for i in range(sm.num_bases)], prev)
    assert t.num_channels == ref.num_channels and t.channel_size == ref.channel_size
    rng = np.random.default_rng(1)
    words = sm.get_initial_state()
    prev_words = None
    for step in range(200):
        sm.update_bases(words)
        if sm.is_terminal():
            words, prev_words = sm.get_initial_state(), None
            continue
        prevs = [prev_words] if (prev and prev_words is not None) else []
        got = ct.to_channels(words, prevs)
        s = games_ref.words_to_state(words)
        exp = ref.to_channels(s, [games_ref.words_to_state(p) for p in prevs])
        assert np.array_equal(got, exp)
        # product python geometry (bases.py state_to_channels) agrees too
        bits = sm.bits(words)
        pbits = [sm.bits(p) for p in prevs]
        assert np.array_equal(t.state_to_channels(bits, pbits).reshape(-1), exp)
        legal = [sm.get_legal_state(r) for r in range(2)]
        prev_words = words
        words = sm.next_state([int(rng.choice(l)) for l in legal])


def test_control_polarity():
    """breakthrough: black->0, white->1; breakthroughSmall reversed (gamedesc.py:144 vs :173)."""
    for game, white_value in (("breakthrough", 1.0), ("breakthroughSmall", 0.0)):
        sm = get_sm(game)
        t = GdlBasesTransformer(sm, templates.default_generation_desc(game, num_previous_states=1))
        x = t.state_to_channels(sm.bits(sm.get_initial_state()))
        assert np.all(x[-1] == white_value)
