"""Generates tests/golden/puct_player.json: per-move root (action, visit count) lists of a Player
search run through the oracle (oracle/puct_ref.py) with the oracle NN on seeded weights."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from galvanise_zero_amd.defs import templates      # noqa: E402
from oracle import puct_ref as P                   # noqa: E402
from puct_harness import Setup                     # noqa: E402


def main():
    game, evals, moves, seed = "breakthroughSmall", 80, 3, 17
    conf_kw = dict(batch_size=4, choose="choose_top_visits", dirichlet_noise_pct=0.25, think_time=-1,
                   converged_visits=1)
    setup = Setup(game)
    conf = templates.base_puct_config(**conf_kw)
    op = P.Player(setup.ref_sm, setup.ref_planes, conf, list(setup.transformer.policy_dist_count),
                  setup.transformer.num_rewards, setup.num_prev_states, seed=seed)
    op.reset(0)
    state = setup.ref_sm.initial_state
    out = []
    for _ in range(moves):
        op.move(state, evals)
        pred = (0, [[]] * 2, [])
        while True:
            buf = op.poll(*pred)
            if buf is None:
                break
            o = setup.nn(buf)
            pred = (o[0].shape[0], o[:-1], o[-1])
        out.append([[a, t] for a, t, _ in op.root_children()])
        lead = 0 if len(setup.ref_sm.legal(state, 0)) > 1 else 1
        mv = op.get_move(lead)[0]
        joint = tuple(mv if r == lead else 0 for r in range(2))
        op.apply_move(joint)
        op.poll(0, [[]] * 2, [])
        state = setup.ref_sm.next_state(state, joint)
    json.dump(dict(game=game, evals=evals, moves=moves, seed=seed, conf=conf_kw, root_visits=out),
              open(os.path.join(HERE, "puct_player.json"), "w"))


if __name__ == "__main__":
    main()
