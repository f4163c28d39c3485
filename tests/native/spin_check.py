"""Subprocess body of tests/test_puct_parity.py::test_spin_fast_path_*: plays breakthrough self-play
through one pool (oracle CPU forward) and prints a digest of every sample plus the pool counters.
The environment (GZ_SPIN_FAST, GZ_VERIFY_FASTPATH) is read once per process by the engine."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(game, games, polls, evals):
    from galvanise_zero_amd.defs import templates
    from galvanise_zero_amd.runner import GamePool
    from puct_harness import Setup
    from oracle import nn_ref
    setup = Setup(game)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    pool = GamePool(setup.sm, setup.transformer, conf, games, identifier="s", seed=5, game_index_base=0)
    n, digest, count = 0, hashlib.sha256(), 0
    for _ in range(polls):
        n = pool.poll(n)
        outs = nn_ref.forward(setup.desc, setup.weights, pool.planes[:n])
        for dst, src in zip(pool.policies + [pool.values], outs):
            dst[:n] = src
        for s in pool.fetch_samples():
            digest.update(json.dumps(s, sort_keys=True).encode())
            count += 1
    st = pool.stats()
    pool.close()
    print(json.dumps({"samples": count, "digest": digest.hexdigest(), "tree_playouts": st["tree_playouts"],
                      "evaluations": st["evaluations"], "games": st["games_completed"]}))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
