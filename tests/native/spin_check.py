"""Subprocess body of tests/test_puct_parity.py::test_spin_fast_path_*: plays breakthrough self-play
through one pool (oracle CPU forward, or with a 5th argument "fake" a cheap synthetic network -- a fixed
random projection of each row's planes to logits and values, a deterministic function of the row -- so
that a run reaches the deep spin regime at 800 evals/move) and prints a digest of every sample plus the
pool counters.  The environment (GZ_SPIN_FAST, GZ_VERIFY_FASTPATH) is read once per process by the
engine."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def fake_forward(desc, planes):
    import numpy as np
    rng = np.random.default_rng(77)
    x = planes.reshape(planes.shape[0], -1).astype(np.float64)
    outs = []
    for p in list(desc.policy_dist_count) + [desc.num_values]:
        w = rng.standard_normal((x.shape[1], p)) * 0.2
        z = np.tanh(x @ w) * 3.0
        z = np.exp(z - z.max(axis=1, keepdims=True))
        outs.append((z / z.sum(axis=1, keepdims=True)).astype(np.float32))
    return outs


def main(game, games, polls, evals, net="oracle"):
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
        if net == "fake":
            outs = fake_forward(setup.desc, pool.planes[:n])
        else:
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
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), *sys.argv[5:6])
