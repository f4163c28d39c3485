"""Multi-GPU sharding path rehearsed on CPU with world-size-2 gloo: the weight blob
reaches every rank bit-identical through shard.broadcast_weights (RCCL on the GPU box), ranks own
disjoint game ranges (shard.game_index_base), and the union of the ranks' self-play samples equals
a single process playing all the games -- a game's trajectory does not depend on its rank or pool.
The network is the oracle's CPU forward (batch-invariant, fp64), standing in for the GPU."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from galvanise_zero_amd import shard
from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.bases import GdlBasesTransformer
from galvanise_zero_amd.nn.desc import NetDesc
from galvanise_zero_amd.nn.weights import from_blob, random_weights, to_blob
from galvanise_zero_amd.runner import GamePool
from galvanise_zero_amd.sm import get_sm

GAMES_PER_RANK = 4
POLLS = 1200
SEED = 11


def _setup():
    sm = get_sm("breakthroughSmall")
    gen = templates.default_generation_desc("breakthroughSmall", num_previous_states=1)
    t = GdlBasesTransformer(sm, gen)
    desc = NetDesc(t.num_channels, t.num_cols, t.num_rows, 64, 1, list(t.policy_dist_count), value_hidden_size=32)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 20
    return sm, t, desc, conf


def _play(sm, t, desc, weights, conf, games, base):
    from oracle import nn_ref
    pool = GamePool(sm, t, conf, games, identifier="g", seed=SEED, game_index_base=base)
    n = 0
    samples = []
    for _ in range(POLLS):
        n = pool.poll(n)
        pol = nn_ref.forward(desc, weights, pool.planes[:n])
        for dst, src in zip(pool.policies + [pool.values], pol):
            dst[:n] = src
        samples += pool.fetch_samples()
    samples += pool.fetch_samples()
    stats = pool.stats()
    pool.close()
    return samples, stats


def _key(s):
    s = dict(s)
    s.pop("match_identifier", None)
    return json.dumps(s, sort_keys=True)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sm, t, desc, conf = _setup()
        ref_blob = to_blob(random_weights(desc, 7921))
        blob = torch.from_numpy(ref_blob.copy()) if rank == 0 else torch.zeros(ref_blob.size, dtype=torch.float32)
        shard.broadcast_weights(blob, src=0)
        weights = from_blob(desc, blob.numpy())
        base = shard.game_index_base(rank, GAMES_PER_RANK)
        samples, stats = _play(sm, t, desc, weights, conf, GAMES_PER_RANK, base)
        totals, tmax = shard.reduce_counters([stats["evaluations"], len(samples)], float(rank + 1))
        with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
            json.dump({"blob_equal": bool(np.array_equal(blob.numpy(), ref_blob)), "base": base,
                       "samples": [_key(s) for s in samples], "evaluations": stats["evaluations"],
                       "totals": totals, "tmax": tmax}, f)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_rank_sharding_matches_single_process():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        ranks = [json.load(open(os.path.join(d, "rank%d.json" % r))) for r in range(world)]
    assert all(r["blob_equal"] for r in ranks)
    assert [r["base"] for r in ranks] == [0, GAMES_PER_RANK]
    # counters: SUM over ranks, time: MAX over ranks
    for r in ranks:
        assert r["totals"] == [sum(x["evaluations"] for x in ranks), sum(len(x["samples"]) for x in ranks)]
        assert r["tmax"] == float(world)

    sm, t, desc, conf = _setup()
    samples, stats = _play(sm, t, desc, random_weights(desc, 7921), conf, world * GAMES_PER_RANK, 0)
    single = sorted(_key(s) for s in samples)
    sharded = sorted(k for r in ranks for k in r["samples"])
    assert len(single) > 0
    assert sharded == single
    assert stats["evaluations"] == sum(r["evaluations"] for r in ranks)


def test_renewal_games_per_sec_aggregates_ranks():
    """bench.per_game_cost's renewal games/s: the rate it is given is per rank, so the
    reported value is world x the per-rank figure (each rank runs the same workload on its own game
    range); the per-rank figure is reported beside it."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    K = 8
    o = {"games": [0] * K, "evals": [0] * K, "tree_playouts": [0] * K, "moves": [0] * K, "spin_epochs": [0] * K,
         "engine_s": [0.0] * K, "cost_hist": [0] * 16, "inflight_games": 4, "inflight_engine_s": 2.0,
         "inflight_evals": 4000, "inflight_games_ord": [4] + [0] * (K - 1),
         "inflight_engine_s_ord": [2.0] + [0.0] * (K - 1), "inflight_evals_ord": [4000] + [0] * (K - 1)}
    one = bench.per_game_cost(o, threads=2, slots=4, run_s=10.0, rate=1000.0, world=1)
    two = bench.per_game_cost(o, threads=2, slots=4, run_s=10.0, rate=1000.0, world=2)
    r1, r2 = one["first_game_cohort"]["games_per_sec_renewal"], two["first_game_cohort"]["games_per_sec_renewal"]
    assert r1["value"] == r1["per_rank"] == 1000.0 / 1000.0
    assert r2["value"] == 2 * r2["per_rank"] and r2["ranks"] == 2
