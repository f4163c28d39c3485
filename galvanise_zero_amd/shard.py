"""Multi-GPU self-play sharding: one process per GPU, games partitioned by global game
index, one collective -- the weight-blob broadcast from rank 0.

Reference counterparts: independent self-play worker processes (src/ggpzero/distributed/worker.py),
each reloading the new generation's weights from disk (worker.py:122-160, cppinterface.py:146-147
update_nn).  Here the new weights travel rank 0 -> every rank as one RCCL broadcast over xGMI
(backend "nccl" on ROCm), or gloo on CPU for the tests.

Game g of the job always uses the RNG streams derived from (seed, g) (engine rng.h), so a game's
trajectory does not depend on which rank, pool or thread runs it.
"""
import torch
import torch.distributed as dist


def game_index_base(rank, games_per_rank):
    """Global index of the first game of `rank` (ranks own contiguous, equal game ranges)."""
    return rank * games_per_rank


def broadcast_weights(blob, src=0):
    """Broadcast the packed float32 weight blob (a torch tensor, device memory under RCCL) from
    `src` to every rank in place.  No-op without an initialised process group of size > 1."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(blob, src=src)
    return blob


def reduce_counters(values, elapsed, device=None):
    """Whole-job totals: SUM of the per-rank counters, MAX of the per-rank elapsed time."""
    vec = torch.tensor(list(values), dtype=torch.float64, device=device)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return vec.tolist(), tmax.item()
