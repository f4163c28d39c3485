"""Benchmark: self-play games/sec + NN leaf-evals/sec, breakthrough 8x8 @ 800 playouts/move
(BASELINE.json configs[1]: 6-block x 128-filter net, eval batch 256), on N GPUs of one node.

One process per GPU (torchrun for N>1).  Each rank runs the native self-play runner on its GPU:
T engine threads x P game pools x 256 games (eval batch 256 per pool, as the reference's
Supervisor batch_size); one launcher thread merges the pools waiting for predictions into
segmented launches of the fused HIP forward.  Games shard across ranks by global game index (no
data-path collective); RCCL is used only to broadcast the weight blob from rank 0 (the
generation-roll hook) before timing.

A "step" = one eval batch (256 leaf evaluations) for every pool of the rank, i.e. T*P*256 leaf
evaluations.  W warmup steps, then exactly K timed steps bracketed by barrier + synchronize; the
time is the max over ranks, `value` is whole-job leaf-evals/sec.  Rank 0 prints one JSON line.

Every game starts from the initial position and the per-leaf host cost grows as games reach their
endgames (the reference's playout loop re-selects finalised children for up to millions of
playouts per move there), so the rate depends on the window.  The default window (W=100, K=10000
steps = 143M leaf evaluations at 14 threads x 4 pools) runs from ~1 s to ~150 s after the start and
covers the first generation of games reaching their endgames; `--steps` larger measures further
into the steady state (DESIGN.md section 6 lists measured long-run rates).
"""
import argparse
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # gfx950 dense bf16 MFMA (MI355X_MICROARCH.md)
# L2-served read rate per CU (MI355X_MICROARCH.md "Indexed rows: gather into LDS": rows shared by
# every workgroup, 66-73 GB/s per CU, 16.8-18.8 TB/s chip-wide).  Every trunk workgroup streams the
# whole conv weight image from its XCD's L2, so below ~1.5 boards per CU the trunk is bound by this
# rate, not by the MFMA peak.
PEAK_L2_GBPS_PER_CU = 70.0
NUM_CUS = 256
# PMC-measured fabric bytes per trunk launch (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE,
# separate rocprofv3 --pmc passes of tools/gpu_pmc.sh at 256 / 640 rows, profiles/r01k_pmc.txt).
# PMC counters cannot be read inside the timed run, so the measured per-launch figure of the same
# kernel at the bench's launch size is reported.
TRAFFIC_PER_LAUNCH = {"gznn::trunk_kernel<128, 8, 8, 1, 1>": (14290.1 * 2 + 320.0) * 1024,
                      "gznn::trunk_kernel<128, 8, 8, 2, 1>": (14722.3 * 2 + 800.0) * 1024}
TRAFFIC_SOURCE = "profiles/r01k_pmc.txt (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, 256- and 640-row launches)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--threads", type=int, default=0, help="host threads per GPU (0: auto)")
    ap.add_argument("--pools", type=int, default=4, help="game pools per thread")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--evals", type=int, default=0, help="evals per move (0: the config's, 800 for cfg2)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="BASELINE.json configs[i-1]; 2 (breakthrough 8x8, 6x128) is the headline workload, "
                         "3-5 (reversi 10x128, hexLG13 12x256, amazons_10x10 20x256) run the same path")
    ap.add_argument("--mode", choices=["template", "literal"], default="template")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--min-launch-rows", type=int, default=1024,
                    help="hold a launch (while one is in flight) until this many rows are queued ...")
    ap.add_argument("--max-launch-wait-us", type=int, default=3000, help="... or its oldest pool waited this long")
    ap.add_argument("--spin-yield", type=int, default=1000,
                    help="yield a game's coroutine after this many NN-free playouts (0: reference behaviour)")
    return ap.parse_args()


def selfplay_conf(mode, evals):
    from galvanise_zero_amd.defs import templates
    if mode == "literal":
        return templates.literal_selfplay_config(evals)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    return conf


def setup_game(config=2):
    from galvanise_zero_amd.defs import templates
    from galvanise_zero_amd.nn.bases import GdlBasesTransformer
    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    from galvanise_zero_amd.sm import get_sm
    cfg = BASELINE_CONFIGS[config]
    sm = get_sm(cfg["game"])
    gen = templates.default_generation_desc(cfg["game"], num_previous_states=1,
                                            draw_head=cfg["desc"].num_values == 3)
    transformer = GdlBasesTransformer(sm, gen)
    desc = cfg["desc"]
    assert (transformer.num_channels, transformer.num_cols, transformer.num_rows) == \
        (desc.input_channels, desc.input_columns, desc.input_rows)
    assert list(transformer.policy_dist_count) == list(desc.policy_dist_count)
    assert transformer.num_rewards == desc.num_values
    return sm, transformer, desc


def cpu_baseline(seconds, evals, mode, batch, config=2):
    """CPU restatement timed on the host: the same engine driven by the reference's Python poll
    loop with the oracle's CPU forward (oracle/nn_ref.py) in place of the GPU."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from galvanise_zero_amd import cppinterface
    from galvanise_zero_amd.nn.weights import random_weights
    from oracle import nn_ref

    sm, transformer, desc = setup_game(config)
    weights = random_weights(desc, 7921)
    cores = min(16, os.cpu_count() or 1)

    class OracleModel(object):
        def predict_on_batch(self, X):
            return nn_ref.forward(desc, weights, X)

    class NN(object):
        gdl_bases_transformer = transformer

        def get_model(self):
            return OracleModel()

    with threadpool_limits(limits=cores):
        sup = cppinterface.Supervisor(sm, NN(), batch_size=batch, seed=1, per_pool_unique_states=True)
        sup.start_self_play(selfplay_conf(mode, evals), 0)
        t0 = time.time()
        sup.poll(do_stats=True)
        rows0 = sup.total_predictions
        t0 = time.time()
        while time.time() - t0 < seconds:
            sup.poll(do_stats=True)
        el = time.time() - t0
        rows = sup.total_predictions - rows0
    return {"value": rows / el, "unit": "leaf-evals/s", "cores": cores, "kind": "port",
            "sample": "%.1f s of %s self-play (%d games inline, batch %d, %d evals/move, %s mode): "
                      "native engine + oracle fp64 numpy forward via the Python poll loop" %
                      (el, sm.game, batch, batch, evals, mode)}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.nn.weights import random_weights, to_blob
    from galvanise_zero_amd.runner import SelfPlayRunner
    from galvanise_zero_amd import shard

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    evals = args.evals or BASELINE_CONFIGS[args.config]["evals"]
    sm, transformer, desc = setup_game(args.config)
    net = HipNet(desc, local_rank)

    # weights: rank 0 creates, RCCL broadcast of the blob (the only collective on the path)
    blob = torch.empty(net.weight_count, dtype=torch.float32, device="cuda")
    if rank == 0:
        blob.copy_(torch.from_numpy(to_blob(random_weights(desc, 7921))))
    shard.broadcast_weights(blob, src=0)
    torch.cuda.synchronize()
    net.set_weights_device(blob.data_ptr(), net.weight_count)

    # the CPUs this process may run on (the GPU box pins 16 per GPU; os.cpu_count() is the machine)
    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 4)
    if world > 1 and cpus >= (os.cpu_count() or cpus):   # unpinned ranks share the machine
        cpus = cpus // world
    threads = args.threads or max(1, min(15, cpus - 1))   # + the launcher (mostly asleep) and main
    runner = SelfPlayRunner(net, sm, transformer, selfplay_conf(args.mode, evals), device=local_rank,
                            num_threads=threads, pools_per_thread=args.pools, batch_size=args.batch,
                            seed=args.seed,
                            game_index_base=shard.game_index_base(rank, threads * args.pools * args.batch),
                            spin_yield_playouts=args.spin_yield, min_launch_rows=args.min_launch_rows,
                            max_launch_wait_us=args.max_launch_wait_us)
    npools = runner.num_pools

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    rows_per_step = npools * args.batch
    t_start = time.perf_counter()

    def heartbeat(st):
        el = time.perf_counter() - t_start
        print("[bench rank %d] %.0fs rows %d (%.0f/s) launches %d games %d" %
              (rank, el, st["rows"], st["rows"] / max(el, 1e-9), st["kernel_launches"], st["games_completed"]),
              file=sys.stderr, flush=True)

    runner.start()
    runner.wait_rows(args.warmup * rows_per_step, timeout_s=3600, progress=heartbeat)
    barrier()
    s0 = runner.stats()
    t0 = time.perf_counter()
    runner.wait_rows((args.warmup + args.steps) * rows_per_step, timeout_s=3600, progress=heartbeat)
    s1 = runner.stats()
    t1 = time.perf_counter()
    barrier()
    t_end = time.perf_counter()
    runner.stop()
    elapsed = t1 - t0

    d = {k: s1[k] - s0[k] for k in s1}
    totals, T = shard.reduce_counters(
        [d["rows"], d["batches"], d["games_completed"], d["games_with_samples"], d["samples"], d["kernel_ms"],
         d["kernel_launches"], d["segments"], s1["games_completed"], s1["completed_game_evals"], d["trunk_ms"],
         d["large_launches"], d["large_rows"], d["large_trunk_ms"], d["engine_idle_ms"],
         d["no_samples"], d["resigns"], d["aborts"], d["dupes"]],
        elapsed, device="cuda")
    (rows, batches, games, games_s, samples, kms, launches, segments, games_all, game_evals_all, tms,
     l_launches, l_rows, l_tms, idle_ms, no_samples, resigns, aborts, dupes) = totals

    if rank == 0:
        flops = desc.flops_per_eval()
        avg_fwd_s = (kms / launches) / 1e3 if launches else float("nan")
        rows_per_launch = rows / launches if launches else float("nan")
        # the trunk kernel runs as one of two variants by launch size; the roofline is reported for
        # the variant that took more trunk time, the other one alongside
        geo = (desc.cnn_filter_size, desc.input_columns, desc.input_rows)
        variants = {
            "gznn::trunk_kernel<%d, %d, %d, 2, 1>" % geo: (l_launches, l_rows, l_tms),
            "gznn::trunk_kernel<%d, %d, %d, 1, 1>" % geo: (launches - l_launches, rows - l_rows, tms - l_tms),
        }
        per_variant = {}
        for name, (vl, vr, vt) in variants.items():
            if vl > 0 and vt > 0:
                per_variant[name] = {"launches": vl, "rows_per_launch": vr / vl, "avg_kernel_ms": vt / vl,
                                     "achieved_tflops": desc.flops_trunk() * vr / (vt / 1e3) / 1e12}
        dom = max(per_variant, key=lambda k: variants[k][2]) if per_variant else None
        # weight stream per trunk workgroup: bf16 3x3 conv weights of every residual conv
        wbytes = 2 * desc.residual_layers * 9 * desc.cnn_filter_size ** 2 * 2
        for name, pv in per_variant.items():
            nb = 2 if name.endswith("2, 1>") else 1
            wg = pv["rows_per_launch"] / nb
            cus = min(wg, NUM_CUS)
            rate = wg * wbytes / (pv["avg_kernel_ms"] / 1e3) / cus / 1e9
            pv["l2_weight_stream"] = {"bytes_per_workgroup": wbytes, "workgroups_per_launch": wg,
                                      "achieved_GBps_per_cu": rate, "peak_GBps_per_cu": PEAK_L2_GBPS_PER_CU,
                                      "frac": rate / PEAK_L2_GBPS_PER_CU}
        achieved = per_variant[dom]["achieved_tflops"] if dom else float("nan")
        out = {
            "metric": "self-play games/sec + NN leaf-evals/sec, breakthrough 8x8 @ 800 playouts/move",
            "value": rows / T,
            "unit": "leaf-evals/s",
            "games_per_sec": games / T,
            # mean NN evaluations of the games completed since start (biased to short games early on)
            "evals_per_completed_game": game_evals_all / games_all if games_all else None,
            "games_completed_total": games_all,
            "sample_games_per_sec": games_s / T,
            "samples_per_sec": samples / T,
            # selfplaymanager.cpp:161-200 counters over the window
            "selfplay_counters": {"no_sample_games": no_samples, "resigns": resigns, "aborts": aborts,
                                  "duplicate_states": dupes},
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * T / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: self-play from the initial position, random-init weights (no .h5 in reference)",
            "config": {"workload": "%s self-play (BASELINE configs[%d]), v1 %dx%d net, %d evals/move (%s mode), "
                                   "eval batch %d" % (sm.game, args.config - 1, desc.residual_layers,
                                                      desc.cnn_filter_size, evals, args.mode, args.batch),
                       "games_per_gpu": npools * args.batch, "threads_per_gpu": threads,
                       "pools_per_thread": args.pools, "eval_batch": args.batch,
                       "launch_batching": {"min_rows": args.min_launch_rows, "max_wait_us": args.max_launch_wait_us}, "parallelism": "games sharded dp%d" % world},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_BF16_TFLOPS, "traffic": TRAFFIC_PER_LAUNCH.get(dom) if args.config == 2 else None,
                         "traffic_unit": "bytes/launch",
                         "traffic_source": TRAFFIC_SOURCE if args.config == 2 and dom in TRAFFIC_PER_LAUNCH else None,
                         "kernel": dom, "avg_kernel_ms": per_variant[dom]["avg_kernel_ms"] if dom else None,
                         "rows_per_launch": per_variant[dom]["rows_per_launch"] if dom else None,
                         "flop_per_leaf_kernel": desc.flops_trunk(), "variants": per_variant,
                         "launch_rows_mean": rows_per_launch,
                         "pools_per_launch": segments / launches if launches else None,
                         "forward_avg_ms": avg_fwd_s * 1e3,
                         "forward_tflops": flops * rows_per_launch / avg_fwd_s / 1e12,
                         "flop_per_leaf": flops, "aggregate_tflops": flops * rows / T / 1e12},
            "gpu_busy_frac": (kms / 1e3) / (T * world) if T > 0 else None,
            "engine_idle_frac": (idle_ms / 1e3) / (T * world * threads) if T > 0 else None,
            "host_peak_rss_gb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6,
        }
        if dom:
            out["roofline"]["l2_weight_stream"] = per_variant[dom]["l2_weight_stream"]
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, evals, args.mode, args.batch, args.config)
        print(json.dumps(out), flush=True)
    runner.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
