"""Benchmark: self-play games/sec + NN leaf-evals/sec, breakthrough 8x8 @ 800 playouts/move
(BASELINE.json configs[1]: 6-block x 128-filter net, eval batch 256), on N GPUs of one node.

One process per GPU.  `python bench.py --gpus N` with N > 1 (and no WORLD_SIZE in the environment)
starts N ranks itself (torch.distributed.run, before any GPU call) and exits with their status;
under torchrun each rank reads RANK / LOCAL_RANK / WORLD_SIZE.  Each rank pins itself to its share
of the process's CPUs and runs the native self-play runner on its GPU: T engine threads x P game
pools x 256 games (eval batch 256 per pool, as the reference's Supervisor batch_size); one launcher
thread merges the pools waiting for predictions into segmented launches of the fused HIP forward.
Games shard across ranks by global game index (no data-path collective); RCCL is used only to
broadcast the weight blob from rank 0 (the generation-roll hook) before timing.

Steady state.  Every game starts from the initial position, and what a leaf costs the host depends
on the game phase (endgames spin through up to millions of NN-free playouts per move), so a
window right after the start measures the opening only, and no game completes in it.  The bench
therefore first AGES the game population: it runs self-play until --age-games completed games per
game slot (default 3.0) or --age-seconds (default 400) elapse.  The population starts in lockstep
and the endgames' share of the host's time keeps growing for several generations: the 660-s curve
of this configuration (profiles/r03p_steady_curve.log) falls from 1.33 M leaf-evals/s at one game
per slot (120 s, the round-2 window) to ~1.04 M at three (360 s) and ~0.95 M at five (600 s), so
the default window sits at three generations, inside the driver's time budget.

A "step" = --step-rows leaf evaluations (default 2^19) per rank.  W warmup steps, then exactly K
timed steps bracketed by barrier + synchronize; the time is the max over ranks; `value` is
whole-job leaf-evals/sec and `games_per_sec` the games completed in the window per second.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import resource
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # gfx950 dense bf16 MFMA (MI355X_MICROARCH.md)
# L2-served read rate per CU (MI355X_MICROARCH.md "Indexed rows: gather into LDS": rows shared by
# every workgroup, 66-73 GB/s per CU).  Every trunk workgroup streams the whole conv weight image
# from its XCD's L2.
PEAK_L2_GBPS_PER_CU = 70.0
NUM_CUS = 256
# PMC-measured fabric bytes per trunk launch (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE,
# separate rocprofv3 --pmc passes, tools/gpu_pmc.sh).  PMC counters cannot be read inside the timed
# run, so the figure measured for the same kernel is reported with its source.
TRAFFIC_PER_LAUNCH = {"gznn::trunk_kernel<128, 4, 1, 1, 1>": (14290.1 * 2 + 320.0) * 1024,
                      "gznn::trunk_kernel<128, 4, 2, 1, 1>": (14722.3 * 2 + 800.0) * 1024,
                      "gznn::trunk_kernel<128, 4, 2, 1, 3>": (58516.6 * 2 + 1280.0) * 1024,
                      "gznn::trunk_kernel_w8<128, 4, 3>": (58403.1 * 2 + 1280.0) * 1024,
                      "gznn::trunk_kernel_h2<128, 4, 3>": (58430.6 * 2 + 1280.0) * 1024}
TRAFFIC_SOURCE = {
    "gznn::trunk_kernel<128, 4, 1, 1, 1>": "profiles/r01k_pmc.txt (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, 256-row launches)",
    "gznn::trunk_kernel<128, 4, 2, 1, 1>": "profiles/r01k_pmc.txt (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, 640-row launches)",
    "gznn::trunk_kernel<128, 4, 2, 1, 3>": "profiles/r04h_pmc_summary.txt (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                           "separate passes, 1024-row launches; FETCH x2 gfx950 correction, 1 KB units)",
    "gznn::trunk_kernel_w8<128, 4, 3>": "profiles/r04u_pmc_summary.txt (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                         "separate passes, 1024-row launches; FETCH x2 gfx950 correction, 1 KB units)",
    "gznn::trunk_kernel_h2<128, 4, 3>": "profiles/r06m_pmc_summary.txt (the final tree; rocprofv3 --pmc FETCH_SIZE / "
                                         "WRITE_SIZE, separate passes, 1024-row launches; FETCH x2 gfx950 correction, "
                                         "1 KB units; round 5's r05b_pmc_summary.txt: identical)"}


PEAK_HBM_GBPS = 8000.0         # MI355X HBM3E (MI355X_MICROARCH.md)
# SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (summed over the 8 XCDs) per launch of the dominant
# kernel at 1,024 rows, from one rocprofv3 --pmc pass (tools/gpu_pmc_r04.sh)
PMC_PER_LAUNCH = {"gznn::trunk_kernel_h2<128, 4, 3>": {
    "mfma_busy_cycles": 682622976.0, "grbm_gui_active": 9254898.8,
    "source": "profiles/r06m_pmc_summary.txt (the final tree; rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES ... GRBM_GUI_ACTIVE, "
              "one pass, 1024-row launches, tools/gpu_pmc_r04.sh; round 5's r05b_pmc_summary.txt: the same kernel, "
              "9249473.5 active cycles): busy cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)"},
    "gznn::trunk_kernel_w8<128, 4, 3>": {
    "mfma_busy_cycles": 682622976.0, "grbm_gui_active": 8828934.5,
    "source": "profiles/r04u_pmc_summary.txt (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES ... GRBM_GUI_ACTIVE, one pass, "
              "1024-row launches, tools/gpu_pmc_r04.sh): busy cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)"},
    "gznn::trunk_kernel<128, 4, 2, 1, 3>": {
    "mfma_busy_cycles": 682622976.0, "grbm_gui_active": 9320148.5,
    "source": "profiles/r04h_pmc_summary.txt (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES ... GRBM_GUI_ACTIVE, one pass, "
              "1024-row launches, tools/gpu_pmc_r04.sh): busy cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)"}}


def per_game_cost(o, threads, slots, run_s, rate=None, world=1):
    """Per-game cost by the game's ordinal within its slot (gz_ordinal_stats of rank 0's runner, the
    whole run): is a slot's k-th game dearer than its first?  Plus the first-game cohort (ordinal 1:
    one game per slot, every game an independent draw from the initial position with its own RNG
    streams): its completed games' costs and the partial costs of the ones still in progress bound
    the stationary per-game cost from below.  The completed games alone are biased towards cheap
    games (the long spins are the ones still running), so `completed_games_evals_per_engine_s`
    overstates the stationary rate."""
    rows = []
    for k in range(len(o["games"])):
        g = o["games"][k]
        if g == 0:
            continue
        rows.append({"ordinal": k + 1 if k + 1 < len(o["games"]) else "%d+" % (k + 1), "games": g,
                     "evals_per_game": o["evals"][k] / g,
                     "nn_free_playouts_per_game": (o["tree_playouts"][k] - o["evals"][k]) / g,
                     "moves_per_game": o["moves"][k] / g, "spin_epochs_per_game": o["spin_epochs"][k] / g,
                     "engine_ms_per_game": 1e3 * o["engine_s"][k] / g,
                     "evals_per_engine_s": o["evals"][k] / o["engine_s"][k] if o["engine_s"][k] > 0 else None,
                     "in_progress": o["inflight_games_ord"][k]})
    ev, es = sum(o["evals"]), sum(o["engine_s"])
    hist = {"<%d ms" % (1 << k): c for k, c in enumerate(o["cost_hist"]) if c}
    c_s = o["engine_s"][0] + o["inflight_engine_s_ord"][0]
    c_e = o["evals"][0] + o["inflight_evals_ord"][0]
    cohort = {"slots": slots, "completed": o["games"][0], "in_progress": o["inflight_games_ord"][0],
              "engine_s_completed": o["engine_s"][0], "engine_s_in_progress": o["inflight_engine_s_ord"][0],
              "evals_completed": o["evals"][0], "evals_in_progress": o["inflight_evals_ord"][0],
              "mean_engine_ms_per_game_lower_bound": 1e3 * c_s / slots if slots else None,
              "evals_per_engine_s_so_far": c_e / c_s if c_s > 0 else None}
    # stationary rate (renewal-reward over games): threads x f x E[evals / game] / E[engine-s / game],
    # f = the share of the engine threads' time spent inside game coroutines over the run.  From the
    # completed games (VERDICT r03 item 3's estimate: biased towards cheap games, an upper bound) and
    # from the first-game cohort so far (completed + in-progress: every slot's first game)
    in_game_s = es + o["inflight_engine_s"]
    f = in_game_s / (threads * run_s) if run_s > 0 and threads else None
    stationary = {"in_game_thread_share": f, "run_s": run_s,
                  "from_completed_games_leaf_evals_per_s": threads * f * ev / es if f and es > 0 else None,
                  "from_first_game_cohort_leaf_evals_per_s": threads * f * c_e / c_s if f and c_s > 0 else None,
                  "note": "completed games are the cheap part of a heavy-tailed per-game cost (DESIGN.md section 6): "
                          "the first figure overstates the stationary rate"}
    # games/s by renewal (SURVEY 8d metric 2 where no game completes in the window -- configs 4 / 5):
    # every poll advances each game of a pool by one evaluation, so each slot completes games at
    # (rate / slots) / E[evals per game].  The first-game cohort's evaluations so far bound
    # E[evals per game] from below (an upper bound on games/s), exactly once every first game completed.
    if rate and slots and c_e > 0:
        mean_e = c_e / slots
        # rate and slots are per rank (every rank runs the same workload on its own game range):
        # the aggregate is world x the per-rank figure
        cohort["games_per_sec_renewal"] = {
            "value": world * rate / mean_e, "per_rank": rate / mean_e, "ranks": world, "evals_per_game": mean_e,
            "kind": "renewal estimate: every slot's first game completed" if o["inflight_games_ord"][0] == 0
            else "upper bound: %d of %d first games still in progress (counted at their evaluations so far)"
                 % (o["inflight_games_ord"][0], slots)}
    return {"by_ordinal": rows, "engine_ms_histogram": hist, "first_game_cohort": cohort,
            "stationary_estimate": stationary,
            "completed_games_evals_per_engine_s": ev / es if es > 0 else None,
            "in_progress": {"games": o["inflight_games"], "engine_s": o["inflight_engine_s"],
                            "evals": o["inflight_evals"],
                            "evals_per_engine_s": o["inflight_evals"] / o["inflight_engine_s"]
                            if o["inflight_engine_s"] > 0 else None}}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--step-rows", type=int, default=1 << 19, help="leaf evaluations per step per rank")
    ap.add_argument("--age-games", type=float, default=3.0,
                    help="steady state: age the game population until this many games per game slot completed ...")
    ap.add_argument("--age-seconds", type=float, default=400.0, help="... or this many seconds passed (0: no aging)")
    ap.add_argument("--threads", type=int, default=0, help="engine threads per GPU (0: the rank's CPU share)")
    ap.add_argument("--pools", type=int, default=2, help="game pools per engine thread")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--evals", type=int, default=0, help="evals per move (0: the config's, 800 for cfg2)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="BASELINE.json configs[i-1]; 2 (breakthrough 8x8, 6x128) is the headline workload, "
                         "3-5 (reversi 10x128, hexLG13 12x256, amazons_10x10 20x256) run the same path")
    ap.add_argument("--mode", choices=["template", "literal"], default="template")
    ap.add_argument("--precision", choices=["bf16x3", "split", "bf16", "fp32"], default=None,
                    help="trunk arithmetic: bf16x3 (alias split) = hi/lo bf16 operands, three MFMAs per "
                         "product, fp32-class accuracy -- about 35x an IEEE fp32 forward's error on cfg2, "
                         "NOT IEEE fp32 (the reference runs fp32 TF); the default, every config; "
                         "bf16 = bf16 operands; fp32 = deprecated alias of bf16x3")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=45.0)
    ap.add_argument("--opening-seconds", type=float, default=30.0,
                    help="also report the GPU leg's rate over the first seconds of aging (the opening phase the "
                         "CPU baseline measures)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--min-launch-rows", type=int, default=1024,
                    help="hold a launch until this many rows are queued ...")
    ap.add_argument("--max-launch-wait-us", type=int, default=3000, help="... or its oldest pool waited this long")
    ap.add_argument("--backend", default="nccl", help="process-group backend (nccl = RCCL; gloo for CPU-side tests)")
    ap.add_argument("--device", type=int, default=-1, help="GPU of every rank (-1: LOCAL_RANK; tests share one GPU)")
    ap.add_argument("--roll", action="store_true",
                    help="a generation roll before the warmup: rank 0's second weight blob goes to every rank "
                         "(RCCL broadcast) and replaces the live runner's network (gz_runner_update_network)")
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, evals, mode, batch, config=2):
    """CPU restatement of the reference's CPU self-play design, timed on this host (the
    reference's own C++ cannot build here -- ggplib / k273 absent): cppinterface.Supervisor with C++
    worker threads (2 pools of `batch` games each, supervisor.cpp:79-99,196-245) running the tree
    search while the Python poll loop (cppinterface.py:131-144) runs the network on the CPU
    (float32 torch, all the rank's cores: oracle/nn_torch.py) -- the same engine and workload as the
    GPU run, only the network moves to the host."""
    import torch
    from galvanise_zero_amd import cppinterface
    from galvanise_zero_amd.nn.weights import random_weights
    from oracle.nn_torch import TorchCPUNet

    sm, transformer, desc = setup_game(config)
    cores = cpu_share()
    torch.set_num_threads(cores)
    # the tree search gets every core but one (C++ worker threads, each with its two pools, as the
    # GPU leg's engine threads); the network's torch threads share the same cores
    workers = max(1, cores - 1)
    model = TorchCPUNet(desc, random_weights(desc, 7921))

    class NN(object):
        gdl_bases_transformer = transformer

        def get_model(self):
            return model

    sup = cppinterface.Supervisor(sm, NN(), batch_size=batch, seed=1, per_pool_unique_states=True)
    t_start = time.time()
    sup.start_self_play(selfplay_conf(mode, evals), workers)
    t_end = time.time() + min(5.0, seconds / 4)          # warm the pools (first batches, torch init)
    while time.time() < t_end:
        sup.poll(do_stats=True)
    rows0 = sup.total_predictions
    t0 = time.time()
    while time.time() - t0 < seconds:
        sup.poll(do_stats=True)
    el = time.time() - t0
    rows = sup.total_predictions - rows0
    return {"value": rows / el, "unit": "leaf-evals/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "worker_threads": workers, "torch_threads": cores,
            "phase": "opening: %.0f-%.0f s after the start of self-play" % (t0 - t_start, t0 - t_start + el),
            "label": "CPU restatement (not the reference's own binary: SURVEY 8c)",
            "sample": "%.1f s of %s self-play from the initial position (%d evals/move, %s mode): CPU restatement "
                      "of the reference's worker-thread design (%d C++ worker threads x 2 pools x %d games, "
                      "Supervisor.poll loop) with a float32 torch-CPU network on %d threads"
                      % (el, sm.game, evals, mode, workers, batch, cores)}


def launch_ranks(args):
    """--gpus N without a process group: start N ranks (one per GPU) with torch.distributed.run
    before anything touches the GPU, and exit with their status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cgroup_cpu_quota():
    """CPUs granted by the cgroup (v2 cpu.max / v1 cfs quota), or None when unlimited: a container
    may see every CPU of the host in its affinity mask but be throttled to a share of them (the
    GPU box: 256 CPUs visible, 16 granted)."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                text = f.read().strip()
        except OSError:
            continue
        if parse is not None:
            quota, period = parse(text)
            if quota == "max":
                return None
            return max(1, int(int(quota) // int(period)))
        quota = int(text)
        if quota <= 0:
            return None
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            return max(1, quota // int(f.read().strip()))
    return None


def cpu_share(local_world=1):
    """CPUs this rank may use: the affinity mask, capped by the cgroup quota, split over the ranks
    of the node."""
    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 4)
    quota = cgroup_cpu_quota()
    if quota is not None:
        cpus = min(cpus, quota)
    return max(1, cpus // max(1, local_world))


def pin_rank_cpus(local_rank, local_world):
    """Split this process's CPUs into contiguous per-rank shares (ranks of one node start with the
    same affinity) when the node's ranks see more CPUs than their quota share; returns the CPU count
    this rank may use."""
    share = cpu_share(local_world)
    if hasattr(os, "sched_getaffinity") and local_world > 1:
        cpus = sorted(os.sched_getaffinity(0))
        if len(cpus) >= share * local_world:
            per = len(cpus) // local_world
            os.sched_setaffinity(0, cpus[local_rank * per:(local_rank + 1) * per])
    return share


def main():
    args = parse()
    if os.environ.get("GZ_SPROF_LIB"):
        # diagnostics: a host sampling profiler (tools/sprof/sprof.c) loaded into this process (its
        # constructor arms SIGPROF; the samples are written at exit)
        import ctypes
        ctypes.CDLL(os.environ["GZ_SPROF_LIB"])
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        print("[bench] note: --gpus %d but WORLD_SIZE %d; using the process group" % (args.gpus, world),
              file=sys.stderr)
    cpus = pin_rank_cpus(local_rank, local_world)

    import torch
    import torch.distributed as dist

    from galvanise_zero_amd._native import HipNet, engine_build_info
    from galvanise_zero_amd.nn.weights import random_weights, to_blob
    from galvanise_zero_amd.runner import SelfPlayRunner
    from galvanise_zero_amd import shard

    device = local_rank if args.device < 0 else args.device
    torch.cuda.set_device(device)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.backend)

    from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
    evals = args.evals or BASELINE_CONFIGS[args.config]["evals"]
    sm, transformer, desc = setup_game(args.config)
    if args.precision is None:
        # bf16x3 split on every BASELINE config (F = 256 on 13 x 13, cfg 4: the two-pass kernel)
        args.precision = "bf16x3"
    net = HipNet(desc, device, args.precision)
    args.precision = net.precision   # canonical: "fp32" / "split" name bf16x3
    heads_fused = net.heads_fused()

    # weights: rank 0 creates, RCCL broadcast of the blob (the only collective on the path)
    blob = torch.empty(net.weight_count, dtype=torch.float32, device="cuda")
    if rank == 0:
        blob.copy_(torch.from_numpy(to_blob(random_weights(desc, 7921))))
    shard.broadcast_weights(blob, src=0)
    torch.cuda.synchronize()
    net.set_weights_device(blob.data_ptr(), net.weight_count)
    blob_sum = float(blob.double().sum().item())

    # one engine thread per CPU of the rank's share (the launcher and main threads mostly sleep):
    # on the 16-CPU box 16 threads ran 13-18 % faster than 15; 20 about 3 % more at 56 % engine idle
    # (quota throttling), 24 slower (profiles/r03t_bench_threads*.log, r03u_bench_threads.txt)
    threads = args.threads or max(1, cpus)
    games_per_rank = threads * args.pools * args.batch
    game_base = shard.game_index_base(rank, games_per_rank)
    runner = SelfPlayRunner(net, sm, transformer, selfplay_conf(args.mode, evals), device=device,
                            num_threads=threads, pools_per_thread=args.pools, batch_size=args.batch,
                            seed=args.seed, game_index_base=game_base,
                            spin_yield_playouts=args.spin_yield, min_launch_rows=args.min_launch_rows,
                            max_launch_wait_us=args.max_launch_wait_us)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    t_start = time.perf_counter()

    def heartbeat(st):
        el = time.perf_counter() - t_start
        print("[bench rank %d] %.0fs rows %d (%.0f/s) launches %d games %d" %
              (rank, el, st["rows"], st["rows"] / max(el, 1e-9), st["kernel_launches"], st["games_completed"]),
              file=sys.stderr, flush=True)

    runner.start()
    # ---- aging: until the population has turned over (or the time limit) ----------------------
    # the first --opening-seconds of it are also reported as the opening-phase rate (the phase the
    # CPU baseline runs in)
    age_target = args.age_games * games_per_rank
    opening = None
    while args.age_seconds > 0:
        st = runner.stats()
        el = time.perf_counter() - t_start
        if opening is None and el >= args.opening_seconds:
            opening = {"seconds": el, "rows": st["rows"], "leaf_evals_per_s": st["rows"] / el}
        if st["games_completed"] >= age_target or el >= args.age_seconds:
            break
        # 2^18 rows, or what the current rate covers until the time limit (at most 10 s) on slow
        # few-slot runs, so aging ends near --age-seconds
        rate = st["rows"] / max(el, 1e-3)
        chunk = int(min(1 << 18, max(1024, rate * min(10.0, max(args.age_seconds - el, 0.5)))))
        runner.wait_rows(st["rows"] + chunk, timeout_s=600)
        if int(el) // 10 != int(time.perf_counter() - t_start) // 10:
            heartbeat(runner.stats())
    aged = runner.stats()
    age_s = time.perf_counter() - t_start
    # ---- optional generation roll on the live runner (worker.py:138-160) ----------------------------
    roll, roll_sum = None, 0.0
    if args.roll:
        blob2 = torch.empty(net.weight_count, dtype=torch.float32, device="cuda")
        if rank == 0:
            blob2.copy_(torch.from_numpy(to_blob(random_weights(desc, 7922))))
        shard.broadcast_weights(blob2, src=0)
        torch.cuda.synchronize()
        tr = time.perf_counter()
        roll = runner.update_network(device_ptr=blob2.data_ptr(), count=net.weight_count, clear_unique_states=True)
        # the caller's wait: handed to the launcher, applied between two launches (BN fold + bf16 pack
        # on the device, gz_net_set_weights_device), filters cleared
        roll["ms"] = (time.perf_counter() - tr) * 1e3
        roll_sum = float(blob2.double().sum().item())
    # ---- warmup + timed steps --------------------------------------------------------------------
    rows_base = aged["rows"]
    runner.wait_rows(rows_base + args.warmup * args.step_rows, timeout_s=3600, progress=heartbeat)
    barrier()
    s0 = runner.stats()
    t0 = time.perf_counter()
    runner.wait_rows(s0["rows"] + args.steps * args.step_rows, timeout_s=3600, progress=heartbeat)
    s1 = runner.stats()
    t1 = time.perf_counter()
    ordinals = runner.ordinal_stats()
    run_s = time.perf_counter() - t_start
    barrier()
    elapsed = t1 - t0

    d = {k: s1[k] - s0[k] for k in s1}
    # every rank's global game range (disjoint by construction; checked here)
    ranges = [(game_base, game_base + games_per_rank)]
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, ranges[0])
        ranges = allr
    disjoint = all(a[1] <= b[0] for a, b in zip(sorted(ranges), sorted(ranges)[1:]))
    totals, T = shard.reduce_counters(
        [d["rows"], d["batches"], d["games_completed"], d["games_with_samples"], d["samples"], d["kernel_ms"],
         d["kernel_launches"], d["segments"], d["completed_game_evals"], d["trunk_ms"],
         d["large_launches"], d["large_rows"], d["large_trunk_ms"], d["engine_idle_ms"],
         d["no_samples"], d["resigns"], d["aborts"], d["dupes"], d["tree_playouts"],
         aged["games_completed"], games_per_rank, blob_sum, d["large_rounds"], d["split_launches"], roll_sum],
        elapsed, device="cuda")
    (rows, batches, games, games_s, samples, kms, launches, segments, game_evals, tms,
     l_launches, l_rows, l_tms, idle_ms, no_samples, resigns, aborts, dupes, tree_playouts,
     aged_games, games_total, blob_sums, l_rounds, split_launches, roll_sums) = totals

    if rank == 0:
        # host budget: leaf evaluations one engine thread sustains (this window) against what the
        # GPU's forward could absorb at its measured per-row time; fewer engine threads than that
        # leave the GPU waiting on the host
        per_thread = rows / T / (threads * world) if T > 0 else float("nan")
        gpu_capacity = rows / (kms / 1e3) / world if kms > 0 else float("nan")
        threads_needed = int(-(-gpu_capacity // per_thread)) if per_thread > 0 else None
        flops = desc.flops_per_eval()
        avg_fwd_s = (kms / launches) / 1e3 if launches else float("nan")
        rows_per_launch = rows / launches if launches else float("nan")
        # the trunk kernel runs as one of two variants by launch size; the roofline is reported for
        # the variant that took more trunk time, the other one alongside
        # the trunk kernels of small / large launches, as rocprofv3 names them (gz_net_kernel_name)
        p = 3 if args.precision == "bf16x3" else 1
        k_large, k_small = net.kernel_name(True), net.kernel_name(False)
        if k_small == k_large:   # one trunk kernel for every launch size (single-image nets)
            variants = {k_large: (launches, rows, tms)}
            whole = {k_large: (s1["kernel_launches"], s1["rows"], s1["trunk_ms"])}
        else:
            variants = {k_large: (l_launches, l_rows, l_tms)}
            # the same over the whole run (aging included): what a rocprofv3 summary of this
            # command averages over
            whole = {k_large: (s1["large_launches"], s1["large_rows"], s1["large_trunk_ms"])}
        if k_small != k_large:
            variants[k_small] = (launches - l_launches, rows - l_rows, tms - l_tms)
            whole[k_small] = (s1["kernel_launches"] - s1["large_launches"], s1["rows"] - s1["large_rows"],
                              s1["trunk_ms"] - s1["large_trunk_ms"])
        # two-image trunk kernels run the dense heads themselves (no heads launch): their algorithmic
        # work per leaf is then the whole forward's
        kernel_flops = desc.flops_per_eval() if heads_fused else desc.flops_trunk()
        per_variant = {}
        for name, (vl, vr, vt) in variants.items():
            if vl > 0 and vr > 0 and vt > 0:
                wl, wr, wt = whole[name]
                per_variant[name] = {"launches": vl, "rows_per_launch": vr / vl, "avg_kernel_ms": vt / vl,
                                     "achieved_tflops": kernel_flops * vr / (vt / 1e3) / 1e12,
                                     "whole_run": {"launches": wl, "rows_per_launch": wr / max(wl, 1),
                                                   "avg_kernel_ms": wt / max(wl, 1)}}
        dom = max(per_variant, key=lambda k: variants[k][2]) if per_variant else None
        # weight stream per trunk workgroup: bf16 3x3 conv weights of every residual conv (hi + lo
        # parts in fp32 mode)
        wbytes = 2 * desc.residual_layers * 9 * desc.cnn_filter_size ** 2 * 2 * (2 if p == 3 else 1)
        # the fp32-accuracy trunk issues 3 bf16 MFMAs per algorithmic product: its ceiling on
        # algorithmic FLOP/s is a third of the dense bf16 peak
        peak = PEAK_BF16_TFLOPS / p
        for name, pv in per_variant.items():
            nb = 2 if name == k_large and k_large != k_small else 1
            wg = pv["rows_per_launch"] / nb
            cus = max(min(wg, NUM_CUS), 1e-9)
            rate = wg * wbytes / (max(pv["avg_kernel_ms"], 1e-9) / 1e3) / cus / 1e9
            if nb == 2 and pv["launches"] > 0:
                # workgroup rounds (one trunk workgroup per CU): rows / (rounds x one round's rows)
                # is how full the launches' last rounds were
                pv["rounds_per_launch"] = l_rounds / pv["launches"]
                pv["row_fill"] = (pv["rows_per_launch"] * pv["launches"]) / (l_rounds * nb * NUM_CUS) if l_rounds else None
            pv["l2_weight_stream"] = {"bytes_per_workgroup": wbytes, "workgroups_per_launch": wg,
                                      "achieved_GBps_per_cu": rate, "peak_GBps_per_cu": PEAK_L2_GBPS_PER_CU,
                                      "frac": rate / PEAK_L2_GBPS_PER_CU}
        achieved = per_variant[dom]["achieved_tflops"] if dom else float("nan")
        out = {
            "metric": "self-play games/sec + NN leaf-evals/sec, breakthrough 8x8 @ 800 playouts/move",
            "value": rows / T,
            "unit": "leaf-evals/s",
            "games_per_sec": games / T,
            "evals_per_completed_game": game_evals / games if games else None,
            "sample_games_per_sec": games_s / T,
            "samples_per_sec": samples / T,
            # selfplaymanager.cpp:161-200 counters over the window
            "selfplay_counters": {"games_completed": games, "no_sample_games": no_samples, "resigns": resigns,
                                  "aborts": aborts, "duplicate_states": dupes},
            "nn_free_playouts_per_leaf": (tree_playouts - rows) / rows if rows else None,
            "steady_state": {"aging_s": age_s, "games_completed_before_window": aged_games,
                             "games_per_slot_before_window": aged_games / games_total if games_total else None,
                             "age_games_target": args.age_games, "age_seconds_limit": args.age_seconds},
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * T / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16x3 split (hi+lo bf16 operands, ~16-bit significand, 3 MFMAs per product, fp32 accumulate)"
                     if p == 3 else "bf16",
            "data": "synthetic: self-play from the initial position, random-init weights (no .h5 in reference)",
            "config": {"workload": "%s self-play (BASELINE configs[%d]), v1 %dx%d net, %d evals/move (%s mode), "
                                   "eval batch %d" % (sm.game, args.config - 1, desc.residual_layers,
                                                      desc.cnn_filter_size, evals, args.mode, args.batch),
                       "step": "%d leaf evaluations per rank" % args.step_rows,
                       "games_per_gpu": games_per_rank, "threads_per_gpu": threads, "cpus_per_gpu": cpus,
                       "cpus_per_rank": cpus,
                       "pools_per_thread": args.pools, "eval_batch": args.batch,
                       "launch_batching": {"min_rows": args.min_launch_rows, "max_wait_us": args.max_launch_wait_us},
                       "parallelism": "games sharded dp%d" % world,
                       "game_ranges": {"per_rank": ranges, "disjoint": disjoint},
                       "weights_broadcast": {"collective": "RCCL broadcast" if world > 1 else "none (1 rank)",
                                             "identical_on_all_ranks": abs(blob_sums - world * blob_sum) <= 1e-6 * max(1.0, abs(world * blob_sum))}},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak,
                         "peak_basis": "dense bf16 MFMA %.0f TFLOP/s / %d MFMAs per algorithmic product" % (PEAK_BF16_TFLOPS, p),
                         "traffic": TRAFFIC_PER_LAUNCH.get(dom) if args.config == 2 else None,
                         "traffic_unit": "bytes/launch",
                         "traffic_source": TRAFFIC_SOURCE.get(dom) if args.config == 2 else None,
                         "kernel": dom, "avg_kernel_ms": per_variant[dom]["avg_kernel_ms"] if dom else None,
                         "rows_per_launch": per_variant[dom]["rows_per_launch"] if dom else None,
                         "flop_per_leaf_kernel": kernel_flops, "heads_fused": heads_fused, "variants": per_variant,
                         "launch_rows_mean": rows_per_launch,
                         "pools_per_launch": segments / launches if launches else None,
                         "forward_avg_ms": avg_fwd_s * 1e3,
                         "forward_tflops": flops * rows_per_launch / avg_fwd_s / 1e12,
                         "flop_per_leaf": flops, "aggregate_tflops": flops * rows / T / 1e12},
            "gpu_busy_frac": (kms / 1e3) / (T * world) if T > 0 else None,
            "split_launches": split_launches,
            "generation_roll": {"launches_before_rank0": roll["launches_before"], "ms_rank0": roll["ms"],
                                "apply_ms_rank0": roll.get("apply_ms"),
                                "collective": "RCCL broadcast" if world > 1 and args.backend == "nccl" else args.backend,
                                "identical_on_all_ranks": abs(roll_sums - world * roll_sum) <= 1e-6 * max(1.0, abs(world * roll_sum))}
                               if roll else None,
            "host_budget": {"leaf_evals_per_s_per_engine_thread": per_thread,
                            "gpu_forward_capacity_leaf_evals_per_s": gpu_capacity,
                            "engine_threads_per_gpu": threads, "engine_threads_needed_per_gpu": threads_needed,
                            "warning": ("host-bound: %d engine threads per GPU, about %d would keep the GPU busy"
                                        % (threads, threads_needed)) if threads_needed and threads < threads_needed
                                       else None},
            "opening": {"leaf_evals_per_s_rank0": opening["leaf_evals_per_s"], "seconds": opening["seconds"]}
                       if opening else None,
            "engine_idle_frac": (idle_ms / 1e3) / (T * world * threads) if T > 0 else None,
            "host_peak_rss_gb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6,
            "engine_build": engine_build_info(),
        }
        if dom:
            out["roofline"]["l2_weight_stream"] = per_variant[dom]["l2_weight_stream"]
            pmc = PMC_PER_LAUNCH.get(dom) if args.config == 2 else None
            if pmc:
                # counter figures of the same kernel from its committed PMC run (PMC counters cannot be
                # read inside the timed run): MFMA pipe busy / (SIMDs x active cycles), and fabric bytes
                # per launch over this window's average launch time against the 8 TB/s HBM peak
                busy = pmc["mfma_busy_cycles"] / (pmc["grbm_gui_active"] / 8 * NUM_CUS * 4)
                gbps = out["roofline"]["traffic"] / (per_variant[dom]["avg_kernel_ms"] / 1e3) / 1e9
                out["roofline"].update({"mfma_busy_frac": busy, "hbm_GBps": gbps, "hbm_peak_GBps": PEAK_HBM_GBPS,
                                        "hbm_frac": gbps / PEAK_HBM_GBPS, "pmc_source": pmc["source"]})
        out["per_game_cost"] = per_game_cost(ordinals, threads, games_per_rank, run_s, rows / T / world if T > 0 else None,
                                             world)
    # The runner is stopped only now: every figure above comes from the snapshots taken at the end
    # of the timed steps.  The stop is bounded (gz_runner_stop cancels the pools: an engine thread
    # inside a long NN-free root spin returns at the game's next playout); its time goes in the line
    # when the line is printed after it.
    line_first = rank == 0 and (world > 1 or args.no_cpu_baseline)
    if line_first:
        print(json.dumps(out), flush=True)
    t_stop = time.time()
    runner.stop()
    if rank == 0:   # (only rank 0 builds the line)
        out["runner_stop_s"] = time.time() - t_stop
    runner.close()   # frees the games' trees before the CPU baseline
    if rank == 0 and not line_first:
        out["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, evals, args.mode, args.batch, args.config)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
