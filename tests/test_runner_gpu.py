"""The benched path against the oracle.

bench.py measures the native runner (csrc/nn/runner.hip): engine threads x game pools whose planes
and predictions live in pinned host memory, merged by one launcher thread into segmented launches
(gz_net_forward_segments) with launch batching (min_launch_rows / max_launch_wait_us), whole-wave
trimming and the two-boards-per-workgroup trunk above 256 rows, and the NN-free-playout yield
(spin_yield_playouts).  These tests run that exact configuration (scaled down in games) and require

  * gz_net_forward_segments over odd-sized (and empty) segments, in device or pinned host memory,
    to equal per-segment gz_net_forward bit for bit (the kernel is batch-invariant);
  * every sample the runner emits for a pool to equal, field for field, the sample the oracle
    (oracle/puct_ref.Manager: the reference's SelfPlayManager, supervisor.cpp:79-99 + 196-245,
    scheduler.cpp:132-205) emits for the same (seed, global game index), replaying the pool with
    the network outputs of the same HIP forward.

Reference: src/cpp/supervisor.cpp:79-99,196-245, src/cpp/scheduler.cpp:132-205,
src/cpp/selfplay.cpp:76-337.
"""
import attr
import numpy as np
import pytest

from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob
from gpu_helpers import Pinned
from puct_harness import Setup, sample_key

pytestmark = pytest.mark.gpu


def _net(desc, seed, device):
    from galvanise_zero_amd._native import HipNet
    w = random_weights(desc, seed)
    net = HipNet(desc, device)
    net.set_weights(to_blob(w))
    return net


@pytest.mark.parametrize("placement", ["device", "pinned"])
@pytest.mark.parametrize("sizes", [(37, 0, 129, 1, 200, 64), (5, 0, 17), (300,)])
def test_forward_segments_match_forward(placement, sizes, hip_device):
    """Segment boundaries inside a two-board workgroup (odd sizes above 256 rows: NB = 2), an empty
    segment, single rows; every segment's outputs equal a gz_net_forward of its rows alone."""
    import torch
    desc = BASELINE_CONFIGS[2]["desc"]
    net = _net(desc, 7921, hip_device)
    C, H, W = desc.input_channels, desc.input_columns, desc.input_rows
    P, V = list(desc.policy_dist_count), desc.num_values
    xs = [random_planes(desc, n, 50 + i) if n else np.zeros((0, C, H, W), np.float32) for i, n in enumerate(sizes)]
    keep, segs, outs = [], [], []
    for x in xs:
        n = x.shape[0]
        if placement == "device":
            tp = torch.from_numpy(x.reshape(-1).copy()).cuda() if n else torch.zeros(1, device="cuda")
            tpol = [torch.full((max(1, n * p),), -1.0, device="cuda") for p in P]
            tval = torch.full((max(1, n * V),), -1.0, device="cuda")
            keep += [tp, tval] + tpol
            segs.append((n, tp.data_ptr(), [t.data_ptr() for t in tpol], tval.data_ptr()))
            outs.append((tpol, tval))
        else:
            bp = Pinned(x.size)
            bp.a[:] = x.reshape(-1)
            bpol = [Pinned(n * p) for p in P]
            bval = Pinned(n * V)
            for b in bpol + [bval]:
                b.a[:] = -1.0
            keep += [bp, bval] + bpol
            segs.append((n, bp.ptr.value, [b.ptr.value for b in bpol], bval.ptr.value))
            outs.append((bpol, bval))
    net.forward_segments(torch.cuda.current_stream().cuda_stream, segs)
    torch.cuda.synchronize()
    for x, (pol, val) in zip(xs, outs):
        n = x.shape[0]
        if n == 0:
            continue
        ref = net.forward(x)
        if placement == "device":
            got = [t[:n * p].cpu().numpy().reshape(n, p) for t, p in zip(pol, P)] + [val[:n * V].cpu().numpy().reshape(n, V)]
        else:
            got = [b.a.reshape(n, p).copy() for b, p in zip(pol, P)] + [val.a.reshape(n, V).copy()]
        for g, r in zip(got, ref):
            assert np.array_equal(g, r)
    if placement == "pinned":
        for b in keep:
            b.free()


def _runner_conf(evals):
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    conf.run_to_end_evals = 4
    return conf


def _oracle_conf(conf, spin):
    d = attr.asdict(conf)
    for k in ("puct_config", "run_to_end_puct_config"):
        d[k]["spin_yield_playouts"] = spin
    return d


def _suffix(s):
    """match_identifier = <pool identifier>_<game slot>_<match count> (selfplay.cpp:187, :323)."""
    s = dict(s)
    s["match_identifier"] = "_".join(s["match_identifier"].split("_")[-2:])
    return s


CASES = {
    # BASELINE configs[1]: breakthrough 8x8 on the 6-block x 128-filter net (the headline workload)
    "breakthrough_cfg2": (2, "breakthrough", 32, 10, 1200, (0, 7, 13, 19)),
    # BASELINE configs[2]: reversi 8x8 with the draw head (3 values), 10-block x 128-filter net
    # (reversi games last ~60 moves of >= 16 evaluations, and the oracle is slow on reversi: pools
    # of 16 games, 20 per thread -- still 640 rows, up to 512 merged)
    "reversi_cfg3": (3, "reversi", 16, 20, 1600, (0, 27)),
}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", list(CASES))
def test_native_runner_matches_oracle(case, hip_device):
    """gz_runner in the bench's configuration: 2 engine threads x 10 pools x 32 games (640 rows),
    launch batching 512 rows / 2 ms (merged launches of several pools, the two-boards-per-workgroup
    trunk, whole-wave trimming beyond 512 rows), spin yield 1000, pinned-host segments.  Pools of
    both engine threads are replayed through the oracle with the outputs of the same HIP forward;
    every runner sample of those pools must be identical to the oracle's."""
    from galvanise_zero_amd.runner import SelfPlayRunner
    from oracle import puct_ref as P
    cfg, game, B, ppt, polls, check_pools = CASES[case]
    desc = BASELINE_CONFIGS[cfg]["desc"]
    setup = Setup(game, draw_head=desc.num_values == 3)
    t = setup.transformer
    assert (t.num_channels, t.num_cols, t.num_rows, list(t.policy_dist_count), t.num_rewards) == \
        (desc.input_channels, desc.input_columns, desc.input_rows, list(desc.policy_dist_count), desc.num_values)
    net = _net(desc, 7921, hip_device)
    conf = _runner_conf(8)
    seed, threads, spin = 20251015, 2, 1000
    r = SelfPlayRunner(net, setup.sm, t, conf, device=hip_device, num_threads=threads, pools_per_thread=ppt,
                       batch_size=B, seed=seed, keep_samples=True, spin_yield_playouts=spin,
                       min_launch_rows=512, max_launch_wait_us=2000)
    r.start()
    r.wait_rows(threads * ppt * B * polls, timeout_s=300)
    r.stop()
    st = r.stats()
    samples = r.fetch_samples()
    r.close()
    # the configuration under test actually ran: merged launches, the two-board trunk
    assert st["segments"] > 1.5 * st["kernel_launches"], st
    assert st["large_launches"] > 0, st
    by_pool = {}
    for s in samples:
        pool = int(s["match_identifier"].split("_")[1][1:])    # gpu<d>_p<i>_<slot>_<count>
        by_pool.setdefault(pool, []).append(s)

    ocfg = _oracle_conf(conf, spin)
    checked = 0
    for pool in check_pools:
        mine = by_pool.get(pool, [])
        man = P.Manager(setup.ref_sm, setup.ref_planes, B, P.UniqueStates(setup.ref_planes.hash_mask(), 1000),
                        "t", seed, pool * B, list(t.policy_dist_count), t.num_rewards, setup.num_prev_states)
        man.start(ocfg)
        pred = (0, [np.zeros(0, np.float32)] * setup.sm.role_count, np.zeros(0, np.float32))
        for it in range(3 * polls):
            if len(man.samples) >= len(mine):
                break
            if it % 200 == 0:
                print("oracle pool %d poll %d: %d/%d samples" % (pool, it, len(man.samples), len(mine)), flush=True)
            buf = man.poll(*pred)
            assert buf is not None
            x = buf.reshape(-1, t.num_channels, t.num_cols, t.num_rows)
            outs = net.forward(x)
            pred = (x.shape[0], outs[:-1], outs[-1])
        n = min(len(mine), len(man.samples))
        assert n >= 1 and n == len(mine), (pool, len(mine), len(man.samples))
        got = [sample_key(setup, _suffix(s), True) for s in mine[:n]]
        exp = [sample_key(setup, _suffix(s), False) for s in man.samples[:n]]
        assert got == exp, pool
        checked += n
    assert checked >= 8
    print("%s: %d samples of %d pools identical to the oracle; runner stats %s" % (case, checked, len(check_pools), st))
