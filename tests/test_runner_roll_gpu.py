"""Generation roll on a live runner (the reference's worker.py:138-160: Supervisor.update_nn +
clear_unique_states while self-play continues; cppinterface.py:146-147, supervisor_impl.cpp:138-144).

gz_runner_update_network swaps the network between two launches (no pool batch runs on two
networks) and clears the duplicate filters: a pool's own filter just before its engine thread
delivers the pool's first batch on the new network, the shared filter at once.  With per-pool
filters the run stays deterministic, so one pool replayed through the oracle -- network A's outputs
for its batches before the roll, B's after, its filter cleared at the same batch -- must emit
exactly the runner's samples.  With the shared filter (the reference's, nondeterministic across
pools by design: quirk 8) the roll must complete, launches continue and the net must compute B.
"""
import numpy as np
import pytest

from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob
from puct_harness import Setup, sample_key

pytestmark = pytest.mark.gpu


def _suffix(s):
    s = dict(s)
    s["match_identifier"] = "_".join(s["match_identifier"].split("_")[-2:])
    return s


@pytest.mark.timeout(900)
@pytest.mark.parametrize("per_pool", [True, False])
def test_generation_roll_live_runner(per_pool, hip_device):
    import attr
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    from oracle import puct_ref as P
    desc = BASELINE_CONFIGS[2]["desc"]
    setup = Setup("breakthrough")
    t = setup.transformer
    wa, wb = to_blob(random_weights(desc, 7921)), to_blob(random_weights(desc, 7922))
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(wa)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 8
    conf.run_to_end_evals = 4
    B, threads, ppt, seed, spin = 32, 2, 4, 20251017, 1000
    r = SelfPlayRunner(net, setup.sm, t, conf, device=hip_device, num_threads=threads, pools_per_thread=ppt,
                       batch_size=B, seed=seed, keep_samples=True, spin_yield_playouts=spin,
                       min_launch_rows=128, max_launch_wait_us=2000, per_pool_unique_states=per_pool)
    r.start()
    r.wait_rows(threads * ppt * B * 300, timeout_s=300)
    before = r.stats()
    roll = r.update_network(wb, clear_unique_states=True)
    r.wait_rows(before["rows"] + threads * ppt * B * 300, timeout_s=300)
    r.stop()
    st = r.stats()
    samples = r.fetch_samples()
    r.close()
    print("roll", roll, "stats before", before, "after", st)
    assert st["kernel_launches"] > roll["launches_before"] > 0
    assert all(k > 0 for k in roll["pool_batches"]), roll
    # the net now computes network B exactly (a fresh net with B's weights, bit for bit)
    x = random_planes(desc, 64, 5)
    fresh = HipNet(desc, hip_device, "bf16x3")
    fresh.set_weights(wb)
    for a, b in zip(net.forward(x), fresh.forward(x)):
        assert np.array_equal(a, b)
    if not per_pool:
        assert st["samples"] > before["samples"]
        return
    # replay one pool through the oracle: A before the roll, B after, filter cleared at the roll
    neta = HipNet(desc, hip_device, "bf16x3")
    neta.set_weights(wa)
    pool = 5
    mine = [s for s in samples if int(s["match_identifier"].split("_")[1][1:]) == pool]
    k = roll["pool_batches"][pool]
    us = P.UniqueStates(setup.ref_planes.hash_mask(), 1000)
    man = P.Manager(setup.ref_sm, setup.ref_planes, B, us, "t", seed, pool * B, list(t.policy_dist_count),
                    t.num_rewards, setup.num_prev_states)
    d = attr.asdict(conf)
    for key in ("puct_config", "run_to_end_puct_config"):
        d[key]["spin_yield_playouts"] = spin
    man.start(d)
    pred = (0, [np.zeros(0, np.float32)] * setup.sm.role_count, np.zeros(0, np.float32))
    batch = 0
    while len(man.samples) < len(mine) and batch < 5000:
        if batch == k + 1:          # this poll delivers batch k, the pool's first on network B
            us.lookup.clear()
        buf = man.poll(*pred)
        assert buf is not None
        xb = buf.reshape(-1, t.num_channels, t.num_cols, t.num_rows)
        outs = (neta if batch < k else net).forward(xb)
        pred = (xb.shape[0], outs[:-1], outs[-1])
        batch += 1
    n = len(mine)
    assert n >= 4 and len(man.samples) >= n, (n, len(man.samples))
    got = [sample_key(setup, _suffix(s), True) for s in mine]
    exp = [sample_key(setup, _suffix(s), False) for s in man.samples[:n]]
    assert got == exp
    print("pool %d: %d samples identical to the oracle across the roll at batch %d" % (pool, n, k))


@pytest.mark.timeout(300)
def test_roll_timeout_withdraws_and_next_roll_succeeds(hip_device):
    """A roll whose wait times out is withdrawn before gz_runner_update_network returns (the caller
    may free its blob at once), or -- when the launcher had already claimed it -- waited for; either
    way the runner keeps playing and the next roll succeeds (no dangling pending roll)."""
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    desc = BASELINE_CONFIGS[2]["desc"]
    setup = Setup("breakthrough")
    wa, wb = to_blob(random_weights(desc, 7921)), to_blob(random_weights(desc, 7922))
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(wa)
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 8
    r = SelfPlayRunner(net, setup.sm, setup.transformer, conf, device=hip_device, num_threads=2, pools_per_thread=2,
                       batch_size=32, seed=3, spin_yield_playouts=1000, min_launch_rows=64, max_launch_wait_us=2000)
    r.start()
    r.wait_rows(128 * 50, timeout_s=120)
    outcomes = []
    for _ in range(5):
        blob = wb.copy()
        try:
            r.update_network(blob, clear_unique_states=False, timeout_s=1e-7)
            outcomes.append("applied")
        except RuntimeError as e:
            assert "(-2)" in str(e), e
            outcomes.append("withdrawn")
        del blob                    # freed right after the call returned
        r.wait_rows(r.stats()["rows"] + 128 * 5, timeout_s=60)
    roll = r.update_network(wa, clear_unique_states=False, timeout_s=60)
    r.wait_rows(r.stats()["rows"] + 128 * 20, timeout_s=60)
    r.stop()
    r.close()
    print("short-timeout rolls:", outcomes, "final roll", roll)
    assert roll["launches_before"] > 0


@pytest.mark.timeout(300)
def test_concurrent_rolls_one_owner(hip_device):
    """Two callers roll at once: a caller arriving while the other's roll is pending,
    being applied or not yet collected is rejected ("already pending"); a call that returns 0 had its
    network applied -- so the net ends on the weights of the last successful call to return."""
    import threading
    import time
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    desc = BASELINE_CONFIGS[2]["desc"]
    setup = Setup("breakthrough")
    blobs = [to_blob(random_weights(desc, 7921 + i)) for i in range(3)]
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(blobs[0])
    conf = templates.selfplay_config_template()
    conf.evals_per_move = 8
    r = SelfPlayRunner(net, setup.sm, setup.transformer, conf, device=hip_device, num_threads=2, pools_per_thread=2,
                       batch_size=32, seed=5, spin_yield_playouts=1000, min_launch_rows=64, max_launch_wait_us=2000)
    r.start()
    r.wait_rows(128 * 50, timeout_s=120)
    x = random_planes(desc, 16, 9)
    refs = []
    for b in blobs:
        f = HipNet(desc, hip_device, "bf16x3")
        f.set_weights(b)
        refs.append(f.forward(x))
    rejected = accepted_both = 0
    for trial in range(6):
        res = {}
        go = threading.Barrier(2)

        def roll(i):
            go.wait()
            try:
                r.update_network(blobs[i], clear_unique_states=False, timeout_s=60)
                res[i] = ("ok", time.perf_counter())
            except RuntimeError as e:
                res[i] = ("err", str(e))

        th = [threading.Thread(target=roll, args=(i,)) for i in (1, 2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        ok = sorted((v[1], i) for i, v in res.items() if v[0] == "ok")
        errs = [v[1] for v in res.values() if v[0] == "err"]
        assert ok, res                                  # at least one caller owns the roll
        for e in errs:
            assert "already pending" in e, e
        rejected += len(errs)
        accepted_both += len(ok) == 2
        last = ok[-1][1]
        r.wait_rows(r.stats()["rows"] + 128 * 5, timeout_s=60)
        got = net.forward(x)
        for a, b in zip(got, refs[last]):
            assert np.array_equal(a, b), (trial, res)
    r.stop()
    r.close()
    print("concurrent rolls: %d rejected, %d trials with both applied in turn" % (rejected, accepted_both))


@pytest.mark.timeout(400)
def test_runner_recreate_reuses_node_memory(hip_device):
    """Trees freed by gz_runner_destroy on the caller's thread go back to the process-wide node pool
    (node_cache_flush), so a second runner's games reuse them: the second create / play / destroy
    cycle adds far less resident memory than the first."""
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    import bench

    def rss_gb():
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * 4096 / 1e9

    sm, t, desc = bench.setup_game(2)
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(to_blob(random_weights(desc, 7921)))
    grow = []
    for cycle in range(2):
        before = rss_gb()
        r = SelfPlayRunner(net, sm, t, bench.selfplay_conf("template", 800), device=hip_device, num_threads=8,
                           pools_per_thread=2, batch_size=64, seed=11, spin_yield_playouts=1000,
                           min_launch_rows=1024, max_launch_wait_us=3000)
        r.start()
        r.wait_rows(2_000_000, timeout_s=150)
        r.stop()
        peak = rss_gb()
        r.close()
        grow.append(peak - before)
        print("cycle %d: rss %.2f -> %.2f GB (+%.2f), after destroy %.2f GB" % (cycle, before, peak, peak - before,
                                                                                rss_gb()))
    assert grow[0] > 0.3, grow                 # the first cycle built real trees
    assert grow[1] < 0.5 * grow[0], grow       # the second reused the freed blocks
