"""The deep BASELINE configs at their real depth through the native runner, against the oracle.

hexLG13 (configs[3], 12 x 256 on 13 x 13: the two-pass split trunk) and amazons_10x10 (configs[4],
20 x 256 on 10 x 10 with 12 planes and 3,041-move policies: the single-image split trunk plus the
policy GEMM and heads launches) run their full nets inside gz_runner's segmented launches (several
pools merged per launch, pinned-host segments, HBM staging), in split precision as bench.py runs
them.  One pool per engine thread is replayed through the oracle (oracle/puct_ref.Manager, the
reference's SelfPlayManager) with the network outputs of the same HIP forward; every sample the
runner emits for it must be identical field for field.

Games are made short with the reference's own resignation knobs so that samples appear within a few
hundred batches: resign0/1 at score < 0.95 in every game (resign*_pct 0), and run-to-end ending
early once the lead's score is below 0.99 from depth 0 (selfplay.cpp:43-74, 171-228).
Reference: src/cpp/selfplay.cpp:76-337, src/cpp/supervisor.cpp:79-99,196-245, model.py:154-296.
"""
import attr
import numpy as np
import pytest

from galvanise_zero_amd.defs import templates
from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS
from galvanise_zero_amd.nn.weights import random_weights, to_blob
from puct_harness import Setup, sample_key

pytestmark = pytest.mark.gpu


def _short_game_conf(evals, sample_every_move=False):
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    if sample_every_move:        # every unique state is sampled (selfplay.cpp:104-118)
        conf.oscillate_sampling_pct = 1.0
    conf.run_to_end_evals = 4
    conf.resign0_score_probability = conf.resign1_score_probability = 0.95
    conf.resign0_pct = conf.resign1_pct = 0.0
    conf.run_to_end_pct = 0.0
    conf.run_to_end_early_score = 0.99
    conf.run_to_end_minimum_game_depth = 0
    return conf


def _suffix(s):
    s = dict(s)
    s["match_identifier"] = "_".join(s["match_identifier"].split("_")[-2:])
    return s


# case: (config, game, batch, polls, evals per move, every move sampled, samples required)
# amazons_cfg5_deep: >= 32 evaluations per sampled move, so the selection over amazons'
# ~2,000-child roots runs many playouts per move on the GPU forward, and >= 50 compared samples
CASES = {"hexLG13_cfg4": (4, "hexLG13", 16, 250, 6, False, 4), "amazons_cfg5": (5, "amazons_10x10", 8, 160, 6, False, 4),
         "amazons_cfg5_deep": (5, "amazons_10x10", 8, 900, 32, True, 50)}


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("case", list(CASES))
def test_deep_config_runner_matches_oracle(case, hip_device):
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    from oracle import puct_ref as P
    cfg, game, B, polls, evals, every_move, need = CASES[case]
    desc = BASELINE_CONFIGS[cfg]["desc"]
    setup = Setup(game)
    t = setup.transformer
    assert (t.num_channels, t.num_cols, t.num_rows, list(t.policy_dist_count)) == \
        (desc.input_channels, desc.input_columns, desc.input_rows, list(desc.policy_dist_count))
    net = HipNet(desc, hip_device, "bf16x3")          # bench.py's arithmetic: bf16x3 split
    net.set_weights(to_blob(random_weights(desc, 7921)))
    conf = _short_game_conf(evals, every_move)
    seed, threads, ppt, spin = 20251019, 2, 2, 1000
    r = SelfPlayRunner(net, setup.sm, t, conf, device=hip_device, num_threads=threads, pools_per_thread=ppt,
                       batch_size=B, seed=seed, keep_samples=True, spin_yield_playouts=spin,
                       min_launch_rows=2 * B, max_launch_wait_us=3000)
    r.start()
    r.wait_rows(threads * ppt * B * polls, timeout_s=400)
    r.stop()
    st = r.stats()
    samples = r.fetch_samples()
    r.close()
    print(case, "runner stats", st)
    assert st["segments"] > 1.2 * st["kernel_launches"], st      # pools merged into launches
    by_pool = {}
    for s in samples:
        by_pool.setdefault(int(s["match_identifier"].split("_")[1][1:]), []).append(s)
    d = attr.asdict(conf)
    for k in ("puct_config", "run_to_end_puct_config"):
        d[k]["spin_yield_playouts"] = spin
    checked = 0
    for pool in (0, ppt):                          # one pool of each engine thread
        mine = by_pool.get(pool, [])
        man = P.Manager(setup.ref_sm, setup.ref_planes, B, P.UniqueStates(setup.ref_planes.hash_mask(), 1000),
                        "t", seed, pool * B, list(t.policy_dist_count), t.num_rewards, setup.num_prev_states)
        man.start(d)
        pred = (0, [np.zeros(0, np.float32)] * setup.sm.role_count, np.zeros(0, np.float32))
        for it in range(4 * polls):
            if len(man.samples) >= len(mine):
                break
            if it % 50 == 0:
                print("oracle pool %d poll %d: %d/%d samples" % (pool, it, len(man.samples), len(mine)), flush=True)
            buf = man.poll(*pred)
            assert buf is not None
            x = buf.reshape(-1, t.num_channels, t.num_cols, t.num_rows)
            outs = net.forward(x)
            pred = (x.shape[0], outs[:-1], outs[-1])
        n = len(mine)
        assert n >= 1 and len(man.samples) >= n, (pool, n, len(man.samples))
        got = [sample_key(setup, _suffix(s), True) for s in mine]
        exp = [sample_key(setup, _suffix(s), False) for s in man.samples[:n]]
        assert got == exp, pool
        checked += n
    print("%s: %d samples of 2 pools identical to the oracle (%d-block x %d net, %d evals per move)" % (
        case, checked, desc.residual_layers, desc.cnn_filter_size, evals))
    assert checked >= need



def _every_move_conf(evals):
    """The self-play template (resignation possible in 1 % of games, run-to-end at 32 evaluations) at
    `evals` evaluations per move with every move sampled: complete games, whose samples appear at
    the game's end (selfplay.cpp:296-337), not opening-only resigns."""
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    conf.oscillate_sampling_pct = 1.0
    return conf


# case: (config, game, games in the pool, evals per move); every game must complete with >= 20
# samples.  hexLG13's and amazons' complete games take minutes each (amazons: 3.3 min on MI355X,
# a 160-move game; the Python oracle's tree work per evaluation dominates): they run with
# GZ_LONG_TESTS=1 (their logs: profiles/r06g*_replay_*.log); reversi runs in every -m gpu pass.
CASES_200 = {"reversi_cfg3_200": (3, "reversi", 2, 200),
             "hexLG13_cfg4_200": (4, "hexLG13", 1, 200),
             "amazons_cfg5_200": (5, "amazons_10x10", 1, 200)}


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("case", list(CASES_200))
def test_deep_config_runner_matches_oracle_200(case, hip_device):
    """cfg3-5's games through the native runner on their full bench nets (bf16x3) at 200 evaluations
    per move, played to the end: the pool replayed through the oracle with the same HIP forward,
    every sample identical, >= 20 per game (the endgame's spins, terminal wins and draws included)."""
    import os
    import time
    from galvanise_zero_amd._native import HipNet
    from galvanise_zero_amd.runner import SelfPlayRunner
    from oracle import puct_ref as P
    cfg, game, B, evals = CASES_200[case]
    if game != "reversi" and not os.environ.get("GZ_LONG_TESTS"):
        pytest.skip("long oracle replay: GZ_LONG_TESTS=1")
    desc = BASELINE_CONFIGS[cfg]["desc"]
    setup = Setup(game, draw_head=(game == "reversi"))
    t = setup.transformer
    assert (t.num_channels, t.num_cols, t.num_rows, list(t.policy_dist_count), t.num_rewards) == \
        (desc.input_channels, desc.input_columns, desc.input_rows, list(desc.policy_dist_count), desc.num_values)
    net = HipNet(desc, hip_device, "bf16x3")
    net.set_weights(to_blob(random_weights(desc, 7921)))
    conf = _every_move_conf(evals)
    seed, spin = 20251020, 1000
    r = SelfPlayRunner(net, setup.sm, t, conf, device=hip_device, num_threads=1, pools_per_thread=1,
                       batch_size=B, seed=seed, keep_samples=True, spin_yield_playouts=spin,
                       min_launch_rows=1, max_launch_wait_us=0)
    r.start()
    t0 = time.time()
    while r.stats()["games_completed"] < B and time.time() - t0 < 600:
        time.sleep(1)
    r.stop()
    st = r.stats()
    samples = r.fetch_samples()
    r.close()
    per_game = {}
    for s in samples:
        per_game[s["match_identifier"]] = per_game.get(s["match_identifier"], 0) + 1
    print(case, "runner", {k: st[k] for k in ("games_completed", "rows", "tree_playouts")}, "samples per game",
          per_game, "%.0f s" % (time.time() - t0), flush=True)
    assert st["games_completed"] >= B, st
    d = attr.asdict(conf)
    for k in ("puct_config", "run_to_end_puct_config"):
        d[k]["spin_yield_playouts"] = spin
    man = P.Manager(setup.ref_sm, setup.ref_planes, B, P.UniqueStates(setup.ref_planes.hash_mask(), 1000),
                    "t", seed, 0, list(t.policy_dist_count), t.num_rewards, setup.num_prev_states)
    man.start(d)
    pred = (0, [np.zeros(0, np.float32)] * setup.sm.role_count, np.zeros(0, np.float32))
    it = 0
    while len(man.samples) < len(samples):
        if it % 2000 == 0:
            print("oracle poll %d: %d/%d samples" % (it, len(man.samples), len(samples)), flush=True)
        buf = man.poll(*pred)
        assert buf is not None
        x = buf.reshape(-1, t.num_channels, t.num_cols, t.num_rows)
        outs = net.forward(x)
        pred = (x.shape[0], outs[:-1], outs[-1])
        it += 1
    n = len(samples)
    got = [sample_key(setup, _suffix(s), True) for s in samples]
    exp = [sample_key(setup, _suffix(s), False) for s in man.samples[:n]]
    assert got == exp
    done = sorted(per_game.values(), reverse=True)[:B]
    assert len(done) == B and min(done) >= 20, per_game
    print("%s: %d samples identical to the oracle, %s per game (%d-block x %d net, %d evals per move)" % (
        case, n, done, desc.residual_layers, desc.cnn_filter_size, evals))
