"""Bit-exact parity of the native PUCT / self-play engine (libgz_engine.so through the reference's
poll protocol) with the oracle restatement (oracle/puct_ref.py): identical planes at every poll,
identical samples (policies, visits, scores, match ids) and identical root visit counts, given the
same network outputs.  Small cases only (the oracle is pure Python)."""
import json
import os

import numpy as np
import pytest

from galvanise_zero_amd import cppinterface
from galvanise_zero_amd.defs import templates
from puct_harness import Setup, run_native_supervisor, run_oracle_supervisor, sample_key
from oracle import games_ref
from oracle import puct_ref as P

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _selfplay_conf(evals, noise, backup_finalised, abort=-1):
    conf = templates.selfplay_config_template()
    conf.evals_per_move = evals
    conf.puct_config.dirichlet_noise_pct = noise
    conf.puct_config.backup_finalised = backup_finalised
    conf.run_to_end_puct_config.dirichlet_noise_pct = noise if noise < 0 else 0.15
    conf.run_to_end_puct_config.backup_finalised = backup_finalised
    conf.abort_max_length = abort
    return conf


@pytest.fixture(scope="module")
def small():
    return Setup("breakthroughSmall")


@pytest.mark.parametrize("noise,bf,abort,seed", [(-1, True, -1, 3), (0.25, True, -1, 4), (0.25, False, 10, 5)])
def test_supervisor_selfplay_parity(small, noise, bf, abort, seed):
    conf = _selfplay_conf(20, noise, bf, abort)
    polls = 1500
    nlog, nsamples, nstats, _ = run_native_supervisor(small, conf, 4, polls, seed=seed)
    olog, osamples, man = run_oracle_supervisor(small, conf, 4, polls, seed=seed, native_log=nlog)
    assert len(nlog) == len(olog) == polls
    a = [sample_key(small, s, True) for s in nsamples]
    b = [sample_key(small, s, False) for s in osamples]
    assert a == b
    if abort < 0:
        assert len(a) > 20
    assert nstats["evaluations"] == sum(x.shape[0] for x in nlog[:-1]) // (small.transformer.num_channels *
                                                                          small.transformer.channel_size)


def _player_run(setup, conf, evals, moves, seed):
    """Play `moves` moves of PlayPoller vs the oracle Player from the initial state; returns the
    per-move root (move, traversals, policy_prob) lists of both."""
    ct = cppinterface.create_c_transformer(setup.transformer)
    cp = cppinterface._CPlayer(setup.sm, ct, conf, seed=seed)
    op = P.Player(setup.ref_sm, setup.ref_planes, conf, list(setup.transformer.policy_dist_count),
                  setup.transformer.num_rewards, setup.num_prev_states, seed=seed)
    cp.player_reset(0)
    op.reset(0)
    words = setup.sm.get_initial_state()
    out_n, out_o = [], []
    for m in range(moves):
        state = games_ref.words_to_state(words)
        cp.player_move(words, evals)
        op.move(state, evals)
        arrays = setup.empty_arrays()
        pred = (0, arrays[:-1], arrays[-1])
        while True:
            bn = cp.poll(len(arrays[0]), arrays)
            bo = op.poll(*pred)
            if bn is None or bo is None:
                assert bn is None and bo is None
                break
            assert np.array_equal(np.array(bn), bo)
            arrays = setup.nn(np.array(bn))
            pred = (arrays[0].shape[0], arrays[:-1], arrays[-1])
        sm = setup.sm
        sm.update_bases(words)
        lead = 0 if len(sm.get_legal_state(0)) > 1 else 1
        gn = cp.player_get_move(lead)
        go = op.get_move(lead)
        assert gn[0] == go[0] and gn[2] == go[2] and abs(gn[1] - go[1]) == 0
        rn, ro = cp.root_children(), op.root_children()
        assert [(a, t) for a, t, _ in rn] == [(a, t) for a, t, _ in ro]
        assert [np.float32(p) for _, _, p in rn] == [np.float32(p) for _, _, p in ro]
        out_n.append(rn)
        joint = [gn[0] if r == lead else 0 for r in range(2)]
        cp.player_apply_move(joint)
        op.apply_move(tuple(joint))
        # drive the apply_move coroutines (no evaluation normally needed)
        arrays = setup.empty_arrays()
        pred = (0, arrays[:-1], arrays[-1])
        while True:
            bn = cp.poll(0, arrays)
            bo = op.poll(*pred)
            if bn is None or bo is None:
                assert bn is None and bo is None
                break
            arrays = setup.nn(np.array(bn))
            bo2 = op.poll(arrays[0].shape[0], arrays[:-1], arrays[-1])
        words = sm.next_state(joint)
        sm.update_bases(words)
        if sm.is_terminal():
            break
    return out_n


@pytest.mark.parametrize("game,batch,choose,evals", [("breakthroughSmall", 1, "choose_top_visits", 60),
                                                     ("breakthroughSmall", 8, "choose_top_visits", 150),
                                                     ("breakthrough", 1, "choose_temperature", 40)])
def test_player_visit_counts_bit_exact(game, batch, choose, evals):
    setup = Setup(game)
    conf = templates.base_puct_config(batch_size=batch, choose=choose, dirichlet_noise_pct=0.25,
                                      think_time=-1, converged_visits=1)
    visits = _player_run(setup, conf, evals, 4, seed=9)
    assert sum(t for _, t, _ in visits[0]) > evals // 2


def test_player_golden_visits():
    """Frozen root visit counts (tests/golden/puct_player.json, made by tests/golden/make_puct_golden.py)."""
    g = json.load(open(os.path.join(GOLDEN, "puct_player.json")))
    setup = Setup(g["game"])
    conf = templates.base_puct_config(**g["conf"])
    visits = _player_run(setup, conf, g["evals"], g["moves"], seed=g["seed"])
    assert [[list(x[:2]) for x in mv] for mv in visits] == g["root_visits"]


def test_workers_deterministic(small):
    """Two worker threads (2 pools each): per-pool RNG streams + per-pool duplicate filter make the
    sample set independent of thread interleaving."""
    conf = _selfplay_conf(16, 0.25, True)
    runs = []
    for _ in range(2):
        _, samples, stats, keep = run_native_supervisor(small, conf, 3, 1200, seed=21, workers=2)
        # samples are collected every poll; flush what remains
        sup = keep[0]
        samples = samples + (sup.fetch_samples() or [])
        runs.append(sorted((s["match_identifier"], s["depth"], json.dumps(s["policies"])) for s in samples))
        del keep
    assert runs[0] == runs[1] and len(runs[0]) > 0


def test_spin_yield_keeps_each_game_identical(small):
    """spin_yield_playouts (build extension, engine/config.h) only reorders coroutines inside a
    pool: every game's own samples are unchanged (per-game RNG, batch-independent predictions).
    Yielding after every NN-free playout is the most disruptive setting."""
    runs = []
    for spin in (0, 1):
        conf = _selfplay_conf(16, 0.25, True)
        conf.puct_config.spin_yield_playouts = spin
        conf.run_to_end_puct_config.spin_yield_playouts = spin
        log, samples, stats, keep = run_native_supervisor(small, conf, 4, 900, seed=31)
        by_game = {}
        for s in samples:
            by_game.setdefault(s["match_identifier"], []).append(sample_key(small, s, True))
        runs.append((by_game, log))
        del keep
    (a, log_a), (b, log_b) = runs
    common = set(a) & set(b)
    assert len(common) >= 3
    for k in common:
        n = min(len(a[k]), len(b[k]))
        assert a[k][:n] == b[k][:n], k
    # the yields did change the batch composition (otherwise the test proves nothing)
    assert any(x.shape != y.shape or not np.array_equal(x, y) for x, y in zip(log_a, log_b))


@pytest.mark.parametrize("spin", [1, 3])
def test_spin_yield_matches_oracle(small, spin):
    """The oracle models the spin-yield extension (puct_ref.Evaluator.playout_main): native and
    oracle stay bit-identical batch by batch with it on, so runner pools (bench default 1000) can
    be replayed through the oracle exactly (tests/test_runner_gpu.py)."""
    import attr
    conf = _selfplay_conf(16, 0.25, False)
    d = attr.asdict(conf)
    for k in ("puct_config", "run_to_end_puct_config"):
        d[k]["spin_yield_playouts"] = spin
    nlog, nsamples, _, _ = run_native_supervisor(small, d, 4, 900, seed=31)
    olog, osamples, _ = run_oracle_supervisor(small, d, 4, 900, seed=31, native_log=nlog)
    assert len(nlog) == len(olog) == 900
    assert [sample_key(small, s, True) for s in nsamples] == [sample_key(small, s, False) for s in osamples]
    assert len(nsamples) > 5


def test_spin_fast_path_identical():
    """The root spin fast path (evaluator.cpp spinRun / spinRunRegs: root -> finalised win playouts
    without the full selection pass) changes nothing: breakthrough 8x8 self-play with it on, off,
    on without the register-resident runs, and on with
    GZ_VERIFY_FASTPATH=1 (every spin playout re-selected by the ordinary path, abort on mismatch)
    gives identical samples; the run reaches the multi-win spin (tree playouts >> evaluations)."""
    import subprocess
    import sys
    script = os.path.join(os.path.dirname(__file__), "native", "spin_check.py")
    outs = []
    # GZ_SPIN_FAST=2: the fast path without the register-resident runs (evaluator.cpp spinRunRegs)
    # GZ_SPIN_VEC: 2 (default) the AVX2 register loops in blocks of eight playouts (evaluator.cpp
    # spin_wins_b), 1 the AVX2 loops per playout (spin_wins_v), 0 the scalar ones (spin_wins)
    # (the six runs are independent processes: run side by side)
    procs = []
    for env in ({"GZ_SPIN_FAST": "0"}, {"GZ_SPIN_FAST": "1"}, {"GZ_SPIN_FAST": "2"},
                {"GZ_SPIN_FAST": "1", "GZ_VERIFY_FASTPATH": "1"}, {"GZ_SPIN_FAST": "1", "GZ_SPIN_VEC": "1"},
                {"GZ_SPIN_FAST": "1", "GZ_SPIN_VEC": "0"}):
        e = dict(os.environ, **env)
        procs.append(subprocess.Popen([sys.executable, script, "breakthrough", "16", "3000", "100"], env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    for pr in procs:
        out, err = pr.communicate(timeout=600)
        assert pr.returncode == 0, err[-2000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
    assert all(o == outs[0] for o in outs[1:])
    assert outs[0]["samples"] > 50 and outs[0]["tree_playouts"] > 3 * outs[0]["evaluations"]


def test_spin_fast_path_identical_root_latch():
    """The spin fast path through the root latch (evaluator.cpp:461-475: past 1,000 root visits each
    reached child draws rng.get() in sorted order and a child holding over 66 % of the traversals is
    left out when its draw exceeds 0.1).  Deep in a multi-win spin one win often holds the latch; the
    register loops read that win's draw at its sorted position and discard the others.  A cheap
    synthetic network takes breakthrough to its deep spins at 400 evals/move; every mode -- fast path
    off (the reference's loop), on, without register runs, verified, each register loop -- gives
    identical samples and counters, and the fast path really read latch draws (GZ_SPIN_STATS)."""
    import subprocess
    import sys
    script = os.path.join(os.path.dirname(__file__), "native", "spin_check.py")
    procs = []
    for env in ({"GZ_SPIN_FAST": "0"}, {"GZ_SPIN_FAST": "1", "GZ_SPIN_STATS": "1"}, {"GZ_SPIN_FAST": "2"},
                {"GZ_SPIN_FAST": "1", "GZ_VERIFY_FASTPATH": "1"}, {"GZ_SPIN_FAST": "1", "GZ_SPIN_VEC": "1"},
                {"GZ_SPIN_FAST": "1", "GZ_SPIN_VEC": "0"}):
        e = dict(os.environ, **env)
        procs.append(subprocess.Popen([sys.executable, script, "breakthrough", "8", "8000", "400", "fake"], env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs, errs = [], []
    for pr in procs:
        out, err = pr.communicate(timeout=900)
        assert pr.returncode == 0, err[-2000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
        errs.append(err)
    assert all(o == outs[0] for o in outs[1:])
    assert outs[0]["samples"] > 20 and outs[0]["tree_playouts"] > 30 * outs[0]["evaluations"]
    stats = [ln for ln in errs[1].splitlines() if ln.startswith("gz spin stats:")]
    assert stats, errs[1][-2000:]
    fields = dict(kv.split("=") for kv in stats[-1].split(":", 1)[1].split())
    assert int(fields["latch_draws"]) > 100000, fields


def test_player_root_latch_bit_exact():
    """Past 1000 root visits the reference's root latch draws the RNG once per reaching child in
    sorted order (evaluator.cpp:461-475); the engine's unsorted fast path must draw identically."""
    setup = Setup("breakthroughSmall")
    conf = templates.base_puct_config(batch_size=1, choose="choose_top_visits", dirichlet_noise_pct=0.25,
                                      think_time=-1, converged_visits=1)
    visits = _player_run(setup, conf, 1400, 2, seed=13)
    assert sum(t for _, t, _ in visits[0]) > 1000


@pytest.mark.parametrize("game,polls,evals", [("reversi", 2500, 12), ("hexLG13", 300, 8), ("amazons_10x10", 120, 6)])
def test_supervisor_selfplay_parity_other_games(game, polls, evals):
    """reversi (3-value draw head, pass moves), hexLG13 (policy heads 170/171), amazons_10x10
    (12 planes, 3041 moves, 4 turn planes): every batch of planes and every sample bit-identical
    between the native engine and the oracle restatement."""
    setup = Setup(game, draw_head=(game == "reversi"))
    conf = _selfplay_conf(evals, 0.25, True, -1)
    conf.run_to_end_evals = 4
    nlog, nsamples, _, _ = run_native_supervisor(setup, conf, 4, polls, seed=11)
    olog, osamples, _ = run_oracle_supervisor(setup, conf, 4, polls, seed=11, native_log=nlog)
    assert len(nlog) == len(olog) == polls
    assert [sample_key(setup, s, True) for s in nsamples] == [sample_key(setup, s, False) for s in osamples]
    if game == "reversi":
        assert len(nsamples) > 0


@pytest.mark.parametrize("game,evals", [("reversi", 40), ("hexLG13", 30), ("amazons_10x10", 20)])
def test_player_visit_counts_bit_exact_other_games(game, evals):
    setup = Setup(game, draw_head=(game == "reversi"))
    conf = templates.base_puct_config(batch_size=4, choose="choose_temperature", dirichlet_noise_pct=0.25,
                                      think_time=-1, converged_visits=1)
    visits = _player_run(setup, conf, evals, 3, seed=13)
    assert sum(t for _, t, _ in visits[0]) > evals // 2
