"""bench.py's own paths on the GPU: the single-rank line carries the contract's keys, and
`--gpus 2` starts two ranks itself (torch.distributed.run) that broadcast the weight blob, load it
with gz_net_set_weights_device, run the native runner on disjoint global game ranges, roll the live
runners to a second broadcast generation (--roll) and report n_gpus = 2.  The two ranks share GPU 0 over gloo here (one GPU per box; RCCL needs one GPU per
rank); the driver's 8-GPU run uses RCCL.  Reference: distributed/worker.py:107-160, SURVEY 8e."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

SMALL = ["--age-seconds", "0", "--warmup", "1", "--steps", "2", "--step-rows", "65536", "--threads", "2",
         "--pools", "2", "--batch", "64", "--no-cpu-baseline"]


def _run(args, timeout=300):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_single_rank_line(hip_device):
    out = _run(["--gpus", "1"] + SMALL)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "games_per_sec", "steady_state"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["value"] > 0
    assert out["roofline"]["bound"] == "mfma" and 0 < out["roofline"]["frac"] < 1


def test_bench_two_ranks(hip_device):
    out = _run(["--gpus", "2", "--backend", "gloo", "--device", "0", "--roll"] + SMALL, timeout=400)
    assert out["n_gpus"] == 2
    assert out["config"]["weights_broadcast"]["identical_on_all_ranks"] is True
    # the mid-run generation roll: broadcast to both ranks, applied by both live runners
    assert out["generation_roll"]["identical_on_all_ranks"] is True
    rng = out["config"]["game_ranges"]
    assert rng["disjoint"] is True and len(rng["per_rank"]) == 2
    assert rng["per_rank"][0][1] - rng["per_rank"][0][0] == out["config"]["games_per_gpu"]
    assert out["value"] > 0
