"""The generation roll's weight load on the device (the reference swaps networks between poll loops:
worker.py:138-160, cppinterface.py:146-147; here the new blob arrives in HBM by an RCCL broadcast,
SURVEY 8e): gz_net_set_weights_device folds BatchNorm and packs the bf16 hi / lo MFMA fragments with
HIP kernels reading the blob in place.  It must build exactly the image the host path
(gz_net_set_weights) builds -- byte for byte, so every forward is bit-identical whichever way the
weights arrived -- for every head and trunk kind: v1 / legacy (conv biases, value BN, sigmoid), v2
(squeeze-excite, pooling and concat-all-layers value heads), large policies (the split GEMM heads'
fragments), both arithmetic modes, padded filter counts."""
import json
import os
import time

import numpy as np
import pytest

from galvanise_zero_amd.nn.desc import BASELINE_CONFIGS, NetDesc
from galvanise_zero_amd.nn.weights import random_planes, random_weights, to_blob

pytestmark = pytest.mark.gpu

with open(os.path.join(os.path.dirname(__file__), "golden", "keras_descs.json")) as _f:
    _FILES = {k: NetDesc(**v["desc"]) for k, v in json.load(_f).items() if "desc" in v}

NETS = {
    "cfg2": BASELINE_CONFIGS[2]["desc"],
    "cfg4": BASELINE_CONFIGS[4]["desc"],
    "cfg5": BASELINE_CONFIGS[5]["desc"],
    "x6_102_legacy": _FILES["breakthrough/models/x6_102.json"],
    "b1_58_v2_gap": _FILES["breakthroughSmall/models/b1_58.json"],
    "f1_581_v2_k0_160": _FILES["draughts_killer/models/f1_581.json"],
    "h2_477_v2_concat_19x19": _FILES["hex19/models/h2_477.json"],
    "v3_leaky_f96": NetDesc(5, 8, 8, 96, 2, [65, 65], num_values=3, leaky_relu=True, flatten_nchw=True),
}


@pytest.mark.parametrize("precision", ["bf16x3", "bf16"])
@pytest.mark.parametrize("name", sorted(NETS))
def test_device_roll_image_identical(name, precision, hip_device):
    import torch
    from galvanise_zero_amd._native import HipNet
    desc = NETS[name]
    blob = to_blob(random_weights(desc, 7922, bias_std=0.2))
    host = HipNet(desc, hip_device, precision)
    host.set_weights(blob)
    dev = HipNet(desc, hip_device, precision)
    t = torch.from_numpy(blob).to("cuda")
    torch.cuda.synchronize()
    dev.set_weights_device(t.data_ptr(), t.numel())
    a, b = host.weight_image(), dev.weight_image()
    assert a.size == b.size and a.size > 0
    diff = np.flatnonzero(a != b)
    assert diff.size == 0, "%d bytes differ of %d; first: %s" % (
        diff.size, a.size, [(int(i), int(a[i]), int(b[i])) for i in diff[:12]])
    x = random_planes(desc, 9, 3)
    for u, v in zip(host.forward(x), dev.forward(x)):
        assert np.array_equal(u, v)
    print("%s %s: %d-byte image identical; device fold + pack %.3f ms" % (name, precision, a.size, dev.last_roll_ms()))
    host.close()
    dev.close()


def test_device_roll_orders_after_async_copy(hip_device):
    """gz_net_set_weights_device needs no caller-side synchronisation: the blob is
    written by an asynchronous pinned-host copy on torch's current stream, with no
    torch.cuda.synchronize() before the call (and a large unrelated copy queued ahead of it, so the
    blob is still in flight when the call starts); the packed image must equal the host path's."""
    import torch
    from galvanise_zero_amd._native import HipNet
    desc = NETS["cfg5"]
    blob = to_blob(random_weights(desc, 7923))
    host = HipNet(desc, hip_device, "bf16x3")
    host.set_weights(blob)
    dev = HipNet(desc, hip_device, "bf16x3")
    for _ in range(3):
        pinned = torch.from_numpy(blob).pin_memory()
        ballast = torch.empty(1 << 28, dtype=torch.uint8).pin_memory()
        d_ballast = torch.empty_like(ballast, device="cuda")
        t = torch.zeros(blob.size, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        d_ballast.copy_(ballast, non_blocking=True)   # 256 MB ahead of the blob on the same stream
        t.copy_(pinned, non_blocking=True)
        dev.set_weights_device(t.data_ptr(), t.numel())
        a, b = host.weight_image(), dev.weight_image()
        assert np.array_equal(a, b), "%d bytes differ" % np.count_nonzero(a != b)
    host.close()
    dev.close()


def test_device_roll_faster_than_round_trip(hip_device, monkeypatch):
    """The device fold / pack against the round trip it replaces (D2H copy of the blob, host fold and
    pack, H2D upload; GZ_HOST_WEIGHT_ROLL=1), on amazons' 20 x 256 net (cfg5: 24.9 M parameters)."""
    import torch
    from galvanise_zero_amd._native import HipNet
    desc = NETS["cfg5"]
    blob = to_blob(random_weights(desc, 7922))
    t = torch.from_numpy(blob).to("cuda")
    net = HipNet(desc, hip_device, "bf16x3")
    times = {}
    for mode in ("device", "round_trip"):
        if mode == "round_trip":
            monkeypatch.setenv("GZ_HOST_WEIGHT_ROLL", "1")
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            net.set_weights_device(t.data_ptr(), t.numel())
            best = min(best, time.perf_counter() - t0)
        times[mode] = best * 1e3
    print("cfg5 weight roll: device %.1f ms (kernels %.2f ms), round trip %.1f ms" %
          (times["device"], net.last_roll_ms(), times["round_trip"]))
    assert times["device"] < times["round_trip"]
    net.close()
