"""Native multi-threaded self-play on one GPU (include/gzero_nn.h gz_runner_*): the steady-state
replacement of the reference's per-batch Python poll loop (cppinterface.py:131-144 driven by
distributed/worker.py:191).  Pools, coroutines, planes and NN launches are all native."""
import ctypes
import json

import numpy as np

from . import _native, cppinterface


class SelfPlayRunner(object):
    def __init__(self, hip_net, sm, transformer, conf, device=0, num_threads=8, pools_per_thread=2,
                 batch_size=256, seed=0, game_index_base=0, keep_samples=False, max_launch_rows=0,
                 spin_yield_playouts=0, min_launch_rows=0, max_launch_wait_us=0, per_pool_unique_states=True):
        self.lib = _native.runner_lib()
        _native.engine_lib()
        self.net = hip_net
        self.sm = sm
        self.c_transformer = cppinterface.create_c_transformer(transformer)
        self.cfg = _native.GzRunnerConfig(device, num_threads, pools_per_thread, batch_size, seed,
                                          game_index_base, int(bool(per_pool_unique_states)),
                                          int(keep_samples), max_launch_rows,
                                          min_launch_rows, max_launch_wait_us)
        self.conf = _native.make_selfplay_config(conf)
        # build extension (engine/config.h): 0 keeps the reference's never-yielding playout loop
        self.conf.puct_config.spin_yield_playouts = spin_yield_playouts
        self.conf.run_to_end_puct_config.spin_yield_playouts = spin_yield_playouts
        ps = list(transformer.policy_dist_count)
        self._ps = (ctypes.c_int * len(ps))(*ps)
        self.handle = self.lib.gz_runner_create(hip_net.handle, sm.handle, self.c_transformer.handle,
                                                ctypes.byref(self.cfg), ctypes.byref(self.conf), self._ps,
                                                len(ps), transformer.num_rewards)
        if not self.handle:
            raise RuntimeError("gz_runner_create: %s" % self.lib.gz_runner_last_error().decode())
        self.num_pools = num_threads * pools_per_thread
        self.batch_size = batch_size

    def start(self):
        if self.lib.gz_runner_start(self.handle) != 0:
            raise RuntimeError("gz_runner_start: %s" % self.lib.gz_runner_last_error().decode())

    def clear_unique_states(self):
        """Supervisor.clear_unique_states (supervisor_impl.cpp:138-144) at a generation roll
        (worker.py:160)."""
        if self.lib.gz_runner_clear_unique_states(self.handle) != 0:
            raise RuntimeError("gz_runner_clear_unique_states: %s" % self.lib.gz_runner_last_error().decode())

    def update_network(self, blob=None, device_ptr=None, count=None, clear_unique_states=True, timeout_s=120.0):
        """Generation roll on the live runner (worker.py:138-160: update_nn + clear_unique_states):
        the launcher swaps in the new weights between two launches, so every pool batch runs on one
        network.  blob: host float32 weight blob, or device_ptr + count (e.g. after an RCCL
        broadcast).  Returns {"pool_batches": [batches of each pool launched on the previous
        network], "launches_before": launches issued before the swap}."""
        if blob is not None:
            blob = np.ascontiguousarray(blob, dtype=np.float32)
            ptr, n, dev = blob.ctypes.data, blob.size, 0
        else:
            ptr, n, dev = device_ptr, count, 1
        rc = self.lib.gz_runner_update_network(self.handle, ctypes.c_void_p(ptr), n, dev, int(bool(clear_unique_states)),
                                               timeout_s)
        if rc != 0:
            raise RuntimeError("gz_runner_update_network (%d): %s" % (rc, self.lib.gz_runner_last_error().decode()))
        pb = (ctypes.c_long * self.num_pools)()
        lb = ctypes.c_long()
        self.lib.gz_runner_roll_info(self.handle, pb, self.num_pools, ctypes.byref(lb))
        # apply_ms: the launcher's wall time applying it (fold / pack / swap); device_ms: the fold +
        # pack kernels of a device blob
        return {"pool_batches": list(pb), "launches_before": lb.value,
                "apply_ms": self.lib.gz_runner_roll_apply_ms(self.handle),
                "device_ms": self.net.last_roll_ms() if dev else None}

    def wait_batches(self, total, timeout_s=600.0):
        rc = self.lib.gz_runner_wait_batches(self.handle, total, timeout_s)
        if rc != 0:
            raise RuntimeError("runner wait failed (%d): %s" % (rc, self.lib.gz_runner_last_error().decode()))

    def wait_rows(self, total, timeout_s=600.0, progress=None, interval_s=10.0):
        """Block until `total` leaf evaluations completed; progress(stats) is called every
        interval_s seconds while waiting (long runs print a heartbeat)."""
        import time
        t_end = time.time() + timeout_s
        while True:
            left = t_end - time.time()
            rc = self.lib.gz_runner_wait_rows(self.handle, total, max(0.001, min(interval_s, left)))
            if rc == 0:
                return
            if rc != -2 or time.time() >= t_end:
                raise RuntimeError("runner wait failed (%d): %s" % (rc, self.lib.gz_runner_last_error().decode()))
            if progress is not None:
                progress(self.stats())

    def fetch_samples(self):
        """Samples produced since the last call (keep_samples=True), as datadesc.Sample dicts."""
        s = _native.take_string(self.lib.gz_runner_fetch_samples(self.handle))
        return json.loads(s) if s else []

    def stats(self):
        st = _native.GzRunnerStats()
        self.lib.gz_runner_stats_get(self.handle, ctypes.byref(st))
        return st.as_dict()

    def ordinal_stats(self):
        """Per-game costs by the game's ordinal within its slot (gz_ordinal_stats)."""
        st = _native.GzOrdinalStats()
        if self.lib.gz_runner_ordinal_stats(self.handle, ctypes.byref(st)) != 0:
            raise RuntimeError("gz_runner_ordinal_stats: %s" % self.lib.gz_runner_last_error().decode())
        return st.as_dict()

    @staticmethod
    def set_verify_fastpath(on):
        """Re-check every engine fast-path decision against the literal reference path from now on
        (process-wide, GZ_VERIFY_FASTPATH at run time; a mismatch aborts the process).  Returns
        the previous setting."""
        return _native.set_verify_fastpath(on)

    def stop(self):
        if self.handle:
            rc = self.lib.gz_runner_stop(self.handle)
            if rc != 0:
                raise RuntimeError("runner failed: %s" % self.lib.gz_runner_last_error().decode())

    def close(self):
        if self.handle:
            self.lib.gz_runner_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GamePool(object):
    """One game pool (the reference's SelfPlayManager, selfplaymanager.cpp:22-159) over caller-owned
    numpy buffers, polled from Python: the unit the native runner schedules, exposed for tests and
    for CPU-side drivers.  poll(pred_count) consumes the predictions written into `policies` /
    `values` for the previous batch and returns the number of rows of planes now in `planes`."""

    def __init__(self, sm, transformer, conf, batch_size, identifier="pool", seed=0, game_index_base=0):
        import numpy as np
        self.lib = _native.engine_lib()
        self.c_transformer = cppinterface.create_c_transformer(transformer)
        t = transformer
        self.planes = np.zeros((batch_size, t.num_channels, t.num_cols, t.num_rows), dtype=np.float32)
        self.policies = [np.zeros((batch_size, p), dtype=np.float32) for p in t.policy_dist_count]
        self.values = np.zeros((batch_size, t.num_rewards), dtype=np.float32)
        fp = ctypes.POINTER(ctypes.c_float)
        self._pol_ptrs = (fp * len(self.policies))(*[p.ctypes.data_as(fp) for p in self.policies])
        self.handle = self.lib.gz_pool_create(sm.handle, self.c_transformer.handle, batch_size,
                                              identifier.encode(), seed, game_index_base, None,
                                              self.planes.ctypes.data_as(fp), self._pol_ptrs,
                                              self.values.ctypes.data_as(fp))
        if not self.handle:
            raise RuntimeError("gz_pool_create: %s" % _native.engine_error())
        self._conf = _native.make_selfplay_config(conf)
        if self.lib.gz_pool_start(self.handle, ctypes.byref(self._conf)) < 0:
            raise RuntimeError("gz_pool_start: %s" % _native.engine_error())

    def poll(self, pred_count):
        n = self.lib.gz_pool_poll(self.handle, pred_count)
        if n < 0:
            raise RuntimeError("gz_pool_poll: %s" % _native.engine_error())
        return n

    def cancel(self):
        """Teardown from any thread (gz_pool_cancel): a poll in progress returns 0 rows at the pool's
        next coroutine switch, and so does every later poll."""
        if self.lib.gz_pool_cancel(self.handle) != 0:
            raise RuntimeError("gz_pool_cancel: %s" % _native.engine_error())

    def fetch_samples(self):
        s = _native.take_string(self.lib.gz_pool_fetch_samples(self.handle))
        return json.loads(s) if s else []

    def ordinal_stats(self):
        """Per-game costs by the game's ordinal within its slot (gz_ordinal_stats)."""
        st = _native.GzOrdinalStats()
        if self.lib.gz_pool_add_ordinal_stats(self.handle, ctypes.byref(st)) != 0:
            raise RuntimeError("gz_pool_add_ordinal_stats: %s" % _native.engine_error())
        return st.as_dict()

    def stats(self):
        st = _native.GzPoolStats()
        self.lib.gz_pool_get_stats(self.handle, ctypes.byref(st))
        return st.as_dict()

    def close(self):
        if self.handle:
            self.lib.gz_pool_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
