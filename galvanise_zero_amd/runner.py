"""Native multi-threaded self-play on one GPU (include/gzero_nn.h gz_runner_*): the steady-state
replacement of the reference's per-batch Python poll loop (cppinterface.py:131-144 driven by
distributed/worker.py:191).  Pools, coroutines, planes and NN launches are all native."""
import ctypes

from . import _native, cppinterface


class SelfPlayRunner(object):
    def __init__(self, hip_net, sm, transformer, conf, device=0, num_threads=8, pools_per_thread=2,
                 batch_size=256, seed=0, game_index_base=0):
        self.lib = _native.runner_lib()
        _native.engine_lib()
        self.net = hip_net
        self.sm = sm
        self.c_transformer = cppinterface.create_c_transformer(transformer)
        self.cfg = _native.GzRunnerConfig(device, num_threads, pools_per_thread, batch_size, seed,
                                          game_index_base, 1)
        self.conf = _native.make_selfplay_config(conf)
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
        self.lib.gz_runner_start(self.handle)

    def wait_batches(self, total, timeout_s=600.0):
        rc = self.lib.gz_runner_wait_batches(self.handle, total, timeout_s)
        if rc != 0:
            raise RuntimeError("runner wait failed (%d): %s" % (rc, self.lib.gz_runner_last_error().decode()))

    def stats(self):
        st = _native.GzRunnerStats()
        self.lib.gz_runner_stats_get(self.handle, ctypes.byref(st))
        return st.as_dict()

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
