"""A CPU stand-in for GeneralizedICP used ONLY by tests/test_bench_launch.py to
rehearse bench.py's multi-rank launch (ORPCD_BENCH_OPTIMIZER) without a GPU.

Its results are a cheap deterministic function of each start (R0, t0) and of
the target's scale, so every rank computes the same value for the same start
and the sharded multistart must reproduce the one-process table.  It records
how many starts each call ran, so the test can check the split.
"""
import json
import os

import numpy as np


class _FakeContext:
    def __init__(self):
        self.reset_stats()

    def reset_stats(self):
        self._st = dict(ms=0.0, launches=0, pairs=0, tiles=0, passes=0, sched_launches=0)

    def set_option(self, name, value):
        pass

    def profiling(self, on):
        pass

    def stats(self):
        return dict(self._st)

    def note(self, starts, iters):
        self._st["launches"] += int(iters.max()) if len(iters) else 0
        self._st["sched_launches"] += int(iters.max()) if len(iters) else 0
        self._st["passes"] += int(iters.sum())
        self._st["pairs"] += int(iters.sum()) * 100
        self._st["ms"] += 0.01 * len(iters)


class FakeGICP:
    zero_rmse_message = "Optimization failed with loss = 0."

    def __init__(self, device=0):
        self.device = device
        self.context = _FakeContext()
        self._exact_nn = True
        self.log = os.environ.get("ORPCD_FAKE_LOG")

    def _one(self, target, R0, t0):
        scale = float(np.abs(target).mean())
        rmse = 0.01 + 0.001 * abs(np.trace(R0) - 1.5) + 0.002 * abs(scale - 0.4) + 1e-4 * float(np.abs(t0).sum())
        iters = 5 + int(abs(np.trace(R0)) * 1000) % 9
        return rmse, iters

    def optimize_batch(self, source, target, R0, t0):
        n = len(R0)
        rm = np.empty(n)
        it = np.empty(n, np.int64)
        for i in range(n):
            rm[i], it[i] = self._one(target, R0[i], t0[i])
        T = np.tile(np.eye(4), (n, 1, 1))
        self.context.note(n, it)
        if self.log:
            with open(self.log, "a") as f:
                f.write(json.dumps({"rank": int(os.environ.get("RANK", "0")), "device": self.device,
                                    "starts": n}) + "\n")
        return dict(T=T, rmse=rm, fitness=np.ones(n), iters=it, ncorr=np.full(n, len(source), np.int64))

    def optimize_batch_multi(self, source, targets, R0s, t0s):
        return [self.optimize_batch(source, g, r, t) for g, r, t in zip(targets, R0s, t0s)]

    def optimize(self, source, target):
        rmse, _ = self._one(target, np.eye(3), np.zeros(3))
        return np.eye(4), rmse
