"""A CPU stand-in for the device context's row-sharded GICP calls
(set_target / set_source_rows / shard_begin / shard_pass / shard_update /
shard_result), built from the oracle's pieces, so that the multi-rank driver
orpcd_amd.parallel.gicp_rows_sharded can be tested with gloo on CPU.  Test
infrastructure only (it calls the oracle)."""
import os

import numpy as np

import oracle


class FakeShardContext:
    def set_target(self, target, epsilon):
        self.tgt = np.ascontiguousarray(target, dtype=np.float64)
        self.tcov = oracle.estimate_normals(self.tgt, 20, -1.0, epsilon)[2]

    # the target's covariance pass by rows (orpcd_set_target_rows), with the
    # library's slicing: blocks of target_slice(m, n) rows (a multiple of the
    # 64-row tile), rank r's block at r * slice, the in-place all-gather into
    # a buffer of slice * n rows whose first m rows are the target's.  The
    # fake's rows are input rows (the library's are Morton rows); a rank keeps
    # its slice only until set_target_cov
    TILE = 64

    @classmethod
    def target_slice(cls, m, nranks):
        return -(-(-(-m // nranks)) // cls.TILE) * cls.TILE

    def set_target_rows(self, target, rank, nranks, epsilon):
        self.tgt = np.ascontiguousarray(target, dtype=np.float64)
        m = len(self.tgt)
        sl = self.target_slice(m, nranks)
        lo, hi = min(m, rank * sl), min(m, rank * sl + sl)
        self.tcov = np.full((m, 3, 3), np.nan)
        self.tcov[lo:hi] = oracle.estimate_normals(self.tgt, 20, -1.0, epsilon)[2][lo:hi]
        if getattr(self, "comm", None) and self.comm[0] == nranks:  # the device all-gather, over the group
            from orpcd_amd import parallel
            send = np.full((sl, 9), np.nan)                # this rank's block of the gather buffer
            send[: hi - lo] = self.tcov[lo:hi].reshape(hi - lo, 9)
            blocks = parallel.allgather_arrays(send)
            assert all(b.shape == (sl, 9) for b in blocks)
            gathered = np.concatenate(blocks)              # slice * nranks rows, block r at r * slice
            assert len(gathered) == sl * nranks >= m and not np.isnan(gathered[:m]).any()
            self.set_target_cov(gathered[:m])
        return lo, hi

    def target_cov_rows(self, lo, hi):
        assert not np.isnan(self.tcov[lo:hi]).any()
        return self.tcov[lo:hi].reshape(hi - lo, 9)

    def set_target_cov(self, cov):
        self.tcov = np.asarray(cov).reshape(len(self.tgt), 3, 3)

    def set_source_rows(self, source, lo, hi):
        self.src_full = np.ascontiguousarray(source, dtype=np.float64)
        self.lo, self.hi = lo, hi

    def shard_begin(self, R0, t0, n_total, epsilon=1e-3, max_correspondence_distance=0.5, max_iteration=100,
                    relative_fitness=1e-6, relative_rmse=1e-6):
        assert np.allclose(R0, np.eye(3)) and np.allclose(t0, 0)
        scov = oracle.estimate_normals(self.src_full, 20, -1.0, epsilon)[2]   # full-cloud neighbourhoods
        self.src, self.scov = self.src_full[self.lo:self.hi], scov[self.lo:self.hi]
        self.n_total, self.r = n_total, max_correspondence_distance
        self.max_iter, self.rf, self.rr = max_iteration, relative_fitness, relative_rmse
        self.T, self.prev, self.pass_, self.done = np.eye(4), (0.0, 0.0), 0, False
        self.fit = self.rmse = 0.0
        self.ncorr = 0

    def shard_pass(self):
        if self.done:
            return np.zeros(29), False
        R, t = self.T[:3, :3], self.T[:3, 3]
        p = self.src @ R.T + t
        c = np.einsum("ij,njk,lk->nil", R, self.scov, R)
        idx, d2 = oracle.nn1_radius(p, self.tgt, self.r)
        JTJ, JTr, _ = oracle.gicp_step(p, c, self.tgt, self.tcov, idx)
        iu = np.triu_indices(6)
        return np.concatenate([JTJ[iu], JTr, [d2[idx >= 0].sum(), float((idx >= 0).sum())]]), True

    def shard_update(self, sums):
        cnt = sums[28]
        fit = cnt / self.n_total if cnt > 0 else 0.0
        rmse = np.sqrt(sums[27] / cnt) if cnt > 0 else 0.0
        conv = self.pass_ >= 1 and abs(self.prev[0] - fit) < self.rf and abs(self.prev[1] - rmse) < self.rr
        if conv or self.pass_ >= self.max_iter:
            self.done, self.fit, self.rmse, self.ncorr = True, fit, rmse, int(cnt)
            return True
        self.prev = (fit, rmse)
        JTJ = np.zeros((6, 6))
        JTJ[np.triu_indices(6)] = sums[:21]
        JTJ = JTJ + np.triu(JTJ, 1).T
        ok, x, _ = oracle.solve_psd6(JTJ, -sums[21:27]) if cnt > 0 else (False, None, 0.0)
        upd = oracle.vec6_to_m4(x) if ok else np.eye(4)
        self.T = upd @ self.T
        self.pass_ += 1
        return False

    def shard_result(self):
        return dict(T=self.T, rmse=self.rmse, fitness=self.fit, iters=self.pass_, ncorr=self.ncorr)

    # device collectives (orpcd_comm_* / orpcd_gicp_shard_run): the same loop,
    # its all-reduce over the process group; the id is recorded to check that
    # every rank joined rank 0's communicator
    def comm_unique_id(self):
        return os.urandom(128)

    def comm_init(self, nranks, rank, uid):
        self.comm = (nranks, rank, bytes(uid))

    def shard_run(self):
        from orpcd_amd import parallel
        n = 0
        while True:
            sums, act = self.shard_pass()
            if not act or self.shard_update(parallel.allreduce_sum(sums)):
                return n
            n += 1

