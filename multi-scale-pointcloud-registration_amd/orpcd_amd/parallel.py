"""Sharding across ranks (one process per GPU).

1. Multistart sharding.  The attempts of one ``multistart_registration``
(Aligner.py:178-202) are independent: every rank replays the identical host RNG stream, runs a
contiguous block of attempts on its own GPU, and one all-gather of a fixed
160-byte record per attempt gives every rank the full table, on which each
applies the reference's strict-< argmin in attempt order.  A speculative
compass iteration (six candidate multistarts) is sharded as one flat,
target-major list of 6 x attempts starts with one all-gather, so a rank's
block spans one or two candidate targets.  No other data-path collective
exists.

2. Row sharding of one start (C5: one GICP over 1M points).  Each rank owns
a contiguous block of source rows (their covariances from the full cloud's
neighbourhoods, computed for its rows only) and the whole target, whose
covariance pass is split by rows too (target_rows_sharded: each rank 1/ws of
the KNN-20 pass, one all-gather); per ICP pass it computes the 29 local
normal-equation sums, one all-reduce(sum) of 232 bytes combines them, and
every rank solves the same 6x6 system (gicp_rows_sharded).  With
``device_collectives=True`` that all-reduce is the library's own RCCL
communicator on its stream (orpcd_comm_init / orpcd_gicp_shard_run): no host
round trip per pass; torch.distributed only hands the 128-byte RCCL id
around.

Backend: ``torch.distributed`` — "nccl" (= RCCL over
xGMI on ROCm) on GPUs, "gloo" for CPU tests.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

REC = 20  # rmse, fitness, iters, ncorr, T(16)


def world() -> Tuple[int, int]:
    import sys
    if "torch.distributed" not in sys.modules:  # no process group can exist: skip importing torch (~1 s)
        return 0, 1
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(B: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of attempts for `rank` (sizes differ by <= 1)."""
    base, rem = divmod(B, world_size)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def pack(r: dict) -> np.ndarray:
    b = len(r["rmse"])
    out = np.zeros((b, REC))
    out[:, 0] = r["rmse"]
    out[:, 1] = r["fitness"]
    out[:, 2] = r["iters"]
    out[:, 3] = r["ncorr"]
    out[:, 4:] = np.asarray(r["T"]).reshape(b, 16)
    return out


def unpack(rec: np.ndarray) -> dict:
    return dict(rmse=rec[:, 0].copy(), fitness=rec[:, 1].copy(), iters=rec[:, 2].astype(np.int64),
                ncorr=rec[:, 3].astype(np.int64), T=rec[:, 4:].reshape(-1, 4, 4).copy())


def allgather_records(local: np.ndarray, B: int) -> np.ndarray:
    """All-gather per-attempt records; returns the (B, REC) table in attempt order."""
    rank, ws = world()
    if ws == 1:
        return local
    import torch
    import torch.distributed as dist

    width = -(-B // ws)  # max block size
    buf = np.zeros((width, REC))
    buf[: len(local)] = local
    if dist.get_backend() == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    t = torch.from_numpy(buf).to(dev)
    outs = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(outs, t)
    allr = torch.stack(outs).cpu().numpy()  # one device-to-host copy for every rank's block
    table = np.zeros((B, REC))
    for r in range(ws):
        lo, hi = shard(B, r, ws)
        table[lo:hi] = allr[r, : hi - lo]
    return table


def allreduce_sum(v: np.ndarray) -> np.ndarray:
    """Sum a small float64 vector over ranks (identity on one rank)."""
    rank, ws = world()
    if ws == 1:
        return v
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def broadcast_bytes(data: bytes, src: int = 0) -> bytes:
    """`data` of rank `src` on every rank of the default group (identity on one rank)."""
    rank, ws = world()
    if ws == 1:
        return data
    import torch.distributed as dist
    obj = [data if rank == src else None]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


def device_comm(ctx):
    """Join ``ctx`` to an RCCL communicator over the default group's ranks
    (once per context and group size): rank 0 makes the id, the group
    broadcasts it."""
    rank, ws = world()
    key = (rank, ws)
    if getattr(ctx, "_orpcd_comm", None) == key:
        return
    uid = broadcast_bytes(ctx.comm_unique_id() if rank == 0 else b"", 0)
    ctx.comm_init(ws, rank, uid)
    ctx._orpcd_comm = key


def allgather_arrays(a: np.ndarray) -> list:
    """Every rank's array (shapes may differ), in rank order (identity on one rank)."""
    rank, ws = world()
    if ws == 1:
        return [a]
    import torch.distributed as dist
    out = [None] * ws
    dist.all_gather_object(out, np.ascontiguousarray(a))
    return out


def target_rows_sharded(ctx, target: np.ndarray, epsilon: float = 1e-3, device_collectives: bool = False):
    """Set ``target`` on every rank's ``ctx`` with its KNN-20 covariance pass
    split by rows (orpcd_set_target_rows): each rank computes 1/ws of the rows;
    one all-gather completes them -- on the device through the context's RCCL
    communicator with ``device_collectives``, else through torch.distributed
    on the host (orpcd_target_cov_rows / orpcd_set_target_cov).  The result is
    the target orpcd_set_target makes, bit for bit."""
    rank, ws = world()
    if ws == 1:
        ctx.set_target(target, epsilon)
        return
    if device_collectives:
        device_comm(ctx)
        ctx.set_target_rows(target, rank, ws, epsilon)
        return
    lo, hi = ctx.set_target_rows(target, rank, ws, epsilon)
    ctx.set_target_cov(np.concatenate(allgather_arrays(ctx.target_cov_rows(lo, hi))))


def gicp_rows_sharded(ctx, source: np.ndarray, target: np.ndarray, R0=None, t0=None, epsilon: float = 1e-3,
                      device_collectives: bool = False, **params) -> dict:
    """One GICP (pose ``source @ R0 + t0``) with the source rows split over the
    ranks of the default process group.  ``ctx`` is this rank's device
    context (``_native.Context`` or any object with the same shard_* calls).
    ``device_collectives``: the per-pass all-reduce runs on the device through
    the library's RCCL communicator (device_comm); else on the host through
    torch.distributed.  Returns the Open3D-convention result (T column
    convention)."""
    rank, ws = world()
    n = len(source)
    if n < ws:
        # every rank sees the same n and ws, so every rank raises here, before
        # any collective (a rank with an empty shard would otherwise leave the
        # others blocked in the per-pass all_reduce)
        raise ValueError(f"gicp_rows_sharded: {n} source rows cannot be split over {ws} ranks")
    lo, hi = shard(n, rank, ws)
    R0 = np.eye(3) if R0 is None else R0
    t0 = np.zeros(3) if t0 is None else t0
    target_rows_sharded(ctx, target, epsilon, device_collectives)
    ctx.set_source_rows(source, lo, hi)
    ctx.shard_begin(R0, t0, n_total=n, epsilon=epsilon, **params)
    if device_collectives:
        device_comm(ctx)
        ctx.shard_run()
        return ctx.shard_result()
    while True:
        sums, active = ctx.shard_pass()
        if not active:
            break
        if ctx.shard_update(allreduce_sum(sums)):
            break
    return ctx.shard_result()
