"""N>1 path on CPU: the multistart sharded over a world_size-2 gloo group must
reproduce the single-process result (and the reference's golden trace G3)."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, speculative=False, interleave=False):
    sys.path[:0] = [PKG, os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from orpcd_amd import Aligner, Preprocessor
    from scripted import ScriptedOptimizer
    from test_host import BatchedScripted, SpeculativeScripted
    g = np.load(f"{GOLDEN}/g3_aligner_trace.npz")
    np.random.seed(7)
    inner = ScriptedOptimizer(g["goal"], mode="scripted")
    opt = (SpeculativeScripted if speculative else BatchedScripted)(inner)
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=4, shard_interleave=interleave)
    T, m, sf, err = al.align(g["src"].copy(), g["tgt"].copy(), refine_registration=False)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), T=T, m=m, sf=sf, err=np.asarray(err),
             batches=np.asarray(opt.batches), rng=np.random.uniform(size=4))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_multistart_matches_reference_trace(tmp_path, world):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    g = np.load(f"{GOLDEN}/g3_aligner_trace.npz")
    shards = []
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["T"], g["scripted_T"]) and z["m"] == g["scripted_metric"]
        assert np.array_equal(z["sf"], g["scripted_sf"]) and np.array_equal(z["err"], g["scripted_errors"])
        assert np.array_equal(z["rng"], g["scripted_rng_after"])  # every rank replays the full RNG stream
        shards.append(z["batches"])
    # attempts (4 per multistart) were split over the ranks, each multistart
    per_ms = np.sum(np.stack(shards), axis=0)
    assert np.all(per_ms == 4) and all(np.all(s < 4) for s in shards)


@pytest.mark.parametrize("world,interleave", [(2, False), (3, False), (5, False), (3, True)])
def test_sharded_speculative_compass_matches_reference_trace(tmp_path, world, interleave):
    """The speculative compass over ranks: each device batch's multistarts
    (the initial one, compass iterations' 6 x 4 starts) are sharded as one
    flat list -- target-major (a rank's block spans one or two candidates) or
    interleaved (every rank an equal slice of every candidate) -- with one
    all-gather per batch; every rank reproduces the reference's align() (G3)
    and its RNG position."""
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), True, interleave), nprocs=world,
                       join=True, start_method="spawn")
    g = np.load(f"{GOLDEN}/g3_aligner_trace.npz")
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["T"], g["scripted_T"]) and z["m"] == g["scripted_metric"]
        assert np.array_equal(z["sf"], g["scripted_sf"]) and np.array_equal(z["err"], g["scripted_errors"])
        assert np.array_equal(z["rng"], g["scripted_rng_after"])


def test_record_pack_roundtrip():
    from orpcd_amd import parallel
    rng = np.random.default_rng(0)
    r = dict(rmse=rng.random(5), fitness=rng.random(5), iters=np.arange(5), ncorr=np.arange(5) * 7,
             T=rng.random((5, 4, 4)))
    u = parallel.unpack(parallel.pack(r))
    for k in r:
        assert np.array_equal(np.asarray(u[k]), np.asarray(r[k]))


def _rows_worker(rank, world, port, out_dir, device_collectives=False):
    sys.path[:0] = [PKG, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from orpcd_amd import parallel
    from shard_fake import FakeShardContext
    from workloads import small_pair
    src, tgt = small_pair(1501, 1400, seed=4)
    ctx = FakeShardContext()
    r = parallel.gicp_rows_sharded(ctx, src, tgt, max_correspondence_distance=0.3,
                                   device_collectives=device_collectives)
    comm = np.frombuffer(ctx.comm[2], np.uint8) if device_collectives else np.zeros(0, np.uint8)
    np.savez(os.path.join(out_dir, f"rows{rank}.npz"), T=r["T"], rmse=r["rmse"], fitness=r["fitness"],
             iters=r["iters"], ncorr=r["ncorr"], comm=comm,
             comm_ranks=ctx.comm[0] if device_collectives else 0, comm_rank=ctx.comm[1] if device_collectives else -1)
    dist.destroy_process_group()


def _rows_too_few_worker(rank, world, port, out_dir):
    sys.path[:0] = [PKG, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from orpcd_amd import parallel
    from shard_fake import FakeShardContext
    from workloads import small_pair
    src, tgt = small_pair(300, 300, seed=4)
    try:
        parallel.gicp_rows_sharded(FakeShardContext(), src[: world - 1], tgt)
        outcome = "returned"
    except ValueError:
        outcome = "ValueError"
    dist.barrier()  # every rank got here: nobody is stuck in a collective
    with open(os.path.join(out_dir, f"few{rank}.txt"), "w") as f:
        f.write(outcome)
    dist.destroy_process_group()


def test_row_sharded_fewer_rows_than_ranks_raises_everywhere(tmp_path):
    """n < world_size: every rank raises ValueError before any collective
    (no rank is left waiting in the per-pass all_reduce)."""
    import torch.multiprocessing as mp
    world = 3
    mp.start_processes(_rows_too_few_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert (tmp_path / f"few{r}.txt").read_text() == "ValueError"


@pytest.mark.parametrize("world,device_collectives", [(2, False), (3, False), (2, True), (3, True)])
def test_row_sharded_gicp_matches_single_process_oracle(tmp_path, world, device_collectives, oracle):
    """C5's multi-GPU path: source rows split over ranks, one all-reduce of
    the 29 normal-equation sums per pass; every rank ends with the result of
    one un-sharded GICP (up to the summation order of the sums).  With
    device_collectives the pass loop is the context's own (orpcd_gicp_shard_run)
    and every rank joins rank 0's communicator id."""
    import torch.multiprocessing as mp
    mp.start_processes(_rows_worker, args=(world, _free_port(), str(tmp_path), device_collectives), nprocs=world,
                       join=True, start_method="spawn")
    if device_collectives:
        ids = [np.load(tmp_path / f"rows{r}.npz")["comm"] for r in range(world)]
        assert all(len(i) == 128 and np.array_equal(i, ids[0]) for i in ids)
        assert [int(np.load(tmp_path / f"rows{r}.npz")["comm_rank"]) for r in range(world)] == list(range(world))
    from workloads import small_pair
    src, tgt = small_pair(1501, 1400, seed=4)
    ref = oracle.gicp(src, tgt, 0.3)
    for r in range(world):
        z = np.load(tmp_path / f"rows{r}.npz")
        assert int(z["iters"]) == ref["iters"] and int(z["ncorr"]) == ref["ncorr"]
        assert np.allclose(z["T"], ref["T"], atol=1e-9, rtol=0)
        assert abs(float(z["rmse"]) - ref["rmse"]) <= 1e-10
