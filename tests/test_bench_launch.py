"""bench.py's multi-rank launch on CPU (gloo): `bench.py --gpus N` with no
WORLD_SIZE starts the N rank processes itself and reports n_gpus = N with
attempts x N starts per step; a --gpus / WORLD_SIZE mismatch fails loudly.
The optimizer is tests/bench_fake.py (deterministic per start), so the
sharded multistart must equal the one-rank run."""
import json
import os
import subprocess
import sys

from conftest import REPO

FAKE = os.path.join(REPO, "tests", "bench_fake.py") + ":FakeGICP"


def _run(args, tmp_path, extra_env=None, timeout=240):
    env = dict(os.environ, ORPCD_BENCH_OPTIMIZER=FAKE, ORPCD_BENCH_BACKEND="gloo",
               ORPCD_FAKE_LOG=str(tmp_path / "calls.jsonl"), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=str(tmp_path),
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


COMMON = ["--steps", "2", "--warmup", "1", "--points", "2000", "--attempts", "30", "--cpu-seconds", "0",
          "--align", "0", "--c4-attempts", "8"]


def test_bench_gpus2_spawns_two_ranks(tmp_path):
    r = _run(["--gpus", "2"] + COMMON, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["devices"] == [0, 1]
    assert line["config"]["attempts_per_step"] == 60 and line["config"]["attempts_per_gpu"] == 30
    assert line["c4"]["n_gpus"] == 2 and line["c4"]["seconds"] > 0
    calls = [json.loads(x) for x in (tmp_path / "calls.jsonl").read_text().splitlines()]
    # every multistart step: 30 starts on each of the two ranks (warm-up + timed + replay = 5 steps)
    step_calls = [c for c in calls if c["starts"] == 30]
    assert {c["rank"] for c in step_calls} == {0, 1}
    assert sum(1 for c in step_calls if c["rank"] == 0) == sum(1 for c in step_calls if c["rank"] == 1) == 5
    # one rank's GICP iterations per step x 2 ranks = the line's
    one = _run(["--gpus", "1"] + COMMON, tmp_path)
    assert one.returncode == 0, one.stderr[-3000:]
    l1 = _line(one.stdout)
    assert l1["n_gpus"] == 1 and l1["config"]["attempts_per_step"] == 30
    # C4 is strong scaling: the same align() at N=1 and N=2 (deterministic optimizer)
    assert line["c4"]["gicp_iterations"] == l1["c4"]["gicp_iterations"]
    assert line["c4"]["scale_factors"] == l1["c4"]["scale_factors"] and line["c4"]["rmse"] == l1["c4"]["rmse"]


def test_bench_gpus_world_size_mismatch_fails(tmp_path):
    r = _run(["--gpus", "3"] + COMMON, tmp_path,
             extra_env=dict(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1"),
             timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_failed_rank_fails_the_launch(tmp_path):
    """A rank that dies makes the launcher exit non-zero (the others are stopped)."""
    r = _run(["--gpus", "2"] + COMMON, tmp_path, extra_env=dict(ORPCD_BENCH_OPTIMIZER="/nonexistent.py:X"),
             timeout=120)
    assert r.returncode != 0


def test_bench_under_torch_distributed_run(tmp_path):
    """The driver's own multi-GPU form: `python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P
    bench.py --gpus 2 ...` (WORLD_SIZE set by the launcher, so bench.py starts
    no processes itself): one JSON line, from rank 0, with n_gpus 2."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, ORPCD_BENCH_OPTIMIZER=FAKE, ORPCD_BENCH_BACKEND="gloo",
               ORPCD_FAKE_LOG=str(tmp_path / "calls.jsonl"), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
                        "--gpus", "2"] + COMMON, env=env, cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["devices"] == [0, 1]
    assert line["config"]["attempts_per_step"] == 60 and line["c4"]["n_gpus"] == 2
