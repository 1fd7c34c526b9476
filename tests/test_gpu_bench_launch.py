"""GPU: `bench.py --gpus 2` starting its own two rank processes, both on this
box's one GPU (gloo collectives: one GPU cannot hold two RCCL ranks).  The
line must report two ranks, 60 starts per step, and a C4 align() -- its
starts sharded over the two ranks -- identical to the committed complete-oracle
run (tests/golden/g7_align_c4.npz): the multi-rank path of the product, end to
end, with the library on the device."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_bench_two_ranks_on_one_gpu(tmp_path):
    env = dict(os.environ, ORPCD_BENCH_BACKEND="gloo", ORPCD_BENCH_DEVICE="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "ORPCD_BENCH_OPTIMIZER"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--cpu-seconds", "0", "--align", "0"], env=env, cwd=str(tmp_path), capture_output=True,
                       text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["devices"] == [0, 0]
    assert line["config"]["attempts_per_step"] == 60 and line["value"] > 0
    c4 = line["c4"]
    assert c4["n_gpus"] == 2
    p = c4["parity_vs_oracle"]
    assert p["scale_factors_identical"] and p["starts"] == p["starts_oracle"] == p["iterations_identical"]
    assert p["max_abs_d_rmse_per_start"] <= 1e-9 and p["d_rmse"] <= 1e-9
    print(f"two ranks: {line['value']:.0f} GICP iterations/s (one GPU shared), C4 {c4['seconds']} s")
