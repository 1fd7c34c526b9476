# Round-4 GPU session: scan microbenchmark, drop-in pass anatomy, C5 row
# projection, the normal-form covariance A/B, and the exact-parity tests.
set -e
mkdir -p gpurun_out/s1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/scan_bench > gpurun_out/s1/scan_bench.json 2> gpurun_out/s1/scan_bench.err
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_gicp.py tests/test_gpu_align.py tests/test_gpu_ties.py tests/test_gpu_shard.py > gpurun_out/s1/tests.log 2>&1
for rep in 1 2; do
  for L in abl/cov6.so head; do
    if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
    for ST in 30 8; do
      echo "== $L starts=$ST" >> gpurun_out/s1/cov_ab.log
      timeout -k 10 120 python3 tools/one_batch.py '{}' --reps 5 --starts $ST >> gpurun_out/s1/cov_ab.log 2>&1
    done
  done
done
unset ORPCD_HIP_LIB
ORPCD_GAPS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 3 --legs batched,dropin > gpurun_out/s1/gaps.log 2>&1
timeout -k 10 400 python3 tools/bench_c5_rows.py --out gpurun_out/s1/c5_rows.json > gpurun_out/s1/c5_rows.log 2>&1
