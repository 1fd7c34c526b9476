# exact_nn: GPU tests (new file first), then timing A/B on C2 batches
set -e
export TMPDIR=/tmp
O=gpurun_out/r2l
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 200 --timeout-method thread > $O/exact_tests.log 2>&1 || { echo "exact tests failed"; tail -40 $O/exact_tests.log; exit 1; }
for st in 1 8 30 64; do
  for cfg in '{"exact_nn":0}' '{"exact_nn":1}'; do
    echo "== starts $st cfg $cfg" >> $O/ab.log
    timeout -k 10 90 python tools/one_batch.py "$cfg" --starts $st --reps 5 2>/dev/null | grep -v WARN >> $O/ab.log
  done
done
