# ordered dispatch v2 (planner block beside the transform): tests, A/B, C5 both ways
set -e
export TMPDIR=/tmp
O=gpurun_out/r2g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for st in 1 8 30 104; do
  for cfg in '{"sched":0}' '{"sched":1}' '{"sched":1,"sched_items":5120}'; do
    echo "== starts $st cfg $cfg" >> $O/ab.log
    timeout -k 10 60 python tools/one_batch.py "$cfg" --starts $st --reps 4 2>/dev/null | grep -v WARN >> $O/ab.log
  done
done
timeout -k 10 300 python3 tools/bench_c5.py --parity 0 --cpu-iters 1 --opt '{"sched":0}' --out $O/c5_0.json > $O/c5_0.log 2>&1
timeout -k 10 300 python3 tools/bench_c5.py --parity 0 --cpu-iters 1 --opt '{"sched":1}' --out $O/c5_1.json > $O/c5_1.log 2>&1
