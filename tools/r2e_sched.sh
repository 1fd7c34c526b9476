# ordered dispatch: GPU tests, A/B against uniform splits (hashes must match), C4 projection, bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for st in 1 8 30 104; do
  for cfg in '{"sched":0}' '{"sched":1}' '{"sched":1,"sched_items":5120}' '{"sched":1,"sched_items":20480}'; do
    echo "== starts $st cfg $cfg" >> $O/ab.log
    timeout -k 10 60 python tools/one_batch.py "$cfg" --starts $st --reps 4 2>/dev/null | grep -v WARN >> $O/ab.log
  done
done
timeout -k 10 300 python3 tools/bench_c4_align.py --out $O/c4.json > $O/c4.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
