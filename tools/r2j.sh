# fused solve + transform: GPU tests, A/B (hashes must match), bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r2j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for st in 1 8 30 104; do
  for cfg in '{"fuse_solve":0}' '{"fuse_solve":1}'; do
    echo "== starts $st cfg $cfg" >> $O/ab.log
    timeout -k 10 60 python tools/one_batch.py "$cfg" --starts $st --reps 4 2>/dev/null | grep -v WARN >> $O/ab.log
  done
done
timeout -k 10 400 python3 bench.py --cpu-seconds 0 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python3 tools/bench_c4_align.py --out $O/c4.json > $O/c4.log 2>&1
