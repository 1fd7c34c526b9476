# Round 5, GPU session 6: lane-per-query KNN parity, split-cap default A/B, C5 call time, bench.
set -e
O=gpurun_out/r5s6; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step sweep
for rep in 1 2; do
  for opt in '{}' '{"sched_cap_us": 0}'; do
    for ST in 30 64; do
      echo "== cap$opt starts=$ST" >> $O/sweep.log
      timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
    done
  done
done
step c5
timeout -k 10 400 python3 tools/bench_c5.py --out $O/c5.json > $O/c5.log 2>&1
step bench
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
step done
