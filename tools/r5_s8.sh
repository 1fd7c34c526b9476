# Round 5, GPU session 8: full GPU suite after the exact re-search bounds fix, split-cap A/B, bench.
set -e
O=gpurun_out/r5s8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
step sweep
for rep in 1 2 3; do
  for opt in '{}' '{"sched_cap_us": 30, "sched_cap_mult": 2}'; do
    for ST in 30 64; do
      echo "== cap$opt starts=$ST" >> $O/sweep.log
      timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
    done
  done
done
step bench
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
step done
