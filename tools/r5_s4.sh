# Round 5, GPU session 4: GPU tests (device tuple test), FGR align (+ phase trace), sched_cap_us sweep, bench.
set -e
O=gpurun_out/r5s4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step fgr_align
timeout -k 10 400 python3 tools/bench_fgr_align.py --out $O/fgr_align.json > $O/fgr_align.log 2>&1
step fgr_trace
ORPCD_FGR_TRACE=1 timeout -k 10 300 python3 tools/bench_fgr_align.py --cpu-seconds 0 > $O/fgr_trace.log 2>&1
step sweep
for rep in 1 2; do
  for opt in '{}' '{"sched_cap_us": 20}' '{"sched_cap_us": 30}' '{"sched_cap_us": 45}' '{"sched_cap_us": 60}'; do
    for ST in 30 64; do
      echo "== cap$opt starts=$ST" >> $O/sweep.log
      timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
    done
  done
done
step bench
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
step done
