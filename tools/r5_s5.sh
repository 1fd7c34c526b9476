# Round 5, GPU session 5: device tuple-test parity, sched_cap_us sweep (results must keep the default's hash).
set -e
O=gpurun_out/r5s5; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fgr.py -m gpu -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step sweep
for rep in 1 2; do
  for opt in '{}' '{"sched_cap_us": 15}' '{"sched_cap_us": 20}' '{"sched_cap_us": 30}' '{"sched_cap_us": 20, "sched_cap_mult": 2}' '{"sched_cap_us": 30, "sched_cap_mult": 2}'; do
    for ST in 30 64; do
      echo "== cap$opt starts=$ST" >> $O/sweep.log
      timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
    done
  done
done
step done
