# Round 5, GPU session 1: counter list, GPU tests, search block-size A/B, wave timelines.
set -e
O=gpurun_out/r5s1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step counters
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
step tests
set +e
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
# assertion failures (rc 1) do not stop the session; a fault, abort or time limit does
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step ab
for rep in 1 2 3; do
  for L in head abl/sw1.so abl/sw2.so; do
    for ST in 30 64; do
      if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
      echo "== $L starts=$ST" >> $O/ab.log
      timeout -k 10 120 python3 tools/one_batch.py '{}' --reps 5 --starts $ST >> $O/ab.log 2>&1
    done
  done
done
unset ORPCD_HIP_LIB
step wavetime
for v in wt wt1; do
  ORPCD_HIP_LIB=abl/$v.so ORPCD_WAVETIME=/tmp/$v.bin timeout -k 10 120 python3 tools/one_batch.py '{}' --reps 1 --starts 30 > $O/$v.run.log 2>&1
  python3 tools/wavetime.py /tmp/$v.bin --every 5 > $O/$v.txt 2>&1
  rm -f /tmp/$v.bin
done
python3 tools/ab_summary.py $O/ab.log > $O/ab_summary.txt 2>&1
step fgr_align
timeout -k 10 300 python3 tools/bench_fgr_align.py --out $O/fgr_align.json > $O/fgr_align.log 2>&1
step done
