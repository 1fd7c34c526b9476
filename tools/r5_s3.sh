# Round 5, GPU session 3: GPU tests, FGR align, C5 (+ lane-per-query KNN A/B, kernel trace), C3, sched sweep, bench.
set -e
O=gpurun_out/r5s3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step fgr_align
set +e
timeout -k 10 400 python3 tools/bench_fgr_align.py --out $O/fgr_align.json > $O/fgr_align.log 2>&1
rc=$?
set -e
echo "fgr_align rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step c5
timeout -k 10 400 python3 tools/bench_c5.py --out $O/c5.json > $O/c5.log 2>&1
ORPCD_KNN_TILES=1 timeout -k 10 400 python3 tools/bench_c5.py --cpu-iters 0 --parity 0 --out $O/c5_knntiles.json > $O/c5_knntiles.log 2>&1
step c5_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5kt -- python3 tools/bench_c5.py --cpu-iters 0 --parity 0 > $O/c5kt.log 2>&1
step fgr_c3
timeout -k 10 300 python3 tools/bench_fgr.py --out $O/fgr_c3.json > $O/fgr_c3.log 2>&1
step sweep
for rep in 1 2; do
  for opt in '{}' '{"sched_items": 7680}' '{"sched_items": 15360}' '{"sched_items": 20480}' '{"search_waves": 49152}' '{"search_waves": 24576}'; do
    for ST in 30 64; do
      echo "== head$opt starts=$ST" >> $O/sweep.log
      timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
    done
  done
done
step fgr_trace
set +e
ORPCD_FGR_TRACE=1 timeout -k 10 300 python3 tools/bench_fgr_align.py --cpu-seconds 0 > $O/fgr_trace.log 2>&1
rc=$?
set -e
echo "fgr_trace rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step wavetime
ORPCD_HIP_LIB=abl/wt.so ORPCD_WAVETIME=/tmp/wt.bin timeout -k 10 120 python3 tools/one_batch.py '{}' --reps 1 --starts 30 > $O/wt.run.log 2>&1
python3 tools/wavetime.py /tmp/wt.bin --every 5 --dump $O/wt_dump.npz > $O/wt.txt 2>&1
rm -f /tmp/wt.bin
step bench
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
step done
