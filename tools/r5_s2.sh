# Round 5, GPU session 2: feature-NN regression diagnosis, GPU tests, FGR align, C5 call time, C3 (+QT=3), wave timelines.
set -e
O=gpurun_out/r5s2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step diag
for L in abl/c0.so abl/c1.so abl/noclamp.so head; do
  if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
  echo "== $L" >> $O/diag.log
  set +e
  timeout -k 10 120 python3 -u -m pytest tests/test_gpu_fgr.py -q -x --timeout 60 --timeout-method thread -k "feature_nn_matches_brute or near_ties_spread" >> $O/diag.log 2>&1
  rc=$?
  set -e
  echo "rc=$rc" >> $O/diag.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
unset ORPCD_HIP_LIB
step tests
set +e
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step fgr_align
timeout -k 10 400 python3 tools/bench_fgr_align.py --out $O/fgr_align.json > $O/fgr_align.log 2>&1 || echo "fgr_align rc=$?" >> $O/steps.log
step c5
timeout -k 10 400 python3 tools/bench_c5.py --out $O/c5.json > $O/c5.log 2>&1
step c5_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5kt -- python3 tools/bench_c5.py --cpu-iters 0 --parity 0 > $O/c5kt.log 2>&1
step fgr_c3
timeout -k 10 300 python3 tools/bench_fgr.py --out $O/fgr_c3.json > $O/fgr_c3.log 2>&1
ORPCD_HIP_LIB=abl/qt3.so timeout -k 10 300 python3 tools/bench_fgr.py --cpu 0 --out $O/fgr_c3_qt3.json > $O/fgr_c3_qt3.log 2>&1
timeout -k 10 300 python3 tools/bench_fgr.py --cpu 0 --out $O/fgr_c3_b.json > $O/fgr_c3_b.log 2>&1
step wavetime
ORPCD_HIP_LIB=abl/wt.so ORPCD_WAVETIME=/tmp/wt.bin timeout -k 10 120 python3 tools/one_batch.py '{}' --reps 1 --starts 30 > $O/wt.run.log 2>&1
python3 tools/wavetime.py /tmp/wt.bin --every 5 > $O/wt.txt 2>&1
rm -f /tmp/wt.bin
step done
