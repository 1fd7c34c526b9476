# Round 5, GPU session 11: split-count limit (64 / 128 / 255) x split cap A/B, wave timeline of the head.
set -e
O=gpurun_out/r5s11; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step sweep
for rep in 1 2; do
  for lib in head abl/smax128.so abl/smax255.so; do
    for opt in '{}' '{"sched_cap_us": 20}' '{"sched_cap_us": 15, "sched_cap_mult": 3}'; do
      for ST in 30 64; do
        echo "== $lib $opt starts=$ST" >> $O/sweep.log
        if [ $lib = head ]; then
          timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
        else
          ORPCD_HIP_LIB=$lib timeout -k 10 120 python3 tools/one_batch.py "$opt" --reps 5 --starts $ST >> $O/sweep.log 2>&1
        fi
      done
    done
  done
done
step wavetime
ORPCD_HIP_LIB=abl/wt.so ORPCD_WAVETIME=/tmp/wt.bin timeout -k 10 120 python3 tools/one_batch.py '{}' --reps 1 --starts 30 > $O/wt.run.log 2>&1
python3 tools/wavetime.py /tmp/wt.bin --every 5 --dump $O/wt_dump.npz > $O/wt.txt 2>&1
rm -f /tmp/wt.bin
step done
