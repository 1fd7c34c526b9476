# Round 5, GPU session 13: persistent ordered dispatch with a static snake order (no atomics) A/B.
set -e
O=gpurun_out/r5s13; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step sweep
for rep in 1 2; do
  for cfg in 'head|{}' 'abl/pst.so|{"sched_persist": 1}' 'abl/pst.so|{"sched_persist": 1, "persist_waves": 10240}' 'abl/pst.so|{"sched_persist": 1, "persist_waves": 20480}' 'abl/pst4.so|{"sched_persist": 1, "persist_waves": 4096}'; do
    lib=${cfg%%|*}; opt=${cfg#*|}
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
step done
