# Historical: the sync_lag option this A/B drives was measured (profiles/r04_sync_lag_ab.log) and
# removed from the library; DESIGN.md §5 (round 4) has the numbers.
# Host-sync variants of the pass loop: the previous library (abl/base.so:
# drained syncs with a done-flag copy per sync) against this tree drained
# (sync_lag 0) and lagged (sync_lag 1), both with the mapped done flags.
#   bash tools/sync_ab.sh [tag]   (on the GPU box)
set -e
T=${1:-sy}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for cfg in "30 {}" "8 {}" '30 {"exact_nn":0}'; do
    st=${cfg%% *}; o=${cfg#* }
    for v in base lag0 lag1; do
      if [ $v = base ]; then export ORPCD_HIP_LIB=abl/base.so; oo="$o"; else unset ORPCD_HIP_LIB
        oo=$(python3 -c "import json,sys; d=json.loads(sys.argv[1]); d['sync_lag']=int(sys.argv[2]); print(json.dumps(d))" "$o" ${v#lag}); fi
      echo "== $v starts=$st opts=$o" >> gpurun_out/$T/ab.log
      timeout -k 10 120 python3 tools/one_batch.py "$oo" --reps 5 --starts $st >> gpurun_out/$T/ab.log 2>&1
    done
  done
done
unset ORPCD_HIP_LIB
