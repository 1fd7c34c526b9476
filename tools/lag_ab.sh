# Historical: the sync_lag option this A/B drives was measured (profiles/r04_sync_lag_ab.log) and
# removed from the library; DESIGN.md §5 (round 4) has the numbers.
# Lagged host syncs (option sync_lag) against drained ones: C2 exact 30 / 8
# starts and fp32 mode 30 starts, interleaved; result hashes must match.
#   bash tools/lag_ab.sh [tag]   (on the GPU box)
set -e
T=${1:-lag}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for cfg in "30 {}" "8 {}" '30 {"exact_nn":0}'; do
    st=${cfg%% *}; o=${cfg#* }
    for lag in 0 1; do
      oo=$(python3 -c "import json,sys; d=json.loads(sys.argv[1]); d['sync_lag']=$lag; print(json.dumps(d))" "$o")
      echo "== lag$lag starts=$st opts=$o" >> gpurun_out/$T/ab.log
      timeout -k 10 120 python3 tools/one_batch.py "$oo" --reps 5 --starts $st >> gpurun_out/$T/ab.log 2>&1
    done
  done
done
