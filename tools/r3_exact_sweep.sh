# Seed-grid build time and the fused re-search's block share, C2 exact batches.
#   bash tools/r3_exact_sweep.sh <tag>
set -e
T=$1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.kt -- python3 tools/one_batch.py "{}" --reps 2 > gpurun_out/$T.kt.log 2>&1
python3 tools/stats_summary.py gpurun_out/$T.kt 8 > gpurun_out/$T.summary.txt
bash tools/sweep_opts.sh $T exact_fused "0 8 16 64 256" "30 8"
