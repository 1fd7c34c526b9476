# Seed-grid build cost (kernel stats) and C2 batches against a reference library.
#   bash tools/r3_grid_ab.sh <tag> <lib>
set -e
T=$1; L=$2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.kt -- python3 tools/time_set_targets.py > gpurun_out/$T.kt.log 2>&1
python3 tools/stats_summary.py gpurun_out/$T.kt 8 > gpurun_out/$T.summary.txt
bash tools/ab.sh $T "{}" 30 $L head
bash tools/ab.sh $T "{}" 8 $L head
