# Kernel statistics of one C2 30-start batch in exact and fast mode, plus an
# 8-start batch.   bash tools/r3_prof.sh [tag]   (on the GPU box)
set -e
T=${1:-pr}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in 1 0; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.kt$m -- python3 tools/one_batch.py "{\"exact_nn\":$m}" --reps 3 > gpurun_out/$T.kt$m.log 2>&1
  timeout -k 10 120 python3 tools/one_batch.py "{\"exact_nn\":$m}" --reps 5 >> gpurun_out/$T.timing.log 2>&1
  timeout -k 10 120 python3 tools/one_batch.py "{\"exact_nn\":$m}" --reps 5 --starts 8 >> gpurun_out/$T.timing.log 2>&1
done
