# Round-3 per-pass anatomy of a C2 batch (exact and fast mode) and the exact
# re-search grid sweep.   bash tools/r3_trace.sh [tag]   (on the GPU box)
set -e
T=${1:-tr}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T.kt_exact -- python3 tools/one_batch.py '{"exact_nn":1}' --reps 2 > gpurun_out/$T.kt_exact.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T.kt_fast -- python3 tools/one_batch.py '{"exact_nn":0}' --reps 2 > gpurun_out/$T.kt_fast.log 2>&1
ORPCD_TRACE=1 timeout -k 10 120 python3 tools/one_batch.py '{"exact_nn":1}' --reps 1 > gpurun_out/$T.trace_exact.log 2>&1
for b in 64 256 1024 4096; do
  echo "exact_blocks $b" >> gpurun_out/$T.sweep.log
  timeout -k 10 120 python3 tools/one_batch.py "{\"exact_blocks\":$b}" --reps 4 >> gpurun_out/$T.sweep.log 2>&1
  timeout -k 10 120 python3 tools/one_batch.py "{\"exact_blocks\":$b}" --reps 4 --starts 8 >> gpurun_out/$T.sweep.log 2>&1
done
for m in 0 1; do
  echo "exact_nn $m" >> gpurun_out/$T.sweep.log
  timeout -k 10 120 python3 tools/one_batch.py "{\"exact_nn\":$m}" --reps 4 >> gpurun_out/$T.sweep.log 2>&1
  timeout -k 10 120 python3 tools/one_batch.py "{\"exact_nn\":$m}" --reps 4 --starts 8 >> gpurun_out/$T.sweep.log 2>&1
done
