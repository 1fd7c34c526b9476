# Cost of the bench's live instrumentation on a C2 30-start batch:
# none / hipEvents only / hipEvents + scanned-quarter counters (and the fp32 mode's quarters)
set -e
T=$1
for rep in 1 2; do
  for o in '{}' '{"profiling":1,"count_tiles":0}' '{"profiling":1}' '{"profiling":1,"exact_nn":0}'; do
    echo "== $o" >> gpurun_out/$T.log
    timeout -k 10 120 python3 tools/one_batch.py "$o" --reps 5 >> gpurun_out/$T.log 2>&1
  done
done
