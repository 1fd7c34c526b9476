# Re-search grid of the fused exact accumulation: exact_blocks x exact_fused, C2 batches.
#   bash tools/r3_exact_blocks.sh <tag>
set -e
T=$1
mkdir -p gpurun_out
for st in 30 8; do
  for eb in 256 512 1024 2048 4096; do
    echo "== exact_blocks $eb starts $st" >> gpurun_out/$T.sweep.log
    timeout -k 10 120 python3 tools/one_batch.py "{\"exact_blocks\":$eb,\"exact_fused\":4096}" --reps 5 --starts $st >> gpurun_out/$T.sweep.log 2>&1
  done
done
