# exact_nn: per-kernel times (kernel trace) of 30- and 8-start C2 batches, exact vs fast
set -e
export TMPDIR=/tmp
O=gpurun_out/r2m
rm -rf $O; mkdir -p $O
for st in 30 8; do
for m in 0 1; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${st}_$m -- python tools/one_batch.py "{\"exact_nn\":$m}" --starts $st --reps 3 > $O/kt_${st}_$m.log 2>&1
done; done
