# per-kernel averages of C2 batches, ordered vs uniform dispatch (rocprofv3 kernel trace)
set -e
export TMPDIR=/tmp
O=gpurun_out/r2f
mkdir -p $O
for st in 1 8 30; do
  for sc in 0 1; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${st}_$sc -o k -- python3 tools/one_batch.py "{\"sched\":$sc}" --starts $st --reps 3 > $O/kt_${st}_$sc.log 2>&1
  done
done
