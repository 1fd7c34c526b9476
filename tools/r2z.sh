# exact_nn kernel breakdown (30-start C2 batches) for profiles/
set -e
export TMPDIR=/tmp
O=gpurun_out/r2z
rm -rf $O; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python tools/one_batch.py '{"exact_nn":1}' --starts 30 --reps 3 > $O/kt.log 2>&1
