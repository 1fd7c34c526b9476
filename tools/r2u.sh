# exact_nn: kernel trace of a 30-start C2 batch (per-launch durations of the re-search kernel)
set -e
export TMPDIR=/tmp
O=gpurun_out/r2u
rm -rf $O; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -- python tools/one_batch.py '{"exact_nn":1}' --starts 30 --reps 2 > $O/kt.log 2>&1
