set -e
mkdir -p gpurun_out/r2c
for st in 1 4 8; do
for w in 1024 2048 4096 8192 16384 32768 65536; do
  echo "== starts $st search_waves $w small_batch 0" >> gpurun_out/r2c/sweep.log
  timeout -k 10 60 python tools/one_batch.py "{\"search_waves\": $w, \"small_batch\": 0}" --starts $st --reps 3 2>/dev/null | grep -v WARN >> gpurun_out/r2c/sweep.log
done
done
