# per-wave search timelines of C2 batches (instrumented library): tools/r2d_wavetime.sh [cfg...]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2d
L=$PWD/multi-scale-pointcloud-registration_amd/orpcd_amd/_lib/liborpcd_hip_wt.so
i=0
for cfg in "$@"; do
  i=$((i+1))
  for st in 30 104; do
    rm -f gpurun_out/r2d/wt.bin
    ORPCD_HIP_LIB=$L ORPCD_WAVETIME=$PWD/gpurun_out/r2d/wt.bin timeout -k 10 120 python3 tools/one_batch.py "$cfg" --starts $st --reps 1 > gpurun_out/r2d/wt${i}_$st.log 2>&1
    python3 tools/wavetime.py gpurun_out/r2d/wt.bin --every 10 > gpurun_out/r2d/wt${i}_$st.txt 2>&1 || true
    rm -f gpurun_out/r2d/wt.bin
  done
done
