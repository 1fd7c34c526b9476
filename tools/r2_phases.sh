# per-pass phase counters (cycles per search wave) of C2 batches: tools/r2_phases.sh OUTDIR
set -e
mkdir -p $1
export ORPCD_HIP_LIB=$PWD/multi-scale-pointcloud-registration_amd/orpcd_amd/_lib/liborpcd_hip_phases.so
for st in 1 8 30; do
  ORPCD_TRACE=1 ORPCD_PHASES=1 timeout -k 10 120 python tools/one_batch.py '{}' --starts $st --reps 1 > $1/ph$st.log 2>&1
done
