# A/B: accumulation queries per thread (4 default, 2, 1)
set -e
export TMPDIR=/tmp
O=gpurun_out/r2bb
rm -rf $O; mkdir -p $O
L=multi-scale-pointcloud-registration_amd/orpcd_amd/_lib
for st in 1 8 30 64; do
  for lib in liborpcd_hip ab_q2 ab_q1; do
    echo "== starts $st lib $lib" >> $O/ab.log
    ORPCD_HIP_LIB=$PWD/$L/$lib.so timeout -k 10 60 python tools/one_batch.py '{}' --starts $st --reps 5 2>/dev/null | grep -v WARN >> $O/ab.log
  done
done
