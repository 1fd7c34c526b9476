# A/B: LDS-staged tile boxes (resident ordered-dispatch search, static or atomic item order) vs per-wave dispatch
set -e
export TMPDIR=/tmp
O=gpurun_out/r2p
rm -rf $O; mkdir -p $O
L=multi-scale-pointcloud-registration_amd/orpcd_amd/_lib
for st in 16 30 64; do
  for lib in liborpcd_hip ab_dyn; do
  for cfg in '{"lds_boxes":0}' '{"lds_boxes":1}'; do
    echo "== starts $st lib $lib cfg $cfg" >> $O/ab.log
    ORPCD_HIP_LIB=$PWD/$L/$lib.so timeout -k 10 60 python tools/one_batch.py "$cfg" --starts $st --reps 5 2>/dev/null | grep -v WARN >> $O/ab.log
  done
  done
done
