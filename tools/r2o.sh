# A/B: exact-mode search register budget / scan unroll variants (C2 batches)
set -e
export TMPDIR=/tmp
O=gpurun_out/r2o
rm -rf $O; mkdir -p $O
L=multi-scale-pointcloud-registration_amd/orpcd_amd/_lib
for st in 8 30; do
  for v in a b c d e; do
    for cfg in '{"exact_nn":0}' '{"exact_nn":1}'; do
      echo "== starts $st lib $v cfg $cfg" >> $O/ab.log
      ORPCD_HIP_LIB=$PWD/$L/ab_$v.so timeout -k 10 60 python tools/one_batch.py "$cfg" --starts $st --reps 4 2>/dev/null | grep -v WARN >> $O/ab.log
    done
  done
done
