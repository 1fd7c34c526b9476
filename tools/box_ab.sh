# the clamped (v_med3) box distance against the
# max-form one, at 16- and 8-point in-tile boxes; exact 30 / 8 starts and
# fp32 mode 30 starts, interleaved, result hashes printed by one_batch.py.
#   bash tools/box_ab.sh   (on the GPU box; libraries built into abl/)
set -e
mkdir -p gpurun_out/box
for rep in 1 2; do
  for cfg in "{} 30" "{} 8" '{"exact_nn":0} 30'; do
    set -- $cfg
    for L in abl/base.so head abl/base_q8.so abl/q8.so; do
      if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
      echo "== $L starts=$2 opts=$1" >> gpurun_out/box/ab.log
      timeout -k 10 120 python3 tools/one_batch.py "$1" --reps 5 --starts $2 >> gpurun_out/box/ab.log 2>&1
    done
  done
done
unset ORPCD_HIP_LIB
