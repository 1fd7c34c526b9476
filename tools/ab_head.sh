# Interleaved A/B of the working-tree library (head) against another build
# (default abl/base.so): exact 30 / 8 starts and fp32 mode 30 starts, result
# hashes printed by tools/one_batch.py.
#   bash tools/ab_head.sh <tag> [lib]   (on the GPU box)
set -e
T=${1:-ab}
OTHER=${2:-abl/base.so}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for cfg in "{} 30" "{} 8" '{"exact_nn":0} 30'; do
    set -- $cfg
    for L in $OTHER head; do
      if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
      echo "== $L starts=$2 opts=$1" >> gpurun_out/$T/ab.log
      timeout -k 10 120 python3 tools/one_batch.py "$1" --reps 5 --starts $2 >> gpurun_out/$T/ab.log 2>&1
    done
  done
done
unset ORPCD_HIP_LIB
