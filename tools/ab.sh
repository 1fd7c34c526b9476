# A/B of C2 batches (tools/one_batch.py) between libraries, interleaved:
#   bash tools/ab.sh <tag> <opts-json> <starts> <lib>...   (lib: path or "head")
# e.g. bash tools/ab.sh x '{}' 30 ab_libs/base.so head
set -e
T=$1; OPTS=$2; ST=$3; shift 3
mkdir -p gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
    echo "== $L starts=$ST opts=$OPTS" >> gpurun_out/$T.ab.log
    timeout -k 10 120 python3 tools/one_batch.py "$OPTS" --reps 5 --starts $ST >> gpurun_out/$T.ab.log 2>&1
  done
done
unset ORPCD_HIP_LIB
