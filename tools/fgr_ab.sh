# Interleaved A/B of the feature-NN builds (tools/fgr_ab.py), then a
# kernel-trace summary of each.   bash tools/fgr_ab.sh <tag> <lib>...   (GPU box)
set -e
T=$1; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
    timeout -k 10 180 python3 tools/fgr_ab.py --tag "$L" >> gpurun_out/$T/ab.log 2>&1
  done
done
unset ORPCD_HIP_LIB
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/kt_$n -o run --output-format csv -- python3 tools/fgr_ab.py --tag "$L" --reps 3 > gpurun_out/$T/kt_$n.log 2>&1
  python3 tools/stats_summary.py gpurun_out/$T/kt_$n > gpurun_out/$T/kt_$n.txt 2>&1 || true
  find gpurun_out/$T/kt_$n -name "*kernel_trace.csv" -delete
done
unset ORPCD_HIP_LIB
ORPCD_TRACE=1 timeout -k 10 180 python3 tools/fgr_ab.py --tag trace --reps 1 2>&1 | grep "feat_nn" | sort | uniq -c > gpurun_out/$T/flagged.txt || true
ORPCD_FGR_TRACE=1 timeout -k 10 180 python3 tools/fgr_ab.py --tag phases --reps 2 > gpurun_out/$T/phases.txt 2>&1 || true
