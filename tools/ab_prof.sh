# Kernel statistics (rocprofv3 --kernel-trace --stats) of one C2 batch per
# library:   bash tools/ab_prof.sh <tag> <opts-json> <starts> <lib>...  (lib: path or "head")
set -e
T=$1; OPTS=$2; ST=$3; shift 3
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in "$@"; do
  if [ "$L" = head ]; then unset ORPCD_HIP_LIB; N=head; else export ORPCD_HIP_LIB=$L; N=$(basename $L .so); fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.$N -- python3 tools/one_batch.py "$OPTS" --reps 3 --starts $ST > gpurun_out/$T.$N.log 2>&1
done
unset ORPCD_HIP_LIB
