# Target set-up time (kernel stats of tools/time_set_targets.py) and C2 batches
# against a reference library:  bash tools/r3_setup_ab.sh <tag> <lib>
set -e
T=$1; L=$2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in $L head; do
  if [ "$lib" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/$T.setup.log
  timeout -k 10 120 python3 tools/time_set_targets.py 2>&1 | grep -v WARN | head -9 >> gpurun_out/$T.setup.log
done
unset ORPCD_HIP_LIB
bash tools/ab.sh $T "{}" 30 $L head
