# A/B of library builds on C2 multistart batches:
#   tools/ab_libs.sh OUTDIR lib1.so lib2.so ...   (paths relative to the repo)
# per build and batch size: batch wall times + result hash, then per-kernel
# average durations of an 8-start batch (rocprofv3 kernel trace).
set -e
out=$1; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for st in 1 8 30 64; do
  for lib in "$@"; do
    echo "== starts $st lib $lib" >> $out/ab.log
    ORPCD_HIP_LIB=$PWD/$lib timeout -k 10 60 python tools/one_batch.py '{}' --starts $st --reps 4 2>/dev/null | grep -v WARN >> $out/ab.log
  done
done
done
i=0
for lib in "$@"; do
  i=$((i+1))
  ORPCD_HIP_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt$i -- python tools/one_batch.py '{}' --starts 8 --reps 4 > $out/kt$i.log 2>&1
done
