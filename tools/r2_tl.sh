# kernel timelines of a 1-start and an 8-start C2 batch under a config: tools/r2_tl.sh OUTDIR 'cfg'
set -e
mkdir -p $1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $1/k1 -- python tools/one_batch.py "$2" --starts 1 --reps 3 > $1/k1.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $1/k8 -- python tools/one_batch.py "$2" --starts 8 --reps 3 > $1/k8.log 2>&1
