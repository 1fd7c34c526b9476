# Round 5, GPU session 14: two halves of a multistart on two streams at once vs one batch.
set -e
O=gpurun_out/r5s14; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/concurrent_halves.py --starts 30 > $O/halves30.log 2>&1
timeout -k 10 200 python3 tools/concurrent_halves.py --starts 64 > $O/halves64.log 2>&1
