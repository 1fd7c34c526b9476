# Round 5, GPU session 10: C4 projection with the imbalance diagnostics (contiguous and interleaved sharding).
set -e
O=gpurun_out/r5s10; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step c4
timeout -k 10 400 python3 tools/bench_c4_align.py --out $O/c4.json > $O/c4.log 2>&1
step c4b
timeout -k 10 400 python3 tools/bench_c4_align.py --out $O/c4b.json > $O/c4b.log 2>&1
step c4i
timeout -k 10 400 python3 tools/bench_c4_align.py --interleave --out $O/c4i.json > $O/c4i.log 2>&1
step done
