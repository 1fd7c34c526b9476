# Round 5, GPU session 9: full GPU suite (row-sharded target and source set-up), C5 row projection with set-up per rank, C5.
set -e
O=gpurun_out/r5s9; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
step c5rows
timeout -k 10 500 python3 tools/bench_c5_rows.py --ranks 1,2,4,8 --out $O/c5_rows.json > $O/c5_rows.log 2>&1
step c5
timeout -k 10 400 python3 tools/bench_c5.py --cpu-iters 0 --parity 0 --out $O/c5.json > $O/c5.log 2>&1
step done
