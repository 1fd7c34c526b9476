# Round 5, GPU session 7: full GPU suite (split cap back to off), then bench.
set -e
O=gpurun_out/r5s7; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "$(date +%T) $1" >> $O/steps.log; }
step tests
set +e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" >> $O/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
step bench
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
step done
