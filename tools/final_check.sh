# End-of-round check on one MI355X: the GPU suite, smoke() and the default bench line.
set -e
O=gpurun_out/final; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set +e
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc" > $O/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke ok" >> $O/steps.log
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "bench ok" >> $O/steps.log
