# full GPU test suite + smoke on the current head
set -e
export TMPDIR=/tmp
O=gpurun_out/r2r
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/tests.log; tail -2 $O/smoke.log
