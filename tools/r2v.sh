# final check on the head: full GPU suite, smoke, bench line
set -e
export TMPDIR=/tmp
O=gpurun_out/r2v
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
tail -2 $O/tests.log; tail -1 $O/smoke.log
