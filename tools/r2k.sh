# Round-2 refresh on the current head: GPU tests, then the bench line.
set -e
export TMPDIR=/tmp
O=gpurun_out/r2k
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
