set -e
export TMPDIR=/tmp
O=gpurun_out/r2h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 tools/bench_c4_align.py --out $O/c4.json > $O/c4.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python3 tools/bench_c5.py --parity 0 --cpu-iters 1 --out $O/c5.json > $O/c5.log 2>&1
