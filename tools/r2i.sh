set -e
export TMPDIR=/tmp
O=gpurun_out/r2i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 tools/bench_c4_align.py --out $O/c4.json > $O/c4.log 2>&1
timeout -k 10 300 python3 tools/bench_c4_align.py --interleave --out $O/c4i.json > $O/c4i.log 2>&1
