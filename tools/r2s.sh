# C4 projection: speculative depth 1 vs auto (2) for the 8 ranks
set -e
export TMPDIR=/tmp
O=gpurun_out/r2s
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 tools/bench_c4_align.py --depth 1 --out $O/c4_d1.json > $O/c4_d1.log 2>&1
timeout -k 10 400 python3 tools/bench_c4_align.py --out $O/c4_auto.json > $O/c4_auto.log 2>&1
timeout -k 10 400 python3 tools/bench_c4_align.py --depth 3 --out $O/c4_d3.json > $O/c4_d3.log 2>&1
