set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 300 python3 tools/bench_c4_align.py --out gpurun_out/r2b/c4_auto.json > gpurun_out/r2b/c4_auto.log 2>&1
timeout -k 10 300 python3 tools/bench_c4_align.py --depth 1 --out gpurun_out/r2b/c4_d1.json > gpurun_out/r2b/c4_d1.log 2>&1
timeout -k 10 300 python3 tools/bench_c4_align.py --no-prefetch --out gpurun_out/r2b/c4_nopf.json > gpurun_out/r2b/c4_nopf.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/r2b/bench.json 2> gpurun_out/r2b/bench.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b/tests.log 2>&1
