set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/bench_c1.py --out gpurun_out/r02_c1.json > gpurun_out/r2x.log 2>&1
tail -1 gpurun_out/r2x.log | cut -c1-300
