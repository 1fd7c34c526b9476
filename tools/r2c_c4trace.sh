# C4 projection with/without RNG prefetch, then a kernel trace of the auto configuration
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2c
timeout -k 10 300 python3 tools/bench_c4_align.py --out gpurun_out/r2c/c4_pf.json > gpurun_out/r2c/c4_pf.log 2>&1
timeout -k 10 300 python3 tools/bench_c4_align.py --no-prefetch --out gpurun_out/r2c/c4_nopf.json > gpurun_out/r2c/c4_nopf.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2c/kt -o c4 -- python3 tools/bench_c4_align.py --out gpurun_out/r2c/c4_traced.json > gpurun_out/r2c/kt.log 2>&1
gzip -f $(find gpurun_out/r2c/kt -name "*kernel_trace.csv")
