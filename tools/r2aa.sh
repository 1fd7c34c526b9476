set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
ORPCD_TRACE=1 timeout -k 10 300 python3 tools/bench_fgr.py --out gpurun_out/fgr_trace.json > gpurun_out/fgr_trace.log 2>&1
grep feat_nn gpurun_out/fgr_trace.log | head -6
