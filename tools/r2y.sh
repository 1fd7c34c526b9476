set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/prof_align_host.py > gpurun_out/r2y.log 2>&1
