# full C2 align(): default and exact_nn GPU runs against the complete CPU oracle run
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python3 -u tools/align_c2_parity.py --out gpurun_out/r02_c2_align_parity.json > gpurun_out/r2q.log 2>&1
tail -3 gpurun_out/r2q.log
