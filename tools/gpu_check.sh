# GPU tests + smoke + bench line + C4 align() projection (one gpurun call).
#   bash tools/gpu_check.sh [tag]     (outputs under gpurun_out/)
# Test failures (pytest rc 1) do not stop the later steps; anything else
# (a crash, an abort, a time limit) does.
set -e
T=${1:-chk}
mkdir -p gpurun_out
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$T.tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/$T.tests.log
if [ "$rc" != 0 ] && [ "$rc" != 1 ]; then exit "$rc"; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/$T.bench.json 2> gpurun_out/$T.bench.err
if [ "${C4:-1}" = 1 ]; then
  timeout -k 10 400 python3 tools/bench_c4_align.py --out gpurun_out/$T.c4_align.json > gpurun_out/$T.c4.log 2>&1
fi
exit "$rc"
