# Drop-in slowdown on re-run: the same drop-in benchmark
# in back-to-back processes, plain and under a kernel trace, so the first and
# a later process can be compared kernel by kernel.
#   bash tools/dropin_repeat.sh [tag]      (on the GPU box)
set -e
T=${1:-dr}
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in 1 2 3; do
  timeout -k 10 200 python3 tools/bench_dropin.py --reps 5 --legs batched,dropin --out gpurun_out/$T/plain$k.json > gpurun_out/$T/plain$k.log 2>&1
done
for k in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt$k -o kt -- python3 tools/bench_dropin.py --reps 5 --legs batched,dropin --out gpurun_out/$T/kt$k.json > gpurun_out/$T/kt$k.log 2>&1
done
