# Drop-in slowdown: A/B of the host environment around
# the same drop-in benchmark, back-to-back processes.
#   bash tools/dropin_env_ab.sh [tag]      (on the GPU box)
set -e
T=${1:-de}
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
nproc > gpurun_out/$T/host.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/$T/host.txt 2>/dev/null || true
echo "OMP=$OMP_NUM_THREADS OPENBLAS=$OPENBLAS_NUM_THREADS" >> gpurun_out/$T/host.txt
for k in 1 2; do
  timeout -k 10 200 python3 tools/bench_dropin.py --reps 5 --legs batched,dropin --out gpurun_out/$T/default$k.json > gpurun_out/$T/default$k.log 2>&1
  OPENBLAS_NUM_THREADS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 5 --legs batched,dropin --out gpurun_out/$T/blas1_$k.json > gpurun_out/$T/blas1_$k.log 2>&1
done
