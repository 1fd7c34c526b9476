# Drop-in slowdown: A/B of the host environment around
# the same drop-in benchmark, back-to-back processes, with the cgroup's CPU
# throttling counters read before and after every run.
#   bash tools/dropin_env_ab.sh [tag]      (on the GPU box)
set -e
T=${1:-de}
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
H=gpurun_out/$T/host.txt
nproc > $H
for f in cpu.max cpu.max.burst; do echo "$f: $(cat /sys/fs/cgroup/$f 2>/dev/null)" >> $H; done
echo "OMP=$OMP_NUM_THREADS OPENBLAS=$OPENBLAS_NUM_THREADS MKL=$MKL_NUM_THREADS" >> $H
python3 -c "import numpy; numpy.show_config()" >> $H 2>&1 || true
run() {  # name, env...
  local name=$1; shift
  echo "== $name before: $(tr '\n' ' ' < /sys/fs/cgroup/cpu.stat 2>/dev/null)" >> $H
  env "$@" timeout -k 10 200 python3 tools/bench_dropin.py --reps 5 --legs batched,dropin,dropin_nospec --out gpurun_out/$T/$name.json > gpurun_out/$T/$name.log 2>&1
  echo "== $name after:  $(tr '\n' ' ' < /sys/fs/cgroup/cpu.stat 2>/dev/null)" >> $H
}
for k in 1 2; do
  run default$k X=1
  run blas1_$k OPENBLAS_NUM_THREADS=1
done
run default3 X=1
