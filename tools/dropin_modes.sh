# Drop-in slowdown: the same drop-in benchmark in fresh
# processes under host-side variants, ORPCD_GAPS on (per batch: device span
# vs host waits).  bash tools/dropin_modes.sh [tag]   (on the GPU box)
set -e
T=${1:-dm}
mkdir -p gpurun_out/$T
for k in 1 2 3; do
  ORPCD_GAPS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 3 --legs batched,dropin > gpurun_out/$T/plain$k.log 2>&1
  ORPCD_GAPS=1 OPENBLAS_NUM_THREADS=1 OMP_NUM_THREADS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 3 --legs batched,dropin > gpurun_out/$T/thr1_$k.log 2>&1
  ORPCD_GAPS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 3 --legs batched,dropin --opt '{"sync_poll": 1}' > gpurun_out/$T/poll$k.log 2>&1
done
