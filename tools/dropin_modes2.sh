# Drop-in slowdown: glibc never returning memory to the
# kernel (no munmap / heap trim between batches) against the default.
#   bash tools/dropin_modes2.sh [tag]   (on the GPU box)
set -e
T=${1:-dm2}
mkdir -p gpurun_out/$T
for k in 1 2 3; do
  ORPCD_GAPS=1 MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=4294967296 timeout -k 10 200 python3 tools/bench_dropin.py --reps 3 --legs batched,dropin > gpurun_out/$T/nomunmap$k.log 2>&1
  ORPCD_GAPS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 3 --legs batched,dropin > gpurun_out/$T/plain$k.log 2>&1
done
