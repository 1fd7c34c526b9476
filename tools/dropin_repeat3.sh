# Drop-in benchmark in three back-to-back processes (VERDICT r03 weak #6
# done-criterion: within 10% of each other, each <= 2.2x the batched path).
#   bash tools/dropin_repeat3.sh [tag]   (on the GPU box)
set -e
T=${1:-d3}
mkdir -p gpurun_out/$T
for k in 1 2 3; do
  ORPCD_GAPS=1 timeout -k 10 200 python3 tools/bench_dropin.py --reps 5 --legs caller_only,batched,dropin --out gpurun_out/$T/run$k.json > gpurun_out/$T/run$k.log 2>&1
done
