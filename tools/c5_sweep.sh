# C5 (one start, 1M <-> 1M) against the split knobs: the small-batch halving
# (small_batch 0 disables it) and the wave target.   bash tools/c5_sweep.sh [tag]
set -e
T=${1:-c5s}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for o in '{}' '{"small_batch":0}' '{"small_batch":0,"search_waves":65536}' '{"search_waves":65536}' '{"search_waves":16384}'; do
    n=$(echo "$o" | tr -dc 'a-z0-9_')
    timeout -k 10 200 python3 tools/bench_c5.py --cpu-iters 0 --parity 0 --opt "$o" --out gpurun_out/$T/${n:-default}_$rep.json > gpurun_out/$T/${n:-default}_$rep.log 2>&1
  done
done
