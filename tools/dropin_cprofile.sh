# Drop-in slowdown: where the host time inside
# optimize() goes, first and second process on the box (cProfile).
#   bash tools/dropin_cprofile.sh [tag]      (on the GPU box)
set -e
T=${1:-dp}
mkdir -p gpurun_out/$T
for k in 1 2; do
  timeout -k 10 200 python3 -m cProfile -o gpurun_out/$T/prof$k.out tools/bench_dropin.py --reps 5 --legs batched,dropin > gpurun_out/$T/run$k.log 2>&1
  python3 -c "import pstats; p = pstats.Stats('gpurun_out/$T/prof$k.out'); p.sort_stats('cumulative').print_stats(45)" > gpurun_out/$T/stats$k.txt
  python3 -c "import pstats; p = pstats.Stats('gpurun_out/$T/prof$k.out'); p.sort_stats('tottime').print_stats(30)" > gpurun_out/$T/tot$k.txt
done
