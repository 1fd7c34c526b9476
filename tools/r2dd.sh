# C4 projection: fractional speculative depths for the 8 ranks
set -e
export TMPDIR=/tmp
O=gpurun_out/r2dd
rm -rf $O; mkdir -p $O
for d in 2 1.5 2.5; do
timeout -k 10 400 python3 tools/bench_c4_align.py --depth $d --out $O/c4_$d.json > $O/c4_$d.log 2>&1
done
