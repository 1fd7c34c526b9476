set -e
export TMPDIR=/tmp
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
