# Sweep one runtime option over C2 batches (tools/one_batch.py):
#   bash tools/sweep_opts.sh <tag> <option> "<values>" "<starts list>" [extra-json-fields]
set -e
T=$1; K=$2; VALS=$3; STARTS=$4; EXTRA=${5:-}
mkdir -p gpurun_out
for st in $STARTS; do
  for v in $VALS; do
    echo "== $K $v starts $st" >> gpurun_out/$T.sweep.log
    timeout -k 10 120 python3 tools/one_batch.py "{\"$K\":$v$EXTRA}" --reps 5 --starts $st >> gpurun_out/$T.sweep.log 2>&1
  done
done
