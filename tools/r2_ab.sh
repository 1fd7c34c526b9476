# A/B of runtime options on C2 multistart batches: tools/r2_ab.sh OUTDIR 'cfgA' 'cfgB' ...
set -e
out=$1; shift
mkdir -p $out
for st in 1 8 30 64; do
  for cfg in "$@"; do
    echo "== starts $st cfg $cfg" >> $out/ab.log
    timeout -k 10 60 python tools/one_batch.py "$cfg" --starts $st --reps 4 2>/dev/null | grep -v WARN >> $out/ab.log
  done
done
