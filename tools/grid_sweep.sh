set -e
for L in ab_libs/g24.so head ab_libs/g48.so ab_libs/g64.so; do
  if [ "$L" = head ]; then unset ORPCD_HIP_LIB; else export ORPCD_HIP_LIB=$L; fi
  for st in 30 8; do echo "== $L $st" >> gpurun_out/r3l.log; timeout -k 10 120 python3 tools/one_batch.py "{}" --reps 5 --starts $st >> gpurun_out/r3l.log 2>&1; done
  echo "== $L set_targets" >> gpurun_out/r3l.log; timeout -k 10 120 python3 tools/time_set_targets.py 2>&1 | grep -v WARN | head -4 >> gpurun_out/r3l.log
done
