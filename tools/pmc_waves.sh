# Search-kernel L2 traffic, 1-wave against 4-wave workgroups:
# the same C2 bench command per library, one kernel-trace pass and one TCC pass each.
#   bash tools/pmc_waves.sh name:lib.so ...   (on the GPU box; outputs under gpurun_out/pmcw/)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmcw
mkdir -p $O
B="python3 bench.py --cpu-seconds 0 --align 0 --c4 0 --steps 5 --warmup 2"
for v in "$@"; do
  n=${v%%:*}; lib=${v#*:}
  echo "$(date +%T) $n kt" >> $O/steps.log
  ORPCD_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n/kt -- $B > $O/$n.kt.log 2>&1
  echo "$(date +%T) $n tcc" >> $O/steps.log
  ORPCD_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/$n/tcc -- $B > $O/$n.tcc.log 2>&1
  echo "$(date +%T) $n tcp" >> $O/steps.log
  ORPCD_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAVES SQ_INSTS_VMEM_RD --output-format csv -d $O/$n/tcp -- $B > $O/$n.tcp.log 2>&1 || echo "$n tcp pass failed" >> $O/steps.log
done
python3 tools/pmc_compare.py $O "$@" > $O/summary.json
rm -rf $O/*/kt $O/*/tcc $O/*/tcp
