# One round's GPU evidence: bench line, rocprofv3 kernel stats + HBM/SQ counter
# passes of the bench command, and the side workloads (C3 FGR, C4 align(), C5, prep, C1, drop-in).
#   bash tools/profile_round.sh [round]   (on the GPU box; outputs under gpurun_out/)
# The raw rocprofv3 CSVs are summarised on the box (tools/summarize_profile.py
# --out-dir gpurun_out/summary) and then deleted: gpurun brings back at most
# 64 MiB of gpurun_out/.  gpurun_out/steps.log names each step as it starts.
set -e
R=${1:-r04}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/kt gpurun_out/fetch gpurun_out/write gpurun_out/sq gpurun_out/summary
step() { echo "$(date +%T) $1" >> gpurun_out/steps.log; }
step bench
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
B="python3 bench.py --cpu-seconds 0 --align 0 --c4 0"  # default steps/warmup: the same kernel mix as the bench line
step kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -- $B > gpurun_out/kt.log 2>&1
step fetch
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch -- $B > gpurun_out/fetch.log 2>&1
step write
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/write -- $B > gpurun_out/write.log 2>&1
step sq
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/sq -- $B > gpurun_out/sq.log 2>&1
step summary
python3 tools/summarize_profile.py --round $R --kt gpurun_out/kt --fetch gpurun_out/fetch --write gpurun_out/write --pmc gpurun_out/sq --out-dir gpurun_out/summary > gpurun_out/summary.log 2>&1
rm -rf gpurun_out/kt gpurun_out/fetch gpurun_out/write gpurun_out/sq
step c4
timeout -k 10 400 python3 tools/bench_c4_align.py --out gpurun_out/c4_align.json > gpurun_out/c4.log 2>&1
step fgr
timeout -k 10 300 python3 tools/bench_fgr.py --out gpurun_out/fgr_c3.json > gpurun_out/fgr.log 2>&1
step c5
timeout -k 10 400 python3 tools/bench_c5.py --out gpurun_out/c5.json > gpurun_out/c5.log 2>&1
step prep
timeout -k 10 300 python3 tools/bench_prep.py --out gpurun_out/prep.json > gpurun_out/prep.log 2>&1
step c1
timeout -k 10 300 python3 tools/bench_c1.py --out gpurun_out/c1.json > gpurun_out/c1.log 2>&1
step dropin
timeout -k 10 300 python3 tools/bench_dropin.py --reps 5 --out gpurun_out/dropin.json > gpurun_out/dropin.log 2>&1
step done
