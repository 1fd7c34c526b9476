set -e
mkdir -p gpurun_out/r2b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ORPCD_TRACE=1 timeout -k 10 120 python tools/one_batch.py '{}' --starts 8 --reps 2 > gpurun_out/r2b/tr8.log 2>&1
ORPCD_TRACE=1 timeout -k 10 120 python tools/one_batch.py '{}' --starts 1 --reps 2 > gpurun_out/r2b/tr1.log 2>&1
timeout -k 10 120 python tools/one_batch.py '{}' --starts 8 --reps 3 > gpurun_out/r2b/b8.log 2>&1
timeout -k 10 120 python tools/one_batch.py '{}' --starts 1 --reps 3 > gpurun_out/r2b/b1.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2b/kt8 -- python tools/one_batch.py '{}' --starts 8 --reps 2 > gpurun_out/r2b/kt8.log 2>&1
