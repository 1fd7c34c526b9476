mkdir -p gpurun_out
ORPCD_TRACE=1 timeout -k 10 200 python tools/one_batch.py '{"search_kernel":0}' --reps 1 > gpurun_out/tr0.log 2>&1
ORPCD_TRACE=1 timeout -k 10 200 python tools/one_batch.py '{"search_kernel":2,"scan_blocks":2560}' --reps 1 > gpurun_out/tr2.log 2>&1
ORPCD_TRACE=1 timeout -k 10 200 python tools/one_batch.py '{"search_kernel":1}' --reps 1 > gpurun_out/tr1.log 2>&1
