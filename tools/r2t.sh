set -e
export TMPDIR=/tmp
O=gpurun_out/r2t
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 200 --timeout-method thread > $O/exact_tests.log 2>&1 || { tail -40 $O/exact_tests.log; exit 1; }
tail -14 $O/exact_tests.log
