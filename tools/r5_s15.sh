# Round 5, GPU session 15: pass-window / resume parity.
set -e
O=gpurun_out/r5s15; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_window.py tests/test_gpu_gicp.py -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
