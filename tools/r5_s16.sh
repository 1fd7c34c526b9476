# Round 5, GPU session 16: window parity tests, C4 re-deal projection.
set -e
O=gpurun_out/r5s16; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_window.py -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 500 python3 tools/bench_c4_redeal.py --passes 8,16,24,32,48 --out $O/redeal.json > $O/redeal.log 2>&1
