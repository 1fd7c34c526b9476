# multi-rank bench rehearsal: two ranks sharing the one GPU over gloo (not a scaling figure)
set -e
export TMPDIR=/tmp
O=gpurun_out/r2w
rm -rf $O; mkdir -p $O
ORPCD_BENCH_DEVICE=0 ORPCD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > $O/bench2.json 2> $O/bench2.err
cat $O/bench2.json
