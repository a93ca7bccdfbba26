# bench.py after the p66 data note: N=1 line and a 2-rank torchrun rehearsal on one GPU.
set -o pipefail
O=gpurun_out/r02zb
mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/n1.json 2> $O/n1.err && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/n2.json 2> $O/n2.err
