# Multi-rank rehearsal of the driver's N>1 launch (2 ranks sharing the box's one GPU), both workloads;
# then config C (k=4) and config D (p130) lines on the final build.
set -o pipefail
O=gpurun_out/r02o
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 4 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 2 --workload p130 --steps 4 --warmup 1 > $O/bench_n2_p130.json 2> $O/bench_n2_p130.err && \
timeout -k 10 400 python bench.py --k 4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_k4.json 2> $O/bench_k4.err && \
timeout -k 10 400 python bench.py --workload p130 --steps 30 --warmup 3 --cpu-seconds 60 > $O/bench_p130.json 2> $O/bench_p130.err
