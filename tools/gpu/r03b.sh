# Round 3: full GPU suite (incl. overflow rescan, EBUSY, epoch intervals), the bench line with the
# device-busy roofline, the same command under a rocprofv3 kernel trace (tools/trace_union.py), and a
# 2-rank torchrun rehearsal of the static -b 66 split on one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 120 ./tools/microbench/valu_cost > $O/valu_cost.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 20 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
T=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_union.py $T --steps 20 --bench $O/trace_bench.json > $O/trace_union.json || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err
echo "n2 rc=$?"
cat $O/trace_union.json
