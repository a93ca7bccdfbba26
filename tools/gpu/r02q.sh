# Batched host centres: GPU suite + candidate/throughput rates incl. small -n.
set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log
timeout -k 10 600 python tools/cand_rate.py > $O/cand_rate.jsonl 2> $O/cand_rate.err
