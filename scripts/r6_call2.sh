#!/bin/bash
# round-6 GPU pass 2: generic transformer lowering on the kernels (tests, throughput vs the
# hand BERT engine and stock PyTorch, steady-state kernel list)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gtransformer_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_tx.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model transformer-base --steps 30 --warmup 10 > $O/tx_base.json 2> $O/tx_base.err &&
timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/bert_base.json 2> $O/bert_base.err &&
timeout -k 10 300 python -u bench.py --model transformer-base --impl torch --steps 30 --warmup 10 > $O/tx_base_torch.json 2> $O/tx_base_torch.err &&
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 20 --warmup 5 > $O/vit_b16.json 2> $O/vit_b16.err &&
timeout -k 10 300 python -u bench.py --model vit-b16 --impl torch --steps 20 --warmup 5 > $O/vit_b16_torch.json 2> $O/vit_b16_torch.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o tx -- python bench.py --model transformer-base --steps 6 --warmup 4 > $O/prof_tx.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o vit -- python bench.py --model vit-b16 --steps 4 --warmup 3 > $O/prof_vit.log 2>&1
rc=$?
tail -3 $O/pytest_tx.log; cat $O/*.json
exit $rc
