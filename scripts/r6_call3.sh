#!/bin/bash
# round-6 GPU pass 3: generic transformer fusions (MLP site, residual epilogues, zero-copy SDPA)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gtransformer_gpu.py tests/test_blaslt_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 20 --warmup 5 > $O/vit_b16.json 2> $O/vit_b16.err &&
timeout -k 10 300 python -u bench.py --model transformer-base --steps 30 --warmup 10 > $O/tx_base32.json 2> $O/tx_base32.err &&
timeout -k 10 300 python -u bench.py --model bert-base --steps 30 --warmup 10 > $O/bert_base.json 2> $O/bert_base.err &&
timeout -k 10 300 python -u bench.py --model transformer-base --impl torch --steps 30 --warmup 10 > $O/tx_base32_torch.json 2> $O/tx_base32_torch.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o vit -- python bench.py --model vit-b16 --steps 4 --warmup 3 > $O/prof_vit.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o tx32 -- python bench.py --model transformer-base --steps 6 --warmup 4 > $O/prof_tx.log 2>&1
rc=$?
tail -3 $O/pytest.log; cat $O/*.json
exit $rc
