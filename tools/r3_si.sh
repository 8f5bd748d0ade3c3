#!/bin/bash
# screen image / HBM kernels (tools/topk_evidence.py) + the parity tests that cover them
export TMPDIR=/tmp
O=gpurun_out/${1:-r3si}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_certificate.py -m gpu -q -k "screen_image or golden or non_finite or certificate or select or unfused or overflow or no_fuse" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u tools/topk_evidence.py > $O/topk_evidence.jsonl 2> $O/topk_evidence.log || { tail -5 $O/topk_evidence.log; exit 1; }
cat $O/topk_evidence.jsonl
