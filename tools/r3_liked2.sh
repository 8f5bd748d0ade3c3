#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3liked2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_capi.py tests/test_gpu_capi_sharded.py tests/test_gpu_certificate.py -m gpu -q -k "liked or golden or user_recs or query_prep or certificate" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/r3_liked.sh ${1:-r3liked2}/b || exit 1
