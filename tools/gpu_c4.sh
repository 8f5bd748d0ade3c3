#!/bin/bash
# Per-row-group hit staging vs HEAD at C5- / C4- / C3-like shapes, then the GPU suite.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c4; mkdir -p $O
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 3 --b 16384 --n 196608 --d 1536 --cscale base new > $O/lab_c5.jsonl 2> $O/lab_c5.log &&
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 3 --b 8192 --n 655360 --d 768 --cscale base new > $O/lab_c4.jsonl 2> $O/lab_c4.log &&
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 3 base new > $O/lab_c3.jsonl 2> $O/lab_c3.log &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
cat $O/lab_c5.jsonl $O/lab_c4.jsonl $O/lab_c3.jsonl | grep variant | cut -c1-330; tail -2 $O/pytest.log
exit $rc
