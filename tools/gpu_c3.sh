#!/bin/bash
# Persistent vs pre-persistent screening GEMM at C5- / C4- / C3-like shapes (interleaved, one
# process each), then the GPU suite and a C2 bench line of the working tree.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c3; mkdir -p $O
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 3 --b 16384 --n 196608 --d 1536 --cscale pre cur > $O/lab_c5.jsonl 2> $O/lab_c5.log &&
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 3 --b 8192 --n 655360 --d 768 --cscale pre cur > $O/lab_c4.jsonl 2> $O/lab_c4.log &&
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 3 pre cur > $O/lab_c3.jsonl 2> $O/lab_c3.log &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.log
rc=$?
cat $O/lab_c5.jsonl $O/lab_c4.jsonl $O/lab_c3.jsonl; tail -2 $O/pytest.log; cut -c1-300 $O/bench_C2.json
exit $rc
