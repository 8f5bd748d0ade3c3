#!/bin/bash
# Multi-process sharded path on a one-GPU box: bench.py --gpus 2 (and 4) launches its own
# ranks, all on GPU 0 over gloo (--share-gpu), and rank 0 checks the merged top-k against the
# host oracle over the whole regenerated catalog. Then the default N = 1 line.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rehearse
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --gpus 2 --share-gpu --steps 5 --warmup 2 > $O/n2.json 2> $O/n2.log &&
timeout -k 10 400 python -u bench.py --gpus 4 --share-gpu --steps 5 --warmup 2 > $O/n4.json 2> $O/n4.log &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/n1.json 2> $O/n1.log
rc=$?
echo "rehearse rc=$rc"
for f in n2 n4 n1; do cut -c1-400 $O/$f.json; python -c "import json;d=json.load(open('$O/$f.json'));print(d.get('parity'))" 2>/dev/null; done
tail -5 $O/n2.log
exit $rc
