#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/cab; mkdir -p $O
for v in pre cur; do
  EBERT_LIB=$GRAFT_REPO_ROOT/_abl/libebert_$v.so timeout -k 10 300 python tools/cert_ab.py --config C5 --n 6250000 >> $O/cert.jsonl 2> $O/cert_$v.log || exit 1
done
cat $O/cert.jsonl
