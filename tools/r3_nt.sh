#!/bin/bash
# non-temporal query loads A/B (_abl/libebert_{base,nt,ntc}.so): in-kernel clock + rate on the
# C3 filter shape and a C5-like batch (16384 queries), then FETCH_SIZE per launch (one --pmc pass each)
export TMPDIR=/tmp
O=gpurun_out/${1:-r3nt}
mkdir -p $O
for v in base nt ntc base nt ntc; do
  timeout -k 10 150 python -u tools/clock_stamp.py --lib _abl/libebert_$v.so --secs 2 > $O/c3_$v.jsonl 2> $O/c3_$v.log || { tail -5 $O/c3_$v.log; exit 1; }
  echo "C3 $v: $(head -1 $O/c3_$v.jsonl | cut -c80-330)"
done
for v in base nt; do
  timeout -k 10 200 python -u tools/clock_stamp.py --lib _abl/libebert_$v.so --secs 3 --b 16384 --n 500000 > $O/c5_$v.jsonl 2> $O/c5_$v.log || { tail -5 $O/c5_$v.log; exit 1; }
  echo "C5-like $v: $(head -1 $O/c5_$v.jsonl | cut -c80-330)"
done
for v in base nt; do
  (cd $O && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm --output-format csv -d pmc_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/clock_stamp.py --lib $GRAFT_REPO_ROOT/_abl/libebert_$v.so --secs 0.3 > pmc_$v.out 2> pmc_$v.log) || exit 1
  python3 -c "
import csv,glob,collections
d=collections.defaultdict(float); n=set()
for f in glob.glob('$O/pmc_$v/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        d[r['Dispatch_Id']]+=float(r['Counter_Value'])
v=sorted(d.values())
print('$v FETCH_SIZE KiB per launch (median of', len(v), '):', v[len(v)//2], '-> GB x2:', round(v[len(v)//2]*1024*2/1e9,2))"
done
