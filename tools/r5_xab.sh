set -o pipefail
O=gpurun_out/${XAB_OUT:-r5xab}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -k "excl or exclusion or user_recs or liked or route" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for c in C2 C3; do
    case $c in C2) A="--steps 50";; C3) A="--steps 20";; esac
    timeout -k 10 600 python -u bench.py --config $c $A --exclude 128 --no-cpu-baseline > $O/${c}_new$i.json 2> $O/${c}_new$i.log || exit 1
    EBERT_LIB=_abl/libebert_prev.so timeout -k 10 600 python -u bench.py --config $c $A --exclude 128 --no-cpu-baseline > $O/${c}_alt$i.json 2> $O/${c}_alt$i.log || exit 1
  done
done
for f in $O/*.json; do python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['stage_ms_per_step']['merge_select'])
" $f; done
