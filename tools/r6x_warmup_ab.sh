# bench.py vs bench_prev.py (`git show HEAD:bench.py > bench_prev.py` before the run: the tree before
# the warm-up-burst edit, which was then reverted); profiles/r6/host_probe/warmup_ab/
set -e
O=gpurun_out/r6x; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/new$i.json 2> $O/new$i.log
  timeout -k 10 600 python -u bench_prev.py --steps 20 --warmup 5 --no-cpu-baseline > $O/old$i.json 2> $O/old$i.log
done
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > $O/c2new$i.json 2> $O/c2new$i.log
  timeout -k 10 600 python -u bench_prev.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > $O/c2old$i.json 2> $O/c2old$i.log
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r6x/*.json')):
    for l in open(f):
        if l.startswith('{'):
            d=json.loads(l); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'])
PY
