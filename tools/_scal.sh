set -e
# per-rank work of strong-scaled C3 (one GPU, --n = rows per rank) + C2
for n in 125000 250000 500000 1000000; do
  timeout -k 10 300 python bench.py --n $n --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sc_$n.json 2> gpurun_out/sc_$n.log
  python -c "import json;d=json.load(open('gpurun_out/sc_$n.json'));print('$n', d['ms_per_step'], d['value'], d['stage_ms_per_step'], d['plan'])"
done
timeout -k 10 300 python bench.py --config C2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sc_c2.json 2> gpurun_out/sc_c2.log
python -c "import json;d=json.load(open('gpurun_out/sc_c2.json'));print('C2', d['ms_per_step'], d['value'], d['stage_ms_per_step'], d['plan'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof125 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 125000 --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2>&1
echo done
