# A/B of the C4 per-rank step: _abl/libebert_prev.so vs the tree's libebert.so, interleaved on
# one box, after the GPU tests and the first-pass certificate statistics
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/cert_stats.py --config C4 --n 1250000 2>/dev/null
for rep in 1 2; do
for v in prev new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_prev.so; fi
  EBERT_LIB=$L timeout -k 10 300 python bench.py --config C4 --n 1250000 --steps 5 --warmup 1 --no-cpu-baseline --device-check 8 > gpurun_out/ab4_$v.json 2> gpurun_out/ab4_$v.log
  python -c "import json;d=json.load(open('gpurun_out/ab4_$v.json'));print('$v C4r', d['ms_per_step'], d['stage_ms_per_step'], d['device_parity']['rows_bit_exact'])"
done
done
for rep in 1 2; do
for v in prev new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_prev.so; fi
  EBERT_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab3_$v.json 2> gpurun_out/ab3_$v.log
  python -c "import json;d=json.load(open('gpurun_out/ab3_$v.json'));print('$v C3', d['ms_per_step'], d['stage_ms_per_step'])"
done
done
