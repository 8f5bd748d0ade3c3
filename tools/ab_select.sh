# A/B of the streaming select: _abl/libebert_prev.so vs the tree's libebert.so, interleaved on one box
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for v in prev new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_prev.so; fi
  echo "== $v"
  EBERT_LIB=$L timeout -k 10 200 python tools/kernel_bench.py --select --select-shapes "4096,65536,200;4096,262144,200;1024,1000000,128;256,1000000,1000" 2>/dev/null
done
done
