set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "select or unfused or exact or large_kprime or retry or overflow" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }; tail -1 gpurun_out/gpu_tests.log

for v in old new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_oldsel.so; fi
  EBERT_LIB=$L timeout -k 10 200 python tools/kernel_bench.py --select --select-shapes "4096,65536,200;4096,262144,200;4096,262144,1024;1024,1000000,100" 2>&1 | grep -v amdgpu | sed "s/^/$v /"
done
