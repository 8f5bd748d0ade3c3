set -e
timeout -k 10 300 python -u -m pytest tests/test_als.py -x -q --timeout 120 --timeout-method thread > gpurun_out/als_tests.log 2>&1 || { tail -40 gpurun_out/als_tests.log; exit 1; }
tail -1 gpurun_out/als_tests.log
timeout -k 10 300 python tools/als_bench.py 2>&1 | grep -v amdgpu.ids
