set -e
run() { # name args...
  local nm=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/cfg_$nm.json 2> gpurun_out/cfg_$nm.log || { echo "$nm FAILED rc=$?"; tail -20 gpurun_out/cfg_$nm.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/cfg_$nm.json'));print('$nm', d['ms_per_step'], d['value'], d['roofline']['frac'], d['plan'], d['stage_ms_per_step'], d.get('parity'), d.get('device_parity'), d.get('host_boundary'))"
}
run C2 --config C2 --steps 5 --warmup 2 --cpu-budget 10 --device-check 32
run C4r --config C4 --n 1250000 --steps 3 --warmup 1 --no-cpu-baseline --device-check 32
run C5r --config C5 --n 6250000 --steps 2 --warmup 1 --no-cpu-baseline --device-check 32
