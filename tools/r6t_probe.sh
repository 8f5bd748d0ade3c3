# bench.py's C2 line against the host probe's loop on one box (tools/host_probe.py), twice
set -e
for i in 1 2; do
  bash tools/gpu.sh bench r6u_bench$i C2 --steps 50 --no-cpu-baseline
  bash tools/gpu.sh bench r6u_bench400_$i C2 --steps 400 --no-cpu-baseline
  bash tools/gpu.sh py r6u_d1_$i tools/host_probe.py --config C2 --steps 400 --timer
  bash tools/gpu.sh py r6u_d2_$i tools/host_probe.py --config C2 --steps 400 --timer --depth 2
  bash tools/gpu.sh py r6u_d1s50_$i tools/host_probe.py --config C2 --steps 50 --timer
done
