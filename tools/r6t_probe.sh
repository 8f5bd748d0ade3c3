# the fixed cost of a timed window (tools/host_probe.py): 50 timed C2 steps after sequential
# warm-up steps vs after one pipelined burst, against 400 steps; C3's 20 steps likewise
set -e
for i in 1 2; do
  bash tools/gpu.sh py r6w_s50_$i tools/host_probe.py --config C2 --steps 50 --timer
  bash tools/gpu.sh py r6w_s50b_$i tools/host_probe.py --config C2 --steps 50 --timer --burst 100
  bash tools/gpu.sh py r6w_s400_$i tools/host_probe.py --config C2 --steps 400 --timer
  bash tools/gpu.sh py r6w_c3s20_$i tools/host_probe.py --config C3 --steps 20 --timer
  bash tools/gpu.sh py r6w_c3s20b_$i tools/host_probe.py --config C3 --steps 20 --timer --burst 10
  bash tools/gpu.sh py r6w_c3s80_$i tools/host_probe.py --config C3 --steps 80 --timer
done
