# per-rank work of the C3 row-sharded step at 8 ranks (tools/shard_sim.py --one-rank)
set -e
cd tools && timeout -k 10 400 python shard_sim.py --one-rank --ranks 8 4 --steps 20 2>&1 | grep -v amdgpu.ids
