# Round-5 probes (gpurun -- bash tools/r5_probe.sh): the persistent walk at a whole C5 filter
# launch (2.08M rows x 16384 queries) with its FETCH_SIZE, and the CU-masked overlap probe under
# the two candidate mask-bit layouts (tools/overlap_probe.py).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5e; mkdir -p $O
for lay in blocked interleaved; do
  EBERT_LIB=_abl/libebert_grid.so EBT_QP_GRID=240 timeout -k 10 400 python -u tools/overlap_probe.py --tail-cus 2 --layout $lay > $O/overlap_$lay.jsonl 2> $O/overlap_$lay.err
  tail -1 $O/overlap_$lay.jsonl
done
timeout -k 10 600 python -u tools/walk_stamp.py --n 2083072 --b 16384 --cscale > $O/walk_c5full.jsonl 2> $O/walk_c5full.err
tail -1 $O/walk_c5full.jsonl
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm --output-format csv -d $O/pmc_c5full -o run -- python3 tools/walk_stamp.py --n 2083072 --b 16384 --cscale --warm 2 > $O/pmc_c5full.log 2>&1
