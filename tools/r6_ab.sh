#!/bin/bash
# Round-6 A/B runs (gpurun -- bash tools/r6_ab.sh MODE OUT): every step under its own time
# limit, stopping at the first failure.
#   shard OUT   the sharded GPU tests, then rank 0's C3/8 replay (tools/rank_sim_capi.py)
#               interleaved: _abl/libebert_r6base.so (round-6 tree before the sharded-step
#               fusions), the current build, twice each
#   lever OUT   the LDS-read-bytes-per-MFMA clock lab (tools/gemm_lab/lds_lever.hip)
#   c5full OUT  C5 on 8 thread ranks at the real 6.25M-row shard size (tools/c5_full_shards.py)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
MODE=$1
O=gpurun_out/$2
mkdir -p "$O"
case "$MODE" in
  shard)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_sharded.py \
      tests/test_gpu_capi_sharded.py tests/test_gpu_sharded_scale.py tests/test_gpu_multiprocess.py \
      -m gpu -q -x --timeout 300 --timeout-method thread -rf > "$O/pytest.log" 2>&1 ||
      { tail -30 "$O/pytest.log"; exit 1; }
    tail -1 "$O/pytest.log"
    for i in 1 2; do
      for v in base new; do
        if [ $v = base ]; then L=_abl/libebert_r6base.so; else L=robot_ebert_amd/libebert.so; fi
        EBERT_LIB=$L timeout -k 10 400 python -u tools/rank_sim_capi.py --config C3 --world 8 \
          --steps 20 > "$O/rs_${v}_$i.json" 2> "$O/rs_${v}_$i.log" ||
          { tail -20 "$O/rs_${v}_$i.log"; exit 1; }
        python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], {k: d[k] for k in d if 'ms' in k})" "$O/rs_${v}_$i.json" "$v$i"
      done
    done
    ;;
  c5full)
    # C5 on 8 thread ranks of 6.25M-row shards, one batch through the C ABI's sharded step
    timeout -k 10 1000 python -u tools/c5_full_shards.py --sample 16 --replay 4 > "$O/c5full.json" \
      2> "$O/c5full.log" || { tail -20 "$O/c5full.log"; exit 1; }
    cat "$O/c5full.json"
    ;;
  lever)
    # tools/gemm_lab/lds_lever.hip built as _abl/lds_lever: LDS-read bytes per MFMA vs clock
    timeout -k 10 300 ./_abl/lds_lever 2.5 3 > "$O/lever.jsonl" 2> "$O/lever.log" ||
      { tail -20 "$O/lever.log"; exit 1; }
    cat "$O/lever.jsonl"
    ;;
esac
