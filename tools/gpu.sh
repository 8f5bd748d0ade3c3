#!/bin/bash
# One wrapper for every GPU evidence run (gpurun -- bash tools/gpu.sh MODE OUT [ARGS...]).
# Output goes under gpurun_out/OUT; every GPU step has its own time limit and the steps stop at
# the first failure.
#   suite  OUT                 the whole -m gpu suite, then __graft_entry__.smoke()
#   tests  OUT EXPR [FILES..]  pytest -m gpu -k EXPR over FILES (default tests/)
#   bench  OUT CONFIG [ARGS..] bench.py --config CONFIG ARGS -> OUT/bench_CONFIG.json (+ .log)
#   prof   OUT CONFIG [STEPS]  rocprofv3 kernel-trace + stats, then FETCH_SIZE and WRITE_SIZE
#                              PMC passes (one counter block each) on the screening GEMM and the
#                              rescore (the top-K roofline's kernel)
#   py     OUT SCRIPT [ARGS..] python SCRIPT ARGS > OUT/out.jsonl (tools/*.py experiments)
#   trace  OUT CMD...          rocprofv3 --kernel-trace --stats of CMD (a kernel timeline)
#   pmc    OUT REGEX CMD...    a trace pass, then one PMC counter group per rocprofv3 run
#                              (occupancy / waits, FETCH_SIZE, LDS, instruction mix) over the
#                              kernels matching REGEX; summarise with tools/pmc_summary.py
#   ab     OUT ALT CFGS [N]    interleaved A/B bench lines (no CPU baseline), N rounds (2) of
#                              every config in CFGS (comma list): the current build, then ALT --
#                              a library (EBERT_LIB=ALT, e.g. _abl/libebert_prev.so from
#                              tools/abl_build.sh) or an environment setting VAR=VALUE
#   epi    OUT LIB...          per-phase filter-epilogue cycles (tools/epi_stamp.py) of C2- and
#                              C3-shaped segments, per -DEBT_EPI_STAMP build _abl/libebert_LIB.so
#   stamp  OUT LIB...          clock-stamp launches (tools/clock_stamp.py) of C2- and C3-shaped
#                              filter segments per -DEBT_CLOCK_STAMP build _abl/libebert_LIB.so
#   recipe NAME                a named evidence run of the table at the end of this file (the
#                              round-4 A/B runs and closing passes, profiles/r4/README.md)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
MODE=$1
O=gpurun_out/$2
shift 2
mkdir -p "$O"
case "$MODE" in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 400 \
      --timeout-method thread -rf --durations=10 > "$O/pytest.log" 2>&1 ||
      { grep -E "FAILED|Error|passed|failed" "$O/pytest.log" | tail -15; exit 1; }
    grep -E "passed|failed" "$O/pytest.log" | tail -1
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ||
      { tail -5 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log"
    ;;
  tests)
    EXPR=$1
    shift
    FILES=${*:-tests}
    timeout -k 10 900 python -u -m pytest $FILES -m gpu -k "$EXPR" -v --maxfail=3 --timeout 400 \
      --timeout-method thread -rf --durations=10 > "$O/pytest.log" 2>&1
    rc=$?
    grep -E "PASSED|FAILED|Error|passed|failed" "$O/pytest.log" | tail -40
    exit $rc
    ;;
  bench)
    CFG=$1
    shift
    timeout -k 10 900 python -u bench.py --config "$CFG" "$@" > "$O/bench_$CFG.json" \
      2> "$O/bench_$CFG.log" || { tail -20 "$O/bench_$CFG.log"; exit 1; }
    python3 - "$O/bench_$CFG.json" <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"].get("workload"), d["n_gpus"], d["value"], d["ms_per_step"],
              (d.get("roofline") or {}).get("frac"), d.get("stage_ms_per_step"),
              (d.get("parity") or {}).get("rows_bit_exact"))
EOF
    ;;
  prof)
    CFG=$1
    STEPS=${2:-5}
    B="python3 bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run \
      -- $B > "$O/trace.json" 2> "$O/trace.log" &&
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'screen_gemm|rescore_kernel' \
      --output-format csv -d "$O/fetch" -o run -- $B > "$O/fetch.json" 2> "$O/fetch.log" &&
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'screen_gemm|rescore_kernel' \
      --output-format csv -d "$O/write" -o run -- $B > "$O/write.json" 2> "$O/write.log"
    rc=$?
    echo "prof $CFG rc=$rc"
    exit $rc
    ;;
  py)
    S=$1
    shift
    timeout -k 10 900 python -u "$S" "$@" > "$O/out.jsonl" 2> "$O/err.log" ||
      { tail -20 "$O/err.log"; exit 1; }
    tail -20 "$O/out.jsonl"
    ;;
  trace)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run \
      -- "$@" > "$O/out.log" 2>&1
    rc=$?
    echo "trace rc=$rc"
    exit $rc
    ;;
  pmc)
    RX=$1
    shift
    P="--kernel-include-regex $RX --output-format csv"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run \
      -- "$@" > "$O/trace.log" 2>&1 &&
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES $P \
      -d "$O/p1" -o run -- "$@" > "$O/p1.log" 2>&1 &&
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE $P -d "$O/p2" -o run -- "$@" > "$O/p2.log" 2>&1 &&
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
      SQ_WAIT_INST_LDS $P -d "$O/p3" -o run -- "$@" > "$O/p3.log" 2>&1 &&
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_SALU \
      SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_MFMA $P -d "$O/p4" -o run -- "$@" > "$O/p4.log" 2>&1
    rc=$?
    echo "pmc rc=$rc"
    exit $rc
    ;;
  ab)
    ALT=$1
    CFGS=$2
    N=${3:-2}
    for i in $(seq "$N"); do
      for c in ${CFGS//,/ }; do
        case $c in C2) A="--steps 400" ;; C3) A="--steps 20" ;; *) A="--steps 5 --warmup 1" ;; esac
        bash "$0" bench "${O#gpurun_out/}/${c}_new$i" "$c" $A --no-cpu-baseline || exit 1
        if [[ $ALT == *=* ]]; then
          env "$ALT" bash "$0" bench "${O#gpurun_out/}/${c}_alt$i" "$c" $A --no-cpu-baseline || exit 1
        else
          EBERT_LIB=$ALT bash "$0" bench "${O#gpurun_out/}/${c}_alt$i" "$c" $A --no-cpu-baseline ||
            exit 1
        fi
      done
    done
    ;;
  epi)
    for v in "$@"; do
      bash "$0" py "${O#gpurun_out/}/c2_$v" tools/epi_stamp.py --lib "_abl/libebert_$v.so" \
        --n 100000 --b 1024 --d 768 --img bf16 --z 2.73 --cscale || exit 1
      bash "$0" py "${O#gpurun_out/}/c3_$v" tools/epi_stamp.py --lib "_abl/libebert_$v.so" || exit 1
    done
    ;;
  stamp)
    for v in "$@"; do
      bash "$0" py "${O#gpurun_out/}/c2_$v" tools/clock_stamp.py --lib "_abl/libebert_$v.so" \
        --n 100000 --b 1024 --d 768 --img bf16 --z 2.73 --cscale --secs 1.5 || exit 1
      bash "$0" py "${O#gpurun_out/}/c3_$v" tools/clock_stamp.py --lib "_abl/libebert_$v.so" \
        --secs 1.5 || exit 1
    done
    ;;
  recipe)
    set -e
    G="bash $0"
    N=${O#gpurun_out/}
    case $N in
      # round 4 (profiles/r4/README.md names each run's output directory)
      r4_walk)     $G suite r4w; $G epi r4w_epi epi_prev epi; $G ab r4w _abl/libebert_prev.so C3,C2 ;;
      r4_evfence)  $G suite r4v; $G ab r4v _abl/libebert_prev.so C2,C3
                   $G trace r4v_trace python3 bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline ;;
      r4_f2key)    $G suite r4k2; $G ab r4k2 _abl/libebert_prev.so C3,C2
                   $G bench r4k2_c2_b512 C2 --steps 50 --no-cpu-baseline --b 512
                   $G bench r4k2_c2_b2048 C2 --steps 50 --no-cpu-baseline --b 2048 ;;
      r4_halfblock) $G suite r4b; $G epi r4b_epi epi_bycol epi; $G ab r4b _abl/libebert_bycol.so C2,C3 ;;
      r4_halfcol)  $G suite r4h2; $G epi r4h2_epi epi_whole epi; $G ab r4h2 _abl/libebert_whole.so C2,C3 ;;
      r4_hitpath)  $G stamp r4h stamp stamp_stageonly stamp_hitnone stamp ;;
      r4_inplace)  $G suite r4i; $G epi r4i_epi epi_staged epi; $G ab r4i _abl/libebert_staged.so C2,C3 ;;
      r4_mred|r4_mslot|r4_rorder)
                   $G suite "$N"; $G ab "$N" _abl/libebert_prev.so C2,C3 ;;
      r4_r4t)      $G suite r4t; $G ab r4t _abl/libebert_head.so C2,C3; $G ab r4t_ldsq EBT_RESCORE_REG=0 C2
                   $G ab r4t_nr1 _abl/libebert_nr1.so C3 1
                   $G bench r4t_c2_streams2 C2 --steps 50 --no-cpu-baseline --streams 2
                   $G stamp r4t_stamp stamp ;;
      r4_sample)   $G ab r4s_d40 _abl/libebert_div40.so C3,C4; $G ab r4s_d30 _abl/libebert_div30.so C3 ;;
      r4_stage)    $G suite r4g; $G epi r4g_epi epi_old epi; $G ab r4g _abl/libebert_head.so C2,C3 ;;
      r4_stores)   $G stamp r4s stamp stamp_nohit stamp_nocnt stamp_none ;;
      r4_final)    $G suite r4f; $G bench r4f C3 --steps 20; $G bench r4f C2 --steps 50
                   $G prof r4f_prof C3 5
                   $G bench r4f C4 --steps 5 --warmup 1 --parity 32
                   $G bench r4f C5 --steps 3 --warmup 1 --parity 32 ;;
      r4_prof_c45) $G prof r4p_c4 C4 3; $G prof r4p_c5 C5 2 ;;
      # round 5 (profiles/r5/README.md)
      r5_lead)     $G ab r5c_ab EBT_SPEC_LEAD=0 C2,C3 2 ;;
      r5_split)    $G ab r5f_ab EBT_FILTER_TPW=0 C5,C4 1 ;;
      r5_walk)     for sh in "c5 --n 520192 --b 16384 --cscale" "c3 --n 333312 --b 4096" \
                             "c5full --n 2083072 --b 16384 --cscale"; do
                     set -- $sh; nm=$1; shift
                     $G py "r5_walk_$nm" tools/walk_stamp.py "$@"
                     timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm \
                       --output-format csv -d "$O/pmc_$nm" -o run -- python3 tools/walk_stamp.py "$@" --warm 2 \
                       > "$O/pmc_$nm.log" 2>&1
                   done ;;
      r5_overlap)  for lay in probe blocked interleaved; do
                     EBERT_LIB=_abl/libebert_grid.so EBT_QP_GRID=240 $G py "r5_overlap_$lay" \
                       tools/overlap_probe.py --tail-cus 2 --layout "$lay"
                   done ;;
      # (A/B builds: tools/abl_build.sh NAME FLAGS, or the previous commit's libebert.so copied
      # to _abl/libebert_prev.so before the change)
      r5_eps)      $G suite r5k; $G ab r5k_ab _abl/libebert_prev.so C3,C2 2 ;;
      r5_sample16) $G ab r5m_s16 _abl/libebert_s16.so C3 2 ;;          # -DEBT_SPEC_SAMPLE_MIN=16
      r5_shardlead) $G trace r5m_rs python3 tools/rank_sim_capi.py --config C3 --world 8 --steps 20
                   EBT_SPEC_LEAD=0 $G py r5m_rs0 tools/rank_sim_capi.py --config C3 --world 8 --steps 20
                   $G py r5m_rs1 tools/rank_sim_capi.py --config C3 --world 8 --steps 20 ;;
      r5_segrate)  $G ab r5s_ab _abl/libebert_prev.so C3 3 ;;
      r5_nr8)      $G ab r5u_ab _abl/libebert_nr8.so C2 3 ;;               # -DEBT_RESCORE_NR_NARROW=8
      r5_final)    $G suite r5t; $G bench r5t C3 --steps 20
                   $G py r5t_rs tools/rank_sim_capi.py --config C3 --world 8 --steps 20
                   $G prof r5t_prof C3 5
                   $G bench r5r_c4 C4 --steps 10; $G bench r5r_c5 C5 --steps 5 --warmup 2
                   $G bench r5r_n2 C3 --gpus 2 --share-gpu --steps 5 --warmup 2 --cpu-budget 4
                   $G bench r5r_n4 C3 --gpus 4 --share-gpu --steps 5 --warmup 2 --cpu-budget 4 ;;
      *) echo "unknown recipe $N" >&2; exit 2 ;;
    esac
    ;;
  *)
    echo "usage: tools/gpu.sh suite|tests|bench|prof|py|trace|pmc|ab|epi|stamp|recipe OUT ..." >&2
    exit 2
    ;;
esac
