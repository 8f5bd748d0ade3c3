#!/bin/bash
# One wrapper for every GPU evidence run (gpurun -- bash tools/gpu.sh MODE OUT [ARGS...]).
# Output goes under gpurun_out/OUT; every GPU step has its own time limit and the steps stop at
# the first failure.
#   suite  OUT                 the whole -m gpu suite, then __graft_entry__.smoke()
#   tests  OUT EXPR [FILES..]  pytest -m gpu -k EXPR over FILES (default tests/)
#   bench  OUT CONFIG [ARGS..] bench.py --config CONFIG ARGS -> OUT/bench_CONFIG.json (+ .log)
#   prof   OUT CONFIG [STEPS]  rocprofv3 kernel-trace + stats, then FETCH_SIZE and WRITE_SIZE
#                              PMC passes (one counter block each) on the screening GEMM
#   py     OUT SCRIPT [ARGS..] python SCRIPT ARGS > OUT/out.jsonl (tools/*.py experiments)
#   trace  OUT CMD...          rocprofv3 --kernel-trace --stats of CMD (a kernel timeline)
#   pmc    OUT REGEX CMD...    a trace pass, then one PMC counter group per rocprofv3 run
#                              (occupancy / waits, FETCH_SIZE, LDS, instruction mix) over the
#                              kernels matching REGEX; summarise with tools/pmc_summary.py
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
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm \
      --output-format csv -d "$O/fetch" -o run -- $B > "$O/fetch.json" 2> "$O/fetch.log" &&
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex screen_gemm \
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
  *)
    echo "usage: tools/gpu.sh suite|tests|bench|prof|py|trace|pmc OUT ..." >&2
    exit 2
    ;;
esac
