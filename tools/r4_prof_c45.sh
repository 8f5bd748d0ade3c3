#!/bin/bash
# Round-4 rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes of the C4 and C5 bench commands
# (gpurun -- bash tools/r4_prof_c45.sh) -> profiles/pmc_C{4,5}_n1.json, profiles/r4_bench_C{4,5}_kernel_stats.csv
set -e
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu.sh prof r4p_c4 C4 3
bash tools/gpu.sh prof r4p_c5 C5 2
