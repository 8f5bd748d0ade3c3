#!/bin/bash
# rocprofv3 evidence of the default C3 bench command with 30 timed steps (the timed launches
# dominate the kernel-stats average), then the PMC traffic passes
export TMPDIR=/tmp
bash tools/prof_bench.sh C3 30 || exit 1
python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/prof_C3/trace.json') if l.startswith('{')][0]
print('profiled bench line', d['value'], d['ms_per_step'], 'avg_ms', d['roofline']['per_launch']['avg_ms'], 'launches', d['roofline']['per_launch']['launches'])"
grep "qp2_kernel<false, 1" $(find gpurun_out/prof_C3/trace -name "*kernel_stats.csv") | cut -d, -f1-4
