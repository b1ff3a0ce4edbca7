#!/bin/bash
# Round-end refresh: rocprof trace + PMC passes of the default workload, traffic.json, config matrix, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/profile.sh prof_final && python tools/summarize_prof.py gpurun_out/prof_final > gpurun_out/prof_final_summary.txt && \
python tools/traffic.py gpurun_out/prof_final aes128gcm/1200/1 gpurun_out/traffic_final.json && \
bash tools/bench_matrix.sh matrix5 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && cat gpurun_out/bench_final.json
