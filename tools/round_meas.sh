set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/profile.sh prof_c2b && python tools/summarize_prof.py gpurun_out/prof_c2b > gpurun_out/prof_c2b_summary.txt && python tools/traffic.py gpurun_out/prof_c2b aes128gcm/1200/1 gpurun_out/traffic_c2b.json && \
bash tools/bench_matrix.sh matrix4 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cat gpurun_out/bench_default.json
