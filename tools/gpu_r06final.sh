# Round-6 final validation on one box: GPU suite, smoke, default bench line, rocprof trace + PMC passes of the default
# workload and of the receive path (traffic for both into gpurun_out/$T/traffic.json), then the BASELINE matrix.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T=${1:-r06z}
bash tools/gpu.sh $T tests smoke bench prof || exit 1
bash tools/gpu.sh ${T}rx "prof:--mode rx" || exit 1
cp gpurun_out/${T}rx/prof_summary.txt gpurun_out/$T/prof_summary_rx.txt
python tools/traffic.py gpurun_out/${T}rx_prof rx:aes128gcm/1200/1 1048576 gpurun_out/$T/traffic.json || exit 1
bash tools/bench_matrix.sh ${T}_matrix || exit 1
echo final done
