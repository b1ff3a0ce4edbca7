set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06b
for m in async async_keep sync; do
  for s in 0xF025 0xF100 0xF101 0xF102; do
    timeout -k 5 60 ./tools/diag/pool_repro $m 300 $s > gpurun_out/r06b/pool_${m}_$s.txt 2>&1; echo "pool $m $s rc=$? $(tail -1 gpurun_out/r06b/pool_${m}_$s.txt)"
  done
done
