set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06a
for m in async sync async_pinned; do
  for s in 0xF025 0xF026 0xF100; do
    timeout -k 5 60 ./tools/diag/pool_repro $m 300 $s > gpurun_out/r06a/pool_${m}_$s.txt 2>&1; echo "pool $m $s rc=$? $(tail -1 gpurun_out/r06a/pool_${m}_$s.txt)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifetime.py tests/test_gpu_packet_server.py tests/test_gpu_servers_device.py tests/test_gpu_threads.py tests/test_gpu_txq_server.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r06a/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r06a/pytest.log; grep -E "^ok frees|evictions" gpurun_out/r06a/pytest.log | head; exit $rc
