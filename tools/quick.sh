set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && tail -2 gpurun_out/gpu_tests.log || exit 1
for a in "" "--pt 8000 --packets 131072" "--suite aes256gcm --keys 64" "--keys 4096 --packets 2097152" "--packets 4096"; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu $a > gpurun_out/q.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/q.json'));c=d['config'];print('$a', d['value'], c['seal_ms'], c['open_ms'])"
done
