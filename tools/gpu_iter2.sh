# one GPU iteration of the AES kernel work: parity tests of the kernel paths, then the headline bench (3x) and a few
# BASELINE configs.  usage (on the box): bash tools/gpu_iter2.sh [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
K=${1:-"jumbo or ragged or full_size or rfc or fixture"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/iter_tests.log 2>&1; rc=$?
tail -3 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit 1
for a in "" "" "" "--pt 1452" "--pt 300 --packets 4194304" "--pt 8000 --packets 131072" "--suite aes256gcm --keys 64" "--keys 4096 --packets 2097152"; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu $a > gpurun_out/q.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/q.json'));c=d['config'];print('$a', d['value'], c['seal_ms'], c['open_ms'], d['roofline']['frac'])"
done
