# round 4 step w: per-packet items of two 64-block passes on two waves (txs_two_wave): the server and packet tests,
# then per-packet latency at 300 / 1200 / 1452 B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04w; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_packet_server.py tests/test_gpu_txq_server.py tests/test_gpu_txrx.py -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; python -c "import json; d=json.load(open('$o/$tag.json')); print('$tag', d['value'], d.get('decrypt_us'), d.get('hp_mask_us'))"; }
for pt in 300 1200 1452; do
  run packet_aes_$pt python bench.py --mode packet --pt $pt --no-cpu || exit 1
done
run packet_aes256_1200 python bench.py --mode packet --suite aes256gcm --no-cpu
