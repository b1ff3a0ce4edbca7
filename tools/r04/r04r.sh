# round 4 step r: the transmit faces per suite and size on the final build: 64-packet flushes (server) and per-packet
# calls at BASELINE configs[3]'s sizes, ChaCha20-Poly1305 and AES-256-GCM beside AES-128-GCM
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04r; mkdir -p $o
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; python -c "import json,sys; d=json.load(open('$o/$tag.json')); print('$tag', d['value'], d.get('unit'), d.get('decrypt_us',''), d.get('hp_mask_us',''))"; }
for suite in aes128gcm aes256gcm chacha20poly1305; do
  for pt in 300 1452 8000; do
    run txq1_${suite}_$pt python bench.py --mode txq --suite $suite --inflight 1 --pt $pt --no-cpu || exit 1
    run packet_${suite}_$pt python bench.py --mode packet --suite $suite --pt $pt --no-cpu || exit 1
  done
done
