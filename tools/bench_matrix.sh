#!/bin/bash
# BASELINE.json configs on one GPU: each line is one bench.py JSON line (device-resident unless --mode e2e).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-matrix}; out=gpurun_out/$tag; mkdir -p $out
run() { name=$1; shift; timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu "$@" > $out/$name.json 2> $out/$name.err || { echo "FAIL $name"; tail -5 $out/$name.err; return 1; }; python -c "import json;d=json.load(open('$out/$name.json'));print('$name', d['value'], d.get('unit'), d.get('ms_per_step'), d.get('roofline',{}).get('frac'))"; }
run c2_aes128_1key && \
run c3_aes256_64keys --suite aes256gcm --keys 64 && \
run c3_chacha_64keys --suite chacha20poly1305 --keys 64 && \
run c4_aes128_pt300 --pt 300 --packets 4194304 && \
run c4_aes128_pt1452 --pt 1452 && \
run c4_aes128_pt8000 --pt 8000 --packets 131072 && \
run c4_txq_pt300 --mode txq --pt 300 --inflight 32 --coalesce 8 && \
run c4_txq_pt1452 --mode txq --pt 1452 --inflight 32 --coalesce 8 && \
run c4_txq_pt8000 --mode txq --pt 8000 --inflight 32 --coalesce 8 && \
run c5_aes128_4ki_keys --keys 4096 --packets 2097152 && \
run rx_aes128 --mode rx && \
run rx_chacha_64keys --mode rx --suite chacha20poly1305 --keys 64 && \
run keys_4ki_aes128 --mode keys --keys 4096 && \
run txq_aes128 --mode txq && \
run txq_chacha --mode txq --suite chacha20poly1305 && \
run packet_aes128 --mode packet && \
run packet_chacha --mode packet --suite chacha20poly1305 && \
run txq_aes128_32inflight --mode txq --inflight 32 --coalesce 8 && \
run txq_chacha_64inflight --mode txq --suite chacha20poly1305 --inflight 64 --coalesce 16 && \
run e2e_aes128 --mode e2e --steps 3 && \
run e2e_c5_4ki_keys_rotating --mode e2e --keys 4096 --packets 2097152 --rotate --steps 3 && \
run c2_aes128_keyruns64_64keys --keys 64 --key-run 64 && \
run c3_aes128_64keys --keys 64 && \
run c3_mixed_66keys --suite mixed --keys 66 && \
run rx_aes128_64keys --mode rx --keys 64 && \
run rx_aes256_64keys --mode rx --suite aes256gcm --keys 64 && \
run rx_mixed_66keys --mode rx --suite mixed --keys 66 && \
run c4_aes128_pt600 --pt 600 --packets 2097152
