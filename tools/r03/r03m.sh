# round-3 matrix on one box: server phase trace, txq latency/sustained, C3, RX many keys, C5 end to end
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r03m
o=gpurun_out/r03m
run() { local tag=$1; shift; timeout -k 10 240 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(cat $o/$tag.json)"; }
QPP_LIB=$PWD/ab/sT.so timeout -k 10 120 python tools/diag/server_trace.py > $o/server_trace.txt 2>&1 && cat $o/server_trace.txt && \
run txq1 python bench.py --mode txq --inflight 1 --no-cpu && \
run txq32 python bench.py --mode txq --inflight 32 --coalesce 8 --no-cpu && \
run c3_aes256_64 python bench.py --suite aes256gcm --keys 64 --no-cpu && \
run c3_aes128_64 python bench.py --keys 64 --no-cpu && \
run c3_chacha_64 python bench.py --suite chacha20poly1305 --keys 64 --no-cpu && \
run rx_aes128_64 python bench.py --mode rx --keys 64 --no-cpu && \
run c5_e2e python bench.py --mode e2e --keys 4096 --rotate --packets 2097152 --steps 6 --warmup 2 --no-cpu && \
run c2 python bench.py
