# round 4 step g: the BASELINE matrix and the receive / transmit faces on the current build, one box
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04g; mkdir -p $o
run() { local tag=$1; shift; timeout -k 10 240 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 300 $o/$tag.json)"; }
run c3_aes256_64 python bench.py --suite aes256gcm --keys 64 --no-cpu && \
run c3_aes128_64 python bench.py --keys 64 --no-cpu && \
run c3_chacha_64 python bench.py --suite chacha20poly1305 --keys 64 --no-cpu && \
run c4_300 python bench.py --pt 300 --packets 4194304 --no-cpu && \
run c4_600 python bench.py --pt 600 --packets 2097152 --no-cpu && \
run c4_1452 python bench.py --pt 1452 --no-cpu && \
run c4_8000 python bench.py --pt 8000 --packets 131072 --no-cpu && \
run rx_aes128_64 python bench.py --mode rx --keys 64 --no-cpu && \
run rx_aes256_64 python bench.py --mode rx --suite aes256gcm --keys 64 --no-cpu && \
run rx_mixed_64 python bench.py --mode rx --suite mixed --keys 66 --no-cpu && \
run c3_mixed_66 python bench.py --suite mixed --keys 66 --no-cpu && \
run txq1_aes python bench.py --mode txq --inflight 1 --no-cpu && \
run txq1_chacha python bench.py --mode txq --suite chacha20poly1305 --inflight 1 --no-cpu && \
run txq32 python bench.py --mode txq --inflight 32 --coalesce 8 --no-cpu && \
run packet python bench.py --mode packet --no-cpu
