# the round-3 matrix on the final build, one box
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r03final; mkdir -p $o
run() { local tag=$1; shift; timeout -k 10 240 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 330 $o/$tag.json)"; }
run c2 python bench.py --no-cpu && \
run c3_aes256_64 python bench.py --suite aes256gcm --keys 64 --no-cpu && \
run c3_aes128_64 python bench.py --keys 64 --no-cpu && \
run c3_chacha_64 python bench.py --suite chacha20poly1305 --keys 64 --no-cpu && \
run c4_300 python bench.py --pt 300 --packets 4194304 --no-cpu && \
run c4_8000 python bench.py --pt 8000 --packets 131072 --no-cpu && \
run rx_aes128_64 python bench.py --mode rx --keys 64 --no-cpu && \
run c5_e2e python bench.py --mode e2e --keys 4096 --rotate --packets 2097152 --steps 6 --warmup 2 --no-cpu && \
run keys python bench.py --mode keys --keys 4096 --no-cpu && \
run txq1 python bench.py --mode txq --inflight 1 --no-cpu && \
run txq32 python bench.py --mode txq --inflight 32 --coalesce 8 --no-cpu && \
run packet python bench.py --mode packet --no-cpu
