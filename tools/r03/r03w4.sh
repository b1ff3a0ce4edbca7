# A/B: quad kernel at 768 (3 waves/SIMD) vs 1024 threads (4 waves/SIMD, a few spills); AES-256 at 1024 too (w1024b)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="ab/base.so:0 ab/w1024.so:0 ab/w1024d6.so:0" ROUNDS=3 bash tools/ab.sh r03w4 && \
CFGS="ab/base.so:0 ab/w1024b.so:0" ROUNDS=2 BENCH_ARGS="--suite aes256gcm --keys 64" bash tools/ab.sh r03w4b
