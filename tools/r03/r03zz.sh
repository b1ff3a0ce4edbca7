# end-of-session validation (r03z.sh), then an AES-256 A/B: quad kernel at 512 threads (no spills) vs 768 (spills)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/r03/r03z.sh && \
CFGS="ab/base.so:0 ab/a512.so:0" ROUNDS=2 BENCH_ARGS="--suite aes256gcm --keys 64" bash tools/ab.sh r03a512
