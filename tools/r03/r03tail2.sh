# tail group variants: 1..4 (ab/tail), {1,3,4} (ab/tail13), {3,4} (ab/base) at 1200 B and 300 B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="ab/base.so:0 ab/tail.so:0 ab/tail13.so:0" ROUNDS=3 bash tools/ab.sh r03t2_1200 && \
CFGS="ab/base.so:0 ab/tail.so:0 ab/tail13.so:0" ROUNDS=2 BENCH_ARGS="--pt 300 --packets 4194304" bash tools/ab.sh r03t2_300
