# round 4 step c: same-box A/B of the quad kernel changes (first AAD block without a product, tail-group write
# deferral) against the previous build (ab/base.so): seal time, then HBM traffic per seal launch
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="ab/base.so:base s2n-quic_amd/libqpp.so:new ab/d2.so:d2" ROUNDS=3 bash tools/ab.sh r04c_ab && \
CFGS="ab/base.so:base s2n-quic_amd/libqpp.so:new" ROUNDS=2 BENCH_ARGS="--pt 300 --packets 4194304" bash tools/ab.sh r04c_ab300 && \
LIBS="ab/base.so s2n-quic_amd/libqpp.so" bash tools/pmc_ab.sh r04c_pmc
