# round 4 step d: same-box A/B -- round keys loaded per round (rk, 768 threads: 0 spills) and 4 waves per SIMD
# (1024 threads; GHASH reads in flight 3 / 6, with the spills that remain) against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="ab/base.so:base ab/prev.so:prev s2n-quic_amd/libqpp.so:rk ab/w1024g3.so:w3 ab/w1024g6.so:w6 " ROUNDS=3 bash tools/ab.sh r04d_ab && \
LIBS="ab/base.so s2n-quic_amd/libqpp.so" bash tools/pmc_ab.sh r04d_pmc
