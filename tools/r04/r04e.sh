# round 4 step e: same-box A/B -- scalar round keys without the tail-group write deferral (new) vs with it (rkdef) vs
# the round-3 layout (base), 1024 threads with 3 GHASH reads in flight (w3); then HBM traffic of plain vs streaming
# payload stores
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="ab/base.so:base ab/rkdef.so:rkdef s2n-quic_amd/libqpp.so:new ab/w1024g3.so:w3" ROUNDS=3 bash tools/ab.sh r04e_ab && \
LIBS="s2n-quic_amd/libqpp.so ab/plainst.so" bash tools/pmc_ab.sh r04e_pmc
