# round 4 step m: same-box A/B of compiler scheduling strategies and pipeline depths on the quad kernel
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="s2n-quic_amd/libqpp.so:new ab/mclause.so:mclause ab/ilp.so:ilp ab/q4d2.so:q4d2 ab/gd12.so:gd12" ROUNDS=3 bash tools/ab.sh r04m_ab
