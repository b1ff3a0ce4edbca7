# round 4 step h: validation of the server-priority build (r04f: full GPU suite incl. TX+RX after the txq server
# tests, smoke, bench, rx trace exit status, PMC profile), then the same-box A/B of the interior payload prefetch
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/r04/r04f.sh && \
CFGS="s2n-quic_amd/libqpp.so:new ab/pf.so:pf ab/base.so:base" ROUNDS=3 bash tools/ab.sh r04h_ab
