# round 4 step a: GPU suite on the AesQ4 build, then same-box A/B of seal time (Q4 vs two-table baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04a; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
CFGS="ab/base.so:base s2n-quic_amd/libqpp.so:q4" ROUNDS=3 bash tools/ab.sh r04a_ab
