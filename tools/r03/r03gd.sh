# A/B: GHASH product with 6 / 9 (default) / 12 LDS reads in flight in the quad kernel
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="ab/base.so:0 ab/gd6.so:0 ab/gd12.so:0" ROUNDS=3 bash tools/ab.sh r03gd
