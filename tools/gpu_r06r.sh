# per-workgroup time spread of the quad kernel (QPP_QUAD_TRACE=2 build): 1 key 1 Mi, 4096 keys 2 Mi
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
o=gpurun_out/r06r; mkdir -p $o
QPP_LIB=$PWD/ab/qtrace2.so timeout -k 10 120 python bench.py --no-cpu --steps 1 --warmup 1 > $o/wg_k1.txt 2>&1 || exit 1
QPP_LIB=$PWD/ab/qtrace2.so timeout -k 10 120 python bench.py --no-cpu --steps 1 --warmup 1 --keys 4096 --packets 2097152 > $o/wg_k4096.txt 2>&1 || exit 1
echo done
