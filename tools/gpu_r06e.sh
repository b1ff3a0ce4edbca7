set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/r06e; mkdir -p $o
export TMPDIR=/tmp
for kp in "4096 2097152" "4096 262144" "1 2097152"; do
  set -- $kp
  QPP_AES_KERNEL=quad QPP_LIB=$PWD/ab/qtrace.so timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 --keys $1 --packets $2 > $o/k$1_n$2.txt 2>&1 || exit 1
  grep "seal 1" $o/k$1_n$2.txt | tail -2
done
