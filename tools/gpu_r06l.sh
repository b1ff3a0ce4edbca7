# receive-path phase trace (round-6 phase A), many-key quad trace and kernel trace (round 6 items 4-5)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
o=gpurun_out/r06l; mkdir -p $o
QPP_LIB=$PWD/ab/rxtrace2.so timeout -k 10 120 python bench.py --mode rx --steps 2 --warmup 1 --no-cpu > $o/rxtrace1.txt 2>&1 || exit 1
QPP_LIB=$PWD/ab/rxtrace2.so timeout -k 10 120 python bench.py --mode rx --keys 64 --steps 2 --warmup 1 --no-cpu > $o/rxtrace64.txt 2>&1 || exit 1
QPP_LIB=$PWD/ab/qtrace.so timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 --keys 4096 --packets 2097152 > $o/qtrace_k4096.txt 2>&1 || exit 1
QPP_LIB=$PWD/ab/qtrace.so timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 --keys 1 --packets 2097152 > $o/qtrace_k1.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_k4096 -o trace -- python3 bench.py --no-cpu --steps 3 --warmup 1 --keys 4096 --packets 2097152 > $o/tr_k4096.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_rx1 -o trace -- python3 bench.py --no-cpu --steps 3 --warmup 1 --mode rx --keys 1 > $o/tr_rx1.log 2>&1 || exit 1
echo done
