# round 4 step j: phase stamps of the server for 1-packet and 64-packet flushes (trace build ab/sT.so)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04j; mkdir -p $o
export QPP_LIB=ab/sT.so
timeout -k 10 120 python tools/diag/server_trace.py 1 1200 2>&1 | tee $o/trace_1.txt && \
timeout -k 10 120 python tools/diag/server_trace.py 64 1200 2>&1 | tee $o/trace_64.txt && \
timeout -k 10 120 python tools/diag/server_trace.py 1 100 2>&1 | tee $o/trace_1_100.txt
# the 300-B row on each AES kernel
for kern in quad wave; do
  QPP_LIB= QPP_AES_KERNEL=$kern timeout -k 10 120 python bench.py --pt 300 --packets 4194304 --no-cpu > $o/c4_300_$kern.json 2> $o/c4_300_$kern.err || exit 1
  echo "$kern: $(head -c 400 $o/c4_300_$kern.json)"
done
