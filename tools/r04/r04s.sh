# round 4 step s: same-box comparison of the GHASH product's reads in flight in the wave-per-packet code (8 with
# schedule barriers = current, 12, and both without the barriers), by the server's phase trace (trace builds)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04s; mkdir -p $o
for r in 1 2; do
  for lib in sT sT_d12 sT_d8f sT_d12f; do
    QPP_LIB=ab/$lib.so timeout -k 10 120 python tools/diag/server_trace.py 1 1200 > $o/${lib}_1_r$r.txt 2>&1 || exit 1
    QPP_LIB=ab/$lib.so timeout -k 10 120 python tools/diag/server_trace.py 64 8000 > $o/${lib}_64x8000_r$r.txt 2>&1 || exit 1
    echo "$r $lib | $(cut -c1-140 $o/${lib}_1_r$r.txt) | $(cut -c1-100 $o/${lib}_64x8000_r$r.txt)"
  done
done
