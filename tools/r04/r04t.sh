# round 4 step t: reads two pass pairs ahead in the wave-per-packet AES (sT_pf2) vs one (sT), server phase trace
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04t; mkdir -p $o
for r in 1 2; do
  for lib in sT sT_pf2; do
    for cfg in "1 1200" "64 8000" "64 1200"; do
      t=$(echo $cfg | tr ' ' x)
      QPP_LIB=ab/$lib.so timeout -k 10 120 python tools/diag/server_trace.py $cfg > $o/${lib}_${t}_r$r.txt 2>&1 || exit 1
      echo "$r $lib $(cut -c1-150 $o/${lib}_${t}_r$r.txt)"
    done
  done
done
