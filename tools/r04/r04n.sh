# round 4 step n: the GSO-burst (txq) sweep on the server path at BASELINE configs[3]'s sizes, one flush in flight and
# 32 in flight, and the per-packet faces with the HP mask
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04n; mkdir -p $o
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 330 $o/$tag.json)"; }
for pt in 300 1200 1452 8000; do
  run txq1_$pt python bench.py --mode txq --inflight 1 --pt $pt --no-cpu || exit 1
  run txq32_$pt python bench.py --mode txq --inflight 32 --coalesce 8 --pt $pt --no-cpu || exit 1
done
run packet_aes python bench.py --mode packet --no-cpu && \
run packet_chacha python bench.py --mode packet --suite chacha20poly1305 --no-cpu
