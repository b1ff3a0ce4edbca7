# C4 small packets: quad kernel vs the wave-item kernel (lane per packet, 4-bit GHASH tables)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r03c4; mkdir -p $o
for pt in 300 600; do for kk in lane wave; do
n=$((1258291200 / pt)); n=$(( n > 4194304 ? 4194304 : n ))
QPP_AES_KERNEL=$kk timeout -k 10 200 python bench.py --pt $pt --packets $n --no-cpu > $o/c4_${pt}_$kk.json 2>$o/err.txt || { tail -3 $o/err.txt; exit 1; }
echo "$pt $kk $(python3 -c "import json;d=json.load(open('$o/c4_${pt}_$kk.json'));print(d['value'],d['config']['seal_ms'],d['config']['open_ms'])")"
done; done
