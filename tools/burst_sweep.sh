#!/bin/bash
# Wave-per-packet (burst) vs lane-per-packet kernels across batch sizes; txq flush latency.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
out=gpurun_out/burst_sweep; mkdir -p $out
for su in ${SUITES:-aes128gcm chacha20poly1305}; do
  for n in ${SIZES:-64 512 4096 16384 65536}; do
    for bm in 0 1000000000; do
      QPP_BURST_MAX=$bm timeout -k 10 120 python bench.py --suite $su --steps 10 --warmup 3 --no-cpu --packets $n > $out/${su}_n${n}_b${bm}.json 2>$out/err.txt || { tail -5 $out/err.txt; exit 1; }
      python -c "import json;d=json.load(open('$out/${su}_n${n}_b${bm}.json'));c=d['config'];print('$su n=$n burst_max=$bm', d['value'], 'GiB/s seal_ms', c['seal_ms'], 'open_ms', c['open_ms'])"
    done
  done
done
for su in aes128gcm aes256gcm chacha20poly1305; do
  timeout -k 10 120 python bench.py --mode txq --suite $su --no-cpu > $out/txq_$su.json 2>$out/err.txt || { tail -5 $out/err.txt; exit 1; }
  cat $out/txq_$su.json
done
