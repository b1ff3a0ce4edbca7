#!/bin/bash
# Same-box A/B of burst-kernel builds over batch sizes: CFGS="ab/x.so ab/y.so" SUITE=aes128gcm bash tools/ab_burst.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/ab_burst
for n in ${SIZES:-64 512 4096 8192}; do
  for lib in $CFGS; do
    QPP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --suite ${SUITE:-aes128gcm} --steps 20 --warmup 3 --no-cpu --packets $n > gpurun_out/ab_burst/o.json 2>gpurun_out/ab_burst/err.txt || { tail -5 gpurun_out/ab_burst/err.txt; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_burst/o.json')); print('n=$n $lib seal_us', round(1e3*d['config']['seal_ms'],1), 'open_us', round(1e3*d['config']['open_ms'],1))"
  done
done
