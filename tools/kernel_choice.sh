# lane vs wave-item AES kernel by key count (1 Mi x 1200 B, AES-128-GCM): the crossover for kWaveKernelPacketsPerKey
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/kc
for k in 16 64 256 512 1024 2048; do
  for kern in lane wave; do
    QPP_AES_KERNEL=$kern timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu --keys $k > gpurun_out/kc/${k}_$kern.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/kc/${k}_$kern.json')); print('keys $k $kern', d['value'], d['config']['seal_ms'], d['config']['open_ms'])"
  done
done
