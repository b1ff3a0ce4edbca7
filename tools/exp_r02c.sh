#!/bin/bash
# e2e pipeline: pinned descriptors/results, rotation cost split out
set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
j() { python3 -c "import json;d=json.load(open('$1'));c=d['config'];print(d['value'],d['ms_per_step'],c.get('rotate_ms_per_step'),c.get('pipeline_ms_per_step'))"; }
E="timeout -k 10 300 python -u bench.py --mode e2e --packets 2097152 --steps 4"
$E --keys 1 > $O/e2e_1key.json && echo "e2e 2Mi 1 key: $(j $O/e2e_1key.json)" || exit 1
$E --keys 4096 > $O/e2e_4096.json && echo "e2e 2Mi 4096 keys static: $(j $O/e2e_4096.json)" || exit 1
for pipe in 65536,96,4 262144,384,4 524288,768,4; do
  $E --keys 4096 --rotate --pipe $pipe > $O/e2e_rot_$pipe.json && echo "e2e c5 rotate pipe $pipe: $(j $O/e2e_rot_$pipe.json)" || exit 1
done
