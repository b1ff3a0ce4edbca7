#!/bin/bash
# does the arena alignment of the payload matter to the lane kernel? (coop chunks straddle 64-B segments at +21)
set -o pipefail
O=gpurun_out/r02f; mkdir -p $O
j() { python3 -c "import json;d=json.load(open('$1'));c=d['config'];print(d['value'],c.get('seal_ms'),c.get('open_ms'))"; }
B="timeout -k 10 200 python -u bench.py --no-cpu --steps 10"
for cfg in "--aad 21" "--aad 21 --stride 1280" "--aad 32" "--aad 32 --stride 1280" "--aad 64 --stride 1280"; do
  $B $cfg > $O/a.json && echo "$cfg: $(j $O/a.json)" || exit 1
done
