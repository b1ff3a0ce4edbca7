#!/bin/bash
set -o pipefail
O=gpurun_out/r02g; mkdir -p $O
j() { python3 -c "import json;d=json.load(open('$1'));c=d['config'];print(d['value'],d['ms_per_step'],c.get('rotate_ms_per_step'))"; }
E="timeout -k 10 300 python -u bench.py --mode e2e --steps 4"
$E > $O/e1.json && echo "e2e 1Mi 1 key auto: $(j $O/e1.json)" || exit 1
$E --pipe 65536,96,4 > $O/e2.json && echo "e2e 1Mi 1 key 64Ki: $(j $O/e2.json)" || exit 1
$E --packets 2097152 --keys 4096 --rotate > $O/e3.json && echo "e2e C5 auto: $(j $O/e3.json)" || exit 1
$E --packets 2097152 > $O/e4.json && echo "e2e 2Mi 1 key auto: $(j $O/e4.json)" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_lifetime.py -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; tail -1 $O/pytest.log
