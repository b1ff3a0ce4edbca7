"""The N>1 path with real HIP work per rank: torch.distributed.run starts 2 ranks on the box's one GPU (each its own
qpp context, key-table replica and packet shard, as bench.py under torchrun), every rank's output is checked against
the oracle, and gloo carries only the control plane (no data-path collective)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_shard_and_match_the_oracle():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "_multirank_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=dict(os.environ))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == 2 and res["packets"] == 8192
    assert res["bad"] == 0  # every byte of both shards equals the oracle, opens round-trip
    assert res["first_pn"] == 0 and res["last_pn"] == 8191  # disjoint PN ranges covering the job
