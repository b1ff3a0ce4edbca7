"""The N>1 path on CPU: two ranks over gloo run the bench's control plane (barrier, max/sum over ranks) and
shard a batch; shards are disjoint, cover the job, and the aggregate throughput formula is weak-scaling."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import multigpu
import qpp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, lr = multigpu.env_rank()
    ctl = multigpu.Control(w)
    sh = multigpu.shard(r, w, 1000, 0x5eed0001)
    descs, arena = qpp.make_batch(sh["count"], 64, [0], seed=sh["seed"], pn_base=sh["pn_base"])
    ctl.barrier()
    t_max = ctl.max(1.0 + r)  # pretend rank r took 1+r seconds
    total = ctl.sum(sh["count"])
    q.put((r, int(descs["pn"][0]), int(descs["pn"][-1]), t_max, total, int(arena[:64].sum())))
    ctl.barrier()
    ctl.close()


@pytest.mark.parametrize("world", [2])
def test_gloo_two_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, a0, b0, t0, n0, s0), (r1, a1, b1, t1, n1, s1) = res
    assert (a0, b0) == (0, 999) and (a1, b1) == (1000, 1999)  # disjoint PN ranges, job covered
    assert t0 == t1 == 2.0  # max over ranks
    assert n0 == n1 == 2000
    assert s0 != s1  # different synthetic data per rank


def test_single_process_control_is_noop():
    ctl = multigpu.Control(1)
    ctl.barrier()
    assert ctl.max(3.5) == 3.5 and ctl.sum(2) == 2.0
    assert multigpu.shard(3, 8, 10, 0)["pn_base"] == 30
