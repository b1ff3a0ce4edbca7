"""One rank of tests/test_gpu_multirank.py (launched by torch.distributed.run): its own qpp context (key-table
replica) on the shared GPU, its own packet shard (multigpu.shard), sealed and opened on the GPU, every packet checked
against the oracle; mismatch counts and PN ranges are summed / gathered over gloo, rank 0 prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "s2n-quic_amd"))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402

import _oracle as orc  # noqa: E402
import multigpu  # noqa: E402
import qpp  # noqa: E402


def main():
    rank, world, _ = multigpu.env_rank()
    ctl = multigpu.Control(world)
    n, pt = 4096, 300
    with qpp.Context(0) as ctx:  # every rank on GPU 0: the box has one
        secrets = [(s, bytes((7 * s + i) & 0xff for i in range(qpp.HASH_LEN[s]))) for s in (1, 2, 3)]
        keys = [ctx.key(s, sec) for s, sec in secrets]
        sh = multigpu.shard(rank, world, n, seed_base=0x5eed0100)
        descs, arena = qpp.make_batch(n, pt, [k.slot for k in keys], seed=sh["seed"], pn_base=sh["pn_base"])
        d_desc, d_arena, d_mask, d_st = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)
        d_desc.upload(descs)
        d_arena.upload(arena)
        ctx.seal_batch(d_desc, n, d_arena, d_mask, d_st, qpp.HP_MASK_OUT)
        got, masks = d_arena.download(), d_mask.download()
        okeys = orc.make_keys([(k.suite, *k.material()) for k in keys])
        od = descs.copy()
        od["key_idx"] = [[k.slot for k in keys].index(int(s)) for s in descs["key_idx"]]
        want = arena.copy()
        want_masks = orc.seal_batch(okeys, od, want, qpp.HP_MASK_OUT)
        bad = int((got != want).sum()) + int(masks.tobytes() != want_masks)
        ctx.open_batch(d_desc, n, d_arena, d_st)
        stride = arena.size // n
        v, a = d_arena.download().reshape(n, stride), arena.reshape(n, stride)
        bad += int((v[:, 21:21 + pt] != a[:, 21:21 + pt]).sum()) + int((d_st.download(dtype=np.int8) != 0).sum())
        for b in (d_desc, d_arena, d_mask, d_st):
            b.free()
        for k in keys:
            k.free()
    ctl.barrier()
    total_bad = ctl.sum(bad)
    lo = ctl.sum(int(descs["pn"][0]) if rank == 0 else 0)
    hi = ctl.sum(int(descs["pn"][-1]) if rank == world - 1 else 0)
    packets = ctl.sum(n)
    if rank == 0:
        print(json.dumps({"world": world, "bad": total_bad, "first_pn": lo, "last_pn": hi, "packets": packets}),
              flush=True)
    ctl.close()


if __name__ == "__main__":
    main()
