#!/usr/bin/env python3
"""Headline benchmark: GiB/s AEAD seal+open, device-resident, 1200 B packets (BASELINE.json metric).

A "step" = one seal pass (AEAD + 5-byte HP mask, as the TX path does) plus one open pass over one batch of
synthetic packets already resident in HBM.  Default workload = BASELINE.json configs[1]:
AES-128-GCM seal+open, 1 Mi x 1200 B packets, single key, per GPU.
Multi-GPU (torchrun, one process per GPU): every rank seals/opens its own shard (weak scaling, no collective);
gloo on CPU tensors carries only the barrier and the max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--suite aes128gcm|aes256gcm|chacha20poly1305]
                    [--packets N | --total-packets T] [--pt BYTES] [--keys K]
                    [--mode device|e2e|rx|keys|txq|packet] [--rotate] [--pipe CHUNK_PKTS,CHUNK_MIB,SLOTS]

BASELINE configs[4] (C5, key-update churn end to end, strong split):
    python bench.py --mode e2e --keys 4096 --rotate --total-packets 16777216
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "s2n-quic_amd"))
import numpy as np  # noqa: E402

import multigpu  # noqa: E402
import qpp  # noqa: E402

qpp.lib()  # load the engine (and its HIP runtime) before anything else touches the GPU

SUITES = {"aes128gcm": 1, "aes256gcm": 2, "chacha20poly1305": 3, "mixed": 0}  # mixed: key i of suite 1 + i % 3
WARMUP_MIN_S = 0.25  # see the warmup loop in main()
METRIC = "GiB/s AEAD seal+open, device-resident, 1200 B packets at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
GiB = float(1 << 30)


def seal_bytes_per_packet(pt, aad, hp=True):
    # read AAD + PT + descriptor(24); write CT + tag(16) + mask(5)
    return aad + pt + 24 + pt + 16 + (5 if hp else 0)


def open_bytes_per_packet(pt, aad):
    # read AAD + CT + tag + descriptor; write PT + status(1)
    return aad + pt + 16 + 24 + pt + 1


def rx_bytes_per_packet(pt, aad):
    """receive path (qpp_unprotect_open_batch), DESIGN.md §4: read the rx descriptor (24), AAD (the header, aad), CT (pt)
    and tag (16; the HP sample lies inside the CT); write the unprotected first byte + PN bytes (5), the packet
    descriptor the call returns (24), the plaintext (pt) and the status (1) -- 2P + aad + 70 (2491 B at P = 1200)"""
    return 24 + aad + pt + 16 + 5 + 24 + pt + 1


LDS_PEAK_CYCLES = 256 * 2.4e9  # LDS-array cycles per second: one array per CU, 256 CUs at the 2.4 GHz spec clock


def aes_lds_cycles_per_packet(pt, aad, nr, hp=True):
    """LDS-array cycles aes_gcm_quad_kernel spends per packet (MI355X_MICROARCH.md §LDS: ds_read_b32 2 and
    ds_read_b128 4 cycles per wave instruction; a wave instruction serves 64 lanes = 16 packets x 4 lanes, so a lane's
    lookup costs 1/64 of it).  Counter slots: J0 + the payload blocks, in groups of 16 slots (4 per lane), the last
    group 12 or 16 -- 133 T-table lookups per block for AES-128 (CtrPage round caching), 197 for AES-256.  GHASH: one
    8-bit-table product (16 ds_read_b128) per AAD block, ciphertext block and the length block, plus each lane's
    final product by H^e (4-bit tables, 32 ds_read_b128).  HP: one AES over the quad (4 lookups per lane and round)."""
    lookups = 133 if nr == 10 else 197
    m = (pt + 15) // 16
    slots = m + 1  # J0 + payload blocks (the length block rides in a slot of its own only when the group has room)
    groups = -(-(slots + 1) // 16)
    tail = slots + 1 - 16 * (groups - 1)
    ctr = 16 * (groups - 1) + (12 if tail <= 12 else 16)
    ghash = (aad + 15) // 16 + m + 1
    lane_instr_cycles = ctr * lookups * 2 + ghash * 16 * 4 + 4 * 32 * 4 + (4 * 4 * nr * 2 if hp else 0)
    return lane_instr_cycles / 64.0


VALU_PEAK_PER_NS = 540.0  # wave-instructions/ns chip-wide for xor/add/alignbit/bitop3/perm/mul_lo (tools/ubench/issue.hip)


def aes_valu_per_packet(pt, aad, nr):
    """VALU wave-instructions aes_gcm_quad_kernel<seal> issues per packet: per wave-block (64 lane-slots: 16 packets x 4
    lanes) of counter slots as in aes_lds_cycles_per_packet, plus a per-packet part (page build, AAD, HP on the quad,
    final GHASH), calibrated on SQ_INSTS_VALU of the 1 Mi x 1200 B AES-128 seal (round 4, profiles/r04f: 402.7 per
    packet at 76 counter slots); AES-256 scales the AES share (213 of the 322 per wave-block) by 14/10 rounds' lookups."""
    m = (pt + 15) // 16
    slots = m + 1
    groups = -(-(slots + 1) // 16)
    tail = slots + 1 - 16 * (groups - 1)
    ctr = 16 * (groups - 1) + (12 if tail <= 12 else 16)
    per_block = 322.0 if nr == 10 else 322.0 + 213.0 * (197.0 / 133.0 - 1.0)
    return ctr * per_block / 64.0 + 20.3


def chacha_valu_per_packet(pt):
    """VALU wave-instructions chacha_kernel issues per packet: 1386 per 64-byte chunk per wave of 64 packets (20-round
    block, 4 Poly1305 blocks of 26-bit-limb products, staging), from SQ_INSTS_VALU = 4.315e8 per 1 Mi x 1200 B seal
    launch (profiles/r01_prof_c3_chacha_summary.txt: 19 chunks x 1386 x 16384 waves)."""
    return 1386.0 * ((pt + 63) // 64) / 64.0


def _cpu_info():
    """CPU model, CPUs visible, the cgroup's CPU quota, and one CPU per physical core among those allowed."""
    info = {"model": None, "nproc": os.cpu_count(), "cpu_max": None}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cpu_max"] = f"{q} {per}"
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        allowed = list(range(os.cpu_count() or 1))
    cores, seen = [], set()
    for c in allowed:  # first hardware thread of every (package, core)
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            key = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            key = ("?", str(c))
        if key not in seen:
            seen.add(key)
            cores.append(c)
    info["allowed"] = len(allowed)
    info["quota_cpus"] = quota
    info["core_cpus"] = cores
    return info


def cpu_baseline(suite, pt, aad, seconds):
    """The reference's per-packet CPU loop (OpenSSL EVP stand-in for aws-lc) on this host: one pinned thread, then one
    pinned thread per physical core (within the cgroup quota and the box's 16-CPU share), plus the raw one-thread
    AEAD rate over 64 KiB messages that separates the cipher from the per-packet EVP overhead."""
    path = os.path.join(ROOT, "oracle", "libcpubase.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.cpubase_run.restype = ctypes.c_double
    L.cpubase_run.argtypes = [ctypes.c_int] * 6 + [ctypes.c_double, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_int)]
    L.cpubase_bulk_seal.restype = ctypes.c_double
    L.cpubase_bulk_seal.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int]
    L.cpubase_impl.restype = ctypes.c_char_p
    info = _cpu_info()
    cores = info["core_cpus"]
    n_all = min(len(cores), 16, info["quota_cpus"] or len(cores))
    cpus = (ctypes.c_int * max(1, n_all))(*cores[:n_all])
    ok1, okn = ctypes.c_int(), ctypes.c_int()
    one = L.cpubase_run(suite, 1, 4096, pt, aad, 1, seconds, ctypes.byref(ok1), cpus)
    alln = L.cpubase_run(suite, n_all, 4096, pt, aad, 1, seconds, ctypes.byref(okn), cpus)
    bulk = L.cpubase_bulk_seal(suite, 65536, min(seconds, 1.0), cores[0])
    return {
        "value": round(alln, 3), "unit": "GiB/s", "cores": n_all, "kind": "port",
        "one_core": round(one, 3), "bulk_seal_one_core": round(bulk, 3),
        "cpu": {"model": info["model"], "nproc": info["nproc"], "allowed": info["allowed"], "cpu_max": info["cpu_max"]},
        "sample": (f"{L.cpubase_impl().decode()} EVP per-packet seal+HP+open loop (stand-in for aws-lc-rs, which cannot "
                   f"be built offline), 4 Ki x {pt} B packets per thread (BASELINE configs[0] shape), {seconds:.1f} s "
                   f"each: 1 pinned thread = {one:.3f} GiB/s, {n_all} threads pinned one per physical core = "
                   f"{alln:.3f} GiB/s; one thread sealing 64 KiB messages (the cipher alone, no per-packet EVP "
                   f"set-up, no HP, no open) = {bulk:.3f} GiB/s; all tags verified={bool(ok1.value and okn.value)}"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--suite", default="aes128gcm", choices=sorted(SUITES))
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU (weak scaling)")
    ap.add_argument("--total-packets", type=int, default=0,
                    help="fixed total split across the ranks (strong scaling; e.g. BASELINE configs[4]: 16 Mi over 8)")
    ap.add_argument("--rotate", action="store_true",
                    help="e2e: key-update churn (BASELINE configs[4]): every step rotates every key "
                         "(qpp_key_update_batch), frees the old ones and re-points the descriptors, inside the timed "
                         "region")
    ap.add_argument("--pt", type=int, default=1200, help="payload bytes per packet")
    ap.add_argument("--aad", type=int, default=21, help="short header: 0x43 || DCID16 || PN4")
    ap.add_argument("--stride", type=int, default=0, help="device mode: arena bytes per packet (0: 16-B rounded)")
    ap.add_argument("--keys", type=int, default=1)
    ap.add_argument("--key-run", type=int, default=1,
                    help="consecutive packets per key run (1: every packet's key drawn independently; 64: GSO bursts)")
    ap.add_argument("--mode", default="device", choices=["device", "e2e", "rx", "keys", "txq", "packet"],
                    help="device: seal+open in HBM (headline); e2e: pinned host -> HBM -> host; rx: receive path "
                         "(unprotect -> PN expand -> open); keys: device key schedule (key-update churn); "
                         "txq: 64-packet GSO-burst flush latency through the transmit queue; packet: per-packet trait-API "
                         "latency")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--pipe", default="auto",
                    help="e2e: host pipeline geometry 'packets per chunk,MiB per chunk,chunk buffers' (auto: the "
                         "engine's default, chunks sized by batch and key count)")
    ap.add_argument("--inflight", type=int, default=1, help="txq: GSO bursts in flight (qpp_txq_flush_async)")
    ap.add_argument("--coalesce", type=int, default=1, help="txq: bursts sent per launch (qpp_txq_set_coalesce)")
    ap.add_argument("--txq-launch", action="store_true",
                    help="txq --inflight 1: the launched path (qpp_txq_create) instead of the persistent server")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-hp", action="store_true", help="seal without the HP mask (diagnostic)")
    ap.add_argument("--no-check", action="store_true", help="skip the warmup open-status check (diagnostic builds)")
    ap.add_argument("--no-server", action="store_true", help="--mode packet: one launch per call (no packet server)")
    args = ap.parse_args()

    rank, world, local_rank = multigpu.env_rank()
    if args.total_packets:  # strong split: rank r owns [r*T/w, (r+1)*T/w)
        lo, hi = args.total_packets * rank // world, args.total_packets * (rank + 1) // world
        args.packets = hi - lo
        args.pn_first = lo
    else:
        args.pn_first = rank * args.packets
    if args.mode == "e2e":
        return e2e(args, rank, world, local_rank)
    ctl = multigpu.Control(world)  # gloo on CPU tensors: barrier + max over ranks only
    barrier, max_over_ranks = ctl.barrier, ctl.max

    suite = SUITES[args.suite]
    if suite == 0 and args.mode not in ("device", "rx"):
        raise SystemExit("--suite mixed: device and rx modes only")
    # QPP_SHARE_DEVICE=1: every rank on GPU 0 (rehearsing the torchrun path on a one-GPU box; never set by the driver)
    ctx = qpp.Context(0 if os.environ.get("QPP_SHARE_DEVICE") == "1" else local_rank)
    rng = np.random.default_rng(0x5eed0000 + 1)
    key_suites = [suite or 1 + i % 3 for i in range(args.keys)]  # mixed: a server whose clients chose every suite
    keys = [ctx.key(ks, rng.integers(0, 256, qpp.HASH_LEN[ks], dtype=np.uint8).tobytes()) for ks in key_suites]
    n, pt, aad = args.packets, args.pt, args.aad
    if args.mode == "keys":
        return keys_churn(args, ctx, suite, rank, world, barrier, max_over_ranks)
    if args.mode == "txq":
        return txq_bursts(args, ctx, keys, rank, world, max_over_ranks)
    if args.mode == "packet":
        return per_packet(args, ctx, keys, rank, world, max_over_ranks)
    sh = multigpu.shard(rank, world, n, seed_base=0x5eed0000 + 1)
    sh["pn_base"] = args.pn_first
    descs, arena = qpp.make_batch(n, pt, [k.slot for k in keys], seed=sh["seed"], aad_len=aad, pn_base=sh["pn_base"],
                                  run=args.key_run, stride=args.stride or None)
    flags = (0 if args.no_hp else qpp.HP_MASK_OUT) | (qpp.ONLY_CHACHA if suite == 3 else qpp.ONLY_AES if suite else 0)
    d_desc, d_mask, d_status = ctx.alloc(descs.nbytes), ctx.alloc(5 * n), ctx.alloc(n)
    d_desc.upload(descs)
    s = ctx.stream

    if args.mode == "rx":
        return rx(args, ctx, keys, descs, arena, d_desc, d_mask, d_status, flags, rank, world, barrier, max_over_ranks)

    d_arena = ctx.alloc(arena.nbytes)
    d_arena.upload(arena)
    del arena

    def step(ev=None):
        if ev:
            ctx.record(ev[0], s)
        ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, flags, stream=s)
        if ev:
            ctx.record(ev[1], s)
        ctx.open_batch(d_desc, n, d_arena, d_status, flags & ~qpp.HP_MASK_OUT, stream=s)
        if ev:
            ctx.record(ev[2], s)

    for _ in range(args.warmup):
        step()
    ctx.sync(s)
    st = d_status.download(dtype=np.int8)
    if not args.no_check and not (st == 0).all():
        raise SystemExit(f"rank {rank}: {int((st != 0).sum())} packets failed to open during warmup")

    evs = [(ctx.event(), ctx.event(), ctx.event()) for _ in range(args.steps)]
    e0, e1 = ctx.event(), ctx.event()
    # Clock ramp: with the host-side check above between warmup and the timed region, a 5-step run measured 12 %
    # below a 20-step run on the same box (the kernels themselves ran slower, per HIP events: the GPU had idled).
    # So the last untimed steps run right before the barrier, for at least WARMUP_MIN_S, queued without host syncs.
    t_w = time.perf_counter()
    while args.warmup and time.perf_counter() - t_w < WARMUP_MIN_S:
        for _ in range(8):
            step()
        ctx.sync(s)
    barrier()
    ctx.sync(s)
    ctx.record(e0, s)
    for k in range(args.steps):
        step(evs[k])
    ctx.record(e1, s)
    ctx.sync(s)
    barrier()
    t_ms = ctx.elapsed_ms(e0, e1)
    seal_ms = [ctx.elapsed_ms(a, b) for a, b, _ in evs]
    open_ms = [ctx.elapsed_ms(b, c) for _, b, c in evs]
    t_max = max_over_ranks(t_ms)

    payload = 2.0 * (args.total_packets or n * world) * pt * args.steps  # seal + open, all ranks
    # HBM bytes per seal launch from the committed PMC profile of this workload (tools/profile.sh + tools/traffic.py);
    # rocprof counters cannot be read from inside this process
    traffic = None
    try:
        tdb = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
        t = tdb.get(f"{args.suite}/{pt}/{args.keys}")
        if t and n == 1 << 20 and "read_bytes" in t:
            traffic = {"bytes": t["traffic_bytes"],
                       "per_alg": round(t["traffic_bytes"] / (n * seal_bytes_per_packet(pt, aad)), 3),
                       "read": t["read_bytes"], "fetch_size_raw": t["fetch_size_raw_bytes"], "write": t["write_bytes"],
                       "read_per_alg": t["read_per_alg"], "write_per_alg": t["write_per_alg"],
                       "source": "profiles/traffic.json: " + t["source"]}
    except (OSError, ValueError, KeyError):
        traffic = None
    value = payload / (t_max / 1e3) / GiB
    seal_avg = float(np.mean(seal_ms))
    burst_max = qpp.BURST_MAX_DEFAULT >> (2 if suite == 3 else 0)  # batches up to this size run one wave per packet
    achieved = n * seal_bytes_per_packet(pt, aad) / (seal_avg / 1e3) / 1e9
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_max / args.steps, 4), "higher_is_better": True,
            "scaling": "strong" if args.total_packets else "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded PCG64 payload bytes, 21 B short-header AAD, PN = base + i)",
            "config": {
                "workload": (f"{qpp.SUITE_NAMES[suite] if suite else 'mixed-suite'} seal(+HP mask)+open, " +
                             (f"{args.total_packets} x {pt} B packets split over {world} GPU(s), " if args.total_packets
                              else f"{n} x {pt} B packets per GPU, ") + f"{args.keys} key(s)" + (" (BASELINE configs[1])" if suite == 1 and pt == 1200 and
                                                     args.keys == 1 and n == 1 << 20 else "")),
                "suite": args.suite, "packets_per_gpu": n, "payload_bytes": pt, "aad_bytes": aad, "keys": args.keys,
                "hp_mask": True, "parallelism": f"packet shards x{world}, no collective",
                "seal_ms": round(seal_avg, 4), "open_ms": round(float(np.mean(open_ms)), 4),
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic["bytes"] if traffic else None,
                "traffic_detail": traffic,
                "kernel": ("plan + aes_gcm_quad_kernel<seal> + chacha_kernel<seal>" if suite == 0 else
                           "chacha_burst_kernel<seal>" if suite == 3 and n <= burst_max else
                           "chacha_kernel<seal>" if suite == 3 else
                           "aes_gcm_burst_kernel<seal>" if n <= burst_max else
                           "aes_gcm_quad_kernel<seal>" + (" + plan (per seal call)" if args.keys > 1 else "")),
                "bytes_per_packet": seal_bytes_per_packet(pt, aad),
            },
            "cpu_baseline": None,
        }
        if suite == 3 and n > burst_max:
            ins = n * chacha_valu_per_packet(pt)
            out["kernel_roofline"] = {
                "bound": "valu", "achieved": round(ins / (seal_avg / 1e3) / 1e9, 1), "peak": VALU_PEAK_PER_NS,
                "unit": "G wave-instructions/s", "frac": round(ins / (seal_avg / 1e3) / (VALU_PEAK_PER_NS * 1e9), 4),
                "model": "bench.chacha_valu_per_packet (SQ_INSTS_VALU); peak measured by tools/ubench/issue.hip",
            }
        if suite in (1, 2) and n > burst_max and args.keys * qpp.WAVE_KERNEL_PACKETS_PER_KEY <= n:
            # the quad kernel's own bounds: the CU's LDS array (T-table + GHASH-table lookups) and VALU issue, not HBM
            nr = 10 if suite == 1 else 14
            cyc = n * aes_lds_cycles_per_packet(pt, aad, nr)
            ins = n * aes_valu_per_packet(pt, aad, nr)
            out["kernel_roofline"] = {
                "bound": "lds", "achieved": round(cyc / (seal_avg / 1e3) / 1e9, 1), "peak": LDS_PEAK_CYCLES / 1e9,
                "unit": "G LDS-array cycles/s", "frac": round(cyc / (seal_avg / 1e3) / LDS_PEAK_CYCLES, 4),
                "model": "bench.aes_lds_cycles_per_packet (quad layout), checked against SQ_LDS_IDX_ACTIVE; "
                         "peak = 256 CUs x 2.4 GHz" + ("" if args.keys == 1 else
                         "; per-packet work only: the per-key-segment table builds are not in the model"),
                "valu": {"achieved": round(ins / (seal_avg / 1e3) / 1e9, 1), "peak": VALU_PEAK_PER_NS,
                         "unit": "G wave-instructions/s", "frac": round(ins / (seal_avg / 1e3) / (VALU_PEAK_PER_NS * 1e9), 4),
                         "model": "bench.aes_valu_per_packet, calibrated on SQ_INSTS_VALU; peak measured by "
                                  "tools/ubench/issue.hip"},
            }
        if world == 1 and not args.no_cpu and suite:
            out["cpu_baseline"] = cpu_baseline(suite, pt, aad, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    ctx.close()


def _host_batch(ctx, n, pt, aad, conn_of, pn_first, seed):
    """A synthetic host-resident batch for the e2e modes, built without a full-size RNG pass: a 64 MiB random block
    tiled over a pinned arena (packets are [AAD | payload | tag] at a fixed stride), short-header first byte 0x43.
    Returns (pinned arena, descriptors with key_idx = connection id, stride)."""
    stride = ((aad + pt + 16 + 15) // 16) * 16
    host = ctx.host_alloc(n * stride)
    block = qpp.xoshiro_bytes(seed, 64 << 20)
    for o in range(0, host.size, block.size):
        m = min(block.size, host.size - o)
        host[o:o + m] = block[:m]
    host.reshape(n, stride)[:, 0] = 0x43
    # descriptors pinned too: a pageable source or destination makes every chunk's copy synchronous (no overlap)
    descs = ctx.host_alloc(n * qpp.PKT_DTYPE.itemsize).view(qpp.PKT_DTYPE)
    descs[:] = 0
    idx = np.arange(n, dtype=np.uint64)
    descs["pn"] = np.uint64(pn_first) + idx
    descs["off"] = 0  # set per window by the caller
    descs["aad_len"], descs["pt_len"], descs["pn_len"] = aad, pt, 4
    descs["key_idx"] = conn_of(idx)
    return host, descs, stride


def e2e(args, rank, world, local_rank):
    """End to end: packets start and end in pinned host memory (the UDP socket buffer of the reference,
    quic/s2n-quic-platform/src/socket/io/tx.rs:204-268) and go through the engine's own host pipeline
    (qpp_host_batch_submit: chunked H2D -> seal(+HP mask) -> open -> D2H on three streams over a ring of device
    buffers).  With --rotate (BASELINE configs[4]) every step first rotates every key (qpp_key_update_batch, the
    device key schedule), frees the old keys (stream-ordered) and re-points the descriptors: key churn inside the
    timed region."""
    ctl = multigpu.Control(world)
    ctx = qpp.Context(0 if os.environ.get("QPP_SHARE_DEVICE") == "1" else local_rank)
    suite = SUITES[args.suite]
    n, pt, aad = args.packets, args.pt, args.aad
    rng = np.random.default_rng(0x5eed0000 + 5)
    hl = qpp.HASH_LEN[suite]
    secrets = [rng.integers(0, 256, hl, dtype=np.uint8).tobytes() for _ in range(args.keys)]
    keys = ctx.keys_batch(suite, secrets, 1) if args.keys > 1 else [ctx.key(suite, secrets[0])]
    nk = len(keys)

    def conn_of(idx):  # packet -> connection (key) id, splitmix-spread like qpp.make_batch
        z = (idx + np.uint64(0x9E3779B97F4A7C15)) * np.uint64(1)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return ((z ^ (z >> np.uint64(31))) % np.uint64(nk)).astype(np.uint32)

    if args.pipe != "auto":
        cp, cmib, cs = (int(x) for x in args.pipe.split(","))
        ctx.set_host_pipe(cp, cmib << 20, cs)
    host, descs, stride = _host_batch(ctx, n, pt, aad, conn_of, args.pn_first, 0x5eed0000 + 7919 * rank)
    # one submit addresses a 4 GiB window of the arena (qpp_pkt.off is 32-bit): split larger shards into windows
    per_win = max(1, ((1 << 32) - stride) // stride)
    wins = []
    for lo in range(0, n, per_win):
        hi = min(n, lo + per_win)
        d = descs[lo:hi]
        d["off"] = (np.arange(hi - lo, dtype=np.uint64) * np.uint64(stride)).astype(np.uint32)
        wins.append((lo, hi, host[lo * stride:hi * stride]))
    masks = ctx.host_alloc(5 * n)  # pinned (see _host_batch)
    status = ctx.host_alloc(n).view(np.int8)
    status[:] = 0
    # descriptors name connections (QPP_KEY_BY_CONN): the device resolves each through the connection -> key table,
    # as the transport's packets name its connection's KeySet (keyset.rs), not a key generation
    flags = qpp.HP_MASK_OUT | qpp.KEY_BY_CONN | (qpp.ONLY_CHACHA if suite == 3 else qpp.ONLY_AES)
    slots = np.array([k.slot for k in keys], dtype=np.uint32)
    ctx.set_conn_keys(slots)

    phase = {"rotate": 0.0, "pipeline": 0.0}

    # The rotation runs in C (tools/txqdrive.c rotate_keys: update_batch, slot_batch, free_batch, set_conn_keys over
    # raw handles, as the transport calls the ABI) when the helper is built; else through the Python wrappers
    rot = None
    if args.rotate and os.path.exists(os.path.join(ROOT, "tools", "libtxqdrive.so")):
        rot = ctypes.CDLL(os.path.join(ROOT, "tools", "libtxqdrive.so")).rotate_keys
        rot.restype = ctypes.c_int
        rot.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        handles = np.array([k.handle for k in keys], dtype=np.uint64)
        for k in keys:
            k.handle = None  # (owned by `handles` from here on)

    def step():
        nonlocal keys, slots
        t0 = time.perf_counter()
        if rot is not None:
            if rot(ctx.handle, handles.ctypes.data, len(handles), slots.ctypes.data) != 0:
                raise SystemExit("rotate_keys failed")
        elif args.rotate:
            new = ctx.update_keys(keys, slots_out=slots)  # the new slots in one call
            ctx.free_keys(keys)
            keys = new
            ctx.set_conn_keys(slots)  # every connection's entry now holds its new key
        t1 = time.perf_counter()
        tickets = [ctx.host_submit(descs[lo:hi], arena, masks[5 * lo:5 * hi], status[lo:hi], flags,
                                   qpp.OP_SEAL | qpp.OP_OPEN) for lo, hi, arena in wins]
        for t in tickets:
            ctx.host_wait(t)
        phase["rotate"] += t1 - t0
        phase["pipeline"] += time.perf_counter() - t1

    for _ in range(args.warmup):
        step()
    ctl.barrier()
    phase.update(rotate=0.0, pipeline=0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t = time.perf_counter() - t0
    ctl.barrier()
    t = ctl.max(t)
    # checks: every open verified; a sample of payloads is the plaintext again (seal -> open round trip)
    assert (status == 0).all(), f"rank {rank}: {int((status != 0).sum())} packets failed to open"
    block = qpp.xoshiro_bytes(0x5eed0000 + 7919 * rank, 64 << 20)
    for i in np.random.default_rng(3).choice(n, min(n, 2000), replace=False):
        o = int(i) * stride
        want = np.array([block[(o + j) % block.size] for j in range(aad + 0, aad + 64)], np.uint8)
        assert (host[o + aad:o + aad + 64] == want).all(), f"rank {rank}: packet {i} did not round-trip"
    total = args.total_packets or n * world
    if rank == 0:
        wl = (f"{qpp.SUITE_NAMES[suite]} seal(+HP mask)+open end to end (pinned host -> HBM -> pinned host, "
              f"qpp_host_batch_submit), {total} x {pt} B packets " +
              (f"split over {world} GPU(s)" if args.total_packets else f"per GPU x {world}") +
              f", {nk} key(s)" + (", every key rotated every step (update + free inside the timed region)"
                                   if args.rotate else ""))
        if args.rotate and nk == 4096 and args.total_packets == 16 << 20:
            wl += " (BASELINE configs[4])"
        print(json.dumps({
            "metric": "GiB/s AEAD seal+open end-to-end (pinned host -> HBM -> pinned host), 1200 B packets",
            "value": round(2.0 * total * pt * args.steps / t / GiB, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * t / args.steps, 3),
            "higher_is_better": True, "scaling": "strong" if args.total_packets else "weak", "dtype": "u8",
            "data": "synthetic (a 64 MiB PCG64 block tiled over the arena)",
            "config": {"workload": wl, "suite": args.suite, "packets_per_gpu": n, "keys": nk, "rotate": args.rotate,
                       "h2d_d2h_bytes_per_step_per_gpu": 2 * n * stride, "windows": len(wins),
                       "pipe": args.pipe, "rotate_ms_per_step": round(1e3 * phase["rotate"] / args.steps, 3),
                       "pipeline_ms_per_step": round(1e3 * phase["pipeline"] / args.steps, 3)},
        }), flush=True)
    for k in keys:
        k.free()
    if rot is not None:
        lib = qpp.lib()
        for h in handles:
            lib.qpp_key_free(ctypes.c_void_p(int(h)))
    ctx.host_free(host)
    ctx.close()


def rx(args, ctx, keys, descs, arena, d_desc, d_mask, d_status, flags, rank, world, barrier, max_over_ranks):
    """Receive path: a GRO batch of protected packets (sealed + header-protected on the device
    first) -> qpp_unprotect_open_batch: HP removal, PN expansion against largest_pn, key choice by key phase, open.
    Each step restores the protected arena (device copy, excluded from the timed kernel events) and opens it."""
    n, pt, aad = args.packets, args.pt, args.aad
    stride = arena.size // n
    # the header's 4 PN bytes carry the packet number (truncated against largest_pn = pn - 1)
    pnb = (descs["pn"] & np.uint64(0xffffffff)).astype(">u4").view(np.uint8).reshape(n, 4)
    arena.reshape(n, stride)[:, aad - 4:aad] = pnb
    d_arena, d_prot = ctx.alloc(arena.nbytes), ctx.alloc(arena.nbytes)
    d_arena.upload(arena)
    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, flags | qpp.HP_APPLY)
    ctx.sync()
    lib = qpp.lib()
    rxd = np.zeros(n, dtype=qpp.RX_DTYPE)
    rxd["largest_pn"] = np.maximum(descs["pn"], np.uint64(1)) - np.uint64(1)
    rxd["key_idx"][:, 0] = descs["key_idx"]
    rxd["key_idx"][:, 1] = descs["key_idx"]
    rxd["off"] = descs["off"]
    rxd["header_len"] = aad - descs["pn_len"]
    rxd["len"] = aad + pt + 16
    d_rx, d_out = ctx.alloc(rxd.nbytes), ctx.alloc(n * qpp.PKT_DTYPE.itemsize)
    d_rx.upload(rxd)
    s = ctx.stream

    def hip_d2d(dst, src):
        ctx._check(lib.qpp_memcpy_d2d(ctx.handle, dst.ptr, src.ptr, arena.nbytes, s), "d2d")

    hip_d2d(d_prot, d_arena)  # keep the protected image
    # every step restores the protected image (device copy) and runs the receive path, back to back on one stream
    # with no host sync in between (as the device-mode bench does): the HIP events around the receive launches time
    # them alone, and the GPU never idles between steps
    evs = [(ctx.event(), ctx.event()) for _ in range(args.warmup + args.steps)]
    for e0, e1 in evs:
        hip_d2d(d_arena, d_prot)
        ctx.record(e0, s)
        ctx.unprotect_open_batch(d_rx, n, d_arena, d_out, d_status, flags & ~qpp.HP_MASK_OUT, stream=s)
        ctx.record(e1, s)
    ctx.sync(s)
    ms = [ctx.elapsed_ms(e0, e1) for e0, e1 in evs[args.warmup:]]
    st = d_status.download(dtype=np.int8)
    assert (st == 0).all(), f"{int((st != 0).sum())} packets failed to open"
    t = max_over_ranks(float(np.mean(ms)))
    if rank == 0:
        out = {
            "metric": "GiB/s receive path (unprotect -> PN expand -> open), device-resident, 1200 B packets",
            "value": round(n * pt * world / (t / 1e3) / GiB, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "ms_per_step": round(t, 4), "suite": args.suite, "packets_per_gpu": n, "keys": args.keys,
        }
        suite = SUITES[args.suite]
        achieved = n * rx_bytes_per_packet(pt, aad) / (t / 1e3) / 1e9
        traffic = None  # HBM bytes per receive launch from the committed PMC profile (tools/traffic.py rx: key)
        try:
            tr = json.load(open(os.path.join(ROOT, "profiles", "traffic.json"))).get(f"rx:{args.suite}/{pt}/{args.keys}")
            if tr and n == 1 << 20 and aad == 21:
                traffic = {"bytes": tr["traffic_bytes"], "per_alg": round(tr["traffic_bytes"] / (n * rx_bytes_per_packet(pt, aad)), 3),
                           "read_per_alg": tr["read_per_alg"], "write_per_alg": tr["write_per_alg"],
                           "source": "profiles/traffic.json: " + tr["source"]}
        except (OSError, ValueError, KeyError):
            traffic = None
        out["roofline"] = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic and traffic["bytes"],
            "traffic_detail": traffic,
            "kernel": "aes_gcm_quad_rx_kernel (one launch: unprotect, group-by key, open)" if suite in (1, 2) else
                      "chacha_kernel<open, RX>" if suite == 3 else "aes_gcm_quad_rx_kernel + chacha_kernel<open, RX>",
            "bytes_per_packet": rx_bytes_per_packet(pt, aad),
        }
        if suite in (1, 2):
            # the open phase is the quad kernel's work (E_K(J0) on the quad in place of the HP mask); the unprotect
            # phase adds one lane-per-packet AES of the sample (16 lookups per round, 2 LDS cycles per wave instruction)
            nr = 10 if suite == 1 else 14
            cyc = n * (aes_lds_cycles_per_packet(pt, aad, nr) + 16 * nr * 2 / 64.0)
            out["kernel_roofline"] = {
                "bound": "lds", "achieved": round(cyc / (t / 1e3) / 1e9, 1), "peak": LDS_PEAK_CYCLES / 1e9,
                "unit": "G LDS-array cycles/s", "frac": round(cyc / (t / 1e3) / LDS_PEAK_CYCLES, 4),
                "model": "bench.aes_lds_cycles_per_packet (quad open) + the unprotect phase's sample AES; "
                         "peak = 256 CUs x 2.4 GHz; checked against SQ_LDS_IDX_ACTIVE (profiles/r06/rx)",
            }
        print(json.dumps(out), flush=True)
    ctx.close()


def keys_churn(args, ctx, suite, rank, world, barrier, max_over_ranks):
    """Device key schedule (BASELINE configs[4] key churn): qpp_key_new_batch derives
    args.keys keys per step (1 "quic ku" update each) -- HKDF, AES expansion and GHASH powers on the GPU."""
    rng = np.random.default_rng(0x5eed0000 + 5)
    hl = qpp.HASH_LEN[suite]
    secrets = [rng.integers(0, 256, hl, dtype=np.uint8).tobytes() for _ in range(args.keys)]
    times = []
    for k in range(args.warmup + args.steps):
        t0 = time.perf_counter()
        ks = ctx.keys_batch(suite, secrets, 1)
        t = time.perf_counter() - t0
        for key in ks:
            key.free()
        if k >= args.warmup:
            times.append(t)
    t = max_over_ranks(float(np.mean(times)))
    if rank == 0:
        print(json.dumps({
            "metric": "keys/s installed (secret -> quic ku -> key/iv/hp -> AES schedule + GHASH powers), host wall",
            "value": round(args.keys * world / t, 1), "unit": "keys/s", "n_gpus": world, "steps": args.steps,
            "ms_per_step": round(1e3 * t, 3), "suite": args.suite, "keys_per_step": args.keys,
        }), flush=True)
    ctx.close()


def txq_bursts(args, ctx, keys, rank, world, max_over_ranks, burst=64):
    """GSO-style bursts (BASELINE configs[3]): the transport encodes `burst` packets into the pinned ring and flushes
    (bursts <= 256 packets are sealed in place on the pinned ring by the wave-per-packet kernels).  --inflight 1: each
    flush waits (qpp_txq_flush), the per-flush latency is reported; --inflight K > 1: qpp_txq_flush_async with up to K
    bursts in flight (each in its own ring region, re-encoded only once its ticket completes), and the sustained
    burst rate is reported."""
    pt, aad = args.pt, args.aad
    stride = ((aad + pt + 16 + 15) // 16) * 16
    K = max(1, args.inflight)
    C = max(1, min(args.coalesce, K))
    # one flush in flight: the persistent server queue (a doorbell instead of a launch per flush) unless --txq-launch
    persistent = K == 1 and not args.txq_launch
    q = (qpp.TxQueue(ctx, K * burst * stride, burst, persistent=True) if persistent else
         qpp.TxQueue(ctx, K * burst * stride, burst * C, in_flight=max(1, K // C)))
    q.set_coalesce(C)
    rng = np.random.default_rng(9)
    q.ring[:] = rng.integers(0, 256, q.ring.size, dtype=np.uint8)
    drive = None
    if K > 1 and os.path.exists(os.path.join(ROOT, "tools", "libtxqdrive.so")):
        drive = ctypes.CDLL(os.path.join(ROOT, "tools", "libtxqdrive.so")).txq_drive
        drive.restype = ctypes.c_double
        drive.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_size_t] * 4 + [ctypes.c_uint64]
    lat, tickets, srv_us = [], [0] * K, []
    pn = 1 << 20
    proto = np.zeros(burst, dtype=qpp.PKT_DTYPE)  # one burst: packet i at i * stride, short header + 4-byte PN
    proto["key_idx"] = [keys[i % len(keys)].slot for i in range(burst)]
    proto["off"] = np.arange(burst) * stride
    proto["aad_len"], proto["pt_len"], proto["pn_len"] = aad, pt, 4
    total = args.warmup + args.steps * 20
    t_start = None
    if K == 1 and os.path.exists(os.path.join(ROOT, "tools", "libtxqdrive.so")):
        # one flush at a time, timed around qpp_txq_flush in C (tools/txqdrive.c txq_latency): the engine's latency,
        # not Python's per-call cost
        lat_fn = ctypes.CDLL(os.path.join(ROOT, "tools", "libtxqdrive.so")).txq_latency
        lat_fn.restype = ctypes.c_int
        lat_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                           ctypes.c_void_p]
        buf = np.zeros(total, dtype=np.float64)
        if lat_fn(q.handle, proto.ctypes.data, burst, total, pn, buf.ctypes.data) != 0:
            raise SystemExit("txq_latency failed")
        lat = list(buf[args.warmup:] * 1e-6)
        wall = max_over_ranks(float(np.sum(buf[args.warmup:])) * 1e-6)
        n_timed = total - args.warmup
        if rank == 0:
            print(json.dumps({
                "metric": f"txq {burst}-packet GSO bursts of {pt} B (sealed + HP in place on the pinned ring), 1 in "
                          f"flight, flush latency median", "unit": "us", "n_gpus": world, "suite": args.suite,
                "bursts": n_timed, "value": round(1e6 * max_over_ranks(float(np.median(lat))), 1),
                "higher_is_better": False, "p10_us": round(1e6 * float(np.percentile(lat, 10)), 1),
                "p90_us": round(1e6 * float(np.percentile(lat, 90)), 1),
                "burst_gib_s": round(n_timed * burst * pt * world / wall / GiB, 3),
                "path": "persistent server (qpp_txq_create_persistent)" if persistent else "launched kernels",
                "driver": "tools/txqdrive.c txq_latency (qpp_txq_flush timed in C)",
                "flushes_served_launched_starts": list(q.info())}), flush=True)
        q.close()
        ctx.close()
        return
    if drive is not None:  # the transport's loop in C (tools/txqdrive.c): the engine, not Python, is measured
        drive(q.handle, proto.ctypes.data, burst, burst * stride, K, max(K, args.warmup * 4), 1 << 40)
        wall = drive(q.handle, proto.ctypes.data, burst, burst * stride, K, args.steps * 20, 1 << 41)
        if wall < 0:
            raise SystemExit(f"txq_drive failed ({wall})")
        wall = max_over_ranks(wall)
        n_timed = args.steps * 20
        rate = n_timed * burst * pt * world / wall / GiB
        if rank == 0:
            print(json.dumps({
                "metric": f"txq {burst}-packet GSO bursts of {pt} B (sealed + HP in place on the pinned ring), "
                          f"{K} in flight, sent {C} per launch", "value": round(rate, 3), "unit": "GiB/s",
                "higher_is_better": True, "n_gpus": world, "suite": args.suite, "bursts": n_timed,
                "us_per_burst": round(1e6 * wall / n_timed, 2), "driver": "tools/txqdrive.c (native push/flush loop)",
            }), flush=True)
        q.close()
        ctx.close()
        return
    for k in range(total):
        if k == args.warmup:
            for t in tickets:
                q.wait(t)
            t_start = time.perf_counter()
        r = k % K
        q.wait(tickets[r])  # the region's previous burst is out of the engine's hands
        base = r * burst * stride
        # the transport's per-packet pushes, as one call (a Python call per packet would be the bottleneck here)
        d = proto.copy()
        d["pn"] = pn + np.arange(burst, dtype=np.uint64)
        d["off"] += base
        q.push_descs(d)
        pn += burst
        t0 = time.perf_counter()
        if K == 1:
            q.flush()
            if k >= args.warmup:
                lat.append(time.perf_counter() - t0)
                if persistent:
                    srv_us.append(q.server_time_us())
        else:
            tickets[r] = q.flush_async()
    for t in tickets:
        q.wait(t)
    wall = max_over_ranks(time.perf_counter() - t_start)
    n_timed = total - args.warmup
    rate = n_timed * burst * pt * world / wall / GiB
    if rank == 0:
        line = {"metric": f"txq {burst}-packet GSO bursts of {pt} B (sealed + HP in place on the pinned ring), "
                          f"{K} in flight, sent {C} per launch", "unit": "GiB/s" if K > 1 else "us", "n_gpus": world, "suite": args.suite,
                "bursts": n_timed, "burst_gib_s": round(rate, 3), "us_per_burst": round(1e6 * wall / n_timed, 2)}
        if K == 1:
            line.update(value=round(1e6 * max_over_ranks(float(np.median(lat))), 1), higher_is_better=False,
                        metric=line["metric"] + ", flush latency median",
                        p90_us=round(1e6 * float(np.percentile(lat, 90)), 1),
                        path="persistent server (qpp_txq_create_persistent)" if persistent else "launched kernels",
                        flushes_served_launched_starts=list(q.info()))
            if srv_us:  # the server's own share: doorbell seen -> completion word written (s_memrealtime)
                line["server_us_median"] = round(float(np.median(srv_us)), 2)
        else:
            line.update(value=round(rate, 3), higher_is_better=True)
        print(json.dumps(line), flush=True)
    q.close()
    ctx.close()


def per_packet(args, ctx, keys, rank, world, max_over_ranks, calls=2000):
    """The trait-shaped per-packet face (Key::encrypt -> qpp_seal, Key::decrypt -> qpp_open): one packet per call,
    as quic/s2n-quic-transport calls it today.  Reports the median call latency, timed around each call in C
    (tools/txqdrive.c packet_latency), through the context's packet server (qpp_ctx_set_packet_server; --no-server:
    one launch per call)."""
    rng = np.random.default_rng(10)
    hdr = bytes([0x43]) + bytes(args.aad - 1)
    pt = rng.integers(0, 256, args.pt, dtype=np.uint8).tobytes()
    k = keys[0]
    if args.no_server:
        ctx.set_packet_server(False)
    drv = ctypes.CDLL(os.path.join(ROOT, "tools", "libtxqdrive.so")).packet_latency
    drv.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                    ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    n = args.warmup + calls
    ts, to, tm = np.zeros(n), np.zeros(n), np.zeros(n)
    rc = drv(k.handle, hdr, len(hdr), pt, len(pt), n, 0, ts.ctypes.data, to.ctypes.data, tm.ctypes.data)
    if rc:
        raise SystemExit(f"per-packet driver failed: {rc}")
    ts, to, tm = ts[args.warmup:], to[args.warmup:], tm[args.warmup:]
    t = max_over_ranks(float(np.median(ts)) * 1e-6)
    calls_srv, starts = ctx.packet_server_info()
    if rank == 0:
        print(json.dumps({
            "metric": f"per-packet Key::encrypt latency ({args.pt} B, qpp_seal), median", "value": round(1e6 * t, 2),
            "unit": "us", "higher_is_better": False, "n_gpus": world, "suite": args.suite,
            "p10_us": round(float(np.percentile(ts, 10)), 2), "p90_us": round(float(np.percentile(ts, 90)), 2),
            "decrypt_us": round(float(np.median(to)), 2), "decrypt_p90_us": round(float(np.percentile(to, 90)), 2),
            "hp_mask_us": round(float(np.median(tm)), 2),
            "calls": calls, "path": "launch per call" if args.no_server else "packet server",
            "server_calls_starts": [calls_srv, starts], "driver": "tools/txqdrive.c packet_latency (timed in C)",
        }), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
