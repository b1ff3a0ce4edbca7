"""Build-time check of the kernel resource remarks (-Rpass-analysis=kernel-resource-usage, one .res file per .hip).

The AES-GCM kernels reserve their LDS (up to the whole 160 KiB) dynamically, so any static LDS the compiler adds (e.g. a private
array it promotes to LDS because of a runtime index) makes every launch fail with an invalid-allocation error; and
the default variants must not touch scratch memory.  usage: python3 check_resources.py *.res"""
import re
import sys

bad = []
for path in sys.argv[1:]:
    name = None
    for line in open(path, errors="replace"):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        if not name:
            continue
        lds = re.search(r"LDS Size \[bytes/block\]: (\d+)", line)
        scr = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        # kernels that address LDS by absolute offset from 0 (dynamic allocation only)
        dyn_lds = any(k in name for k in ("aes_gcm_quad_kernel", "aes_gcm_quad_rx_kernel", "aes_gcm_wave_kernel",
                                          "aes_gcm_burst_kernel", "txq_server_kernel"))
        # the throughput kernels whose hot loops must not spill (AES-128: the headline)
        default = ("aes_gcm_wave_kernel" in name or re.search(r"aes_gcm_quad_kernelILb[01]ELi10E", name)
                   or re.search(r"aes_gcm_quad_rx_kernelILi10E", name))  # (the AES-128-only receive instance)
        if lds and dyn_lds and int(lds.group(1)) != 0:
            bad.append(f"{name}: {lds.group(1)} B of static LDS on top of the dynamic 160 KiB")
        # (a few per-packet spills outside the group loop are tolerated: tools/isa_report.py shows where they are)
        if scr and default and int(scr.group(1)) > 32:
            bad.append(f"{name}: {scr.group(1)} B/lane of scratch")
if bad:
    sys.exit("kernel resource check failed:\n  " + "\n  ".join(bad))
