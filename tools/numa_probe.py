#!/usr/bin/env python3
"""Host topology of the GPU box as this process sees it (diagnostic): NUMA
nodes and their CPUs, the CPUs this process may run on, the GPU's PCI address
and NUMA node, and the node of freshly allocated / pinned host pages.  Used to
explain the BaoHasher's process-to-process spread."""
import ctypes
import json
import os
from pathlib import Path


def cpulist(s: str) -> list:
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def nodes() -> dict:
    res = {}
    for d in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        try:
            res[int(d.name[4:])] = cpulist((d / "cpulist").read_text())
        except OSError:
            pass
    return res


def gpu_pci(dev: int = 0) -> str | None:
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return None
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, dev) != 0:
        return None
    return buf.value.decode().lower()


def page_node(addr: int) -> int:
    """NUMA node of the page at addr (move_pages with nodes = NULL)."""
    libc = ctypes.CDLL(None, use_errno=True)
    SYS_move_pages = 279  # x86_64
    pages = (ctypes.c_void_p * 1)(addr & ~4095)
    status = (ctypes.c_int * 1)(-1)
    rc = libc.syscall(SYS_move_pages, 0, 1, pages, None, status, 0)
    return status[0] if rc == 0 else -1000 - ctypes.get_errno()


def main():
    import numpy as np
    nd = nodes()
    aff = sorted(os.sched_getaffinity(0))
    out = {"nodes": {n: f"{c[0]}-{c[-1]} ({len(c)} cpus)" if c else "" for n, c in nd.items()},
           "affinity": aff, "affinity_by_node": {n: len(set(c) & set(aff)) for n, c in nd.items()}}
    a = np.ones(64 << 20, np.uint8)
    out["numpy_page_nodes"] = [page_node(a.ctypes.data + off) for off in range(0, a.size, 8 << 20)]
    import torch
    pci = gpu_pci(0)
    out["gpu0_pci"] = pci
    if pci:
        p = Path("/sys/bus/pci/devices") / pci
        try:
            out["gpu0_numa_node"] = int((p / "numa_node").read_text())
            out["gpu0_local_cpulist"] = (p / "local_cpulist").read_text().strip()
        except OSError as e:
            out["gpu0_sysfs"] = str(e)
    pin = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
    out["torch_pinned_page_nodes"] = [page_node(pin.data_ptr() + off) for off in range(0, pin.numel(), 8 << 20)]
    out["cpu_count"] = os.cpu_count()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
