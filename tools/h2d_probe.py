#!/usr/bin/env python3
"""H2D copy rate from pinned host memory by transfer size (diagnostic for
the BaoHasher line): 1 GiB moved as back-to-back hipMemcpyAsync calls of
one size on one stream, the way the library's staging ring issues them, and
the same through the library's own staged path (pageable source)."""
import ctypes
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    dev = torch.device("cuda", 0)
    total = 1 << 30
    src = torch.empty(total, dtype=torch.uint8).pin_memory()
    src.random_(0, 256)
    dst = torch.empty(total, dtype=torch.uint8, device=dev)
    dst2 = torch.empty(total, dtype=torch.uint8, device=dev)
    out = {}
    for mib in (1, 2, 4, 8, 16, 64, 256):
        piece = mib << 20
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for off in range(0, total, piece):
                dst[off:off + piece].copy_(src[off:off + piece], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        out[f"pinned_{mib}MiB_GBps"] = round(total / best / 1e9, 2)
    # both directions at once (encode() E2E moves ~18 MB each way per object):
    # H2D on one stream, D2H on another, 16 MiB pieces, pinned both sides
    back = torch.empty(total, dtype=torch.uint8).pin_memory()
    s_up, s_down = torch.cuda.Stream(), torch.cuda.Stream()
    piece = 16 << 20
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for off in range(0, total, piece):
            with torch.cuda.stream(s_up):
                dst[off:off + piece].copy_(src[off:off + piece], non_blocking=True)
            with torch.cuda.stream(s_down):
                back[off:off + piece].copy_(dst2[off:off + piece], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    out["duplex_16MiB_each_way_GBps"] = round(total / best / 1e9, 2)
    out["duplex_16MiB_total_GBps"] = round(2 * total / best / 1e9, 2)
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for off in range(0, total, piece):
            back[off:off + piece].copy_(dst2[off:off + piece], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    out["d2h_16MiB_GBps"] = round(total / best / 1e9, 2)
    # the library's staged path: a pageable source through the pinned ring (4 MiB pieces)
    from carbonado_amd.utils import BaoHasher
    import numpy as np
    host = src.numpy().copy()  # pageable
    for piece_mib in (4, 16, 64):
        piece = piece_mib << 20
        best = 1e9
        for _ in range(3):
            h = BaoHasher()
            t0 = time.perf_counter()
            for off in range(0, total, piece):
                h.update(host[off:off + piece])
            h.finalize()
            best = min(best, time.perf_counter() - t0)
            del h
        out[f"hasher_{piece_mib}MiB_appends_GiBps"] = round(total / best / 2**30, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
