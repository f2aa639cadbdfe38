"""Diagnostic: device encode() level 12 (zfec fused into the bao layout) vs the
oracle for a few object sizes; prints diff runs (stream offsets) when they differ.
Run on the GPU box from the repo root: python3 tools/pipeline_diff.py"""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from carbonado_amd import device
from oracle import oracle as O
L = device._lib.lib()
for n in (616565, 70001, 12288, 1 << 20, 3 << 20):
    host = np.random.default_rng(n).integers(0, 256, (2, (n + 31) // 16 * 16), dtype=np.uint8)
    inp = torch.from_numpy(host).cuda()
    enc, h, _ = O.encode(host[0, :n].tobytes(), 12)
    out = torch.full((2, (len(enc) + 15) // 16 * 16), 0xEE, dtype=torch.uint8, device="cuda")
    hs = torch.zeros((2, 32), dtype=torch.uint8, device="cuda")
    sc = device.encode_scratch(12, n, 2)
    olen, info = device.encode_batch(12, inp, n, out, hs, sc)
    torch.cuda.synchronize()
    g = out[0, :olen].cpu().numpy()
    e = np.frombuffer(enc, np.uint8)
    d = np.nonzero(g != e)[0]
    N = 8 * info.chunk_len // 1024
    offs = [L.chip_bao_encoded_len(0)]  # placeholder
    print(n, "C", info.chunk_len, "Cc", info.chunk_len // 1024, "N", N, "diffs", len(d), "hash ok", hs[0].cpu().numpy().tobytes() == h)
    if len(d):
        # classify diffs: find runs
        runs = []
        s = d[0]; p = d[0]
        for x in d[1:]:
            if x != p + 1:
                runs.append((s, p)); s = x
            p = x
        runs.append((s, p))
        print(" runs", len(runs), [(int(a), int(b)) for a, b in runs[:12]])
        print(" got", g[d[:8]], "exp", e[d[:8]])
