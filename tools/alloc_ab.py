"""In-process A/B of buffer layouts for the 1024 x 16 MiB 4-of-8 encode
(calibration tool, not product code): one allocation per direction vs the
batch split over two allocations (launched back to back, or concurrently on
two streams), interleaved rounds in ONE process so that the comparison does
not depend on which process got which HBM placement.
    python tools/alloc_ab.py [rounds=5] [one-first|one-last]
"""
import sys

import torch

sys.path.insert(0, ".")
from carbonado_amd import device  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
N, COUNT, K, M = 16 << 20, 1024, 4, 8
C = N // K
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def rnd(shape):
    t = torch.empty(shape, dtype=torch.uint8, device=dev)
    flat = t.view(-1)
    g = torch.Generator(device=dev).manual_seed(7)
    for off in range(0, flat.numel(), 1 << 30):
        n = min(1 << 30, flat.numel() - off)
        flat[off:off + n].copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g))
    return t


ORDER = sys.argv[2] if len(sys.argv) > 2 else "one-first"
if ORDER == "one-first":
    one_in, one_out = rnd((COUNT, N)), torch.empty((COUNT, M * C), dtype=torch.uint8, device=dev)
h_in = [rnd((COUNT // 2, N)), rnd((COUNT // 2, N))]
h_out = [torch.empty((COUNT // 2, M * C), dtype=torch.uint8, device=dev) for _ in range(2)]
q_in = [rnd((COUNT // 4, N)) for _ in range(4)]
q_out = [torch.empty((COUNT // 4, M * C), dtype=torch.uint8, device=dev) for _ in range(4)]
if ORDER != "one-first":
    one_in, one_out = rnd((COUNT, N)), torch.empty((COUNT, M * C), dtype=torch.uint8, device=dev)
s2 = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def one():
    device.zfec_encode_batch(one_in, N, one_out, K, M)


def halves_seq():
    for i in range(2):
        device.zfec_encode_batch(h_in[i], N, h_out[i], K, M)


def halves_conc():
    cur = torch.cuda.current_stream()
    for i in range(2):
        s2[i].wait_stream(cur)
        with torch.cuda.stream(s2[i]):
            device.zfec_encode_batch(h_in[i], N, h_out[i], K, M)
    for i in range(2):
        cur.wait_stream(s2[i])


def quarters_seq():
    for i in range(4):
        device.zfec_encode_batch(q_in[i], N, q_out[i], K, M)


cases = {"one allocation": one, "two allocations, back to back": halves_seq,
         "two allocations, two streams": halves_conc, "four allocations, back to back": quarters_seq}
print("allocation order:", ORDER)
for f in cases.values():  # the library's self-tuning, then warm
    for _ in range(3):
        f()
torch.cuda.synchronize()
res = {k: [] for k in cases}
for _ in range(R):
    for k, f in cases.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        b.synchronize()
        res[k].append(a.elapsed_time(b))
for k, v in res.items():
    v.sort()
    ms = v[len(v) // 2]
    gbs = 3 * N * COUNT / (ms * 1e-3) / 1e9
    print(f"{k:34s} median {ms:7.3f} ms  {gbs:7.1f} GB/s  {gbs / 8000:.4f} of 8 TB/s  "
          f"({COUNT * N / (ms * 1e-3) / 2**30:.1f} GiB/s of input)")
