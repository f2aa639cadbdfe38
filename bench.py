#!/usr/bin/env python3
"""Headline benchmark: device-resident zfec 4-of-8 encode of 16 MiB objects
(BASELINE.json metric; configs[1]: 1024 x 16 MiB random buffers per GPU).

A step = one zfec encode launch over the whole per-GPU batch (1024 objects x
16 MiB = 16 GiB in, 32 GiB out), inputs already resident in HBM.  Objects
are independent, so N ranks each encode their own batch (weak scaling, no
data-path collective); the driver's N>1 launch uses torch.distributed only
for the barrier and the max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--objects 1024]
                    [--object-mib 16] [--k 4 --m 8] [--mode encode|decode|bao]

Rank 0 prints one JSON line (metric/value/unit/... + roofline + cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch  # first: the HIP runtime is shared with libcarbonado_hip (see _lib.py)
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from carbonado_amd import _lib, device  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s device-resident zfec 4-of-8 encode, 16 MiB objects; % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--objects", type=int, default=1024, help="objects per GPU")
    ap.add_argument("--object-mib", type=float, default=16.0)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--mode", choices=["encode", "decode", "bao"], default="encode")
    ap.add_argument("--erase", default="1,2", help="decode mode: shards dropped")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--traffic-json", default="auto",
                    help="PMC summary (profiles/*_pmc.json, tools/pmc_summary.py) with the measured HBM "
                         "bytes per launch of this kernel; 'auto' = newest matching file, 'none' = null")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()


def fill_random(t: torch.Tensor, seed: int) -> None:
    """Uniform random bytes on the device, in 1 GiB slabs (bounded temporaries)."""
    g = torch.Generator(device=t.device).manual_seed(seed)
    flat = t.view(-1)
    slab = 1 << 30
    for off in range(0, flat.numel(), slab):
        n = min(slab, flat.numel() - off)
        flat[off:off + n].copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device=t.device, generator=g))


def measured_traffic(spec: str, kernel_sym: str, alg_bytes: int):
    """HBM bytes per launch from a committed rocprofv3 PMC summary of the same
    kernel and workload (profiles/<tag>_pmc.json), else None."""
    if spec == "none":
        return None
    files = sorted((ROOT / "profiles").glob("*_pmc.json"), key=lambda p: p.stat().st_mtime) if spec == "auto" \
        else [Path(spec)]
    for f in reversed(files):
        try:
            tj = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        hb = tj.get("hbm_bytes_per_launch")
        if hb and kernel_sym in (tj.get("kernel") or "") and abs(hb - alg_bytes) < 0.25 * alg_bytes:
            return round(hb), str(f.relative_to(ROOT))
    return None, None


def cpu_baseline(args, n: int, sample_obj: bytes | None):
    """Time the CPU oracle (scalar fec.c-style restatement of zfec-rs) on
    whole 16 MiB objects, 1 thread, until ~cpu_seconds of work."""
    from oracle import oracle as O
    import numpy as np
    obj = np.frombuffer(sample_obj, np.uint8) if sample_obj is not None else O.fill_object(0xCA4B0AD0, 0, n)
    done = 0
    t0 = time.perf_counter()
    while True:
        if args.mode == "bao":
            O.bao_encode(obj)
        elif args.mode == "decode":
            pass
        else:
            O.zfec_encode(obj, args.k, args.m)
        done += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or done >= 4096:
            break
    return {"value": done * n / el / 2**30, "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{done} x {n} B objects ({'bao' if args.mode == 'bao' else 'zfec %d-of-%d encode' % (args.k, args.m)}), "
                      f"oracle/carbonado_oracle.c scalar fec.c-style restatement, 1 thread, {el:.1f} s"}


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    L = _lib.lib()
    rc = L.chip_init(local)
    if rc != 0:
        raise SystemExit(f"libcarbonado_hip: no usable gfx950 device ({rc})")
    k, m = args.k, args.m
    n = int(args.object_mib * (1 << 20))
    count = args.objects
    pad, C = 0, 0
    import ctypes
    p32, c32 = ctypes.c_uint32(), ctypes.c_uint32()
    L.chip_calc_padding_len(n, k, ctypes.byref(p32), ctypes.byref(c32))
    pad, C = p32.value, c32.value
    dev = torch.device("cuda", local)

    inp = torch.empty((count, n), dtype=torch.uint8, device=dev)
    fill_random(inp, 0xCA4B0AD0 + rank)
    if args.mode == "encode":
        out = torch.empty((count, m * C), dtype=torch.uint8, device=dev)
        step = lambda: device.zfec_encode_batch(inp, n, out, k, m)  # noqa: E731
        alg_bytes = count * (n + m * C)  # read input + write all m shards
        kernel = f"gf_apply_kernel<{k},{(m - k + 3) // 4}>"
        kernel_sym = f"gf_apply_kernel<{k}, {(m - k + 3) // 4},"
        unit_bytes = n
    elif args.mode == "decode":
        enc = torch.empty((count, m * C), dtype=torch.uint8, device=dev)
        device.zfec_encode_batch(inp, n, enc, k, m)
        erased = {int(x) for x in args.erase.split(",") if x}
        keep = [i for i in range(m) if i not in erased]
        out = torch.empty((count, k * C), dtype=torch.uint8, device=dev)
        step = lambda: device.zfec_decode_batch(enc, C, keep, out, k, m)  # noqa: E731
        alg_bytes = count * (2 * k * C)  # read k shares + write k data shards
        kernel = f"gf_apply_kernel<{k},1> (decode, erased {sorted(erased)})"
        kernel_sym = f"gf_apply_kernel<{k}, 1,"
        unit_bytes = n
    else:
        blen = L.chip_bao_encoded_len(n)
        out = torch.empty((count, (blen + 15) // 16 * 16), dtype=torch.uint8, device=dev)
        hashes = torch.empty((count, 32), dtype=torch.uint8, device=dev)
        scratch = device.bao_scratch(n, count, dev)
        step = lambda: device.bao_encode_batch(inp, n, out, hashes, scratch)  # noqa: E731
        alg_bytes = count * (n + blen)
        kernel = "bao_chunk_kernel<0> + bao_parent_kernel<0> levels"
        kernel_sym = "bao_chunk_kernel"
        unit_bytes = n
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    elapsed = t1 - t0
    launch_ms = [a.elapsed_time(b) for a, b in evs]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    max_elapsed = float(t.item())

    verified = None
    sample = None
    if rank == 0 and not args.no_verify:
        from oracle import oracle as O
        sample = inp[0].cpu().numpy().tobytes()
        if args.mode == "encode":
            verified = out[0].cpu().numpy().tobytes() == O.zfec_encode(sample, k, m)[0]
        elif args.mode == "decode":
            verified = out[0, :n].cpu().numpy().tobytes() == sample
        else:
            verified = hashes[0].cpu().numpy().tobytes() == O.blake3(sample)

    if rank == 0:
        total_units = world * count * unit_bytes * args.steps
        value = total_units / max_elapsed / 2**30
        avg_ms = sum(launch_ms) / len(launch_ms)
        achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = measured_traffic(args.traffic_json, kernel_sym, alg_bytes)
        res = {
            "metric": METRIC if args.mode == "encode" and (k, m) == (4, 8) else
            f"GiB/s device-resident {args.mode} ({k}-of-{m}), {args.object_mib:g} MiB objects",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes generated on device)",
            "config": {"workload": f"zfec {k}-of-{m} {args.mode}, {count} x {args.object_mib:g} MiB objects per GPU"
                       if args.mode != "bao" else f"bao encode, {count} x {args.object_mib:g} MiB objects per GPU",
                       "objects_per_gpu": count, "object_bytes": n, "chunk_len": C, "k": k, "m": m,
                       "global_objects": world * count,
                       "parallelism": f"objects partitioned over {world} rank(s), no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kernel, "alg_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": round(avg_ms, 4), "min_launch_ms": round(min(launch_ms), 4)},
            "verified_object0": verified,
        }
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(args, n, sample)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
