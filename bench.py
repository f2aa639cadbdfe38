#!/usr/bin/env python3
"""Headline benchmark: device-resident zfec 4-of-8 encode of 16 MiB objects
(BASELINE.json metric; configs[1]: 1024 x 16 MiB random buffers per GPU).

A step = one zfec encode launch over the whole per-GPU batch (1024 objects x
16 MiB = 16 GiB in, 32 GiB out), inputs already resident in HBM.  Objects
are independent, so N ranks each encode their own contiguous range of the
global object set (weak scaling, no data-path collective).  torch.distributed
(gloo) carries only the control plane: barrier and max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5]
                    [--objects 1024] [--object-mib 16] [--k 4 --m 8]
                    [--mode encode|decode|bao|...] [--alloc chip|contiguous|torch]
                    [--scatter] [--dry-run]

--gpus N with N > 1 and no WORLD_SIZE in the environment: this process
starts the N rank processes itself (RANK/LOCAL_RANK/WORLD_SIZE,
MASTER_ADDR=127.0.0.1) before anything touches the GPU, waits for them and
exits with their status; under torch.distributed.run WORLD_SIZE must equal N.
Rank 0 prints one JSON line (metric/value/unit/... + roofline + cpu_baseline).
"""
from __future__ import annotations

import argparse
import datetime
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import torch  # first: the HIP runtime is shared with libcarbonado_hip (see _lib.py)
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from carbonado_amd.sharding import max_over_ranks, object_range  # noqa: E402

# BLAKE3 ceiling, measured (tools/valu_probe.hip, profiles/r6q_valu_probe.txt): the product's b3_compress
# (four G's issued step by step, b3_g4) in a register-only loop at 8 waves/SIMD runs 6.125e10
# compressions/s = 41.2 T "672-op" lane-ops/s.  gfx950 issues the VOP2 int ops (v_add_u32, v_xor_b32)
# and v_bitop3_b32 at the full SIMD-32 rate (~69 T lane-ops/s measured, 78.6 nominal) but v_add3_u32,
# v_alignbit_b32, v_perm_b32, v_lshl_add_u32 and SDWA forms at half rate (~38 T); half of a
# compression's instructions are of the second kind.
VALU_PEAK_TOPS = 41.2
VALU_PEAK_SRC = ("measured BLAKE3 ceiling: the product's b3_compress (b3_g4 order) in a register loop, 8 waves/SIMD, "
                 "6.125e10 compressions/s x 672 (tools/valu_probe.hip VAR 3, profiles/r6q_valu_probe.txt); VOP2 "
                 "add/xor issue at ~69 T lane-ops/s, the VOP3 add3/alignbit at ~38 T")
# hardware VALU issue peak: a wave64 VOP2 op every 2 cycles per SIMD = 32 lane-ops/cycle x 4 SIMDs x
# 256 CUs x 2.4 GHz (measured ~69 T for v_add/v_xor at 2 waves/SIMD; half of BLAKE3's ops issue at half rate)
HW_VALU_PEAK_TOPS = 78.6
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s device-resident zfec 4-of-8 encode, 16 MiB objects; % HBM roofline"
SEED = 0xCA4B0AD0


# BASELINE.json configs as presets (configs[1..4]; configs[0] is the CPU
# round trip of tests/test_oracle.py and tests/test_gpu_pipeline.py)
CONFIGS = {
    "cfg2": dict(mode="encode", k=4, m=8, objects=1024),                     # zfec 4-of-8 encode, 1024 x 16 MiB
    "cfg3": dict(mode="decode", k=4, m=8, objects=1024, erase="1,2"),        # decode, 2 shards dropped
    "cfg4": dict(mode="e2e", k=4, m=8, objects=1024, level=15),              # full encode(), host -> host
    "cfg5": dict(mode="encode", k=8, m=16, objects=1024),                    # 8-of-16, 1024 per GPU (8192 on 8)
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py starts them itself")
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="BASELINE.json config preset (sets mode, k, m, objects, erase, level)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--objects", type=int, default=1024, help="objects per GPU")
    ap.add_argument("--object-mib", type=float, default=16.0)
    ap.add_argument("--object-bytes", type=int, default=0,
                    help="object size in bytes (overrides --object-mib), e.g. 16779371: a 16 MiB object after "
                         "level 15's snap + ECIES stages, zfec shards of 4,195,328 B")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--mode", choices=["encode", "decode", "bao", "bao-decode", "pipeline", "pipeline-decode", "e2e", "e2e-decode", "scrub",
                                       "scrub-batch", "hasher", "file", "latency"],
                    default="encode",
                    help="bao-decode: device-resident decoding::bao (verify every node, return the content); "
                         "pipeline: device-resident encode() at --level (Bao/Zfec bits; 12 = zfec fused into "
                         "bao); e2e: encode() at --level from pinned HOST memory to host memory (H2D+kernels+D2H); "
                         "scrub: scrub() of level-12 streams with one corrupted shard (host API, decoding.rs:151-212); "
                         "scrub-batch: scrub() of device-resident level-12 streams, every --scrub-every-th one damaged "
                         "(chip_scrub_batch_dev); "
                         "hasher: BaoHasher update()+finalize() over the objects in 4 MiB appends (utils.rs:104-137); "
                         "file: file::encode of flat files on disk to .c<level> files (file.rs:409-440); "
                         "latency: one object per call through the C-ABI (tools/abi_latency: the library call, the "
                         "Rust patch's call sequence, round 5's) at --latency-levels x --latency-sizes, the C "
                         "oracle's single-thread time per call beside each row")
    ap.add_argument("--latency-levels", default="12,4,8,15", help="latency mode: Format levels")
    ap.add_argument("--latency-sizes", default="1024,1048576,16777216", help="latency mode: object bytes")
    ap.add_argument("--latency-reps", type=int, default=40, help="latency mode: calls per form and row")
    ap.add_argument("--file-dir", default=None, help="file mode: working directory (default $TMPDIR/carbonado_files)")
    ap.add_argument("--fsync", action="store_true", help="file mode: fsync every output file")
    ap.add_argument("--file-slice", type=int, default=64, help="file mode: files per pipeline slice")
    ap.add_argument("--io-threads", type=int, default=16, help="file mode: reader / writer threads per stage")
    ap.add_argument("--level", type=int, default=12, help="e2e mode: Format bits (Bao|Zfec = 12)")
    ap.add_argument("--slots", type=int, default=3, help="e2e mode: pipeline slots (streams)")
    ap.add_argument("--slice-mib", type=int, default=256, help="e2e mode: input bytes per pipeline slice")
    ap.add_argument("--in-pad-kib", type=int, default=0, help="encode/decode: extra bytes per input object row")
    ap.add_argument("--out-pad-kib", type=int, default=0, help="encode/decode: extra bytes per output object row")
    ap.add_argument("--bao-stream-offset", type=int, default=56,
                    help="bao / bao-decode: each stream starts this many bytes into its 256-B multiple row (56, the "
                         "default: every chunk and node on a 64-B boundary; bao encode 2233 -> 2320 GiB/s, "
                         "profiles/r10j_session)")
    ap.add_argument("--stream-offset", type=int, default=56,
                    help="pipeline at Zfec|Bao: each stream starts this many bytes into its 256-B multiple row "
                         "(56, the default: every chunk and node on a 64-B boundary, include/carbonado_hip.h; "
                         "0: streams at the row start, +4 to +11 %% slower, profiles/r10i_session)")
    ap.add_argument("--prealloc-gib", type=float, default=0, help="allocate (and keep) this much HBM first")
    ap.add_argument("--alloc", choices=["chip", "contiguous", "torch"], default="chip",
                    help="device batch buffers: the library's class-balanced allocator (chip_device_alloc via "
                         "carbonado_amd.device.empty_batch; DESIGN.md §2), physically contiguous HBM "
                         "(CHIP_ALLOC=contiguous), or torch's caching allocator")
    ap.add_argument("--host-threads", type=int, default=16,
                    help="e2e mode: host threads for the Snappy/Ecies stages (the GPU box's CPU share is 16)")
    ap.add_argument("--erase", default="1,2", help="decode mode: shards dropped")
    ap.add_argument("--scrub-every", type=int, default=64,
                    help="scrub-batch mode: one object in this many has a corrupted byte in a data shard")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of each CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="second CPU baseline with objects in parallel on this many host threads (SURVEY 8d: "
                         "'all host cores'; the GPU box's CPU share is 16); 0 or 1 = the 1-thread one only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--verify-all", action="store_true",
                    help="pipeline mode: check EVERY object bit-exact (encode mode does by default): BLAKE3 of "
                         "each object's output on the GPU vs the C oracle's zfec (or encode()) + BLAKE3 on 16 host "
                         "threads, outside the timed region")
    ap.add_argument("--no-verify-all", action="store_true",
                    help="encode / decode / e2e / bao / bao-decode modes (which check every object by default): "
                         "object 0 only")
    ap.add_argument("--no-aliased", action="store_true",
                    help="encode mode: skip the second, in-place (aliased data shards) measurement")
    ap.add_argument("--no-box-ceiling", action="store_true",
                    help="encode mode: skip the box-ceiling diagnostic (the same memory pattern without the GF "
                         "arithmetic, with GPU clocks and partition modes), run after the checks")
    ap.add_argument("--scatter", action="store_true",
                    help="N>1: rank 0 generates every object and scatters them over RCCL/xGMI (timed "
                         "separately, outside `value`)")
    ap.add_argument("--scatter-gib", type=float, default=1.0,
                    help="N>1 without --scatter: GiB per rank that rank 0 scatters over RCCL/xGMI once, timed and "
                         "reported as `scatter` (the inputs themselves are generated on each rank); 0 = none")
    ap.add_argument("--dry-run", action="store_true", help="no device: exercise the multi-rank control plane")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="leave the process's CPUs and memory policy alone (default: once the GPU is known, the "
                         "main thread runs on the GPU's NUMA node and allocates host memory there)")
    ap.add_argument("--traffic-json", default="auto",
                    help="PMC summary (profiles/*_pmc.json, tools/pmc_summary.py) with the measured HBM "
                         "bytes per launch of this kernel; 'auto' = newest matching file, 'none' = null; used "
                         "when the live PMC passes are off or fail")
    ap.add_argument("--live-pmc", choices=["auto", "on", "off"], default="auto",
                    help="measure roofline.traffic in this run: two child processes of the same workload under "
                         "`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (one pass each) before this process "
                         "touches the GPU; auto = on at N=1 for the device-resident modes with one dominant kernel")
    args = ap.parse_args(argv)
    if args.object_bytes:
        args.object_mib = args.object_bytes / 2**20  # exact: an integer over a power of two
    if args.config:
        explicit = {a.dest for a in ap._actions if any(o in (argv if argv is not None else sys.argv[1:])
                                                       for o in a.option_strings)}
        for key, val in CONFIGS[args.config].items():
            if key not in explicit:
                setattr(args, key, val)
    if args.mode in ("scrub", "hasher") and args.objects == ap.get_default("objects"):
        args.objects = 64  # host-API paths: a bounded host-memory working set
    if args.mode == "file" and args.objects == ap.get_default("objects"):
        args.objects = 128  # 2 GiB of input files + 2.1 GiB of output files on the box's disk
    if args.mode not in ("encode", "decode", "e2e", "bao", "bao-decode", "pipeline-decode", "e2e-decode", "scrub",
                         "scrub-batch", "file"):
        args.no_verify_all = True
    return args


def spawn_ranks(n: int) -> int:
    """Start the n rank processes of `bench.py --gpus n` (this process never
    touches the GPU), wait for them, return the worst exit status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    procs = [subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:],
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def visible_gpus_no_hip() -> int:
    """GPUs this process may use, counted without initialising HIP (a rank
    decides whether to profile itself before it touches the GPU: torch's
    device_count can fall back to hipGetDeviceCount): the visibility
    variable if set, else the KFD topology's GPU nodes (simd_count > 0)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip():
            return len([x for x in v.split(",") if x.strip()])
    gpus = 0
    for props in Path("/sys/class/kfd/kfd/topology/nodes").glob("*/properties"):
        try:
            kv = dict(line.split()[:2] for line in props.read_text().splitlines() if len(line.split()) >= 2)
        except OSError:
            continue
        gpus += int(kv.get("simd_count", "0")) > 0
    return gpus


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or leave WORLD_SIZE unset")
    if world > 1:
        dist.init_process_group("gloo")  # control plane only: no bytes of the path cross it
    return world, rank, local


def gather_floats(value: float, world: int) -> list:
    """Every rank's value (gloo control plane), in rank order."""
    if world == 1:
        return [float(value)]
    out = [None] * world
    dist.all_gather_object(out, float(value))
    return [float(v) for v in out]


def verify_threads(world: int) -> int:
    """Host threads each rank may use for its checks: the ranks share the
    host's CPUs (os.cpu_count() // world), at most 16 each (a GPU's share of
    the box)."""
    return max(1, min(16, (os.cpu_count() or 1) // max(1, world)))


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
    kernel and workload (profiles/<tag>_pmc.json), else (None, None)."""
    if spec == "none":
        return None, None
    # newest round/session tag last (r1…, r2a … r2z sort in the order they were taken)
    files = sorted((ROOT / "profiles").glob("*_pmc.json")) if spec == "auto" else [Path(spec)]
    for f in reversed(files):
        try:
            tj = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        hb = tj.get("hbm_bytes_per_launch")
        if hb and kernel_sym in (tj.get("kernel") or "") and abs(hb - alg_bytes) < 0.25 * alg_bytes:
            return round(hb), str(f.relative_to(ROOT))
    return None, None


def pmc_kernel_sym(args) -> str | None:
    """Substring of the rocprofv3 kernel name of the mode's dominant kernel
    (the Workload's kernel_sym) for the device-resident modes the live PMC
    covers: one launch of it per step."""
    fused = os.environ.get("CHIP_FUSED", "1") != "0"
    n = int(args.object_mib * (1 << 20))
    if args.mode == "encode":
        return f"zfec_apply_kernel<{args.k}, {(args.m - args.k + 3) // 4}>"
    if args.mode == "decode":
        return f"zfec_apply_kernel<{args.k}, 1>"
    if fused and args.mode == "bao" and n >= 65536:
        return "bao_content_fused_kernel"
    if fused and args.mode == "pipeline" and args.level & 12 == 12:
        return "zfec_bao_fused_kernel"
    if args.mode == "bao-decode" or (args.mode == "pipeline-decode" and args.level & 4):
        return "bao_chunk_kernel_verify"
    return None


DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
            "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
            "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE", "TORCH_NCCL_ASYNC_ERROR_HANDLING")


def child_env(local_rank: int | None) -> dict:
    """Environment of a profiled single-GPU child: no torch.distributed
    variables (it runs alone), and at N > 1 only this rank's GPU visible."""
    env = {k: v for k, v in os.environ.items() if k not in DIST_ENV}
    env["TMPDIR"] = "/tmp"
    if local_rank is not None:
        picked = False
        for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
            if env.get(var):
                ids = [x for x in env[var].split(",") if x.strip()]
                env[var] = ids[local_rank % len(ids)]
                picked = True
        if not picked:
            env["HIP_VISIBLE_DEVICES"] = str(local_rank)
    return env


def live_traffic(args, argv: list, timeout_s: float = 240.0, local_rank: int | None = None) -> dict:
    """roofline.traffic measured in this run: the same workload in two child
    processes under rocprofv3, one counter pass each (FETCH_SIZE uses 3 TCC
    counters and WRITE_SIZE 2, so they cannot share a pass), then the
    MI355X_MICROARCH.md HBM recipe: bytes = 2 x FETCH_SIZE (gfx950 reports
    half of a wide streaming read; tools/fetch_calib pins the factor for this
    access shape) + WRITE_SIZE, both KiB, averaged over the timed launches
    (the last `steps` dispatches of the kernel: decode's child also runs the
    encode that builds its shares).  Runs before this process initialises the
    GPU; every child runs in its own process group and is killed (SIGKILL) at
    the time limit.  Returns {"bytes": ...} or {"error": ...}."""
    import csv
    import shutil
    import signal
    import subprocess
    import tempfile
    sym = pmc_kernel_sym(args)
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if sym is None or not Path(prof).exists():
        return {"error": "no rocprofv3" if sym else f"no live PMC for mode {args.mode}"}
    steps = 2
    child = [sys.executable, str(Path(__file__).resolve())] + list(argv) + [
        "--steps", str(steps), "--warmup", "1", "--live-pmc", "off", "--no-cpu-baseline", "--no-verify",
        "--no-verify-all", "--no-aliased", "--no-box-ceiling", "--traffic-json", "none", "--gpus", "1"]
    tmp = Path(tempfile.mkdtemp(prefix="chip_pmc_", dir="/tmp"))
    env = child_env(local_rank)
    vals, name = {}, None
    t0 = time.perf_counter()
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        tag = ctr.split("_")[0].lower()
        cmd = [prof, "--pmc", ctr, "-d", str(tmp / tag), "-o", tag, "--output-format", "csv", "--"] + child
        with open(tmp / f"{tag}.log", "wb") as log:
            p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT,
                                 start_new_session=True)
            try:
                rc = p.wait(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return {"error": f"{ctr} pass killed after {timeout_s:.0f} s"}
        if rc != 0:
            return {"error": f"{ctr} pass exit status {rc}"}
        rows = []
        for f in sorted((tmp / tag).rglob("*counter_collection.csv")):
            rows += [r for r in csv.DictReader(open(f)) if sym in r.get("Kernel_Name", "")]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        if len(rows) < steps:
            return {"error": f"{ctr} pass: {len(rows)} dispatches of {sym!r}"}
        name = rows[-1]["Kernel_Name"]
        vals[ctr] = sum(float(r["Counter_Value"]) for r in rows[-steps:]) / steps
    shutil.rmtree(tmp, ignore_errors=True)
    return {"bytes": round(2 * vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024),
            "FETCH_SIZE_KiB": vals["FETCH_SIZE"], "WRITE_SIZE_KiB": vals["WRITE_SIZE"], "kernel": name,
            "seconds": round(time.perf_counter() - t0, 1)}


def cpu_baseline(args, n: int, sample_obj: bytes | None, threads: int = 1, seconds: float | None = None):
    """Time the CPU oracle (scalar fec.c-style restatement of zfec-rs / the
    BLAKE3+bao restatement) on whole objects for ~cpu_seconds: 1 thread (the
    reference crate is single-threaded), or `threads` host threads each
    working through objects of its own (ctypes releases the GIL)."""
    from oracle import oracle as O
    import numpy as np
    obj = np.frombuffer(sample_obj, np.uint8) if sample_obj is not None else O.fill_object(SEED, 0, n)
    if args.mode in ("e2e", "e2e-decode", "file") and args.level & 1:
        import hashlib
        eph = hashlib.sha256(b"cpu baseline eph").digest()
        pub = O.c_public_key(hashlib.sha256(b"carbonado-amd bench receiver").digest())
    else:
        eph = pub = b""
    if args.mode == "e2e-decode":
        import hashlib
        sk = hashlib.sha256(b"carbonado-amd bench receiver").digest()
        enc_obj, h_obj, inf_obj = O.c_encode_full(obj, args.level, pub, eph if eph else bytes(32), bytes(16))
    if args.mode == "bao-decode":
        bstream, bhash = O.bao_encode(obj)
    if args.mode == "pipeline-decode":
        enc_obj, h_obj, inf_obj = O.encode(obj, args.level)
    if args.mode == "scrub-batch":
        enc_obj, h_obj, inf_obj = O.encode(obj, 12)
    if args.mode == "scrub":
        enc_obj, h_obj, inf_obj = O.encode(obj, 12)
        bad = bytearray(enc_obj)
        bad[scrub_corrupt_offset(len(obj), 0)] ^= 0x40
        zc, zpad, zC = O.zfec_encode(obj, 4, 8)
    if args.mode == "decode":
        z, pad, C = O.zfec_encode(obj, args.k, args.m)
        keep = [i for i in range(args.m) if str(i) not in args.erase.split(",")]
        shares = [z[i * C:(i + 1) * C] for i in keep]
    def one():
        if args.mode == "bao":
            O.bao_encode(obj)
        elif args.mode == "bao-decode":
            O.bao_decode(bstream, bhash)
        elif args.mode == "hasher":
            O.blake3(obj)
        elif args.mode == "scrub":
            # the reference's scrub: bao decode (fails), zfec decode of the
            # intact shards, re-encode; restated with the C oracle's pieces
            try:
                O.bao_decode(bytes(bad), h_obj)
            except Exception:
                pass
            keep_s = [i for i in range(8) if i != 0][:4]
            O.encode(O.zfec_decode_shares([zc[i * zC:(i + 1) * zC] for i in keep_s], keep_s, zpad), 12)
        elif args.mode == "pipeline-decode":
            O.decode(h_obj, enc_obj, inf_obj["padding_len"], args.level)
        elif args.mode == "scrub-batch":  # an intact stream: scrub()'s bao_decode succeeds
            O.bao_decode(enc_obj, h_obj)
        elif args.mode == "e2e-decode":
            cur = O.decode(h_obj, enc_obj, inf_obj["padding_len"], args.level & 12) if args.level & 12 else enc_obj
            if args.level & 1:
                cur = O.c_ecies_decrypt(sk, cur)
            if args.level & 2:
                cur = O.c_snap_decompress(cur, n + 1024)
        elif args.mode in ("e2e", "pipeline", "file"):
            if args.level & 3:  # host stages too: the all-C restatement (oracle/host_oracle.c)
                O.c_encode_full(obj, args.level, pub, eph, bytes(16))
            else:
                O.encode(obj, args.level)
        elif args.mode == "decode":
            O.zfec_decode_shares(shares, keep, pad, args.k, args.m)
        else:
            O.zfec_encode(obj, args.k, args.m)

    def worker(deadline):
        c = 0
        while True:
            one()
            c += 1
            if time.perf_counter() >= deadline or c >= 4096:
                return c
    budget = args.cpu_seconds if seconds is None else seconds
    t0 = time.perf_counter()
    if threads <= 1:
        done = worker(t0 + budget)
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(worker, [t0 + budget] * threads))
    el = time.perf_counter() - t0
    what = {"bao": "bao encode", "bao-decode": "bao decode (verify + content)", "e2e": f"encode() level {args.level}", "pipeline": f"encode() level {args.level}",
            "file": f"encode() level {args.level} (in memory, no file I/O, no header)",
            "hasher": "BLAKE3 of the content", "scrub": "scrub() restated: bao decode + zfec decode + encode()", "e2e-decode": f"decode() level {args.level}",
            "pipeline-decode": f"decode() level {args.level}",
            "scrub-batch": "scrub() of an intact level-12 stream: bao decode of the stream",
            "decode": f"zfec {args.k}-of-{args.m} decode, erased {args.erase}"}.get(
        args.mode, f"zfec {args.k}-of-{args.m} encode")
    return {"value": round(done * n / el / 2**30, 4), "unit": "GiB/s", "cores": max(1, threads), "kind": "port",
            "sample": f"{done} x {n} B objects ({what}) through oracle/carbonado_oracle.c"
                      f"{' + host_oracle.c' if args.mode in ('e2e', 'e2e-decode', 'file') and args.level & 3 else ''}, scalar "
                      f"restatement of the reference crates, "
                      f"{'1 thread' if threads <= 1 else f'{threads} threads, objects in parallel'}, {el:.1f} s"}


PCIE_SPEC_GBS = 63.0  # PCIe Gen5 x16, per direction (spec)
# one direction alone, pinned host memory, the runtime's DMA path (tools/pageable_probe.hip,
# profiles/r1w_pageable_probe.txt): the practical per-direction ceilings on the GPU box
PCIE_MEASURED_GBS = {"h2d": 55.6, "d2h": 55.0}
# both directions at once: two pinned 16 MiB-piece copy streams side by side
# (tools/h2d_probe.py, profiles/r9q_session/h2d_probe.log: 47.1 GB/s each way)
PCIE_MEASURED_DUPLEX_GBS = 94.2


class ClockSampler:
    """The GPU's current SCLK / MCLK / FCLK (the `*` level of sysfs
    pp_dpm_*) sampled every 10 ms on a host thread between start() and
    stop(), plus its compute / memory partition modes, read from the PCI
    device directory the library reports (chip_host_topology's gpu_pci).
    Diagnostic only: anything unreadable is reported as such."""

    FILES = ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk")

    def __init__(self, dev):
        import threading
        self.base, self.err = None, None
        try:
            from carbonado_amd import device
            pci = device.host_topology().get("gpu_pci")
            if pci and Path(f"/sys/bus/pci/devices/{pci}").is_dir():
                self.base = Path(f"/sys/bus/pci/devices/{pci}")
            else:
                self.err = f"no sysfs directory for gpu_pci={pci!r}"
        except Exception as e:  # diagnostic only
            self.err = f"{type(e).__name__}: {e}"[:200]
        self.samples = {f: [] for f in self.FILES}
        self.stop_ev = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)

    @staticmethod
    def current_mhz(text: str):
        for line in text.splitlines():
            if line.rstrip().endswith("*"):
                for tok in line.split():
                    if tok.lower().endswith("mhz"):
                        try:
                            return int(float(tok[:-3]))
                        except ValueError:
                            return None
        return None

    def _read(self, name: str):
        try:
            return (self.base / name).read_text()
        except OSError:
            return None

    def _run(self):
        while not self.stop_ev.is_set():
            for f in self.FILES:
                t = self._read(f)
                v = self.current_mhz(t) if t else None
                if v is not None:
                    self.samples[f].append(v)
            self.stop_ev.wait(0.01)

    def start(self):
        if self.base is not None:
            self.thread.start()

    def stop(self) -> dict:
        if self.base is None:
            return {"unavailable": self.err}
        self.stop_ev.set()
        self.thread.join()
        out = {"sysfs": str(self.base)}
        for f in self.FILES:
            s = self.samples[f]
            out[f[7:] + "_MHz"] = {"min": min(s), "max": max(s), "samples": len(s)} if s else None
        for f in ("current_compute_partition", "current_memory_partition"):
            t = self._read(f)
            out[f.replace("current_", "")] = t.strip() if t else None
        return out


def bao_data_region_len(N: int) -> int:
    """End of the data region of a Zfec|Bao stream of N chunks: the end of chunk
    N/2 - 1 (bao pre-order: chunk i at 8 + 1024 i + 64 (P(i) + c(i)), c(s) the
    parents whose leftmost chunk is s; bao_kernels.hip header)."""
    def ceil_log2(x):
        return (x - 1).bit_length()

    def c(s):
        return ceil_log2(N) if s == 0 else min((s & -s).bit_length() - 1, ceil_log2(N - s))
    last = N // 2 - 1
    return 8 + 1024 * last + 64 * (sum(c(s) for s in range(last)) + c(last)) + 1024


def pcie_roofline(h2d_bytes: int, d2h_bytes: int, step_s: float, duplex_achieved: float) -> dict:
    """Roofline of a host-buffer path (H2D and D2H overlapped): each direction
    priced separately, since the traffic is asymmetric (encode() writes ~2x
    what it reads).  `bound` names the binding direction, the one at the
    higher fraction of its own peak; the duplex sum is kept alongside."""
    rate = {d: b / step_s / 1e9 for d, b in (("h2d", h2d_bytes), ("d2h", d2h_bytes))}
    bind = max(rate, key=lambda d: rate[d] / PCIE_SPEC_GBS)
    return {"bound": f"pcie-{bind}", "achieved": round(rate[bind], 2), "peak": PCIE_SPEC_GBS, "unit": "GB/s",
            "frac": round(rate[bind] / PCIE_SPEC_GBS, 4),
            "frac_of_measured": round(rate[bind] / PCIE_MEASURED_GBS[bind], 4),
            "peak_measured": PCIE_MEASURED_GBS[bind],
            "h2d_GBps": round(rate["h2d"], 2), "d2h_GBps": round(rate["d2h"], 2),
            "h2d_frac": round(rate["h2d"] / PCIE_SPEC_GBS, 4), "d2h_frac": round(rate["d2h"] / PCIE_SPEC_GBS, 4),
            "duplex_GBps": round(duplex_achieved, 2), "duplex_frac": round(duplex_achieved / (2 * PCIE_SPEC_GBS), 4),
            "duplex_peak_measured": PCIE_MEASURED_DUPLEX_GBS,
            "duplex_frac_of_measured": round((rate["h2d"] + rate["d2h"]) / PCIE_MEASURED_DUPLEX_GBS, 4),
            "note": ("PCIe Gen5 x16: 63 GB/s per direction (spec); peak_measured = that direction alone from "
                     "pinned memory on the GPU box (profiles/r1w_pageable_probe.txt); duplex_peak_measured = both "
                     "directions at once (profiles/r9q_session/h2d_probe.log); H2D and D2H overlap, rates over "
                     "the whole step's wall time")}


def bind_to_gpu_node() -> dict:
    """A NUMA-aware host for one GPU: the calling (main) thread moves to the
    CPUs of the GPU's NUMA node and prefers that node for the memory it
    touches first, so the host buffers the workload makes next sit next to
    the GPU's PCIe root (the library already keeps its staging ring and copy
    threads there).  The GPU box is two sockets; without this the process
    lands on either (BaoHasher)."""
    import ctypes
    from carbonado_amd.device import host_topology
    t = host_topology()
    node, pci = t.get("gpu_node", -1), t.get("gpu_pci", "")
    if node is None or node < 0 or not pci:
        return {"bound": False, "why": "GPU NUMA node unknown"}
    try:
        cpus = set()
        for part in Path(f"/sys/bus/pci/devices/{pci}/local_cpulist").read_text().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    except (OSError, ValueError) as e:
        return {"bound": False, "why": f"local_cpulist: {e}"}
    cpus &= os.sched_getaffinity(0)
    if not cpus:
        return {"bound": False, "why": "none of the GPU's CPUs are allowed"}
    os.sched_setaffinity(0, cpus)
    libc = ctypes.CDLL(None, use_errno=True)
    mask = ctypes.c_ulong(1 << node)
    MPOL_PREFERRED, SYS_set_mempolicy = 1, 238  # x86_64
    pol = libc.syscall(SYS_set_mempolicy, MPOL_PREFERRED, ctypes.byref(mask), 64 + 1) == 0
    return {"bound": True, "gpu_node": node, "cpus": len(cpus), "mempolicy_preferred": pol}


def scrub_corrupt_offset(n: int, o: int) -> int:
    """Stream offset of a content byte inside data shard o % 4 of a level-12
    encoding of n bytes (one byte per object is flipped for --mode scrub):
    chunk i of the bao stream sits at 8 + 1024 i + 64 (P(i) + c(i))."""
    unit = 1024 * 4
    C = -(-n // unit) * unit // 4
    N = 8 * C // 1024

    def clog2(x):
        return 0 if x <= 1 else (x - 1).bit_length()

    def c_at(s):
        cl = clog2(N - s)
        return cl if s == 0 else min((s & -s).bit_length() - 1, cl)

    def p_before(s):
        total, cnt, L = 0, N, 1
        while cnt > 1:
            total += min((s + (1 << L) - 1) >> L, cnt // 2)
            cnt = (cnt + 1) // 2
            L += 1
        return total
    i = (o % 4) * (C // 1024) + (C // 1024) // 3
    return 8 + 1024 * i + 64 * (p_before(i) + c_at(i)) + 517


def _lib_len(n: int) -> int:
    from carbonado_amd import _lib
    return _lib.lib().chip_bao_encoded_len(n)


class Workload:
    """The per-rank batch and its step function (device buffers from torch)."""

    def __init__(self, args, rank: int, local: int, world: int):
        from carbonado_amd import _lib, device
        self.args = args
        L = _lib.lib()
        self.dev = dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
        if L.chip_init(dev.index) != 0:
            raise SystemExit(f"libcarbonado_hip: no usable gfx950 device: {L.chip_last_device_error().decode()}")
        # before any host buffer of the workload exists
        self.host_binding = {"bound": False, "why": "--no-numa-bind"} if args.no_numa_bind else bind_to_gpu_node()
        self.k, self.m = k, m = args.k, args.m
        self.n = n = int(args.object_mib * (1 << 20))
        self.count = count = args.objects
        p32, c32 = ctypes.c_uint32(), ctypes.c_uint32()
        L.chip_calc_padding_len(n, k, ctypes.byref(p32), ctypes.byref(c32))
        self.C = C = c32.value
        self.prealloc = (torch.empty(int(args.prealloc_gib * 2**30), dtype=torch.uint8, device=dev)
                         if args.prealloc_gib else None)
        if args.alloc == "contiguous":
            os.environ["CHIP_ALLOC"] = "contiguous"  # read by chip_device_alloc at each call
        device_mode = args.mode in ("encode", "decode", "bao", "bao-decode", "pipeline", "pipeline-decode",
                                    "scrub-batch")
        self.alloc_info = {}

        def batch_buf(shape, name=None):
            """Device batch buffer: the library's allocator (class-balanced from 1 GiB up) or torch's."""
            if args.alloc != "torch" and device_mode:
                t = device.empty_batch(shape, dev)
                if name:
                    f, u, sec = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_double()
                    if L.chip_device_alloc_info(ctypes.c_void_p(t.data_ptr()), ctypes.byref(f), ctypes.byref(u),
                                                ctypes.byref(sec)) == 0:
                        self.alloc_info[name] = {"classes_found": f.value, "classes_used": u.value,
                                                 "alloc_s": round(sec.value, 3)}
                return t
            return torch.empty(shape, dtype=torch.uint8, device=dev)
        self.batch_buf = batch_buf
        # bao, pipeline modes: object rows at a 256-B pitch for any n (the batch entry points take
        # 16-B multiples; at 16 B every 128-B piece a wave loads straddles two lines and K13 fetches
        # 1.21x the input, tools/k13_fetch, profiles/r10c_session), handed over whole
        row = ((n + 255) // 256 * 256 if args.mode in ("bao", "pipeline", "pipeline-decode", "bao-decode") else n) + \
            args.in_pad_kib * 1024
        self.inp_full = batch_buf((count, row), "in")
        self.inp = self.inp_full[:, :n] if row != n else self.inp_full
        self.scatter_s = None
        rng = object_range(rank, world, world * count)
        if args.scatter and world > 1:
            self.scatter_s = self._scatter_inputs(rank, world)
        else:
            fill_random(self.inp_full, SEED + rng.start)
        if args.mode == "encode":
            self.out = batch_buf((count, m * C + args.out_pad_kib * 1024), "out")
            self.step = lambda: device.zfec_encode_batch(self.inp_full, n, self.out, k, m)
            self.alg_bytes = count * (n + m * C)  # read the input + write all m shards
            ng = (m - k + 3) // 4
            self.kernel = f"zfec_apply_kernel<{k}, {ng}>"
            self.kernel_sym = f"zfec_apply_kernel<{k}, {ng}>"
        elif args.mode == "decode":
            self.enc = batch_buf((count, m * C), "enc")
            device.zfec_encode_batch(self.inp, n, self.enc, k, m)
            erased = {int(x) for x in args.erase.split(",") if x}
            self.keep = [i for i in range(m) if i not in erased]
            self.out = batch_buf((count, k * C), "out")
            self.step = lambda: device.zfec_decode_batch(self.enc, C, self.keep, self.out, k, m)
            self.alg_bytes = count * (2 * k * C)  # read k shares + write k data shards
            self.kernel = f"zfec_apply_kernel<{k}, 1> (decode, erased {sorted(erased)})"
            self.kernel_sym = f"zfec_apply_kernel<{k}, 1>"
        elif args.mode == "pipeline":
            lv = args.level
            if lv & 3:
                raise SystemExit("--mode pipeline runs the device-only levels (Bao/Zfec bits); use --mode e2e")
            zlen = m * C if lv & 8 else n
            self.blen = blen = L.chip_bao_encoded_len(zlen) if lv & 4 else zlen
            self.soff = off = args.stream_offset if lv & 12 == 12 else 0
            self.out = batch_buf((count, (off + blen + 255) // 256 * 256), "out")
            self.hashes = torch.empty((count, 32), dtype=torch.uint8, device=dev)
            self.scratch = device.encode_scratch(lv, n, count, dev)
            self.step = lambda: device.encode_batch(lv, self.inp_full, n, self.out, self.hashes, self.scratch,
                                                    out_offset=off)
            # HBM bytes: the object read once, its stream written once.  At Zfec|Bao the fused
            # kernel (K13) hashes the shards on chip; CHIP_FUSED=0 runs K1-BL + K3, which
            # read the 8C bytes of shards back (counted then)
            two = lv & 12 == 12 and os.environ.get("CHIP_FUSED", "1") == "0"
            self.alg_bytes = count * (n + zlen + zlen + (blen - zlen)) if two else count * (n + blen)
            self.zlen = zlen
            if lv & 12 == 12 and not two:
                self.kernel = (f"encode() level {lv} on the device: zfec_bao_fused_kernel_full/_general (zfec 4-of-8 + chunk "
                               "hashing + tree levels 1-3 in one pass) + parent levels from level 4")
                self.kernel_sym = "zfec_bao_fused_kernel"
            elif two:
                self.kernel = (f"encode() level {lv} on the device: gf_apply_bl_kernel + bao_chunk_kernel_inplace + parent "
                               "levels (zfec writes the shards into their bao chunk slots; bao hashes in place)")
            elif lv & 4:
                self.kernel = f"encode() level {lv} on the device: bao_content_fused_kernel / bao_chunk_kernel_encode + parent levels"
            else:
                self.kernel = f"encode() level {lv} on the device: zfec_apply_kernel"
            if not (lv & 12 == 12 and not two):
                self.kernel_sym = "pipeline"
        elif args.mode == "pipeline-decode":
            lv = args.level
            if lv & 3:
                raise SystemExit("--mode pipeline-decode runs the device-only levels (Bao/Zfec bits); use --mode "
                                 "e2e-decode")
            zlen = m * C if lv & 8 else n
            self.blen = blen = L.chip_bao_encoded_len(zlen) if lv & 4 else zlen
            self.zlen = zlen
            self.soff = off = args.stream_offset if lv & 12 == 12 else 0
            self.enc = batch_buf((count, (off + blen + 255) // 256 * 256), "enc")
            self.hashes = torch.empty((count, 32), dtype=torch.uint8, device=dev)
            esc = device.encode_scratch(lv, n, count, dev)
            _, info = device.encode_batch(lv, self.inp_full, n, self.enc, self.hashes, esc, out_offset=off)
            torch.cuda.synchronize()
            del esc
            self.pad = info.padding_len
            self.out = batch_buf((count, (n + 255) // 256 * 256), "out")
            self.status = torch.full((count,), -1, dtype=torch.int32, device=dev)
            self.scratch = device.decode_scratch(lv, blen, count, dev)
            self.step = lambda: device.decode_batch(lv, self.enc, blen, self.hashes, self.pad, self.out, self.status,
                                                    self.scratch, in_offset=off)
            # read each encoding once (every byte verified) and write the decoded object once;
            # without Bao only the primaries' bytes are read
            self.alg_bytes = count * (blen + n) if lv & 4 else count * 2 * n
            if lv & 4:
                self.kernel = (f"decode() level {lv} on the device: bao_chunk_kernel_verify (every chunk and "
                               f"parent verified{', only the 4 data shards written' if lv & 8 else ''}) + parent "
                               "check levels")
            else:
                self.kernel = f"decode() level {lv} on the device: primaries' bytes copied"
            self.kernel_sym = "pipeline"
        elif args.mode == "scrub":
            import numpy as np
            import carbonado_amd as ca
            host = self.inp.cpu().numpy()
            del self.inp
            torch.cuda.empty_cache()
            self.inp = torch.from_numpy(host)
            self.encs, self.hashes_h, self.infos, self.bads = [], [], [], []
            for o in range(count):
                enc, h, info = ca.encode(b"", host[o], 12)
                bad = np.frombuffer(enc, np.uint8).copy()
                bad[scrub_corrupt_offset(n, o)] ^= 0x40
                self.encs.append(enc)
                self.hashes_h.append(h)
                self.infos.append(info)
                self.bads.append(bad)
            self.fixed = [None] * count

            def step():
                for o in range(count):
                    self.fixed[o] = ca.decoding.scrub(self.bads[o], self.hashes_h[o], self.infos[o])
            self.step = step
            self.blen = len(self.encs[0])
            self.alg_bytes = count * 2 * self.blen  # PCIe: the damaged stream up, the repaired stream down
            self.h2d_bytes, self.d2h_bytes = count * self.blen, count * self.blen
            self.kernel = ("scrub(): H2D + bao node check + zfec decode of intact shards + fused re-encode + D2H, "
                           "one call per object (host API)")
            self.kernel_sym = "scrub"
        elif args.mode == "scrub-batch":
            zlen = m * C
            self.zlen = zlen
            self.blen = blen = L.chip_bao_encoded_len(zlen)
            self.soff = soff = args.stream_offset
            row = (soff + blen + 255) // 256 * 256
            self.enc = batch_buf((count, row), "enc")
            self.hashes = torch.empty((count, 32), dtype=torch.uint8, device=dev)
            esc = device.encode_scratch(12, n, count, dev)
            _, info = device.encode_batch(12, self.inp, n, self.enc, self.hashes, esc, out_offset=soff)
            torch.cuda.synchronize()
            del esc
            self.pad = info.padding_len
            self.sample0 = self.inp[0].cpu().numpy().tobytes()
            self.inp = self.inp[:1]  # only object 0's input is kept (the oracle check)
            torch.cuda.empty_cache()
            every = max(1, args.scrub_every)
            self.damaged = list(range(every // 2 % count, count, every))
            self.orig = {o: self.enc[o, soff:soff + blen].clone() for o in self.damaged}
            for o in self.damaged:  # one byte of a data shard's chunk
                off = scrub_corrupt_offset(n, o)
                self.enc[o, soff + off] ^= 0x40
            self.out = batch_buf((count, row), "out")
            self.scratch = device.scrub_scratch(blen, count, dev)
            self.scrub_status = None

            def step():
                self.scrub_status = device.scrub_batch(self.enc, blen, self.hashes, self.pad, C, self.out,
                                                       self.scratch, offset=soff)
            self.step = step
            # VALU: every chunk and parent of every stream re-hashed (node check), plus the
            # damaged streams' re-encode (zfec + bao); HBM bytes: the streams read once
            self.scrub_comps = (count + len(self.damaged)) * (zlen // 64 + zlen // 1024 - 1)
            self.alg_bytes = count * blen + len(self.damaged) * (2 * blen + zlen)
            self.kernel = (f"scrub() of {count} device-resident level-12 streams, {len(self.damaged)} damaged: "
                           "bao_chunk_kernel_check + bao_parent_check_kernel (every node), scrub_mask_kernel, "
                           "then per damaged stream gather + zfec decode + fused re-encode")
            self.kernel_sym = "scrub-batch"
        elif args.mode == "hasher":
            import numpy as np
            from carbonado_amd.utils import BaoHasher
            host = self.inp.cpu().numpy().reshape(-1)
            del self.inp
            torch.cuda.empty_cache()
            self.inp = torch.from_numpy(host.reshape(count, n))
            piece = 4 << 20
            self.pieces = [host[i:i + piece] for i in range(0, host.size, piece)]
            self.digest = None

            self.finalize_ms = []

            def step():
                h = BaoHasher()
                for p in self.pieces:
                    h.update(p)
                t0 = time.perf_counter()
                self.digest = bytes(h.finalize())
                self.finalize_ms.append((time.perf_counter() - t0) * 1e3)
            self.step = step
            self.alg_bytes = host.size  # PCIe: the content up (the hash comes back)
            self.h2d_bytes, self.d2h_bytes = host.size, 0
            self.kernel = ("BaoHasher: H2D appends into a grow-only HBM buffer, chunk CVs hashed during update() "
                           "(64-chunk units with bytes past them), finalize(): last chunks + slot layout + parent "
                           "levels")
            self.kernel_sym = "hasher"
        elif args.mode == "file":
            import hashlib
            import tempfile
            from carbonado_amd import file as cfile
            base = Path(args.file_dir or os.path.join(tempfile.gettempdir(), "carbonado_files"))
            self.in_dir, self.out_dir = base / f"in{rank}", base / f"out{rank}"
            import shutil
            for d in (self.in_dir, self.out_dir):
                shutil.rmtree(d, ignore_errors=True)
                d.mkdir(parents=True)
            host = self.inp.cpu().numpy()
            del self.inp
            torch.cuda.empty_cache()
            self.inp = torch.from_numpy(host)
            self.paths = []
            for o in range(count):
                p = self.in_dir / f"object{o:05d}.bin"
                host[o].tofile(p)
                self.paths.append(p)
            self.sk = hashlib.sha256(b"carbonado-amd bench file key").digest()
            lv = args.level

            self.file_stats = {}
            self.file_step = 0

            def step():
                # each step writes new files into a directory of its own, as an archive
                # would (rewriting the same names measures page-cache truncation instead)
                d = self.out_dir / f"s{self.file_step}"
                d.mkdir(exist_ok=True)
                self.file_step += 1
                self.file_stats = {}
                self.results = cfile.encode_files(self.paths, d, self.sk, lv, slice_objects=args.file_slice,
                                                  host_threads=args.host_threads, fsync=args.fsync,
                                                  io_threads=args.io_threads,
                                                  stats=self.file_stats)
            self.step = step
            step()
            self.final_len = max(r[1].output_len for r in self.results) + 160
            self.alg_bytes = count * (n + self.final_len)  # PCIe bytes: H2D input + D2H encoding
            self.h2d_bytes, self.d2h_bytes = count * n, count * self.final_len
            self.kernel = (f"file::encode level {lv}: read files -> pinned -> H2D + zfec/bao kernels (+ host "
                           f"snap/ecies) -> D2H -> header (BIP-340) + body written{' + fsync' if args.fsync else ''}")
            self.kernel_sym = "file"
        elif args.mode == "e2e-decode":
            import hashlib
            from carbonado_amd.encoding import public_key
            cap = L.chip_encode_max_len(n)
            lv, slots = args.level, args.slots
            self.sk = hashlib.sha256(b"carbonado-amd bench receiver").digest()
            self.pub = public_key(self.sk) if lv & 1 else b""
            h_in = torch.empty((count, n), dtype=torch.uint8, pin_memory=True)
            h_in.copy_(self.inp.cpu())
            del self.inp
            torch.cuda.empty_cache()
            self.inp = h_in
            self.h_enc = torch.empty((count, cap), dtype=torch.uint8, pin_memory=True)
            self.h_hash = torch.empty((count, 32), dtype=torch.uint8, pin_memory=True)
            self.enc_len, infos = device.encode_host_batch(lv, h_in, n, self.h_enc, self.h_hash, slots,
                                                           pubkey=self.pub, host_threads=args.host_threads)
            self.pads = [i.padding_len for i in infos]
            self.h_out = torch.empty((count, n + 1024), dtype=torch.uint8, pin_memory=True)

            def step():
                self.dec_len, self.dec_status = device.decode_host_batch(
                    lv, self.h_enc, self.enc_len, self.h_hash, self.pads, self.h_out, secret_key=self.sk,
                    nslots=slots, slice_bytes=args.slice_mib << 20, host_threads=args.host_threads)
            self.step = step
            step()
            self.alg_bytes = count * (max(self.enc_len) + n)  # PCIe bytes: H2D encoding + D2H content
            self.h2d_bytes, self.d2h_bytes = count * max(self.enc_len), count * n
            stages = ("ecies + " if lv & 1 else "") + ("unsnap + " if lv & 2 else "")
            host = f" + host {stages[:-3]} on {args.host_threads} threads" if stages else ""
            self.kernel = f"decode() level {lv}: H2D + bao verify kernels + D2H{host}, {slots} slots"
            self.kernel_sym = "e2e"
        elif args.mode == "e2e":
            cap = L.chip_encode_max_len(n)
            self.h_in = torch.empty((count, n), dtype=torch.uint8, pin_memory=True)
            self.h_in.copy_(self.inp.cpu())
            del self.inp
            torch.cuda.empty_cache()
            self.inp = self.h_in  # object 0 for verification lives on the host
            self.h_out = torch.empty((count, cap), dtype=torch.uint8, pin_memory=True)
            self.h_hash = torch.empty((count, 32), dtype=torch.uint8, pin_memory=True)
            self.final_len = cap
            lv, slots = args.level, args.slots
            # ECIES (level & 1): a fixed receiver key; the ephemeral key and
            # nonce of every object are injected so object 0 can be checked
            # bit for bit against the C oracle.
            self.pub = b""
            self.eph = self.nonce = None
            if lv & 1:
                import hashlib
                import numpy as np
                from carbonado_amd.encoding import public_key
                self.pub = public_key(hashlib.sha256(b"carbonado-amd bench receiver").digest())
                self.eph = np.stack([np.frombuffer(hashlib.sha256(b"eph%d" % o).digest(), np.uint8)
                                     for o in range(count)])
                self.nonce = np.stack([np.frombuffer(hashlib.sha256(b"nonce%d" % o).digest()[:16], np.uint8)
                                       for o in range(count)])

            def step():
                olens, _ = device.encode_host_batch(lv, self.h_in, n, self.h_out, self.h_hash, slots,
                                                    slice_bytes=args.slice_mib << 20,
                                                    pubkey=self.pub, ephemeral_sk=self.eph, nonce=self.nonce,
                                                    host_threads=args.host_threads)
                self.final_len = max(olens)
                self.olens = olens
            self.step = step
            step()
            self.alg_bytes = count * (n + self.final_len)  # PCIe bytes: H2D input + D2H encoding
            self.h2d_bytes, self.d2h_bytes = count * n, count * self.final_len
            self.copy_back = "whole stream"
            if lv & 12 == 12 and os.environ.get("CHIP_E2E_SPLIT", "1") != "0":
                # split copy-back (api_encode.cpp SplitGeo): the host writes each stream's
                # header and data-shard chunks (zl/2 bytes, zl = the bao header) itself;
                # the nodes between them and the tail cross PCIe
                host_made = sum(8 + int.from_bytes(self.h_out[o, :8].numpy().tobytes(), "little") // 2
                                for o in range(count))
                self.d2h_bytes = sum(self.olens) - host_made + 32 * count
                self.copy_back = (f"split: host writes header + data chunks ({host_made // count} B/object), "
                                  f"{self.d2h_bytes // count} B/object D2H")
                if lv & 3 and os.environ.get("CHIP_E2E_DIRECT", "1") != "0":
                    # direct: the host-stage output is written into the stream's data region in
                    # host memory, and that region [0, t0) is what crosses H2D
                    zls = [int.from_bytes(self.h_out[o, :8].numpy().tobytes(), "little") for o in range(count)]
                    self.h2d_bytes = sum(bao_data_region_len(z // 1024) for z in zls)
                    self.copy_back += f"; direct: {self.h2d_bytes // count} B/object H2D (the data region)"
                self.alg_bytes = self.h2d_bytes + self.d2h_bytes
            stages = ("snap + " if lv & 2 else "") + ("ecies + " if lv & 1 else "")
            host = f"host {stages[:-3]} on {args.host_threads} threads + " if stages else ""
            self.kernel = f"encode() level {lv}: {host}H2D + gf_apply + bao kernels + D2H, {slots} slots"
            self.kernel_sym = "e2e"
        elif args.mode == "bao-decode":
            blen = L.chip_bao_encoded_len(n)
            off = args.bao_stream_offset
            self.enc = batch_buf((count, (off + blen + 255) // 256 * 256), "enc")
            self.hashes = torch.empty((count, 32), dtype=torch.uint8, device=dev)
            self.scratch = device.bao_scratch(n, count, dev)
            device.bao_encode_batch(self.inp_full, n, self.enc, self.hashes, self.scratch, out_offset=off)
            self.out = batch_buf((count, n), "out")
            self.status = torch.full((count,), -1, dtype=torch.int32, device=dev)
            self.step = lambda: device.bao_decode_batch(self.enc, n, self.hashes, self.out, self.status, self.scratch,
                                                        in_offset=off)
            if off:
                self.soff = off
            self.alg_bytes = count * (blen + n)  # read the stream, write the content
            self.kernel = "bao_chunk_kernel_verify (verify + content) + bao_parent_kernel<1> levels"
            self.kernel_sym = "bao_chunk_kernel_verify"
        else:
            self.blen = blen = L.chip_bao_encoded_len(n)
            self.soff = off = args.bao_stream_offset
            self.out = batch_buf((count, (off + blen + 255) // 256 * 256), "out")
            self.hashes = torch.empty((count, 32), dtype=torch.uint8, device=dev)
            self.scratch = device.bao_scratch(n, count, dev)
            self.step = lambda: device.bao_encode_batch(self.inp_full, n, self.out, self.hashes, self.scratch,
                                                        out_offset=off)
            self.alg_bytes = count * (n + blen)
            fused = n >= 65536 and os.environ.get("CHIP_FUSED", "1") != "0"
            self.kernel = ("bao_content_fused_kernel (K13 content mode: chunk hashing + tree levels 1-3, 64 consecutive "
                           "chunks per wave) + bao_parent_kernel levels from level 4"
                           + ("" if n % 65536 == 0 else " + bao_tail_kernel (the last < 64 chunks)") if fused else
                           "bao_chunk_kernel_encode + bao_parent_kernel levels")
            self.kernel_sym = "bao_content_fused_kernel" if fused else "bao_chunk_kernel_encode"
        torch.cuda.synchronize()

    def _scatter_inputs(self, rank: int, world: int) -> float:
        """Rank 0 generates all world*count objects and scatters them (RCCL)."""
        grp = dist.new_group(backend="nccl", timeout=datetime.timedelta(seconds=180))  # a stuck collective ends the run, not the node's slot
        full = None
        if rank == 0:
            full = torch.empty((world * self.count, self.n), dtype=torch.uint8, device=self.dev)
            fill_random(full, SEED)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        chunks = [c.contiguous() for c in full.chunk(world, dim=0)] if rank == 0 else None
        dist.scatter(self.inp, chunks, src=0, group=grp)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        del full, chunks
        torch.cuda.empty_cache()
        return el

    def scatter_sample(self, rank: int, world: int, gib: float) -> dict:
        """N > 1: rank 0 scatters `gib` GiB to every rank over RCCL (xGMI),
        once, timed between barriers; the inputs of the timed steps are
        generated on each rank, so this only shows RCCL seeing N ranks and
        the per-link rate of the input-staging collective."""
        grp = dist.new_group(backend="nccl", timeout=datetime.timedelta(seconds=180))  # a stuck collective ends the run, not the node's slot
        res = scatter_sample(rank, world, int(gib * 2**30), self.dev, grp)
        torch.cuda.empty_cache()
        res["how"] = ("RCCL scatter (backend nccl) from rank 0 over xGMI, outside the timed region; the timed "
                      "steps' inputs are generated on each rank")
        return res

    def time_steps(self, steps: int, warmup: int, world: int, step=None):
        step = step or self.step
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            evs[i][0].record(stream)  # the library launches on torch's current stream
            step()
            evs[i][1].record(stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier(world)
        return t1 - t0, [a.elapsed_time(b) for a, b in evs]

    def verify_all(self, threads: int = 16):
        """SURVEY.md 8d cfg2 check: all objects bit-exact, compared through
        BLAKE3 digests of the m shards (computed on the device by the bao
        kernels, hash-only) against oracle/carbonado_oracle.c's zfec + BLAKE3
        of the same inputs (ctypes releases the GIL: the checks run in
        parallel on `threads` host threads).  cfg3 (decode): every decoded
        object equals its resident input, compared on the device.  cfg4
        (e2e): every object's encoding in host memory equals the C oracle's
        encode() (orc_encode_full with the same injected ECIES values)."""
        if self.args.mode == "decode":
            return self._verify_all_decode()
        if self.args.mode == "e2e":
            return self._verify_all_e2e(threads)
        if self.args.mode in ("bao-decode", "pipeline-decode"):
            return self._verify_all_bao_decode()
        if self.args.mode == "e2e-decode":
            return self._verify_all_e2e_decode(threads)
        if self.args.mode in ("scrub", "scrub-batch", "file"):
            return self._verify_all_repaired(threads)
        from concurrent.futures import ThreadPoolExecutor
        from carbonado_amd import device
        from oracle import oracle as O
        t0 = time.perf_counter()
        count, k, m, C = self.count, self.k, self.m, self.C
        pipeline = self.args.mode == "pipeline"
        bao = self.args.mode == "bao"
        olen = self.blen if (pipeline or bao) else m * C  # bytes of each object's output
        digests = torch.empty((count, 32), dtype=torch.uint8, device=self.dev)
        off = getattr(self, "soff", 0) if (pipeline or bao) else 0
        if off:  # streams 8-B aligned in their rows: hashed from 16-B aligned copies, 64 rows at a time
            scratch = device.bao_scratch(olen, 64, self.dev)
            for o0 in range(0, count, 64):
                o1 = min(count, o0 + 64)
                rows = self.out[o0:o1, off:off + olen].contiguous()
                device.bao_encode_batch(rows, olen, None, digests[o0:o1], scratch)
                del rows
        else:
            scratch = device.bao_scratch(olen, count, self.dev)
            device.bao_encode_batch(self.out, olen, None, digests, scratch)
        torch.cuda.synchronize()
        gpu = digests.cpu().numpy()
        hashes = self.hashes.cpu().numpy() if (pipeline or bao) else None
        del scratch
        host_in = self.inp.cpu().numpy()

        def check(o):
            if bao:  # encoding::bao (encoding.rs:38-44): the stream and its hash
                stream, h = O.bao_encode(host_in[o].tobytes())
                return O.blake3(stream) == gpu[o].tobytes() and h == hashes[o].tobytes()
            if pipeline:
                enc, h, _ = O.encode(host_in[o].tobytes(), self.args.level)
                return O.blake3(enc) == gpu[o].tobytes() and (not self.args.level & 4 or
                                                              h == hashes[o].tobytes())
            return O.blake3(O.zfec_encode(host_in[o], k, m)[0]) == gpu[o].tobytes()
        with ThreadPoolExecutor(threads) as ex:
            oks = list(ex.map(check, range(count)))
        bad = [o for o, ok in enumerate(oks) if not ok]
        return {"ok": not bad, "objects": count, "mismatched": bad[:16], "seconds": round(time.perf_counter() - t0, 1),
                "how": (f"BLAKE3 of each object's bao stream on the GPU + its bao hash vs the oracle's bao encode "
                        f"(stream BLAKE3 + root hash) on {threads} threads" if bao else
                        f"BLAKE3 of each object's level-{self.args.level} encoding on the GPU + its bao hash vs the "
                        f"oracle's encode() + BLAKE3 on {threads} threads" if pipeline else
                        f"BLAKE3 of each object's {m} shards on the GPU vs oracle zfec + BLAKE3 on {threads} threads")}

    def _verify_all_decode(self):
        """decoding::zfec of every object (decoding.rs:21-51): the k data
        shards' first n bytes equal the object's input, both resident in HBM
        (compared 64 objects at a time)."""
        t0 = time.perf_counter()
        n, bad = self.n, []
        for o0 in range(0, self.count, 64):
            o1 = min(self.count, o0 + 64)
            diff = (self.out[o0:o1, :n] != self.inp[o0:o1, :n]).any(dim=1)
            bad += [o0 + int(i) for i in torch.nonzero(diff).flatten().tolist()]
        torch.cuda.synchronize()
        return {"ok": not bad, "objects": self.count, "mismatched": bad[:16],
                "seconds": round(time.perf_counter() - t0, 1),
                "how": "every decoded object's n bytes vs its resident input, compared on the device"}

    def _verify_all_bao_decode(self):
        """decoding::bao of every object (decoding.rs:53-60), or decode() at a
        device-only level (decoding.rs:80-114) for pipeline-decode: every
        status is 0 (every node verified) and every decoded content equals
        the object's resident input, compared on the device 64 objects at a
        time."""
        t0 = time.perf_counter()
        n, bad = self.n, []
        st = self.status.cpu().tolist()
        bad_status = [o for o, v in enumerate(st) if v != 0]
        for o0 in range(0, self.count, 64):
            o1 = min(self.count, o0 + 64)
            diff = (self.out[o0:o1, :n] != self.inp[o0:o1, :n]).any(dim=1)
            bad += [o0 + int(i) for i in torch.nonzero(diff).flatten().tolist()]
        torch.cuda.synchronize()
        return {"ok": not bad and not bad_status, "objects": self.count, "mismatched": bad[:16],
                "bad_status": bad_status[:16], "seconds": round(time.perf_counter() - t0, 1),
                "how": "every object's status == 0 and its decoded content vs its resident input, on the device"}

    def _verify_all_e2e_decode(self, threads: int):
        """decode() of every object from host memory (decoding.rs:80-114):
        every status is 0, every decoded length is n and every decoded
        object's bytes equal its input (pinned host memory, compared on
        `threads` host threads; numpy releases the GIL)."""
        from concurrent.futures import ThreadPoolExecutor
        import numpy as np
        t0 = time.perf_counter()
        n, got, want = self.n, self.h_out.numpy(), self.inp.numpy()
        bad_status = [o for o, v in enumerate(self.dec_status) if v != 0]

        def check(o):
            return self.dec_len[o] == n and np.array_equal(got[o, :n], want[o])
        with ThreadPoolExecutor(threads) as ex:
            oks = list(ex.map(check, range(self.count)))
        bad = [o for o, ok in enumerate(oks) if not ok]
        return {"ok": not bad and not bad_status, "objects": self.count, "mismatched": bad[:16],
                "bad_status": bad_status[:16], "seconds": round(time.perf_counter() - t0, 1),
                "how": f"every object's status == 0, decoded length == n and decoded bytes (host memory) vs its "
                       f"input, on {threads} threads"}

    def _verify_all_repaired(self, threads: int):
        """scrub() (decoding.rs:159-212) and file::decode (file.rs:395-440)
        of every object: scrub — every repaired stream equals the intact
        encoding and every status is what the damage calls for; file — every
        written file decodes (header signature checked, the device decode
        path) back to its input."""
        t0 = time.perf_counter()
        mode = self.args.mode
        if mode == "scrub":
            bad = [o for o in range(self.count) if self.fixed[o] != self.encs[o]]
            how = "every object's scrub() output vs its intact level-12 encoding (host API)"
            return {"ok": not bad, "objects": self.count, "mismatched": bad[:16],
                    "seconds": round(time.perf_counter() - t0, 1), "how": how}
        if mode == "scrub-batch":
            st = self.scrub_status
            want = [0 if o in self.orig else 12 for o in range(self.count)]
            bad_status = [o for o in range(self.count) if st is None or st[o] != want[o]]
            so = getattr(self, "soff", 0)
            bad = [o for o in self.orig if not torch.equal(self.out[o, so:so + self.blen], self.orig[o])]
            return {"ok": not bad and not bad_status, "objects": self.count, "repaired": len(self.orig),
                    "mismatched": bad[:16], "bad_status": bad_status[:16],
                    "seconds": round(time.perf_counter() - t0, 1),
                    "how": "every object's status (damaged: 0 = repaired, intact: 12 = UnnecessaryScrub) and every "
                           "repaired stream vs its pre-damage bytes, on the device"}
        from concurrent.futures import ThreadPoolExecutor
        from carbonado_amd import file as cfile
        host = self.inp.numpy()

        def check(o):
            path, info = self.results[o]
            hdr, back = cfile.decode(self.sk, path.read_bytes())
            return (back == host[o].tobytes() and hdr.format == self.args.level and
                    hdr.encoded_len == info.output_len)
        with ThreadPoolExecutor(min(threads, 4)) as ex:
            oks = list(ex.map(check, range(self.count)))
        bad = [o for o, ok in enumerate(oks) if not ok]
        return {"ok": not bad, "objects": self.count, "mismatched": bad[:16],
                "seconds": round(time.perf_counter() - t0, 1),
                "how": f"every written file read back, file::decode (header + signature + decode() on the device) "
                       f"vs its input, on {min(threads, 4)} threads"}

    def _verify_all_e2e(self, threads: int):
        """encode() of every object (encoding.rs:86-172) against the C oracle
        on `threads` host threads: at levels with host stages
        orc_encode_full with the object's injected ephemeral key and nonce
        (host_oracle.c), else the device-stage oracle; bytes and hash."""
        from concurrent.futures import ThreadPoolExecutor
        from oracle import oracle as O
        t0 = time.perf_counter()
        lv, host_in = self.args.level, self.h_in.numpy()
        out, hashes = self.h_out.numpy(), self.h_hash.numpy()

        def check(o):
            if lv & 3:
                eph = self.eph[o].tobytes() if self.eph is not None else bytes(32)
                nonce = self.nonce[o].tobytes() if self.nonce is not None else bytes(16)
                enc, h, _ = O.c_encode_full(host_in[o].tobytes(), lv, self.pub, eph, nonce)
            else:
                enc, h, _ = O.encode(host_in[o].tobytes(), lv)
            return (self.olens[o] == len(enc) and out[o, :len(enc)].tobytes() == enc and
                    (not lv & 4 or hashes[o].tobytes() == h))
        with ThreadPoolExecutor(threads) as ex:
            oks = list(ex.map(check, range(self.count)))
        bad = [o for o, ok in enumerate(oks) if not ok]
        return {"ok": not bad, "objects": self.count, "mismatched": bad[:16],
                "seconds": round(time.perf_counter() - t0, 1),
                "how": (f"every object's level-{lv} encoding (host memory) and hash vs the C oracle's "
                        f"{'orc_encode_full (same injected ECIES values)' if lv & 3 else 'encode()'} on "
                        f"{threads} threads")}

    def time_aliased(self, steps: int, warmup: int, world: int):
        """the same encode with the data shards aliased (in
        place: the input already sits in the first n bytes of each output
        slot, only parity is written).  Reported next to, not instead of, the
        48 MiB/object figure."""
        from carbonado_amd import device
        n, k, m = self.n, self.k, self.m
        self.out[:, :n].copy_(self.inp)
        step = lambda: device.zfec_encode_batch(self.out, n, self.out, k, m)  # noqa: E731
        el, ms = self.time_steps(steps, warmup, world, step)
        from oracle import oracle as O
        ok = self.out[0].cpu().numpy().tobytes() == O.zfec_encode(self.inp[0].cpu().numpy().tobytes(), k, m)[0]
        return el, ms, ok

    def box_ceiling(self, reps: int = 5) -> dict:
        """What this box's HBM gives the headline's access pattern on the
        same buffers: chip_hbm_pattern_batch_dev (the encode's loads, stores,
        grid and run queue, no GF arithmetic) timed with HIP events, one
        warm-up + `reps` launches, outside the timed region and after every
        check (it overwrites the output).  GPU clocks and partition modes are
        sampled from sysfs while it runs."""
        from carbonado_amd import device
        n, k, m = self.n, self.k, self.m
        launch = lambda: device.hbm_pattern_batch(self.inp_full, n, self.out, k, m)  # noqa: E731
        launch()
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        sampler = ClockSampler(self.dev)
        sampler.start()
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            launch()
            b.record(stream)
            b.synchronize()
            ms.append(a.elapsed_time(b))
        clocks = sampler.stop()
        ms.sort()
        med = ms[len(ms) // 2]
        ach = self.alg_bytes / (med * 1e-3) / 1e9
        return {"GBps": round(ach, 1), "frac_of_peak": round(ach / HBM_PEAK_GBS, 4), "median_ms": round(med, 4),
                "min_ms": round(ms[0], 4), "launches": reps, "clocks": clocks,
                "how": f"chip_hbm_pattern_batch_dev: the encode's {k}-read/{m}-write pattern on the same buffers, "
                       f"grid and run queue without the GF arithmetic, HIP events, median of {reps}"}

    def verify_object0(self):
        from oracle import oracle as O
        sample = self.inp[0].cpu().numpy().tobytes()
        if self.args.mode == "encode":
            ok = self.out[0].cpu().numpy().tobytes() == O.zfec_encode(sample, self.k, self.m)[0]
        elif self.args.mode == "e2e":
            lv = self.args.level
            if lv & 3:
                eph = self.eph[0].tobytes() if self.eph is not None else bytes(32)
                nonce = self.nonce[0].tobytes() if self.nonce is not None else bytes(16)
                enc, h, _ = O.c_encode_full(sample, lv, self.pub, eph, nonce)
            else:
                enc, h, _ = O.encode(sample, lv)
            ok = (self.h_out[0, :len(enc)].numpy().tobytes() == enc and
                  self.h_hash[0].numpy().tobytes() == h)
        elif self.args.mode == "decode":
            ok = self.out[0, :self.n].cpu().numpy().tobytes() == sample
        elif self.args.mode == "bao-decode":
            # every object verified (status 0) and object 0's content is the input;
            # the stream itself is checked against the oracle's bao encoding
            blen = _lib_len(self.n)
            ok = (bool((self.status == 0).all()) and self.out[0].cpu().numpy().tobytes() == sample and
                  self.enc[0, :blen].cpu().numpy().tobytes() == O.bao_encode(sample)[0])
        elif self.args.mode == "scrub":
            ok = all(self.fixed[o] == self.encs[o] for o in range(self.count))
        elif self.args.mode == "scrub-batch":
            # intact streams: UnnecessaryScrub (12); damaged: repaired (0) to the original stream;
            # object 0's stream is the oracle's encode()
            sample = self.sample0
            st = self.scrub_status
            want = [0 if o in self.orig else 12 for o in range(self.count)]
            ok = (st is not None and list(st) == want and
                  all(torch.equal(self.out[o, self.soff:self.soff + self.blen], self.orig[o]) for o in self.orig) and
                  self.enc[0, self.soff:self.soff + self.blen].cpu().numpy().tobytes() == O.encode(sample, 12)[0])
        elif self.args.mode == "hasher":
            ok = self.digest == O.blake3(self.inp.numpy().reshape(-1))
        elif self.args.mode == "pipeline":
            enc, h, _ = O.encode(sample, self.args.level)
            ok = (self.out[0, self.soff:self.soff + self.blen].cpu().numpy().tobytes() == enc and
                  (self.hashes[0].cpu().numpy().tobytes() == h if self.args.level & 4 else True))
        elif self.args.mode == "e2e-decode":
            ok = self.h_out[0, :self.n].numpy().tobytes() == sample
        elif self.args.mode == "pipeline-decode":
            # object 0: status 0, decoded bytes equal the input, and its encoding is the
            # oracle's encode() (every object's status and bytes: verified_all_objects)
            enc, h, _ = O.encode(sample, self.args.level)
            ok = (int(self.status[0]) == 0 and torch.equal(self.out[0, :self.n], self.inp[0, :self.n]) and
                  self.enc[0, self.soff:self.soff + self.blen].cpu().numpy().tobytes() == enc)
        elif self.args.mode == "file":
            from carbonado_amd import file as cfile
            path, info = self.results[0]
            hdr, back = cfile.decode(self.sk, path.read_bytes())
            ok = back == sample and hdr.format == self.args.level and hdr.encoded_len == info.output_len
        else:
            ok = self.hashes[0].cpu().numpy().tobytes() == O.blake3(sample)
        return ok, sample


def scatter_sample(rank: int, world: int, per: int, dev, group) -> dict:
    """Rank 0 scatters `per` bytes to every rank once (after one warm-up
    scatter), timed between barriers; every rank checks its slice (a
    counter pattern, so each rank knows what it must receive)."""
    gpu = dev.type == "cuda"
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    local = torch.empty(per, dtype=torch.uint8, device=dev)
    chunks = None
    base = torch.arange(256, dtype=torch.uint8, device=dev).repeat(per // 256 + 1)[:per]

    def slice_of(r):  # rank r's bytes: a byte ramp shifted by 37 r (uint8 arithmetic wraps)
        return base + (37 * r) % 256
    if rank == 0:
        chunks = [slice_of(r) for r in range(world)]
    dist.scatter(local, chunks, src=0, group=group)  # warm the communicator
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    dist.scatter(local, chunks, src=0, group=group)
    sync()
    el = max_over_ranks(time.perf_counter() - t0)
    oks = [None] * world
    dist.all_gather_object(oks, bool(torch.equal(local, slice_of(rank))))
    del local, chunks, base
    return {"ranks": world, "bytes_per_rank": per, "seconds": round(el, 4),
            "GiB_per_s_total": round((world - 1) * per / el / 2**30, 2),
            "GiB_per_s_per_receiver": round(per / el / 2**30, 2), "every_slice_ok": all(oks)}


class DryRun:
    """Control-plane rehearsal without a device (CPU gloo tests)."""

    def __init__(self, args, rank: int):
        n = int(args.object_mib * (1 << 20))
        self.rank = rank
        self.alg_bytes = args.objects * 3 * n
        self.kernel = self.kernel_sym = "dry-run"
        self.C = n // args.k
        self.scatter_s = None
        self.alloc_info = {"in": {"classes_found": 0, "classes_used": 0, "alloc_s": 0.0, "rank": rank}}
        self.scrub_comps = args.objects * (args.m * self.C // 64)  # scrub-batch's VALU count (placeholder)

    def box_ceiling(self, reps: int = 5) -> dict:
        """The box-ceiling record's keys with placeholder timings (no device)."""
        sampler = ClockSampler(None)
        sampler.start()
        clocks = sampler.stop()
        return {"GBps": 6000.0, "frac_of_peak": 0.75, "median_ms": 1.0, "min_ms": 1.0, "launches": reps,
                "clocks": clocks, "how": "dry run: placeholder timings, no device"}

    def time_steps(self, steps: int, warmup: int, world: int):
        barrier(world)
        t0 = time.perf_counter()
        time.sleep(0.01 * steps * (1 + 0.1 * self.rank))
        t1 = time.perf_counter()
        barrier(world)
        return t1 - t0, [10.0] * steps


def run_latency(args) -> None:
    """--mode latency: single-object call latency (the reference's real unit,
    a segment of about 1 MB, README.md:107-111).  The GPU side is
    tools/abi_latency (C++ over the C-ABI only, no Python in the timed
    calls); the cpu_baseline leg times oracle/carbonado_oracle.c (+
    host_oracle.c at levels with Snappy/Ecies) on one thread per call for
    the same rows.  One JSON line; `value` = level 12 at 1 MiB, lib encode."""
    import statistics
    import subprocess

    import numpy as np
    tool = ROOT / "tools" / "abi_latency"
    if not tool.exists():
        subprocess.run(["g++", "-std=c++17", "-O2", str(ROOT / "tools" / "abi_latency.cpp"), "-I" + str(ROOT / "include"),
                        "-L" + str(ROOT / "carbonado_amd" / "lib"), "-lcarbonado_hip",
                        "-Wl,-rpath," + str(ROOT / "carbonado_amd" / "lib"), "-o", str(tool)], check=True)
    r = subprocess.run([str(tool), str(args.latency_reps), args.latency_levels, args.latency_sizes],
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise SystemExit("abi_latency failed: " + r.stdout[-2000:] + r.stderr[-2000:])
    cols = ["lib_enc", "lib_dec", "patch_enc", "patch_dec", "r5_enc", "r5_dec"]
    rows = []
    for line in r.stdout.splitlines():
        f = line.split()
        if len(f) == 8 and f[0].isdigit():
            row = {"level": int(f[0]), "bytes": int(f[1])}
            row.update({c: (None if v == "-" else float(v)) for c, v in zip(cols, f[2:])})
            rows.append(row)
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import host_oracle as H
        from oracle import oracle as O
        sk = H.sha256(b"latency receiver")
        pub, eph, nonce = H.public_key(sk), H.sha256(b"latency eph"), H.sha256(b"latency nonce")[:16]
        rng = np.random.default_rng(5)
        for row in rows:
            lv, nb = row["level"], row["bytes"]
            d = rng.integers(0, 256, nb, dtype=np.uint8).tobytes()
            te, td = [], []
            budget = time.perf_counter() + 6.0  # bounded sample per row
            for _ in range(5):
                t0 = time.perf_counter()
                if lv & 3:
                    enc, h, info = O.c_encode_full(d, lv, pub, eph, nonce)
                else:
                    enc, h, info = O.encode(d, lv)
                t1 = time.perf_counter()
                if lv & 3:  # all in C: bao -> zfec, then ecies -> snap (host_oracle.c)
                    cur = O.decode(h, enc, info["padding_len"], lv & 12) if lv & 12 else enc
                    if lv & 1:
                        cur = O.c_ecies_decrypt(sk, cur)
                    back = O.c_snap_decompress(cur, nb + 1024) if lv & 2 else cur
                else:
                    back = O.decode(h, enc, info["padding_len"], lv) if lv & 12 else enc
                t2 = time.perf_counter()
                assert back == d
                te.append((t1 - t0) * 1e6)
                td.append((t2 - t1) * 1e6)
                if time.perf_counter() > budget:
                    break
            row["cpu_enc"] = round(statistics.median(te), 1)
            row["cpu_dec"] = round(statistics.median(td), 1)
        cpu = {"unit": "us per call", "cores": 1, "kind": "port",
               "sample": "median of up to 5 calls per row, 6 s per row at most: encode() and decode() through "
                         "oracle/carbonado_oracle.c (+ host_oracle.c for the Snappy/Ecies stages), all C"}
    head = next((x for x in rows if x["level"] == 12 and x["bytes"] == 1 << 20), rows[0] if rows else None)
    print(json.dumps({
        "metric": "single_object_latency", "value": head["lib_enc"] if head else None, "unit": "us",
        "higher_is_better": False, "n_gpus": 1, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "one object per call through the C-ABI (tools/abi_latency)",
                   "levels": args.latency_levels, "sizes": args.latency_sizes, "reps": args.latency_reps},
        "columns": {"lib": "chip_encode / chip_decode, caller buffers reused",
                    "patch": "carbonado-hip/reroute.patch's call sequence, a fresh buffer per output",
                    "r5": "round 5's patch at Zfec|Bao: zfec -> host Vec -> bao",
                    "cpu": "the C oracle, one thread (cpu_baseline)"},
        "rows": rows, "cpu_baseline": cpu}))


def main():
    args = parse()
    if args.mode == "latency":
        return run_latency(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, local = setup_dist(args)
    n = int(args.object_mib * (1 << 20))
    live = None
    under_profiler = any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or \
        "rocprofiler" in os.environ.get("LD_PRELOAD", "")
    if (not args.dry_run and not under_profiler and
            (args.live_pmc == "on" or (args.live_pmc == "auto" and pmc_kernel_sym(args) is not None))):
        # before this process touches the GPU; at N > 1 every rank profiles its own GPU in
        # parallel (a rehearsal with several ranks on one GPU skips it: they would share it)
        if world == 1:
            live = live_traffic(args, sys.argv[1:])
        elif visible_gpus_no_hip() >= world:
            live = live_traffic(args, sys.argv[1:], timeout_s=150.0, local_rank=local)
    wl = DryRun(args, rank) if args.dry_run else Workload(args, rank, local, world)
    scatter = None
    if world > 1 and args.dry_run and args.scatter_gib > 0:  # the same collective over gloo, CPU tensors
        scatter = scatter_sample(rank, world, 1 << 20, torch.device("cpu"), None)
        scatter["how"] = "dry run: the RCCL sample's scatter over gloo with 1 MiB CPU tensors per rank"
    if world > 1 and not args.dry_run and not args.scatter and args.scatter_gib > 0:
        if torch.cuda.device_count() >= world:
            try:  # outside the metric: an RCCL failure is reported, not fatal to the measurement
                scatter = wl.scatter_sample(rank, world, args.scatter_gib)
            except (RuntimeError, ValueError) as e:
                scatter = {"error": f"{type(e).__name__}: {e}"[:300]}
                torch.cuda.synchronize()
                barrier(world)
        else:  # a rehearsal with several ranks on one GPU: RCCL refuses two ranks on one device
            scatter = {"skipped": f"{world} ranks share {torch.cuda.device_count()} GPU(s); RCCL needs one GPU per rank"}
    elapsed, launch_ms = wl.time_steps(args.steps, args.warmup, world)
    max_elapsed = max_over_ranks(elapsed)
    rank_avg_ms = gather_floats(sum(launch_ms) / len(launch_ms), world)
    rank_live = [live]
    if world > 1:
        rank_live = [None] * world
        dist.all_gather_object(rank_live, live)
    rank_alloc = [getattr(wl, "alloc_info", {})]
    if world > 1:  # each rank's buffers' memory classes (placement differs per GPU)
        rank_alloc = [None] * world
        dist.all_gather_object(rank_alloc, getattr(wl, "alloc_info", {}))

    verified, sample = None, None
    if rank == 0 and not args.no_verify and not args.dry_run:
        verified, sample = wl.verify_object0()
    verified_all = None
    want_all = ((args.mode in ("encode", "decode", "e2e", "bao", "bao-decode", "pipeline-decode", "e2e-decode",
                               "scrub", "scrub-batch", "file") and not args.no_verify_all) or
                (args.mode == "pipeline" and args.verify_all))
    if want_all and not args.no_verify and not args.dry_run:
        # every rank checks its own objects (N > 1: the whole global set), rank 0 reports;
        # the host threads are split over the ranks (16 per GPU is the box's CPU share)
        mine = wl.verify_all(threads=verify_threads(world))
        if world > 1:
            every = [None] * world
            dist.all_gather_object(every, mine)
            verified_all = {"ok": all(v["ok"] for v in every), "objects": sum(v["objects"] for v in every),
                            "ranks": world, "mismatched_by_rank": {r: v["mismatched"] for r, v in enumerate(every)
                                                                   if v["mismatched"]},
                            "seconds_max": max(v["seconds"] for v in every), "how": mine["how"] + ", on every rank"}
        else:
            verified_all = mine
    if args.mode == "hasher" and verified is not None:
        # one stream over every object's bytes: the object-0 check above is already the whole input
        verified_all = {"ok": bool(verified), "objects": args.objects,
                        "how": "the hasher's one digest over all objects' bytes (4 MiB appends) vs the oracle's "
                               "BLAKE3 of the same bytes"}
    aliased = None
    if args.mode == "encode" and not args.dry_run and not args.no_aliased:
        a_el, a_ms, a_ok = wl.time_aliased(args.steps, args.warmup, world)
        aliased = (max_over_ranks(a_el), a_ms, a_ok)
    box = None
    if args.mode == "encode" and not args.no_box_ceiling and (args.k, args.m) in ((4, 8), (8, 16)):
        try:  # diagnostic, after the checks (it overwrites the outputs); every rank on its own GPU
            box = wl.box_ceiling()
        except Exception as e:
            box = {"error": f"{type(e).__name__}: {e}"[:300]}
        if world > 1:
            every = [None] * world
            dist.all_gather_object(every, box.get("GBps"))
            box["GBps_by_rank"] = every

    if rank == 0:
        k, m = args.k, args.m
        total_units = world * args.objects * n * args.steps
        value = total_units / max_elapsed / 2**30
        avg_ms = sum(launch_ms) / len(launch_ms)
        achieved = wl.alg_bytes / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = None, None
        if live and "bytes" in live:
            traffic = live["bytes"]
            traffic_src = (f"live: this run's rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the same workload "
                           f"(2 x FETCH_SIZE + WRITE_SIZE per launch, {live['seconds']} s)")
        else:
            traffic, traffic_src = measured_traffic(args.traffic_json, wl.kernel_sym, wl.alg_bytes)
            if live:
                traffic_src = f"{traffic_src or 'none'} (live PMC failed: {live['error']})"
            elif world > 1 and traffic_src:
                traffic_src = (f"committed fallback {traffic_src}: no live PMC at this N (ranks sharing a GPU, or "
                               "the passes are off)")
        if args.mode == "bao":
            workload = f"bao encode, {args.objects} x {args.object_mib:g} MiB objects per GPU"
        elif args.mode == "bao-decode":
            workload = f"bao decode (verify + content), {args.objects} x {args.object_mib:g} MiB objects per GPU"
        elif args.mode == "pipeline":
            workload = f"encode() level {args.level}, {args.objects} x {args.object_mib:g} MiB objects per GPU"
        elif args.mode == "pipeline-decode":
            workload = f"decode() level {args.level}, {args.objects} x {args.object_mib:g} MiB objects per GPU"
        elif args.mode == "scrub":
            workload = (f"scrub() of {args.objects} level-12 streams of {args.object_mib:g} MiB objects, one "
                        f"corrupted byte each, host buffers")
        elif args.mode == "scrub-batch":
            workload = (f"scrub() of {args.objects} device-resident level-12 streams of {args.object_mib:g} MiB "
                        f"objects per GPU, 1 in {args.scrub_every} damaged")
        elif args.mode == "hasher":
            workload = f"BaoHasher over {args.objects} x {args.object_mib:g} MiB in 4 MiB appends, host buffers"
        elif args.mode == "e2e":
            workload = (f"encode() level {args.level} host->HBM->host (pinned), {args.objects} x "
                        f"{args.object_mib:g} MiB objects per GPU")
        elif args.mode == "e2e-decode":
            workload = (f"decode() level {args.level} host->HBM->host (pinned), {args.objects} x "
                        f"{args.object_mib:g} MiB objects per GPU")
        elif args.mode == "file":
            workload = (f"file::encode level {args.level}: {args.objects} flat files of {args.object_mib:g} MiB "
                        f"on disk -> .c{args.level} files (header + body) on disk")
        else:
            workload = f"zfec {k}-of-{m} {args.mode}, {args.objects} x {args.object_mib:g} MiB objects per GPU"
        res = {
            "metric": METRIC if args.mode == "encode" and (k, m) == (4, 8) and n == 16 << 20 else
            (f"GiB/s {workload}" if args.mode.startswith("e2e") or args.mode in ("scrub", "hasher", "file")
             else f"GiB/s device-resident {workload}"),
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
            "config": {"workload": workload, "objects_per_gpu": args.objects, "object_bytes": n,
                       "chunk_len": wl.C, "k": k, "m": m, "global_objects": world * args.objects,
                       "parallelism": f"objects partitioned over {world} rank(s), no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": wl.kernel,
                         "alg_bytes_per_launch": wl.alg_bytes, "avg_launch_ms": round(avg_ms, 4),
                         "min_launch_ms": round(min(launch_ms), 4)},
            "verified_object0": verified,
        }
        if getattr(wl, "soff", 0):
            res["config"]["stream_offset"] = wl.soff
        if args.mode == "file":
            res["config"].update(file_slice=args.file_slice, io_threads=args.io_threads)
        if live and "bytes" in live:
            res["roofline"].update({"traffic_ratio": round(live["bytes"] / wl.alg_bytes, 4),
                                    "pmc_KiB_per_launch": {"FETCH_SIZE": live["FETCH_SIZE_KiB"],
                                                           "WRITE_SIZE": live["WRITE_SIZE_KiB"]},
                                    "pmc_kernel": live["kernel"]})
        if args.mode.startswith("e2e") or args.mode in ("scrub", "hasher", "file"):
            res["roofline"].update(pcie_roofline(getattr(wl, "h2d_bytes", 0), getattr(wl, "d2h_bytes", 0),
                                                 max_elapsed / args.steps, achieved))
            res["data"] = ("synthetic (uniform random bytes), pinned host buffers" if args.mode.startswith("e2e")
                           else "synthetic (uniform random bytes) in files on the box's local disk, read and "
                                "written through the page cache" if args.mode == "file"
                           else "synthetic (uniform random bytes), pageable host buffers (numpy / bytes)")
        pipe = args.mode in ("pipeline", "pipeline-decode", "scrub-batch")
        if args.mode in ("bao", "bao-decode", "scrub-batch") or (pipe and args.level & 4):
            # BLAKE3 compressions: one per 64-B block of content plus one per parent node;
            # 7 rounds x 8 G x 12 VALU lane-ops (a+b+m as one v_add3_u32).
            hashed = getattr(wl, "zlen", n) if pipe else n
            chunks = max(1, -(-hashed // 1024))
            comps = (wl.scrub_comps if args.mode == "scrub-batch" else
                     args.objects * (max(1, -(-hashed // 64)) + (chunks - 1)))
            ops = comps * 7 * 8 * 12
            tops = ops / (avg_ms * 1e-3) / 1e12
            hbm = res["roofline"]
            res["roofline"] = {"bound": "valu", "achieved": round(tops, 2), "peak": VALU_PEAK_TOPS, "unit": "TOPS",
                               "frac": round(tops / VALU_PEAK_TOPS, 4), "traffic": hbm["traffic"],
                               "traffic_source": hbm["traffic_source"], "kernel": wl.kernel,
                               "alg_ops_per_launch": ops, "hbm_achieved_GBps": hbm["achieved"],
                               "avg_launch_ms": hbm["avg_launch_ms"], "min_launch_ms": hbm["min_launch_ms"],
                               "peak_source": VALU_PEAK_SRC,
                               "peak_kind": "measured BLAKE3-loop ceiling (the product's own best compression "
                                            "loop), not a hardware figure",
                               "hw_valu_peak_TOPS": HW_VALU_PEAK_TOPS,
                               "frac_of_hw_valu": round(tops / HW_VALU_PEAK_TOPS, 4),
                               "note": "ops = 672 per BLAKE3 compression (content blocks + parents); peak = the "
                                       "measured compression ceiling x 672"
                                       + ("; achieved over the whole step (every kernel of the level)"
                                          if pipe else "")}
            for key in ("traffic_ratio", "pmc_KiB_per_launch", "pmc_kernel", "alg_bytes_per_launch"):
                if key in hbm:
                    res["roofline"][key] = hbm[key]
            if args.mode == "pipeline" and args.level & 12 == 12:
                # why K13 (encode() at Zfec|Bao) sits near 0.65 of the loop ceiling
                res["roofline"]["note_bound"] = (
                    "K13 bound (DESIGN.md section 3, K13): one launch per 256 x 16 MiB objects takes 3.61 ms = "
                    "1.36x the larger of its two halves measured alone (the BLAKE3 hashing ~2.6 ms; the GF(2^8) "
                    "products, loads and line stores ~2.65 ms): two waves per SIMD alternate between a VALU phase "
                    "and a store/LDS phase.  PMC traffic is 1.04x the algorithmic bytes, so nothing is wasted on "
                    "HBM; every lever measured (a third wave, two states per lane, role-split waves, priorities, "
                    "four orders) was neutral or slower (profiles/NOT_KEPT.md).  Recorded as the bound.")
            if pipe and "pmc_kernel" in hbm:
                res["roofline"]["note_traffic"] = ("traffic: the one dominant kernel's launch (the parent-level "
                                                   "kernels after it move a few % more); alg bytes: the whole step")
        if world > 1 and any(r and "bytes" in r for r in rank_live):
            res["roofline"]["per_rank_traffic_ratio"] = [
                round(r["bytes"] / wl.alg_bytes, 4) if r and "bytes" in r else None for r in rank_live]
            res["roofline"]["per_rank_traffic_note"] = ("each rank's own rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                                        "passes on its own GPU, before the timed region")
        if world > 1:
            fr = [wl.alg_bytes / (ms * 1e-3) / 1e9 / (HBM_PEAK_GBS if res["roofline"]["unit"] == "GB/s" else 1)
                  for ms in rank_avg_ms]
            res["roofline"]["per_rank_avg_launch_ms"] = [round(x, 4) for x in rank_avg_ms]
            if res["roofline"]["bound"] == "hbm":
                res["roofline"]["per_rank_frac_min"] = round(min(fr), 4)
                res["roofline"]["per_rank_frac_max"] = round(max(fr), 4)
            res["roofline"]["note_ranks"] = "achieved/frac above: rank 0's launches; per-rank averages listed"
        if not args.dry_run and args.mode not in ("e2e", "e2e-decode", "scrub", "hasher", "file"):
            res["alloc"] = {"kind": {"chip": "chip_device_alloc (class-balanced from 1 GiB, DESIGN.md §2)",
                                     "contiguous": "hipDeviceMallocContiguous (CHIP_ALLOC=contiguous)",
                                     "torch": "torch caching allocator (hipMalloc)"}[args.alloc],
                            "buffers": wl.alloc_info}
            if world > 1:
                res["alloc"]["buffers_by_rank"] = rank_alloc
        if world > 1:
            res["verify_threads_per_rank"] = verify_threads(world)
        if verified_all is not None:
            res["verified_all_objects"] = verified_all
        if box is not None:
            res["box_ceiling"] = box
            if box.get("GBps"):
                res["roofline"]["box_ceiling_GBps"] = box["GBps"]
                res["roofline"]["frac_of_box_ceiling"] = round(achieved / box["GBps"], 4)
        if aliased is not None:
            a_max, a_ms, a_ok = aliased
            a_bytes = args.objects * (n + (m - k) * wl.C)
            a_avg = sum(a_ms) / len(a_ms)
            a_ach = a_bytes / (a_avg * 1e-3) / 1e9
            res["aliased_data_shards"] = {
                "value": round(world * args.objects * n * args.steps / a_max / 2**30, 2), "unit": "GiB/s",
                "ms_per_step": round(a_max / args.steps * 1e3, 4), "alg_bytes_per_launch": a_bytes,
                "achieved": round(a_ach, 1), "peak": HBM_PEAK_GBS, "frac": round(a_ach / HBM_PEAK_GBS, 4),
                "verified_object0": a_ok,
                "note": ("SURVEY.md 8d: in-place encode, the input already sits in the output slot and only the "
                         "parity shards are written (16 MiB read + 16 MiB written per object); `value` above "
                         "(all 8 shards written, 48 MiB per object) is the graded figure")}
        if scatter is not None:
            res["scatter"] = scatter
        if not args.dry_run:
            res["host_binding"] = getattr(wl, "host_binding", None)
        if getattr(wl, "copy_back", None):
            res["copy_back"] = wl.copy_back
        if args.mode == "hasher" and not args.dry_run:
            from carbonado_amd import device as _dev
            try:
                res["host_topology"] = _dev.host_topology()
            except Exception as e:  # diagnostic only
                res["host_topology"] = {"error": str(e)[:200]}
            fm = sorted(wl.finalize_ms[-args.steps:])
            res["finalize_ms"] = {"median": round(fm[len(fm) // 2], 3), "max": round(fm[-1], 3),
                                  "how": "host wall time of finalize() after the last update() of each timed step "
                                         f"({args.objects * args.object_mib:g} MiB in 4 MiB appends)"}
        if args.mode == "file" and not args.dry_run:
            res["file_stages_last_step"] = dict(wl.file_stats, note="busy seconds of each overlapped stage")
        if wl.scatter_s is not None:
            res["scatter"] = {"seconds": round(wl.scatter_s, 4),
                              "GiB_per_s": round(world * args.objects * n / wl.scatter_s / 2**30, 2),
                              "how": "RCCL scatter from rank 0 over xGMI (outside the timed region)"}
        if args.dry_run:
            res["dry_run"] = True
        if not args.no_cpu_baseline:
            # rank 0, after the timed region and the checks, at any N (the other ranks are done)
            res["cpu_baseline"] = cpu_baseline(args, n, sample, seconds=0.5 if args.dry_run else None)
            threads = min(args.cpu_threads, os.cpu_count() or 1)
            if threads > 1 and not args.dry_run:
                res["cpu_baseline_all_cores"] = cpu_baseline(args, n, sample, threads)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
