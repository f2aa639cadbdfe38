"""Multi-rank control plane on CPU (gloo, world_size 2): object partition,
max-over-ranks timing, sum of processed objects and the input scatter used
by bench.py for N > 1.  No GPU needed."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from carbonado_amd.sharding import (max_over_ranks, object_range, scatter_objects,
                                    sum_over_ranks)


def test_object_range_partition():
    for total in [0, 1, 7, 1024, 8192, 8193]:
        for world in [1, 2, 3, 4, 8]:
            rs = [object_range(r, world, total) for r in range(world)]
            assert rs[0].start == 0 and rs[-1].stop == total
            assert all(a.stop == b.start for a, b in zip(rs, rs[1:]))
            assert max(r.count for r in rs) - min(r.count for r in rs) <= 1
    assert object_range(3, 8, 8192).start == 3072  # cfg5: 1024 per GPU


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = object_range(rank, world, 10)
        got_max = max_over_ranks(1.5 + rank)
        got_sum = sum_over_ranks(rng.count)
        per = 3
        full = torch.arange(world * per * 4, dtype=torch.uint8).reshape(world * per, 4) if rank == 0 else None
        local = torch.empty((per, 4), dtype=torch.uint8)
        scatter_objects(local, full, src=0)
        expect = torch.arange(world * per * 4, dtype=torch.uint8).reshape(world * per, 4)[rank * per:(rank + 1) * per]
        q.put((rank, got_max, got_sum, bool(torch.equal(local, expect))))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_control_plane():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, mx, sm, ok in res:
        assert mx == 2.5 and sm == 10 and ok, (rank, mx, sm, ok)


@pytest.mark.parametrize("world", [2])
def test_bench_world2_cpu_dry_run(world):
    """bench.py's multi-rank reduction logic (value = all ranks' bytes / max
    time) exercised with gloo on CPU via --dry-run (no device)."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(root / "bench.py"), "--gpus", str(world),
           "--steps", "3", "--warmup", "1", "--dry-run"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    import json
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["scaling"] == "weak"
    assert res["config"]["global_objects"] == world * res["config"]["objects_per_gpu"]


def test_bench_spawns_its_own_ranks_dry_run():
    """`bench.py --gpus 2` with no WORLD_SIZE starts the two rank processes
    itself (the driver's N>1 command line without torch.distributed.run) and
    rank 0 prints one line with n_gpus 2."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--dry-run"], capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_objects"] == 2 * res["config"]["objects_per_gpu"]
    assert len(res["roofline"]["per_rank_avg_launch_ms"]) == 2
    assert res["box_ceiling"]["GBps"] > 0 and "frac_of_box_ceiling" in res["roofline"]
    assert res["box_ceiling"]["clocks"].keys() & {"unavailable", "sclk_MHz"}


def test_bench_refuses_world_size_mismatch():
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=120, cwd=root, env=env)
    assert out.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in out.stderr


def test_bench_config_presets():
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    a = bench.parse(["--config", "cfg5"])
    assert (a.mode, a.k, a.m, a.objects) == ("encode", 8, 16, 1024)
    a = bench.parse(["--config", "cfg3", "--objects", "64"])
    assert (a.mode, a.erase, a.objects) == ("decode", "1,2", 64)
    a = bench.parse(["--config", "cfg4"])
    assert (a.mode, a.level) == ("e2e", 15)
    a = bench.parse([])
    assert (a.mode, a.k, a.m, a.objects, a.alloc) == ("encode", 4, 8, 1024, "chip")


def test_bench_cfg5_eight_ranks_dry_run():
    """The driver's SCALE command shape for cfg5 (8192 x 16 MiB objects over 8
    GPUs), rehearsed with 8 gloo ranks on CPU: one line, per-rank arrays 8
    long, 8192 global objects, verify threads split over the ranks."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, str(root / "bench.py"), "--config", "cfg5", "--gpus", "8", "--steps", "2",
                          "--warmup", "1", "--dry-run"], capture_output=True, text=True, timeout=600, cwd=root,
                         env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 8 and res["config"]["global_objects"] == 8192
    assert (res["config"]["k"], res["config"]["m"]) == (8, 16)
    assert len(res["roofline"]["per_rank_avg_launch_ms"]) == 8
    assert 1 <= res["verify_threads_per_rank"] <= 16
    # the N>1 line carries the CPU baseline (rank 0, after the timed region) and the
    # scatter sample (gloo stands in for RCCL in the dry run): every rank got its slice
    cb = res["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] == "port" and "8-of-16" in cb["sample"]
    sc = res["scatter"]
    assert sc["ranks"] == 8 and sc["every_slice_ok"] is True and sc["bytes_per_rank"] > 0
    # the box-ceiling diagnostic: every rank's ceiling, the headline priced against it,
    # clocks / partition modes (reported unavailable without a device)
    box = res["box_ceiling"]
    assert len(box["GBps_by_rank"]) == 8 and all(g > 0 for g in box["GBps_by_rank"])
    assert "clocks" in box and res["roofline"]["box_ceiling_GBps"] == box["GBps"]
    assert 0 < res["roofline"]["frac_of_box_ceiling"]


@pytest.mark.parametrize("mode", ["encode", "decode", "bao", "bao-decode", "pipeline", "pipeline-decode", "e2e",
                                  "e2e-decode", "scrub", "scrub-batch", "hasher", "file"])
def test_bench_every_mode_dry_run(mode):
    """Every bench mode's control plane runs without a device and prints one
    line with the contract's keys (scrub-batch's VALU count once lacked a dry
    placeholder)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, str(root / "bench.py"), "--mode", mode, "--steps", "2", "--warmup", "1",
                          "--dry-run"], capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "config", "roofline"):
        assert key in res, key
