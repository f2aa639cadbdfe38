"""RCCL (torch.distributed's "nccl" backend on ROCm) on the box's GPU before
the driver's 8-GPU run: world size 1, the control plane bench.py uses at N > 1
(barrier, the MAX / SUM all-reduces) and sharding.scatter_objects on a 64 MiB
object batch, bytes asserted (objects partitioned over ranks,
the scatter only stages inputs).  The ranks of a real N > 1 run are separate
processes; this one runs in a child process so RCCL's threads and its
communicator end with it."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

_CHILD = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist
from carbonado_amd.sharding import object_range, scatter_objects
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="file://" + sys.argv[2], rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
try:
    assert dist.get_backend() == "nccl"
    world, rank = dist.get_world_size(), dist.get_rank()
    per, n = 4, 16 << 20  # 4 objects of 16 MiB: the 64 MiB batch
    g = torch.Generator(device="cuda").manual_seed(5)
    full = torch.randint(0, 256, (world * per, n), dtype=torch.uint8, device="cuda", generator=g)
    local = torch.zeros((per, n), dtype=torch.uint8, device="cuda")
    scatter_objects(local, full, src=0)
    r = object_range(rank, world, world * per)
    assert torch.equal(local, full[r.start:r.stop]), "scatter bytes"
    t = torch.tensor([3.5], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([r.count], dtype=torch.int64, device="cuda")
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.barrier()
    torch.cuda.synchronize()
    assert t.item() == 3.5 and s.item() == per
    print("RCCL_OK", torch.cuda.get_device_name(0), flush=True)
finally:
    dist.destroy_process_group()
"""


def test_rccl_world1_scatter_and_control_plane(gpu, tmp_path):
    root = str(Path(__file__).resolve().parents[1])
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, "-c", _CHILD, root, str(tmp_path / "store")], env=env,
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "RCCL_OK" in out.stdout, out.stdout[-3000:] + out.stderr[-3000:]
