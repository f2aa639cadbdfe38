"""CPU tests of bench.py's host-side helpers (no device)."""
import sys
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


@pytest.mark.parametrize("n", [4096 * 3, 70_001, 1 << 20, (1 << 20) + 37])
def test_scrub_corrupt_offset_lands_in_a_chunk(n):
    """--mode scrub flips one byte per object at scrub_corrupt_offset(n, o): a
    content byte of data shard o % 4 in the level-12 stream (the layout
    formula 8 + 1024 i + 64 (P(i) + c(i)), checked against the oracle's
    encode)."""
    import bench
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, _, _ = O.encode(d, 12)
    z, _, C = O.zfec_encode(d)
    for o in range(4):
        off = bench.scrub_corrupt_offset(n, o)
        i = o * (C // 1024) + (C // 1024) // 3  # the chunk the helper aims at
        assert enc[off - 517:off - 517 + 1024] == z[1024 * i:1024 * (i + 1)]


FAKE_ROCPROF = r'''#!/usr/bin/env python3
# stand-in for rocprofv3 --pmc CTR -d DIR -o TAG --output-format csv -- cmd...
import sys
from pathlib import Path
a = sys.argv[1:]
ctr, d, tag = a[a.index("--pmc") + 1], Path(a[a.index("-d") + 1]), a[a.index("-o") + 1]
cmd = a[a.index("--") + 1:]
assert "--live-pmc" in cmd and cmd[cmd.index("--live-pmc") + 1] == "off", cmd
assert cmd[-2:] == ["--gpus", "1"], cmd  # the child runs alone on one GPU
import os
exp = os.environ.get("EXPECT_HIP")
if exp is not None:  # a rank's child: only its GPU visible, no torch.distributed variables
    assert os.environ.get("HIP_VISIBLE_DEVICES") == exp, os.environ.get("HIP_VISIBLE_DEVICES")
    assert "WORLD_SIZE" not in os.environ and "RANK" not in os.environ and "MASTER_PORT" not in os.environ
d.mkdir(parents=True, exist_ok=True)
val = {"FETCH_SIZE": [999.0, 100.0, 200.0], "WRITE_SIZE": [5.0, 300.0, 500.0]}[ctr]
with open(d / f"{tag}_counter_collection.csv", "w") as f:
    f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n")
    f.write("1,at::fill_kernel,%s,1\n" % ctr)
    for i, v in enumerate(val):
        f.write('%d,"chip::(anonymous namespace)::zfec_apply_kernel<4, 1>(chip::zf::ApplyArgs)",%s,%s\n' % (i + 2, ctr, v))
'''


def test_live_traffic_two_passes(tmp_path, monkeypatch):
    """bench.live_traffic: one rocprofv3 pass per counter, the kernel's last
    `steps` dispatches averaged, bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB)."""
    import shutil
    import bench
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE_ROCPROF)
    fake.chmod(0o755)
    monkeypatch.setattr(shutil, "which", lambda name: str(fake))
    args = bench.parse([])
    r = bench.live_traffic(args, [], timeout_s=60)
    assert r["FETCH_SIZE_KiB"] == 150.0 and r["WRITE_SIZE_KiB"] == 400.0, r
    assert r["bytes"] == (2 * 150 + 400) * 1024
    assert "zfec_apply_kernel<4, 1>" in r["kernel"]
    # a mode without an HBM-bound kernel gets no passes
    assert "error" in bench.live_traffic(bench.parse(["--mode", "bao"]), [])


@pytest.mark.parametrize("visible,expect", [(None, "3"), ("4,5,6,7", "7")])
def test_live_traffic_per_rank_child(tmp_path, monkeypatch, visible, expect):
    """N > 1: every rank profiles its own GPU before the timed region; the
    child sees only that GPU (LOCAL_RANK-th of the visible ones) and none of
    the torch.distributed variables, and runs with --gpus 1."""
    import shutil
    import bench
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE_ROCPROF)
    fake.chmod(0o755)
    monkeypatch.setattr(shutil, "which", lambda name: str(fake))
    for k, v in {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3", "MASTER_PORT": "29500",
                 "MASTER_ADDR": "127.0.0.1", "EXPECT_HIP": expect}.items():
        monkeypatch.setenv(k, v)
    if visible is None:
        monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    else:
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", visible)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    r = bench.live_traffic(bench.parse(["--gpus", "8"]), ["--gpus", "8"], timeout_s=60, local_rank=3)
    assert r.get("bytes") == (2 * 150 + 400) * 1024, r


def test_pcie_roofline_names_the_binding_direction():
    """E2E lines price each PCIe direction on its own:
    cfg4 moves ~2.1x as many bytes D2H as H2D, so D2H binds and the frac is
    against one direction's 63 GB/s, not the 126 GB/s duplex sum."""
    import bench
    n, out = 16 << 20, 35_660_232
    r = bench.pcie_roofline(1024 * n, 1024 * out, 0.7088, 75.5)
    assert r["bound"] == "pcie-d2h" and r["peak"] == 63.0 and r["unit"] == "GB/s"
    assert abs(r["d2h_GBps"] - 1024 * out / 0.7088 / 1e9) < 0.01
    assert abs(r["frac"] - r["d2h_GBps"] / 63.0) < 1e-3 and 0.8 < r["frac"] < 0.84
    assert r["h2d_GBps"] < r["d2h_GBps"] and r["achieved"] == r["d2h_GBps"]
    assert abs(r["frac_of_measured"] - r["d2h_GBps"] / 55.0) < 1e-3
    assert r["duplex_frac"] == round(75.5 / 126.0, 4)
    # decode reads the stream up and writes the content down: H2D binds
    r = bench.pcie_roofline(1024 * out, 1024 * n, 0.8, 0)
    assert r["bound"] == "pcie-h2d" and r["peak_measured"] == 55.6
    # the hasher only uploads
    assert bench.pcie_roofline(1 << 30, 0, 0.05, 0)["bound"] == "pcie-h2d"


@pytest.mark.parametrize("N", [2, 8, 10, 16, 34, 40, 64])
def test_bao_data_region_len_matches_the_oracle_stream(N):
    """bench.bao_data_region_len(N) = end of chunk N/2 - 1 in the oracle's bao
    stream of N distinct chunks (the H2D bytes of the direct e2e path)."""
    content = b"".join(bytes([i % 251 + 1]) * 1024 for i in range(N))
    enc, _ = O.bao_encode(content)
    last = N // 2 - 1
    off = enc.find(bytes([last % 251 + 1]) * 1024)
    import bench
    assert off > 0 and bench.bao_data_region_len(N) == off + 1024
