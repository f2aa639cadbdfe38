#!/usr/bin/env python3
"""Summarise a gpurun_out/<tag> rocprofv3 session into profiles/<tag>_*.

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slots), both
in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

usage: tools/pmc_summary.py TAG [kernel-substring]
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def avg_counter(path: Path, kern: str):
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    vals = [float(r["Counter_Value"]) for r in rows]
    return (sum(vals) / len(vals) if vals else None), len(vals), (rows[0]["Kernel_Name"] if rows else None)


def main():
    tag = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "zfec_apply_kernel"
    src = ROOT / "gpurun_out" / tag
    tag = tag.replace("/", "_")  # a session's sub-run (gpu_session.sh prof15s: TAG/p15s)
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    stats = src / "prof" / "stats_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, dst / f"{tag}_kernel_stats.csv")
    fetch, nf, name = avg_counter(src / "pmc_fetch" / "fetch_counter_collection.csv", kern)
    write, nw, _ = avg_counter(src / "pmc_write" / "write_counter_collection.csv", kern)
    avg_ns = None
    if stats.exists():
        for r in csv.DictReader(open(stats)):
            if kern in r["Name"]:
                avg_ns = float(r["AverageNs"])
    out = {
        "tag": tag,
        "kernel": name,
        "dispatches_fetch_pass": nf,
        "dispatches_write_pass": nw,
        "FETCH_SIZE_KiB_avg": fetch,
        "WRITE_SIZE_KiB_avg": write,
        "hbm_bytes_per_launch": (2 * fetch * 1024 + write * 1024) if fetch and write else None,
        "correction": "2 x FETCH_SIZE (gfx950 reports half of wide streaming reads) + WRITE_SIZE, KiB->B",
        "rocprof_avg_ns": avg_ns,
        "commands": {
            "stats": "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 2",
            "fetch": "rocprofv3 --pmc FETCH_SIZE -- python3 bench.py --steps 2 --warmup 1",
            "write": "rocprofv3 --pmc WRITE_SIZE -- python3 bench.py --steps 2 --warmup 1",
        },
    }
    (dst / f"{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
    for f in sorted(src.glob("bench_*.log")):
        lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
        if lines:
            (dst / f"{tag}_{f.stem}.json").write_text(lines[-1] + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
