#!/usr/bin/env python3
"""Pair tools/k13_fetch's variants with their rocprofv3 FETCH_SIZE and
WRITE_SIZE counters (one pass each).  The tool launches each variant
1 + reps times in the order it prints ("VARIANT <label> dispatches <d> ..."),
so the zfec_bao_fused_kernel dispatches of a pass, in dispatch order, are
the variants' launches in that order; the warm-up launch of each is dropped.

usage: tools/k13_fetch_summary.py SESSION_DIR  (gpurun_out/<tag>)
writes SESSION_DIR/k13_fetch_summary.json and prints a table
"""
import csv
import json
import re
import sys
from pathlib import Path


def dispatches(csv_path: Path):
    rows = [r for r in csv.DictReader(open(csv_path)) if "zfec_bao_fused_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows]


def variants(log: Path):
    out = []
    for line in log.read_text().splitlines():
        m = re.match(r"VARIANT (.+?)\s+dispatches (\d+)\s+median\s+([\d.]+) ms", line)
        if m:
            out.append((m.group(1).strip(), int(m.group(2)), float(m.group(3))))
    return out


def main():
    d = Path(sys.argv[1])
    fetch = dispatches(next(d.glob("kf/**/*counter_collection.csv")))
    write = dispatches(next(d.glob("kw/**/*counter_collection.csv")))
    vs = variants(d / "k13_fetch_pmc_fetch.log")
    res, i = [], 0
    for label, nd, ms in vs:
        f = fetch[i + 1:i + nd]  # drop the warm-up launch
        w = write[i + 1:i + nd]
        i += nd
        res.append({"variant": label, "median_ms_under_pmc": ms,
                    "FETCH_SIZE_KiB": round(sum(f) / len(f)) if f else None,
                    "WRITE_SIZE_KiB": round(sum(w) / len(w)) if w else None})
    assert i == len(fetch) == len(write), (i, len(fetch), len(write))
    base = res[0]["FETCH_SIZE_KiB"]
    for r in res:
        r["fetch_vs_first"] = round(r["FETCH_SIZE_KiB"] / base, 4) if base and r["FETCH_SIZE_KiB"] else None
    (d / "k13_fetch_summary.json").write_text(json.dumps(res, indent=1) + "\n")
    print(f"{'variant':46s} {'FETCH KiB':>12s} {'x first':>8s} {'WRITE KiB':>12s}")
    for r in res:
        print(f"{r['variant']:46s} {r['FETCH_SIZE_KiB']:12d} {r['fetch_vs_first']:8.4f} {r['WRITE_SIZE_KiB']:12d}")


if __name__ == "__main__":
    main()
