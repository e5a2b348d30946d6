#!/usr/bin/env python3
"""Summarise rocprofv3 runs into per-kernel duration and HBM traffic.

Usage:
  collect_pmc.py trace <kernel_trace_dir> <out.json>
  collect_pmc.py pmc <fetch_dir> <write_dir> <workload> [out.json]

HBM bytes follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE are collected in SEPARATE --pmc passes (TCC slots),
both in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
coalesced streaming read (16 B/lane), so the read side is doubled.  WRITE_SIZE
reads 16-B-per-lane streaming stores exactly.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys


def rows(d: str, pattern: str):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name: str) -> str:
    if "k_encode" in name:
        return "encode"
    if "k_reconstruct" in name:
        return "reconstruct"
    if "k_gf_vect_mul" in name:
        return "gf_vect_mul"
    return "other"


def per_kernel_counter(d: str, counter: str):
    vals: dict[str, list[float]] = {}
    for r in rows(d, "*counter_collection*.csv"):
        if r.get("Counter_Name") != counter:
            continue
        vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def pmc(fetch_dir: str, write_dir: str, workload: str, out: str | None) -> dict:
    fetch = per_kernel_counter(fetch_dir, "FETCH_SIZE")
    write = per_kernel_counter(write_dir, "WRITE_SIZE")
    res: dict = {"workload": workload, "kernels": {},
                 "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                           "hbm = 2*FETCH_SIZE*1024 (gfx950 half-count correction) + "
                           "WRITE_SIZE*1024, median over dispatches"}
    for name in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch.get(name, [0.0])) * 1024.0
        w = statistics.median(write.get(name, [0.0])) * 1024.0
        res["kernels"][name] = {"kind": short(name), "fetch_bytes_raw": f,
                                "fetch_bytes_corrected": 2.0 * f, "write_bytes": w,
                                "hbm_bytes": 2.0 * f + w,
                                "dispatches": len(fetch.get(name, []))}
    for kind in ("encode", "reconstruct"):
        c = [v for v in res["kernels"].values() if v["kind"] == kind]
        if c:
            best = max(c, key=lambda v: v["dispatches"])
            res[f"{kind}_hbm_bytes_per_launch"] = best["hbm_bytes"]
            res[f"{kind}_read_bytes_per_launch"] = best["fetch_bytes_corrected"]
            res[f"{kind}_write_bytes_per_launch"] = best["write_bytes"]
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
    return res


def trace(d: str, out: str | None) -> dict:
    durs: dict[str, list[float]] = {}
    for r in rows(d, "*kernel_trace*.csv"):
        name = r.get("Kernel_Name", "")
        t = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-3  # ns -> us
        durs.setdefault(name, []).append(t)
    res = {name: {"kind": short(name), "calls": len(v), "avg_us": statistics.mean(v),
                  "median_us": statistics.median(v), "min_us": min(v), "max_us": max(v)}
           for name, v in durs.items()}
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
    return res


if __name__ == "__main__":
    if sys.argv[1] == "pmc":
        r = pmc(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else None)
    else:
        r = trace(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    print(json.dumps(r, indent=1))
