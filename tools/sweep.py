#!/usr/bin/env python3
"""In-process A/B sweep of the RAID6 8+2 kernels: memory layout x kernel variant.

Rounds are interleaved inside one process (cdna_hip_programming.md §5.4 rule 24)
and the median / min over rounds is reported.  Times come from HIP events on
the launching stream.

  python tools/sweep.py [--rounds 5] [--iters 10] [--stripes 4096] [--strip-kib 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
sys.path.insert(0, ROOT)
# kernel variants live in the lab build of the library only
os.environ.setdefault("DRAID_EC_LIB",
                      os.path.join(ROOT, "draid-spdk_amd", "liblab", "libdraid_ec.so"))

VARIANTS = {0: "default (64 lanes U1)", 1: "U2", 2: "512 lanes U1", 3: "128 lanes",
            4: "chunk-major map", 5: "persistent", 6: "scalar plan", 7: "persist 512 scalar",
            8: "1024 lanes", 9: "64 lanes", 10: "256 lanes U1", 11: "512 lanes U2", 12: "U4",
            13: "DIAG no-plan U2", 14: "DIAG no-plan U1", 15: "DIAG no-plan no-mul U1",
            16: "XCD-aware map", 17: "XCD-aware 512 lanes",
            18: "64 lanes U2", 19: "64 lanes U4", 20: "64 lanes XCD-aware",
            21: "64 lanes nt loads only", 22: "64 lanes nt stores only", 23: "64 lanes no nt",
            24: "st buffer nt", 25: "st sc1", 26: "st sc1 nt", 27: "st sc0 sc1 nt",
            28: "st sc0 nt", 29: "ld buffer nt", 30: "ld sc1 nt", 31: "ld sc0 sc1 nt",
            32: "ld sc0 nt", 33: "ld sc1 st sc1", 34: "ld buf nt st sc1 nt",
            35: "ld buf nt st buf nt", 36: "ld buf nt st sc1", 37: "ld sc0sc1nt st sc1nt",
            38: "XCD-aware, enc policy", 39: "XCD-aware, rec policy",
            40: "enc G16 diagonal", 41: "enc G16 same chunk", 42: "enc G4 diagonal",
            43: "enc G4 same chunk", 44: "rec G16 diagonal", 45: "rec G4 diagonal"}


def probe(torch, dev, nbytes, rounds, iters):
    """Pure read / write / copy ceilings from tools/probe/libprobe.so."""
    import ctypes as C
    L = C.CDLL(os.path.join(ROOT, "tools", "probe", "libprobe.so"))
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev).random_(0, 256)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    sink = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = C.c_void_p(stream.cuda_stream)
    out = []
    for grid in (2048, 4096, 8192, 16384):
        ops = {"read": (lambda: L.probe_read(C.c_void_p(a.data_ptr()), C.c_uint64(nbytes),
                                             C.c_void_p(sink.data_ptr()), grid, sh), nbytes),
               "write": (lambda: L.probe_write(C.c_void_p(b.data_ptr()), C.c_uint64(nbytes), grid,
                                               sh), nbytes),
               "copy": (lambda: L.probe_copy(C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()),
                                             C.c_uint64(nbytes), grid, sh), 2 * nbytes)}
        for name, (fn, moved) in ops.items():
            ts = []
            for _ in range(rounds):
                fn()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(iters):
                    fn()
                e1.record(stream)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / iters)
            med = float(np.median(ts))
            out.append({"probe": name, "grid": grid, "median_us": round(med, 2),
                        "gb_s": round(moved / (med * 1e-6) / 1e9, 1)})
            print(f"probe {name:5s} grid {grid:6d} {med:9.2f} us {out[-1]['gb_s']:8.1f} GB/s")
    del a, b
    return out


def make_layout(torch, name, k, m, S, B, dev):
    n = k + m
    if name.startswith("stripe_major"):
        gap = int(name.split("gap")[1]) if "gap" in name else 0
        ss = S + gap
        buf = torch.empty(B * n * ss, dtype=torch.uint8, device=dev)
        idx = torch.arange(B * n, dtype=torch.int64, device=dev)
        table = buf.data_ptr() + idx * ss
    elif name == "parity_apart":
        # data strips stripe-major, every stripe's P (Q) in a second region
        buf = torch.empty(B * n * S, dtype=torch.uint8, device=dev)
        s = torch.arange(B, dtype=torch.int64, device=dev).repeat_interleave(n)
        j = torch.arange(n, dtype=torch.int64, device=dev).repeat(B)
        off = torch.where(j < k, (s * k + j) * S, B * k * S + (s * m + (j - k)) * S)
        table = buf.data_ptr() + off
    elif name.startswith("stripe_shuffled"):
        # stripe-major slots, stripes assigned to slots in a seeded random order
        # (stripe_shuffled_gG: runs of G consecutive slots stay together)
        G = int(name.split("_g")[1]) if "_g" in name else 1
        buf = torch.empty(B * n * S, dtype=torch.uint8, device=dev)
        g = torch.Generator(device="cpu")
        g.manual_seed(7)
        blk = torch.randperm((B + G - 1) // G, generator=g)
        order = blk.repeat_interleave(G) * G + torch.arange(G).repeat(len(blk))
        order = order[order < B]
        slot = order.to(dev).repeat_interleave(n)
        j = torch.arange(n, dtype=torch.int64, device=dev).repeat(B)
        table = buf.data_ptr() + (slot * n + j) * S
    elif name == "strip_major":
        buf = torch.empty(n * B * S, dtype=torch.uint8, device=dev)
        s = torch.arange(B, dtype=torch.int64, device=dev).repeat_interleave(n)
        j = torch.arange(n, dtype=torch.int64, device=dev).repeat(B)
        table = buf.data_ptr() + j * (B * S) + s * S
    else:
        raise ValueError(name)
    buf.random_(0, 256)
    return buf, table.contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--strip-kib", type=int, default=64)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--failures", default="dual", choices=["dual", "single"])
    ap.add_argument("--layouts", default="stripe_major,stripe_major_gap256,stripe_major_gap4096,strip_major")
    ap.add_argument("--variants", default="0,1,2,8,10,11,12")
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--fail-order", default="random", choices=["random", "sorted", "fixed"],
                    help="per-stripe failure pairs: seeded random (bench), the same pairs "
                         "sorted so neighbouring stripes share one, or one pair everywhere")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.json"))
    args = ap.parse_args()

    import torch
    import draid_ec as ec
    import bench

    dev = torch.device("cuda", 0)
    k, S, B = args.k, args.strip_kib * 1024, args.stripes
    m = 1 if k == 4 else 2
    probes = probe(torch, dev, (k + m) * S * B, args.rounds, args.iters) if args.probe else []
    fgen = bench.failure_pairs if args.failures == "dual" else bench.failure_single
    fnp0 = fgen(B, k, 0x1234)
    if args.fail_order == "sorted":
        fnp0 = fnp0[np.lexsort((fnp0[:, 1], fnp0[:, 0]))].copy()
    elif args.fail_order == "fixed":
        fnp0 = np.repeat(fnp0[:1], B, axis=0).copy()
    fail = torch.from_numpy(fnp0.reshape(-1)).to(dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    layouts = {}
    for name in args.layouts.split(","):
        buf, table = make_layout(torch, name, k, m, S, B, dev)
        layouts[name] = (buf, table, ec.make_batch(k, m, S, B, table))
    variants = [int(v) for v in args.variants.split(",")]
    verified = {}
    if "stripe_major" in layouts:
        # every variant must produce the default's bytes: erase its outputs, rerun, compare
        buf, _, batch = layouts["stripe_major"]
        view = buf.view(B, k + m, S)
        ec.set_variant(0)
        ec.encode(batch, sh)
        torch.cuda.synchronize(dev)
        good = view.clone()
        fnp = fnp0
        rows = torch.arange(B, device=dev)
        for v in variants:
            ec.set_variant(v)
            view[:, k:] = 0
            ec.encode(batch, sh)
            torch.cuda.synchronize(dev)
            ok = torch.equal(view, good)
            for slot in range(2):
                idx = np.nonzero(fnp[:, slot] != 0xFF)[0]
                if len(idx):
                    ii = torch.from_numpy(idx).to(dev)
                    view[rows[ii], torch.from_numpy(fnp[idx, slot].astype(np.int64)).to(dev)] = 0
            ec.reconstruct(batch, fail, sh)
            torch.cuda.synchronize(dev)
            verified[v] = ok and torch.equal(view, good)
            print(f"verify v{v}: {'ok' if verified[v] else 'MISMATCH'}")
        del good
        ec.set_variant(0)
    res = {f"{l}|{v}|{op}": [] for l in layouts for v in variants for op in ("enc", "rec")}
    nbytes = (k + m) * S * B
    rec_nbytes = bench.reconstruct_bytes_per_stripe(k, m, S, args.failures) * B
    for r in range(args.rounds):
        for lname, (_, _, batch) in layouts.items():
            for v in variants:
                ec.set_variant(v)
                for op in ("enc", "rec"):
                    fn = (lambda: ec.encode(batch, sh)) if op == "enc" else \
                         (lambda: ec.reconstruct(batch, fail, sh))
                    fn()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        fn()
                    e1.record(stream)
                    e1.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / args.iters
                    res[f"{lname}|{v}|{op}"].append(us)
    ec.set_variant(0)
    summary = []
    for key, vals in res.items():
        lname, v, op = key.split("|")
        med = float(np.median(vals))
        summary.append({"layout": lname, "variant": int(v), "desc": VARIANTS[int(v)], "op": op,
                        "verified": verified.get(int(v)),
                        "median_us": round(med, 2), "min_us": round(min(vals), 2),
                        "hbm_gb_s": round((nbytes if op == "enc" else rec_nbytes) / (med * 1e-6)
                                          / 1e9, 1)})
    summary.sort(key=lambda d: (d["op"], d["median_us"]))
    for d in summary:
        print(f'{d["op"]} {d["layout"]:24s} v{d["variant"]} {d["desc"]:22s} '
              f'{d["median_us"]:9.2f} us  {d["hbm_gb_s"]:8.1f} GB/s')
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"config": vars(args), "results": summary, "probes": probes}, f, indent=1)


if __name__ == "__main__":
    main()
