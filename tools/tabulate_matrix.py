"""Prints a gpu_shape_matrix.sh result file as a table: one row per (shape, kernel), one
column per library build, microseconds per launch."""
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
shapes, libs = [], []
for r in rows:
    if r["shape"] not in shapes:
        shapes.append(r["shape"])
    if r["lib"] not in libs:
        libs.append(r["lib"])
print("shape".ljust(24), " ".join(l.rjust(7) for l in libs))
for s in shapes:
    d = {r["lib"]: r for r in rows if r["shape"] == s}
    for key in ("enc_ms", "rec_ms"):
        print((s + " " + key[:3]).ljust(24),
              " ".join((f"{d[l][key] * 1000:.1f}" if l in d else "-").rjust(7) for l in libs))
print("all verified:", all(r["verified"] for r in rows), len(rows), "runs")
