"""Reduces rocprofv3 --pmc JSON output to per-instance (XCD x channel) totals for the
draid kernels: for each kernel and counter, the spread of the per-instance values
(min, max, mean, max/mean) -- a balanced kernel has max/mean close to 1."""
import glob
import json
import os
import sys


def load(d):
    for f in glob.glob(os.path.join(d, "**", "*results.json"), recursive=True):
        with open(f) as fh:
            yield json.load(fh)


def main(root):
    out = {}
    for cdir in sorted(glob.glob(os.path.join(root, "TCC_*"))):
        if not os.path.isdir(cdir):
            continue
        for doc in load(cdir):
            for sdk in doc.get("rocprofiler-sdk-tool", []):
                names = {}
                for k in sdk.get("kernel_symbols", []):
                    names[k.get("kernel_id")] = k.get("formatted_kernel_name") or k.get("kernel_name", "")
                counters = {}
                for agent in sdk.get("counters", []):
                    counters[agent.get("id", {}).get("handle")] = agent
                cc = sdk.get("callback_records", {}).get("counter_collection", []) or \
                    sdk.get("buffer_records", {}).get("counter_collection", [])
                for rec in cc:
                    kid = rec.get("dispatch_data", {}).get("dispatch_info", {}).get("kernel_id")
                    name = names.get(kid, "?")
                    kind = "encode" if "k_encode" in name else "reconstruct" if "k_reconstruct" in name else None
                    if not kind:
                        continue
                    vals = {}
                    for r in rec.get("records", []):
                        cid = r.get("counter_id", {}).get("handle")
                        cname = counters.get(cid, {}).get("name", str(cid))
                        vals.setdefault(cname, []).append(r.get("value", 0.0))
                    for cname, v in vals.items():
                        key = f"{kind}:{cname}"
                        ent = out.setdefault(key, {"dispatches": 0, "instances": len(v), "per_instance": [0.0] * len(v)})
                        if len(v) == len(ent["per_instance"]):
                            ent["dispatches"] += 1
                            ent["per_instance"] = [a + b for a, b in zip(ent["per_instance"], v)]
    for key, ent in out.items():
        p = [x / max(1, ent["dispatches"]) for x in ent["per_instance"]]
        mean = sum(p) / max(1, len(p))
        ent["per_launch"] = {"min": min(p), "max": max(p), "mean": mean, "sum": sum(p),
                             "max_over_mean": (max(p) / mean) if mean else None,
                             "min_over_mean": (min(p) / mean) if mean else None}
        ent["per_instance"] = [round(x, 1) for x in p]
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
