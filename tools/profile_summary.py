"""Summarise rocprofv3 output of a bench.py run into profiles/<round>/ (kernel groups as bench.py names them).

  python tools/profile_summary.py stats <kernel_stats.csv> [bench.json]      -> per-group calls / avg / total
  python tools/profile_summary.py traffic <fetch_pmc.csv> <write_pmc.csv>    -> HBM bytes per launch per group

Groups: "gemm" = dense GEMM instantiations (A mode 0), "conv3x3" = implicit-GEMM convs (A mode 1), "attention",
"layernorm", "other".  FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB; on gfx950 FETCH_SIZE counts
half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section), so fetch bytes are doubled.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def group(name: str) -> str:
    m = re.search(r"gemm_big_kernel<(\d)", name)
    if m:
        return "conv3x3" if m.group(1) == "1" else "gemm"
    m = re.search(r"gemm_kernel<[^,]*Traits\w+, (\d)", name)
    if m:
        return "conv3x3" if m.group(1) == "1" else "gemm"
    if "attn_fwd" in name:
        return "attention"
    if "layernorm" in name:
        return "layernorm"
    return "other"


def stats(path, bench=None):
    g = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    for r in csv.DictReader(open(path)):
        k = group(r["Name"])
        g[k]["calls"] += int(r["Calls"])
        g[k]["total_ns"] += float(r["TotalDurationNs"])
    out = {k: dict(v, avg_us=v["total_ns"] / v["calls"] / 1e3) for k, v in g.items()}
    if bench:
        b = json.loads(open(bench).read().strip().splitlines()[-1])
        rf = b.get("roofline") or {}
        out["bench_dominant"] = {"kernel": rf.get("kernel"), "avg_launch_us": rf.get("avg_launch_us")}
        if rf.get("kernel") in out:
            out["bench_dominant"]["rocprof_avg_us"] = out[rf["kernel"]]["avg_us"]
            out["bench_dominant"]["ratio"] = rf["avg_launch_us"] / out[rf["kernel"]]["avg_us"]
    return out


def traffic(fetch_csv, write_csv):
    acc = defaultdict(lambda: defaultdict(list))
    for path, counter in ((fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            acc[group(r["Kernel_Name"])][counter].append(float(r["Counter_Value"]))
    out = {}
    for k, c in acc.items():
        f = c.get("FETCH_SIZE", [])
        w = c.get("WRITE_SIZE", [])
        if not f or not w:
            continue
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / len(w)
        out[k] = {"launches": len(f), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": fb + wb,
                  "note": "FETCH_SIZE x 2 (gfx950 16-B streaming-read correction) + WRITE_SIZE, KiB -> bytes"}
    return out


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        print(json.dumps(stats(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None), indent=1))
    else:
        print(json.dumps(traffic(sys.argv[2], sys.argv[3]), indent=1))
