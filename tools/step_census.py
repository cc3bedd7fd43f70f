"""Per-step kernel census of an eager rocprofv3 kernel trace of bench.py (tools/trace_step.sh): launches and GPU time
per kernel symbol per infer, the small-launch tail (kernels under 20 us) listed separately.
Usage: python tools/step_census.py gpurun_out/prof_e [infers=3] [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)", "anon")
    n = re.sub(r"\(.*$", "", n)  # drop the argument list
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"<.*>", "<..>", n)
    return n.split("::")[-1]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_e"
    infers = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    out = sys.argv[3] if len(sys.argv) > 3 else None
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one infer: every MapAnything call starts with the fault-word reset; the census covers the last `infers` calls
    # (the weight loading / packing before the first call is left out)
    starts = [i for i, r in enumerate(rows) if "fault_reset_kernel" in r["Kernel_Name"]]
    if len(starts) >= infers:
        rows = rows[starts[-infers]:]
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per = {k: {"launches_per_infer": c / infers, "us_per_infer": t / infers, "avg_us": t / c} for k, (c, t) in agg.items()}
    total_l = sum(v["launches_per_infer"] for v in per.values())
    total_t = sum(v["us_per_infer"] for v in per.values())
    small = {k: v for k, v in per.items() if v["avg_us"] < 20}
    print(f"per infer (trace / {infers}): {total_l:.0f} launches, {total_t / 1e3:.2f} ms of kernel time; "
          f"kernels under 20 us: {sum(v['launches_per_infer'] for v in small.values()):.0f} launches, "
          f"{sum(v['us_per_infer'] for v in small.values()) / 1e3:.3f} ms")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]["us_per_infer"]):
        print(f"{v['launches_per_infer']:7.1f} x {v['avg_us']:8.2f} us = {v['us_per_infer'] / 1e3:7.3f} ms  {k}")
    if out:
        json.dump({"infers": infers, "launches_per_infer": total_l, "ms_per_infer": total_t / 1e3, "kernels": per},
                  open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
