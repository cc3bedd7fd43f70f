"""Summarise rocprofv3 output of a bench.py run into profiles/<round>/ (kernel groups as bench.py names them).

  python tools/profile_summary.py stats <kernel_stats.csv> [bench.json]      -> per-group calls / avg / total
  python tools/profile_summary.py traffic <fetch_pmc.csv> <write_pmc.csv>    -> HBM bytes per launch per group
  python tools/profile_summary.py mfma <kernel-regex> <pmc.csv>...           -> MFMA-pipe utilisation at the real clock
  python tools/profile_summary.py mfma_groups <pmc.csv> [launch_log.json]   -> the same per kernel group (bench run)
  python tools/profile_summary.py kinds <kernel_trace.csv> <launch_log.json> -> per bench.py kind (calls / avg / total)
  python tools/profile_summary.py shapes <kernel_trace.csv> <launch_log.json> -> per kind and problem shape (a log
                                                                               written with MAPA_LAUNCH_SHAPES=1)
  python tools/profile_summary.py headline <kernel_trace.csv> <bench.json>   -> groups over the headline infers only
  python tools/profile_summary.py agree <kernel_kinds_eager.json> <bench.json> -> bench vs rocprof for the roofline class

With a launch log (MAPA_LAUNCH_LOG, mapanything/_native.py) every GEMM / attention dispatch is named exactly as
bench.py names it ("gemm", "gemm_ln", "gemm_split", "conv3x3", "conv3x3_split", "attention", "attention_global"): the n-th
GEMM-kernel dispatch of the trace is the n-th GEMM call of the log (one dispatch per mapa_gemm call), the n-th
attn_fwd dispatch the n-th attention call.

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
    if "conv_halo_kernel" in name:
        return "conv3x3"
    if "gemm_pers" in name:  # gemm_pers.hip: dense A only (the transformer linears, persistent register epilogue)
        return "gemm"
    m = re.search(r"gemm_(?:big|8p|w4|sk)_kernel<(?:[^,<>]*P8Cfg<[^>]*>, )?(\d)", name)
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


def _is_gemm(name):
    return "gemm_big_kernel" in name or "gemm_kernel<" in name or "gemm_sk_kernel" in name or \
        "gemm_pp_kernel" in name or "conv_halo_kernel" in name or "gemm_pers" in name


def dispatch_kinds(names, log_path, keep_shape=False):
    """names: kernel names of the dispatches in order -> the bench kind of each (None for other kernels).  Log
    entries written with MAPA_LAUNCH_SHAPES=1 carry the problem shape after a colon ("gemm:10960x3072x1024");
    keep_shape keeps it, otherwise only the kind is returned."""
    log = json.load(open(log_path))
    if not keep_shape:
        log = [k.split(":")[0] for k in log]
    g_log = [k for k in log if k.startswith(("gemm", "conv3x3"))]
    a_log = [k for k in log if k.startswith("attention")]
    gi = ai = 0
    out = []
    prev_ln = False
    for n in names:
        # an LN-fused call is cut into launches of at most the co-resident grid (gemm_big.hip launch_gemm_big_ln):
        # back-to-back LN-kernel dispatches are one logged call
        is_ln = re.search(r"gemm_big_kernel<[^>]*, true>", n) is not None
        if is_ln and prev_ln:
            out.append(out[-1])
        elif _is_gemm(n):
            out.append(g_log[gi] if gi < len(g_log) else None)
            gi += 1
        elif "attn_fwd" in n:
            out.append(a_log[ai] if ai < len(a_log) else None)
            ai += 1
        else:
            out.append(None)
        prev_ln = is_ln
    if gi != len(g_log) or ai != len(a_log):
        raise SystemExit(f"launch log does not match the trace: {gi}/{len(g_log)} gemm, {ai}/{len(a_log)} attention")
    return out


def kinds(trace_csv, log_path, keep_shape=False):
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = dispatch_kinds([r["Kernel_Name"] for r in rows], log_path, keep_shape)
    g = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    for r, k in zip(rows, ks):
        k = k or group(r["Kernel_Name"])
        g[k]["calls"] += 1
        g[k]["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {k: dict(v, avg_us=v["total_ns"] / v["calls"] / 1e3) for k, v in g.items()}


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


def headline(trace_csv, bench):
    """Per-group launch stats over the bench's HEADLINE infers only, from the kernel trace of the driver's full command
    (which also runs the fast mode and the 100-view strong job): dispatches are cut into infers at every
    patchify_kernel launch (one per infer) and the first warmup + steps (graph replay) + steps (the eager timing pass)
    infers are kept — the launches bench.py's roofline times."""
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    n_keep = b["warmup"] + 2 * b["steps"]
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    g = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    infer = 0
    for r in rows:
        if "patchify_kernel" in r["Kernel_Name"]:
            infer += 1
        if infer < 1 or infer > n_keep:
            continue
        k = group(r["Kernel_Name"])
        g[k]["calls"] += 1
        g[k]["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {k: dict(v, avg_us=v["total_ns"] / v["calls"] / 1e3) for k, v in g.items()}
    rf = b.get("roofline") or {}
    out["infers"] = n_keep
    out["bench_dominant"] = {"kernel": rf.get("kernel"), "avg_launch_us": rf.get("avg_launch_us")}
    if rf.get("kernel") in out:
        out["bench_dominant"]["rocprof_avg_us"] = out[rf["kernel"]]["avg_us"]
        out["bench_dominant"]["ratio"] = rf["avg_launch_us"] / out[rf["kernel"]]["avg_us"]
    return out


def traffic(fetch_csv, write_csv, fetch_log=None, write_log=None):
    acc = defaultdict(lambda: defaultdict(list))
    for path, counter, log in ((fetch_csv, "FETCH_SIZE", fetch_log), (write_csv, "WRITE_SIZE", write_log)):
        rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        ks = dispatch_kinds([r["Kernel_Name"] for r in rows], log) if log else [None] * len(rows)
        for r, k in zip(rows, ks):
            acc[k or group(r["Kernel_Name"])][counter].append(float(r["Counter_Value"]))
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


def mfma(pattern, paths):
    """Per-dispatch MFMA-pipe busy fraction of the kernels matching `pattern`, at the clock the chip actually ran.

    SQ counters are summed over the 32 shader engines.  SQ_VALU_MFMA_BUSY_CYCLES sums busy cycles over all 1024
    SIMDs (it equals SQ_INSTS_MFMA x 32 for v_mfma_f32_32x32x16_bf16), so the busy fraction over the cycles the
    sequencers had work = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x SQ_BUSY_CYCLES / 32), and the clock = SQ_BUSY_CYCLES / 32
    / duration.  (SQ_CYCLES / 32 / duration reads above the 2.4 GHz maximum on short kernels — its window is wider
    than the dispatch timestamps — so it is reported only as an upper-bound clock.)"""
    per = defaultdict(dict)  # (file, dispatch) -> counters
    for path in paths:
        for r in csv.DictReader(open(path)):
            if not re.search(pattern, r["Kernel_Name"]):
                continue
            d = per[(path, r["Dispatch_Id"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = defaultdict(list)
    for d in per.values():
        for k, v in d.items():
            agg[k].append(v)
    mean = {k: sum(v) / len(v) for k, v in agg.items()}
    out = {"dispatches_per_pass": len(per) // max(1, len(paths)), "counters_mean": mean}
    if "SQ_BUSY_CYCLES" in mean:
        out["clock_ghz"] = mean["SQ_BUSY_CYCLES"] / 32.0 / mean["dur_ns"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            out["mfma_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * mean["SQ_BUSY_CYCLES"] / 32.0)
    if "SQ_CYCLES" in mean:
        out["clock_ghz_upper"] = mean["SQ_CYCLES"] / 32.0 / mean["dur_ns"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            out["mfma_busy_frac_lower"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * mean["SQ_CYCLES"] / 32.0)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "SQ_VALU_MFMA_COEXEC_CYCLES" in mean:
        out["valu_coexec_frac_of_mfma_busy"] = mean["SQ_VALU_MFMA_COEXEC_CYCLES"] / mean["SQ_VALU_MFMA_BUSY_CYCLES"]
    if "SQ_INSTS_VALU" in mean and "SQ_INSTS_MFMA" in mean:
        out["valu_insts_per_mfma"] = (mean["SQ_INSTS_VALU"] - mean["SQ_INSTS_MFMA"]) / mean["SQ_INSTS_MFMA"]
    if "SQ_WAIT_INST_ANY" in mean and "SQ_WAVE_CYCLES" in mean:
        out["wait_inst_frac_of_wave_cycles"] = mean["SQ_WAIT_INST_ANY"] / mean["SQ_WAVE_CYCLES"]
    return out


def _dispatch_order(per):
    return sorted(per, key=lambda d: int(d))


def mfma_groups(path, log_path=None):
    """Per kernel group (as bench.py names them): MFMA-pipe busy fraction over the sequencer-busy cycles and the
    clock (see mfma()), time-weighted over every dispatch of a PMC pass with SQ_BUSY_CYCLES +
    SQ_VALU_MFMA_BUSY_CYCLES."""
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = per[r["Dispatch_Id"]]
        d["group"] = group(r["Kernel_Name"])
        d["name"] = r["Kernel_Name"]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if log_path:
        order = _dispatch_order(per)
        for did, k in zip(order, dispatch_kinds([per[i]["name"] for i in order], log_path)):
            if k:
                per[did]["group"] = k
    acc = defaultdict(lambda: {"launches": 0, "busy": 0.0, "sq_busy": 0.0, "ns": 0.0})
    for d in per.values():
        if "SQ_BUSY_CYCLES" not in d or "SQ_VALU_MFMA_BUSY_CYCLES" not in d or d["dur_ns"] <= 0:
            continue
        a = acc[d["group"]]
        a["launches"] += 1
        a["busy"] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["sq_busy"] += d["SQ_BUSY_CYCLES"] / 32.0
        a["ns"] += d["dur_ns"]
    return {k: {"launches": v["launches"], "mfma_busy_frac": v["busy"] / (1024.0 * v["sq_busy"]),
                "clock_ghz": v["sq_busy"] / v["ns"],
                "note": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x SQ_BUSY_CYCLES / 32 SEs), summed over launches"}
            for k, v in acc.items() if v["sq_busy"] > 0}


def agree(kinds_json, bench):
    """The bench line's dominant kernel class: its HIP-event average launch vs rocprofv3's average for the same class
    in the eager per-kind trace (launch-log-named dispatches, so split / LayerNorm-fused GEMMs are told apart)."""
    b = json.load(open(bench))
    r = b["roofline"]
    k = json.load(open(kinds_json)).get(r["kernel"], {})
    return {"kernel": r["kernel"], "bench_avg_launch_us": r["avg_launch_us"], "rocprof_eager_avg_us": k.get("avg_us"),
            "ratio": (r["avg_launch_us"] / k["avg_us"]) if k.get("avg_us") else None, "rocprof_calls": k.get("calls")}


if __name__ == "__main__":
    a = sys.argv
    if a[1] == "mfma_groups":
        print(json.dumps(mfma_groups(a[2], a[3] if len(a) > 3 else None), indent=1))
    elif a[1] == "mfma":
        print(json.dumps(mfma(a[2], a[3:]), indent=1))
    elif a[1] == "stats":
        print(json.dumps(stats(a[2], a[3] if len(a) > 3 else None), indent=1))
    elif a[1] == "headline":
        print(json.dumps(headline(a[2], a[3]), indent=1))
    elif a[1] == "kinds":
        print(json.dumps(kinds(a[2], a[3]), indent=1))
    elif a[1] == "agree":
        print(json.dumps(agree(a[2], a[3]), indent=1))
    elif a[1] == "shapes":
        per = kinds(a[2], a[3], keep_shape=True)
        print(json.dumps(dict(sorted(per.items(), key=lambda kv: -kv[1]["total_ns"])), indent=1))
    else:
        print(json.dumps(traffic(a[2], a[3], *(a[4:6] if len(a) > 5 else (None, None))), indent=1))
