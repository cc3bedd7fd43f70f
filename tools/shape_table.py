"""Per-shape table of the path GEMMs and split-precision head convs from tools/shape_pmc.sh output:
time and TF/s (kbench, HIP events, random data) next to hipBLASLt on the same box, L2-fabric traffic (FETCH_SIZE x 2
+ WRITE_SIZE, rocprofv3 PMC) against the algorithmic bytes (A + W read once, the bf16 output written once), the
operand bytes the tile schedule stages into LDS (tiles x (BM + BN) x K x 2), and the MFMA-pipe busy fraction at
the clock the chip ran.  Usage: python tools/shape_table.py gpurun_out/shape > profiles/r2/gemm_shapes.json"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import _is_gemm  # noqa: E402

V, T = 8, 1369
R, L = V * (T + 1), V * T + 1
GEMMS = [("enc.qkv", R, 3072, 1024), ("enc.proj", R, 1024, 1024), ("enc.fc1", R, 4096, 1024),
         ("enc.fc2", R, 1024, 4096), ("aat.qkv", L, 2304, 768), ("aat.proj", L, 768, 768),
         ("aat.fc1", L, 3072, 768), ("aat.fc2", L, 768, 3072), ("pose.res", V * T, 784, 784)]
CONVS = [("l1rn@148", 148, 288, 256), ("l2rn@74", 74, 576, 256), ("l3rn@37", 37, 1152, 256), ("l4rn@19", 19, 2304, 256),
         ("rn4@19", 19, 768, 256), ("rn3@37", 37, 768, 256), ("rn2@74", 74, 768, 256), ("rn1@148", 148, 768, 256),
         ("reg1@296", 296, 768, 128), ("reg2@518", 518, 384, 128)]
PER = 8  # dispatches per shape per function in a PMC run (3 warm-up + 5)


def dispatches(path):
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = per[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [per[k] for k in sorted(per)]


def chunks(ds, pred, n):
    sel = [d for d in ds if pred(d["name"])]
    return [sel[i * PER:(i + 1) * PER] for i in range(n)]


def mean(xs, key):
    v = [x[key] for x in xs if key in x]
    return sum(v) / len(v) if v else None


def tile_of(name):
    if "conv_halo_kernel" in name:
        return None  # halo conv: staged bytes are not (BM + BN) x K
    m = re.search(r"gemm_big_kernel<(\d), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", name)
    if m:
        return int(m.group(8)), int(m.group(2))
    if "gemm_sk_kernel" in name:
        m = re.search(r"gemm_sk_kernel<\d, (\d+)", name)
        return 256, int(m.group(1))
    if "gemm_kernel<" in name:
        return 128, 128
    return None


def timings(log, kind):
    ours, blas = {}, {}
    for line in open(log):
        m = re.match(rf"{kind} (\S+)\s+v0\s.*:\s+([\d.]+) us\s+([\d.]+) TF/s", line)
        if m:
            ours[m.group(1)] = (float(m.group(2)), float(m.group(3)))
        m = re.match(rf"{kind} (\S+)\s+hipBLASLt via torch:\s+([\d.]+) us\s+([\d.]+) TF/s", line)
        if m:
            blas[m.group(1)] = (float(m.group(2)), float(m.group(3)))
    return ours, blas


def table(root, kind):
    shapes = GEMMS if kind == "gemm" else CONVS
    f = dispatches(glob.glob(f"{root}/f_{kind}/**/*counter_collection.csv", recursive=True)[0])
    w = dispatches(glob.glob(f"{root}/w_{kind}/**/*counter_collection.csv", recursive=True)[0])
    m = dispatches(glob.glob(f"{root}/m_{kind}/**/*counter_collection.csv", recursive=True)[0])
    ours_t, blas_t = timings(f"{root}/kb_{kind}.log", kind)
    cf, cw, cm = (chunks(x, _is_gemm, len(shapes)) for x in (f, w, m))
    bl = lambda n: n.startswith("Cijk")  # noqa: E731
    bf, bw, bm = (chunks(x, bl, len(shapes)) for x in (f, w, m)) if kind == "gemm" else ([], [], [])
    out = []
    for i, sh in enumerate(shapes):
        if kind == "gemm":
            name, M, N, K = sh
            alg = (M * K + N * K + M * N) * 2
        else:
            name, hw, C, N = sh
            M, K = V * hw * hw, 9 * C
            alg = (V * hw * hw * (2 * C // 3) + N * K + M * N) * 2  # compact split input [hi | lo], out once
        flop = 2.0 * M * N * K
        row = {"shape": name, "M": M, "N": N, "K": K, "gflop": flop / 1e9, "algorithmic_bytes": alg}
        if name in ours_t:
            row["us"], row["tflops"] = ours_t[name]
        if name in blas_t:
            row["hipblaslt_us"], row["hipblaslt_tflops"] = blas_t[name]
            row["vs_hipblaslt"] = row["hipblaslt_us"] / row["us"]
        k = cf[i][0]["name"] if cf[i] else ""
        row["kernel"] = re.sub(r"\(mapa_gemm_impl::GemmArgs.*|\(mapa_gemm_impl::\(anonymous.*", "", k).replace(
            "void mapa_gemm_impl::(anonymous namespace)::", "")
        fb, wb = mean(cf[i], "FETCH_SIZE"), mean(cw[i], "WRITE_SIZE")
        if fb is not None and wb is not None:
            row["fabric_bytes"] = 2048.0 * fb + 1024.0 * wb
            row["fabric_over_algorithmic"] = row["fabric_bytes"] / alg
        t = tile_of(k)
        if t:
            bm_, bn_ = t
            tiles = -(-M // bm_) * -(-N // bn_)
            row["tile"] = f"{bm_}x{bn_}"
            row["tiles"] = tiles
            row["staged_bytes"] = tiles * (bm_ + bn_) * K * 2
            if "us" in row:
                row["staged_tb_per_s"] = row["staged_bytes"] / row["us"] / 1e6
        busy, sqb, ns = mean(cm[i], "SQ_VALU_MFMA_BUSY_CYCLES"), mean(cm[i], "SQ_BUSY_CYCLES"), mean(cm[i], "ns")
        if busy and sqb:
            row["mfma_busy_frac"] = busy / (1024.0 * sqb / 32.0)
            row["clock_ghz"] = sqb / 32.0 / ns
        if kind == "gemm" and bf and bf[i]:
            fb2, wb2 = mean(bf[i], "FETCH_SIZE"), mean(bw[i], "WRITE_SIZE")
            if fb2 is not None and wb2 is not None:
                row["hipblaslt_fabric_bytes"] = 2048.0 * fb2 + 1024.0 * wb2
            b2, s2, n2 = mean(bm[i], "SQ_VALU_MFMA_BUSY_CYCLES"), mean(bm[i], "SQ_BUSY_CYCLES"), mean(bm[i], "ns")
            if b2 and s2:
                row["hipblaslt_mfma_busy_frac"] = b2 / (1024.0 * s2 / 32.0)
                row["hipblaslt_clock_ghz"] = s2 / 32.0 / n2
        out.append(row)
    return out


if __name__ == "__main__":
    root = sys.argv[1]
    print(json.dumps({"gemm": table(root, "gemm"), "conv3x3_split": table(root, "conv"),
                      "note": "8 views at 518x518 (M = 10960 / 10953 rows); random data; fabric bytes = FETCH_SIZE x 2 "
                              "(gfx950 16-B streaming-read correction) + WRITE_SIZE per launch, Infinity-Cache hits "
                              "included; staged = operand bytes the tile schedule moves L2 -> LDS"}, indent=1))
