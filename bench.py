"""MapAnything feed-forward inference benchmark on MI355X (views/sec, N-view 518x518 bf16).

  python bench.py                        # N=1: configs[1] = 8 views 518x518 bf16 image-only infer on 1 GPU
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
      bench.py --gpus N                  # 8 views per GPU (weak scaling), global-attention K/V all-gathered
  python bench.py --gpus N               # the same: without WORLD_SIZE in the environment and N > 1 this process
                                         # (which never touches the GPU) starts that torch.distributed.run itself
                                         # and exits with its status; rank 0's JSON line is the output
  ... bench.py --gpus N --total-views 100  # configs[2]: a fixed 100-view job split over the N ranks (strong)
  python bench.py --gpus 2 --dry-run     # launcher rehearsal on CPU: gloo ranks, no GPU, a placeholder step

One step = one full `MapAnything.infer(views)` (validation, forward, post-processing with edge masks) over
synthetic images with inputs already resident in HBM, in the reference's own GPU precision recipe: bf16 autocast
encoder and transformer; geometric encoders and heads with autocast disabled (model.py:1377 / 1774), i.e. at the
TF32 precision the reference's fp32 convs / linears run at on its GPUs (cudnn's default, matmul.allow_tf32 at
model.py:93) — here binary16 operands at TF32's 11 significant bits with fp32 accumulation (--head-precision tf32, the
default), with the binary16 range closed by power-of-two weight scales and an automatic fp32-exact re-run of a call
whose head activations leave binary16's range (`range_fallbacks` counts them; expect 0).  The same JSON line carries,
as nested objects: the fp32-exact heads (`fp32_exact_heads`, split-precision bf16 x3), the opt-in bf16-heads fast
mode (N=1; not the reference's recipe, never the headline), the forward-only time (`forward_only`: the raw
MapAnything.forward without input validation / pre- and post-processing), and the configs[2] strong-scaling job (a
fixed 100 views over the N ranks: `strong_scaling`, measured at every N so the curve can be read off the driver's
per-N lines).  At N > 1 (or --shard-rehearsal on one GPU) `kv_overlap` reports each global layer's K/V all-gather
time on the communicator's stream beside the local- and remote-key attention and the join's exposed wait.  On one GPU
the engine's launches are replayed from a captured HIP graph (MapAnything.hip_graphs); per-kernel timing for the
roofline comes from a second, eager pass of the same steps with an event pair around every native call.  Prints ONE
JSON line on rank 0.
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "map-anything_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
PROFILE_ROUND = "r6"          # profiles/<round>/: the rocprofv3 PMC summaries the roofline / attention objects cite


def enc_linear_flops_per_view(T):
    """DINOv2 linears + patch-embed per view (2*M*N*K), M = T+1 tokens (T for patch embed)."""
    R = T + 1
    per_block = 2 * R * (1024 * 3072 + 1024 * 1024 + 1024 * 4096 * 2)
    return 24 * per_block + 2 * T * 588 * 1024


_JSON_FD = None  # a private dup of the real stdout: the one JSON line goes there (_protect_stdout)


def _protect_stdout():
    """Native libraries write to fd 1 — RCCL prints its version banner to stdout when a communicator is created (the
    N > 1 path and --shard-rehearsal) — which would put non-JSON lines in front of rank 0's JSON line.  Keep a dup of
    the real stdout for that line and point fd 1 (and with it Python's own prints) at stderr."""
    global _JSON_FD
    if _JSON_FD is not None:
        return
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)


def _emit(obj):
    """The bench's one JSON line, on the real stdout."""
    line = json.dumps(obj) + "\n"
    if _JSON_FD is None:
        sys.stdout.write(line)
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line.encode())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--views-per-gpu", type=int, default=8)
    ap.add_argument("--total-views", type=int, default=0,
                    help="strong scaling: this many views split over the ranks (configs[2]: 100), else views-per-gpu")
    ap.add_argument("--res", type=int, default=518)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="autocast operand dtype of the encoder / transformer (infer(amp_dtype=...)); fp32 = use_amp off")
    ap.add_argument("--head-precision", default="tf32", choices=["tf32", "tf32x2", "fp32", "bf16"],
                    help="tf32 (default) = the reference's GPU recipe for its autocast-disabled heads (TF32-equivalent "
                         "binary16 operands, fp32 accumulation); tf32x2 = 22-bit activations; fp32 = fp32-exact "
                         "split-bf16 heads; bf16 = fast mode (not the reference's recipe)")
    ap.add_argument("--shard-rehearsal", action="store_true",
                    help="N=1 only: run the view-sharded path on a one-rank RCCL group with MAPA_FORCE_OVERLAP=1 (the "
                         "N > 1 global layers' overlapped all-gather branch) and report kv_overlap")
    ap.add_argument("--no-forward-only", action="store_true", help="skip the forward-only timing")
    ap.add_argument("--from-files-src", type=int, default=1024,
                    help="N=1: also time infer from JPEG files (this many pixels a side, resized to 518 on the host "
                         "by the reference's pipeline, prefetched one scene ahead); 0 = skip")
    ap.add_argument("--no-fast-mode", action="store_true", help="skip the bf16-heads fast-mode measurement")
    ap.add_argument("--strong-views", type=int, default=100,
                    help="also time a fixed job of this many views over the N ranks (configs[2]); 0 = skip")
    ap.add_argument("--strong-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--batch-scenes", type=int, default=2,
                    help="N=1: also time B scenes of views-per-gpu views per infer (batched scenes); 0 = skip")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--geometric", action="store_true",
                    help="cfg4 inputs: + intrinsics, 90%%-sparse depth_z, is_metric_scale on every view")
    ap.add_argument("--cfg4-views", type=int, default=32,
                    help="N=1: also time configs[3] (this many views, images + intrinsics + 90%%-sparse depth, "
                         "metric) as the nested multimodal_cfg4 object; 0 = skip")
    ap.add_argument("--cfg4-steps", type=int, default=5)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", PROFILE_ROUND, "pmc_traffic.json"),
                    help="HBM bytes per launch from rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/profile_summary.py)")
    ap.add_argument("--mfma-pmc-json", default=os.path.join(REPO, "profiles", PROFILE_ROUND, "pmc_mfma.json"),
                    help="per-kernel-group MFMA busy fraction + clock from a rocprofv3 SQ pass (tools/gpu_pmc.sh)")
    ap.add_argument("--attn-pmc-json", default=None,
                    help="global-attention MFMA busy fraction from rocprofv3 PMC passes (tools/attn_pmc.sh); default: "
                         f"profiles/{PROFILE_ROUND}/attn_global_pmc.json (8 views) or attn_global_v100_pmc.json (>= 100 views)")
    ap.add_argument("--lib", default=None, help="A/B only: load this libmapa.so build (tools/ab_build.sh)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal without a GPU: gloo process group, placeholder CPU step (tests only)")
    ap.add_argument("--fail-rank", type=int, default=-1, help="dry-run only: this rank exits with an error")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    _protect_stdout()
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.lib:
        from mapanything import _native

        _native.load_library(args.lib)

    observed_world = 1
    sharded = world > 1 or args.shard_rehearsal
    if sharded:
        import torch.distributed as dist

        from mapanything.parallel import init_distributed

        if args.shard_rehearsal:
            if world != 1:
                raise SystemExit("bench.py: --shard-rehearsal is a one-GPU rehearsal of the N > 1 path")
            os.environ["MAPA_FORCE_OVERLAP"] = "1"  # parallel.force_overlap: the overlapped multi-rank branch
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local_rank)
        _, observed_world = init_distributed("nccl", torch.device("cuda", local_rank))
        assert observed_world == args.gpus, (observed_world, args.gpus)
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from mapanything.models import MapAnything
    from mapanything.utils import synthetic
    from tests_helpers import released_config

    V_total = args.total_views or args.views_per_gpu * world
    H = W = args.res
    model = MapAnything(**released_config(), precision=args.precision,
                        head_precision=args.head_precision).load_synthetic_weights().to(dev).eval()
    if sharded:
        model.enable_view_sharding(dist.group.WORLD)
    imgs = synthetic.synthetic_images(V_total, H, W, seed=2)
    views = [{"img": torch.from_numpy(i).to(dev), "data_norm_type": ["dinov2"]} for i in imgs]
    if args.geometric:
        Ks = synthetic.synthetic_intrinsics(V_total, H, W, seed=4)
        Ds = synthetic.synthetic_sparse_depth(V_total, H, W, seed=4)
        for v, K, D in zip(views, Ks, Ds):
            v.update(intrinsics=torch.from_numpy(K).to(dev), depth_z=torch.from_numpy(D).to(dev),
                     is_metric_scale=torch.ones(1, dtype=torch.bool, device=dev))

    amp = dict(use_amp=args.precision != "fp32", amp_dtype=args.precision if args.precision != "fp32" else "bf16")

    def step():
        return model.infer(views, **amp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng = model.engine()
    shard_check = shard_graph_self_check(model, step, dist, dev) if sharded else None

    def timed(k):
        return timed_fn(step, k)

    def timed_fn(fn, k):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    # timed region: the production path (the engine's launches replayed from a HIP graph: one GPU, or a view shard
    # whose K/V all-gathers run on RCCL inside the graph)
    dt = timed(args.steps)
    ktimes, instr_ms = {}, None
    if not args.no_kernel_timing:
        # per-launch HIP events cannot ride inside a graph replay: the same K steps again, launched eagerly with
        # an event pair around every native call, give each kernel family's average launch duration
        eng.enable_kernel_timing()
        instr_ms = timed(args.steps) / args.steps * 1e3
        ktimes = eng.collect_kernel_timing()
    ms = dt / args.steps * 1e3
    value = V_total * args.steps / dt

    fwd = None
    if not args.no_forward_only:
        # the raw forward (model.py:1657-2152) on the same views, preprocessed once outside the timed region: the
        # infer() time minus input validation / preprocessing and the post-processing masks
        from mapanything.utils.inference import preprocess_input_views_for_inference, validate_input_views_for_inference

        pre = preprocess_input_views_for_inference(validate_input_views_for_inference(
            [dict(v) for v in views]))
        fprec = args.precision
        model.forward(pre, precision=fprec)
        fdt = timed_fn(lambda: model.forward(pre, precision=fprec), args.steps)
        fwd = {"ms_per_step": fdt / args.steps * 1e3, "value": V_total * args.steps / fdt, "unit": "views/s",
               "steps": args.steps, "what": "MapAnything.forward on preprocessed views (no validation / "
                                            "preprocessing / post-processing masks), same HIP-graph path"}
        del pre

    def other_heads(hp):
        fm = MapAnything(**released_config(), precision=args.precision, head_precision=hp).to(dev).eval()
        fm._sd = model._sd
        for _ in range(args.warmup):
            fm.infer(views, **amp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fm.infer(views, **amp)
        torch.cuda.synchronize()
        fdt = time.perf_counter() - t0
        del fm
        torch.cuda.empty_cache()
        return {"value": V_total * args.steps / fdt, "unit": "views/s", "ms_per_step": fdt / args.steps * 1e3,
                "head_precision": hp}

    fast = exact = None
    if world == 1 and not args.no_fast_mode and args.head_precision != "bf16" and args.precision == "bf16":
        # opt-in bf16-heads fast mode on the same workload (NOT the reference's recipe; reported, never headline)
        fast = other_heads("bf16")
        fast["note"] = ("opt-in fast mode: DPT / pose heads on plain bf16 operands (the reference runs them with "
                        "autocast disabled, model.py:1774); not like-for-like, not the headline")
        if args.head_precision == "tf32":  # the fp32-exact split-bf16 heads beside the TF32-equivalent headline
            exact = other_heads("fp32")
            exact["note"] = ("heads fp32-exact (split bf16 x3, ~2^-16 relative per product) instead of the reference's "
                             "TF32 recipe: the previous rounds' headline configuration")

    batched = None
    if world == 1 and args.batch_scenes > 1 and not args.geometric and not args.total_views:
        # B scenes x V views per infer (each view's img (B, 3, H, W)), run as one batched engine call
        B = args.batch_scenes
        b_imgs = synthetic.synthetic_images(V_total, H, W, seed=2, batch=B)
        b_views = [{"img": torch.from_numpy(i).to(dev), "data_norm_type": ["dinov2"]} for i in b_imgs]
        del b_imgs
        for _ in range(max(1, args.warmup)):
            model.infer(b_views, **amp)
        bdt = timed_fn(lambda: model.infer(b_views, **amp), args.steps)
        batched = {"scenes": B, "views_per_scene": V_total, "value": B * V_total * args.steps / bdt, "unit": "views/s",
                   "ms_per_step": bdt / args.steps * 1e3, "steps": args.steps,
                   "workload": f"{B} scenes x {V_total} views {H}x{W} per infer (batched: one engine call)",
                   "vs_single_scene": (B * V_total * args.steps / bdt) / value}
        del b_views
        torch.cuda.empty_cache()

    files = None
    if world == 1 and args.from_files_src and not args.geometric and not args.total_views and H == 518:
        files = bench_from_files(model, amp, V_total, args, timed_fn)

    cfg4 = None
    if world == 1 and args.cfg4_views and not args.geometric and not args.total_views:
        cfg4 = bench_cfg4(model, amp, dev, H, W, args, timed_fn)

    strong = None
    if args.strong_views and not args.total_views and not args.geometric and args.strong_views >= world:
        # configs[2]: a fixed job of strong_views views split over the N ranks (strong scaling)
        s_imgs = synthetic.synthetic_images(args.strong_views, H, W, seed=3)
        s_views = [{"img": torch.from_numpy(i).to(dev), "data_norm_type": ["dinov2"]} for i in s_imgs]
        del s_imgs
        model.infer(s_views, **amp)  # warm-up (graph capture)
        sdt = timed_fn(lambda: model.infer(s_views, **amp), args.strong_steps)
        strong = {"views": args.strong_views, "value": args.strong_views * args.strong_steps / sdt, "unit": "views/s",
                  "ms_per_step": sdt / args.strong_steps * 1e3, "steps": args.strong_steps, "warmup": 1,
                  "scaling": "strong", "views_per_gpu": args.strong_views / world,
                  "workload": f"{args.strong_views}-view {H}x{W} image-only MapAnything.infer (configs[2]), "
                              f"views sharded over {world} rank(s)"}
        del s_views
        torch.cuda.empty_cache()

    if rank == 0:
        T = (H // 14) * (W // 14)
        roofline = None
        if ktimes:
            # dominant kernel by total time inside the timed region
            kind = max(ktimes, key=lambda k: ktimes[k]["ms"])
            kt = ktimes[kind]
            achieved = kt["flops"] / (kt["ms"] * 1e-3) / 1e12 if kt["flops"] else None
            traffic = None
            if os.path.exists(args.traffic_json):
                tj = json.load(open(args.traffic_json)).get(kind)
                traffic = tj["hbm_bytes_per_launch"] if tj else None
            mfma_pmc = None
            if os.path.exists(args.mfma_pmc_json):
                # MFMA-pipe busy fraction + clock of this kernel class from a rocprofv3 SQ-counter pass
                mfma_pmc = json.load(open(args.mfma_pmc_json)).get(kind)
            roofline = {"kernel": kind, "bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                        "unit": "TFLOP/s", "frac": (achieved / PEAK_BF16_TFLOPS) if achieved else None,
                        "traffic": traffic,
                        "traffic_unit": "bytes/launch: L2 fabric fetch (FETCH_SIZE x2, Infinity-Cache hits included) + WRITE_SIZE, rocprofv3 PMC, " + os.path.relpath(args.traffic_json, REPO),
                        "pmc": mfma_pmc,
                        "launches": kt["count"], "avg_launch_us": kt["ms"] * 1e3 / kt["count"],
                        "timing_pass": {"ms_per_step": instr_ms, "launch": "eager, event pair per native call",
                                        "note": "same K steps re-run after the timed region"},
                        "per_kernel": {k: {"ms_per_step": v["ms"] / args.steps,
                                           "tflops": (v["flops"] / (v["ms"] * 1e-3) / 1e12) if v["flops"] else None}
                                       for k, v in ktimes.items()}}
        xattn = None
        if ktimes.get("attention_global", {}).get("flops"):
            # north_star target: >= 40 % MFMA utilisation in the cross-view (global AAT) attention kernel
            v = ktimes["attention_global"]
            tf = v["flops"] / (v["ms"] * 1e-3) / 1e12
            xattn = {"kernel": "attn_fwd_bf16 (global AAT layers, L = V*1369+1 keys)", "achieved": tf,
                     "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": tf / PEAK_BF16_TFLOPS, "target_frac": 0.40,
                     "ms_per_step": v["ms"] / args.steps, "launches_per_step": v["count"] / args.steps}
            attn_pmc = args.attn_pmc_json or os.path.join(
                REPO, "profiles", PROFILE_ROUND, "attn_global_v100_pmc.json" if V_total >= 100 else "attn_global_pmc.json")
            if os.path.exists(attn_pmc):
                # MFMA-pipe busy fraction at the clock the chip really ran (rocprofv3 PMC pass, tools/attn_pmc.sh)
                pj = json.load(open(attn_pmc))
                xattn["pmc"] = {k: pj.get(k) for k in ("mfma_busy_frac", "mfma_busy_frac_lower", "clock_ghz",
                                                       "clock_ghz_upper", "valu_insts_per_mfma",
                                                       "valu_coexec_frac_of_mfma_busy")}
                xattn["pmc"]["source"] = os.path.relpath(attn_pmc, REPO)
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not args.geometric:
            cpu = cpu_baseline(model, imgs, H, W)
        kvo = kv_overlap(ktimes) if ktimes else None
        L = V_total * T + 1
        gf_view = (1870.9e9 + 36864.0 * L * L / V_total + (165.6e9 if args.geometric else 0.0)) / 1e12 \
            if H == 518 else None
        line = {
            "metric": "views/sec + ms/infer, N-view 518x518 bf16 at 1/2/4/8 MI355X",
            "value": value, "unit": "views/s", "n_gpus": world, "world_size_observed": observed_world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "strong" if args.total_views else "weak",
            "vs_baseline": None,
            "dtype": args.precision, "data": "synthetic (seeded uint8 images, named-PRNG synthetic weights)",
            "head_precision": args.head_precision,
            "precision_recipe": {
                "tf32": "reference GPU recipe: bf16 autocast encoder + transformer; geometric encoders and heads "
                        "(autocast disabled, model.py:1377 / 1774) at the TF32 precision the reference's fp32 convs / "
                        "linears run at on its GPUs (cudnn default, matmul.allow_tf32 at model.py:93): binary16 "
                        "operands (TF32's 11 significant bits), fp32 accumulation",
                "tf32x2": "as tf32 with 22-bit activations (binary16 [hi | lo] x f16 weights, 2x the head work)",
                "fp32": "reference autocast recipe with fp32-exact geometric encoders and heads (split-precision bf16 "
                        "GEMMs)",
                "bf16": "bf16 heads (fast mode, not the reference recipe)"}[args.head_precision],
            "config": {"workload": f"{V_total}-view {H}x{W} " + (
                           "images+intrinsics+sparse depth (cfg4 inputs)" if args.geometric else
                           ("image-only MapAnything.infer (fixed job, strong scaling)" if args.total_views else
                            "image-only MapAnything.infer (configs[1] at N=1)")),
                       "views": V_total, "views_per_gpu": V_total / world, "height": H, "width": W,
                       "batch_per_view": 1,
                       "parallelism": f"view-sharded x{world} + RCCL K/V all-gather" if world > 1 else
                       ("one-rank RCCL shard rehearsal (MAPA_FORCE_OVERLAP=1)" if sharded else "single")},
            # algorithmic TFLOP/s of the whole job (global attention grows as (V*1369)^2: per-view work rises with
            # the total view count, so weak-scaling views/s alone understates the per-GPU throughput at N > 1)
            "tflops_effective": (gf_view * value) if gf_view else None,
            "tflops_effective_per_gpu": (gf_view * value / world) if gf_view else None,
            "tflop_per_view": gf_view,
            "roofline": roofline,
            "cross_view_attention": xattn,
            "cpu_baseline": cpu,
            "batched_scenes": batched,
            "multimodal_cfg4": cfg4,
            "fast_mode_bf16_heads": fast,
            "fp32_exact_heads": exact,
            "strong_scaling": strong,
            "forward_only": fwd,
            "from_files": files,
            "kv_overlap": kvo,
            "range_fallbacks": MapAnything.range_fallbacks,
            # one GPU, or a view shard over RCCL (kernels and collectives captured together; MAPA_SHARD_GRAPHS=0 or a
            # failed capture on any rank: eager, with the reason)
            "hip_graphs": bool(model.hip_graphs and (not sharded or model._shard_graphs)),
            "hip_graph_fallback": None if not sharded else model.shard_graph_fallback,
            "shard_graph_check": shard_check,
        }
        _emit(line)
    if dist is not None:
        dist.destroy_process_group()


def bench_from_files(model, amp, V, args, timed_fn):
    """End to end from image files: V square JPEGs of --from-files-src pixels a side per scene, decoded, Lanczos-
    resized to 518x518 and normalised by the input pipeline (utils/image.py, the reference's load_images), then
    infer().  Sequential (load_images then infer, per scene) and prefetched (iter_load_images: the next scene's host
    decode runs on host threads under this scene's GPU work), for the GPU resize (default) and the host PIL resize.
    Not the headline: it includes the host's JPEG decode rate."""
    import tempfile

    import PIL.Image

    from mapanything.utils.image import iter_load_images, load_images
    from tests_helpers import synthetic_image

    S = args.from_files_src
    tmp = tempfile.mkdtemp(prefix="mapa_bench_")
    paths = []
    for i in range(V):  # smooth seeded photographs-like images (gradients, discs, mild noise)
        p = os.path.join(tmp, f"view_{i:03d}.jpg")
        PIL.Image.fromarray(synthetic_image(S, S, 100 + i)).save(p, quality=95)
        paths.append(p)
    steps = max(2, args.steps // 2)

    def leg(gpu_resize):
        model.infer(load_images(paths, gpu_resize=gpu_resize), **amp)  # warm-up
        seq = timed_fn(lambda: model.infer(load_images(paths, gpu_resize=gpu_resize), **amp), steps)
        t_load = timed_fn(lambda: load_images(paths, gpu_resize=gpu_resize), steps)

        def prefetched():
            for views in iter_load_images([paths] * steps, prefetch=1, gpu_resize=gpu_resize):
                model.infer(views, **amp)
        pre = timed_fn(prefetched, 1)
        return {"sequential": {"value": V * steps / seq, "unit": "views/s", "ms_per_step": seq / steps * 1e3},
                "prefetched": {"value": V * steps / pre, "unit": "views/s", "ms_per_step": pre / steps * 1e3},
                "load_only": {"value": V * steps / t_load, "unit": "views/s", "ms_per_step": t_load / steps * 1e3}}
    gpu = leg(True)
    pil = leg(False)
    for p in paths:
        os.remove(p)
    os.rmdir(tmp)
    threads = min(16, os.cpu_count() or 1)
    return {"views": V, "src": f"{S}x{S} JPEG (q95) -> 518x518 Lanczos (fixed_mapping)", "steps": steps,
            **gpu, "host_threads": threads,
            "pil_resize": pil,
            "note": "default loader: host JPEG decode (PIL, thread pool) + GPU resize / crop / normalise "
                    "(mapa_resize_normalize, bit-identical with PIL's Image.resize); pil_resize: the host PIL resize "
                    "path.  load_only = the loader alone (decode + H2D + resize, synchronised).  The in-HBM "
                    "headline excludes the loader"}


def kv_overlap(ktimes):
    """The overlapped global layer of the view-sharded path (engine._block_global_sharded), per layer, from the eager
    timing pass: the K/V all-gather on the communicator's stream, the local- and remote-key attention on the compute
    stream, and the join's exposed wait (local attention done -> gathered slots visible).  overlap_frac = 1 - wait /
    all-gather: the share of the all-gather hidden under the local-key attention.  None without a sharded run."""
    g, la = ktimes.get("kv_allgather"), ktimes.get("kv_local_attention")
    ra, wt = ktimes.get("kv_remote_attention"), ktimes.get("kv_gather_wait")
    if not (g and la and ra and wt):
        return None
    ag = g["ms"] / g["count"]
    wait = wt["ms"] / wt["count"]
    return {"allgather_ms_per_layer": ag, "local_attn_ms": la["ms"] / la["count"],
            "remote_attn_ms": ra["ms"] / ra["count"], "gather_wait_ms": wait,
            "overlap_frac": max(0.0, min(1.0, 1.0 - wait / ag)) if ag > 0 else None, "layers_timed": g["count"],
            "source": "eager timing pass: HIP events on the communicator's stream (all-gather) and the compute "
                      "stream (attention, join)"}


def bench_cfg4(model, amp, dev, H, W, args, timed_fn):
    """configs[3]: 32 views 518x518, images + intrinsics + 90 %-sparse depth_z + is_metric_scale on every view, one
    infer per step on one GPU (the geometric encoders fp32-exact as split-precision GEMMs; HIP-graph replayed with
    the ray / depth / camera inputs refreshed into the graph's static buffers), plus its own per-kernel times from
    an eager timing pass of 2 steps."""
    from mapanything.utils import synthetic

    V = args.cfg4_views
    imgs = synthetic.synthetic_images(V, H, W, seed=5)
    Ks = synthetic.synthetic_intrinsics(V, H, W, seed=5)
    Ds = synthetic.synthetic_sparse_depth(V, H, W, seed=5)
    views = [{"img": torch.from_numpy(i).to(dev), "data_norm_type": ["dinov2"], "intrinsics": torch.from_numpy(K).to(dev),
              "depth_z": torch.from_numpy(D).to(dev), "is_metric_scale": torch.ones(1, dtype=torch.bool)}
             for i, K, D in zip(imgs, Ks, Ds)]
    del imgs, Ks, Ds

    def step():
        return model.infer(views, **amp)

    step()  # warm-up: geometric weights packed, graph captured
    graphs = sum(1 for k in model._graphs if k[5] is not None)
    step()
    dt = timed_fn(step, args.cfg4_steps)
    per_kernel = None
    if not args.no_kernel_timing:
        eng = model.engine()
        eng.enable_kernel_timing()
        timed_fn(step, 2)
        kt = eng.collect_kernel_timing()
        per_kernel = {k: {"ms_per_step": v["ms"] / 2,
                          "tflops": (v["flops"] / (v["ms"] * 1e-3) / 1e12) if v["flops"] else None}
                      for k, v in kt.items()}
    out = {"views": V, "value": V * args.cfg4_steps / dt, "unit": "views/s", "ms_per_step": dt / args.cfg4_steps * 1e3,
           "steps": args.cfg4_steps, "warmup": 2, "hip_graphs": graphs > 0,
           "workload": f"{V}-view {H}x{W} images + intrinsics + 90%-sparse depth_z + is_metric_scale, "
                       "MapAnything.infer on 1 GPU (configs[3])",
           "per_kernel": per_kernel}
    del views
    torch.cuda.empty_cache()
    return out


def shard_graph_self_check(model, step, dist, dev):
    """N > 1: the first graph replay of the sharded forward against one eager sharded forward of the same views,
    bitwise, on every rank (the warm-up captured the graph; a replay and an eager run issue the same kernels and
    collectives in the same order).  Returns what every rank saw (MIN over ranks) and the collective path taken."""
    from mapanything.parallel import RcclComm

    graphs = sum(1 for k in model._graphs if k[-1] is not None)
    was = model.hip_graphs
    model.hip_graphs = False
    eager = step()
    model.hip_graphs = was
    replay = step()
    torch.cuda.synchronize()
    keys = [k for k in ("pts3d", "conf", "depth_along_ray", "ray_directions", "cam_quats", "cam_trans",
                        "metric_scaling_factor", "mask") if replay and replay[0] is not None and k in replay[0]]
    same = all(torch.equal(a[k], b[k]) for a, b in zip(replay, eager) if a is not None for k in keys)
    flags = torch.tensor([1 if same else 0, graphs], dtype=torch.int32, device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    return {"graph_eq_eager_all_ranks": bool(flags[0].item()), "sharded_graphs_min_over_ranks": int(flags[1].item()),
            "communicator": "direct RCCL (captured)" if isinstance(model._comm, RcclComm) else "process group (eager)",
            "keys": keys}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run (one process per GPU, env://
    rendezvous on 127.0.0.1) as CHILD processes — this process never initialises the GPU — relay their output, and
    return a non-zero status if any rank fails (torch.distributed.run stops the others then)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", env.get("OMP_NUM_THREADS", "16"))
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        print(f"bench.py: {n}-rank job failed with status {rc}", file=sys.stderr, flush=True)
    return rc


def dry_run(args, world, rank):
    """The multi-rank control path of the bench (launcher, rendezvous, timed barrier + max-over-ranks, rank-0 JSON
    line) over gloo with a placeholder CPU step, for the CPU test-suite (tests/test_bench_launcher.py)."""
    import torch.distributed as dist

    from mapanything.parallel import CommError, DistComm, init_distributed

    observed = 1
    if world > 1:
        _, observed = init_distributed("gloo")
    if os.environ.get("MAPA_BENCH_STDOUT_NOISE"):  # test hook: a native library writing to fd 1 (RCCL's banner)
        os.write(1, b"RCCL version : (native stdout noise)\n")
        print("python-level stdout noise", flush=True)
    if rank == args.fail_rank:
        raise SystemExit(f"rank {rank}: injected failure (--fail-rank)")
    comm = DistComm() if world > 1 else None
    x = torch.ones(64, 64)

    phases = {"kv_allgather": [], "kv_local_attention": [], "kv_remote_attention": [], "kv_gather_wait": []}

    def step():
        # placeholder of one overlapped global layer: "local" product, the slot all-gather, "remote" product (CPU:
        # sequential, so the gather is fully exposed)
        t0 = time.perf_counter()
        y = x @ x
        t1 = time.perf_counter()
        if comm is not None:
            t = torch.zeros(world * 4, 4)
            t[rank * 4:(rank + 1) * 4] = y[:4, :4]
            comm.allgather_slots(t, 4)
        t2 = time.perf_counter()
        y = y @ x
        t3 = time.perf_counter()
        for k, v in (("kv_local_attention", t1 - t0), ("kv_allgather", t2 - t1), ("kv_gather_wait", t2 - t1),
                     ("kv_remote_attention", t3 - t2)):
            phases[k].append(v * 1e3)
        return y

    try:
        for _ in range(args.warmup):
            step()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
    except CommError as e:
        raise SystemExit(f"rank {rank}: {e}")
    if rank == 0:
        kvo = kv_overlap({k: {"ms": sum(v), "count": len(v)} for k, v in phases.items()}) if world > 1 else None
        _emit({"metric": "dry-run (launcher rehearsal, no GPU)", "value": args.steps / dt, "unit": "steps/s",
               "n_gpus": world, "world_size_observed": observed, "steps": args.steps, "warmup": args.warmup,
               "dry_run": True, "kv_overlap": kvo})
    if world > 1:
        dist.destroy_process_group()


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(model, imgs, H, W, budget_s=80.0, max_reps=3):
    """The fp32 CPU oracle (oracle/mapa_oracle.py, test infrastructure) timed on this host's cores on the same
    8-view workload: three full infers (one takes ~22 s on 16 EPYC 9575F threads), the median reported; fewer only if
    the next one would push the total past ~budget_s.  Threads:
    OMP_NUM_THREADS (the GPU box's CPU share: 16 cores of the host per GPU; os.cpu_count() there reports the whole
    machine), else every core of this host."""
    from oracle.mapa_oracle import MapAnythingOracle

    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    torch.set_num_threads(cores)
    oracle = MapAnythingOracle(model._sd)
    views = [{"img": torch.from_numpy(i), "data_norm_type": ["dinov2"]} for i in imgs]
    times = []
    t_start = time.perf_counter()
    while not times or (len(times) < max_reps and (time.perf_counter() - t_start) + times[-1] < budget_s):
        t0 = time.perf_counter()
        with torch.no_grad():
            oracle.infer(views)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    return {"value": len(views) / dt, "unit": "views/s", "cores": cores, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus_visible": os.cpu_count(), "reps": len(times),
            "sample": f"{len(views)} views {H}x{W}, median of {len(times)} infer (apply_mask=False), fp32 torch-CPU "
                      f"oracle on {cores} threads",
            "seconds": dt}


if __name__ == "__main__":
    main()
