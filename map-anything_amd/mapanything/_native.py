"""ctypes binding of libmapa.so (the gfx950 HIP kernels behind include/mapa.h).

There is no fallback: if the library or a gfx950 device is missing, `lib()` raises.  Tensors are passed as
raw device pointers on torch's current HIP stream (torch is the allocator and stream owner, nothing more).
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libmapa.so")
_lib = None

F32, BF16, BF16X3, F16, F16X2 = 0, 1, 2, 3, 4
A_DENSE, A_CONV3X3 = 0, 1
OUT_ROWMAJOR, OUT_PIXSHUF = 0, 1
ACT_NONE, ACT_GELU, ACT_RELU, ACT_GELU_POST = 0, 1, 2, 3

# Every extern "C" symbol declared in include/mapa.h (checked by tests/test_capi.py).
EXPORTED = (
    "mapa_last_error", "mapa_version", "mapa_device_check", "mapa_gemm", "mapa_gemm_workspace_bytes",
    "mapa_gemm_set_variant", "mapa_attention", "mapa_attention_workspace_bytes", "mapa_layernorm",
    "mapa_patchify", "mapa_assemble_tokens", "mapa_add_rowvec", "mapa_bilinear_ac", "mapa_mean_tokens",
    "mapa_linear_small", "mapa_pose_scale_finalize", "mapa_dense_head_out", "mapa_convert_rows",
    "mapa_fill_splitmix", "mapa_postprocess_mask", "mapa_recover_intrinsics", "mapa_denorm_image",
    "mapa_pixel_unshuffle", "mapa_depth_norm_factors", "mapa_pose_inputs", "mapa_add_view_vectors", "mapa_add_f32",
    "mapa_split_bf16x3", "mapa_split_rows", "mapa_view_rays", "mapa_apply_mask", "mapa_confidence_mask", "mapa_attn_merge", "mapa_dense_adaptor",
    "mapa_normalize_image", "mapa_normal_cos_threshold", "mapa_rope2d", "mapa_gemm_tune",
    "mapa_regressor_head_out", "mapa_stream_check", "mapa_fault_slot_create", "mapa_fault_slot_destroy",
    "mapa_fault_publish", "mapa_fault_status", "mapa_fault_reset",
    "mapa_comm_unique_id_bytes", "mapa_comm_get_unique_id", "mapa_comm_init", "mapa_comm_allgather_kv",
    "mapa_comm_broadcast", "mapa_comm_check", "mapa_comm_destroy",
    "mapa_resize_plan_bytes", "mapa_resize_plan_build", "mapa_resize_workspace_bytes", "mapa_resize_normalize",
)
FAULT_LN_BARRIER = 1  # include/mapa.h MAPA_FAULT_LN_BARRIER
FAULT_F16_RANGE = 2  # include/mapa.h MAPA_FAULT_F16_RANGE
RESAMPLE_LANCZOS, RESAMPLE_BILINEAR, RESAMPLE_BICUBIC = 1, 2, 3  # include/mapa.h MAPA_RESAMPLE_* (PIL numbering)


class ResizePlan(ctypes.Structure):
    """include/mapa.h mapa_resize_plan (the header of a resize plan blob)."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "in_w", "in_h", "rs_w", "rs_h", "crop_left", "crop_top", "out_w", "out_h", "filter", "need_h", "need_v",
        "kh", "kv", "row0", "nrows", "off_hb", "off_hk", "off_vb", "off_vk", "int32s")]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int), ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
        ("A", ctypes.c_void_p), ("lda", ctypes.c_int64), ("W", ctypes.c_void_p), ("ldw", ctypes.c_int64),
        ("a_mode", ctypes.c_int), ("conv_C", ctypes.c_int), ("conv_IH", ctypes.c_int), ("conv_IW", ctypes.c_int),
        ("conv_OH", ctypes.c_int), ("conv_OW", ctypes.c_int), ("conv_stride", ctypes.c_int),
        ("bias", ctypes.c_void_p), ("bias_mod", ctypes.c_int), ("gamma", ctypes.c_void_p), ("act", ctypes.c_int),
        ("resid1", ctypes.c_void_p), ("resid2", ctypes.c_void_p), ("out_f32", ctypes.c_void_p),
        ("out_lp", ctypes.c_void_p), ("out_lp_relu", ctypes.c_void_p), ("ldo", ctypes.c_int64),
        ("out_mode", ctypes.c_int), ("ps_s", ctypes.c_int), ("ps_h", ctypes.c_int), ("ps_w", ctypes.c_int),
        ("ps_cout", ctypes.c_int), ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_int64),
        ("out_s3", ctypes.c_void_p), ("out_s3_relu", ctypes.c_void_p), ("a_split", ctypes.c_int),
        ("conv_kblock", ctypes.c_int), ("ln_w", ctypes.c_void_p), ("ln_b", ctypes.c_void_p), ("ln_eps", ctypes.c_float),
        ("ln_out", ctypes.c_void_p), ("ln_ldo", ctypes.c_int64),
    ]


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int), ("batch", ctypes.c_int), ("heads", ctypes.c_int), ("seq_q", ctypes.c_int),
        ("seq_kv", ctypes.c_int), ("q", ctypes.c_void_p), ("k", ctypes.c_void_p), ("v", ctypes.c_void_p),
        ("o", ctypes.c_void_p), ("q_bstride", ctypes.c_int64), ("q_rstride", ctypes.c_int64),
        ("k_bstride", ctypes.c_int64), ("k_rstride", ctypes.c_int64), ("v_bstride", ctypes.c_int64),
        ("v_rstride", ctypes.c_int64), ("o_bstride", ctypes.c_int64), ("o_rstride", ctypes.c_int64),
        ("lse", ctypes.c_void_p), ("kv_nseg", ctypes.c_int), ("kv_seg_start", ctypes.c_int * 16),
        ("kv_seg_len", ctypes.c_int * 16), ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_int64),
        ("scale", ctypes.c_float),
    ]


class NativeError(RuntimeError):
    pass


class DeviceFault(NativeError):
    """A kernel set the library's device fault word (include/mapa.h MAPA_FAULT_*); `bits` holds the word."""

    def __init__(self, bits: int):
        super().__init__(_fault_message(bits))
        self.bits = int(bits)

    @property
    def range_only(self) -> bool:
        """Only MAPA_FAULT_F16_RANGE: a binary16 operand left binary16's range (the run is valid in another recipe)."""
        return self.bits == FAULT_F16_RANGE


def lib_path() -> str:
    return _LIB_PATH


def load_library(path: Optional[str] = None):
    """dlopen libmapa.so and declare argtypes (no device needed)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or _LIB_PATH
    if not os.path.exists(p):
        raise NativeError(f"libmapa.so not found at {p}: build it with `make -C map-anything_amd/csrc` "
                          f"(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(p)
    vp, i, i64, f, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64
    L.mapa_last_error.restype = ctypes.c_char_p
    L.mapa_version.restype = i
    L.mapa_device_check.argtypes = [i]
    L.mapa_gemm.argtypes = [ctypes.POINTER(GemmDesc), vp]
    L.mapa_gemm_workspace_bytes.argtypes = [ctypes.POINTER(GemmDesc)]
    L.mapa_gemm_workspace_bytes.restype = i64
    L.mapa_gemm_set_variant.argtypes = [i]
    L.mapa_gemm_tune.argtypes = [i, i]
    L.mapa_attention.argtypes = [ctypes.POINTER(AttnDesc), vp]
    L.mapa_attention_workspace_bytes.argtypes = [ctypes.POINTER(AttnDesc)]
    L.mapa_attention_workspace_bytes.restype = i64
    L.mapa_layernorm.argtypes = [vp, i64, i, i, vp, vp, f, vp, vp, i, i64, i, i64, i, vp]
    L.mapa_patchify.argtypes = [vp, i, i, i, vp, i, i, vp]
    L.mapa_assemble_tokens.argtypes = [vp, vp, vp, i, i, i, vp, vp]
    L.mapa_add_rowvec.argtypes = [vp, i64, i, i, i, vp, vp]
    L.mapa_bilinear_ac.argtypes = [vp, i, i, i, i, i, i, i, i, i, vp, i, vp]
    L.mapa_mean_tokens.argtypes = [vp, i, i, i, vp, vp, vp]
    L.mapa_linear_small.argtypes = [vp, i, i, vp, vp, i, i, vp, vp]
    L.mapa_pose_scale_finalize.argtypes = [vp, vp, i, i, vp, vp, vp, vp]
    L.mapa_dense_head_out.argtypes = [vp, i, i, i, vp, vp, vp, vp, i, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mapa_regressor_head_out.argtypes = [vp] * 5 + [i] + [vp] * 7 + [vp]
    L.mapa_convert_rows.argtypes = [vp, i64, i, i, vp, i, i64, vp]
    L.mapa_fill_splitmix.argtypes = [vp, i64, u64, f, f, vp]
    L.mapa_postprocess_mask.argtypes = [vp, vp, vp, vp, i, i, i, f, f, i, vp, vp]
    L.mapa_normal_cos_threshold.argtypes = [ctypes.c_double]
    L.mapa_normal_cos_threshold.restype = f
    L.mapa_recover_intrinsics.argtypes = [vp, i, i, i, vp, vp]
    L.mapa_denorm_image.argtypes = [vp, i, i, i, vp, vp, vp, vp]
    L.mapa_pixel_unshuffle.argtypes = [vp, i, i, i, i, i, vp, i, vp, i, i64, vp]
    L.mapa_depth_norm_factors.argtypes = [vp, i, i, vp, vp, vp, vp]
    L.mapa_pose_inputs.argtypes = [vp, vp, vp, i, vp, vp, vp, vp]
    L.mapa_add_view_vectors.argtypes = [vp, i, i, i, vp, vp, i, vp]
    L.mapa_add_f32.argtypes = [vp, vp, i64, vp]
    L.mapa_split_bf16x3.argtypes = [vp, i64, i64, i, i, vp, vp]
    L.mapa_split_rows.argtypes = [vp, i64, i64, i, i, vp, i, vp]
    L.mapa_view_rays.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp]
    L.mapa_apply_mask.argtypes = [vp, vp, vp, vp, i64, vp]
    L.mapa_confidence_mask.argtypes = [vp, vp, vp, i, i64, f, vp]
    L.mapa_attn_merge.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i, i64, vp]
    L.mapa_dense_adaptor.argtypes = [vp, i, i64, vp, vp, vp, vp, vp]
    L.mapa_normalize_image.argtypes = [vp, i, i, i, vp, vp, vp, vp]
    L.mapa_rope2d.argtypes = [vp, i, i, i, i, i, i64, i64, i64, vp, f, f, vp]
    L.mapa_stream_check.argtypes = [vp, ctypes.c_char_p]
    pu32 = ctypes.POINTER(ctypes.c_uint32)
    L.mapa_fault_slot_create.argtypes = [ctypes.POINTER(pu32), ctypes.POINTER(pu32)]
    L.mapa_fault_slot_destroy.argtypes = [pu32]
    L.mapa_fault_publish.argtypes = [pu32, vp]
    L.mapa_fault_status.argtypes = [i]
    L.mapa_fault_reset.argtypes = [vp]
    L.mapa_comm_get_unique_id.argtypes = [vp]
    L.mapa_comm_init.argtypes = [ctypes.POINTER(vp), i, i, vp, i, ctypes.c_double]
    L.mapa_comm_allgather_kv.argtypes = [vp, vp, i64, vp]
    L.mapa_comm_broadcast.argtypes = [vp, vp, i64, i, vp]
    L.mapa_comm_check.argtypes = [vp]
    L.mapa_comm_destroy.argtypes = [vp, i]
    L.mapa_resize_plan_bytes.argtypes = [i, i, i, i, i]
    L.mapa_resize_plan_bytes.restype = i64
    L.mapa_resize_plan_build.argtypes = [i, i, i, i, i, i, i, i, i, vp, i64]
    L.mapa_resize_workspace_bytes.argtypes = [vp]
    L.mapa_resize_workspace_bytes.restype = i64
    L.mapa_resize_normalize.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, i64, vp]
    _lib = L
    return L


def lib():
    """The loaded library, after checking that a gfx950 device is present (raises otherwise)."""
    L = load_library()
    if not getattr(L, "_device_ok", False):
        if not torch.cuda.is_available():
            raise NativeError("no HIP device visible: the MapAnything MI355X engine has no CPU path")
        dev = torch.cuda.current_device()
        if L.mapa_device_check(dev) != 1:
            raise NativeError(L.mapa_last_error().decode())
        L._device_ok = True
    return L


def _serialize_from_env() -> bool:
    """Debug / serialize mode: MAPA_SERIALIZE=1, or the HIP runtime's own switches (AMD_SERIALIZE_KERNEL >= 1,
    HIP_LAUNCH_BLOCKING=1) — every launch is followed by a stream synchronise + device-error check."""
    if os.environ.get("MAPA_SERIALIZE", "0") not in ("", "0"):
        return True
    if os.environ.get("AMD_SERIALIZE_KERNEL", "0") not in ("", "0"):
        return True
    return os.environ.get("HIP_LAUNCH_BLOCKING", "0") not in ("", "0")


SERIALIZE = _serialize_from_env()


def set_serialize(on: bool):
    global SERIALIZE
    SERIALIZE = bool(on)


def check(rc: int, what: str):
    if rc != 0:
        raise NativeError(f"{what}: {_lib.mapa_last_error().decode()}")
    if SERIALIZE and not torch.cuda.is_current_stream_capturing():
        if _lib.mapa_stream_check(stream(), what.encode()) != 0:
            raise NativeError(_lib.mapa_last_error().decode())


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dt_code(dtype: torch.dtype) -> int:
    if dtype == torch.bfloat16:
        return BF16
    if dtype == torch.float32:
        return F32
    if dtype == torch.float16:
        return F16
    raise NativeError(f"unsupported dtype {dtype}")


# ------------------------------------------------------------------------------------------- fault channel
def _fault_message(bits: int) -> str:
    if bits & FAULT_LN_BARRIER:
        return ("a LayerNorm-fused GEMM band barrier timed out on the device (include/mapa.h MAPA_FAULT_LN_BARRIER): "
                "the normalised rows of that launch are invalid, so this call's outputs were discarded")
    if bits & FAULT_F16_RANGE:
        return ("a binary16 operand (the TF32-equivalent heads, or the fp16 recipe) left binary16's range (include/"
                "mapa.h MAPA_FAULT_F16_RANGE): this call's outputs were discarded; head_precision='fp32' runs the heads "
                "fp32-exact")
    return f"device fault word 0x{bits:x}"


def fault_status(reset: bool = True) -> int:
    """Synchronous read of the library's sticky device fault word (mapa_fault_status), reset when `reset`."""
    v = int(lib().mapa_fault_status(1 if reset else 0))
    if v < 0:
        raise NativeError(lib().mapa_last_error().decode())
    return v


def check_faults():
    """Raise NativeError if a kernel set the device fault word since the last check (synchronises the device)."""
    v = fault_status(reset=True)
    if v:
        raise DeviceFault(v)


class FaultTimeout(NativeError):
    """The device did not reach a fault publish within the caller's bound (a hung kernel or collective)."""


class FaultSlot:
    """A host-visible slot the device writes its fault word into, stream-ordered (mapa_fault_publish): the host
    arms it (slot = 0), enqueues work + publish(), and wait() polls the slot — without synchronising the stream, so
    the kernels queued after the publish keep the GPU busy while the host checks.  One slot per captured graph (its
    publish node is baked into the graph with this slot's address) and one per eager caller."""

    def __init__(self):
        L = lib()
        if _DEFERRED_SLOTS and not torch.cuda.is_current_stream_capturing():
            while _DEFERRED_SLOTS:
                L.mapa_fault_slot_destroy(_DEFERRED_SLOTS.pop())
        h, d = ctypes.POINTER(ctypes.c_uint32)(), ctypes.POINTER(ctypes.c_uint32)()
        if L.mapa_fault_slot_create(ctypes.byref(h), ctypes.byref(d)) != 0:
            raise NativeError(L.mapa_last_error().decode())
        self._h, self._d = h, d
        self._word = ctypes.c_uint32.from_address(ctypes.addressof(h.contents))
        self.armed = False

    def arm(self):
        self._word.value = 0
        self.armed = True

    def publish(self):
        """Enqueue the publish on the current stream (also inside a graph capture)."""
        check(lib().mapa_fault_publish(self._d, stream()), "mapa_fault_publish")

    @staticmethod
    def reset():
        """Enqueue the fault word's reset on the current stream (the start of a call; also inside a capture)."""
        check(lib().mapa_fault_reset(stream()), "mapa_fault_reset")

    def wait(self, timeout_s: float = 600.0, poll=None):
        """Poll until the armed publish has run; raise NativeError if it carried a fault (the device word is reset).
        The poll sleeps ~50 us between reads, calls `poll()` (e.g. a communicator's asynchronous-error check) every
        ~10 ms, and raises FaultTimeout past timeout_s, or NativeError if the stream drains without the publish."""
        import time

        if not self.armed:
            return
        self.armed = False
        t0, s = time.monotonic(), torch.cuda.current_stream()
        t_poll = t0
        while True:
            v = self._word.value
            if v:
                break
            if s.query():  # the stream is idle: the publish ran (re-read once) or never was enqueued
                v = self._word.value
                if not v:
                    raise NativeError("fault publish slot armed but never written (the publish was not enqueued)")
                break
            now = time.monotonic()
            if now - t0 > timeout_s:
                raise FaultTimeout(f"fault publish not reached within {timeout_s:.0f} s")
            if poll is not None and now - t_poll > 0.01:
                poll()
                t_poll = now
            time.sleep(5e-5)
        bits = v >> 1
        if bits:
            fault_status(reset=True)
            raise DeviceFault(bits)

    def __del__(self):
        # a slot can be collected at any allocation — also while a HIP graph is being captured on this thread (a
        # cyclic reference freed by the garbage collector), where a host free would invalidate the capture: then the
        # free waits for the next slot made outside a capture
        try:
            if _lib is not None and getattr(self, "_h", None):
                if torch.cuda.is_current_stream_capturing():
                    _DEFERRED_SLOTS.append(self._h)
                else:
                    _lib.mapa_fault_slot_destroy(self._h)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


_DEFERRED_SLOTS = []  # FaultSlot host words collected during a capture, freed by the next FaultSlot()


class CComm:
    """The library's own RCCL communicator (include/mapa.h mapa_comm_*): what a non-Python host of libmapa.so uses for
    the sharded forward's K/V all-gather and scale-token broadcast.  `uid` = rank 0's mapa_comm_get_unique_id bytes
    (CComm.unique_id()), handed to every rank by the caller."""

    @staticmethod
    def unique_id() -> bytes:
        L = lib()
        buf = ctypes.create_string_buffer(int(L.mapa_comm_unique_id_bytes()))
        if L.mapa_comm_get_unique_id(buf) != 0:
            raise NativeError(L.mapa_last_error().decode())
        return buf.raw

    def __init__(self, world: int, rank: int, uid: bytes, device: int, timeout_s: float = 600.0):
        L = lib()
        self._c = ctypes.c_void_p()
        if L.mapa_comm_init(ctypes.byref(self._c), world, rank, uid, device, float(timeout_s)) != 0:
            raise NativeError(L.mapa_last_error().decode())
        self.world, self.rank = world, rank

    def allgather_slots(self, full: torch.Tensor, rows_per_slot: int):
        slot = rows_per_slot * full[0].numel() * full.element_size()
        check(lib().mapa_comm_allgather_kv(self._c, ctypes.c_void_p(full.data_ptr()), slot, stream()),
              "mapa_comm_allgather_kv")

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        check(lib().mapa_comm_broadcast(self._c, ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(), src,
                                        stream()), "mapa_comm_broadcast")

    def check_async(self):
        check(lib().mapa_comm_check(self._c), "mapa_comm_check")

    def close(self, abort: bool = False):
        if self._c:
            rc = lib().mapa_comm_destroy(self._c, 1 if abort else 0)
            self._c = ctypes.c_void_p()
            if rc != 0:
                raise NativeError(lib().mapa_last_error().decode())


# --------------------------------------------------------------------------------------- kernel timing
# Optional per-launch HIP-event timing (bench.py's roofline numbers): events are recorded on the stream the
# kernel is launched on, around the launch, and only read after the timed region.
_timing = None


def timing_start():
    global _timing
    _timing = {}


def timing_stop():
    """-> {kind: {"ms": total, "count": launches, "flops": total algorithmic flops}} (synchronises)."""
    global _timing
    t, _timing = _timing, None
    if not t:
        return {}
    torch.cuda.synchronize()
    out = {}
    for kind, recs in t.items():
        ms = sum(a.elapsed_time(b) for a, b, _ in recs)
        out[kind] = {"ms": ms, "count": len(recs), "flops": float(sum(f for _, _, f in recs))}
    return out


def mark(stream=None):
    """An event recorded now on `stream` (default: the current stream) while kernel timing is on, else None."""
    if _timing is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


def span(kind, start, end):
    """Record the interval between two mark() events under `kind` (no flops: a phase, not a kernel)."""
    if _timing is not None and start is not None and end is not None:
        _timing.setdefault(kind, []).append((start, end, 0.0))


def _tic():
    if _timing is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _toc(tok, kind, flops=0.0):
    if tok is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    _timing.setdefault(kind, []).append((tok, e, flops))


# Optional launch log for profiling (MAPA_LAUNCH_LOG=<path>): the kind of every GEMM / attention call in launch
# order, written at exit, so tools/profile_summary.py can name each rocprofv3 dispatch the way bench.py does (the
# split-precision head GEMMs share kernel symbols with the plain ones).
_LAUNCH_LOG = [] if os.environ.get("MAPA_LAUNCH_LOG") else None
_LAUNCH_SHAPES = os.environ.get("MAPA_LAUNCH_SHAPES", "0") == "1"  # log "kind:shape" (profile_summary.py shapes)
if _LAUNCH_LOG is not None:
    import atexit
    import json as _json

    atexit.register(lambda: open(os.environ["MAPA_LAUNCH_LOG"], "w").write(_json.dumps(_LAUNCH_LOG)))


# ------------------------------------------------------------------------------------------------ wrappers
_WS_NEED = {}
_WS = {}
_AWS = {}
_WS_RETIRED = []  # grown-out GEMM workspaces, kept alive for graphs captured against them


def gemm_workspace(nbytes: int, ln: bool = False) -> torch.Tensor:
    """Zero-filled GEMM scratch (stream-K / split-K tickets and slabs; with ln=True the LayerNorm-fused linears' band
    generation words and statistics granules, in a buffer of their own) for the current device and stream —
    include/mapa.h's workspace contract: zeroed once, then owned by mapa_gemm.  One buffer per stream (and kind)
    because concurrent calls must not share it.  Grown (re-allocated zeroed, stream-ordered) when a larger problem
    needs more."""
    key = (torch.cuda.current_device(), torch.cuda.current_stream().cuda_stream, bool(ln))
    ws = _WS.get(key)
    if ws is None or ws.numel() < nbytes:
        if ws is not None:
            # a captured HIP graph may hold the old buffer's address: never free a workspace once used
            _WS_RETIRED.append(ws)
        ws = _WS[key] = torch.zeros(max(nbytes, 0 if ws is None else ws.numel()), dtype=torch.uint8,
                                    device="cuda")
    return ws


def attention_workspace(d) -> torch.Tensor:
    """Scratch for the stream-K attention partials (fp32 rows + LSE of the tasks that a workgroup range cuts);
    one buffer per device and stream, sized once by mapa_attention_workspace_bytes (it depends on the device's
    resident workgroup count only).  Contents are never read across calls."""
    key = (torch.cuda.current_device(), torch.cuda.current_stream().cuda_stream)
    ws = _AWS.get(key)
    if ws is None:
        need = int(lib().mapa_attention_workspace_bytes(ctypes.byref(d)))
        ws = _AWS[key] = torch.empty(max(need, 16), dtype=torch.uint8, device="cuda")
    return ws


TUNE_CONV_HALO, TUNE_TAIL_STREAMK, TUNE_HALO_SPLIT, TUNE_TILE_GROUP, TUNE_LN_FUSE = 0, 1, 2, 3, 4
TUNE_LN_SPIN, TUNE_LN_TEST_SKIP, TUNE_DIAG_GRID, TUNE_PERS, TUNE_PERS_LN, TUNE_PERS_STAGGER = 5, 6, 7, 8, 9, 10


def gemm_tune(key: int, value: int):
    """A-B hooks of the automatic kernel choice (include/mapa.h mapa_gemm_tune): TUNE_CONV_HALO (stride-1 head convs
    on the LDS halo-window kernel, default on), TUNE_TAIL_STREAMK (tail-only stream-K for nearly empty last waves),
    TUNE_HALO_SPLIT (K part count of the flat-raster halo conv, 0 = automatic), TUNE_TILE_GROUP (tile rows per group
    in the 256-row GEMM kernels' tile order, 0 = the default 4), TUNE_LN_FUSE (LayerNorm fused into the residual
    linears: 2 = default, whatever the tile choice; 1 = where it is the 192-row kernel; 0 = off), TUNE_LN_SPIN (polls
    of the fused LayerNorm's band barrier before it gives up, 0 = default), TUNE_LN_TEST_SKIP (test hook: the next n
    fused launches drop one tile's statistics, so a band times out and the fault word is raised)."""
    check(lib().mapa_gemm_tune(key, value), "mapa_gemm_tune")
    _WS_NEED.clear()


def gemm_set_variant(variant: int = 0):
    """Force one GEMM kernel variant (0 = automatic); see include/mapa.h."""
    check(lib().mapa_gemm_set_variant(variant), "mapa_gemm_set_variant")
    _WS_NEED.clear()


def _wscale_epilogue(W, N, bias, gamma, act, head_out):
    """Epilogue operands for a weight stored as 2^s x w (W._mapa_wscale = s, engine._f16_pack: a binary16 head weight
    whose largest element sits outside [2^-4, 2^12] is rescaled by a power of two so that its small elements stay
    normal binary16 numbers, as TF32 — fp32's exponent — keeps them).  The accumulator is then exactly 2^s x the
    unscaled one, so the epilogue takes bias x 2^s and gamma x 2^-s (or a gamma of 2^-s), and the fused regressor
    tail's 1x1 weights x 2^-s: all exact powers of two through a positively homogeneous activation (none or ReLU),
    so every output bit equals the unscaled arithmetic's.  The scaled copies are made once per (weight, bias, gamma)
    and kept on the weight tensor (before any graph capture: the engine's eager warm-up)."""
    s = W._mapa_wscale
    if act not in (ACT_NONE, ACT_RELU):
        raise NativeError("a power-of-two scaled weight needs a linear or ReLU epilogue")
    cache = W.__dict__.setdefault("_mapa_wsc_cache", [])
    w6 = head_out[0] if head_out is not None else None
    for b0, g0, w60, ent in cache:
        if b0 is bias and g0 is gamma and w60 is w6:
            b2, g2, w62 = ent
            break
    else:
        up, dn = 2.0 ** s, 2.0 ** -s
        b2 = None if bias is None else (bias.float() * up).contiguous()
        if head_out is not None:  # the fused regressor tail applies no gamma: its 1x1 weights take the 2^-s
            g2, w62 = None, (w6.float() * dn).contiguous()
        else:
            g2 = (gamma.float() * dn).contiguous() if gamma is not None else \
                torch.full((N,), dn, dtype=torch.float32, device=W.device)
            w62 = None
        cache.append((bias, gamma, w6, (b2, g2, w62)))
    if head_out is not None:
        return b2, gamma, (w62,) + tuple(head_out[1:])
    return b2, g2, head_out


def gemm(A, W, M, N, K, *, lda=None, bias=None, bias_mod=0, gamma=None, act=ACT_NONE, resid1=None, resid2=None,
         out_f32=None, out_lp=None, out_lp_relu=None, out_s3=None, out_s3_relu=None, ldo=None, conv=None,
         pixshuf=None, head_out=None, ln=None):
    """C = A W^T with fused epilogue (see include/mapa.h). conv=(C, IH, IW, OH, OW, stride); pixshuf=(s, h, w, cout).
    out_s3 / out_s3_relu: split-precision operand outputs (bf16 [rows][2*ldo], [hi | lo]).  A weight packed for split
    operands (W._mapa_split, engine._split_pack) marks A as a compact split operand (mapa_gemm_desc.a_split): K is
    then the logical 3C, the stored A row 2C wide.  A conv weight tagged W._mapa_kblock = B holds its columns in the
    channel-block-major K order (mapa_gemm_desc.conv_kblock).
    head_out=(w6, b6, pose_out, scale, views_per_scale, pts3d, pts3d_cam, rays, depth, conf, logits, mask): the conv
    is the regressor's conv2 and its hidden map goes straight into the dense head (mapa_regressor_head_out; no other
    outputs; image i uses scale[i // views_per_scale]).
    ln=(w, b, eps, out): the LayerNorm of out_f32's rows into out (the GEMM's 16-bit dtype; mapa_gemm_desc.ln_*), fused
    into the residual linear where the library can (include/mapa.h)."""
    if getattr(W, "_mapa_wscale", 0):
        bias, gamma, head_out = _wscale_epilogue(W, N, bias, gamma, act, head_out)
    d = GemmDesc()
    d.dtype = dt_code(A.dtype)
    assert W.dtype == A.dtype
    d.M, d.N, d.K = M, N, K
    d.A = A.data_ptr()
    split_a = W.dtype == torch.bfloat16 and getattr(W, "_mapa_split", False)
    d.a_split = 1 if split_a else 0
    d.lda = lda if lda is not None else (2 * K // 3 if split_a else K)
    d.W = W.data_ptr()
    d.ldw = W.stride(0)
    if conv is not None:
        d.a_mode = A_CONV3X3
        d.conv_C, d.conv_IH, d.conv_IW, d.conv_OH, d.conv_OW, d.conv_stride = conv
        d.conv_kblock = getattr(W, "_mapa_kblock", 0)  # weights packed channel-block-major (engine.hconv3)
        d.lda = K
    d.bias = None if bias is None else bias.data_ptr()
    d.bias_mod = bias_mod
    d.gamma = None if gamma is None else gamma.data_ptr()
    d.act = act
    d.resid1 = None if resid1 is None else resid1.data_ptr()
    d.resid2 = None if resid2 is None else resid2.data_ptr()
    d.out_f32 = None if out_f32 is None else out_f32.data_ptr()
    d.out_lp = None if out_lp is None else out_lp.data_ptr()
    d.out_lp_relu = None if out_lp_relu is None else out_lp_relu.data_ptr()
    for t in (out_s3, out_s3_relu):  # MAPA_BF16X3 rows from a bf16 GEMM, MAPA_F16X2 rows from an f16 one
        if t is not None and t.dtype != (torch.float16 if A.dtype == torch.float16 else torch.bfloat16):
            raise NativeError("split outputs are [rows][2*ld] of the GEMM's 16-bit dtype (bf16 or f16)")
    d.out_s3 = None if out_s3 is None else out_s3.data_ptr()
    d.out_s3_relu = None if out_s3_relu is None else out_s3_relu.data_ptr()
    d.ldo = ldo if ldo is not None else N
    if pixshuf is not None:
        d.out_mode = OUT_PIXSHUF
        d.ps_s, d.ps_h, d.ps_w, d.ps_cout = pixshuf
    if ln is not None:
        lw, lb, leps, lout = ln
        d.ln_w, d.ln_b, d.ln_eps, d.ln_out, d.ln_ldo = lw.data_ptr(), lb.data_ptr(), float(leps), lout.data_ptr(), \
            lout.stride(0)
    key = (d.dtype, M, N, K, d.a_mode, d.a_split, d.conv_kblock, ln is not None) + \
        (tuple(conv) if conv is not None else ())
    need = _WS_NEED.get(key)
    if need is None:
        need = _WS_NEED[key] = int(lib().mapa_gemm_workspace_bytes(ctypes.byref(d)))
    if need:
        ws = gemm_workspace(need, ln=ln is not None)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    tok = _tic()
    if head_out is not None:
        w6, b6, po, sc, vps, *outs = head_out
        check(lib().mapa_regressor_head_out(ctypes.byref(d), ptr(w6), ptr(b6), ptr(po), ptr(sc), int(vps),
                                            *(ptr(t) for t in outs), stream()),
              "mapa_regressor_head_out")
    else:
        check(lib().mapa_gemm(ctypes.byref(d), stream()), "mapa_gemm")
    # split-precision GEMMs (K = 3 x the logical K) are timed as their own class: executed MFMA flops; residual
    # linears with their output LayerNorm (ln=) too ("gemm_ln": the GEMM flops over the fused launch's time)
    kind = ("conv3x3" if conv is not None else "gemm") + ("_split" if getattr(W, "_mapa_split", False) else "") + \
        ("_ln" if ln is not None else "")
    if _LAUNCH_LOG is not None:
        _LAUNCH_LOG.append(f"{kind}:{M}x{N}x{K}" + (f":{conv[1]}x{conv[2]}s{conv[5]}" if conv is not None else "")
                           if _LAUNCH_SHAPES else kind)
    _toc(tok, kind, 2.0 * M * N * K)


def attention(q, k, v, o, *, batch, heads, seq_q, seq_kv, q_bstride, q_rstride, k_bstride, k_rstride,
              v_bstride, v_rstride, o_bstride, o_rstride, lse=None, kv_segments=None, kind="attention", scale=None):
    """q/k/v/o are tensors whose data_ptr is the (b=0, h=0, i=0, d=0) element.  `kind` labels the launch for the
    per-kernel timing (bench.py: "attention_global" = the cross-view AAT layers)."""
    d = AttnDesc()
    d.dtype = dt_code(q.dtype)
    d.batch, d.heads, d.seq_q, d.seq_kv = batch, heads, seq_q, seq_kv
    d.q, d.k, d.v, d.o = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr()
    d.q_bstride, d.q_rstride = q_bstride, q_rstride
    d.k_bstride, d.k_rstride = k_bstride, k_rstride
    d.v_bstride, d.v_rstride = v_bstride, v_rstride
    d.o_bstride, d.o_rstride = o_bstride, o_rstride
    d.lse = None if lse is None else lse.data_ptr()
    d.scale = 0.0 if scale is None else float(scale)  # 0 -> 1/sqrt(64)
    if d.dtype in (BF16, F16):
        ws = attention_workspace(d)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    if kv_segments:
        if len(kv_segments) > 16:
            raise NativeError("at most 16 K/V segments")
        d.kv_nseg = len(kv_segments)
        for i, (st, ln) in enumerate(kv_segments):
            d.kv_seg_start[i], d.kv_seg_len[i] = st, ln
    if _LAUNCH_LOG is not None:
        _LAUNCH_LOG.append(f"{kind}:{batch}x{heads}x{seq_q}x{seq_kv}" if _LAUNCH_SHAPES else kind)
    tok = _tic()
    check(lib().mapa_attention(ctypes.byref(d), stream()), "mapa_attention")
    _toc(tok, kind, 4.0 * batch * heads * seq_q * seq_kv * 64)


def layernorm(x, rows, dim, w, b, *, eps=1e-6, ldx=None, y_f32=None, y_lp=None, y_s3=None, ldy=None, group=0,
              group_stride=0, row_off=0):
    """y_s3: split-precision operand rows ([rows][2*ldy], [hi | lo]: bf16 = MAPA_BF16X3, f16 = MAPA_F16X2) instead of
    y_lp."""
    if y_s3 is not None:
        if y_lp is not None or y_s3.dtype not in (torch.bfloat16, torch.float16):
            raise NativeError("layernorm: y_s3 (bf16 or f16 split rows) replaces y_lp")
        y_lp, lp_dtype = y_s3, (F16X2 if y_s3.dtype == torch.float16 else BF16X3)
    else:
        lp_dtype = dt_code(y_lp.dtype) if y_lp is not None else F32
    tok = _tic()
    check(lib().mapa_layernorm(ptr(x), ldx if ldx is not None else dim, rows, dim, ptr(w), ptr(b), eps, ptr(y_f32),
                               ptr(y_lp), lp_dtype, ldy if ldy is not None else dim, group, group_stride, row_off,
                               stream()), "mapa_layernorm")
    _toc(tok, "layernorm")


def patchify(img, n, H, W, out, kpad):
    check(lib().mapa_patchify(ptr(img), n, H, W, ptr(out), dt_code(out.dtype), kpad, stream()), "mapa_patchify")


def assemble_tokens(patch, cls, pos, n, T, dim, x):
    check(lib().mapa_assemble_tokens(ptr(patch), ptr(cls), ptr(pos), n, T, dim, ptr(x), stream()),
          "mapa_assemble_tokens")


def add_rowvec(x, ldx, r0, r1, dim, vec):
    check(lib().mapa_add_rowvec(ptr(x), ldx, r0, r1, dim, ptr(vec), stream()), "mapa_add_rowvec")


def bilinear_ac(inp, n, IH, IW, C, OHf, OWf, OH, OW, out, split_out=False):
    """split_out: out is a split-precision operand ([pixels][2*C], [hi | lo]: bf16 = MAPA_BF16X3, f16 =
    MAPA_F16X2)."""
    if split_out and out.dtype not in (torch.bfloat16, torch.float16):
        raise NativeError("bilinear_ac: split output is bf16 or f16")
    sdt = (F16X2 if out.dtype == torch.float16 else BF16X3) if split_out else dt_code(out.dtype)
    check(lib().mapa_bilinear_ac(ptr(inp), dt_code(inp.dtype), n, IH, IW, C, OHf, OWf, OH, OW, ptr(out), sdt,
                                 stream()), "mapa_bilinear_ac")


def mean_tokens(x, n, T, C, y):
    work = torch.empty(n * 32 * C, device=x.device, dtype=torch.float32)
    check(lib().mapa_mean_tokens(ptr(x), n, T, C, ptr(y), ptr(work), stream()), "mapa_mean_tokens")


def linear_small(x, M, K, w, b, N, act, y):
    check(lib().mapa_linear_small(ptr(x), M, K, ptr(w), ptr(b), N, act, ptr(y), stream()), "mapa_linear_small")


def pose_scale_finalize(pose_raw, scale_raw, nviews, batch, pose_out, scale_out, poses44=None):
    check(lib().mapa_pose_scale_finalize(ptr(pose_raw), ptr(scale_raw), nviews, batch, ptr(pose_out),
                                         ptr(scale_out), ptr(poses44), stream()), "mapa_pose_scale_finalize")


def dense_head_out(hidden, n, HW, w6, b6, pose_out, scale, batch, pts3d, pts3d_cam, rays, depth, conf, logits,
                   mask):
    check(lib().mapa_dense_head_out(ptr(hidden), dt_code(hidden.dtype), n, HW, ptr(w6), ptr(b6), ptr(pose_out),
                                    ptr(scale), batch, ptr(pts3d), ptr(pts3d_cam), ptr(rays), ptr(depth), ptr(conf),
                                    ptr(logits), ptr(mask), stream()), "mapa_dense_head_out")


def convert_rows(src, lds, rows, cols, dst, ldd):
    check(lib().mapa_convert_rows(ptr(src), lds, rows, cols, ptr(dst), dt_code(dst.dtype), ldd, stream()),
          "mapa_convert_rows")


def split_bf16x3(x, rows, cols, cols_padded, y, ldx=None):
    """x fp32 [rows][cols] -> y bf16 [rows][2*cols_padded] = [hi | lo] (mapa.h mapa_split_bf16x3)."""
    if x.dtype != torch.float32 or y.dtype != torch.bfloat16 or y.numel() < rows * 2 * cols_padded:
        raise AssertionError("split_bf16x3: fp32 input, bf16 output of rows x 2*cols_padded")
    check(lib().mapa_split_bf16x3(ptr(x), cols if ldx is None else ldx, rows, cols, cols_padded, ptr(y), stream()),
          "mapa_split_bf16x3")


def split_rows(x, rows, cols, cols_padded, y, ldx=None):
    """x fp32 [rows][cols] -> y [rows][2*cols_padded] = [hi | lo]: the bf16 split (MAPA_BF16X3) for a bf16 y, the
    TF32-equivalent binary16 split (MAPA_F16X2) for an f16 y (mapa.h mapa_split_rows)."""
    if x.dtype != torch.float32 or y.dtype not in (torch.bfloat16, torch.float16) or \
            y.numel() < rows * 2 * cols_padded:
        raise AssertionError("split_rows: fp32 input, bf16 / f16 output of rows x 2*cols_padded")
    check(lib().mapa_split_rows(ptr(x), cols if ldx is None else ldx, rows, cols, cols_padded, ptr(y),
                                F16X2 if y.dtype == torch.float16 else BF16X3, stream()), "mapa_split_rows")


def fill_splitmix(out, seed, half, mid):
    check(lib().mapa_fill_splitmix(ptr(out), out.numel(), seed, half, mid, stream()), "mapa_fill_splitmix")


def postprocess_mask(pts3d, pts3d_cam, mask_in, mask_out, n, H, W, normal_cos_thr, depth_rtol, use_edges, work):
    check(lib().mapa_postprocess_mask(ptr(pts3d), ptr(pts3d_cam), ptr(mask_in), ptr(mask_out), n, H, W,
                                      float(normal_cos_thr), depth_rtol, int(use_edges), ptr(work), stream()),
          "mapa_postprocess_mask")


def resize_plan(in_w, in_h, rs_w, rs_h, crop_left, crop_top, out_w, out_h, filter_):
    """Host-only (no device): PIL's fixed-point resampling plan for an in_w x in_h -> rs_w x rs_h resize followed by
    the crop (crop_left, crop_top, +out_w, +out_h), as an int32 numpy blob (include/mapa.h mapa_resize_plan_build)."""
    import numpy as np
    L = load_library()
    nb = L.mapa_resize_plan_bytes(in_w, in_h, rs_w, rs_h, filter_)
    if nb < 0:
        raise NativeError(L.mapa_last_error().decode())
    blob = np.zeros(nb // 4, np.int32)
    check(L.mapa_resize_plan_build(in_w, in_h, rs_w, rs_h, crop_left, crop_top, out_w, out_h, filter_,
                                   blob.ctypes.data, nb), "mapa_resize_plan_build")
    return blob


def resize_plan_header(blob) -> ResizePlan:
    return ResizePlan.from_buffer_copy(blob[:ctypes.sizeof(ResizePlan) // 4].tobytes())


def resize_workspace_bytes(blob) -> int:
    return int(load_library().mapa_resize_workspace_bytes(blob.ctypes.data))


def resize_normalize(src_u8, src_row_bytes, blob, plan_dev, mean=None, std=None, out=None, out_u8=None,
                     workspace=None):
    """src_u8 (device, HWC RGB rows of src_row_bytes) -> out [3][out_h][out_w] f32 normalised and / or out_u8
    [out_h][out_w][3]; blob: the host plan, plan_dev: its device copy (include/mapa.h mapa_resize_normalize)."""
    m = s = None
    if out is not None:
        m = (ctypes.c_float * 3)(*[float(x) for x in mean])
        s = (ctypes.c_float * 3)(*[float(x) for x in std])
    ws = resize_workspace_bytes(blob)
    if ws and (workspace is None or workspace.numel() * workspace.element_size() < ws):
        raise NativeError(f"resize_normalize: workspace of {ws} bytes needed")
    check(lib().mapa_resize_normalize(ptr(src_u8), int(src_row_bytes), blob.ctypes.data, ptr(plan_dev),
                                      ctypes.cast(m, ctypes.c_void_p) if m is not None else None,
                                      ctypes.cast(s, ctypes.c_void_p) if s is not None else None, ptr(out),
                                      ptr(out_u8), ptr(workspace) if ws else None, ws, stream()),
          "mapa_resize_normalize")


def normal_cos_threshold(tol_deg: float) -> float:
    """The library's host-side boundary (double arccos rounded to float32), include/mapa.h."""
    return float(load_library().mapa_normal_cos_threshold(float(tol_deg)))


def recover_intrinsics(rays, n, H, W, K):
    check(lib().mapa_recover_intrinsics(ptr(rays), n, H, W, ptr(K), stream()), "mapa_recover_intrinsics")


def denorm_image(img, n, H, W, mean, std, out):
    check(lib().mapa_denorm_image(ptr(img), n, H, W, ptr(mean), ptr(std), ptr(out), stream()), "mapa_denorm_image")


def pixel_unshuffle(inp, n, H, W, C, r, out, *, ldo=None, view_div=None):
    """NHWC f32 [n][H][W][C] -> token rows [n*(H/r)*(W/r)][C*r*r]; view_div given: depth log-normalisation."""
    check(lib().mapa_pixel_unshuffle(ptr(inp), n, H, W, C, r, ptr(view_div), 1 if view_div is not None else 0,
                                     ptr(out), dt_code(out.dtype), ldo if ldo is not None else C * r * r,
                                     stream()), "mapa_pixel_unshuffle")


def depth_norm_factors(depth, n, HW, nf, log_nf=None):
    work = torch.empty(n * 128, device=depth.device, dtype=torch.float32)
    check(lib().mapa_depth_norm_factors(ptr(depth), n, HW, ptr(nf), ptr(log_nf), ptr(work), stream()),
          "mapa_depth_norm_factors")


def pose_inputs(quats, trans, cam_mask, V, out_q, out_t, out_log_nf):
    check(lib().mapa_pose_inputs(ptr(quats), ptr(trans), ptr(cam_mask), V, ptr(out_q), ptr(out_t), ptr(out_log_nf),
                                 stream()), "mapa_pose_inputs")


def add_view_vectors(x, T, C, nviews, vecs, scales, nvec):
    check(lib().mapa_add_view_vectors(ptr(x), T, C, nviews, ptr(vecs), ptr(scales), nvec, stream()),
          "mapa_add_view_vectors")


def add_f32(dst, src, n):
    check(lib().mapa_add_f32(ptr(dst), ptr(src), n, stream()), "mapa_add_f32")


def view_rays(n, H, W, rays, *, K=None, rays_in=None, depth_z=None, depth_along_ray=None):
    check(lib().mapa_view_rays(ptr(K), ptr(rays_in), ptr(depth_z), n, H, W, ptr(rays), ptr(depth_along_ray),
                               stream()), "mapa_view_rays")


def apply_mask(pts3d, pts3d_cam, depth_along_ray, mask, npix):
    check(lib().mapa_apply_mask(ptr(pts3d), ptr(pts3d_cam), ptr(depth_along_ray), ptr(mask), npix, stream()),
          "mapa_apply_mask")


def confidence_mask(conf, mask_in, mask_out, n, HW, q):
    check(lib().mapa_confidence_mask(ptr(conf), ptr(mask_in), ptr(mask_out), n, HW, float(q), stream()),
          "mapa_confidence_mask")


def attn_merge(o_a, lse_a, o_b, lse_b, o_out, rows, heads, ld, lse_out=None):
    check(lib().mapa_attn_merge(ptr(o_a), ptr(lse_a), ptr(o_b), ptr(lse_b), ptr(o_out), ptr(lse_out),
                                dt_code(o_a.dtype), rows, heads, ld, stream()), "mapa_attn_merge")


def dense_adaptor(raw, n, HW, value, conf, logits, mask):
    """raw [n][HW][6] f32 -> value [n][4][HW], conf / logits / mask [n][HW] (NCHW planes; include/mapa.h)."""
    check(lib().mapa_dense_adaptor(ptr(raw), n, HW, ptr(value), ptr(conf), ptr(logits), ptr(mask), stream()),
          "mapa_dense_adaptor")


def normalize_image(hwc_u8, n, H, W, mean, std, out):
    """hwc_u8 [n][H][W][3] uint8 (device) -> out [n][3][H][W] f32 = (x / 255 - mean) / std (include/mapa.h)."""
    m = (ctypes.c_float * 3)(*[float(x) for x in mean])
    s = (ctypes.c_float * 3)(*[float(x) for x in std])
    check(lib().mapa_normalize_image(ptr(hwc_u8), n, H, W, ctypes.cast(m, ctypes.c_void_p),
                                     ctypes.cast(s, ctypes.c_void_p), ptr(out), stream()), "mapa_normalize_image")


def rope2d(tokens, positions, B, H, N, D, sb, sh, sn, base, f0):
    """In-place RoPE-2D on tokens (B, H, N, D) with element strides (sb, sh, sn); positions int64 (B, N, 2)."""
    if positions.dtype != torch.int64 or not positions.is_contiguous():
        raise NativeError("rope2d: positions must be contiguous int64 (B, N, 2)")
    check(lib().mapa_rope2d(ptr(tokens), dt_code(tokens.dtype), B, H, N, D, sb, sh, sn, ptr(positions), float(base),
                            float(f0), stream()), "mapa_rope2d")
