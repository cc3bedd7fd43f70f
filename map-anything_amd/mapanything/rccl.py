"""Direct RCCL binding for the HIP-graph-captured view-sharded forward.

The sharded forward's collectives (one K/V all-gather per global layer, the scale-token broadcast) must be enqueued
on the device inside a HIP graph capture.  Issued through torch.distributed's ProcessGroupNCCL they cannot be: its
watchdog thread polls the completion events of the captured work (hipEventQuery on an event recorded in a capturing
stream), which invalidates the capture on ROCm 7 (measured on MI355X: `operation failed due to a previous error during
capture`, then the watchdog aborts the process).  So the sharded path talks to RCCL itself — the same librccl.so
torch loaded — on a communicator of its own: ncclAllGather / ncclBroadcast go straight onto the caller's stream, no
events, no host-side bookkeeping, capturable like any kernel.  The unique id is exchanged over the existing process
group (the reference's own setup: mapanything/utils/train_tools.py:389-402), which also keeps the host-side
collectives (output gather, the capture agreement).
"""

from __future__ import annotations

import ctypes
import os
import time
from typing import Optional

import torch

NCCL_DTYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
               torch.float64: 8, torch.bfloat16: 9}  # ncclDataType_t (rccl.h)


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES


NCCL_SUCCESS, NCCL_IN_PROGRESS = 0, 7  # ncclResult_t
_UNDEF_INT = -2 ** 31                  # NCCL_CONFIG_UNDEF_INT


class Config(ctypes.Structure):
    """ncclConfig_t in its 2.17 layout (ncclConfig_v21700: the fields every RCCL since 2.17 reads; the library copies
    `size` bytes and keeps its defaults for the rest), as NCCL_CONFIG_INITIALIZER fills it, non-blocking."""
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int), ("minCTAs", ctypes.c_int),
                ("maxCTAs", ctypes.c_int), ("netName", ctypes.c_char_p), ("splitShare", ctypes.c_int)]

    @classmethod
    def nonblocking(cls):
        c = cls()
        c.size, c.magic, c.version = ctypes.sizeof(cls), 0xCAFEBEEF, 21700
        c.blocking = 0
        c.cgaClusterSize = c.minCTAs = c.maxCTAs = c.splitShare = _UNDEF_INT
        c.netName = None
        return c


_lib = None


def lib_path() -> str:
    """torch's bundled librccl.so (the library its process groups already loaded), else the system one."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(lib_path())
        vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), i, UniqueId, i]
        L.ncclCommInitRankConfig.argtypes = [ctypes.POINTER(vp), i, UniqueId, i, ctypes.POINTER(Config)]
        L.ncclCommGetAsyncError.argtypes = [vp, ctypes.POINTER(i)]
        L.ncclCommAbort.argtypes = [vp]
        L.ncclCommFinalize.argtypes = [vp]
        L.ncclAllGather.argtypes = [vp, vp, sz, i, vp, vp]
        L.ncclBroadcast.argtypes = [vp, vp, sz, i, i, vp, vp]
        L.ncclCommDestroy.argtypes = [vp]
        L.ncclGetErrorString.argtypes = [i]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        for f in (L.ncclGetUniqueId, L.ncclCommInitRank, L.ncclCommInitRankConfig, L.ncclCommGetAsyncError,
                  L.ncclCommAbort, L.ncclCommFinalize, L.ncclAllGather, L.ncclBroadcast, L.ncclCommDestroy):
            f.restype = i
        _lib = L
    return _lib


class RcclError(RuntimeError):
    pass


class RcclTimeout(RcclError):
    pass


def _err(L, rc: int) -> str:
    return f"{L.ncclGetErrorString(rc).decode()} (ncclResult {rc})"


def check(rc: int, what: str):
    if rc != 0:
        raise RcclError(f"{what}: {_err(lib(), rc)}")


def _timeout_s() -> float:
    from .parallel import comm_timeout

    return comm_timeout().total_seconds()


class Communicator:
    """One RCCL communicator over the ranks of a torch.distributed group; collectives on the caller's stream.

    Created NON-BLOCKING (ncclCommInitRankConfig, blocking = 0): the init returns at once and the connection set-up
    is polled with ncclCommGetAsyncError against comm_timeout(), so a rank whose peers fail inside their own init
    (or never arrive) raises RcclTimeout here instead of hanging in ncclCommInitRank, and its half-built
    communicator is torn down with ncclCommAbort.  A collective that returns ncclInProgress (the non-blocking
    launch path) is polled the same way before the next call.  `lib_` replaces the RCCL binding (tests drive the
    init protocol with a fake library on a gloo group)."""

    def __init__(self, group=None, device: Optional[torch.device] = None, lib_=None, timeout_s: Optional[float] = None):
        import torch.distributed as dist

        L = lib_ if lib_ is not None else lib()
        self._L = L
        self.timeout_s = _timeout_s() if timeout_s is None else float(timeout_s)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        uid = UniqueId()
        obj = [None]
        if self.rank == 0:  # rank 0 always reaches the broadcast: an error travels to every rank as a string
            rc = L.ncclGetUniqueId(ctypes.byref(uid))
            obj = [ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid)) if rc == 0
                   else f"ncclGetUniqueId: {L.ncclGetErrorString(rc).decode()} (ncclResult {rc})"]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if isinstance(obj[0], str):
            raise RcclError(obj[0])
        ctypes.memmove(ctypes.addressof(uid), obj[0], ctypes.sizeof(uid))
        if device is None and lib_ is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self._comm = ctypes.c_void_p()
        cfg = Config.nonblocking()
        if device is not None and lib_ is None:
            with torch.cuda.device(device):
                rc = L.ncclCommInitRankConfig(ctypes.byref(self._comm), self.world, uid, self.rank, ctypes.byref(cfg))
        else:
            rc = L.ncclCommInitRankConfig(ctypes.byref(self._comm), self.world, uid, self.rank, ctypes.byref(cfg))
        if rc not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
            self.abort()
            raise RcclError(f"ncclCommInitRankConfig: {_err(L, rc)}")
        self.wait_ready("ncclCommInitRankConfig")

    def async_state(self) -> int:
        """ncclCommGetAsyncError of the communicator (NCCL_SUCCESS, NCCL_IN_PROGRESS or an error code)."""
        st = ctypes.c_int(NCCL_SUCCESS)
        rc = self._L.ncclCommGetAsyncError(self._comm, ctypes.byref(st))
        return rc if rc != NCCL_SUCCESS else st.value

    def wait_ready(self, what: str, timeout_s: Optional[float] = None):
        """Poll until the communicator's pending operation (init, a non-blocking launch) completes; on an error or
        past the timeout abort the communicator and raise (RcclError / RcclTimeout)."""
        deadline = time.monotonic() + (self.timeout_s if timeout_s is None else timeout_s)
        pause = 1e-4
        while True:
            st = self.async_state()
            if st == NCCL_SUCCESS:
                return
            if st != NCCL_IN_PROGRESS:
                self.abort()
                raise RcclError(f"{what}: {_err(self._L, st)} (rank {self.rank} of {self.world})")
            if time.monotonic() > deadline:
                self.abort()
                raise RcclTimeout(f"{what}: not complete after {self.timeout_s:.0f} s on rank {self.rank} of "
                                  f"{self.world} (communicator aborted)")
            time.sleep(pause)
            pause = min(pause * 2, 0.02)

    def check_async(self, what: str = "RCCL"):
        """Raise (after aborting) if the communicator reports an asynchronous error — a peer lost mid-collective."""
        st = self.async_state() if self._comm else NCCL_SUCCESS
        if st not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
            self.abort()
            raise RcclError(f"{what}: asynchronous error {_err(self._L, st)} on rank {self.rank} of {self.world}")

    def _issue(self, rc: int, what: str):
        if rc == NCCL_IN_PROGRESS:
            self.wait_ready(what)
        elif rc != NCCL_SUCCESS:
            raise RcclError(f"{what}: {_err(self._L, rc)}")

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        if t.dtype not in NCCL_DTYPES:
            raise RcclError(f"no RCCL datatype for {t.dtype}")
        return NCCL_DTYPES[t.dtype]

    def all_gather_(self, full: torch.Tensor, rows_per_slot: int, stream: torch.cuda.Stream):
        """In place: slot r of full ([world * rows_per_slot, ...]) = rank r's slot."""
        mine = full.narrow(0, self.rank * rows_per_slot, rows_per_slot)
        self._issue(self._L.ncclAllGather(mine.data_ptr(), full.data_ptr(), mine.numel(), self._dt(full), self._comm,
                                          stream.cuda_stream), "ncclAllGather")

    def broadcast_(self, t: torch.Tensor, src: int, stream: torch.cuda.Stream):
        self._issue(self._L.ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), src, self._comm,
                                          stream.cuda_stream), "ncclBroadcast")

    def abort(self):
        """ncclCommAbort: tear the communicator down without waiting for its peers (an error, a timeout, a
        collective that never completes — RCCL's kernels stop on the abort flag)."""
        if self._comm:
            self._L.ncclCommAbort(self._comm)
            self._comm = ctypes.c_void_p()

    def close(self, abort: bool = False):
        """Normal teardown: ncclCommFinalize (flushes the issued collectives; polled against the timeout) then
        ncclCommDestroy; abort=True (or a finalize that fails) aborts instead."""
        if not self._comm:
            return
        if not abort:
            try:
                self._issue(self._L.ncclCommFinalize(self._comm), "ncclCommFinalize")
                self._L.ncclCommDestroy(self._comm)
                self._comm = ctypes.c_void_p()
                return
            except RcclError:
                pass  # wait_ready aborted already, or fall through to the abort
        self.abort()
