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
from typing import Optional

import torch

NCCL_DTYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
               torch.float64: 8, torch.bfloat16: 9}  # ncclDataType_t (rccl.h)


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES


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
        L.ncclAllGather.argtypes = [vp, vp, sz, i, vp, vp]
        L.ncclBroadcast.argtypes = [vp, vp, sz, i, i, vp, vp]
        L.ncclCommDestroy.argtypes = [vp]
        L.ncclGetErrorString.argtypes = [i]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        for f in (L.ncclGetUniqueId, L.ncclCommInitRank, L.ncclAllGather, L.ncclBroadcast, L.ncclCommDestroy):
            f.restype = i
        _lib = L
    return _lib


class RcclError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc != 0:
        raise RcclError(f"{what}: {lib().ncclGetErrorString(rc).decode()} (ncclResult {rc})")


class Communicator:
    """One RCCL communicator over the ranks of a torch.distributed group; collectives on the caller's stream."""

    def __init__(self, group=None, device: Optional[torch.device] = None):
        import torch.distributed as dist

        L = lib()
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
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(L.ncclCommInitRank(ctypes.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        if t.dtype not in NCCL_DTYPES:
            raise RcclError(f"no RCCL datatype for {t.dtype}")
        return NCCL_DTYPES[t.dtype]

    def all_gather_(self, full: torch.Tensor, rows_per_slot: int, stream: torch.cuda.Stream):
        """In place: slot r of full ([world * rows_per_slot, ...]) = rank r's slot."""
        mine = full.narrow(0, self.rank * rows_per_slot, rows_per_slot)
        check(lib().ncclAllGather(mine.data_ptr(), full.data_ptr(), mine.numel(), self._dt(full), self._comm,
                                  stream.cuda_stream), "ncclAllGather")

    def broadcast_(self, t: torch.Tensor, src: int, stream: torch.cuda.Stream):
        check(lib().ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), src, self._comm,
                                  stream.cuda_stream), "ncclBroadcast")

    def close(self):
        if self._comm:
            lib().ncclCommDestroy(self._comm)
            self._comm = ctypes.c_void_p()
