"""View-sharded multi-GPU execution.

One process per GPU.  The V input views are split into contiguous blocks (view 0 -> rank 0, sizes differ by at
most one: 100 views on 8 ranks -> 13,13,13,13,12,12,12,12).  Every stage of the path is per-view except the
12 global layers of the alternating-attention transformer (alternating_attention_transformer.py:658-661): there
each rank computes Q for its own tokens and attends to the K/V of ALL tokens, so K/V are all-gathered once per
global layer (RCCL over xGMI; backend "nccl" of torch.distributed IS RCCL on ROCm).  The scale token is carried
by every rank as a replica whose K/V are contributed once, by rank 0; the replicas are NOT bit-identical (each
rank's query block count, attention chunking and partial-merge order differ, so they round differently), so the
final scale-token feature of rank 0 is broadcast before the scale head: every rank derives the same
metric_scaling_factor.  Outputs stay on the rank that owns the view, or are gathered (to rank 0 or to every
rank) when the model asks for it (MapAnything.enable_view_sharding(gather_outputs=...)).

Gathered K/V layout: [world][max_rows][2*C] with rank r's block in slot r (its valid rows first, padding after);
the attention kernel reads the valid rows through its K/V segment table, so no compaction copy is needed.
"""

from __future__ import annotations

import datetime
import os
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch


def force_collectives() -> bool:
    """Debug switch MAPA_FORCE_COLLECTIVES=1: a one-rank shard still runs the K/V all-gather (gather-first form) and
    the scale-token broadcast through its communicator, so the collective path — RCCL under HIP-graph capture
    included — runs on a single GPU.  Implied by MAPA_FORCE_OVERLAP=1."""
    return os.environ.get("MAPA_FORCE_COLLECTIVES", "0") == "1" or force_overlap()


def force_overlap() -> bool:
    """Debug switch MAPA_FORCE_OVERLAP=1: a one-rank shard runs the OVERLAPPED global layer of the multi-rank path —
    the asynchronous all-gather on the communicator's side stream, attention of the local queries over the first
    half of its own keys (treated as "local") with LSE, the join, attention over the second half (treated as
    "remote"), and the LSE merge — so the N > 1 production branch (RCCL fork / join under HIP-graph capture
    included) executes on a single GPU (engine._block_global_sharded)."""
    return os.environ.get("MAPA_FORCE_OVERLAP", "0") == "1"


class CommError(RuntimeError):
    """A collective of the view-sharded path failed or timed out (dead peer, RCCL / gloo error).  Raised instead of
    hanging; the process is expected to exit non-zero (bench.py does)."""


def comm_timeout() -> datetime.timedelta:
    """Timeout for communicator init and for every collective: MAPA_COMM_TIMEOUT_S seconds (default 300)."""
    return datetime.timedelta(seconds=float(os.environ.get("MAPA_COMM_TIMEOUT_S", "300")))


def init_distributed(backend: str = "nccl", device: Optional[torch.device] = None):
    """One process per GPU, env:// rendezvous (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, as torchrun sets them;
    the reference's own setup is mapanything/utils/train_tools.py:389-402).  Differences that matter for a serving
    job: the process group gets an explicit timeout (comm_timeout()), RCCL's watchdog tears the process down when a
    collective exceeds it (TORCH_NCCL_ASYNC_ERROR_HANDLING=1 unless set), and a first all-reduce proves that every
    peer is up — a rank that cannot reach the others raises CommError within the timeout instead of hanging.
    Returns (rank, world)."""
    import torch.distributed as dist

    timeout = comm_timeout()
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    try:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
        probe = torch.ones(1, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(probe)
        if backend == "nccl":
            torch.cuda.synchronize(device)
    except Exception as e:  # noqa: BLE001 — every init failure becomes one error type
        raise CommError(f"communicator init ({backend}) failed: {e}") from e
    world = dist.get_world_size()
    if int(probe.item()) != world:
        raise CommError(f"communicator init: probe all-reduce saw {int(probe.item())} of {world} ranks")
    return dist.get_rank(), world


@dataclass
class ShardPlan:
    """Views of one scene split over `world` ranks in contiguous runs (counts / starts).  scenes = B > 1: B batched
    scenes share the split (rank r holds views starts[r] .. +counts[r] of every scene, scene-major: local image
    b * counts[r] + i), and its K/V slot holds the B scenes' token rows then the B scale-token replicas."""
    num_views: int
    world: int
    rank: int
    tokens_per_view: int
    scenes: int = 1
    counts: List[int] = field(init=False)
    starts: List[int] = field(init=False)

    def __post_init__(self):
        V, P = self.num_views, self.world
        if V < P:
            raise ValueError(f"{V} views cannot be sharded over {P} ranks (need at least one view per rank)")
        if self.scenes < 1:
            raise ValueError(f"scenes must be >= 1, got {self.scenes}")
        self.counts = [V // P + (1 if r < V % P else 0) for r in range(P)]
        self.starts = [sum(self.counts[:r]) for r in range(P)]

    @property
    def local_views(self) -> range:
        return range(self.starts[self.rank], self.starts[self.rank] + self.counts[self.rank])

    def local_rows(self, r: Optional[int] = None) -> int:
        """AAT rows held by rank r: its views' tokens + the scale-token replica (of every scene)."""
        r = self.rank if r is None else r
        return self.scenes * (self.counts[r] * self.tokens_per_view + 1)

    def kv_valid_rows(self, r: int) -> int:
        """K/V rows rank r contributes to the global set (scale token only from rank 0); one scene."""
        return self.counts[r] * self.tokens_per_view + (1 if r == 0 else 0)

    @property
    def max_rows(self) -> int:
        return max(self.local_rows(r) for r in range(self.world))

    @property
    def total_kv(self) -> int:
        """Keys one global-attention query sees: its scene's tokens + its scale token."""
        return self.num_views * self.tokens_per_view + 1

    def kv_segments(self) -> List[Tuple[int, int]]:
        if self.scenes != 1:
            raise ValueError("kv_segments: one scene; use scene_kv_segments(b)")
        return [(r * self.max_rows, self.kv_valid_rows(r)) for r in range(self.world)]

    def scene_kv_segments(self, b: int) -> List[Tuple[int, int]]:
        """Scene b's keys in the gathered [world][max_rows] K/V: each rank's run of the scene's token rows, then the
        scene's scale token from rank 0's slot (one segment with rank 0's tokens when they are adjacent: B = 1)."""
        if self.scenes == 1:
            return self.kv_segments()
        T, B = self.tokens_per_view, self.scenes
        segs = [(r * self.max_rows + b * self.counts[r] * T, self.counts[r] * T) for r in range(self.world)]
        return segs + [(B * self.counts[0] * T + b, 1)]


class DistComm:
    """K/V exchange over a torch.distributed process group (RCCL on MI355X, gloo on CPU tests)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # ProcessGroupNCCL's collectives cannot be captured into a HIP graph (its watchdog polls the captured work's
        # events; rccl.py): the captured sharded forward uses RcclComm instead
        self.graph_safe = False

    def _call(self, what, fn, *a, **k):
        """Run one collective; a backend error (gloo raises on a dead peer / timeout, RCCL's watchdog on a timed-out
        collective) becomes CommError naming the collective and this rank."""
        try:
            return fn(*a, **k)
        except CommError:
            raise
        except RuntimeError as e:
            raise CommError(f"{what} failed on rank {self.rank} of {self.world}: {e}") from e

    def allgather_slots(self, full: torch.Tensor, rows_per_slot: int):
        """full: [world * rows_per_slot, C]; this rank's slot already written in place."""
        mine = full.narrow(0, self.rank * rows_per_slot, rows_per_slot)
        self._call("K/V all-gather", self.dist.all_gather_into_tensor, full, mine, group=self.group)

    def allgather_slots_async(self, full: torch.Tensor, rows_per_slot: int):
        """Start the slot all-gather on the communicator's stream (it waits for the current stream's K/V
        projection); the returned handle's wait() makes the current stream wait for the gathered slots."""
        mine = full.narrow(0, self.rank * rows_per_slot, rows_per_slot)
        work = self._call("K/V all-gather", self.dist.all_gather_into_tensor, full, mine, group=self.group,
                          async_op=True)
        comm = self

        class _Handle:
            def wait(self_inner):
                comm._call("K/V all-gather (wait)", work.wait)

        return _Handle()

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        """In place: every rank's t = rank src's t."""
        self._call("scale-token broadcast", self.dist.broadcast, t, src, group=self.group)

    def close(self, abort: bool = False):
        """Nothing to release: the process group belongs to the caller."""

    def check_async(self):
        """Device-side collectives of this communicator have no asynchronous error state of their own."""

    def all_agree(self, ok: bool, device) -> bool:
        """True on every rank iff ok on every rank (an eager MIN all-reduce of one int, never captured)."""
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        self._call("agreement all-reduce", self.dist.all_reduce, flag, op=self.dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item())

    def all_agree_host(self, ok: bool) -> bool:
        """all_agree over a gloo group of the same ranks on a CPU tensor: no device work and no stream
        synchronisation (the per-call fault agreement, MapAnything._await_faults, while the GPU still runs the heads).
        The group is made on first use — every rank reaches that call at the same point of the same call."""
        if getattr(self, "_host_group", None) is None:
            ranks = None if self.group is None else self.dist.get_process_group_ranks(self.group)
            self._host_group = self.dist.new_group(ranks=ranks, backend="gloo")
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        self._call("agreement all-reduce (host)", self.dist.all_reduce, flag, op=self.dist.ReduceOp.MIN,
                   group=self._host_group)
        return bool(flag.item())

    def gather_views(self, local: torch.Tensor, counts: List[int], dst: Optional[int]) -> Optional[torch.Tensor]:
        """View-major local rows [counts[rank], ...] -> [sum(counts), ...] in rank order on rank dst (None: on
        every rank); other ranks get None.  Slots are padded to max(counts) so one collective moves them."""
        if local.dtype == torch.bool:  # moved as bytes
            out = self.gather_views(local.view(torch.uint8), counts, dst)
            return None if out is None else out.view(torch.bool)
        mx = max(counts)
        slot = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        slot[:local.shape[0]].copy_(local)
        if dst is None:
            full = torch.empty((self.world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            self._call("output all-gather", self.dist.all_gather_into_tensor, full, slot, group=self.group)
        else:
            lst = [torch.empty_like(slot) for _ in range(self.world)] if self.rank == dst else None
            self._call("output gather", self.dist.gather, slot, lst, dst=dst, group=self.group)
            if self.rank != dst:
                return None
            full = torch.cat(lst, 0)
        return torch.cat([full[r * mx:r * mx + c] for r, c in enumerate(counts)], 0)


class RcclComm(DistComm):
    """DistComm whose device-side collectives (the per-global-layer K/V all-gather, the scale-token broadcast) go to
    RCCL directly on a communicator of its own (mapanything/rccl.py), so they can be captured with the kernels into
    the sharded forward's HIP graph; the host-side ones (output gather, the capture agreement) stay on the process
    group.  The overlapped all-gather runs on a side stream forked from and joined back into the caller's stream
    (event record / wait: captured as graph edges).  The communicator is created non-blocking and its init polled
    against comm_timeout() (rccl.Communicator: a peer that fails inside its init makes this rank raise CommError
    instead of hanging); an RCCL error raises CommError.  Captured collectives have no watchdog of their own: the
    model's per-call fault wait (MapAnything._await_faults, bounded by comm_timeout()) polls check_async() and, if
    the forward does not reach its fault publish in time, aborts the communicator (abort() stops RCCL's kernels)
    and raises CommError."""

    def __init__(self, group=None, device=None):
        super().__init__(group)
        self.graph_safe = True
        from . import rccl

        self._rccl_mod = rccl
        try:
            self._nccl = rccl.Communicator(group, device)
        except Exception as e:  # noqa: BLE001 — init failures become CommError like the process group's
            raise CommError(f"RCCL communicator init failed on rank {self.rank} of {self.world}: {e}") from e
        self._side = torch.cuda.Stream(self._nccl.device)

    def _rc(self, what, fn, *a):
        try:
            fn(*a)
        except self._rccl_mod.RcclError as e:
            raise CommError(f"{what} failed on rank {self.rank} of {self.world}: {e}") from e

    def check_async(self):
        try:
            self._rc("RCCL", self._nccl.check_async)
        except CommError:
            self.graph_safe = False  # check_async aborted the communicator
            raise

    def abort(self):
        """ncclCommAbort; the communicator is unusable afterwards (graphs captured against it must not replay)."""
        self._nccl.abort()
        self.graph_safe = False

    def close(self, abort: bool = False):
        """Release the RCCL communicator (ncclCommFinalize + ncclCommDestroy, or ncclCommAbort after an error)."""
        self._nccl.close(abort=abort)

    def allgather_slots(self, full: torch.Tensor, rows_per_slot: int):
        self._rc("K/V all-gather", self._nccl.all_gather_, full, rows_per_slot, torch.cuda.current_stream())

    def allgather_slots_async(self, full: torch.Tensor, rows_per_slot: int):
        from . import _native as nat

        cur = torch.cuda.current_stream()
        side = self._side
        side.wait_stream(cur)  # the K/V projection into this rank's slot is done
        g0 = nat.mark(side)  # eager timing pass only (bench.py kv_overlap): the gather on the communicator's stream
        self._rc("K/V all-gather", self._nccl.all_gather_, full, rows_per_slot, side)
        nat.span("kv_allgather", g0, nat.mark(side))

        class _Handle:
            def wait(self_inner):
                cur.wait_stream(side)

        return _Handle()

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        self._rc("scale-token broadcast", self._nccl.broadcast_, t, src, torch.cuda.current_stream())


class ThreadComm:
    """In-process communicator for tests: P threads (one engine each, same device) exchange slots through a
    barrier; the exchanged bytes are identical to what all_gather_into_tensor delivers.  Each rank thread must
    launch on its own HIP stream (as separate processes do): the library's scratch buffers are per stream."""

    graph_safe = False  # host synchronisation inside every exchange

    def __init__(self, world: int):
        self.world = world
        self._barrier = threading.Barrier(world)
        self._bufs = [None] * world
        self._local = threading.local()

    def bind(self, rank: int):
        self._local.rank = rank
        return self

    @property
    def rank(self):
        return self._local.rank

    def allgather_slots(self, full: torch.Tensor, rows_per_slot: int):
        r = self.rank
        torch.cuda.current_stream().synchronize() if full.is_cuda else None
        self._bufs[r] = full
        self._barrier.wait()
        for s in range(self.world):
            if s != r:
                src = self._bufs[s].narrow(0, s * rows_per_slot, rows_per_slot)
                full.narrow(0, s * rows_per_slot, rows_per_slot).copy_(src)
        if full.is_cuda:
            torch.cuda.current_stream().synchronize()
        self._barrier.wait()

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if t.is_cuda:
            torch.cuda.current_stream().synchronize()
        self._bufs[self.rank] = t
        self._barrier.wait()
        if self.rank != src:
            t.copy_(self._bufs[src])
            if t.is_cuda:
                torch.cuda.current_stream().synchronize()
        self._barrier.wait()

    def all_agree_host(self, ok: bool) -> bool:
        return self.all_agree(ok)

    def all_agree(self, ok: bool, device=None) -> bool:
        """True on every rank thread iff ok on every one (barrier-exchanged flags)."""
        self._bufs[self.rank] = bool(ok)
        self._barrier.wait()
        res = all(bool(b) for b in self._bufs)
        self._barrier.wait()
        return res

    def gather_views(self, local: torch.Tensor, counts: List[int], dst: Optional[int]) -> Optional[torch.Tensor]:
        if local.is_cuda:
            torch.cuda.current_stream().synchronize()
        self._bufs[self.rank] = local
        self._barrier.wait()
        out = None
        if dst is None or self.rank == dst:
            out = torch.cat([self._bufs[r].to(local.device) for r in range(self.world)], 0)
            if local.is_cuda:
                torch.cuda.current_stream().synchronize()
        self._barrier.wait()
        return out

    def allgather_slots_async(self, full: torch.Tensor, rows_per_slot: int):
        """Deferred exchange: this rank's slot is final now (synchronised), the other slots are filled at wait();
        work enqueued in between may read only this rank's own slot, exactly as with the RCCL overlap."""
        comm = self
        if full.is_cuda:
            torch.cuda.current_stream().synchronize()

        class _Handle:
            def wait(self_inner):
                comm.allgather_slots(full, rows_per_slot)

        return _Handle()
