"""View-sharding host logic (mapanything/parallel.py) on CPU: shard plan, in-place slot all-gather over a real
torch.distributed group (gloo, world_size 2 and 3), and the sharded global-attention algorithm (local Q, gathered
K/V read through the segment table) against unsharded attention.  The GPU version of the same algorithm is
tests/test_gpu_sharded.py."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from mapanything.parallel import DistComm, ShardPlan


def test_shard_plan_layout():
    p = ShardPlan(100, 8, 0, 1369)
    assert p.counts == [13, 13, 13, 13, 12, 12, 12, 12]
    assert p.starts[:3] == [0, 13, 26]
    assert list(ShardPlan(100, 8, 5, 1369).local_views) == list(range(64, 76))
    assert p.max_rows == 13 * 1369 + 1
    segs = p.kv_segments()
    assert segs[0] == (0, 13 * 1369 + 1) and segs[7] == (7 * p.max_rows, 12 * 1369)
    assert sum(n for _, n in segs) == p.total_kv == 100 * 1369 + 1
    with pytest.raises(ValueError):
        ShardPlan(3, 4, 0, 10)


def test_shard_plan_batched_scenes():
    """B scenes share the view split; each rank's slot holds [scene][view][token] rows then the B scale-token
    replicas, and scene b's segments select exactly its tokens on every rank plus its scale token from rank 0."""
    V, world, T, B = 7, 3, 5, 4
    plans = [ShardPlan(V, world, r, T, scenes=B) for r in range(world)]
    p = plans[0]
    assert p.counts == [3, 2, 2] and p.max_rows == B * (3 * T + 1) and p.total_kv == V * T + 1
    # global K/V laid out as the engine writes it: rank r's slot row of (scene b, local view i, token t)
    full = -torch.ones(world * p.max_rows, dtype=torch.int64)
    for r, pr in enumerate(plans):
        c = pr.counts[r]
        for b in range(B):
            for i in range(c):
                for t in range(T):
                    full[r * p.max_rows + (b * c + i) * T + t] = b * 1000 + (pr.starts[r] + i) * T + t
            full[r * p.max_rows + B * c * T + b] = b * 1000 + V * T  # scale-token replica
    for b in range(B):
        segs = p.scene_kv_segments(b)
        assert len(segs) == world + 1 and sum(n for _, n in segs) == p.total_kv
        got = torch.cat([full[st:st + n] for st, n in segs]).tolist()
        assert sorted(got) == [b * 1000 + k for k in range(V * T + 1)]
    # one scene: the B = 1 layout and segments
    assert ShardPlan(V, world, 0, T, scenes=1).scene_kv_segments(0) == ShardPlan(V, world, 0, T).kv_segments()
    with pytest.raises(ValueError):
        p.kv_segments()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gather_rows(full, segs):
    return torch.cat([full[st:st + n] for st, n in segs], 0)


def _attn_lse(qh, kh, vh):
    s = qh @ kh.transpose(-1, -2) / 8.0
    lse = torch.logsumexp(s, -1)
    return torch.softmax(s, -1) @ vh, lse


def _worker(rank, world, port, V, T, C, q, overlap=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        heads, hd = C // 64, 64
        # the same global token set on every rank (view-major, scale token last)
        tokens_q = torch.randn(V * T + 1, C, generator=g)
        tokens_kv = torch.randn(V * T + 1, 2 * C, generator=g)
        plan = ShardPlan(V, world, rank, T)
        comm = DistComm()
        lv = list(plan.local_views)
        rows = torch.cat([torch.arange(v * T, (v + 1) * T) for v in lv] + [torch.tensor([V * T])])
        full = torch.zeros(world * plan.max_rows, 2 * C)
        L = plan.local_rows()
        full[rank * plan.max_rows:rank * plan.max_rows + L] = tokens_kv[rows]
        segs = plan.kv_segments()
        if overlap:
            # the engine's overlapped global layer: own-key partial while the gather is in flight, remote partial
            # after wait(), LSE merge (engine._block_global_sharded / mapa_attn_merge)
            h = comm.allgather_slots_async(full, plan.max_rows)
            qh0 = tokens_q[rows].view(L, C // 64, 64).transpose(0, 1)
            own = _gather_rows(full, [segs[rank]])
            o_l, l_l = _attn_lse(qh0, own[:, :C].reshape(-1, C // 64, 64).transpose(0, 1),
                                 own[:, C:].reshape(-1, C // 64, 64).transpose(0, 1))
            h.wait()
            rest = _gather_rows(full, [sg for r, sg in enumerate(segs) if r != rank])
            o_r, l_r = _attn_lse(qh0, rest[:, :C].reshape(-1, C // 64, 64).transpose(0, 1),
                                 rest[:, C:].reshape(-1, C // 64, 64).transpose(0, 1))
            m = torch.maximum(l_l, l_r)
            wl, wr = torch.exp(l_l - m)[..., None], torch.exp(l_r - m)[..., None]
            merged = (wl * o_l + wr * o_r) / (wl + wr)
        else:
            comm.allgather_slots(full, plan.max_rows)
        kv = _gather_rows(full, segs)
        assert kv.shape[0] == plan.total_kv
        # sharded attention for the local queries
        qh = tokens_q[rows].view(L, heads, hd).transpose(0, 1)
        kh = kv[:, :C].reshape(-1, heads, hd).transpose(0, 1)
        vh = kv[:, C:].reshape(-1, heads, hd).transpose(0, 1)
        got = F.scaled_dot_product_attention(qh[None], kh[None], vh[None])[0]
        # unsharded reference
        ref = F.scaled_dot_product_attention(tokens_q.view(-1, heads, hd).transpose(0, 1)[None],
                                             tokens_kv[:, :C].reshape(-1, heads, hd).transpose(0, 1)[None],
                                             tokens_kv[:, C:].reshape(-1, heads, hd).transpose(0, 1)[None])[0]
        err = (got - ref[:, rows]).abs().max().item()
        if overlap:
            err = max(err, (merged - ref[:, rows]).abs().max().item())
        q.put((rank, err, sorted(kv[:, 0].tolist()) == sorted(tokens_kv[:, 0].tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("world,V", [(2, 5), (3, 7)])
def test_sharded_global_attention_gloo(world, V, overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, V, 16, 128, q, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, same_set in res:
        assert same_set, f"rank {rank}: gathered K/V set differs from the global token set"
        assert err < 1e-5, f"rank {rank}: sharded attention differs by {err}"


def _gather_worker(rank, world, port, q):
    """DistComm.broadcast_ (the scale-token feature), all_agree and gather_views (outputs to rank 0 / to every rank) over a
    real gloo group, and MapAnything._finish assembling the reference's per-view list from them."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mapanything.models.mapanything.model import MapAnything

        V = 7
        plan = ShardPlan(V, world, rank, 4)
        comm = DistComm()
        tok = torch.full((1, 8), float(rank + 1))
        comm.broadcast_(tok, 0)
        ok_bcast = bool((tok == 1.0).all())
        # the sharded graph-capture fallback's agreement: one failing rank makes every rank fall back
        ok_bcast &= comm.all_agree(True, "cpu") and not comm.all_agree(rank != world - 1, "cpu")
        lv = list(plan.local_views)
        local = {"pts3d": torch.stack([torch.full((1, 2, 2, 3), float(v)) for v in lv], 0).view(len(lv), 2, 2, 3),
                 "non_ambiguous_mask": torch.tensor([[[v % 2 == 0]] for v in lv]).view(len(lv), 1, 1),
                 "metric_scaling_factor": torch.ones(1, 1)}
        m = MapAnything.__new__(MapAnything)  # host glue only: no weights, no device
        m._comm = comm
        res = {}
        for mode in ("rank0", "all", None):
            m._gather = mode
            out = m._finish(dict(local), plan, V, with_post=False)
            got = [None if o is None else float(o["pts3d"].flatten()[0]) for o in out]
            masks = [None if o is None else bool(o["non_ambiguous_mask"].flatten()[0]) for o in out]
            res[mode] = (got, masks)
        # B = 2 batched scenes: local rows scene-major (scene b, local view i), value 100 b + global view
        B = 2
        plan2 = ShardPlan(V, world, rank, 4, scenes=B)
        lv = list(plan2.local_views)
        vals = [100 * b + v for b in range(B) for v in lv]
        local2 = {"pts3d": torch.tensor(vals, dtype=torch.float32).view(-1, 1, 1, 1).expand(-1, 2, 2, 3).contiguous(),
                  "metric_scaling_factor": torch.ones(B, 1)}
        for mode in ("rank0", "all", None):
            m._gather = mode
            out = m._finish(dict(local2), plan2, V, with_post=False, scenes=B)
            res[("b2", mode)] = [None if o is None else o["pts3d"][:, 0, 0, 0].tolist() for o in out]
        q.put((rank, ok_bcast, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scale_token_broadcast_and_output_gather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    V = 7
    every = [float(v) for v in range(V)]
    every_mask = [v % 2 == 0 for v in range(V)]
    for rank, ok_bcast, r in res:
        assert ok_bcast, rank
        plan = ShardPlan(V, world, rank, 4)
        own = [float(v) if v in plan.local_views else None for v in range(V)]
        assert r["all"] == (every, every_mask)
        assert r["rank0"][0] == (every if rank == 0 else own)
        assert r[None][0] == own
        every2 = [[float(v), float(100 + v)] for v in range(V)]  # per view: its (B,) values, scene order
        own2 = [e if v in plan.local_views else None for v, e in enumerate(every2)]
        assert r[("b2", "all")] == every2
        assert r[("b2", "rank0")] == (every2 if rank == 0 else own2)
        assert r[("b2", None)] == own2


class _FakeRccl:
    """Stands in for librccl.so in rccl.Communicator (the init protocol only): the last rank fails inside its own
    ncclCommInitRankConfig; the others see their non-blocking init stay in progress (peers that never arrive) or,
    with mode "async_error", turn into an asynchronous error after a few polls."""

    def __init__(self, rank, world, mode):
        self.rank, self.world, self.mode = rank, world, mode
        self.aborted, self.polls, self.blocking = 0, 0, None

    def ncclGetUniqueId(self, uid):
        return 0

    def ncclCommInitRankConfig(self, pcomm, nranks, uid, rank, cfg):
        self.blocking = cfg._obj.blocking
        pcomm._obj.value = 0x1234  # the communicator object exists before the connection set-up
        if rank == self.world - 1:
            return 2  # ncclSystemError inside this rank's init
        return 7  # ncclInProgress

    def ncclCommGetAsyncError(self, comm, pst):
        self.polls += 1
        pst._obj.value = 3 if (self.mode == "async_error" and self.polls > 5) else 7
        return 0

    def ncclCommAbort(self, comm):
        self.aborted += 1
        return 0

    def ncclGetErrorString(self, rc):
        return {2: b"unhandled system error", 3: b"internal error", 7: b"in progress"}.get(rc, b"?")


def _rccl_init_worker(rank, world, port, mode, q):
    """rccl.Communicator's non-blocking init with a peer failing inside its init: every rank raises RcclError within
    the timeout (the waiting ranks abort their half-built communicator), then the ranks agree to fall back — the
    sequence MapAnything.enable_view_sharding runs before it keeps the process-group communicator."""
    import time

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mapanything import rccl

        fake = _FakeRccl(rank, world, mode)
        t0 = time.monotonic()
        err = None
        try:
            rccl.Communicator(None, None, lib_=fake, timeout_s=2.0)
        except rccl.RcclError as e:
            err = e
        dt = time.monotonic() - t0
        agreed = DistComm().all_agree(err is None, "cpu")
        q.put((rank, type(err).__name__ if err else None, str(err), dt, fake.aborted, fake.blocking, agreed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["timeout", "async_error"])
@pytest.mark.parametrize("world", [2, 3])
def test_rccl_init_failure_raises_on_every_rank_within_timeout(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rccl_init_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, kind, msg, dt, aborted, blocking, agreed in res:
        assert blocking == 0, "the communicator must be created non-blocking"
        assert kind is not None, f"rank {rank} did not raise"
        assert not agreed, "every rank must agree to fall back"
        assert dt < 10.0, (rank, dt)
        if rank == world - 1:
            assert kind == "RcclError" and "system error" in msg and aborted == 1
        elif mode == "timeout":
            assert kind == "RcclTimeout" and dt >= 2.0 and aborted == 1, (rank, kind, dt, aborted)
        else:
            assert kind == "RcclError" and "internal error" in msg and aborted == 1, (rank, kind, msg)
