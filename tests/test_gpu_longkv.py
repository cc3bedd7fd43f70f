"""Long-sequence global attention at the BASELINE key counts, checked independently of the model.

configs[2] (100 views over 8 ranks) runs every global AAT layer over 100*1369+1 = 136 901 keys, configs[4]
(2000 views, memory_efficient_inference) over 2 738 001 keys (8.4 GB of bf16 K/V per layer, reference
uniception/models/utils/transformer_blocks.py:198-201).  The attention kernel is run on a few thousand query rows
against K/V laid out exactly as the sharded layer lays them out (8 rank slots of a [world][max_rows][2C] buffer read
through the segment table, parallel.ShardPlan) and compared with a chunked fp32 softmax in torch on the same device
(online max / sum over key chunks: the whole score matrix would not fit).  Few query rows leave most of the chip's
workgroup slots empty, so the kernel cuts the key range into chunks and combines them in attn_split_merge; more rows
take the whole-range path; the local-slot / remote-slots split of the overlapped all-gather is merged through the
LSEs with mapa_attn_merge.  Any mis-indexed segment or chunk shows up as an O(1) error: with near-uniform attention
the output is the mean of V over exactly the right key set.

A second test runs rank 0's share of the configs[4] job (250 of 2000 views at 518^2, memory_efficient_inference)
through the sharded model path with a replica communicator standing in for the 7 other ranks."""

import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu

HEADS, C = 12, 768


@pytest.fixture(scope="module")
def nat():
    from mapanything import _native

    _native.lib()
    return _native


def _layout(num_views, world=8, T=1369):
    from mapanything.parallel import ShardPlan

    p = ShardPlan(num_views, world, 0, T)
    return p.world * p.max_rows, p.kv_segments(), p.total_kv


def _ref_attention(q, kv, segs, chunk=1 << 17):
    """fp32 softmax(q k^T / 8) v over the logical keys (segment order), per head, chunked over keys."""
    Sq = q.shape[0]
    out = torch.empty(Sq, C, device="cuda")
    lse = torch.empty(HEADS, Sq, device="cuda")
    for h in range(HEADS):
        qh = q[:, h * 64:(h + 1) * 64].float() / 8.0
        m = torch.full((Sq,), float("-inf"), device="cuda")
        l = torch.zeros(Sq, device="cuda")
        acc = torch.zeros(Sq, 64, device="cuda")
        for st, n in segs:
            for c0 in range(st, st + n, chunk):
                c1 = min(c0 + chunk, st + n)
                k = kv[c0:c1, h * 64:(h + 1) * 64].float()
                v = kv[c0:c1, C + h * 64:C + (h + 1) * 64].float()
                s = qh @ k.t()
                mn = torch.maximum(m, s.amax(1))
                p = torch.exp(s - mn[:, None])
                sc = torch.exp(m - mn)
                l = l * sc + p.sum(1)
                acc = acc * sc[:, None] + p @ v
                m = mn
                del s, p
        out[:, h * 64:(h + 1) * 64] = acc / l[:, None]
        lse[h] = m + torch.log(l)
    return out, lse


def _run(nat, q, kv, segs, lse=None):
    Sq = q.shape[0]
    o = torch.empty(Sq, C, device="cuda", dtype=torch.bfloat16)
    nat.attention(q, kv, kv[:, C:], o, batch=1, heads=HEADS, seq_q=Sq, seq_kv=sum(n for _, n in segs), q_bstride=0,
                  q_rstride=C, k_bstride=0, k_rstride=2 * C, v_bstride=0, v_rstride=2 * C, o_bstride=0, o_rstride=C,
                  lse=lse, kv_segments=segs, kind="attention_global")
    return o


@pytest.mark.parametrize("views,Sq", [(100, 16384), (100, 2048), (2000, 2048), (2000, 8192)])
def test_long_kv_attention_matches_chunked_fp32(nat, views, Sq):
    rows, segs, total = _layout(views)
    g = torch.Generator(device="cuda").manual_seed(views * 7 + Sq)
    kv = torch.randn(rows, 2 * C, device="cuda", dtype=torch.bfloat16, generator=g)
    q = (1.5 * torch.randn(Sq, C, device="cuda", generator=g)).to(torch.bfloat16)
    lse = torch.empty(1, HEADS, Sq, device="cuda")
    o = _run(nat, q, kv, segs, lse)
    torch.cuda.synchronize()
    assert sum(n for _, n in segs) == total
    ref, ref_lse = _ref_attention(q, kv, segs)
    e, el = rel_l2(o.float().cpu(), ref.cpu()), rel_l2(lse[0].cpu(), ref_lse.cpu())
    print(f"\n[{total} keys, {Sq} query rows] rel-L2 out {e:.2e}  lse {el:.2e}")
    assert torch.isfinite(o.float()).all()
    assert e < 8e-3 and el < 1e-4, (e, el)


def test_long_kv_local_remote_split_merges_through_lse(nat):
    """The overlapped all-gather path at configs[4] size: rank 0's own slot first (with LSE), the 7 remote slots
    after the gather, the two partials merged by mapa_attn_merge (engine._block_global_sharded)."""
    rows, segs, total = _layout(2000)
    Sq = 4096
    g = torch.Generator(device="cuda").manual_seed(5)
    kv = torch.randn(rows, 2 * C, device="cuda", dtype=torch.bfloat16, generator=g)
    q = (1.5 * torch.randn(Sq, C, device="cuda", generator=g)).to(torch.bfloat16)
    lse_l = torch.empty(HEADS, Sq, device="cuda")
    lse_r = torch.empty(HEADS, Sq, device="cuda")
    o_l = _run(nat, q, kv, segs[:1], lse_l)
    o_r = _run(nat, q, kv, segs[1:], lse_r)
    o = torch.empty_like(o_l)
    nat.attn_merge(o_l, lse_l, o_r, lse_r, o, Sq, HEADS, C)
    ref, _ = _ref_attention(q, kv, segs)
    e = rel_l2(o.float().cpu(), ref.cpu())
    print(f"\n[{total} keys, local + remote merged] rel-L2 {e:.2e}")
    assert e < 8e-3, e


class ReplicaComm:
    """Rank 0 of an 8-rank job whose other ranks hold copies of rank 0's K/V slot: the gathered buffer has the
    configs[4] shape and content of the right magnitude, so rank 0 does exactly its share of the work."""

    world, rank = 8, 0

    def allgather_slots(self, full, rows_per_slot):
        mine = full.narrow(0, 0, rows_per_slot)
        for r in range(1, self.world):
            full.narrow(0, r * rows_per_slot, rows_per_slot).copy_(mine)

    def allgather_slots_async(self, full, rows_per_slot):
        comm = self

        class _H:
            def wait(self_inner):
                comm.allgather_slots(full, rows_per_slot)

        return _H()

    def broadcast_(self, t, src=0):
        pass

    def gather_views(self, local, counts, dst):
        return local


def test_cfg5_rank_share_memory_efficient():
    """configs[4] per-rank load: 250 local views of a 2000-view 518^2 job, memory_efficient_inference=True,
    2 738 001 keys per global layer; outputs finite, shaped as the reference returns them, mask-consistent."""
    import time

    from mapanything.models import MapAnything
    from mapanything.parallel import ShardPlan
    from mapanything.utils import synthetic
    from tests_helpers import released_config

    V, H = 2000, 518
    plan = ShardPlan(V, 8, 0, 1369)
    assert plan.counts[0] == 250 and plan.total_kv == 2738001
    base = torch.from_numpy(synthetic.synthetic_images(1, H, H, seed=31)[0][0]).cuda()
    imgs = [base.roll(shifts=7 * i, dims=-1).unsqueeze(0) for i in range(8)]
    views = [{"img": imgs[i % 8], "data_norm_type": ["dinov2"]} for i in range(V)]
    model = MapAnything(**released_config()).load_synthetic_weights().to("cuda").eval()
    model.enable_view_sharding(comm=ReplicaComm())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = model.infer(views, memory_efficient_inference=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"\n[cfg5 rank-0 share] 250 local views of 2000, {dt:.1f} s")
    assert sum(o is not None for o in out) == 250 and all(o is not None for o in out[:250])
    for o in out[:250:31]:
        assert o["pts3d"].shape == (1, H, H, 3) and o["conf"].shape == (1, H, H)
        for k in ("pts3d", "pts3d_cam", "ray_directions", "depth_along_ray", "conf", "cam_trans", "cam_quats"):
            assert torch.isfinite(o[k]).all(), k
        assert torch.equal(o["non_ambiguous_mask"], torch.sigmoid(o["non_ambiguous_mask_logits"]) > 0.5)
        assert torch.all(o["mask"][..., 0] <= o["non_ambiguous_mask"])
        assert torch.allclose(o["ray_directions"].norm(dim=-1), torch.ones(1, device="cuda"), atol=1e-5)
    s = out[0]["metric_scaling_factor"]
    assert all(torch.equal(o["metric_scaling_factor"], s) for o in out[:250])
