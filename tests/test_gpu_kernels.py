"""Per-kernel parity of libmapa.so against PyTorch fp32 references of the same op (needs an MI355X)."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    from mapanything import _native

    _native.lib()
    return _native


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).cuda()


# ------------------------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 200, 264), (129, 130, 72), (1370, 1024, 1024),
                                   (37, 784, 784), (5, 7, 16)])
def test_gemm_plain(nat, dtype, M, N, K):
    A = _rand(M, K, seed=1).to(dtype)
    W = _rand(N, K, scale=K ** -0.5, seed=2).to(dtype)
    b = _rand(N, seed=3)
    out = torch.empty(M, N, device="cuda")
    nat.gemm(A, W, M, N, K, bias=b, out_f32=out)
    ref = A.float() @ W.float().t() + b
    tol = 1e-5 if dtype == torch.float32 else 1e-4
    assert rel_l2(out.cpu(), ref.cpu()) < tol


def test_gemm_epilogues(nat):
    M, N, K = 333, 384, 192
    A = _rand(M, K, seed=4).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=5).to(torch.bfloat16)
    b, g = _rand(N, seed=6), _rand(N, seed=7)
    r1, r2 = _rand(M, N, seed=8), _rand(M, N, seed=9)
    acc = A.float() @ W.float().t() + b
    # gelu -> bf16
    o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=o)
    assert rel_l2(o.float().cpu(), F.gelu(acc).cpu()) < 5e-3
    # resid1 + resid2 + gamma * relu(acc) -> f32 + relu copy
    of = torch.empty(M, N, device="cuda")
    orl = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nat.gemm(A, W, M, N, K, bias=b, gamma=g, act=nat.ACT_RELU, resid1=r1, resid2=r2, out_f32=of, out_lp_relu=orl)
    ref = r1 + r2 + g * torch.relu(acc)
    assert rel_l2(of.cpu(), ref.cpu()) < 1e-4
    assert rel_l2(orl.float().cpu(), torch.relu(ref).cpu()) < 5e-3
    # in-place residual (x = x + gamma * acc), the transformer-block pattern
    x = r1.clone()
    nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=x, out_f32=x)
    assert rel_l2(x.cpu(), (r1 + g * acc).cpu()) < 1e-4


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_gelu_epilogue_fp32_exactness(nat, dtype):
    """The GELU epilogue's erf (mapa_common.h erf_fast: <= 1.2 ulp of fp32 erff) against the exact-erf GELU of the
    SAME kernel's pre-activation (a second launch without the activation, so only the GELU evaluation differs):
    within a few fp32 ulp everywhere, including the negative tail and |x| > 4 (the 8-column epilogue path and its
    4-column tail: N = 200 is not a multiple of 8).  The round-2 Abramowitz-Stegun erf (5e-7 absolute) fails this
    in the tail, where GELU is ~1e-5 and that error is a few percent."""
    M, N, K = 513, 200, 64
    A = (_rand(M, K, seed=70) * 1.5).to(dtype)
    W = _rand(N, K, scale=K ** -0.5, seed=71).to(dtype)
    b = _rand(N, seed=72)
    out = torch.empty(M, N, device="cuda")
    pre = torch.empty(M, N, device="cuda")
    nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_f32=out)
    nat.gemm(A, W, M, N, K, bias=b, out_f32=pre)
    ref = F.gelu(pre.double())
    assert float(pre.abs().max()) > 4.0 and float(pre.min()) < -4.0  # the tails are exercised
    ulp = torch.finfo(torch.float32).eps * ref.abs().clamp_min(torch.finfo(torch.float32).tiny)
    err = (out.double() - ref).abs()
    # 0.5 * x * (1 + erf): a few ulp of the result from the products, plus 0.5|x| times the erf's error near +-1
    # (<= 1.2 ulp of 1 = 7e-8: the 1e-7 |x| term; in the negative tail 1 + erf cancels exactly, so that term is the
    # whole error there — the round-2 erf's 5e-7 would put 2.5e-7 |x| there and fail)
    assert bool((err <= 8 * ulp + 1e-7 * pre.abs().double()).all()), float((err / (ulp + 1e-30)).max())


@pytest.mark.parametrize("variant", [0, 2570, 2571, 2574])
def test_gemm_gelu_bf16_output(nat, variant):
    """The bf16-only GELU epilogue (epi_mode 1, the transformer fc1: mapa_common.h gelu_bf16out, a degree-9 fit of
    the normal tail, 3.2e-5 relative): every output within one bf16 rounding of torch's exact-erf GELU of the same
    kernel's fp32 pre-activation, and rounded differently from it in well under 1 % of the elements."""
    M, N, K = 2741, 3072, 768
    A = (_rand(M, K, seed=90) * 1.5).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=91).to(torch.bfloat16)
    b = _rand(N, seed=92)
    pre = torch.empty(M, N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(A, W, M, N, K, bias=b, out_f32=pre)
        nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=out)
        torch.cuda.synchronize()
    finally:
        nat.gemm_set_variant(0)
    # x * Phi(x) with an accurate tail (F.gelu's 0.5 x (1 + erf(x / sqrt 2)) cancels to -0 below x ~ -5.9 even in
    # fp64; the kernel keeps the true tail, e.g. GELU(-8.38) = -2.2e-16)
    xd = pre.double()
    ref = xd * 0.5 * torch.special.erfc(-xd * 0.7071067811865476)  # Phi(x) through erfc: no cancellation
    assert float(pre.abs().max()) > 4.0 and float(pre.min()) < -6.0  # the tail is exercised
    err = (out.double() - ref).abs()
    assert bool((err <= ref.abs() * 2.0 ** -8 + 1e-30).all()), float((err / ref.abs().clamp_min(1e-30)).max())
    flips = (out != ref.float().to(torch.bfloat16)).float().mean().item()
    assert flips < 5e-3, flips
    # against torch's own GELU: identical up to those tail values (absolute 1e-15) and rounding flips
    assert float((out.double() - F.gelu(xd)).abs().max()) <= float(F.gelu(xd).abs().max()) * 2.0 ** -8


@pytest.mark.parametrize("variant", [2580, 2581, 2582, 2571, 2568, 2572, 2573, 2574, 2587])
@pytest.mark.parametrize("M,N,K", [(10960, 1024, 4096), (10960, 768, 3072), (3000, 200, 264), (513, 136, 72),
                                   (3000, 200, 256), (10960, 3072, 1024), (700, 4100, 128)])
def test_gemm_big_and_streamk_variants(nat, variant, M, N, K):
    """Every 256-row schedule, incl. the stream-K ones (split tiles summed by the last arriver), on the path's
    narrow-N shapes, on more tiles than CUs and on ragged tails; stream-K must be bit-reproducible and leave its
    workspace tickets zeroed."""
    A = _rand(M, K, seed=21).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=22).to(torch.bfloat16)
    b, g, r = _rand(N, seed=23), _rand(N, seed=24), _rand(M, N, seed=25)
    ref = r + g * (A.float() @ W.float().t() + b)
    out = torch.empty(M, N, device="cuda")
    lp = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=r, out_f32=out, out_lp=lp)
        again = torch.empty_like(out)
        nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=r, out_f32=again)
        inplace = r.clone()  # the transformer's residual update: x += gamma * (A W^T + b), residual loaded ahead
        nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=inplace, out_f32=inplace)
        torch.cuda.synchronize()
    finally:
        nat.gemm_set_variant(0)
    assert rel_l2(out.cpu(), ref.cpu()) < 1e-4
    assert rel_l2(lp.float().cpu(), ref.cpu()) < 5e-3
    assert torch.equal(out, again)
    assert torch.equal(out, inplace)
    if 2580 <= variant <= 2582:  # tickets (the workspace head) back to zero for the next call
        ws = nat.gemm_workspace(0)
        assert ws.numel() > 0 and int(ws[: 4 * 65536].count_nonzero()) == 0


@pytest.mark.parametrize("variant", [0, 2600, 2601, 2602, 2603])
@pytest.mark.parametrize("M,N,K", [(10960, 3072, 1024), (10953, 768, 768), (3001, 200, 264), (513, 136, 72),
                                   (700, 4100, 128), (5, 12, 8)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm_persistent_register_epilogue(nat, variant, M, N, K, dtype):
    """The persistent register-epilogue kernel (gemm_pers.hip; 0 = the automatic choice, which takes it for these
    epilogues; 2600..2603 = each tile shape) on both transformer patterns — act(acc + bias) -> 16-bit (GELU and
    plain) and the in-place fp32 residual x += gamma * (acc + bias) — on ragged M / N / K, with more tiles than
    resident workgroups (several rounds) and fewer; deterministic, and bitwise equal to the data-parallel tile kernels
    (same MFMA products and K order, only the operand order and the store path differ)."""
    A = _rand(M, K, seed=31).to(dtype)
    W = _rand(N, K, scale=K ** -0.5, seed=32).to(dtype)
    b, g, r = _rand(N, seed=33), _rand(N, seed=34), _rand(M, N, seed=35)
    acc = A.float() @ W.float().t() + b
    outs = {}
    for tag, var, pers in (("pers", variant, 1), ("tiles", 0, 0)):
        nat.gemm_set_variant(var)
        nat.gemm_tune(nat.TUNE_PERS, pers)
        try:
            o = torch.empty(M, N, device="cuda", dtype=dtype)
            og = torch.empty(M, N, device="cuda", dtype=dtype)
            x = r.clone()
            nat.gemm(A, W, M, N, K, bias=b, out_lp=o)
            nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=og)
            nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=x, out_f32=x)
            og2 = torch.empty_like(og)
            nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=og2)
            torch.cuda.synchronize()
        finally:
            nat.gemm_set_variant(0)
            nat.gemm_tune(nat.TUNE_PERS, 1)
        outs[tag] = (o, og, x)
        assert torch.equal(og, og2)
    o, og, x = outs["pers"]
    assert rel_l2(o.float().cpu(), acc.cpu()) < 5e-3
    assert rel_l2(og.float().cpu(), F.gelu(acc).cpu()) < 5e-3
    assert rel_l2(x.cpu(), (r + g * acc).cpu()) < 1e-4
    # the plain and residual outputs bitwise; the GELU one bitwise where both use the bf16 GELU epilogue (the 128x128
    # kernels of small problems evaluate the fp32 erf form: rounding flips only)
    assert torch.equal(outs["pers"][0], outs["tiles"][0]) and torch.equal(outs["pers"][2], outs["tiles"][2])
    assert rel_l2(outs["pers"][1].float().cpu(), outs["tiles"][1].float().cpu()) < 5e-3
    if M >= 10000:  # the path shapes: both on the 16-bit GELU epilogue
        assert torch.equal(outs["pers"][1], outs["tiles"][1])


def _ln_flag(nat):
    """The library's device fault word (include/mapa.h fault channel): MAPA_FAULT_LN_BARRIER if a band barrier of a
    LayerNorm-fused launch gave up."""
    return nat.fault_status(reset=False)


# (M, N, K, gamma): the path's residual linears at 8 views (enc proj / fc2 on 192x256 tiles, aat proj / fc2 on
# 192x192), a one-band problem, a ragged last band, and B = 2 scenes (more tiles than CUs: fused only if the 192-row
# tile is still the automatic choice, else the library's GEMM + LayerNorm)
@pytest.mark.parametrize("M,N,K,gamma", [(10960, 1024, 1024, True), (10960, 1024, 4096, True), (10953, 768, 768, False),
                                         (10953, 768, 3072, False), (150, 768, 768, False), (4001, 1024, 1024, True),
                                         (21905, 768, 3072, False), (80001, 1024, 1024, True),
                                         (136901, 768, 768, False)])
@pytest.mark.parametrize("pers_ln", [0, 1, 2])
def test_gemm_layernorm_fused(nat, M, N, K, gamma, pers_ln):
    """mapa_gemm with ln_out (the next sub-block's LayerNorm fused into the residual linear): the fp32 residual
    stream bitwise equal to the plain GEMM's, the bf16 normalised rows within one bf16 rounding of the standalone
    two-pass LayerNorm of that stream (mapa_layernorm) and of torch's fp32 LayerNorm, repeatable bit for bit, and no
    band barrier timed out.  MAPA_TUNE_LN_FUSE=0 (GEMM, then LayerNorm) is the A side, 1 fuses only where the tile
    choice is the 192-row kernel, 2 (the default) whatever it is.  pers_ln = 1: the fused forms on the persistent
    register-epilogue kernel (MAPA_TUNE_PERS_LN; whole 192-row bands per round); 2: that form where K <= 1024, the
    LNF tiles above."""
    A = _rand(M, K, seed=61).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=62).to(torch.bfloat16)
    b = _rand(N, seed=63)
    g = _rand(N, scale=0.1, seed=64) if gamma else None
    x0 = _rand(M, N, seed=65) + 3.0 * _rand(1, N, seed=66)  # per-channel offsets, as the residual stream carries
    lw, lb = 1.0 + 0.2 * _rand(N, seed=67), 0.1 * _rand(N, seed=68)

    def run(fuse):
        nat.gemm_tune(nat.TUNE_LN_FUSE, fuse)
        nat.gemm_tune(nat.TUNE_PERS_LN, pers_ln)
        x = x0.clone()
        y = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=x, out_f32=x, ln=(lw, lb, 1e-6, y))
        torch.cuda.synchronize()
        return x, y
    try:
        xs, ys = run(0)
        xf, yf = run(1)
        xf2, yf2 = run(1)
        xa, ya = run(2)  # the default: the fused kernel whatever the tile choice (B = 2: more tiles than CUs)
    finally:
        nat.gemm_tune(nat.TUNE_LN_FUSE, 2)  # the default
        nat.gemm_tune(nat.TUNE_PERS_LN, 0)  # the default
    assert _ln_flag(nat) == 0
    assert torch.equal(xf, xs) and torch.equal(xf2, xf) and torch.equal(yf2, yf)
    assert not torch.isnan(yf.float()).any() and not torch.isnan(ya.float()).any()
    ref = F.layer_norm(xs, (N,), lw, lb, 1e-6)
    ulp = ref.abs().clamp_min(1e-3) * 2.0 ** -7  # one bf16 rounding (8 significant bits)
    for y in (ys, yf, ya):
        assert ((y.float() - ref).abs() <= ulp).all()
    for y in (yf, ya):
        diff = (y.float() != ys.float()).float().mean().item()
        assert diff < 1e-3, diff  # statistics rounded differently flip at most a few bf16 roundings
    assert rel_l2(xa.cpu(), xs.cpu()) < 1e-6  # another tile kernel for the residual when the choice differed


def test_gemm_layernorm_forms_interleave_in_one_workspace(nat):
    """MAPA_TUNE_PERS_LN = 2 alternates the persistent LayerNorm form (K <= 1024: the proj linears) with the LNF tiles
    (K = 4096: fc2) on one stream's workspace, as a transformer block does.  Both forms key their row statistics on the
    same 192-row bands and per-band generation words, so a granule left by one form never carries the epoch the other
    waits for: every call of an interleaved sequence equals the same call run alone, bit for bit."""
    M, N = 10960, 1024
    lw, lb = 1.0 + 0.2 * _rand(N, seed=91), 0.1 * _rand(N, seed=92)
    shapes = [1024, 4096, 1024, 4096, 1024]
    ops = []
    for i, K in enumerate(shapes):
        A = _rand(M, K, seed=100 + i).to(torch.bfloat16)
        W = _rand(N, K, scale=K ** -0.5, seed=200 + i).to(torch.bfloat16)
        ops.append((A, W, K, _rand(N, seed=300 + i), _rand(M, N, seed=400 + i)))

    def run(op):
        A, W, K, b, x0 = op
        x = x0.clone()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        nat.gemm(A, W, M, N, K, bias=b, resid1=x, out_f32=x, ln=(lw, lb, 1e-6, y))
        return x, y

    nat.gemm_tune(nat.TUNE_PERS_LN, 2)
    alone = []
    for op in ops:  # each call after a fresh call of the same shape only
        run(op)
        alone.append(run(op))
    torch.cuda.synchronize()
    for _ in range(2):
        seq = [run(op) for op in ops]
        torch.cuda.synchronize()
        for (xa, ya), (xs, ys) in zip(alone, seq):
            assert torch.equal(xa, xs) and torch.equal(ya, ys)
    nat.gemm_tune(nat.TUNE_PERS_LN, 0)  # the default
    assert _ln_flag(nat) == 0


@pytest.mark.parametrize("pers_ln", [0, 1, 2])
def test_gemm_layernorm_barrier_timeout_is_reported(nat, pers_ln):
    """A band that never completes (the test hook drops tile (0, 0)'s statistics publish; MAPA_TUNE_LN_SPIN shortens
    the bounded wait) must not hang and must not pass silently: the fault word carries MAPA_FAULT_LN_BARRIER, a
    FaultSlot published after the launch raises, check_faults raises and resets, and the next call is clean — its
    residual stream still bitwise the plain GEMM's, its LayerNorm rows identical to an undisturbed fused run."""
    M, N, K = 10953, 768, 768
    A = _rand(M, K, seed=81).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=82).to(torch.bfloat16)
    b, x0 = _rand(N, seed=83), _rand(M, N, seed=84)
    lw, lb = 1.0 + 0.2 * _rand(N, seed=85), 0.1 * _rand(N, seed=86)

    def run():
        x = x0.clone()
        y = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        nat.gemm(A, W, M, N, K, bias=b, resid1=x, out_f32=x, ln=(lw, lb, 1e-6, y))
        return x, y

    nat.gemm_tune(nat.TUNE_PERS_LN, pers_ln)
    assert nat.fault_status(reset=True) == 0
    x_ok, y_ok = run()
    slot = nat.FaultSlot()
    nat.gemm_tune(nat.TUNE_LN_SPIN, 4096)
    nat.gemm_tune(nat.TUNE_LN_TEST_SKIP, 1)
    try:
        slot.arm()
        x_bad, y_bad = run()
        slot.publish()
        with pytest.raises(nat.NativeError, match="LayerNorm"):
            slot.wait(timeout_s=60)
    finally:
        nat.gemm_tune(nat.TUNE_LN_SPIN, 0)
        nat.gemm_tune(nat.TUNE_LN_TEST_SKIP, 0)
    assert nat.fault_status(reset=False) == 0  # the slot's raise reset the word
    # the synchronous form reports it too
    nat.gemm_tune(nat.TUNE_LN_SPIN, 4096)
    nat.gemm_tune(nat.TUNE_LN_TEST_SKIP, 1)
    try:
        run()
        torch.cuda.synchronize()
    finally:
        nat.gemm_tune(nat.TUNE_LN_SPIN, 0)
        nat.gemm_tune(nat.TUNE_LN_TEST_SKIP, 0)
    assert nat.fault_status(reset=False) & nat.FAULT_LN_BARRIER
    with pytest.raises(nat.NativeError, match="LayerNorm"):
        nat.check_faults()
    assert nat.fault_status(reset=False) == 0
    assert torch.equal(x_bad, x_ok)  # the residual stream never depends on the barrier
    assert torch.equal(y_bad[192:], y_ok[192:])  # only band 0's normalised rows are invalid
    x2, y2 = run()
    torch.cuda.synchronize()
    nat.gemm_tune(nat.TUNE_PERS_LN, 0)  # the default
    assert nat.fault_status(reset=False) == 0
    assert torch.equal(x2, x_ok) and torch.equal(y2, y_ok)


def test_fault_words_are_per_thread(nat):
    """Two host threads, each on its own stream (the in-thread sharded ranks, a server with a model per stream):
    thread A raises MAPA_FAULT_LN_BARRIER (the test hook) and stops before its publish; thread B then starts a call —
    reset, clean work, publish — on its own word.  B's publish is clean and B's reset does not clear A's fault, which
    A's publish still carries (with one shared word a concurrent caller's per-call reset dropped another caller's
    fault: a range fault lost that way left the TF32-equivalent heads' overflow in the outputs)."""
    import threading

    M, N, K = 10953, 768, 768
    A = _rand(M, K, seed=91).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=92).to(torch.bfloat16)
    b, x0 = _rand(N, seed=93), _rand(M, N, seed=94)
    lw, lb = 1.0 + 0.2 * _rand(N, seed=95), 0.1 * _rand(N, seed=96)
    bar, res, errs = threading.Barrier(2, timeout=120), {}, []

    def outcome(slot):
        try:
            slot.wait(timeout_s=60)
            return "clean"
        except nat.NativeError as e:
            return str(e)

    def thread_a():
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                nat.fault_status(reset=True)
                slot = nat.FaultSlot()
                slot.arm()
                x = x0.clone()
                y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                nat.gemm_tune(nat.TUNE_LN_SPIN, 4096)
                nat.gemm_tune(nat.TUNE_LN_TEST_SKIP, 1)
                try:
                    nat.gemm(A, W, M, N, K, bias=b, resid1=x, out_f32=x, ln=(lw, lb, 1e-6, y))
                    s.synchronize()  # the fault is in A's word now
                finally:
                    nat.gemm_tune(nat.TUNE_LN_SPIN, 0)
                    nat.gemm_tune(nat.TUNE_LN_TEST_SKIP, 0)
                bar.wait()  # B runs its whole call
                bar.wait()
                slot.publish()
                res["a"] = outcome(slot)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            bar.abort()

    def thread_b():
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                bar.wait()
                slot = nat.FaultSlot()
                slot.arm()
                nat.FaultSlot.reset()
                o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                nat.gemm(A, W, M, N, K, bias=b, out_lp=o)
                slot.publish()
                res["b"] = outcome(slot)
                bar.wait()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            bar.abort()

    th = [threading.Thread(target=thread_a), threading.Thread(target=thread_b)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    torch.cuda.synchronize()
    assert not errs, errs
    assert res["b"] == "clean", res
    assert "LayerNorm" in res["a"], res
    assert nat.fault_status(reset=False) == 0  # this thread's word saw neither


@pytest.mark.parametrize("variant", [2580, 2581, 2582, 2572, 2573, 2574])
def test_conv3x3_big_variants(nat, variant):
    n, H, W, C, Co = 2, 37, 37, 256, 256
    x = _rand(n, C, H, W, seed=26).to(torch.bfloat16)
    w = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=27).to(torch.bfloat16)
    ref = F.conv2d(x.float(), w.float(), None, padding=1)
    out = torch.empty(n * H * W, Co, device="cuda")
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(x.permute(0, 2, 3, 1).contiguous(), w.permute(0, 2, 3, 1).reshape(Co, -1).contiguous(), n * H * W,
                 Co, 9 * C, out_f32=out, conv=(C, H, W, H, W, 1))
    finally:
        nat.gemm_set_variant(0)
    assert rel_l2(out.view(n, H, W, Co).permute(0, 3, 1, 2).cpu(), ref.cpu()) < 1e-4


@pytest.mark.parametrize("variant,dtype", [(0, torch.bfloat16), (0, torch.float32), (2568, torch.bfloat16),
                                           (2571, torch.bfloat16), (2580, torch.bfloat16)])
@pytest.mark.parametrize("n,H,W,C,Co,stride", [(2, 37, 37, 96, 256, 1), (1, 19, 19, 768, 128, 2)])
def test_conv3x3_channel_block_k_order(nat, variant, dtype, n, H, W, C, Co, stride):
    """conv_kblock = 32: the K index walks the 9 taps of each 32-channel slice (weights packed [out][C/32][tap][32])
    and gives the conv of the tap-major packing, for every tile schedule."""
    x = _rand(n, C, H, W, seed=40)
    w = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=41)
    b = _rand(Co, seed=42)
    xl, wl = x.to(dtype), w.to(dtype)
    ref = F.conv2d(xl.float(), wl.float(), b, stride=stride, padding=1)
    OH, OW = ref.shape[-2:]
    x_nhwc = xl.permute(0, 2, 3, 1).contiguous()
    wkb = wl.permute(0, 2, 3, 1).reshape(Co, 9, C // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
    wkb._mapa_kblock = 32
    out = torch.empty(n * OH * OW, Co, device="cuda")
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(x_nhwc, wkb, n * OH * OW, Co, 9 * C, bias=b, out_f32=out, conv=(C, H, W, OH, OW, stride))
        torch.cuda.synchronize()
    finally:
        nat.gemm_set_variant(0)
    got = out.view(n, OH, OW, Co).permute(0, 3, 1, 2)
    assert rel_l2(got.cpu(), ref.cpu()) < (1e-5 if dtype == torch.float32 else 1e-4)


@pytest.mark.parametrize("variant", [2584, 2586, 2588])
@pytest.mark.parametrize("n,H,W,C,Co", [(2, 37, 29, 96, 256), (1, 50, 48, 256, 128), (3, 16, 16, 32, 256),
                                        (1, 148, 148, 256, 256), (2, 13, 21, 64, 256)])
def test_conv3x3_halo_window(nat, variant, n, H, W, C, Co):
    """The LDS halo-window conv (16x16-pixel blocks, 18x18 window per 32-channel slice, the 9 taps read at shifted
    window addresses; 2588: 8x16 blocks, 10x18 windows, 256-wide tiles): ragged blocks at the image edges, zero
    padding, fused epilogue (bias, ReLU, residual, bf16 + fp32 + split outputs), both tile widths."""
    if variant == 2588 and Co % 256:
        pytest.skip("8-row blocks come with 256-wide tiles")
    x = _rand(n, C, H, W, seed=50)
    w = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=51)
    b, r = _rand(Co, seed=52), _rand(n * H * W, Co, seed=53)
    xl, wl = x.to(torch.bfloat16), w.to(torch.bfloat16)
    ref = F.conv2d(xl.float(), wl.float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    ref = r + torch.relu(ref)
    x_nhwc = xl.permute(0, 2, 3, 1).contiguous()
    wkb = wl.permute(0, 2, 3, 1).reshape(Co, 9, C // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
    wkb._mapa_kblock = 32
    M = n * H * W
    out = torch.empty(M, Co, device="cuda")
    lp = torch.empty(M, Co, device="cuda", dtype=torch.bfloat16)
    s3 = torch.empty(M, 2 * Co, device="cuda", dtype=torch.bfloat16)
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(x_nhwc, wkb, M, Co, 9 * C, bias=b, act=nat.ACT_RELU, resid1=r, out_f32=out, out_lp=lp, out_s3=s3,
                 conv=(C, H, W, H, W, 1))
        again = torch.empty_like(out)
        nat.gemm(x_nhwc, wkb, M, Co, 9 * C, bias=b, act=nat.ACT_RELU, resid1=r, out_f32=again,
                 conv=(C, H, W, H, W, 1))
        torch.cuda.synchronize()
    finally:
        nat.gemm_set_variant(0)
    assert rel_l2(out.cpu(), ref.cpu()) < 1e-4
    assert rel_l2(lp.float().cpu(), ref.cpu()) < 5e-3
    assert torch.equal(s3, _split_expect(out))
    assert torch.equal(out, again)


@pytest.mark.parametrize("split", [0, 1, 2, 3, 7])
@pytest.mark.parametrize("n,H,W,C,Co", [(2, 37, 37, 256, 256), (1, 19, 19, 96, 128), (2, 37, 29, 64, 256),
                                        (3, 13, 21, 32, 128), (1, 61, 61, 64, 128), (2, 5, 7, 32, 128)])
def test_conv3x3_halo_flat_split(nat, split, n, H, W, C, Co):
    """The halo conv on flat-raster blocks (256 consecutive positions of the images' raster with one zero column per
    row and one zero row per image; 1-D window of 256 + 2(W+1) + 2 positions) with the 32-channel slices split over
    `split` workgroups per tile (0 = automatic; the parts meet in fp32 slabs, summed in part order by the last
    arriver): every epilogue output, blocks straddling rows and images, maps up to 61 pixels wide, bitwise repeatable,
    tickets back to zero."""
    x = _rand(n, C, H, W, seed=56)
    w = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=57)
    b, r = _rand(Co, seed=58), _rand(n * H * W, Co, seed=59)
    xl, wl = x.to(torch.bfloat16), w.to(torch.bfloat16)
    ref = F.conv2d(xl.float(), wl.float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    ref = r + torch.relu(ref)
    x_nhwc = xl.permute(0, 2, 3, 1).contiguous()
    wkb = wl.permute(0, 2, 3, 1).reshape(Co, 9, C // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
    wkb._mapa_kblock = 32
    M = n * H * W
    out = torch.full((M, Co), float("nan"), device="cuda")
    lp = torch.empty(M, Co, device="cuda", dtype=torch.bfloat16)
    s3 = torch.empty(M, 2 * Co, device="cuda", dtype=torch.bfloat16)
    nat.gemm_set_variant(2589)
    nat.gemm_tune(nat.TUNE_HALO_SPLIT, split)
    try:
        nat.gemm(x_nhwc, wkb, M, Co, 9 * C, bias=b, act=nat.ACT_RELU, resid1=r, out_f32=out, out_lp=lp, out_s3=s3,
                 conv=(C, H, W, H, W, 1))
        again = torch.empty_like(out)
        nat.gemm(x_nhwc, wkb, M, Co, 9 * C, bias=b, act=nat.ACT_RELU, resid1=r, out_f32=again,
                 conv=(C, H, W, H, W, 1))
        torch.cuda.synchronize()
    finally:
        nat.gemm_set_variant(0)
        nat.gemm_tune(nat.TUNE_HALO_SPLIT, 0)
    assert rel_l2(out.cpu(), ref.cpu()) < 1e-4
    assert rel_l2(lp.float().cpu(), ref.cpu()) < 5e-3
    assert torch.equal(s3, _split_expect(out))
    assert torch.equal(out, again)
    ws = nat.gemm_workspace(0)
    assert int(ws[: 4 * (65536 - 16384)].count_nonzero()) == 0  # the ticket words (the top 64 KiB: LN generations)


def test_split_precision_conv_halo_flat(nat):
    """Split-precision activations through the flat-raster split-K halo conv at the DPT's 37^2 (automatic choice:
    no forced variant) stay within ~1e-5 of the fp64 conv."""
    n, h, w, C, Co = 3, 37, 37, 256, 256
    x = _rand(n, C, h, w, seed=60)
    wt = _rand(Co, C, 3, 3, scale=C ** -0.5 / 3, seed=61)
    ref = F.conv2d(x.cpu().double(), wt.cpu().double(), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    M = n * h * w
    xr = x.permute(0, 2, 3, 1).reshape(M, C).contiguous()
    a = torch.empty(M, 2 * C, dtype=torch.bfloat16, device="cuda")
    nat.split_bf16x3(xr, M, C, C, a)
    wk = wt.permute(0, 2, 3, 1).reshape(Co, 9, C)
    whi = wk.to(torch.bfloat16)
    wlo = (wk - whi.float()).to(torch.bfloat16)
    wp = torch.stack([whi, wlo, whi], 2).reshape(Co, 9, 3 * C)
    wp = wp.reshape(Co, 9, 3 * C // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
    wp._mapa_split = True
    wp._mapa_kblock = 32
    out = torch.empty(M, Co, device="cuda")
    nat.gemm(a, wp, M, Co, 9 * 3 * C, out_f32=out, conv=(3 * C, h, w, h, w, 1))
    assert rel_l2(out.cpu(), ref) < 2e-5


def test_split_precision_conv_halo_window(nat):
    """Split-precision activations ([hi | lo] stored, [hi | hi | lo] logical, 32-channel slices mapped per slice)
    through the halo-window conv stay within ~1e-5 of the fp64 conv."""
    n, h, w, C, Co = 2, 37, 37, 256, 256
    x = _rand(n, C, h, w, seed=54)
    wt = _rand(Co, C, 3, 3, scale=C ** -0.5 / 3, seed=55)
    ref = F.conv2d(x.cpu().double(), wt.cpu().double(), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    M = n * h * w
    xr = x.permute(0, 2, 3, 1).reshape(M, C).contiguous()
    a = torch.empty(M, 2 * C, dtype=torch.bfloat16, device="cuda")
    nat.split_bf16x3(xr, M, C, C, a)
    wk = wt.permute(0, 2, 3, 1).reshape(Co, 9, C)
    whi = wk.to(torch.bfloat16)
    wlo = (wk - whi.float()).to(torch.bfloat16)
    wp = torch.stack([whi, wlo, whi], 2).reshape(Co, 9, 3 * C)  # [out][tap][hi | lo | hi]
    wp = wp.reshape(Co, 9, 3 * C // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
    wp._mapa_split = True
    wp._mapa_kblock = 32
    out = torch.empty(M, Co, device="cuda")
    nat.gemm_set_variant(2584)
    try:
        nat.gemm(a, wp, M, Co, 9 * 3 * C, out_f32=out, conv=(3 * C, h, w, h, w, 1))
    finally:
        nat.gemm_set_variant(0)
    assert rel_l2(out.cpu(), ref) < 2e-5


def test_regressor_head_out_repeatable(nat):
    """The fused regressor head is bit-for-bit repeatable launch to launch (tools/ho_det.py: with -O3 SLP packing of
    dense_head_pixel into v_pk_*_f32, one 16-lane row per wave of the pts3d y components came out different from
    launch to launch on MI355X; conv_halo.o is built with -fno-slp-vectorize)."""
    n, H, W, C = 2, 518, 518, 128
    M = n * H * W
    xr = _rand(M, C, seed=70).relu()
    wk = _rand(C, 9, C, scale=(9 * C) ** -0.5, seed=71)
    b2, w6, b6 = _rand(C, seed=72), _rand(6, C, scale=C ** -0.5, seed=73), _rand(6, seed=74)
    a = torch.empty(M, 2 * C, dtype=torch.bfloat16, device="cuda")
    nat.split_bf16x3(xr, M, C, C, a)
    whi = wk.to(torch.bfloat16)
    wlo = (wk - whi.float()).to(torch.bfloat16)
    wp = torch.stack([whi, wlo, whi], 2).reshape(C, 9, 3 * C).reshape(C, 9, 12, 32).permute(0, 2, 1, 3)
    wp = wp.contiguous().reshape(C, -1)
    wp._mapa_split = True
    wp._mapa_kblock = 32
    pose_out, scale = torch.empty(n, 19, device="cuda"), torch.empty(1, device="cuda")
    nat.pose_scale_finalize(_rand(n, 7, seed=75), _rand(1, seed=76), n, 1, pose_out, scale,
                            torch.empty(n, 4, 4, device="cuda"))

    def run():
        o = [torch.empty((n, H, W, 3), device="cuda") for _ in range(3)] + [torch.empty((n, H, W, 1), device="cuda")] + \
            [torch.empty((n, H, W), device="cuda") for _ in range(2)] + \
            [torch.empty((n, H, W), dtype=torch.uint8, device="cuda")]
        nat.gemm(a, wp, M, C, 9 * 3 * C, bias=b2, act=nat.ACT_RELU, conv=(3 * C, H, W, H, W, 1),
                 head_out=(w6, b6, pose_out, scale, n, *o))
        return o
    first = run()
    for _ in range(6):
        for x, y in zip(first, run()):
            assert torch.equal(x, y)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("n,H,W", [(2, 37, 29), (1, 48, 64), (3, 16, 16)])
def test_regressor_head_out_fused(nat, split, n, H, W):
    """mapa_regressor_head_out (regressor conv2 + ReLU + 1x1 128->6 + dense head in one launch) against the two-launch
    path with an fp32 hidden map (conv out_f32 + mapa_dense_head_out): same fp32 math, other summation order; the
    mask may differ only where the logit is ~0."""
    C = 128
    x = _rand(n, C, H, W, seed=60)
    wt = _rand(C, C, 3, 3, scale=(9 * C) ** -0.5, seed=61)
    b2, w6, b6 = _rand(C, seed=62), _rand(6, C, scale=C ** -0.5, seed=63), _rand(6, seed=64)
    M = n * H * W
    xr = x.permute(0, 2, 3, 1).reshape(M, C).contiguous()
    wk = wt.permute(0, 2, 3, 1).reshape(C, 9, C)
    if split:
        a = torch.empty(M, 2 * C, dtype=torch.bfloat16, device="cuda")
        nat.split_bf16x3(xr, M, C, C, a)
        whi = wk.to(torch.bfloat16)
        wlo = (wk - whi.float()).to(torch.bfloat16)
        wp = torch.stack([whi, wlo, whi], 2).reshape(C, 9, 3 * C)
        Cl = 3 * C
    else:
        a, wp, Cl = xr.to(torch.bfloat16), wk.to(torch.bfloat16), C
    wp = wp.reshape(C, 9, Cl // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(C, -1)
    wp._mapa_split = split
    wp._mapa_kblock = 32
    pose_out = torch.empty(n, 19, device="cuda")
    scale = torch.empty(1, device="cuda")
    nat.pose_scale_finalize(_rand(n, 7, seed=65), _rand(1, seed=66), n, 1, pose_out, scale,
                            torch.empty(n, 4, 4, device="cuda"))

    def outs():
        f = dict(device="cuda")
        return [torch.full((n, H, W, 3), float("nan"), **f) for _ in range(3)] + \
            [torch.full((n, H, W, 1), float("nan"), **f)] + [torch.full((n, H, W), float("nan"), **f) for _ in range(2)] + \
            [torch.full((n, H, W), 7, dtype=torch.uint8, device="cuda")]

    conv = (Cl, H, W, H, W, 1)
    hid = torch.empty(M, C, device="cuda")
    nat.gemm(a, wp, M, C, 9 * Cl, bias=b2, act=nat.ACT_RELU, out_f32=hid, conv=conv)
    ref = outs()
    nat.dense_head_out(hid, n, H * W, w6, b6, pose_out, scale, 1, *ref)
    got = outs()
    nat.gemm(a, wp, M, C, 9 * Cl, bias=b2, act=nat.ACT_RELU, conv=conv, head_out=(w6, b6, pose_out, scale, n, *got))
    torch.cuda.synchronize()
    for r, g in zip(ref[:6], got[:6]):
        assert torch.isfinite(g).all()
        assert rel_l2(g.cpu(), r.cpu()) < 1e-5
    # one metric scale per image (batched scenes, views_per_scale = 1) against the unfused head with batch = n
    scales = torch.rand(n, device="cuda") + 0.5
    ref_b, got_b = outs(), outs()
    nat.dense_head_out(hid, n, H * W, w6, b6, pose_out, scales, n, *ref_b)
    nat.gemm(a, wp, M, C, 9 * Cl, bias=b2, act=nat.ACT_RELU, conv=conv, head_out=(w6, b6, pose_out, scales, 1, *got_b))
    torch.cuda.synchronize()
    for r, g in zip(ref_b[:6], got_b[:6]):
        assert rel_l2(g.cpu(), r.cpu()) < 1e-5
    logits = ref[5].cpu()
    decided = logits.abs() > 1e-4
    assert torch.equal(got[6].cpu()[decided], ref[6].cpu()[decided])
    assert int(got[6].cpu().gt(1).sum()) == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,H,W,C,Co,stride", [(2, 19, 19, 96, 256, 1), (1, 37, 37, 768, 768, 2),
                                              (3, 16, 20, 128, 128, 1), (1, 8, 8, 256, 6, 1)])
def test_conv3x3_implicit_gemm(nat, dtype, n, H, W, C, Co, stride):
    x = _rand(n, C, H, W, seed=10)
    w = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=11)
    b = _rand(Co, seed=12)
    xl, wl = x.to(dtype), w.to(dtype)
    ref = F.conv2d(xl.float(), wl.float(), b, stride=stride, padding=1)
    OH, OW = ref.shape[-2:]
    x_nhwc = xl.permute(0, 2, 3, 1).contiguous()
    wmat = wl.permute(0, 2, 3, 1).reshape(Co, -1).contiguous()
    out = torch.empty(n * OH * OW, Co, device="cuda")
    nat.gemm(x_nhwc, wmat, n * OH * OW, Co, 9 * C, bias=b, out_f32=out, conv=(C, H, W, OH, OW, stride))
    got = out.view(n, OH, OW, Co).permute(0, 3, 1, 2)
    tol = 1e-5 if dtype == torch.float32 else 1e-4
    assert rel_l2(got.cpu(), ref.cpu()) < tol


@pytest.mark.parametrize("s,ci,co", [(4, 96, 96), (2, 192, 192)])
def test_convtranspose_pixel_shuffle(nat, s, ci, co):
    n, h, w = 2, 7, 9
    x = _rand(n, ci, h, w, seed=13).to(torch.bfloat16)
    wt = _rand(ci, co, s, s, scale=ci ** -0.5, seed=14).to(torch.bfloat16)
    b = _rand(co, seed=15)
    ref = F.conv_transpose2d(x.float(), wt.float(), b, stride=s)
    A = x.permute(0, 2, 3, 1).reshape(n * h * w, ci).contiguous()
    Wm = wt.permute(2, 3, 1, 0).reshape(s * s * co, ci).contiguous()
    out = torch.empty(n, h * s, w * s, co, device="cuda")
    nat.gemm(A, Wm, n * h * w, s * s * co, ci, bias=b, bias_mod=co, out_f32=out, pixshuf=(s, h, w, co))
    assert rel_l2(out.permute(0, 3, 1, 2).cpu(), ref.cpu()) < 1e-4


# ------------------------------------------------------------------------------------------------- attention
def _sdpa_ref(q, k, v):
    return F.scaled_dot_product_attention(q.float(), k.float(), v.float())


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 8e-3), (torch.float32, 2e-5)])
@pytest.mark.parametrize("B,Hh,S", [(2, 16, 1370), (3, 12, 1369), (1, 12, 200), (1, 2, 64), (1, 1, 1), (2, 3, 65)])
def test_attention_packed_qkv(nat, dtype, tol, B, Hh, S):
    C = Hh * 64
    qkv = _rand(B * S, 3 * C, seed=16).to(dtype)
    o = torch.empty(B * S, C, device="cuda", dtype=dtype)
    rs = 3 * C
    nat.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B, heads=Hh, seq_q=S, seq_kv=S, q_bstride=S * rs,
                  q_rstride=rs, k_bstride=S * rs, k_rstride=rs, v_bstride=S * rs, v_rstride=rs, o_bstride=S * C,
                  o_rstride=C)
    t = qkv.view(B, S, 3, Hh, 64).permute(2, 0, 3, 1, 4)
    ref = _sdpa_ref(t[0], t[1], t[2]).transpose(1, 2).reshape(B * S, C)
    assert rel_l2(o.float().cpu(), ref.cpu()) < tol


def test_attention_cross_lengths_and_lse(nat):
    """Q rows attend to a different-length K/V set (the sharded global layer) + LSE output."""
    Hh, Sq, Skv = 12, 300, 1111
    q = _rand(Sq, Hh * 64, seed=17).to(torch.bfloat16)
    kv = _rand(Skv, 2 * Hh * 64, seed=18).to(torch.bfloat16)
    o = torch.empty(Sq, Hh * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(1, Hh, Sq, device="cuda")
    C = Hh * 64
    nat.attention(q, kv, kv[:, C:], o, batch=1, heads=Hh, seq_q=Sq, seq_kv=Skv, q_bstride=0, q_rstride=C,
                  k_bstride=0, k_rstride=2 * C, v_bstride=0, v_rstride=2 * C, o_bstride=0, o_rstride=C, lse=lse)
    qh = q.view(Sq, Hh, 64).transpose(0, 1)[None]
    kh = kv[:, :C].reshape(Skv, Hh, 64).transpose(0, 1)[None]
    vh = kv[:, C:].reshape(Skv, Hh, 64).transpose(0, 1)[None]
    ref = _sdpa_ref(qh, kh, vh)[0].transpose(0, 1).reshape(Sq, C)
    assert rel_l2(o.float().cpu(), ref.cpu()) < 8e-3
    s = (qh.float() @ kh.float().transpose(-1, -2)) / 8.0
    assert rel_l2(lse.cpu(), torch.logsumexp(s, -1).cpu()) < 1e-4


def test_attention_softmax_rescale_branch(nat):
    """A key block late in the sweep carries a spiked score so the running max jumps (rule 26)."""
    Hh, S = 1, 1024
    qkv = _rand(S, 3 * 64, scale=0.5, seed=19)
    qkv[:, 64:128][900] *= 40.0
    qkv = qkv.to(torch.bfloat16)
    o = torch.empty(S, 64, device="cuda", dtype=torch.bfloat16)
    nat.attention(qkv, qkv[:, 64:], qkv[:, 128:], o, batch=1, heads=1, seq_q=S, seq_kv=S, q_bstride=0, q_rstride=192,
                  k_bstride=0, k_rstride=192, v_bstride=0, v_rstride=192, o_bstride=0, o_rstride=64)
    t = qkv.view(1, S, 3, 1, 64).permute(2, 0, 3, 1, 4)
    ref = _sdpa_ref(t[0], t[1], t[2])[0, 0]
    assert rel_l2(o.float().cpu(), ref.cpu()) < 8e-3


@pytest.mark.parametrize("trend", [1.0, -1.0])
def test_attention_score_drift_past_exp2_range(nat, trend):
    """Scores drift by ~±600 (log2 units) along the keys: with a growing drift every later tile exceeds the
    first tile's max by far more than exp2's range, so the reference-max softmax must rebase (repeatedly);
    with a falling drift everything after the first tiles underflows to 0, exactly as in fp32."""
    Hh, S = 2, 1000
    q = _rand(S, Hh * 64, scale=0.2, seed=40)
    q[:, 0::64] = 4.0  # a constant component so that score ~ 4 * k[:, 0] / 8 for every query
    k = _rand(S, Hh * 64, scale=0.2, seed=41)
    drift = trend * torch.linspace(-300.0, 300.0, S, device="cuda")
    k[:, 0::64] = drift[:, None] * 2.0 * 0.6931471805599453  # score = k0 / 2 (natural log) = drift (log2)
    v = _rand(S, Hh * 64, seed=42)
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    o = torch.empty(S, Hh * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(1, Hh, S, device="cuda")
    C = Hh * 64
    nat.attention(q, k, v, o, batch=1, heads=Hh, seq_q=S, seq_kv=S, q_bstride=0, q_rstride=C, k_bstride=0,
                  k_rstride=C, v_bstride=0, v_rstride=C, o_bstride=0, o_rstride=C, lse=lse)
    qh, kh, vh = (t.view(S, Hh, 64).transpose(0, 1)[None] for t in (q, k, v))
    ref = _sdpa_ref(qh, kh, vh)[0].transpose(0, 1).reshape(S, C)
    assert torch.isfinite(o.float()).all()
    assert rel_l2(o.float().cpu(), ref.cpu()) < 8e-3
    # the kernel's scores are bf16(q * log2(e) / 8) . k in the log2 domain (one documented bf16 rounding of the
    # scaled Q, ~2^-9 relative per score); at |score| ~ 200 that alone moves the LSE by ~0.4, so the LSE is held
    # to the log2-domain reference of those same scores
    log2e = 1.4426950408889634
    s2 = (qh.float() * (log2e / 8.0)).to(torch.bfloat16).float() @ kh.float().transpose(-1, -2)
    assert rel_l2(lse.cpu(), (torch.logsumexp(s2 / log2e, -1)).cpu()) < 1e-5


@pytest.mark.parametrize("segs", [[(0, 100), (300, 37), (500, 200), (800, 64)], [(64, 128), (0, 64), (700, 1)]])
def test_attention_kv_segments(nat, segs):
    """Logical keys = concatenation of physical K/V row ranges (the sharded layer's slot table); segment
    boundaries both on and off the 64-key tile grid."""
    Hh, Sq = 3, 150
    C = Hh * 64
    kv = _rand(1024, 2 * C, seed=43).to(torch.bfloat16)
    q = _rand(Sq, C, seed=44).to(torch.bfloat16)
    o = torch.empty(Sq, C, device="cuda", dtype=torch.bfloat16)
    skv = sum(n for _, n in segs)
    nat.attention(q, kv, kv[:, C:], o, batch=1, heads=Hh, seq_q=Sq, seq_kv=skv, q_bstride=0, q_rstride=C,
                  k_bstride=0, k_rstride=2 * C, v_bstride=0, v_rstride=2 * C, o_bstride=0, o_rstride=C,
                  kv_segments=segs)
    rows = torch.cat([torch.arange(s0, s0 + n) for s0, n in segs]).cuda()
    kvl = kv[rows]
    qh = q.view(Sq, Hh, 64).transpose(0, 1)[None]
    kh = kvl[:, :C].reshape(skv, Hh, 64).transpose(0, 1)[None]
    vh = kvl[:, C:].reshape(skv, Hh, 64).transpose(0, 1)[None]
    ref = _sdpa_ref(qh, kh, vh)[0].transpose(0, 1).reshape(Sq, C)
    assert rel_l2(o.float().cpu(), ref.cpu()) < 8e-3


# ----------------------------------------------------------------------------------------------- others
@pytest.mark.parametrize("dim", [768, 1024])
def test_layernorm(nat, dim):
    rows = 517
    x = _rand(rows + 7, dim, scale=3.0, seed=20) + 1.5
    w, b = _rand(dim, seed=21), _rand(dim, seed=22)
    yf = torch.empty(rows, dim, device="cuda")
    yl = torch.empty(rows, dim, device="cuda", dtype=torch.bfloat16)
    nat.layernorm(x, rows, dim, w, b, y_f32=yf, y_lp=yl)
    ref = F.layer_norm(x[:rows], (dim,), w, b, 1e-6)
    assert rel_l2(yf.cpu(), ref.cpu()) < 1e-6
    assert rel_l2(yl.float().cpu(), ref.cpu()) < 5e-3
    # grouped rows: drop the first row of every group of T+1 (DINOv2 cls)
    T = 10
    yg = torch.empty(30, dim, device="cuda")
    nat.layernorm(x, 30, dim, w, b, y_f32=yg, group=T, group_stride=T + 1, row_off=1)
    idx = torch.tensor([g * (T + 1) + 1 + t for g in range(3) for t in range(T)])
    assert rel_l2(yg.cpu(), F.layer_norm(x[idx], (dim,), w, b, 1e-6).cpu()) < 1e-6


@pytest.mark.parametrize("n,IH,IW,OHf,OWf,OH,OW", [(2, 19, 19, 38, 38, 37, 37), (2, 37, 37, 74, 74, 74, 74),
                                                   (2, 296, 296, 518, 518, 518, 518), (2, 16, 16, 224, 224, 224, 224),
                                                   (1, 19, 19, 38, 38, 37, 37), (3, 7, 5, 13, 9, 13, 9)])
def test_bilinear_align_corners(nat, n, IH, IW, OHf, OWf, OH, OW):
    """Row pairs share source rows (odd row counts, pairs straddling two images included)."""
    C = 128
    x = _rand(n, C, IH, IW, seed=23)
    ref = F.interpolate(x, size=(OHf, OWf), mode="bilinear", align_corners=True)[:, :, :OH, :OW]
    out = torch.empty(n, OH, OW, C, device="cuda")
    nat.bilinear_ac(x.permute(0, 2, 3, 1).contiguous(), n, IH, IW, C, OHf, OWf, OH, OW, out)
    assert rel_l2(out.permute(0, 3, 1, 2).cpu(), ref.cpu()) < 3e-5  # fp32 op-order vs ATen GPU kernel


def test_splitmix_fill_matches_numpy(nat):
    from mapanything.utils.synthetic import GLOBAL_SEED, fnv1a64, named_uniform

    name = "encoder.model.blocks.3.mlp.fc1.weight"
    ref = named_uniform(name, (4096, 1024), -0.054, 0.054)
    out = torch.empty(4096 * 1024, device="cuda")
    half = np.float32(0.054)
    nat.fill_splitmix(out, fnv1a64(name) ^ GLOBAL_SEED, float(half), 0.0)
    assert np.array_equal(out.cpu().numpy().reshape(4096, 1024), ref)


def test_patchify_and_tokens(nat):
    n, H, W = 2, 56, 70
    img = _rand(n, 3, H, W, seed=24)
    out = torch.empty(n * (H // 14) * (W // 14), 640, device="cuda")
    nat.patchify(img, n, H, W, out, 640)
    ref = F.unfold(img, 14, stride=14).transpose(1, 2).reshape(-1, 588)
    assert torch.equal(out[:, :588].cpu(), ref.cpu())
    assert torch.count_nonzero(out[:, 588:]).item() == 0


# ------------------------------------------------------------------------------------------ geometric inputs
def test_gemm_gelu_after_residual(nat):
    """ResidualBlock tail (dense_rep_encoder.py:44-52): gelu(conv2(x) + b + identity)."""
    M, N, K = 300, 96, 128
    A, W, b, r = _rand(M, K, seed=21), _rand(N, K, scale=K ** -0.5, seed=22), _rand(N, seed=23), _rand(M, N, seed=24)
    out = torch.empty(M, N, device="cuda")
    nat.gemm(A, W, M, N, K, bias=b, resid1=r, act=nat.ACT_GELU_POST, out_f32=out)
    ref = F.gelu(A @ W.t() + b + r)
    assert rel_l2(out.cpu(), ref.cpu()) < 1e-5


@pytest.mark.parametrize("C,lognorm", [(3, False), (1, True)])
def test_pixel_unshuffle(nat, C, lognorm):
    n, H, W, r = 2, 42, 56, 14
    x = _rand(n, H, W, C, seed=31).abs() if lognorm else _rand(n, H, W, C, seed=31)
    div = torch.tensor([1.7, 0.4], device="cuda") if lognorm else None
    out = torch.empty(n * (H // r) * (W // r), C * r * r, device="cuda")
    nat.pixel_unshuffle(x, n, H, W, C, r, out, view_div=div)
    y = x
    if lognorm:
        y = y / div.view(-1, 1, 1, 1)
        nrm = y.norm(dim=-1, keepdim=True)
        y = y / nrm.clip(min=1e-8) * torch.log1p(nrm)
    ref = F.pixel_unshuffle(y.permute(0, 3, 1, 2), r).permute(0, 2, 3, 1).reshape(out.shape)
    assert rel_l2(out.cpu(), ref.cpu()) < 1e-6


def test_depth_norm_factors(nat):
    n, H, W = 3, 64, 80
    d = _rand(n, H, W, seed=41).abs() * 5
    d[d < 4] = 0
    d[2] = 0  # a view without valid depth: nf = clip(0, 1e-8)
    nf = torch.empty(n, device="cuda")
    lnf = torch.empty(n, device="cuda")
    nat.depth_norm_factors(d, n, H * W, nf, lnf)
    valid = d > 0
    ref = ((d * valid).sum((1, 2)) / (valid.sum((1, 2)) + 1e-8)).clip(min=1e-8)
    assert torch.allclose(nf, ref, rtol=1e-5)
    assert torch.allclose(lnf, torch.log(ref + 1e-8), rtol=1e-5)


def test_pose_inputs_match_oracle(nat):
    import importlib

    orc = importlib.import_module("oracle.mapa_oracle")
    V = 4
    g = torch.Generator().manual_seed(5)
    q = torch.randn(V, 4, generator=g)
    q = q / q.norm(dim=1, keepdim=True)
    t = torch.randn(V, 3, generator=g)
    mask = torch.tensor([1, 1, 0, 1], dtype=torch.uint8)
    oq, ot, ol = torch.empty(V, 4, device="cuda"), torch.empty(V, 3, device="cuda"), torch.empty(V, device="cuda")
    nat.pose_inputs(q.cuda(), t.cuda(), mask.cuda(), V, oq, ot, ol)
    rq, rt = torch.tensor([[0.0, 0, 0, 1]]).repeat(V, 1), torch.zeros(V, 3)
    for v in range(V):
        if mask[v]:
            a, b = orc._pose_2_to_1(q[:1], t[:1], q[v:v + 1], t[v:v + 1])
            rq[v], rt[v] = a[0], b[0]
    assert float(ot[0].abs().max()) == 0.0  # the reference view's own translation cancels exactly
    dis = rt.norm(dim=-1)
    nf = (dis.sum() / ((dis > 0).sum() + 1e-8)).clip(min=1e-8)
    assert torch.allclose(oq.cpu(), rq, atol=1e-6)
    assert torch.allclose(ot.cpu(), rt / nf, atol=1e-5)
    assert torch.allclose(ol.cpu(), torch.log(nf + 1e-8).repeat(V), atol=1e-6)


def test_add_view_vectors(nat):
    V, T, C = 3, 10, 64
    x = _rand(V * T, C, seed=51)
    vecs = _rand(2, V, C, seed=52)
    sc = torch.tensor([[1.0, 0.0, 1.0], [0.0, 1.0, 1.0]], device="cuda")
    ref = x.view(V, T, C) + (sc[:, :, None, None] * vecs[:, :, None, :]).sum(0)
    nat.add_view_vectors(x, T, C, V, vecs, sc, 2)
    assert torch.allclose(x.view(V, T, C), ref, atol=1e-6)


def test_view_rays_and_depth_along_ray(nat):
    """preprocess_input_views_for_inference per pixel (inference.py:222-311) vs its torch restatement."""
    n, H, W = 2, 48, 64
    K = torch.tensor([[[50.0, 0, 31.5], [0, 52.0, 23.0], [0, 0, 1]], [[70.0, 0, 30.0], [0, 66.0, 25.0], [0, 0, 1]]])
    dz = (torch.rand(n, H, W, generator=torch.Generator().manual_seed(3)) * 5).cuda()
    rays = torch.empty(n, H, W, 3, device="cuda")
    dar = torch.empty(n, H, W, 1, device="cuda")
    nat.view_rays(n, H, W, rays, K=K.cuda(), depth_z=dz, depth_along_ray=dar)
    x, y = torch.meshgrid(torch.arange(W).float(), torch.arange(H).float(), indexing="xy")
    d = torch.stack(((x - K[:, 0, 2, None, None]) / K[:, 0, 0, None, None],
                     (y - K[:, 1, 2, None, None]) / K[:, 1, 1, None, None], torch.ones(n, H, W)), -1)
    ref = d / torch.norm(d, dim=-1, keepdim=True)
    assert torch.allclose(rays.cpu(), ref, atol=1e-6)
    ref_d = torch.norm(dz.cpu()[..., None] * (ref / ref[..., 2:3]), dim=-1, keepdim=True)
    assert torch.allclose(dar.cpu(), ref_d, rtol=1e-5)
    raw = _rand(n, H, W, 3, seed=7)
    nat.view_rays(n, H, W, rays, rays_in=raw)
    assert torch.allclose(rays, raw / (torch.norm(raw, dim=-1, keepdim=True) + 1e-8), atol=1e-6)


@pytest.mark.parametrize("q", [0.0, 0.1, 0.5, 0.937, 1.0])
def test_confidence_mask_matches_torch_quantile(nat, q):
    n, HW = 3, 50_000
    g = torch.Generator().manual_seed(11)
    conf = (1.0 + torch.rand(n, HW, generator=g).mul(7.0).round().div(3.0)).cuda()  # many duplicates
    conf[1] = 1.0 + torch.rand(HW, generator=g).cuda()
    m_in = (torch.rand(n, HW, generator=g) > 0.2).cuda()
    out = torch.empty(n, HW, dtype=torch.bool, device="cuda")
    nat.confidence_mask(conf, m_in, out, n, HW, q)
    thr = torch.quantile(conf, q, dim=1, keepdim=True)
    assert torch.equal(out, m_in & (conf > thr))


def test_apply_mask_zeroes_geometry(nat):
    n = 1000
    p, pc, d = _rand(n, 3, seed=1), _rand(n, 3, seed=2), _rand(n, 1, seed=3)
    m = (torch.rand(n, generator=torch.Generator().manual_seed(4)) > 0.5).cuda()
    ref = (p * m[:, None], pc * m[:, None], d * m[:, None])
    nat.apply_mask(p, pc, d, m, n)
    assert torch.equal(p, ref[0]) and torch.equal(pc, ref[1]) and torch.equal(d, ref[2])


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1e-2), (torch.float32, 2e-5)])
def test_attention_partials_merge_to_full(nat, dtype, tol):
    """Local-key + remote-key partials merged through their LSEs == attention over all keys (sharded overlap)."""
    H, Sq, Skv, C = 4, 200, 333, 256
    q = _rand(Sq, C, seed=61).to(dtype)
    kv = _rand(Skv, 2 * C, seed=62).to(dtype)
    st = dict(batch=1, heads=H, seq_q=Sq, q_bstride=0, q_rstride=C, k_bstride=0, k_rstride=2 * C, v_bstride=0,
              v_rstride=2 * C, o_bstride=0, o_rstride=C)
    full = torch.empty(Sq, C, device="cuda", dtype=dtype)
    nat.attention(q, kv, kv[:, C:], full, seq_kv=Skv, **st)
    segs_a, segs_b = [(0, 100)], [(100, 150), (250, 83)]
    oa, ob = torch.empty_like(full), torch.empty_like(full)
    la, lb = torch.empty(H, Sq, device="cuda"), torch.empty(H, Sq, device="cuda")
    nat.attention(q, kv, kv[:, C:], oa, seq_kv=100, kv_segments=segs_a, lse=la, **st)
    nat.attention(q, kv, kv[:, C:], ob, seq_kv=233, kv_segments=segs_b, lse=lb, **st)
    nat.attn_merge(oa, la, ob, lb, oa, Sq, H, C)
    assert rel_l2(oa.float().cpu(), full.float().cpu()) < tol


# ------------------------------------------------------------------------------------- split-precision operands
@pytest.mark.parametrize("rows,cols,cp", [(37, 588, 592), (1369, 196, 200), (10, 1024, 1024)])
def test_split_bf16x3_is_bit_exact(nat, rows, cols, cp):
    """[hi | lo] blocks: hi = bf16(x) (RNE), lo = bf16(x - hi), zero padding — bit-exact vs torch."""
    x = _rand(rows, cols, scale=3.0, seed=11)
    y = torch.full((rows, 2 * cp), 7.0, dtype=torch.bfloat16, device="cuda")
    nat.split_bf16x3(x, rows, cols, cp, y)
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    ref = torch.zeros(rows, 2, cp, dtype=torch.bfloat16, device="cuda")
    ref[:, 0, :cols], ref[:, 1, :cols] = hi, lo
    assert torch.equal(y.view(torch.int16), ref.reshape(rows, -1).view(torch.int16))


@pytest.mark.parametrize("variant", [0, 2568])
def test_split_precision_conv_matches_fp32(nat, variant):
    """A 3x3 conv run as one bf16 implicit-GEMM over split activations (stored [hi | lo], read [hi | hi | lo]) and
    [hi | lo | hi] weights (the geometric encoders' bf16-mode path) stays within ~1e-5 of the fp32 conv (plain
    bf16: ~3e-3)."""
    n, h, w, C, Co = 2, 37, 37, 588, 768
    x = _rand(n, C, h, w, seed=12)
    wt = _rand(Co, C, 3, 3, scale=C ** -0.5 / 3, seed=13)
    ref = F.conv2d(x.cpu().double(), wt.cpu().double(), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    M, cp = n * h * w, 592
    xr = x.permute(0, 2, 3, 1).reshape(M, C).contiguous()
    a = torch.empty(M, 2 * cp, dtype=torch.bfloat16, device="cuda")
    nat.split_bf16x3(xr, M, C, cp, a)
    wk = wt.permute(0, 2, 3, 1).reshape(Co, 9, C)
    whi = wk.to(torch.bfloat16)
    wlo = (wk - whi.float()).to(torch.bfloat16)
    wp = torch.zeros(Co, 9, 3, cp, dtype=torch.bfloat16, device="cuda")
    wp[:, :, 0, :C], wp[:, :, 1, :C], wp[:, :, 2, :C] = whi, wlo, whi
    wp = wp.reshape(Co, -1)
    wp._mapa_split = True  # A is a compact split operand
    out = torch.empty(M, Co, device="cuda")
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(a, wp, M, Co, 9 * 3 * cp, out_f32=out, conv=(3 * cp, h, w, h, w, 1))
    finally:
        nat.gemm_set_variant(0)
    assert rel_l2(out.cpu(), ref) < 2e-5


# ------------------------------------------------------------- split-precision operand outputs (fp32 heads)
def _split_expect(v):
    """[hi | lo] of fp32 rows v [R][C] (mapa_split_bf16x3's layout)."""
    hi = v.to(torch.bfloat16)
    lo = (v - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], 1)


@pytest.mark.parametrize("M,N,K", [(333, 384, 192), (100, 6, 24), (257, 130, 64)])
def test_gemm_split_outputs_bit_exact(nat, M, N, K):
    """out_s3 / out_s3_relu rows are exactly [hi | lo] of the fp32 epilogue value (the out_f32 output)."""
    A = _rand(M, K, seed=31).to(torch.bfloat16)
    W = _rand(N, K, scale=K ** -0.5, seed=32).to(torch.bfloat16)
    b, r1 = _rand(N, seed=33), _rand(M, N, seed=34)
    of = torch.empty(M, N, device="cuda")
    s3 = torch.full((M, 2 * N), 7.0, device="cuda", dtype=torch.bfloat16)
    s3r = torch.full((M, 2 * N), 7.0, device="cuda", dtype=torch.bfloat16)
    nat.gemm(A, W, M, N, K, bias=b, resid1=r1, out_f32=of, out_s3=s3, out_s3_relu=s3r)
    assert torch.equal(s3, _split_expect(of))
    assert torch.equal(s3r, _split_expect(torch.relu(of)))


def test_gemm_split_output_pixel_shuffle(nat):
    """ConvTranspose k=s=2 through the pixel-shuffle epilogue into split rows (2*cout per output pixel)."""
    n, h, w, ci, co, s = 2, 5, 7, 64, 48, 2
    A = _rand(n * h * w, ci, seed=35).to(torch.bfloat16)
    W = _rand(s * s * co, ci, scale=ci ** -0.5, seed=36).to(torch.bfloat16)
    b = _rand(co, seed=37)
    of = torch.empty(n * h * s * w * s, co, device="cuda")
    s3 = torch.empty(n * h * s * w * s, 2 * co, device="cuda", dtype=torch.bfloat16)
    nat.gemm(A, W, n * h * w, s * s * co, ci, bias=b, bias_mod=co, out_f32=of, out_s3=s3, pixshuf=(s, h, w, co))
    assert torch.equal(s3, _split_expect(of))


def test_split_chain_matches_fp32(nat):
    """A split-output GEMM feeding a split-operand conv3x3 ([hi | lo | hi] weights, A stored [hi | lo]): the fp32
    product to ~2^-16 (plain bf16 operands: ~3e-3) — the precision of the heads in bf16 mode."""
    from mapanything.models.mapanything.engine import _split_pack

    n, H, W_, C, Co = 2, 9, 11, 64, 40
    x = _rand(n * H * W_, C, seed=38)
    w1 = _rand(C, C, scale=C ** -0.5, seed=39)
    b1 = _rand(C, seed=40)
    wc = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=41)
    xs = torch.empty(n * H * W_, 2 * C, device="cuda", dtype=torch.bfloat16)
    nat.split_bf16x3(x, n * H * W_, C, C, xs)
    w1s = _split_pack(w1.cpu().numpy().reshape(C, 1, C), "cuda")
    y = torch.empty(n * H * W_, 2 * C, device="cuda", dtype=torch.bfloat16)
    nat.gemm(xs, w1s, n * H * W_, C, 3 * C, bias=b1, act=nat.ACT_RELU, out_s3=y)
    wcs = _split_pack(wc.permute(0, 2, 3, 1).reshape(Co, 9, C).cpu().numpy(), "cuda")
    out = torch.empty(n * H * W_, Co, device="cuda")
    nat.gemm(y, wcs, n * H * W_, Co, 27 * C, out_f32=out, conv=(3 * C, H, W_, H, W_, 1))
    yr = torch.relu(x.double() @ w1.double().t() + b1.double())
    ref = F.conv2d(yr.view(n, H, W_, C).permute(0, 3, 1, 2), wc.double(), padding=1).permute(0, 2, 3, 1)
    assert rel_l2(out.double().cpu(), ref.reshape(-1, Co).cpu()) < 2e-5


def test_layernorm_split_output(nat):
    rows, dim = 77, 768
    x = _rand(rows, dim, seed=42)
    w, b = _rand(dim, seed=43), _rand(dim, seed=44)
    yf = torch.empty(rows, dim, device="cuda")
    ys = torch.empty(rows, 2 * dim, device="cuda", dtype=torch.bfloat16)
    nat.layernorm(x, rows, dim, w, b, y_f32=yf, y_s3=ys)
    assert torch.equal(ys, _split_expect(yf))


def test_bilinear_split_output(nat):
    n, IH, IW, C, OH, OW = 2, 19, 23, 128, 38, 46
    x = _rand(n * IH * IW, C, seed=45)
    yf = torch.empty(n * OH * OW, C, device="cuda")
    ys = torch.empty(n * OH * OW, 2 * C, device="cuda", dtype=torch.bfloat16)
    nat.bilinear_ac(x, n, IH, IW, C, OH, OW, OH, OW, yf)
    nat.bilinear_ac(x, n, IH, IW, C, OH, OW, OH, OW, ys, split_out=True)
    assert torch.equal(ys, _split_expect(yf))


# ------------------------------------------------------------------------------------------- RoPE-2D
def test_rope2d_matches_reference_fixture():
    """uniception croco RoPE2D (pos_embed.py:101-155 / curope kernels.cu:17-82) through the RoPE2D op: fp32 to
    within the sincos rounding of the reference's own outputs (fixture from the reference, make_rope_golden.py)."""
    import os

    from conftest import GOLDEN
    from uniception.models.libs.croco.pos_embed import RoPE2D

    g = np.load(os.path.join(GOLDEN, "golden_rope2d.npz"))
    t = torch.from_numpy(g["grid_tokens"]).cuda()
    out = RoPE2D(freq=100.0)(t, torch.from_numpy(g["grid_pos"]).cuda())
    assert out.data_ptr() == t.data_ptr()  # in place, as cuRoPE2D
    assert (out.cpu() - torch.from_numpy(g["grid_out"])).abs().max() < 2e-5
    for base in (100, 10000):
        t = torch.from_numpy(g["rand_tokens"]).cuda()
        RoPE2D(freq=float(base))(t, torch.from_numpy(g["rand_pos"]).cuda())
        assert (t.cpu() - torch.from_numpy(g[f"rand_out_base{base}"])).abs().max() < 2e-5, base


def test_rope2d_bf16_on_packed_qkv_rows(nat):
    """The same rotation in place on the Q and K column blocks of a packed [rows][3C] bf16 qkv buffer (what an
    attention with RoPE positions reads), V untouched; against the oracle on the fp32 values."""
    from oracle.mapa_oracle import rope2d

    N, H = 300, 12
    C = 64 * H
    qkv = _rand(N, 3 * C, seed=51).to(torch.bfloat16)
    pos = torch.randint(0, 40, (1, N, 2), generator=torch.Generator().manual_seed(3)).cuda()
    ref = qkv.float().cpu()
    work = qkv.clone()
    for blk in (0, 1):  # Q then K: (B=1, H, N, 64) views with strides (., 64, 3C)
        nat.rope2d(work[:, blk * C:], pos, 1, H, N, 64, 0, 64, 3 * C, 100.0, 1.0)
    for blk in (0, 1):
        x = ref[:, blk * C:(blk + 1) * C].view(N, H, 64).permute(1, 0, 2)[None]
        want = rope2d(x, pos.cpu())[0].permute(1, 0, 2).reshape(N, C)
        got = work[:, blk * C:(blk + 1) * C].float().cpu()
        assert rel_l2(got, want) < 4e-3
    assert torch.equal(work[:, 2 * C:], qkv[:, 2 * C:])



# ----------------------------------------------------------------------- fp16 operands (the fp16 autocast recipe)
@pytest.mark.parametrize("variant", [0, 2568, 2570, 2571, 2574, 2587, 1282, 643])
@pytest.mark.parametrize("M,N,K", [(300, 200, 264), (1370, 1024, 1024), (2737, 768, 3072)])
def test_gemm_fp16_operands(nat, variant, M, N, K):
    """infer(amp_dtype="fp16"): fp16 A / W on the f16 MFMA in every tile kernel the automatic choice uses (and the
    128x128 fallbacks), fp32 accumulate; plain, GELU -> fp16 and in-place residual epilogues."""
    A = _rand(M, K, seed=80).to(torch.float16)
    W = _rand(N, K, scale=K ** -0.5, seed=81).to(torch.float16)
    b, g = _rand(N, seed=82), _rand(N, seed=83) * 0.1
    acc = A.float() @ W.float().t() + b
    nat.gemm_set_variant(variant)
    try:
        out = torch.empty(M, N, device="cuda")
        nat.gemm(A, W, M, N, K, bias=b, out_f32=out)
        assert rel_l2(out.cpu(), acc.cpu()) < 1e-5
        o = torch.empty(M, N, device="cuda", dtype=torch.float16)
        nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=o)
        assert o.dtype == torch.float16 and rel_l2(o.float().cpu(), F.gelu(acc).cpu()) < 1e-3
        x0 = _rand(M, N, seed=84)
        x = x0.clone()
        nat.gemm(A, W, M, N, K, bias=b, gamma=g, resid1=x, out_f32=x)
        assert rel_l2(x.cpu(), (x0 + g * acc).cpu()) < 1e-5
    finally:
        nat.gemm_set_variant(0)


@pytest.mark.parametrize("B,Hh,S", [(2, 16, 1370), (1, 12, 10953), (3, 12, 65)])
def test_attention_fp16_operands(nat, B, Hh, S):
    """The flash kernel on fp16 q / k / v (f16 MFMAs, P rounded to fp16) against fp32 SDPA of the same inputs,
    including the split-merge path (few query blocks) and the LSE."""
    C = Hh * 64
    qkv = _rand(B * S, 3 * C, seed=85).to(torch.float16)
    o = torch.empty(B * S, C, device="cuda", dtype=torch.float16)
    lse = torch.empty(B, Hh, S, device="cuda")
    rs = 3 * C
    nat.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B, heads=Hh, seq_q=S, seq_kv=S, q_bstride=S * rs,
                  q_rstride=rs, k_bstride=S * rs, k_rstride=rs, v_bstride=S * rs, v_rstride=rs, o_bstride=S * C,
                  o_rstride=C, lse=lse)
    t = qkv.view(B, S, 3, Hh, 64).permute(2, 0, 3, 1, 4)
    ref = _sdpa_ref(t[0], t[1], t[2]).transpose(1, 2).reshape(B * S, C)
    assert rel_l2(o.float().cpu(), ref.cpu()) < 2e-3
    s = (t[0].float() @ t[1].float().transpose(-1, -2)) / 8.0
    assert rel_l2(lse.cpu(), torch.logsumexp(s, -1).cpu()) < 1e-4
    # the overlapped all-gather's partial merge in fp16
    half = S // 2
    if half >= 1 and B == 1:
        q = qkv[:, :C]
        oa, ob = torch.empty_like(o), torch.empty_like(o)
        la, lb = torch.empty(Hh, S, device="cuda"), torch.empty(Hh, S, device="cuda")
        common = dict(batch=1, heads=Hh, seq_q=S, q_bstride=0, q_rstride=rs, k_bstride=0, k_rstride=rs, v_bstride=0,
                      v_rstride=rs, o_bstride=0, o_rstride=C)
        nat.attention(q, qkv[:, C:], qkv[:, 2 * C:], oa, seq_kv=half, lse=la, **common)
        nat.attention(q, qkv[half:, C:], qkv[half:, 2 * C:], ob, seq_kv=S - half, lse=lb, **common)
        om = torch.empty_like(o)
        nat.attn_merge(oa, la, ob, lb, om, S, Hh, C)
        assert rel_l2(om.float().cpu(), ref.cpu()) < 2e-3


def test_layernorm_fp16_output(nat):
    rows, dim = 517, 1024
    x = _rand(rows, dim, scale=3.0, seed=86) + 1.5
    w, b = _rand(dim, seed=87), _rand(dim, seed=88)
    y = torch.empty(rows, dim, device="cuda", dtype=torch.float16)
    nat.layernorm(x, rows, dim, w, b, y_lp=y)
    ref = F.layer_norm(x, (dim,), w, b, 1e-6)
    assert y.dtype == torch.float16 and rel_l2(y.float().cpu(), ref.cpu()) < 1e-3
    y7 = torch.empty(rows, 768, device="cuda", dtype=torch.float16)
    nat.layernorm(x[:, :768].contiguous(), rows, 768, w[:768], b[:768], y_lp=y7)
    ref7 = F.layer_norm(x[:, :768], (768,), w[:768], b[:768], 1e-6)
    assert rel_l2(y7.float().cpu(), ref7.cpu()) < 1e-3
