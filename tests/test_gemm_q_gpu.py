"""Numerics of the four-wave 256x256 GEMM kernel (gemm_q.hip, variant 32) against
fp32 PyTorch references: every operand
layout, ragged M / N / K edges (incl. the k-contiguous K tail), each fused
epilogue, fp32 beta-accumulate and the split-K in-launch combine."""
import pytest
import torch

import ldnn  # noqa: F401
from ldnn.ops import _ext

pytestmark = pytest.mark.gpu

KERNELS = [32]


def C():
    return _ext.C()


def _ref(a, b, a_kc, b_kc):
    A = a.float() if a_kc else a.float().t()
    B = b.float().t() if b_kc else b.float()
    return A @ B


def _ops(M, N, K, a_kc, b_kc, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = (torch.randn(M, K, device="cuda", generator=g) if a_kc else
         torch.randn(K, M, device="cuda", generator=g)).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) if b_kc else
         torch.randn(K, N, device="cuda", generator=g)).bfloat16()
    return a, b


@pytest.mark.parametrize("variant", KERNELS)
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (520, 776, 520), (296, 264, 4200), (1024, 512, 1040),
                                   (264, 784, 1016), (64, 16, 4096)])
def test_layouts_ragged(variant, a_kc, b_kc, M, N, K):
    a, b = _ops(M, N, K, a_kc, b_kc)
    ref = _ref(a, b, a_kc, b_kc)
    c = torch.full((M, N), float("nan"), device="cuda")
    C().gemm(a, b, c, a_kc, b_kc, tile=256, variant=variant)
    torch.cuda.synchronize()
    assert (c - ref).abs().max().item() <= 1e-3 * K ** 0.5 + 1e-3
    cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C().gemm(a, b, cb, a_kc, b_kc, tile=256, variant=variant)
    assert ((cb.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("variant", KERNELS)
def test_asymmetric_identity(variant):
    """A = I with an asymmetric B catches a transposed or mis-placed C write (exact)."""
    n = 512
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda").reshape(n, n).float().remainder(97).bfloat16()
    c = torch.empty(n, n, device="cuda")
    C().gemm(a, b, c, True, True, tile=256, variant=variant)
    assert torch.equal(c, b.float().t())
    C().gemm(a, b, c, True, False, tile=256, variant=variant)
    assert torch.equal(c, b.float())
    C().gemm(a.t().contiguous(), b, c, False, False, tile=256, variant=variant)
    assert torch.equal(c, b.float())


@pytest.mark.parametrize("variant", KERNELS)
@pytest.mark.parametrize("epi", ["bias", "relu", "sigmoid"])
def test_fwd_epilogues(variant, epi):
    M, N, K = 600, 520, 1104
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    code = {"bias": C().EPI_BIAS, "relu": C().EPI_BIAS_RELU, "sigmoid": C().EPI_BIAS_SIGMOID}[epi]
    C().gemm(x, w, y, True, True, code, bias=bias, tile=256, variant=variant)
    ref = x.float() @ w.float().t() + bias
    ref = ref.relu() if epi == "relu" else ref.sigmoid() if epi == "sigmoid" else ref
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("variant", KERNELS)
@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_dgrad_epilogue_and_dbias(variant, act):
    M, N, K = 776, 1040, 520   # dX[M,K] = dY[M,N] @ W[N,K]
    g = torch.Generator(device="cuda").manual_seed(2)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    yprev = torch.randn(M, K, device="cuda", generator=g)
    yprev = (yprev.relu() if act == "relu" else yprev.sigmoid()).bfloat16()
    dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(K, device="cuda")
    code = C().EPI_DRELU if act == "relu" else C().EPI_DSIGMOID
    C().gemm(dy, w, dx, True, False, code, aux=yprev, dbias=db, tile=256, variant=variant)
    gr = dy.float() @ w.float()
    y = yprev.float()
    ref = gr * (y > 0) if act == "relu" else gr * y * (1 - y)
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(db, dx.float().sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("variant", KERNELS)
def test_wgrad_beta_accumulate(variant):
    B, N, K = 1100, 264, 784   # dW[N,K] = dY^T X
    g = torch.Generator(device="cuda").manual_seed(3)
    dy = torch.randn(B, N, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, K, device="cuda", generator=g).bfloat16()
    dw = torch.randn(N, K, device="cuda", generator=g)
    base = dw.clone()
    C().gemm(dy, x, dw, False, False, beta=1.0, tile=256, variant=variant)
    torch.testing.assert_close(dw, base + dy.float().t() @ x.float(), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("variant", KERNELS)
@pytest.mark.parametrize("splitk", [2, 3, 4])
@pytest.mark.parametrize("case", ["wgrad", "fwd_relu", "dgrad_drelu"])
def test_splitk_inlaunch_combine(variant, splitk, case):
    """Split-K over gridDim.y with the deterministic in-launch slab combine: the
    result equals the fp32 reference and is bit-identical across repeats."""
    g = torch.Generator(device="cuda").manual_seed(4)
    if case == "wgrad":
        B, M, N = 4160, 520, 784
        a = torch.randn(B, M, device="cuda", generator=g).bfloat16()
        b = torch.randn(B, N, device="cuda", generator=g).bfloat16()
        out = torch.empty(M, N, device="cuda")
        ref = a.float().t() @ b.float()
        args = (a, b, out, False, False)
        kw = {}
        tol = 1e-3 * B ** 0.5 + 1e-3
    elif case == "fwd_relu":
        M, N, K = 300, 264, 4096
        a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        b = (torch.randn(N, K, device="cuda", generator=g) * 0.02).bfloat16()
        bias = torch.randn(N, device="cuda", generator=g)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = (a.float() @ b.float().t() + bias).relu()
        args = (a, b, out, True, True, C().EPI_BIAS_RELU)
        kw = dict(bias=bias)
        tol = 3e-2
    else:
        M, N, K = 264, 4096, 520
        a = (torch.randn(M, N, device="cuda", generator=g) * 0.05).bfloat16()
        b = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
        yprev = torch.randn(M, K, device="cuda", generator=g).relu().bfloat16()
        out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        ref = (a.float() @ b.float()) * (yprev.float() > 0)
        db = torch.zeros(K, device="cuda")
        args = (a, b, out, True, False, C().EPI_DRELU)
        kw = dict(aux=yprev, dbias=db)
        tol = 3e-2
    ne, nc = C().gemm_q_ws(out.shape[0], out.shape[1], splitk)
    ws = torch.empty(ne, device="cuda")
    cnt = torch.zeros(nc, device="cuda", dtype=torch.int32)
    C().gemm(*args, tile=256, variant=variant, splitk=splitk, ws=ws, cnt=cnt, **kw)
    first = out.clone()
    assert (out.float() - ref).abs().max().item() <= tol
    if case == "dgrad_drelu":
        torch.testing.assert_close(db, out.float().sum(0), rtol=1e-3, atol=1e-2)
        kw["dbias"] = torch.zeros(K, device="cuda")
    C().gemm(*args, tile=256, variant=variant, splitk=splitk, ws=ws, cnt=cnt, **kw)
    assert torch.equal(out, first)
    assert int(cnt.abs().sum().item()) == 0   # counters left zero for the next launch


def test_auto_picks_q_for_long_k():
    """tile=0 / variant=0 routes long-K shapes with a full 256-tile grid (>= 192 tiles)
    to gemm_q: bit-identical to variant 32."""
    a, b = _ops(3584, 3584, 1024, True, True, seed=5)
    c0 = torch.empty(3584, 3584, device="cuda")
    c1 = torch.empty_like(c0)
    C().gemm(a, b, c0, True, True)
    C().gemm(a, b, c1, True, True, tile=256, variant=32)
    assert torch.equal(c0, c1)


@pytest.mark.parametrize("M,N,K", [(520, 776, 784), (1024, 512, 1040)])
def test_relu_mask_forward_and_dgrad(M, N, K):
    """EPI_BIAS_RELU_MASK writes the bf16 output AND mask bits (bit q of byte [m][n/8] =
    out[m][n+q] > 0); EPI_DRELU_MASK reading those bits equals EPI_DRELU reading the bf16
    activation (same accumulators, same derivative, same bias-gradient sums)."""
    c = C()
    x, w = _ops(M, N, K, True, True, seed=3)
    bias = torch.randn(N, device="cuda")
    h_ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    h = torch.empty_like(h_ref)
    mask = torch.full((M, (N + 7) // 8), 0xAA, dtype=torch.uint8, device="cuda")
    c.gemm(x, w, h_ref, True, True, c.EPI_BIAS_RELU, bias=bias, tile=256, variant=32)
    c.gemm(x, w, h, True, True, c.EPI_BIAS_RELU, bias=bias, mask_out=mask)
    assert torch.equal(h, h_ref)
    bits = ((h.float() > 0).view(M, -1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(-1)
    assert torch.equal(mask[:, : N // 8].to(torch.int32), bits)
    # dgrad: dz_prev = (dz W2) * relu'(h), K2 = 640 outputs of the next layer
    dz, w2 = _ops(M, N, 640, True, False, seed=4)   # dz [M][640], w2 [640][N] (k-strided B)
    out_a, out_m = (torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    db_a, db_m = torch.zeros(N, device="cuda"), torch.zeros(N, device="cuda")
    c.gemm(dz, w2, out_a, True, False, c.EPI_DRELU, aux=h, dbias=db_a, tile=256, variant=32)
    c.gemm(dz, w2, out_m, True, False, c.EPI_DRELU, dbias=db_m, mask_in=mask)
    assert torch.equal(out_a, out_m)
    torch.testing.assert_close(db_m, db_a, rtol=1e-5, atol=1e-3)
    ref = (dz.float() @ w2.float()) * (h.float() > 0)
    torch.testing.assert_close(out_m.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("sk", [2, 4])
def test_split_slabs_plus_slab_sum(sk):
    """Split-K partial products into [sk][M][N] slabs (no in-launch combine) + slab_sum."""
    c = C()
    M, N, K = 1032, 784, 4096
    a, b = _ops(M, N, K, False, False, seed=5)
    slabs = torch.full((sk, M, N), float("nan"), device="cuda")
    out = torch.empty(M, N, device="cuda")
    c.gemm(a, b, slabs, False, False, tile=256, splitk=sk)
    c.slab_sum(slabs, out)
    ref = _ref(a, b, False, False)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)
    one = torch.empty(M, N, device="cuda")
    c.gemm(a, b, one, False, False, tile=256, variant=32)
    torch.testing.assert_close(out, one, rtol=1e-5, atol=1e-3)  # fp32 summation order only


def test_transpose_and_slab_sum_cols():
    c = C()
    x = torch.randn(520, 776, device="cuda").bfloat16()
    out = torch.empty(776, 520, device="cuda", dtype=torch.bfloat16)
    c.transpose_bf16(x, out)
    assert torch.equal(out, x.t())
    for r, cc in ((4096, 4096), (64, 64), (8, 1032), (1032, 8)):   # whole / single / ragged tiles
        x = torch.randn(r, cc, device="cuda").bfloat16()
        out = torch.empty(cc, r, device="cuda", dtype=torch.bfloat16)
        c.transpose_bf16(x, out)
        assert torch.equal(out, x.t()), (r, cc)
    ws = torch.randn(3, 264, 792, device="cuda")
    dst = torch.full((264, 784), float("nan"), device="cuda")
    extra = torch.full((264,), float("nan"), device="cuda")
    c.slab_sum_cols(ws, dst, extra)
    tot = ws.sum(0)
    torch.testing.assert_close(dst, tot[:, :784], rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(extra, tot[:, 784], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (512, 784, 2048)])
def test_gemm_opt_epilogue_equals_gemm_then_optimizer(kind, M, N, K):
    """gemm_opt: a weight-gradient GEMM whose epilogue applies SGD (momentum, weight decay) /
    Adam / AdamW to the fp32 master and refreshes the bf16 shadow -- the four-wave kernel's
    row-staged update at 4096 x 4096 x 4096 (gemm_q EPI_OPT_*), gemm.hip's at the smaller
    shape -- == the plain fp32-out GEMM followed by the separate fused optimizer launch."""
    torch.manual_seed(0)
    C = _ext.C()
    dz = (torch.randn(K, M, device="cuda") * 0.1).bfloat16()   # [batch][out]
    h = torch.randn(K, N, device="cuda").bfloat16()            # [batch][in]
    master0 = torch.randn(M, N, device="cuda") * 0.05
    hp = torch.tensor([1e-2 if kind == "sgd" else 1e-3, 3.0], device="cuda")   # lr, Adam step (already bumped)
    wd = 1e-2
    # reference: gradient GEMM, then the flat optimizer kernel
    g = torch.empty(M, N, device="cuda")
    # (the tiling gemm_opt takes, unsplit: the same fp32 accumulation order)
    C.gemm(dz, h, g, False, False, tile=256 if M * N >= 192 * 65536 else 128, splitk=1)
    torch.testing.assert_close(g, dz.float().t() @ h.float(), rtol=2e-3, atol=2e-3)
    mr, m1, v1 = master0.clone(), torch.randn(M, N, device="cuda") * 1e-3, torch.rand(M, N, device="cuda") * 1e-5
    sr = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    mf, m2, v2 = master0.clone(), m1.clone(), v1.clone()
    sf = torch.empty_like(sr)
    if kind == "sgd":
        C.sgd_step(mr.view(-1), g.view(-1), m1.view(-1), sr.view(-1), hp, 0.5, 0.9, 0.0, wd, False, False)
        C.gemm_opt(dz, h, mf, False, False, "sgd", m=m2, shadow=sf, hp=hp, grad_scale=0.5, momentum=0.9,
                   weight_decay=wd)
        states = ((m2, m1),)
    else:
        C.adam_step(mr.view(-1), g.view(-1), m1.view(-1), v1.view(-1), sr.view(-1), hp, 0.5, 0.9, 0.999, 1e-8, wd,
                    kind == "adamw")
        C.gemm_opt(dz, h, mf, False, False, kind, m=m2, v=v2, shadow=sf, hp=hp, grad_scale=0.5, weight_decay=wd)
        states = ((m2, m1), (v2, v1))
    torch.cuda.synchronize()
    # the same gradient (fp32 accumulate, tile order identical), the same update arithmetic
    torch.testing.assert_close(mf, mr, rtol=1e-5, atol=1e-7)
    for a, b in states:
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-9)
    assert (sf.float() - sr.float()).abs().max().item() <= 2 ** -7 * mr.abs().max().item()
