"""hsg_gemm_f32 (fp32-accurate 3-limb bf16 split on v_mfma_f32_32x32x16_bf16) and
hsg_gemm_f32_mfma (exact-f32 v_mfma_f32_32x32x2_f32) against an fp64 torch
reference: every operand layout, ragged shapes, each epilogue, split-K, and the
split path's error class (per element, in units of sum_k |a||b|, no worse than
the exact-f32 instruction's)."""
import pytest
import torch

from helpers import skip_unless_dev

pytestmark = pytest.mark.gpu

SHAPES = [(19200 // 8, 512, 300), (1000, 300, 512), (67, 45, 33), (1120, 64, 512), (300, 512, 2400),
          (128, 128, 32), (5, 7, 3)]


def ref(A, B, a_t, b_t):
    a = A.double().t() if a_t else A.double()
    b = B.double().t() if b_t else B.double()
    return a @ b


def mk(rows, cols):
    # row stride padded to a multiple of 4 when needed (16-byte aligned rows)
    ld = (cols + 3) // 4 * 4
    return torch.randn(rows, ld, device="cuda")[:, :cols]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("a_t,b_t", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("dtype", ["f32", "f32mfma"])
def test_layouts(M, N, K, a_t, b_t, dtype):
    from hetersumgraph_amd.dense import gemm
    torch.manual_seed(M + N + K)
    A = mk(K, M) if a_t else mk(M, K)
    B = mk(N, K) if b_t else mk(K, N)
    C = gemm(A, B, a_t, b_t, dtype=dtype)
    R = ref(A, B, a_t, b_t)
    err = (C.double() - R).abs().max().item()
    assert err <= 1e-5 * max(1.0, K ** 0.5) * 4, err


@pytest.mark.parametrize("splits", [2, 7, 16])
def test_split_k(splits):
    from hetersumgraph_amd.dense import gemm
    torch.manual_seed(splits)
    A = torch.randn(4000, 300, device="cuda")
    B = torch.randn(4000, 512, device="cuda")
    C = gemm(A, B, a_t=True, splits=splits)          # dW-shaped: A^T B
    R = A.double().t() @ B.double()
    assert (C.double() - R).abs().max().item() < 2e-3
    C2 = gemm(A, B, a_t=True, splits=splits)
    assert torch.equal(C, C2)                          # deterministic


def test_epilogues():
    from hetersumgraph_amd.dense import gemm
    torch.manual_seed(0)
    X = torch.randn(777, 300, device="cuda")
    W = torch.randn(512, 300, device="cuda")
    b = torch.randn(512, device="cuda")
    H = gemm(X, W, b_t=True, bias=b, relu=True)
    Hr = torch.relu(X.double() @ W.double().t() + b.double())
    assert (H.double() - Hr).abs().max().item() < 1e-4
    G = torch.randn(777, 300, device="cuda")
    W2 = torch.randn(300, 512, device="cuda")
    dH = gemm(G, W2, relu_mask=H)
    dHr = (G.double() @ W2.double()) * (Hr > 0)
    assert (dH.double() - dHr).abs().max().item() < 1e-4
    acc = torch.randn(777, 300, device="cuda")
    acc0 = acc.clone()
    gemm(dH, W, out=acc, add=acc)
    accr = acc0.double() + dH.double() @ W.double()
    assert (acc.double() - accr).abs().max().item() < 2e-3


def test_speed_smoke():
    """Reports TFLOP/s of the dominant FFN GEMM shape (no assertion on speed)."""
    from hetersumgraph_amd.dense import gemm
    X = torch.randn(19200, 300, device="cuda")
    W = torch.randn(512, 300, device="cuda")
    b = torch.randn(512, device="cuda")
    for _ in range(3):
        gemm(X, W, b_t=True, bias=b, relu=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        gemm(X, W, b_t=True, bias=b, relu=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    tf = 2 * 19200 * 300 * 512 / (ms * 1e-3) / 1e12
    print(f"ffn gemm1 19200x512x300: {ms * 1e3:.1f} us, {tf:.1f} TFLOP/s")
    e0.record()
    for _ in range(20):
        torch.nn.functional.linear(X, W, b)
    e1.record()
    torch.cuda.synchronize()
    ms2 = e0.elapsed_time(e1) / 20
    print(f"torch linear same shape: {ms2 * 1e3:.1f} us, {2 * 19200 * 300 * 512 / (ms2 * 1e-3) / 1e12:.1f} TFLOP/s")


# ---- hsg_gemm_bf16: bf16-rounded operands, fp32 accumulation (config 5) ----------
def bf16_ref(A, B, a_t, b_t):
    """fp64 GEMM of the operands rounded to bf16 (RNE, as v_cvt_pk_bf16_f32): every
    bf16 x bf16 product is exact in fp32, so only the fp32 summation differs."""
    return ref(A.bfloat16().float(), B.bfloat16().float(), a_t, b_t)


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("a_t,b_t", [(False, False), (False, True), (True, False), (True, True)])
def test_bf16_layouts(M, N, K, a_t, b_t):
    from hetersumgraph_amd.dense import gemm
    torch.manual_seed(M + N + K + 1)
    A = mk(K, M) if a_t else mk(M, K)
    B = mk(N, K) if b_t else mk(K, N)
    C = gemm(A, B, a_t, b_t, dtype="bf16")
    err = (C.double() - bf16_ref(A, B, a_t, b_t)).abs().max().item()
    assert err <= 1e-5 * max(1.0, K ** 0.5) * 4, err
    # and it is a real reduced-precision result: far from the fp32 GEMM at large K
    if K >= 300:
        assert (C.double() - ref(A, B, a_t, b_t)).abs().max().item() > 1e-4


def test_bf16_epilogue_and_split_k():
    from hetersumgraph_amd.dense import gemm, gemm_dtype
    torch.manual_seed(5)
    X = torch.randn(777, 300, device="cuda")
    W = torch.randn(512, 300, device="cuda")
    b = torch.randn(512, device="cuda")
    with gemm_dtype("bf16"):
        H = gemm(X, W, b_t=True, bias=b, relu=True)
        A = torch.randn(4000, 300, device="cuda")
        B = torch.randn(4000, 512, device="cuda")
        C = gemm(A, B, a_t=True, splits=7)
    Hr = torch.relu(bf16_ref(X, W, False, True) + b.double())
    assert (H.double() - Hr).abs().max().item() < 1e-4
    assert (C.double() - bf16_ref(A, B, True, False)).abs().max().item() < 2e-3


@pytest.mark.parametrize("M,N,K,a_t,b_t", [(19200, 512, 300, False, True), (19200, 300, 512, False, True),
                                           (19200, 512, 300, False, False), (4000, 300, 512, False, False),
                                           (777, 64, 300, False, True), (3000, 1350, 300, False, True)])
def test_split_is_fp32_class(M, N, K, a_t, b_t):
    """Per output element, |C - C_fp64| / sum_k |a_k b_k| of the 3-limb split path is
    within 1.5x of the exact-f32 instruction's and below 2e-6 (fp32 unit roundoff is
    6e-8 per rounding), on operands with a wide dynamic range."""
    from hetersumgraph_amd.dense import gemm
    torch.manual_seed(K)
    A = (mk(K, M) if a_t else mk(M, K)) * torch.exp(2 * torch.randn(1, device="cuda"))
    B = mk(N, K) if b_t else mk(K, N)
    A = A * torch.exp(torch.randn_like(A))               # entries spread over many binades
    a64 = (A.t() if a_t else A).double()
    b64 = (B.t() if b_t else B).double()
    ref, unit = a64 @ b64, a64.abs() @ b64.abs()
    e = {}
    for dt in ("f32", "f32mfma"):
        C = gemm(A, B, a_t, b_t, dtype=dt)
        e[dt] = ((C.double() - ref).abs() / unit).max().item()
    print(f"{M}x{N}x{K}: split {e['f32']:.2e}, f32 mfma {e['f32mfma']:.2e}")
    assert e["f32"] <= 1.5 * e["f32mfma"] + 1e-8 and e["f32"] < 2e-6


# ---- hsg_wsplit + hsg_gemm_f32_psw: pre-split weight operand ----------------------
PSW_SHAPES = [(1, 1, 4), (33, 17, 20), (130, 300, 300), (777, 512, 300), (1000, 300, 512), (257, 64, 300),
              (19200, 512, 300)]


@pytest.mark.parametrize("plan", ["1", "2", "3", "4", "5", "6", "7", "27", "30"])
@pytest.mark.parametrize("M,N,K", PSW_SHAPES)
@pytest.mark.parametrize("trans", [False, True])
def test_psw_layouts(M, N, K, trans, plan, monkeypatch):
    """Every tile plan, row/column/K tails, both weight orientations: fp32-class error
    against fp64 (the same bound as hsg_gemm_f32's test_layouts)."""
    from hetersumgraph_amd.dense import gemm_psw, split_weights
    skip_unless_dev(plan == "27")
    monkeypatch.setenv("HSG_GEMM5", plan)
    torch.manual_seed(M + N + K)
    A = mk(M, K)
    W = mk(K, N) if trans else mk(N, K)
    (S,) = split_weights((W, trans))
    C = gemm_psw(A, S)
    R = A.double() @ (W.double() if trans else W.double().t())
    err = (C.double() - R).abs().max().item()
    assert err <= 1e-5 * max(1.0, K ** 0.5) * 4, err


@pytest.mark.parametrize("M,N,K", [(19200, 512, 300), (19200, 300, 512), (1600, 300, 512), (777, 512, 300)])
@pytest.mark.parametrize("plan", ["7", "27"])
def test_psw_split_is_fp32_class(M, N, K, plan, monkeypatch):
    """The pre-split-weight GEMM (in-kernel split of the fp32 activation operand) is
    fp32-class: per element |C - C_fp64| / sum_k |a_k b_k| within 1.5x of the exact-f32
    instruction's and below 2e-6, on operands spread over many binades."""
    from hetersumgraph_amd.dense import gemm, gemm_psw, split_weights
    skip_unless_dev(plan == "27")
    monkeypatch.setenv("HSG_GEMM5", plan)
    torch.manual_seed(K + 1)
    A = mk(M, K) * torch.exp(2 * torch.randn(1, device="cuda"))
    A = A * torch.exp(torch.randn_like(A))
    W = mk(N, K) * torch.exp(torch.randn(N, K, device="cuda"))
    (S,) = split_weights((W, False))
    ref = A.double() @ W.double().t()
    unit = A.double().abs() @ W.double().abs().t()
    e_psw = ((gemm_psw(A, S).double() - ref).abs() / unit).max().item()
    e_f32 = ((gemm(A, W, b_t=True, dtype="f32mfma").double() - ref).abs() / unit).max().item()
    print(f"{M}x{N}x{K} plan {plan}: psw {e_psw:.2e}, f32 mfma {e_f32:.2e}")
    assert e_psw <= 1.5 * e_f32 + 1e-8 and e_psw < 2e-6


def test_psw_epilogues_and_colsums():
    from hetersumgraph_amd.dense import gemm, gemm_psw, row_tiles, split_weights
    torch.manual_seed(1)
    X = torch.randn(777, 300, device="cuda")
    W1 = torch.randn(512, 300, device="cuda")
    W2 = torch.randn(300, 512, device="cuda")
    b = torch.randn(512, device="cuda")
    s1, s2t, s1t = split_weights((W1, False), (W2, True), (W1, True))
    H = gemm_psw(X, s1, bias=b, relu=True)
    Hr = torch.relu(X.double() @ W1.double().t() + b.double())
    assert (H.double() - Hr).abs().max().item() < 1e-4
    G = torch.randn(777, 300, device="cuda")
    hpart = torch.zeros(row_tiles(777, 512, 300) * 512, device="cuda")
    dH = gemm_psw(G, s2t, relu_mask=H, colsum_part=hpart)
    dHr = (G.double() @ W2.double()) * (Hr > 0)
    assert (dH.double() - dHr).abs().max().item() < 1e-4
    # 64-row column partials, as hsg_gemm_f32 writes them
    hpart_ref = torch.zeros_like(hpart)
    gemm(G, W2, relu_mask=H, splits=1, colsum_part=hpart_ref)
    assert torch.allclose(hpart.view(-1, 512).sum(0), hpart_ref.view(-1, 512).sum(0), rtol=1e-5, atol=1e-3)
    for t in range(row_tiles(777, 512, 300)):
        blk = dH[64 * t:64 * (t + 1)].double().sum(0)
        assert torch.allclose(hpart.view(-1, 512)[t].double(), blk, rtol=1e-6, atol=1e-3)
    acc = torch.randn(777, 300, device="cuda")
    acc0 = acc.clone()
    gemm_psw(dH, s1t, out=acc, add=acc)
    accr = acc0.double() + dH.double() @ W1.double()
    assert (acc.double() - accr).abs().max().item() < 2e-3


@pytest.mark.parametrize("M", [19200, 28800, 10001])
def test_resident_b_gemm(M, monkeypatch):
    """Dev-only k_gemm12 (HSG_GEMM12=1; the wide FFN GEMMs with K <= 320, B resident in
    LDS, A straight to registers; measured slower than k_gemm7): C within the split's
    fp32 class of fp64 for the bias + ReLU and the ReLU-mask epilogues, 32-row column
    partials equal to the band sums, and C bitwise equal to k_gemm7 (same fragments,
    same product order) with the same column totals."""
    from hetersumgraph_amd.dense import gemm_psw, psw_row_tiles, split_weights
    from helpers import dev_lib
    if not dev_lib():
        pytest.skip("k_gemm12 is in the dev library only (HSG_LIB_PATH=.../libhsg_dev.so)")
    monkeypatch.setenv("HSG_GEMM12", "1")
    torch.manual_seed(M)
    N, K = 512, 300
    X = torch.randn(M, K, device="cuda")
    W1 = torch.randn(N, K, device="cuda") * 0.05
    W2 = torch.randn(K, N, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    s1, s2t = split_weights((W1, False), (W2, True))
    rt = psw_row_tiles(M, N, K)
    assert rt == (M + 31) // 32
    H = gemm_psw(X, s1, bias=b, relu=True)
    Hr = torch.relu(X.double() @ W1.double().t() + b.double())
    unit = X.double().abs() @ W1.double().abs().t() + b.double().abs()
    assert ((H.double() - Hr).abs() / unit).max().item() < 2e-6
    G = torch.randn(M, K, device="cuda")
    part = torch.full((rt, N), float("nan"), device="cuda")
    dH = gemm_psw(G, s2t, relu_mask=H, colsum_part=part)
    dHr = (G.double() @ W2.double()) * (H.double() > 0)
    unit = (G.double().abs() @ W2.double().abs())
    assert ((dH.double() - dHr).abs() / unit).max().item() < 2e-6
    bands = torch.nn.functional.pad(dH.double(), (0, 0, 0, rt * 32 - M)).view(rt, 32, N).sum(1)
    assert torch.allclose(part.double(), bands, rtol=1e-6, atol=1e-4)
    monkeypatch.setenv("HSG_GEMM12", "0")
    assert psw_row_tiles(M, N, K) == (M + 63) // 64
    part7 = torch.zeros((M + 63) // 64, N, device="cuda")
    assert torch.equal(gemm_psw(X, s1, bias=b, relu=True), H)
    assert torch.equal(gemm_psw(G, s2t, relu_mask=H, colsum_part=part7), dH)
    assert torch.allclose(part7.sum(0), part.sum(0), rtol=1e-5, atol=1e-3)


def test_psw_rejects_bad_operands():
    from hetersumgraph_amd._lib import HSG_EINVAL, load
    lib = load()
    A = torch.randn(64, 30, device="cuda")            # K % 4 != 0
    planes = torch.empty(3 * 128 * 32, dtype=torch.bfloat16, device="cuda")
    C = torch.empty(64, 64, device="cuda")
    assert lib.hsg_gemm_f32_psw(64, 64, 30, A.data_ptr(), 30, planes.data_ptr(), C.data_ptr(), 64, None, None,
                                0, 0, 0, None, None) == HSG_EINVAL


# ---- hsg_gemm_f32_slabs + hsg_slab_reduce (the stack's deferred reductions) ------
def test_slab_batch_sums_segments_in_one_launch():
    from hetersumgraph_amd.reduce import SlabBatch
    torch.manual_seed(3)
    b = SlabBatch()
    outs, refs = [], []
    # job 1: three segments (applications), pitch/offset into a [rows][3][d] slab
    d = 70
    parts = [torch.randn(r, 3, d, device="cuda") for r in (5, 17, 1)]
    for off in range(3):
        o = torch.full((d,), 7.0, device="cuda")
        for prt in parts:
            b.add(("ln", off), o, d, 3 * d, off * d, 1.0, False, prt, prt.shape[0])
        outs.append(o)
        refs.append(sum(prt[:, off].double().sum(0) for prt in parts))
    # job 2: scaled, accumulating, more than 4 segments (chained launches)
    o2 = torch.randn(1000, device="cuda")
    base = o2.double().clone()
    segs = [torch.randn(r, 1000, device="cuda") for r in (3, 9, 1, 4, 2, 8)]
    for sg in segs:
        b.add("w", o2, 1000, 1000, 0, 0.5, True, sg, sg.shape[0])
    b.flush()
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.allclose(o.double(), r, rtol=1e-5, atol=1e-4)
    r2 = base + 0.5 * sum(sg.double().sum(0) for sg in segs)
    assert torch.allclose(o2.double(), r2, rtol=1e-5, atol=1e-4)


def test_gemm_slabs_reduce_to_the_product():
    from hetersumgraph_amd.dense import gemm_slabs
    from hetersumgraph_amd.reduce import SlabBatch
    torch.manual_seed(4)
    A = torch.randn(9000, 300, device="cuda")
    B = torch.randn(9000, 512, device="cuda")
    ws, splits = gemm_slabs(A, B, a_t=True)
    assert splits > 1
    out = torch.empty(300, 512, device="cuda")
    b = SlabBatch()
    b.add("dw", out.view(-1), 300 * 512, 300 * 512, 0, 1.0, False, ws, splits)
    b.flush()
    R = A.double().t() @ B.double()
    assert (out.double() - R).abs().max().item() < 2e-3


def test_slab_batch_staged_rows():
    """out_rows > 1: row b of the output sums the b-th of out_rows equal row ranges of
    every segment (the attention-parameter stage layout)."""
    from hetersumgraph_amd.reduce import SlabBatch
    torch.manual_seed(6)
    segs = [torch.randn(r, 88, device="cuda") for r in (4096, 301, 7)]
    R = 64
    out = torch.empty(R * 88, device="cuda")
    b = SlabBatch()
    for sg in segs:
        b.add("stage", out, 88, 88, 0, 1.0, False, sg, sg.shape[0], out_rows=R)
    b.flush()
    ref = torch.zeros(R, 88, dtype=torch.float64, device="cuda")
    for sg in segs:
        per = (sg.shape[0] + R - 1) // R
        for r in range(R):
            ref[r] += sg[r * per:(r + 1) * per].double().sum(0)
    assert torch.allclose(out.view(R, 88).double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("cols,pitch,coff,out_rows", [(1000, 1000, 0, 1), (300, 904, 300, 1), (88, 88, 0, 64),
                                                      (70, 210, 70, 1)])
def test_slab_reduce_float4_columns_bitwise_equal_scalar(cols, pitch, coff, out_rows, monkeypatch):
    """hsg_slab_reduce reads 16-byte column pieces when the job's geometry is aligned
    (cols, pitch, offset multiples of 4); the per-column summation order is the scalar
    form's, so the sums are bitwise equal (HSG_SLAB_VEC=1 forces the scalar form: dev library)."""
    skip_unless_dev(False)
    from hetersumgraph_amd.reduce import SlabBatch
    torch.manual_seed(7)
    segs = [torch.randn(r, pitch, device="cuda") for r in (4096, 301, 7, 64)]

    def run():
        out = torch.full((out_rows * cols,), 3.0, device="cuda")
        b = SlabBatch()
        for sg in segs:
            b.add("j", out, cols, pitch, coff, 0.75, True, sg, sg.shape[0], out_rows=out_rows)
        b.flush()
        torch.cuda.synchronize()
        return out

    vec = run()
    monkeypatch.setenv("HSG_SLAB_PRED", "0")        # dev: clamped loads of rows past a range
    pred = run()
    monkeypatch.setenv("HSG_SLAB_VEC", "1")
    scalar = run()
    assert torch.equal(vec, scalar)
    assert torch.equal(vec, pred)
    per = [(sg.shape[0] + out_rows - 1) // out_rows for sg in segs]
    ref = torch.full((out_rows, cols), 3.0, dtype=torch.float64, device="cuda")
    for sg, pr in zip(segs, per):
        for r in range(out_rows):
            ref[r] += 0.75 * sg[r * pr:(r + 1) * pr, coff:coff + cols].double().sum(0)
    assert torch.allclose(vec.view(out_rows, cols).double(), ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,N,K", [(19200, 512, 300), (1000, 300, 512), (777, 64, 300), (33, 20, 20)])
def test_psw_bf16_mode_is_the_rounded_product(M, N, K):
    """bf16 GEMM mode on the pre-split weight (hsg_gemm_bf16_psw; plane 0 = RNE(W)):
    equals an fp32 GEMM of the bf16-rounded operands up to summation order, and agrees
    with hsg_gemm_bf16 on the unsplit weight (which it falls back to for ragged N)."""
    from hetersumgraph_amd.dense import gemm, gemm_dtype, gemm_psw, split_weights
    torch.manual_seed(M + N)
    A = mk(M, K)
    W = mk(N, K)
    with gemm_dtype("bf16"):
        (S,) = split_weights((W, False))
        assert S.mode == "bf16"
        b = torch.randn(N, device="cuda")
        C = gemm_psw(A, S, bias=b, relu=True)
        C2 = gemm(A, W, b_t=True, bias=b, relu=True)
    ref = torch.relu(A.bfloat16().double() @ W.bfloat16().double().t() + b.double())
    scale = max(1.0, ref.abs().max().item())
    assert (C.double() - ref).abs().max().item() <= 1e-5 * scale * max(1.0, K ** 0.5)
    assert (C2.double() - ref).abs().max().item() <= 1e-5 * scale * max(1.0, K ** 0.5)


# ---- hsg_gemm_dw_slabs: a layer's two FFN weight gradients in one launch ------------
DW_PAIRS = [((38400, 300, 512), None),            # cfg2 S2W: dW2 = dY^T H, dW1 = dH^T X
            ((3360, 64, 512), None),              # cfg2 W2S
            ((1000, 20, 36), None),               # K tail (1000 = 31.25 tiles), ragged tiles
            ((4096, 300, 512), 3)]                # explicit splits


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("shape,splits", DW_PAIRS)
def test_dw_slabs_pair(shape, splits, dtype):
    """Both weight gradients of a layer in ONE hsg_gemm_dw_slabs launch, slabs summed by
    hsg_slab_reduce: 'f32' fp32-class per element (|err| / sum_k |a_k b_k| < 2e-6, the
    split GEMM's bound), 'bf16' equal to an fp64 GEMM of the RNE-rounded operands up to
    fp32 summation (< 2e-6 of sum |a b|); the pair's second job is the transposed shape."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_dw_slabs
    from hetersumgraph_amd.reduce import SlabBatch
    K, d, dh = shape
    torch.manual_seed(K + d)
    A1, B1 = mk(K, d), mk(K, dh)                    # dW2 = A1^T B1: [d, dh]
    A2, B2 = mk(K, dh), mk(K, d)                    # dW1 = A2^T B2: [dh, d]
    A1 = A1 * torch.exp(torch.randn_like(A1))
    with gemm_dtype(dtype):
        res = gemm_dw_slabs([(A1, B1), (A2, B2)], splits=splits)
    assert res is not None
    b = SlabBatch()
    outs = []
    for q, ((A, B), (ws, sp)) in enumerate(zip([(A1, B1), (A2, B2)], res)):
        if splits is not None:
            assert sp == splits
        out = torch.full((A.shape[1] * B.shape[1],), 7.0, device="cuda")
        b.add(q, out, out.numel(), out.numel(), 0, 1.0, False, ws, sp)
        outs.append(out.view(A.shape[1], B.shape[1]))
    b.flush()
    torch.cuda.synchronize()
    for (A, B), C in zip([(A1, B1), (A2, B2)], outs):
        a64, b64 = A.double(), B.double()
        if dtype == "bf16":
            a64, b64 = A.bfloat16().double(), B.bfloat16().double()
        ref, unit = a64.t() @ b64, a64.abs().t() @ b64.abs()
        err = ((C.double() - ref).abs() / unit.clamp_min(1e-30)).max().item()
        print(f"{dtype} K={K} {A.shape[1]}x{B.shape[1]}: max err / sum|ab| = {err:.2e}")
        assert err < 2e-6


# ---- k_gemm11: one round of big tiles for the cfg2-class FFN GEMMs -------------------
BIG_SHAPES = [(19200, 512, 300), (19200, 300, 512), (18000, 512, 300), (20000, 300, 512)]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("M,N,K", BIG_SHAPES)
def test_big_tile_psw_epilogues(M, N, K, dtype, monkeypatch):
    """The pre-split-weight GEMM on the cfg2-class shapes, where hsg_gemm_*_psw runs one
    round of 160 x 256 / 192 x 160 tiles (k_gemm11; hsg_gemm_psw_row_tiles reports its
    80- / 48-row column-partial bands): every epilogue the FFN uses -- bias + ReLU,
    ReLU' mask with column partials, accumulate, and the ELU-gate epilogue -- against
    fp64 ('f32': fp32-class, |err| / sum_k |a_k b_k| < 2e-6; 'bf16': the GEMM of the
    RNE-rounded operands).  Dev library with HSG_GEMM11=1 (measured slower than k_gemm7)."""
    skip_unless_dev(False)
    monkeypatch.setenv("HSG_GEMM11", "1")
    from hetersumgraph_amd.dense import gemm_dtype, gemm_psw, gemm_psw_elug, psw_row_tiles, split_weights
    torch.manual_seed(M + N)
    A = mk(M, K)
    W = mk(N, K) * 0.5
    with gemm_dtype(dtype):
        (S,) = split_weights((W, False))
    rt = psw_row_tiles(M, N, K, dtype)
    assert rt == (M + (159 if N > 320 else 191)) // (160 if N > 320 else 192) * (2 if N > 320 else 4)
    a64 = A.double() if dtype == "f32" else A.bfloat16().double()
    w64 = W.double() if dtype == "f32" else W.bfloat16().double()
    ref, unit = a64 @ w64.t(), a64.abs() @ w64.abs().t()
    tol = 2e-6

    def rel(C, R):
        return ((C.double() - R).abs() / unit.clamp_min(1e-30)).max().item()

    bias = torch.randn(N, device="cuda")
    C = gemm_psw(A, S, bias=bias, relu=True)
    assert rel(C, torch.relu(ref + bias.double())) < tol
    mask = torch.randn(M, N, device="cuda")
    hpart = torch.empty(rt, N, device="cuda")
    C = gemm_psw(A, S, relu_mask=mask, colsum_part=hpart)
    R = torch.where(mask.double() > 0, ref, torch.zeros_like(ref))
    assert rel(C, R) < tol
    colsum = hpart.double().sum(0)
    assert (colsum - C.double().sum(0)).abs().max().item() <= 1e-4 * max(1.0, C.double().abs().sum(0).max().item())
    add = torch.randn(M, N, device="cuda")
    C = gemm_psw(A, S, add=add.clone())
    assert rel(C, ref + add.double()) < tol
    # ELU gate: x = elu(h) + origin, G = dx * elu'(h) from e = x - origin
    origin = torch.randn(M, N, device="cuda")
    h = 2 * torch.randn(M, N, device="cuda")
    x = torch.nn.functional.elu(h) + origin
    out, G = add.clone(), torch.empty(M, N, device="cuda")
    assert gemm_psw_elug(A, S, out, x, origin, G)
    assert rel(out, ref + add.double()) < tol
    e = x.double() - origin.double()
    gref = torch.where(e > 0, out.double(), out.double() * (e + 1))
    assert (G.double() - gref).abs().max().item() <= 1e-6 * max(1.0, gref.abs().max().item())


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("M,p_drop", [(19200, 0.1), (19200, 0.0), (28800, 0.1), (17000, 0.1)])
def test_psw_ln_epilogue_equals_gemm_plus_ln(M, p_drop, dtype):
    """hsg_gemm_psw_ln (the wide FFN's second GEMM with dropout + residual + LayerNorm in
    its epilogue, GATLayer.py:39-42) against gemm_psw + hsg_ln_fwd on the same operands
    and dropout stream: y, out, mean and rstd bitwise equal (the same accumulation and
    the arithmetic of k_ln_fwd4).  Dev library (measured break-even: the product
    library declines and the FFN runs the GEMM and hsg_ln_fwd)."""
    skip_unless_dev(False)
    from hetersumgraph_amd import rng as hsg_rng
    from hetersumgraph_amd._lib import load, ptr, stream_of
    from hetersumgraph_amd.dense import gemm_dtype, gemm_psw, gemm_psw_ln, split_weights
    N, K = 300, 512
    torch.manual_seed(M)
    Hm = torch.relu(torch.randn(M, K, device="cuda"))
    W2 = torch.randn(N, K, device="cuda") / K ** 0.5
    b2, gamma, beta = (torch.randn(N, device="cuda") for _ in range(3))
    x = torch.randn(M, N, device="cuda")
    with gemm_dtype(dtype):
        (S,) = split_weights((W2, False))
    hsg_rng.manual_seed(77)
    seed_t, off = hsg_rng.get(x.device).take() if p_drop > 0 else (None, 0)
    y1, out1 = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
    mean1, rstd1 = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    from hetersumgraph_amd._lib import path_options
    with path_options(HSG_FFN_LN_EPI="1"):
        assert gemm_psw_ln(Hm, S, b2, x, gamma, beta, 1e-5, p_drop, seed_t, off, y1, out1, mean1, rstd1)
    y2 = gemm_psw(Hm, S, bias=b2)
    out2, mean2, rstd2 = torch.empty_like(out1), torch.empty_like(mean1), torch.empty_like(rstd1)
    lib = load()
    assert lib.hsg_ln_fwd(M, N, ptr(y2), ptr(x), ptr(gamma), ptr(beta), 1e-5, float(p_drop), ptr(seed_t), off,
                          ptr(out2), ptr(mean2), ptr(rstd2), stream_of(x)) == 0
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.equal(mean1, mean2) and torch.equal(rstd1, rstd2)
    assert torch.equal(out1, out2)


def test_psw_ln_declines_without_plan():
    from hetersumgraph_amd.dense import gemm_psw_ln, split_weights
    M, N, K = 1000, 300, 512                      # 11 tiles: far from one round of the GPU
    A = torch.randn(M, K, device="cuda")
    (S,) = split_weights((torch.randn(N, K, device="cuda"), False))
    t = torch.empty(M, N, device="cuda")
    v = torch.ones(N, device="cuda")
    assert not gemm_psw_ln(A, S, v, t, v, v, 1e-5, 0.0, None, 0, t.clone(), t.clone(), torch.empty(M, device="cuda"),
                           torch.empty(M, device="cuda"))


# ---- the bf16 mode on bf16 activations (round 5) -----------------------------------
def _bf16_rows(t, pad_to=8):
    """t as bf16 rows with the pitch rounded up to ``pad_to`` (zeros in the pad)."""
    n, d = t.shape
    ld = (d + pad_to - 1) // pad_to * pad_to
    buf = torch.zeros(n, ld, dtype=torch.bfloat16, device=t.device)
    buf[:, :d] = t.bfloat16()
    return buf[:, :d]


@pytest.mark.parametrize("M,N,K", [(28800, 512, 300), (28800, 300, 512), (777, 512, 300), (130, 64, 96)])
def test_bf16_io_gemms_bitwise_equal_fp32_io(M, N, K):
    """hsg_gemm_bf16_psw_io against hsg_gemm_bf16_psw on the same values: a bf16 A
    (io 1) holds exactly what the fp32-A path rounds at fragment read, a bf16 C (io 2)
    is the fp32 result rounded to nearest even, a bf16 relu' mask (io 4) gates as the
    fp32 one (RNE keeps the sign): bitwise equal, column partials too."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_psw, psw_row_tiles, split_weights
    torch.manual_seed(M + N + K)
    A = mk(M, K)
    Ab = _bf16_rows(A)
    A_r = Ab.float().contiguous()                       # the same values as fp32 rows
    W = mk(N, K) * 0.5
    with gemm_dtype("bf16"):
        (S,) = split_weights((W, False))
    bias = torch.randn(N, device="cuda")
    # io 2: x W^T + b, relu -> bf16 C
    ref = gemm_psw(A, S, bias=bias, relu=True)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    gemm_psw(A, S, bias=bias, relu=True, out=Cb)
    assert torch.equal(Cb, ref.bfloat16())
    # io 1: bf16 A -> fp32 C
    assert torch.equal(gemm_psw(Ab, S, bias=bias), gemm_psw(A_r, S, bias=bias))
    # io 7: bf16 A, bf16 relu' mask, bf16 C, column partials
    Hm = torch.randn(M, N, device="cuda")
    rt = psw_row_tiles(M, N, K, "bf16")
    p1, p2 = torch.empty(rt, N, device="cuda"), torch.empty(rt, N, device="cuda")
    ref = gemm_psw(A_r, S, relu_mask=Hm.bfloat16().float(), colsum_part=p1)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    gemm_psw(Ab, S, relu_mask=Hm.bfloat16(), colsum_part=p2, out=Cb)
    torch.cuda.synchronize()
    assert torch.equal(Cb, ref.bfloat16()) and torch.equal(p1, p2)


@pytest.mark.parametrize("M", [28800, 777])
def test_bf16_io_elug_rho_bitwise(M):
    """The dx GEMM with the ELU gate and rho on a bf16 dH (hsg_gemm_bf16_psw_elug_rho_a16)
    against the fp32-A call on the same values: bitwise equal dx, G and rho."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_psw_elug, split_weights
    N, K, D = 300, 512, 50
    torch.manual_seed(M)
    dH = torch.randn(M, K, device="cuda")
    dHb = _bf16_rows(dH)
    W1 = torch.randn(K, N, device="cuda") / K ** 0.5
    with gemm_dtype("bf16"):
        (S,) = split_weights((W1, True))
    ds = torch.randn(M, N, device="cuda")
    origin = torch.randn(M, N, device="cuda")
    x = torch.nn.functional.elu(2 * torch.randn(M, N, device="cuda")) + origin
    outs = []
    for A, gdt in ((dHb.float().contiguous(), torch.float32), (dHb, torch.float32), (dHb, torch.bfloat16)):
        out, G = ds.clone(), torch.empty_like(ds, dtype=gdt)
        rho = torch.empty(M, (N + 63) // 64, 3, device="cuda")          # the bf16 mode: 64-column groups
        assert gemm_psw_elug(A, S, out, x, origin, G, rho, D)
        outs.append((out, G, rho))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    # G as bf16 rows: the fp32 G rounded to nearest even; dx and rho (from the fp32 G) unchanged
    assert torch.equal(outs[2][0], outs[0][0]) and torch.equal(outs[2][2], outs[0][2])
    assert torch.equal(outs[2][1], outs[0][1].bfloat16())


@pytest.mark.parametrize("n,p_drop", [(28800, 0.1), (1001, 0.0)])
def test_ln_bwd_bf16_dy_bitwise(n, p_drop):
    """hsg_ln_bwd_dy16: dy stored as bf16 rows (pitch 304, zero pad) = RNE of
    hsg_ln_bwd's fp32 dy; dx and the dgamma / dbeta / db2 partials bitwise equal."""
    from hetersumgraph_amd import rng as hsg_rng
    from hetersumgraph_amd._lib import load, ptr
    lib = load()
    d = 300
    torch.manual_seed(n)
    dout, y, x = (torch.randn(n, d, device="cuda") for _ in range(3))
    gamma = 1 + 0.1 * torch.randn(d, device="cuda")
    mean, rstd = torch.randn(n, device="cuda"), torch.rand(n, device="cuda") + 0.5
    hsg_rng.manual_seed(5)
    seed_t, off = hsg_rng.get(x.device).take() if p_drop > 0 else (None, 0)
    nb = lib.hsg_ln_bwd_blocks(n)
    dy, dx, part = torch.empty_like(x), torch.empty_like(x), x.new_empty(nb, 3, d)
    assert lib.hsg_ln_bwd(n, d, ptr(dout), ptr(y), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), p_drop, ptr(seed_t),
                          off, ptr(dy), ptr(dx), ptr(part), None) == 0
    dyb = torch.full((n, 304), float("nan"), device="cuda").bfloat16()
    dx2, part2 = torch.empty_like(x), torch.empty_like(part)
    assert lib.hsg_ln_bwd_dy16(n, d, ptr(dout), ptr(y), 0, ptr(x), ptr(gamma), ptr(mean), ptr(rstd), p_drop,
                               ptr(seed_t), off, ptr(dyb), 304, ptr(dx2), ptr(part2), None) == 0
    torch.cuda.synchronize()
    assert torch.equal(dyb[:, :d], dy.bfloat16()) and torch.equal(dyb[:, d:].float(), torch.zeros(n, 4, device="cuda"))
    assert torch.equal(dx, dx2) and torch.equal(part, part2)


def test_dw_pair_bf16_operands_bitwise():
    """hsg_gemm_dw_slabs_io (bf16 dY, H, dH; fp32 X) against hsg_gemm_dw_slabs in the
    bf16 mode on the same values: bitwise equal partial slabs."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_dw_slabs
    K, d, dh = 38400, 300, 512
    torch.manual_seed(3)
    DY = _bf16_rows(torch.randn(K, d, device="cuda"))
    Hh = torch.randn(K, dh, device="cuda").bfloat16()
    DH = torch.randn(K, dh, device="cuda").bfloat16()
    X = torch.randn(K, d, device="cuda")
    with gemm_dtype("bf16"):
        a = gemm_dw_slabs([(DY, Hh), (DH, X)])
        b = gemm_dw_slabs([(DY.float().contiguous(), Hh.float()), (DH.float(), X)])
    torch.cuda.synchronize()
    assert a is not None and b is not None
    for (wa, sa), (wb, sb) in zip(a, b):
        assert sa == sb and torch.equal(wa, wb)


@pytest.mark.parametrize("n,p_drop", [(28800, 0.1), (1001, 0.0)])
def test_ln_fwd_bf16_y_equals_fp32_on_the_same_values(n, p_drop):
    """hsg_ln_fwd_y16 (the bf16 mode's bf16 LayerNorm input y) against hsg_ln_fwd on
    the same (bf16-rounded) y: out, mean, rstd bitwise equal; and hsg_ln_bwd_dy16 with
    y_bf16 against y_bf16 = 0 on the fp32 copy of those values."""
    from hetersumgraph_amd import rng as hsg_rng
    from hetersumgraph_amd._lib import load, ptr
    lib = load()
    d = 300
    torch.manual_seed(n + 1)
    yb = torch.randn(n, d, device="cuda").bfloat16()
    yf = yb.float().contiguous()
    x = torch.randn(n, d, device="cuda")
    gamma, beta = 1 + 0.1 * torch.randn(d, device="cuda"), 0.1 * torch.randn(d, device="cuda")
    hsg_rng.manual_seed(9)
    seed_t, off = hsg_rng.get(x.device).take() if p_drop > 0 else (None, 0)
    outs = []
    for y, f in ((yf, lib.hsg_ln_fwd), (yb, lib.hsg_ln_fwd_y16)):
        out, mean, rstd = torch.empty_like(x), x.new_empty(n), x.new_empty(n)
        assert f(n, d, ptr(y), ptr(x), ptr(gamma), ptr(beta), 1e-5, p_drop, ptr(seed_t), off, ptr(out), ptr(mean),
                 ptr(rstd), None) == 0
        outs.append((out, mean, rstd))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    mean, rstd = outs[0][1], outs[0][2]
    dout = torch.randn(n, d, device="cuda")
    nb = lib.hsg_ln_bwd_blocks(n)
    res = []
    for y, flag in ((yf, 0), (yb, 1)):
        dy = torch.zeros(n, 304, device="cuda").bfloat16()
        dx, part = torch.empty_like(x), x.new_empty(nb, 3, d)
        assert lib.hsg_ln_bwd_dy16(n, d, ptr(dout), ptr(y), flag, ptr(x), ptr(gamma), ptr(mean), ptr(rstd), p_drop,
                                   ptr(seed_t), off, ptr(dy), 304, ptr(dx), ptr(part), None) == 0
        res.append((dy, dx, part))
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.equal(a, b)
