"""Per-head-dropout head projection kernels vs a PyTorch fp64 reference that uses
the same keep-mask bits (fwd, dX, dW), plus mask statistics."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def unpack(bits, n):
    """[H, NWI, in] int32 words (32 rows per word) -> bool [H, n, in]."""
    H, NWI, d_in = bits.shape
    b = bits.to(torch.int64) & 0xFFFFFFFF
    j = torch.arange(32, device=bits.device)
    m = ((b.unsqueeze(-1) >> j) & 1).bool()                   # [H, NWI, in, 32]
    return m.permute(0, 1, 3, 2).reshape(H, NWI * 32, d_in)[:, :n]


@pytest.mark.parametrize("n,d_in,H,D", [(19200 // 4, 300, 8, 8), (1120, 64, 6, 50), (333, 70, 3, 16),
                                         (65, 33, 1, 64), (200, 40, 3, 5), (130, 50, 2, 75),
                                         (97, 300, 16, 25), (1000, 64, 16, 4), (257, 128, 3, 16),
                                         (70, 300, 8, 8), (19200, 300, 8, 8), (100, 20, 2, 8), (50, 304, 4, 12),
                                         (33, 8, 16, 4)])
def test_head_projection_matches_masked_reference(n, d_in, H, D):
    from hetersumgraph_amd import _lib, rng
    from hetersumgraph_amd.hproj import _HeadProj
    p = 0.1
    torch.manual_seed(n)
    X = torch.randn(n, d_in, device="cuda", requires_grad=True)
    W = (torch.randn(H * D, d_in, device="cuda") / d_in ** 0.5).requires_grad_()
    r = rng.get("cuda")
    off0 = r.offset
    Z = _HeadProj.apply(X, W, H, D, p)
    R = torch.randn_like(Z)
    (Z * R).sum().backward()
    # regenerate the same bits: same seed, same offset
    r.offset = off0
    from hetersumgraph_amd.hproj import dropmask_bits
    bits = dropmask_bits(X.detach(), H, p)
    keep = unpack(bits, n).double()                            # [H, n, d_in]
    scale = 1.0 / (1.0 - float(int(p * 65536)) / 65536)
    rate = 1 - keep.mean().item()
    assert abs(rate - p) < 0.01 + 3 / (n * d_in * H) ** 0.5, rate
    Xd = X.detach().double().requires_grad_()
    Wd = W.detach().double().requires_grad_()
    Zr = torch.einsum("kic,kdc->ikd", keep * Xd.unsqueeze(0) * scale, Wd.view(H, D, d_in)).reshape(n, H * D)
    (Zr * R.double()).sum().backward()
    assert (Z.detach().double() - Zr.detach()).abs().max().item() < 1e-4
    assert (X.grad.double() - Xd.grad).abs().max().item() < 1e-4 * max(1, Xd.grad.abs().max().item())
    assert (W.grad.double() - Wd.grad).abs().max().item() < 1e-4 * max(1, Wd.grad.abs().max().item())


def test_masks_independent_across_heads_and_calls():
    from hetersumgraph_amd.hproj import dropmask_bits
    X = torch.randn(4096, 300, device="cuda")
    a = unpack(dropmask_bits(X, 8, 0.1), 4096).float()
    b = unpack(dropmask_bits(X, 8, 0.1), 4096).float()
    # heads differ from each other and calls differ from each other
    assert (a[0] != a[1]).float().mean().item() > 0.1
    assert (a != b).float().mean().item() > 0.1
    # pairwise independence: P(keep_k and keep_j) ~ (1-p)^2
    both = (a[0] * a[1]).mean().item()
    assert abs(both - 0.81) < 0.01


@pytest.mark.parametrize("n,d_in,H,D", [(19200 // 8, 300, 8, 8), (1120, 64, 6, 50), (333, 72, 3, 16), (77, 40, 2, 64),
                                         (130, 20, 4, 5), (50, 16, 1, 33)])
def test_fused_source_logits_match_split_kernel(n, d_in, H, D):
    """hsg_hproj_fwd_logits: Z is bitwise the plain projection's, and sigma = <Z_k, a1_k>
    agrees with the split hsg_attn_src_logits to fp32 summation-order noise; shapes
    whose slots do not fit a wave's slot group (ceil(D/16) = 3) fall back (None)."""
    from hetersumgraph_amd import _lib, rng
    from hetersumgraph_amd.hproj import hproj_fwd
    torch.manual_seed(n + D)
    X = torch.randn(n, d_in, device="cuda")
    W = torch.randn(H * D, d_in, device="cuda") / d_in ** 0.5
    a1 = torch.randn(H, D, device="cuda")
    rng.manual_seed(3)
    Z0, _ = hproj_fwd(X, W, H, D, 0.1)
    rng.manual_seed(3)
    Z1, _, sigma = hproj_fwd(X, W, H, D, 0.1, a1=a1)
    torch.cuda.synchronize()
    assert torch.equal(Z0, Z1)
    if (D + 15) // 16 == 3:
        assert sigma is None
        return
    lib = _lib.load()
    ref = torch.empty(n, H, device="cuda")
    _lib.check(lib.hsg_attn_src_logits(n, H, D, Z0.data_ptr(), a1.data_ptr(), ref.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream), "logits")
    torch.cuda.synchronize()
    tol = 1e-5 * max(1.0, ref.abs().max().item())
    assert (sigma - ref).abs().max().item() <= tol


def test_batched_dropmask_equals_single_launches():
    """hsg_dropmask_multi (the fused stack's one launch for all its head projections)
    draws bit-for-bit the masks of one hsg_dropmask launch per job."""
    from hetersumgraph_amd._lib import load, ptr, stream_of
    from hetersumgraph_amd.hproj import dropmasks
    lib = load()
    seed = torch.tensor([12345], dtype=torch.int64, device="cuda")
    jobs = [(19200, 300, 8, 0.1, seed, 3), (1120, 64, 6, 0.1, seed, 5), (777, 33, 3, 0.4, seed, 9),
            (1, 1, 1, 0.5, seed, 11), (40, 300, 8, 0.0, seed, 12)]
    got = dropmasks(jobs, torch.device("cuda"), None)
    for (n, d_in, H, p, s, off), g in zip(jobs, got):
        ref = torch.empty(lib.hsg_dropmask_words(n, d_in, H), dtype=torch.int32, device="cuda")
        assert lib.hsg_dropmask(n, d_in, H, float(p), ptr(s), off, ptr(ref), None) == 0
        torch.cuda.synchronize()
        assert torch.equal(g, ref), (n, d_in, H, p, off)


@pytest.mark.parametrize("n,d_in,H,D", [(1120, 64, 6, 50), (333, 72, 3, 16), (65, 33, 1, 64), (130, 50, 2, 75),
                                         (200, 40, 3, 5), (19200 // 4, 300, 8, 8)])
def test_hproj_bwd_one_launch_equals_two(monkeypatch, n, d_in, H, D):
    """hsg_hproj_bwd (round 5: dX and the dW slabs of the S2W shape in ONE launch,
    k_hproj_bwd_hw) against hsg_hproj_dx + hsg_hproj_dw (HSG_HPROJ_BWD_MERGE=0, dev
    library): bitwise equal dX and partial slabs (shapes it does not merge take the
    two launches either way)."""
    from helpers import skip_unless_dev
    skip_unless_dev(False)
    from hetersumgraph_amd._lib import load, ptr
    from hetersumgraph_amd.hproj import dropmask_bits
    lib = load()
    torch.manual_seed(n + D)
    X = torch.randn(n, d_in, device="cuda")
    W = torch.randn(H * D, d_in, device="cuda") / d_in ** 0.5
    dZ = torch.randn(n, H * D, device="cuda")
    bits = dropmask_bits(X, H, 0.1)
    chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("HSG_HPROJ_BWD_MERGE", flag)
        dX = torch.full_like(X, 0.5)                              # accumulate onto it
        part = X.new_empty(chunks * H * D * d_in)
        assert lib.hsg_hproj_bwd(n, d_in, H, D, ptr(dZ), H * D, ptr(W), ptr(X), d_in, ptr(bits), 0.1, ptr(dX), d_in,
                                 1, ptr(part), None) == 0
        outs.append((dX, part))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("n,d_in,H,D,acc", [(19200, 300, 8, 8, 1), (19200, 300, 8, 8, 0), (4800, 300, 8, 8, 1),
                                             (2570, 300, 5, 8, 0), (1001, 68, 8, 8, 1)])
def test_narrow_bwd_one_launch_equals_dx_and_dw(n, d_in, H, D, acc):
    """hsg_hproj_bwd on the narrow-head (W2S) shape runs dX and the dW slabs in ONE
    launch (round 6, k_hproj_bwd_n8: the k_hproj_dx_n8 tiles and single-image
    k_hproj_dw_mf blocks) -- bitwise equal to hsg_hproj_dx + hsg_hproj_dw (product
    library: those entries launch the separate kernels)."""
    from hetersumgraph_amd._lib import load, ptr
    from hetersumgraph_amd.hproj import dropmask_bits
    lib = load()
    torch.manual_seed(n + H)
    X = torch.randn(n, d_in, device="cuda")
    W = torch.randn(H * D, d_in, device="cuda") / d_in ** 0.5
    dZ = torch.randn(n, H * D, device="cuda")
    bits = dropmask_bits(X, H, 0.1)
    chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
    dX1, dX2 = torch.full_like(X, 0.5), torch.full_like(X, 0.5)
    p1, p2 = X.new_empty(chunks * H * D * d_in), X.new_empty(chunks * H * D * d_in)
    assert lib.hsg_hproj_bwd(n, d_in, H, D, ptr(dZ), H * D, ptr(W), ptr(X), d_in, ptr(bits), 0.1, ptr(dX1), d_in,
                             acc, ptr(p1), None) == 0
    assert lib.hsg_hproj_dx(n, d_in, H, D, ptr(dZ), H * D, ptr(W), ptr(bits), 0.1, ptr(dX2), d_in, acc, None) == 0
    assert lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), 0.1, ptr(p2), None, 0, None) == 0
    torch.cuda.synchronize()
    assert torch.equal(dX1, dX2)
    assert torch.equal(p1, p2)


@pytest.mark.parametrize("n,d_in,H,D", [(19200, 300, 8, 8), (1000, 64, 16, 4), (257, 128, 3, 16), (70, 300, 8, 8)])
def test_dw_4x4x1_equals_16x16x4_kernel(monkeypatch, n, d_in, H, D):
    """The unpadded 4x4x1 dW kernel (k_hproj_dw_m4, round 5) against the 16x16x4 slot
    kernel on the same keep bits and the same row chunks (HSG_HPROJ_DWM4=0, dev
    library): fp32 summation-order noise only, relative to the summed magnitudes."""
    from helpers import skip_unless_dev
    skip_unless_dev(False)
    from hetersumgraph_amd._lib import load, ptr
    from hetersumgraph_amd.hproj import dropmask_bits
    lib = load()
    torch.manual_seed(n + d_in)
    X = torch.randn(n, d_in, device="cuda")
    dZ = torch.randn(n, H * D, device="cuda")
    bits = dropmask_bits(X, H, 0.1)
    outs = []
    monkeypatch.setenv("HSG_HPROJ_DWMF", "0")                 # off the round-5 bf16 limb kernel
    for flag in ("1", "0"):
        monkeypatch.setenv("HSG_HPROJ_DWM4", flag)
        chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
        part = X.new_empty(chunks * H * D * d_in)
        dW = X.new_empty(H * D, d_in)
        assert lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), 0.1, ptr(part), ptr(dW), 0,
                                None) == 0
        outs.append(dW)
    torch.cuda.synchronize()
    keep = unpack(bits, n).double()
    mag = torch.einsum("kic,ikd->kdc", keep * X.double().abs().unsqueeze(0),
                       dZ.double().abs().view(n, H, D)).reshape(H * D, d_in)
    err = ((outs[0].double() - outs[1].double()).abs() / mag.clamp_min(1e-30)).max().item()
    print(f"4x4x1 vs 16x16x4 dW: max |diff| / sum|terms| = {err:.2e}")
    assert err < 1e-6


@pytest.mark.parametrize("n,d_in,H", [(19200, 300, 8), (70, 300, 8), (100, 20, 2), (50, 304, 4), (33, 8, 5),
                                      (1000, 64, 8)])
def test_fwd_mfma_limbs_match_fp64_and_valu_kernel(n, d_in, H):
    """hsg_hproj_fwd_mf (D = 8 on bf16 limb MFMAs, W as hsg_wsplit planes) against the
    fp64 masked reference and the VALU kernel hsg_hproj_fwd_t8 on the same keep bits:
    Z and the fused source logits to fp32 rounding."""
    from hetersumgraph_amd._lib import load, ptr, stream_of
    from hetersumgraph_amd.dense import split_dims, split_weights
    from hetersumgraph_amd.hproj import dropmask_bits, transposed_weight
    lib = load()
    D, p = 8, 0.1
    torch.manual_seed(n + H)
    X = torch.randn(n, d_in, device="cuda")
    W = torch.randn(H * D, d_in, device="cuda") / d_in ** 0.5
    a1 = torch.randn(H, D, device="cuda")
    bits = dropmask_bits(X, H, p)
    (sw,) = split_weights((W, False))
    Np, Kp = split_dims(H * D, d_in)
    outs = []
    for kind in ("mf", "t8"):
        Z = torch.full((n, H * D), float("nan"), device="cuda")
        sg = torch.full((n, H), float("nan"), device="cuda")
        if kind == "mf":
            rc = lib.hsg_hproj_fwd_mf(n, d_in, H, ptr(X), d_in, ptr(sw.planes), Np, Kp, ptr(bits), p, ptr(Z), H * D,
                                      ptr(a1), ptr(sg), stream_of(X))
        else:
            wt = transposed_weight(W, H, D)
            rc = lib.hsg_hproj_fwd_t8(n, d_in, H, ptr(X), d_in, ptr(wt), ptr(bits), p, ptr(Z), H * D, ptr(a1),
                                      ptr(sg), stream_of(X))
        assert rc == 0
        outs.append((Z, sg))
    torch.cuda.synchronize()
    keep = unpack(bits, n).double()
    scale = 1.0 / (1.0 - float(int(p * 65536)) / 65536)
    Zr = torch.einsum("kic,kdc->ikd", keep * X.double().unsqueeze(0) * scale, W.double().view(H, D, d_in))
    sr = (Zr * a1.double().unsqueeze(0)).sum(-1)
    Zr = Zr.reshape(n, H * D)
    tol = 2e-6 * max(1.0, Zr.abs().max().item())
    for Z, sg in outs:
        assert (Z.double() - Zr).abs().max().item() < tol
        assert (sg.double() - sr).abs().max().item() < 4 * tol * max(1.0, a1.abs().max().item())


@pytest.mark.parametrize("n,d_in,H", [(19200, 300, 8), (70, 300, 8), (100, 20, 2), (50, 304, 4), (33, 8, 5),
                                      (1000, 64, 8), (4800, 300, 8)])
def test_dw_mfma_limbs_match_fp64(n, d_in, H):
    """hsg_hproj_dw for D = 8 (round 5: k_hproj_dw_mf, bf16 limb MFMAs, the keep byte
    through the LDS table) against the fp64 masked reference dW = s sum_i dZ_k^T (M_k o X),
    both as the summed partial slabs and through k_sum_parts: fp32 rounding relative to
    the summed magnitudes."""
    from hetersumgraph_amd._lib import load, ptr
    from hetersumgraph_amd.hproj import dropmask_bits
    lib = load()
    D, p = 8, 0.1
    torch.manual_seed(n + 7 * H)
    X = torch.randn(n, d_in, device="cuda")
    dZ = torch.randn(n, H * D, device="cuda")
    bits = dropmask_bits(X, H, p)
    chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
    part = torch.full((chunks * H * D * d_in,), float("nan"), device="cuda")
    dW = X.new_empty(H * D, d_in)
    assert lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), p, ptr(part), ptr(dW), 0,
                            None) == 0
    torch.cuda.synchronize()
    keep = unpack(bits, n).double()
    scale = 1.0 / (1.0 - float(int(p * 65536)) / 65536)
    ref = torch.einsum("kic,ikd->kdc", keep * X.double().unsqueeze(0), dZ.double().view(n, H, D)) * scale
    mag = torch.einsum("kic,ikd->kdc", keep * X.double().abs().unsqueeze(0), dZ.double().abs().view(n, H, D)) * scale
    ref, mag = ref.reshape(H * D, d_in), mag.reshape(H * D, d_in)
    assert torch.isfinite(part).all()
    sums = part.view(chunks, H * D, d_in).double().sum(0) * scale
    for got in (dW.double(), sums):
        err = ((got - ref).abs() / mag.clamp_min(1e-30)).max().item()
        assert err < 2e-6, err
