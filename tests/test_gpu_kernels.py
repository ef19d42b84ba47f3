"""Kernel-level GPU tests: each HIP entry point against an independent reference
(torch fp64 for the GEMM, the numpy oracle for the embedding/FM/pooling math).
Integer/index outputs (gathered rows, pooling counts) are compared bit-exact."""
import ctypes as C
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402


def _s():
    return _lib.stream_handle()


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(300, 400, 432), (257, 416, 400), (64, 10, 16), (1000, 128, 64),
                                   (256, 400, 448), (384, 416, 400), (128, 80, 16)])   # last three: FAST path
def test_gemm_f32_matches_fp64(hip_lib, ta, tb, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    r4 = lambda x: (x + 3) // 4 * 4
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    ref = A.double() @ B.double()
    # store in the requested orientations with padded leading dims (zero pads)
    if ta:
        lda = r4(M) + 4
        Ad = torch.zeros(K, lda); Ad[:, :M] = A.t()
    else:
        lda = r4(K) + 4
        Ad = torch.zeros(M, lda); Ad[:, :K] = A
    if tb:
        ldb = r4(K)
        Bd = torch.zeros(N, ldb); Bd[:, :K] = B.t()
    else:
        ldb = r4(N)
        Bd = torch.zeros(K, ldb); Bd[:, :N] = B
    Ad, Bd = Ad.cuda(), Bd.cuda()
    ldc = N + 3
    C = torch.full((M, ldc), 7.0, device="cuda")
    call("dl_gemm_f32", ta, tb, M, N, K, ptr(Ad), lda, ptr(Bd), ldb, ptr(C), ldc, 0, None, 0, 1, 0, _s())
    torch.cuda.synchronize()
    out = C[:, :N].double().cpu()
    scale = (A.abs().double() @ B.abs().double()).clamp(min=1.0)
    assert ((out - ref).abs() / scale).max().item() < 2e-6
    assert (C[:, N:].cpu() == 7.0).all()   # columns >= N untouched


def test_gemm_f32_epilogues_and_split(hip_lib):
    g = torch.Generator().manual_seed(1)
    M, N, K = 512, 80, 2048
    A = torch.randn(K, M, generator=g).cuda()     # stored [r][i] (ta=1)
    B = torch.randn(K, N, generator=g).cuda()
    ref = (A.t().double() @ B.double()).cpu()
    splits = 8
    slab = torch.zeros(splits, M, N, device="cuda")
    call("dl_gemm_f32", 1, 0, M, N, K, ptr(A), M, ptr(B), N, ptr(slab), N, 3, None, 0, splits, M * N, _s())
    torch.cuda.synchronize()
    assert torch.allclose(slab.double().sum(0).cpu(), ref, rtol=1e-5, atol=1e-3)
    # relu + mask epilogues
    X = torch.randn(M, K, generator=g).cuda()
    C = torch.zeros(M, N, device="cuda")
    call("dl_gemm_f32", 0, 0, M, N, K, ptr(X), K, ptr(B), N, ptr(C), N, 1, None, 0, 1, 0, _s())
    mask = torch.randn(M, N, generator=g).cuda()
    C2 = torch.zeros(M, N, device="cuda")
    call("dl_gemm_f32", 0, 0, M, N, K, ptr(X), K, ptr(B), N, ptr(C2), N, 2, ptr(mask), N, 1, 0, _s())
    torch.cuda.synchronize()
    r = (X.double() @ B.double())
    assert torch.allclose(C.double(), r.clamp(min=0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(C2.double(), torch.where(mask > 0, r, torch.zeros_like(r)), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,N,K,splits", [(416, 400, 8192, 8), (432, 400, 4096 + 16, 3), (208, 160, 65536, 64),
                                            (144, 80, 5000 * 4, 5), (416, 400, 65536, 64)])
def test_gemm_f32_tall_split_tiles(hip_lib, M, N, K, splits):
    """Weight-gradient products (ta=1, split-K slabs; M a multiple of 144 and N of 80 run
    on the tall 5-wave tiles, the others on the 128-row tiles with the wave skip): slab
    sums against fp64."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(K, M, generator=g).cuda()     # x stored [k][m]
    B = torch.randn(K, N, generator=g).cuda()     # dh stored [k][n]
    ref = (A.t().double() @ B.double()).cpu()
    slab = torch.full((splits, M, N), 7.0, device="cuda")
    call("dl_gemm_f32", 1, 0, M, N, K, ptr(A), M, ptr(B), N, ptr(slab), N, 3, None, 0, splits, M * N, _s())
    torch.cuda.synchronize()
    from deep_learning_amd.engine import _num_splits
    used = _num_splits(K, splits)
    got = slab[:used].double().sum(0).cpu()
    scale = (A.abs().t().double() @ B.abs().double()).cpu().clamp(min=1.0)
    assert ((got - ref).abs() / scale).max().item() < 2e-6


def _planes(W, transpose):
    """dl_split3 planes of the f32 matrix W [rows][cols] (or of W^T) as int16 [3][..]."""
    rows, cols = W.shape
    ld = rows if transpose else cols
    n = rows * cols
    P = torch.zeros(3 * n, dtype=torch.int16, device="cuda")
    call("dl_split3", ptr(W), rows, cols, cols, 1 if transpose else 0, ptr(P), ld, n, _s())
    return P


@pytest.mark.parametrize("kind", ["s3", "bf16"])
@pytest.mark.parametrize("rows,cols,reg_kind", [(432, 400, 0), (416, 400, 1), (37, 24, 0)])
def test_adam_dense_split3_equals_adam_then_split(hip_lib, rows, cols, reg_kind, kind):
    """dl_adam_dense_split3 (the tower weight's Adam update writing its own s3 planes) against
    dl_adam_dense_reg followed by the two dl_split3 launches it replaces: W, m, v and both plane
    layouts bit-identical, the regulariser sum (block atomics) within 1e-5 relative; a poisoned
    step leaves all unchanged."""
    g = torch.Generator().manual_seed(rows + cols + reg_kind)
    n = rows * cols
    nslab = 5
    W0 = (torch.randn(rows, cols, generator=g) * 0.05).cuda()
    m0 = (torch.randn(rows, cols, generator=g) * 1e-3).cuda()
    v0 = (torch.rand(rows, cols, generator=g) * 1e-6).cuda()
    slab = (torch.randn(nslab, n, generator=g) * 1e-3).cuda()
    opt = torch.zeros(_lib.OPT_LEN)
    opt[3], opt[4], opt[5], opt[6], opt[7] = 1e-3, 0.9, 0.999, 1e-8, 10
    out = []
    for fused in (False, True):
        W, m, v, o = W0.clone(), m0.clone(), v0.clone(), opt.clone().cuda()
        wp = torch.zeros(3 * n, dtype=torch.int16, device="cuda")
        wtp = torch.zeros(3 * n, dtype=torch.int16, device="cuda")
        if fused:
            call("dl_adam_dense_split3" if kind == "s3" else "dl_adam_dense_bf16", ptr(W), ptr(m), ptr(v), ptr(slab),
                 nslab, n, rows, cols, 1e-4, n - cols, reg_kind, ptr(o), ptr(o[8:]), ptr(wp), ptr(wtp), _s())
        else:
            call("dl_adam_dense_reg", ptr(W), ptr(m), ptr(v), ptr(slab), nslab, n, n, 1e-4, n - cols, reg_kind,
                 ptr(o), None, ptr(o[8:]), _s())
            if kind == "s3":
                call("dl_split3", ptr(W), rows, cols, cols, 0, ptr(wp), cols, n, _s())
                call("dl_split3", ptr(W), rows, cols, cols, 1, ptr(wtp), rows, n, _s())
            else:   # the bf16 tower's refresh (engine._refresh_wb)
                call("dl_cast_bf16", ptr(W), rows, cols, cols, ptr(wp), cols, _s())
                call("dl_transpose_bf16", ptr(W), 1, rows, cols, cols, ptr(wtp), rows, _s())
        torch.cuda.synchronize()
        out.append((W, m, v, o[8].item(), wp, wtp))
    for a, b in zip(out[0], out[1]):
        if isinstance(a, float):   # the regulariser sum: one float atomic per block, in any order
            assert abs(a - b) <= 1e-5 * abs(a)
        else:
            assert torch.equal(a, b)
    # a poisoned step (the step guard's skip word) applies nothing and writes no plane
    W, m, v, o = W0.clone(), m0.clone(), v0.clone(), opt.clone()
    o[_lib.OPT_SKIP] = 1
    o = o.cuda()
    wp = torch.full((3 * n,), 7, dtype=torch.int16, device="cuda")
    wtp = torch.full((3 * n,), 7, dtype=torch.int16, device="cuda")
    call("dl_adam_dense_split3" if kind == "s3" else "dl_adam_dense_bf16", ptr(W), ptr(m), ptr(v), ptr(slab), nslab,
         n, rows, cols, 1e-4, n - cols, reg_kind, ptr(o), ptr(o[8:]), ptr(wp), ptr(wtp), _s())
    torch.cuda.synchronize()
    assert torch.equal(W, W0) and torch.equal(m, m0) and (wp == 7).all() and (wtp == 7).all()


def test_split3_is_exact(hip_lib):
    """hi + mid + lo reconstructs every (normal) f32 exactly, each plane a bf16 rounding."""
    g = torch.Generator().manual_seed(3)
    W = (torch.randn(37, 24, generator=g) * torch.logspace(-20, 20, 24)).cuda()
    P = _planes(W, False).view(3, 37, 24)
    f = lambda t: (t.to(torch.int32) << 16).view(torch.float32)
    back = (f(P[0]) + f(P[1])) + f(P[2])
    assert torch.equal(back, W)
    assert torch.equal(f(P[0]), W.bfloat16().float())
    PT = _planes(W, True).view(3, 24, 37)
    # the transposed layout's rows have K = 37 (one whole 32-deep chunk): natural order back
    pos = torch.tensor([_s3_kpos(k, 37) for k in range(37)], device="cuda")
    assert torch.equal(PT[0][:, pos], P[0].t())
    # a whole-chunk row length in both layouts: K = 64 (W^T rows) and 96 (W rows)
    W2 = (torch.randn(64, 96, generator=g)).cuda()
    P2 = _planes(W2, False).view(3, 64, 96)
    PT2 = _planes(W2, True).view(3, 96, 64)
    p96 = torch.tensor([_s3_kpos(k, 96) for k in range(96)], device="cuda")
    p64 = torch.tensor([_s3_kpos(k, 64) for k in range(64)], device="cuda")
    assert torch.equal(P2[:, :, p96][0], PT2[:, :, p64][0].t())
    assert torch.equal(f(P2[0][:, p96]), W2.bfloat16().float())


def _s3_kpos(k, K):
    """Position of k in a plane row of length K (include/dlamd.h dl_split3, DL_S3_KPERM)."""
    if not _lib.lib().dl_s3_kperm() or (k | 31) >= K:
        return k
    kk = k & 31
    return (k & ~31) | (8 * (kk >> 2) + (kk & 3) if kk < 16 else 8 * ((kk - 16) >> 2) + 4 + (kk & 3))


@pytest.mark.parametrize("ldc_pad", [3, 4])   # ldc % 4 == 0 (pad 4, N % 4 == 0): the register epilogue
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(65536, 400, 432), (300, 400, 416), (257, 416, 400), (1000, 80, 64),
                                   (513, 16, 8), (100, 213, 40)])
def test_gemm_s3_nt_matches_fp64(hip_lib, epi, M, N, K, ldc_pad):
    """C = A . B^T (+ ReLU / ReluGrad mask) on the three-plane split, against fp64: the same
    2e-6 relative bound as the f32 kernel; columns past N untouched."""
    if M == 65536 and (epi == 2 or ldc_pad == 3):
        pytest.skip("one full-size case per epilogue pair is enough")
    g = torch.Generator().manual_seed(M + 3 * N + K + epi)
    lda = K + 4
    A = torch.zeros(M, lda)
    A[:, :K] = torch.randn(M, K, generator=g)
    Bm = torch.randn(N, K, generator=g) * 0.05
    ref = A[:, :K].double() @ Bm.double().t()
    scale = (A[:, :K].abs().double() @ Bm.abs().double().t()).clamp(min=1e-3)
    mask = torch.randn(M, N + 5, generator=g)
    if epi == 1:
        ref = ref.clamp(min=0)
    elif epi == 2:
        ref = torch.where(mask[:, :N] > 0, ref, torch.zeros_like(ref))
    Ad, mk = A.cuda(), mask.cuda()
    Bp = _planes(Bm.cuda(), False)     # B given as [N][K]: planes with ld K
    ldb = K
    ldc = N + ldc_pad
    C = torch.full((M, ldc), 7.0, device="cuda")
    call("dl_gemm_s3_nt", M, N, K, ptr(Ad), lda, ptr(Bp), ldb, N * K, ptr(C), ldc, epi,
         ptr(mk) if epi == 2 else None, N + 5, _s())
    torch.cuda.synchronize()
    out = C[:, :N].double().cpu()
    assert ((out - ref).abs() / scale).max().item() < 2e-6
    assert (C[:, N:].cpu() == 7.0).all()


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("M,N,K", [(65536, 400, 416), (300, 400, 416), (257, 213, 40), (513, 16, 8), (77, 48, 72)])
def test_gemm_s3_relu_bitmask_round_trip(hip_lib, M, N, K, aligned):
    """dl_gemm_s3_nt_bits: the ReLU forward writes bit (c & 15) of halfword [i][c >> 4] =
    (h[i][c] > 0) (checked against the f32 output it writes beside it, every bit of every
    row, padding halfwords untouched), and the bitmask ReluGrad epilogue (epi 3) gives exactly
    the f32-mask epilogue's output (epi 2 with the same activations as the mask)."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K + 4, generator=g).cuda()
    Bm = (torch.randn(N, K, generator=g) * 0.05).cuda()
    Bp = _planes(Bm, False)
    # aligned: ldc % 4 == 0 and an even ldbits (the engine's layout: 32 halfwords a row), which
    # selects the register epilogue (DIRECT) wherever N % 4 == 0; else the LDS epilogue
    ldc, ldb16 = (N + 4, 32) if aligned else (N + 3, (N + 15) // 16 + 2)
    h = torch.full((M, ldc), 7.0, device="cuda")
    bits = torch.full((M, ldb16), -1, dtype=torch.int16, device="cuda")
    call("dl_gemm_s3_nt_bits", M, N, K, ptr(A), K + 4, ptr(Bp), K, N * K, ptr(h), ldc, 1, None, 0,
         ptr(bits), ldb16, _s())
    torch.cuda.synchronize()
    nh = (N + 15) // 16
    words = bits[:, :nh].to(torch.int32) & 0xFFFF
    got = ((words[:, :, None] >> torch.arange(16, device="cuda")) & 1).reshape(M, nh * 16)[:, :N].bool()
    assert torch.equal(got, h[:, :N] > 0)
    assert (bits[:, nh:] == -1).all()
    # dX-shaped use: the same bitmask against the f32 mask it encodes
    dY = torch.randn(M, K + 4, generator=g).cuda()
    c2 = torch.full((M, ldc), 5.0, device="cuda")
    c3 = torch.full((M, ldc), 5.0, device="cuda")
    call("dl_gemm_s3_nt", M, N, K, ptr(dY), K + 4, ptr(Bp), K, N * K, ptr(c2), ldc, 2, ptr(h), ldc, _s())
    call("dl_gemm_s3_nt_bits", M, N, K, ptr(dY), K + 4, ptr(Bp), K, N * K, ptr(c3), ldc, 3, None, 0,
         ptr(bits), ldb16, _s())
    torch.cuda.synchronize()
    assert torch.equal(c2, c3)


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("M,N,K,F,E,tld", [(65536, 400, 432, 26, 16, 32), (300, 400, 432, 26, 16, 16),
                                           (257, 213, 72, 8, 8, 8), (77, 48, 96, 3, 32, 32),
                                           (513, 16, 64, 1, 64, 64), (40, 400, 416, 26, 16, 32)])
def test_gemm_s3_nt_gather_equals_lookup_then_gemm(hip_lib, M, N, K, F, E, tld, aligned):
    """dl_gemm_s3_nt_gather (the deep lookup inside the first tower layer's A stream) against
    the same GEMM over an x0 whose first F * E columns hold the looked-up rows: output and ReLU
    bitmask bit-identical.  Ids include the zero row (zero_row0), ids past the table and
    negative ids after the offset (all read as zeros), the slot plane's stride (tld = 2E) and a
    batch that is not a multiple of the 256-row block."""
    g = torch.Generator().manual_seed(M + N + K + F)
    n_rows, off = 5000, 3
    table = torch.randn(n_rows, tld, generator=g)
    ids = torch.randint(0, n_rows - off, (M, F + 2), generator=g, dtype=torch.int64)
    ids[::7, 0] = -off                      # row 0 (zero_row0)
    ids[5::11, F - 1] = n_rows              # past the table
    ids[3::13, F // 2] = -off - 1           # negative row
    rows = ids[:, :F] + off
    valid = (rows > 0) & (rows < n_rows)
    look = table[rows.clamp(0, n_rows - 1)][:, :, :E] * valid[:, :, None]
    A = torch.randn(M, K + 4, generator=g)
    A_ref = A.clone()
    A_ref[:, :F * E] = look.reshape(M, F * E)
    A[:, :F * E] = float("nan")             # never read by the gather
    Bm = (torch.randn(N, K, generator=g) * 0.05).cuda()
    Bp = _planes(Bm, False)
    ldc, ldb16 = (N + 4, 32) if aligned else (N + 3, (N + 15) // 16 + 2)
    Ad, Ar, Td, Id = A.cuda(), A_ref.cuda(), table.cuda(), ids.cuda()
    h_ref = torch.full((M, ldc), 7.0, device="cuda")
    h = torch.full((M, ldc), 7.0, device="cuda")
    b_ref = torch.full((M, ldb16), -1, dtype=torch.int16, device="cuda")
    b = torch.full((M, ldb16), -1, dtype=torch.int16, device="cuda")
    call("dl_gemm_s3_nt_bits", M, N, K, ptr(Ar), K + 4, ptr(Bp), K, N * K, ptr(h_ref), ldc, 1, None, 0,
         ptr(b_ref), ldb16, _s())
    call("dl_gemm_s3_nt_gather", M, N, K, ptr(Ad), K + 4, ptr(Td), n_rows, tld, ptr(Id), F + 2, off, 1, F, E,
         ptr(Bp), K, N * K, ptr(h), ldc, 1, ptr(b), ldb16, _s())
    torch.cuda.synchronize()
    assert torch.equal(h, h_ref)
    assert torch.equal(b, b_ref)
    # the store epilogue, no bitmask
    c_ref = torch.full((M, ldc), 5.0, device="cuda")
    c = torch.full((M, ldc), 5.0, device="cuda")
    call("dl_gemm_s3_nt", M, N, K, ptr(Ar), K + 4, ptr(Bp), K, N * K, ptr(c_ref), ldc, 0, None, 0, _s())
    call("dl_gemm_s3_nt_gather", M, N, K, ptr(Ad), K + 4, ptr(Td), n_rows, tld, ptr(Id), F + 2, off, 1, F, E,
         ptr(Bp), K, N * K, ptr(c), ldc, 0, None, 0, _s())
    torch.cuda.synchronize()
    assert torch.equal(c, c_ref)


@pytest.mark.parametrize("M,N,K,F,E,tld", [(65536, 400, 432, 26, 16, 32), (300, 400, 432, 26, 16, 16),
                                           (257, 213, 72, 8, 8, 8), (77, 48, 96, 3, 32, 32),
                                           (513, 16, 64, 1, 64, 64), (40, 400, 480, 26, 16, 32)])
def test_gemm_s3_nt_gather_tab_equals_x0_gemm(hip_lib, M, N, K, F, E, tld):
    """dl_gemm_s3_nt_gather_tab (predict's table form: the rows' byte offsets resolved beforehand
    and staged as they stand) against dl_gemm_s3_nt_bits over the x0 that holds the looked-up
    rows: output and ReLU bitmask bit-identical.  The offset table is built here by the layout
    rule (common.h kGtab*) with masked entries and junk in the pitch padding; x0's gathered
    columns are NaN (never read); a ragged batch."""
    g = torch.Generator().manual_seed(M + N + K + F)
    n_rows = 5000
    table = torch.randn(n_rows, tld, generator=g)
    rows = torch.randint(0, n_rows, (M, F), generator=g, dtype=torch.int64)
    masked = torch.rand(M, F, generator=g) < 0.1
    look = table[rows][:, :, :E] * (~masked)[:, :, None]
    tiles = (M + 255) // 256
    gt = np.full((tiles, F, 272), 0x12345678, dtype=np.uint32)   # pad entries: never read
    m = np.arange(M)
    gt[m // 256, :, m % 256] = np.where(masked.numpy(), 0xFFFFFF00, rows.numpy() * tld * 4).astype(np.uint32)
    A_ref = torch.randn(M, K + 4, generator=g)
    A_ref[:, :F * E] = look.reshape(M, F * E)
    Ax = A_ref.clone()
    Ax[:, :F * E] = float("nan")
    Bm = (torch.randn(N, K, generator=g) * 0.05).cuda()
    Bp = _planes(Bm, False)
    ldc, ldb16 = N + 4, 32
    Ar, Ad, Td = A_ref.cuda(), Ax.cuda(), table.cuda()
    Gd = torch.from_numpy(gt.view(np.int32).reshape(-1)).cuda()
    for epi, bits in ((1, True), (0, False)):
        h_ref = torch.full((M, ldc), 7.0, device="cuda")
        h = torch.full((M, ldc), 7.0, device="cuda")
        b_ref = torch.full((M, ldb16), -1, dtype=torch.int16, device="cuda")
        b = torch.full((M, ldb16), -1, dtype=torch.int16, device="cuda")
        bb = lambda t: (ptr(t), ldb16) if bits else (None, 0)
        call("dl_gemm_s3_nt_bits", M, N, K, ptr(Ar), K + 4, ptr(Bp), K, N * K, ptr(h_ref), ldc, epi, None, 0,
             *bb(b_ref), _s())
        call("dl_gemm_s3_nt_gather_tab", M, N, K, ptr(Ad), K + 4, ptr(Td), n_rows, tld, ptr(Gd), F, E, ptr(Bp), K,
             N * K, ptr(h), ldc, epi, *bb(b), _s())
        torch.cuda.synchronize()
        assert torch.equal(h, h_ref)
        assert torch.equal(b, b_ref)


def test_gemm_s3_nt_gather_argument_checks(hip_lib):
    """The gather's preconditions fail loudly: a partial 32-deep chunk, too many fields, an
    emb_dim outside {8..64}, the mask epilogue, a table past one 32-bit buffer range."""
    A = torch.zeros(64, 440, device="cuda")
    Bp = _planes(torch.zeros(16, 432, device="cuda"), False)
    T = torch.zeros(100, 16, device="cuda")
    I = torch.zeros(64, 30, dtype=torch.int64, device="cuda")
    C_ = torch.zeros(64, 16, device="cuda")
    base = lambda F, E, epi=1, n_rows=100: (64, 16, 432, ptr(A), 440, ptr(T), n_rows, 16, ptr(I), 30, 0, 1, F, E,
                                            ptr(Bp), 432, 16 * 432, ptr(C_), 16, epi, None, 0, _s())
    for args, msg in [(base(3, 16), "32-deep"), (base(41, 8), "fields"), (base(8, 4), "emb_dim"),
                      (base(2, 16, epi=2), "epilogue"), (base(2, 16, n_rows=1 << 26), "buffer range")]:
        with pytest.raises(_lib.DLError, match=msg):
            call("dl_gemm_s3_nt_gather", *args)
    G = torch.zeros(26 * 272 + 1, dtype=torch.int32, device="cuda")
    with pytest.raises(_lib.DLError, match="offset table"):
        call("dl_gemm_s3_nt_gather_tab", 64, 16, 432, ptr(A), 440, ptr(T), 100, 16, None, 26, 16, ptr(Bp), 432,
             16 * 432, ptr(C_), 16, 1, None, 0, _s())
    with pytest.raises(_lib.DLError, match="16-B aligned"):
        call("dl_gemm_s3_nt_gather_tab", 64, 16, 432, ptr(A), 440, ptr(T), 100, 16, ptr(G[1:]), 26, 16, ptr(Bp),
             432, 16 * 432, ptr(C_), 16, 1, None, 0, _s())


@pytest.mark.parametrize("M,N,K,splits", [(432, 400, 65536, 64), (416, 400, 8192, 8), (428, 396, 5000, 3),
                                            (64, 16, 100, 1), (16, 416, 4096, 16), (400, 400, 8192, 8),
                                            (404, 400, 2048, 2), (144, 400, 1024, 1)])
def test_gemm_s3_tn_split_slabs(hip_lib, M, N, K, splits):
    """Weight gradients X^T . dY as split-K slabs (K chunks rounded to 64): slab sums against
    fp64, slabs past the used count untouched."""
    g = torch.Generator().manual_seed(M + N + K)
    X = torch.randn(K, M, generator=g).cuda()
    Y = (torch.randn(K, N, generator=g) * 1e-3).cuda()
    ref = (X.t().double() @ Y.double()).cpu()
    from deep_learning_amd.engine import _num_splits
    used = _num_splits(K, splits, 64)
    slab = torch.full((used + 1, M, N), 7.0, device="cuda")
    call("dl_gemm_s3_tn", M, N, K, ptr(X), M, ptr(Y), N, ptr(slab), N, splits, M * N, _s())
    torch.cuda.synchronize()
    got = slab[:used].double().sum(0).cpu()
    scale = (X.abs().t().double() @ Y.abs().double()).cpu().clamp(min=1e-6)
    assert ((got - ref).abs() / scale).max().item() < 2e-6
    assert (slab[used].cpu() == 7.0).all()


def test_gemm_bf16(hip_lib):
    g = torch.Generator().manual_seed(2)
    M, N, K = 300, 200, 256
    A = torch.randn(M, K, generator=g).bfloat16()
    B = torch.randn(K, N, generator=g).bfloat16()
    ref = A.double() @ B.double()
    Ad, Bd = A.cuda(), B.cuda()
    C = torch.zeros(M, N, device="cuda")
    call("dl_gemm_bf16", 0, 0, M, N, K, ptr(Ad), K, ptr(Bd), N, ptr(C), N, 0, 0, None, 0, 1, 0, _s())
    torch.cuda.synchronize()
    assert torch.allclose(C.double().cpu(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("ta,tb,epi,cbf", [(1, 0, 3, 0), (0, 1, 2, 1), (0, 1, 0, 0), (0, 0, 1, 1), (0, 1, 3, 0), (0, 1, 1, 1)])
def test_gemm_bf16_variants(hip_lib, ta, tb, epi, cbf):
    """The bf16 tower's products: dW (A^T, split-K slabs), dX (B^T, ReluGrad mask, bf16 out),
    dx0 (B^T, fp32 out), forward (ReLU, bf16 out) — against fp64 on the same bf16 inputs."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 272, 208, 320
    A = torch.randn(M, K, generator=g).bfloat16()
    B = torch.randn(K, N, generator=g).bfloat16()
    mask = (torch.rand(M, N, generator=g) > 0.5).bfloat16()
    ref = A.double() @ B.double()
    if epi == 1:
        ref = ref.clamp_min(0)
    if epi == 2:
        ref = ref * mask.double()
    Ad = (A.t().contiguous() if ta else A).cuda()
    Bd = (B.t().contiguous() if tb else B).cuda()
    lda = M if ta else K
    ldb = K if tb else N
    splits = 4 if epi == 3 else 1
    C = torch.zeros(splits * M * N, dtype=torch.bfloat16 if cbf else torch.float32, device="cuda")
    md = mask.cuda()
    call("dl_gemm_bf16", ta, tb, M, N, K, ptr(Ad), lda, ptr(Bd), ldb, ptr(C), N, cbf, epi,
         ptr(md) if epi == 2 else None, N, splits, M * N, _s())
    torch.cuda.synchronize()
    got = C.double().cpu().view(splits, M, N).sum(0)
    tol = 2e-2 if cbf else 1e-3          # bf16 output: one bf16 rounding (2^-8 relative)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=tol, atol=tol)


def _engine(model, **kw):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    spec = ModelSpec(model, **kw)
    return spec, CTREngine(spec, max_batch=kw.pop("B", 256) if "B" in kw else 256, init="none")


def test_embed_fwd_bit_exact_gather(hip_lib):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    from oracle import ctr_ref as R
    cfg = R.make_cfg("deepfm_pipeline", C=13, S=26, E=16, cate_index_size=5000, hidden=[32, 16])
    spec = ModelSpec("deepfm_pipeline", C=13, S=26, E=16, cate_index_size=5000, hidden=[32, 16])
    eng = CTREngine(spec, max_batch=200, init="none")
    P = R.init_params(cfg, np.random.default_rng(0))
    eng.load_params(P)
    b = make_batch(200, cate_index_size=5000, seed=5)
    b["cate_feats"][0, :3] = 0          # row-0 / cont-row collisions
    b["cate_feats"][1, :] = np.arange(26) % 13
    eng.stage(b)
    eng._forward(200, _s())
    torch.cuda.synchronize()
    fw = R.forward(cfg, P, b)
    x0 = eng.x0.cpu().numpy()
    # gathered embeddings are copies: bit-exact
    np.testing.assert_array_equal(x0[:, :26 * 16], fw["x0"][:, 13:13 + 26 * 16])
    np.testing.assert_array_equal(x0[:, 26 * 16:26 * 16 + 13], fw["x0"][:, :13])
    fo = eng.fm_out.cpu().numpy()
    np.testing.assert_array_equal(fo[:, :39], fw["first"])           # single multiply: exact
    np.testing.assert_allclose(fo[:, 39:55], fw["second"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(eng.z[:200].cpu().numpy(), fw["z"], atol=1e-5)


def test_pool_counts_bit_exact(hip_lib):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    from oracle import ctr_ref as R
    ranges = [[0, 30, "a"], [30, 90, "b"], [90, 97, "c"]]
    cfg = R.make_cfg("deepfm_multi_cate", V=4, S=5, E=16, cate_index_size=3000, hidden=[32, 16],
                     multi_ranges=ranges)
    spec = ModelSpec("deepfm_multi_cate", V=4, S=5, E=16, cate_index_size=3000, hidden=[32, 16],
                     multi_ranges=ranges)
    eng = CTREngine(spec, max_batch=128, init="none")
    P = R.init_params(cfg, np.random.default_rng(1))
    P["feats_emb"][17] = 0.0            # an id whose row sums to zero: not counted
    eng.load_params(P)
    rng = np.random.default_rng(3)
    b = make_batch(128, cont=0, vector=4, cate_fields=5, cate_index_size=3000, seed=9, cate_only=True)
    multi = rng.integers(1, 3000, size=(128, 97))
    multi[rng.random((128, 97)) < 0.5] = 0
    multi[0] = 0
    multi[1, :5] = 17
    b["cate_feats"] = np.concatenate([b["cate_feats"], multi], 1)
    eng.stage(b)
    eng._forward(128, _s())
    torch.cuda.synchronize()
    fw = R.forward(cfg, P, b)
    np.testing.assert_array_equal(eng.cnt_emb.cpu().numpy(), fw["cnt_emb"])
    np.testing.assert_array_equal(eng.cnt_first.cpu().numpy(), fw["cnt_first"])
    x0 = eng.x0.cpu().numpy()
    np.testing.assert_allclose(x0[:, 80:80 + 48], fw["pooled"].reshape(128, -1), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(eng.z[:128].cpu().numpy(), fw["z"], atol=1e-5)


def test_out_of_range_id_raises(hip_lib):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    spec = ModelSpec("dnn_pipeline", C=13, S=26, E=8, cate_index_size=1000, hidden=[16])
    eng = CTREngine(spec, max_batch=64)
    b = make_batch(64, cate_index_size=1000, seed=1)
    b["cate_feats"][3, 4] = 1000
    with pytest.raises(_lib.DLError, match="out of range"):
        eng.predict(b)


def test_index_build_matches_numpy(hip_lib):
    """Sort/dedup/inverse map: bit-exact against numpy (unique rows, segment
    boundaries, per-owner counts) for a sharded key encoding."""
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    B, world, C = 300, 4, 13
    spec = ModelSpec("deepfm_pipeline", C=C, S=26, E=16, cate_index_size=2000, hidden=[16])
    eng = CTREngine(spec, max_batch=B, init="none")
    b = make_batch(B, cate_index_size=2000, seed=4)
    b["cate_feats"][0, :5] = [0, 0, 3, 3, 1999]
    eng.stage(b)
    L = eng.layout
    L.batch = B
    import ctypes
    n = B * 52
    ws = torch.zeros(hip_lib.dl_index_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    keys = torch.zeros(n, dtype=torch.int32, device="cuda")
    refs = torch.zeros(n, dtype=torch.int32, device="cuda")
    uniq = torch.zeros(n, dtype=torch.int32, device="cuda")
    off = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    nu = torch.zeros(1, dtype=torch.int32, device="cuda")
    inv = torch.zeros(n, dtype=torch.int32, device="cuda")
    oc = torch.zeros(world + 1, dtype=torch.int32, device="cuda")
    call("dl_index_build", ctypes.byref(L), ptr(eng.in_cate), world, C, ptr(ws), ws.numel(), ptr(keys), ptr(refs),
         ptr(uniq), ptr(off), ptr(nu), ptr(inv), ptr(oc), ptr(eng.err), _s())
    torch.cuda.synchronize()
    cate = b["cate_feats"].astype(np.int64)
    rows = np.concatenate([cate + C, cate], 1).reshape(-1)          # FM slots then deep slots
    ref_rows = np.concatenate([cate[:, :, None] + C, cate[:, :, None]], 2)  # not used: order check below
    rows = np.concatenate([cate + C, cate], 1)                       # [B, 52]
    flat = rows.reshape(-1)
    valid = flat > 0
    own = np.where(flat < C, world, flat % world)
    loc = np.where(flat < C, flat, flat // world)
    key = (own.astype(np.uint64) << 27) | loc.astype(np.uint64)
    key = np.where(valid, key, 0xFFFFFFFF)
    u_ref, cnt_ref = np.unique(key[valid], return_counts=True)
    nuv = int(nu.item())
    assert nuv == len(u_ref)
    got_u = uniq[:nuv].cpu().numpy().astype(np.uint32).astype(np.uint64)
    np.testing.assert_array_equal(got_u, u_ref)
    np.testing.assert_array_equal(np.diff(off[:nuv + 1].cpu().numpy()), cnt_ref)
    invc = inv.cpu().numpy()
    np.testing.assert_array_equal(invc[~valid], -1)
    np.testing.assert_array_equal(u_ref[invc[valid]], key[valid])
    own_u = (u_ref >> 27).astype(np.int64)
    np.testing.assert_array_equal(oc.cpu().numpy(), np.bincount(own_u, minlength=world + 1))


@pytest.mark.parametrize("B", [300, 2048])
def test_index_build_pair_equals_two_builds(hip_lib, B):
    """dl_index_build_pair (the wdl table ids and wide ids in one sort, index.hip) against
    dl_index_build run once per id set: unique rows, counts, segment offsets, the sorted
    references inside every segment and both inverse maps bit-identical — row-0 references
    (dropped when the layout's zero-row rule applies), repeated ids and wide ids on the
    deep-output rows included."""
    import ctypes
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    Fw, H = 26, 32
    spec = ModelSpec("wdl", C=13, S=26, E=16, cate_index_size=8000, hidden=[64, H], Fw=Fw)
    eng = CTREngine(spec, max_batch=B, init="none", adam="lazy")
    assert eng.index_pair
    b = make_batch(B, cate_index_size=8000, wide_fields=Fw, seed=B)
    b["cate_feats"][0, :4] = [0, 0, 5, 5]
    b["wide_feats"][1, :3] = [Fw, Fw + H - 1, Fw]
    eng.stage(b)
    eng._pre(B)
    torch.cuda.synchronize()
    nt, nw = int(eng.idx_n[0].item()), int(eng.widx_n[0].item())
    got = dict(u=eng.idx_uniq[:nt].cpu().numpy(), off=eng.idx_off[:nt + 1].cpu().numpy(),
               inv=eng.idx_inv[:eng.n_refs].cpu().numpy(), refs=eng.idx_refs.cpu().numpy(),
               wu=eng.widx_uniq[:nw].cpu().numpy(), woff=eng.widx_off[:nw + 1].cpu().numpy(),
               winv=eng.winv[:B * Fw].cpu().numpy(), wrefs=eng.widx_refs.cpu().numpy())

    def one(L, cate, n):
        ws = torch.zeros(hip_lib.dl_index_workspace_bytes(n), dtype=torch.uint8, device="cuda")
        t = [torch.zeros(n + 1, dtype=torch.int32, device="cuda") for _ in range(6)]
        call("dl_index_build", ctypes.byref(L), ptr(cate), 1, 0, ptr(ws), ws.numel(), ptr(t[0]), ptr(t[1]), ptr(t[2]),
             ptr(t[3]), ptr(t[4]), ptr(t[5]), None, ptr(eng.err), _s())
        torch.cuda.synchronize()
        k = int(t[4][0].item())
        return k, t[2][:k].cpu().numpy(), t[3][:k + 1].cpu().numpy(), t[5][:n].cpu().numpy(), t[1].cpu().numpy()

    L = eng.layout
    L.batch = B
    k1, u1, off1, inv1, refs1 = one(L, eng.in_cate, eng.n_refs)
    WL = eng.wlayout
    WL.batch = B
    k2, u2, off2, inv2, refs2 = one(WL, eng.in_wide, B * Fw)
    assert (nt, nw) == (k1, k2)
    same = np.testing.assert_array_equal
    same(got["u"], u1)
    same(got["off"], off1)
    same(got["inv"], inv1)
    same(got["refs"][:off1[-1]], refs1[:off1[-1]])
    same(got["wu"], u2)
    same(got["woff"], off2)
    same(got["winv"], inv2)
    same(got["wrefs"][:off2[-1]], refs2[:off2[-1]])


@pytest.mark.parametrize("model", ["deepfm_pipeline", "dnn_pipeline"])
def test_sorted_backward_equals_atomic(hip_lib, model):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    spec = ModelSpec(model, C=13, V=0, S=26, E=16, cate_index_size=3000, hidden=[32, 16])
    outs = []
    for mode in ("atomic", "sorted"):
        eng = CTREngine(spec, max_batch=700, seed=3, bwd=mode)
        for i in range(3):
            eng.train_step(make_batch(700, cate_index_size=3000, seed=20 + i))
        torch.cuda.synchronize()
        outs.append(eng.params())
    for k in outs[0]:
        np.testing.assert_allclose(outs[0][k], outs[1][k], atol=2e-6, rtol=0, err_msg=k)


def test_chain_apply_equals_sorted_segment_apply(hip_lib):
    """Owner update of the sharded path: arrival chains (dl_rec_chain_link +
    dl_rec_apply_chain) and the stash form (dl_rec_gather's moments at every arrival) against
    the sort + segment form (dl_sort_unique + dl_rec_apply_segments) on the same arrivals — 8 senders with unique ids each, so
    rows arrive up to 8 times, some rows lagging several steps: records bit-identical,
    chain heads back to -1."""
    E, ld, rows, W, per, hist_len = 16, 64, 5000, 8, 900, 8
    g = torch.Generator().manual_seed(5)
    rec0 = torch.zeros(rows, ld)
    rec0[:, :E + 3] = torch.randn(rows, E + 3, generator=g) * 0.1
    rec0[:, E + 4: 3 * E + 4] = torch.rand(rows, 2 * E, generator=g) * 0.01
    stamps = torch.randint(3, 10, (rows,), generator=g, dtype=torch.int32)
    rec0.view(torch.int32)[:, E + 3] = stamps
    ids = torch.cat([torch.randperm(rows, generator=g)[:per] for _ in range(W)]).to(torch.int32)
    n = ids.numel()
    gr = torch.randn(n, E, generator=g)
    g1 = torch.randn(n, generator=g)
    hist = torch.rand(hist_len, generator=g) * 1e-3
    opt = torch.zeros(32)   # DL_OPT_LEN: Adam scalars, sums, status word
    opt[3], opt[4], opt[5], opt[6], opt[7] = 1e-3, 0.9, 0.999, 1e-8, 10   # alpha, b1, b2, eps, step
    ids_d, gr_d, g1_d, hist_d, opt_d = ids.cuda(), gr.cuda(), g1.cuda(), hist.cuda(), opt.cuda()
    # sort + segments
    recA = rec0.clone().cuda()
    z = lambda *sh: torch.zeros(*sh, dtype=torch.int32, device="cuda")
    ws = torch.zeros(hip_lib.dl_index_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    keys, pos, uniq, off, nu = z(n), z(n), z(n), z(n + 1), z(4)
    call("dl_sort_unique", ptr(ids_d), n, 13, ptr(ws), ws.numel(), ptr(keys), ptr(pos), ptr(uniq), ptr(off),
         ptr(nu), None, _s())
    call("dl_rec_apply_segments", ptr(recA), ld, E, 1, ptr(uniq), ptr(off), ptr(nu), n, n, ptr(pos), ptr(gr_d),
         ptr(g1_d), None, None, None, ptr(hist_d), hist_len, ptr(opt_d), _s())
    # with the owner gather's stash (rows + moments caught up to step 9 at every arrival
    # position): the record is only written, and must come out the same
    recC = rec0.clone().cuda()
    L = _lib.EmbLayout()
    L.n_rows, L.batch, L.emb_dim = rows, 1, E
    rows_u, rows_u1 = torch.empty(n, E, device="cuda"), torch.empty(n, device="cuda")
    mv = torch.empty(n, hip_lib.dl_rec_stash_floats(E), device="cuda")   # the moment stash (rec.hip)
    call("dl_rec_gather", C.byref(L), ptr(recC), ld, 1, 0, ptr(ids_d), None, n, 1, ptr(hist_d), hist_len,
         ptr(opt_d), 1, ptr(rows_u), ptr(rows_u1), ptr(mv), _s())
    call("dl_rec_apply_segments", ptr(recC), ld, E, 1, ptr(uniq), ptr(off), ptr(nu), n, n, ptr(pos), ptr(gr_d),
         ptr(g1_d), ptr(rows_u), ptr(rows_u1), ptr(mv), ptr(hist_d), hist_len, ptr(opt_d), _s())
    # chains
    recB = rec0.clone().cuda()
    head = torch.full((rows,), -1, dtype=torch.int32, device="cuda")
    nxt = z(n)
    call("dl_rec_chain_link", ptr(ids_d), n, ptr(head), ptr(nxt), _s())
    call("dl_rec_apply_chain", ptr(recB), ld, E, 1, ptr(ids_d), n, ptr(head), ptr(nxt), ptr(gr_d), ptr(g1_d),
         ptr(hist_d), hist_len, ptr(opt_d), _s())
    torch.cuda.synchronize()
    assert int(nu[0]) == len(np.unique(ids.numpy()))
    np.testing.assert_array_equal(recB.cpu().numpy().view(np.int32), recA.cpu().numpy().view(np.int32))
    np.testing.assert_array_equal(recC.cpu().numpy().view(np.int32)[:, :3 * E + 4],
                                  recA.cpu().numpy().view(np.int32)[:, :3 * E + 4])
    assert bool((head == -1).all())
    touched = np.unique(ids.numpy())
    assert (recB.view(torch.int32)[:, E + 3].cpu().numpy()[touched] == 10).all()


@pytest.mark.parametrize("E", [8, 16])
def test_pool_weighted_matches_oracle(hip_lib, E):
    """dl_pool_fwd_weighted / dl_pool_bwd_weighted (dnn_multi_textline.py:89-103) against
    oracle.pool_weighted: counts bit-exact, pooled vectors and table gradients at 1e-6."""
    from oracle import ctr_ref as R
    rng = np.random.default_rng(E)
    B, N, W, S = 300, 5000, 97, 3
    ranges = [[0, 30, "a"], [30, 90, "b"], [90, 97, "c"]]
    V = rng.standard_normal((N, E)).astype(np.float32) * 0.1
    V[11] = 0.0                                           # a real id with a zero row
    ids = np.zeros((B, S + W), np.int64)                  # [S singles | multi block]
    ids[:, :S] = rng.integers(1, N, (B, S))
    multi = rng.integers(1, N, (B, W))
    multi[rng.random((B, W)) < 0.5] = 0
    multi[0] = 0
    multi[1, :7] = 11
    ids[:, S:] = multi
    vals = (rng.random((B, W)) * 2).astype(np.float32)
    vals[2, :10] = 0.0
    Vz = V.copy(); Vz[0] = 0
    ref_pooled, ref_cnt = R.pool_weighted(Vz, multi, vals, ranges)
    M = len(ranges)
    x0_ld, pool_col = 64 + M * E, 64
    L = _lib.EmbLayout(n_rows=N, batch=B, emb_dim=E, cate_fields=S, cate_ld=S + W, use_fm=0, zero_row0=1,
                       x0_ld=x0_ld, x0_pool_col=pool_col, dx0_ld=x0_ld)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    tab, idt, vt = dev(V), dev(ids), dev(vals)
    s0 = torch.tensor([r[0] for r in ranges], dtype=torch.int32, device="cuda")
    s1 = torch.tensor([r[1] for r in ranges], dtype=torch.int32, device="cuda")
    x0 = torch.zeros(B, x0_ld, device="cuda")
    cnt = torch.zeros(B, M, device="cuda")
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    call("dl_pool_fwd_weighted", C.byref(L), ptr(tab), ptr(idt), S, ptr(vt), W, ptr(s0), ptr(s1), M,
         ptr(x0), ptr(cnt), ptr(err), _s())
    torch.cuda.synchronize()
    assert int(err[0]) == 0
    np.testing.assert_array_equal(cnt.cpu().numpy(), ref_cnt)
    got = x0[:, pool_col:].cpu().numpy().reshape(B, M, E)
    np.testing.assert_allclose(got, ref_pooled, rtol=1e-5, atol=1e-6)
    assert (x0[:, :pool_col] == 0).all()
    # backward: dx0 at the pooled columns
    d = rng.standard_normal((B, M, E)).astype(np.float32)
    dx0 = torch.zeros(B, x0_ld, device="cuda")
    dx0[:, pool_col:] = dev(d.reshape(B, -1))
    g = torch.zeros(N, E, device="cuda")
    touched = torch.zeros(N, dtype=torch.uint8, device="cuda")
    call("dl_pool_bwd_weighted", C.byref(L), ptr(idt), S, ptr(vt), W, ptr(s0), ptr(s1), M, ptr(dx0), pool_col,
         ptr(cnt), ptr(g), ptr(touched), _s())
    torch.cuda.synchronize()
    G = R.pool_weighted_bwd(N, multi, vals.astype(np.float64), ranges, ref_cnt.astype(np.float64),
                            d.astype(np.float64))
    np.testing.assert_allclose(g.cpu().numpy(), G, rtol=1e-5, atol=1e-6)
    want_touched = np.zeros(N, np.uint8)
    for a, b_, _ in ranges:
        want_touched[multi[:, a:b_].reshape(-1)] = 1
    want_touched[0] = 0
    np.testing.assert_array_equal(touched.cpu().numpy(), want_touched)


@pytest.mark.gpu
def test_textline_pooling_frozen_tag_slot(hip_lib):
    """deep_learning_amd.textline (dnn_multi_textline.py:69-103): slots 'a', 'b' pooled from the
    trainable table (row 0 zeroed), slot 'tag' from the frozen word2vec table (:45-47,85-88: read
    directly, row 0 not zeroed, no gradient); counts bit-exact, pooled vectors and the table
    gradient (non-tag slots only) against oracle.pool_weighted / pool_weighted_bwd."""
    from oracle import ctr_ref as R
    from deep_learning_amd.textline import TextlinePooling
    rng = np.random.default_rng(5)
    B, N, Nw, E = 257, 3000, 2000, 16
    ranges = [[0, 20, "a"], [20, 50, "tag"], [50, 64, "b"]]
    W = 64
    V = (rng.standard_normal((N, E)) * 0.1).astype(np.float32)
    w2v = (rng.standard_normal((Nw, E)) * 0.1).astype(np.float32)   # row 0 nonzero: tag padding counts
    ids = rng.integers(1, Nw, (B, W))
    ids[rng.random((B, W)) < 0.4] = 0
    vals = (rng.random((B, W)) * 2).astype(np.float32)
    Vz = V.copy()
    Vz[0] = 0
    ref, ref_cnt = [], []
    for r in ranges:
        tab = w2v if r[2] == "tag" else Vz
        p, c = R.pool_weighted(tab, ids, vals, [r])
        ref.append(p)
        ref_cnt.append(c)
    ref, ref_cnt = np.concatenate(ref, 1), np.concatenate(ref_cnt, 1)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    tp = TextlinePooling(ranges, E, N, w2v=dev(w2v))
    pooled, cnt = tp.forward(dev(V), dev(ids), dev(vals))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cnt.cpu().numpy(), ref_cnt)
    np.testing.assert_allclose(pooled.cpu().numpy().reshape(B, 3, E), ref, rtol=1e-5, atol=1e-6)
    d = rng.standard_normal((B, 3, E)).astype(np.float32)
    g = torch.zeros(N, E, device="cuda")
    touched = torch.zeros(N, dtype=torch.uint8, device="cuda")
    tp.backward(dev(d.reshape(B, -1)), dev(ids), dev(vals), g, touched)
    torch.cuda.synchronize()
    keep = [0, 2]
    G = R.pool_weighted_bwd(N, ids, vals.astype(np.float64), [ranges[m] for m in keep],
                            ref_cnt[:, keep].astype(np.float64), d[:, keep].astype(np.float64))
    np.testing.assert_allclose(g.cpu().numpy(), G, rtol=1e-5, atol=1e-6)


def test_auc_gpu_matches_sklearn_goldens_and_oracle(hip_lib):
    """dl_auc (metrics.hip) against the committed sklearn goldens and the oracle on a
    tie-heavy 2M-sample set (float32 scores, as the reference's score tensor)."""
    import os
    from deep_learning_amd.metrics import AucAccumulator, roc_auc
    from oracle import ctr_ref as R
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "auc_golden.npz"))
    for case in ("ties", "random", "all_tied"):
        y, s = d[case + "_y"], d[case + "_s"].astype(np.float32)
        assert abs(roc_auc(y, s) - R.auc(y, s)) < 1e-12
        assert abs(roc_auc(y, s) - d[case + "_auc"][0]) < 1e-7
    rng = np.random.default_rng(11)
    n = 2_000_003
    s = (np.round(rng.random(n) * 1000) / 1000 - 0.5).astype(np.float32)   # ties, both signs
    s[:1000] = -0.0                                                        # -0.0 ties with +0.0
    s[1000:2000] = 0.0
    y = (rng.random(n) < 0.5 + 0.3 * s).astype(np.float32)
    acc = AucAccumulator()
    for a in range(0, n, 700_001):                                        # ragged batches
        acc.add(torch.from_numpy(y[a:a + 700_001]).cuda(), torch.from_numpy(s[a:a + 700_001]).cuda())
    assert abs(acc.result() - R.auc(y, s)) < 1e-12
    # tiny sets: one positive and one negative (either order, tied), a tie group holding every class
    assert roc_auc(np.array([0, 1]), np.array([0.1, 0.2])) == 1.0
    assert roc_auc(np.array([1, 0]), np.array([0.1, 0.2])) == 0.0
    assert roc_auc(np.array([1, 0]), np.array([0.3, 0.3])) == 0.5
    y3, s3 = np.array([1, 0, 1, 0, 0]), np.array([0.5, 0.5, 0.9, -1.0, 0.5], np.float32)
    assert abs(roc_auc(y3, s3) - R.auc(y3, s3)) < 1e-12
    with pytest.raises(ValueError, match="one class"):
        roc_auc(np.ones(10), np.arange(10.0))
    with pytest.raises(ValueError, match="one class"):
        roc_auc(np.zeros(1), np.zeros(1))


@pytest.mark.parametrize("n,distinct", [(1, 1), (4096 * 3, 5), (100_003, 50), (262_147, 200_000), (5000, 4999)])
def test_sort_unique_matches_numpy(hip_lib, n, distinct):
    """dl_sort_unique (radix sort + the two-pass segmented unique): unique keys, segment
    bounds, positions in stable order and the inverse map bit-exact against numpy, with
    segments that span many 4096-key chunks and ragged tails."""
    rng = np.random.default_rng(n)
    ids = rng.integers(0, distinct, n).astype(np.int32)
    d = torch.from_numpy(ids).cuda()
    ws = torch.zeros(hip_lib.dl_index_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    z = lambda m: torch.full((m,), -7, dtype=torch.int32, device="cuda")
    keys, pos, uniq, off, nu, inv = z(n), z(n), z(n), z(n + 1), z(1), z(n)
    call("dl_sort_unique", ptr(d), n, 18, ptr(ws), ws.numel(), ptr(keys), ptr(pos), ptr(uniq), ptr(off), ptr(nu),
         ptr(inv), _s())
    torch.cuda.synchronize()
    u_ref, first, inv_ref, cnt_ref = np.unique(ids, return_index=True, return_inverse=True, return_counts=True)
    k = int(nu.item())
    assert k == len(u_ref)
    np.testing.assert_array_equal(uniq[:k].cpu().numpy(), u_ref)
    o = off[:k + 1].cpu().numpy()
    assert o[0] == 0 and o[-1] == n
    np.testing.assert_array_equal(np.diff(o), cnt_ref)
    np.testing.assert_array_equal(inv.cpu().numpy(), inv_ref.reshape(-1))
    np.testing.assert_array_equal(pos.cpu().numpy(), np.argsort(ids, kind="stable"))


@pytest.mark.parametrize("M,N,K,epi,cbf", [(65536, 400, 432, 1, 1), (9000, 400, 400, 2, 1), (5000, 416, 400, 0, 0),
                                           (4100, 37, 200, 1, 0), (8192, 400, 416, 1, 0), (300, 209, 40, 2, 1),
                                           (777, 208, 8, 1, 1), (1000, 100, 1000, 2, 0), (257, 400, 432, 0, 1),
                                           (1000, 300, 72, 2, 0), (129, 416, 48, 1, 1), (65536, 416, 400, 0, 0)])
@pytest.mark.parametrize("ldc_pad", [3, 4])   # ldc % 4 == 0 (pad 4, N % 4 == 0): the register epilogue
def test_gemm_bf16_b_resident(hip_lib, M, N, K, epi, cbf, ldc_pad):
    """The tall-skinny bf16 path (ta=0, tb=1: the streamed-weight kernel gemm_bf16_nt_kernel,
    the B-resident kernel where it declines): relu / ReluGrad-mask / store epilogues, bf16 or
    f32 output, ragged M, N and K chunks (K past one chunk, not a multiple of 32, beyond the
    B-resident limit), against an fp64 product of the same bf16 operands."""
    g = torch.Generator().manual_seed(M + N + K)
    lda = (K + 7) // 8 * 8 + 8
    A = torch.randn(M, lda, generator=g).bfloat16()
    A[:, K:] = 7.0                                  # pad past K must not be read
    Bt = torch.randn(N, lda, generator=g).bfloat16()
    Bt[:, K:] = -3.0
    ldm = (N + 7) // 8 * 8
    mask = torch.randn(M, ldm, generator=g).bfloat16()
    ref = A[:, :K].double() @ Bt[:, :K].double().t()
    if epi == 1:
        ref = ref.clamp(min=0)
    elif epi == 2:
        ref = torch.where(mask[:, :N].double() > 0, ref, torch.zeros_like(ref))
    ldc = N + ldc_pad
    C = torch.full((M, ldc), 5.0, device="cuda", dtype=torch.bfloat16 if cbf else torch.float32)
    md, Ad, Bd = mask.cuda(), A.cuda(), Bt.cuda()    # held for the launch (no freed temporaries)
    call("dl_gemm_bf16", 0, 1, M, N, K, ptr(Ad), lda, ptr(Bd), lda, ptr(C), ldc, cbf, epi,
         ptr(md) if epi == 2 else None, ldm, 1, 0, _s())
    torch.cuda.synchronize()
    out = C[:, :N].double().cpu()
    scale = (A[:, :K].double().abs() @ Bt[:, :K].double().abs().t()).clamp(min=1.0)
    tol = 1e-2 if cbf else 1e-5                      # bf16 output rounding vs fp32 accumulation
    assert ((out - ref).abs() / scale).max().item() < tol
    assert (C[:, N:].float().cpu() == 5.0).all()


@pytest.mark.parametrize("M,N,K,splits", [(432, 400, 65536, 64), (416, 400, 40000, 7), (264, 208, 1000, 3),
                                          (64, 16, 96, 1), (432, 400, 65536, 85), (416, 400, 65536, 85),
                                          (136, 120, 4096, 5), (288, 392, 2048, 1)])
def test_gemm_bf16_dw_transposed_reads(hip_lib, M, N, K, splits):
    """Weight gradients of the bf16 tower from batch-major operands (ta=1, tb=0, split slabs):
    the transposing-LDS-read kernels against an fp64 product of the same bf16 inputs, with
    ragged M tiles, K steps and splits (K % 32 == 0: the LDS-DMA ring kernel, 144 x 400 blocks;
    K = 1000: the two-buffer kernel)."""
    g = torch.Generator().manual_seed(M + N + K)
    X = torch.randn(K, M, generator=g).bfloat16()
    Y = torch.randn(K, N, generator=g).bfloat16()
    ref = X.double().t() @ Y.double()
    slab = torch.full((splits, M, N), 0.0, device="cuda")
    Xd, Yd = X.cuda(), Y.cuda()     # held: a freed temporary's block can be handed to the next .cuda()
    call("dl_gemm_bf16", 1, 0, M, N, K, ptr(Xd), M, ptr(Yd), N, ptr(slab), N, 0, 3, None, 0, splits,
         M * N, _s())
    torch.cuda.synchronize()
    got = slab.double().sum(0).cpu()
    scale = (X.double().abs().t() @ Y.double().abs()).clamp(min=1.0)
    assert ((got - ref).abs() / scale).max().item() < 5e-4


@pytest.mark.parametrize("B", [3000, 70])
def test_wdl_head_bf16_dy_is_rounded_f32_dy(hip_lib, B):
    """dl_wdl_head_fwd_bwd_bf16 (the C5 head writing the bf16 tower's dY itself, with the
    wide ids and weights loaded ahead of the sample being reduced): score, z, dz and the
    block partials bit-identical to the f32 head, dY equal to the f32 dY rounded to
    nearest-even, z against an fp64 restatement of models/wdl.py:225-264."""
    g = torch.Generator().manual_seed(B)
    Fw, H, rows, ldh = 26, 400, 5000, 404
    wide = torch.randint(0, rows, (B, Fw), generator=g)
    h = torch.randn(B, ldh, generator=g).clamp_min(0)
    w = torch.randn(rows, generator=g) * 0.1
    bias = torch.tensor([0.1, 0.0, 0.0, 0.0])
    label = (torch.rand(B, generator=g) > 0.5).float()
    wide_d, h_d, w_d, bias_d, label_d = wide.cuda(), h.cuda(), w.cuda(), bias.cuda(), label.cuda()
    grid = _lib.lib().dl_wdl_head_grid(B)
    outs = []
    for bf in (0, 1):
        score, z, dz = (torch.zeros(B, device="cuda") for _ in range(3))
        dh = torch.zeros(B, ldh, device="cuda", dtype=torch.bfloat16 if bf else torch.float32)
        gw = torch.zeros(rows, device="cuda", dtype=torch.int64)   # fixed point, 2^-48 units
        touched = torch.zeros(rows, device="cuda", dtype=torch.uint8)
        slab = torch.zeros(grid * (H + 2), device="cuda")
        err = torch.zeros(4, device="cuda", dtype=torch.int32)
        call("dl_wdl_head_fwd_bwd_bf16" if bf else "dl_wdl_head_fwd_bwd", B, Fw, H, ptr(wide_d), Fw, ptr(h_d), ldh,
             ptr(w_d), ptr(bias_d), rows, ptr(label_d), 1e-7, 1.0 / B, ptr(score), ptr(z), ptr(dz), ptr(dh), ptr(gw),
             ptr(touched), ptr(slab), grid, ptr(err), _s())
        torch.cuda.synchronize()
        assert err.cpu().sum().item() == 0
        outs.append((score.cpu(), z.cpu(), dz.cpu(), dh[:, :H].cpu(), gw.cpu(), touched.cpu(), slab.cpu()))
    f, b = outs
    for i in (0, 1, 2, 4, 5, 6):   # wide gradient too: integer atomics, order-independent
        assert torch.equal(f[i], b[i])
    assert torch.equal(b[3], f[3].bfloat16())
    # the wide segment sum against fp64 (every dz term quantised to 2^-48)
    gref = torch.zeros(rows, dtype=torch.float64).index_add_(0, wide.reshape(-1), f[2].double().repeat_interleave(Fw))
    np.testing.assert_allclose(f[4].double().numpy() / 2.0 ** 48, gref.numpy(), rtol=0, atol=1e-12)
    z_ref = w.double()[wide].sum(1) + h[:, :H].double() @ w.double()[Fw:Fw + H] + 0.1
    np.testing.assert_allclose(f[1].double().numpy(), z_ref.numpy(), rtol=0, atol=1e-4)


@pytest.mark.parametrize("n", [1003, 4096 * 256 * 4 * 2 + 4 * 100 + 3])
@pytest.mark.parametrize("flags", [0, _lib.ROWS_SPARSE_ADAM, _lib.ROWS_GRAD_FIXED,
                                   _lib.ROWS_GRAD_FIXED | _lib.ROWS_SPARSE_ADAM])
def test_adam_rows_width1_sweep(hip_lib, n, flags):
    """dl_adam_rows at width 1 (first-order / wdl wide weights, optim.hip adam_rows1_kernel):
    every row steps (touched rows with their gradient, the rest with g = l2*p), the consumed
    gradients and flags are reset, sq = sum p^2; n with a 3-row tail, and large enough that
    each thread takes two groups per round.  p
    goes through the hardware reciprocal; all three are held to f32-rounding tolerances."""
    rng = np.random.default_rng(n + flags)
    p = rng.standard_normal(n).astype(np.float32)
    m = (rng.standard_normal(n) * 1e-2).astype(np.float32)
    v = (rng.random(n) * 1e-3).astype(np.float32)
    touched = (rng.random(n) < 0.3).astype(np.uint8)
    fixed = bool(flags & _lib.ROWS_GRAD_FIXED)
    if not fixed:   # the first-order tables' root state s = sqrt(v) (common.h adam_elem_root)
        v = np.sqrt(v.astype(np.float64)).astype(np.float32)
    # the gradient table's invariant: zero outside the touched rows
    gf = np.where(touched == 1, rng.standard_normal(n) * 1e-2, 0).astype(np.float32)
    if fixed:
        gq = np.round(gf.astype(np.float64) * 2.0 ** 48).astype(np.int64)
        g_d = torch.from_numpy(gq).cuda()
        g_eff = (gq.astype(np.float64) * 2.0 ** -48).astype(np.float32)
    else:
        g_d = torch.from_numpy(gf).cuda()
        g_eff = gf
    g_eff = np.where(touched == 1, g_eff, np.float32(0))
    l2 = np.float32(1e-3)
    b1, b2, eps, alpha = np.float32(0.9), np.float32(0.999), np.float32(1e-8), np.float32(1e-3)
    opt = torch.zeros(_lib.OPT_LEN, dtype=torch.float32)
    opt[3], opt[4], opt[5], opt[6] = float(alpha), float(b1), float(b2), float(eps)
    opt = opt.cuda()
    sq = torch.zeros(1, dtype=torch.int64, device="cuda")   # fixed point (DL_REG_SUM_SCALE)
    pd, md, vd = (torch.from_numpy(a.copy()).cuda() for a in (p, m, v))
    td = torch.from_numpy(touched.copy()).cuda()
    call("dl_adam_rows", ptr(pd), ptr(md), ptr(vd), ptr(g_d), ptr(td), n, 1, float(l2),
         flags | _lib.ROWS_CLEAR_TOUCHED, ptr(opt), ptr(sq), _s())
    torch.cuda.synchronize()
    g = (g_eff + l2 * p).astype(np.float32)
    omb1, omb2 = np.float32(1) - b1, np.float32(1) - b2
    # first-order tables keep the root state s = sqrt(v) (common.h adam_elem_root): the input
    # array is s, the output is s'; the wide weights (fixed-point form) keep v
    v_in = v if fixed else (v * v).astype(np.float32)
    if flags & _lib.ROWS_SPARSE_ADAM:
        m1 = (m * b1 + g * omb1).astype(np.float32)
        v1 = (v_in * b2 + (g * g) * omb2).astype(np.float32)
    else:
        m1 = (m + (g - m) * omb1).astype(np.float32)
        v1 = (v_in + (g * g - v_in) * omb2).astype(np.float32)
    p1 = (p - (m1 * alpha) / (np.sqrt(v1) + eps)).astype(np.float32)
    # g + l2*p may contract to an fma on the device: m, v within f32 rounding, not bit-equal
    np.testing.assert_allclose(md.cpu().numpy(), m1, rtol=2e-6, atol=2e-9)
    v_out = vd.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(v_out if fixed else v_out * v_out, v1, rtol=4e-6, atol=2e-11)
    np.testing.assert_allclose(pd.cpu().numpy(), p1, rtol=1e-6, atol=1e-7)
    assert int(td.sum()) == 0
    assert not torch.any(g_d != 0)
    np.testing.assert_allclose(_lib.reg_sum(sq), float(np.sum(p.astype(np.float64) ** 2)), rtol=1e-4)
