"""Weight-gradient GEMMs (gr_wgrad / gr_wgrad2 / gr_wgrad2_bf16) against an fp64 torch
reference: C[ka][nb] = sum_m A'(m, ka) Bm(m, nb), colsum[ka] = sum_m A'(m, ka), with
A' = (A - mean) * rstd from the saved row stats (or A itself), over jagged rows.

Shapes cover the panel widths (NT 4 / 8 / 13 / 16), Nb an exact multiple of the panel
width (the colsum then has no padding column to ride in) and ragged Ka / Nb.
Tolerances: fp32 path 1e-5 relative to the largest |C| (f32 MFMA, split-K over rows);
bf16 operands: against the reference on bf16-rounded A' and Bm, 1e-5 likewise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from mygenerativerecommenders_amd import _lib
    return _lib


def _case(rows_per_seq, Ka, Nb, seed, stats=True):
    g = torch.Generator(device="cuda").manual_seed(seed)
    dev = torch.device("cuda")
    lens = torch.tensor(rows_per_seq, dtype=torch.int64)
    offs = torch.zeros(len(rows_per_seq) + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(lens, 0)
    total = int(offs[-1])
    cap = total + 37  # rows past offsets[B] must not contribute
    a = torch.randn(cap, Ka, device=dev, generator=g) * 2 + 0.5
    b = torch.randn(cap, Nb, device=dev, generator=g)
    st = None
    if stats:
        mean = a[:, :Ka].mean(1)
        rstd = torch.rsqrt(a[:, :Ka].var(1, unbiased=False) + 1e-6)
        st = torch.stack([mean, rstd], 1).contiguous()
    return offs.to(dev), total, cap, a, b, st


def _ref(a, b, st, total, bf16=False):
    if bf16:  # the kernel applies the LN in fp32, then rounds both operands to bf16
        a32 = a[:total]
        if st is not None:
            a32 = (a32 - st[:total, 0:1]) * st[:total, 1:2]
        a64 = a32.bfloat16().double()
        b64 = b[:total].bfloat16().double()
    else:
        a64 = a[:total].double()
        if st is not None:
            a64 = (a64 - st[:total, 0:1].double()) * st[:total, 1:2].double()
        b64 = b[:total].double()
    return a64.t() @ b64, a64.sum(0)


def _check(got, ref, what):
    scale = ref.abs().max().item() + 1.0
    err = (got.double() - ref).abs().max().item()
    assert err <= 1e-5 * scale, (what, err, scale)


@pytest.mark.parametrize("stream", [1, 0])
@pytest.mark.parametrize("Ka,Nb", [(50, 200), (256, 1024), (256, 256), (64, 64), (33, 17),
                                   (256, 257), (128, 128), (16, 250), (64, 256), (50, 1),
                                   (64, 32), (62, 30), (40, 100), (64, 130)])
def test_wgrad_single_with_colsum(Ka, Nb, stream):
    """stream = GR_OPT_WGRAD_STREAM (Ka <= 64, Nb <= 256: the streaming form or the
    LDS-staged panels; other shapes ignore it)."""
    L = _lib()
    if stream == 0 and (Ka > 64 or Nb > 256):
        pytest.skip("the option only selects among the narrow forms")
    with L.option("WGRAD_STREAM", stream):
        _single_with_colsum(L, Ka, Nb)


def _single_with_colsum(L, Ka, Nb):
    offs, total, cap, a, b, st = _case([700, 1, 333, 64, 1000], Ka, Nb, Ka + Nb)
    lib = L.lib()
    ws_n = lib.gr_wgrad_workspace_size(cap, Ka, Nb)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device="cuda")
    c = torch.full((Ka, Nb), float("nan"), device="cuda")
    cs = torch.full((Ka,), float("nan"), device="cuda")
    L.call("gr_wgrad", a.data_ptr(), Ka, st.data_ptr(), b.data_ptr(), Nb, offs.data_ptr(),
           offs.numel() - 1, cap, Ka, Nb, c.data_ptr(), cs.data_ptr(), ws.data_ptr(), ws_n,
           L.stream_handle())
    torch.cuda.synchronize()
    rc, rcs = _ref(a, b, st, total)
    _check(c, rc, "C")
    _check(cs, rcs, "colsum")
    # deterministic: a second run is bit-identical
    c2 = torch.empty_like(c)
    cs2 = torch.empty_like(cs)
    L.call("gr_wgrad", a.data_ptr(), Ka, st.data_ptr(), b.data_ptr(), Nb, offs.data_ptr(),
           offs.numel() - 1, cap, Ka, Nb, c2.data_ptr(), cs2.data_ptr(), ws.data_ptr(), ws_n,
           L.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(c, c2) and torch.equal(cs, cs2)


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("D,n_out,hv", [(50, 200, 50), (256, 1024, 256), (128, 512, 128),
                                        (64, 256, 64), (64, 128, 32), (48, 160, 40)])
def test_wgrad2_layer_shapes(bf16, D, n_out, hv):
    """The layer's pair: (_uvqk: LN(x)^T d_uvqk, no colsum) + (_o: dy^T o_in, colsum)."""
    L = _lib()
    offs, total, cap, x, duvqk, st = _case([211, 5, 2048, 90], D, n_out, D + n_out)
    _, _, _, dy, o_in, _ = _case([211, 5, 2048, 90], D, hv, 3 * D + hv, stats=False)
    lib = L.lib()
    ws_n = lib.gr_wgrad2_workspace_size(cap, D, n_out, D, hv)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device="cuda")
    c0 = torch.full((D, n_out), float("nan"), device="cuda")
    c1 = torch.full((D, hv), float("nan"), device="cuda")
    cs1 = torch.full((D,), float("nan"), device="cuda")
    L.call("gr_wgrad2_bf16" if bf16 else "gr_wgrad2", x.data_ptr(), D, st.data_ptr(),
           duvqk.data_ptr(), n_out, D, n_out, c0.data_ptr(), None, dy.data_ptr(), D, None,
           o_in.data_ptr(), hv, D, hv, c1.data_ptr(), cs1.data_ptr(), offs.data_ptr(),
           offs.numel() - 1, cap, ws.data_ptr(), ws_n, L.stream_handle())
    torch.cuda.synchronize()
    r0, _ = _ref(x, duvqk, st, total, bf16)
    r1, rcs = _ref(dy, o_in, None, total, bf16)
    _check(c0, r0, "C0")
    _check(c1, r1, "C1")
    _check(cs1, rcs, "colsum1")


@pytest.mark.parametrize("Ka,Nb", [(256, 1024), (256, 256)])
def test_wgrad_single_wide_many_rows(Ka, Nb):
    """gr_wgrad at 128 < Ka <= 256 takes the wide plan; at C3 row counts (~65K rows) its
    slabs are larger than the narrow plan's, so gr_wgrad_workspace_size must size for it
    (the single-GEMM paths: frozen _o or frozen _uvqk at D = 256)."""
    L = _lib()
    offs, total, cap, a, b, st = _case([2059] * 32, Ka, Nb, 7 + Ka + Nb)
    lib = L.lib()
    ws_n = lib.gr_wgrad_workspace_size(cap, Ka, Nb)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device="cuda")
    c = torch.full((Ka, Nb), float("nan"), device="cuda")
    cs = torch.full((Ka,), float("nan"), device="cuda")
    L.call("gr_wgrad", a.data_ptr(), Ka, st.data_ptr(), b.data_ptr(), Nb, offs.data_ptr(),
           offs.numel() - 1, cap, Ka, Nb, c.data_ptr(), cs.data_ptr(), ws.data_ptr(), ws_n,
           L.stream_handle())
    torch.cuda.synchronize()
    rc, rcs = _ref(a, b, st, total)
    _check(c, rc, "C")
    _check(cs, rcs, "colsum")


def test_wgrad_stream_operand_over_1gib():
    """the streaming form masks padding k-steps and out-of-range
    columns with a buffer voffset that must fail the range check at ANY operand size.
    Rounds 1-5 used 2^30: with an operand over 1 GiB those lanes read real data there and
    added it into C.  Here A (no row stats, the _o problem's dy) and B are 1.1 GB each;
    the masked offset is now 2^31 (common.h OOB_OFF), above every num_records."""
    L = _lib()
    Ka = Nb = 64
    rows = [1_100_000, 1_050_001, 1_100_003, 1_050_000]  # 4.3 M rows: 1.1 GB per operand
    offs, total, cap, a, b, _ = _case(rows, Ka, Nb, 11, stats=False)
    assert a.numel() * 4 > (1 << 30) and b.numel() * 4 > (1 << 30)
    lib = L.lib()
    with L.option("WGRAD_STREAM", 1):
        ws_n = lib.gr_wgrad_workspace_size(cap, Ka, Nb)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device="cuda")
        c = torch.full((Ka, Nb), float("nan"), device="cuda")
        cs = torch.full((Ka,), float("nan"), device="cuda")
        L.call("gr_wgrad", a.data_ptr(), Ka, None, b.data_ptr(), Nb, offs.data_ptr(),
               offs.numel() - 1, cap, Ka, Nb, c.data_ptr(), cs.data_ptr(), ws.data_ptr(), ws_n,
               L.stream_handle())
        torch.cuda.synchronize()
    rc, rcs = _ref(a, b, None, total)
    _check(c, rc, "C")
    _check(cs, rcs, "colsum")
