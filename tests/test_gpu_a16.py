"""bf16 activations (ABI 16, the ``*_a16`` entries): HSTU(autocast_dtype=bfloat16) at wide
heads keeps uvqk, h_pre, o_in and d_uvqk in HBM as bf16 (reference hstu.py:439-480: under
autocast those mm outputs and their gradients are bf16).

Each a16 entry runs the same kernel as its ``*_bf16`` counterpart on the same bf16
operands, so the parity bar here is BIT-EXACT against that counterpart fed the
bf16-rounded inputs (fp32 in, fp32 out), with bf16 outputs compared to the counterpart's
fp32 output rounded to bf16.  The counterparts themselves are checked against the fp32
oracle in test_gpu_attention.py / test_gpu_hstu.py; the whole encoder in a16 mode is
checked against the oracle at C3 geometry in test_gpu_hstu.py::test_hstu_bf16_mode_vs_oracle
and below against the fp32-activation bf16 path."""
import numpy as np
import pytest
import torch

from mygenerativerecommenders_amd import _lib, ops

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _offsets(lengths):
    lens = torch.tensor(lengths, dtype=torch.int64)
    offs = torch.zeros(len(lengths) + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(lens, 0)
    return offs.to(DEV), int(offs[-1])


def _eq(a, b, what):
    assert a.shape == b.shape, what
    if a.dtype == torch.bfloat16:
        a, b = a.view(torch.int16), b.view(torch.int16)
    bad = (a != b)
    if a.is_floating_point():
        bad &= ~(torch.isnan(a) & torch.isnan(b))
    assert not bad.any(), f"{what}: {int(bad.sum())} of {a.numel()} differ"


def _bf(t):
    return t.to(torch.bfloat16)


def _img(w, transpose):
    """bf16 [N][K] weight image through gr_weight_images_bf16, checked against torch's
    round-to-nearest-even cast of the same matrix."""
    src = w.contiguous()
    R, C = src.shape
    out = torch.empty((C, R) if transpose else (R, C), dtype=torch.bfloat16, device=DEV)
    desc = np.array([[src.data_ptr(), R, C, 1 if transpose else 0, out.data_ptr()]], dtype=np.int64)
    _lib.call("gr_weight_images_bf16", desc.ctypes.data, 1, _lib.stream_handle())
    torch.cuda.synchronize()
    _eq(out, _bf(src.t().contiguous() if transpose else src), "weight image")
    return out


@pytest.mark.parametrize("D,n_out", [(256, 1024), (192, 768)])
def test_ln_uvqk_fwd_a16_bitexact(D, n_out):
    offs, total = _offsets([700, 1, 333, 2048, 64])
    cap = total + 21
    g = torch.Generator(device="cuda").manual_seed(D)
    x = torch.randn(cap, D, device=DEV, generator=g) * 1.5 + 0.3
    w = torch.randn(D, n_out, device=DEV, generator=g) * 0.05
    st = _lib.stream_handle()
    B = offs.numel() - 1
    xs32 = torch.empty(cap, 2, device=DEV)
    h32 = torch.empty(cap, n_out, device=DEV)
    u32 = torch.empty(cap, n_out, device=DEV)
    _lib.call("hstu_ln_uvqk_fwd_bf16", x.data_ptr(), D, offs.data_ptr(), B, cap, D, w.data_ptr(),
              n_out, 1e-6, 1, xs32.data_ptr(), h32.data_ptr(), u32.data_ptr(), n_out, st)
    xs = torch.empty(cap, 2, device=DEV)
    h16 = torch.empty(cap, n_out, dtype=torch.bfloat16, device=DEV)
    u16 = torch.empty(cap, n_out, dtype=torch.bfloat16, device=DEV)
    xn = torch.empty(cap, D, dtype=torch.bfloat16, device=DEV)
    wt = _img(w, True)
    _lib.call("hstu_ln_uvqk_fwd_a16", x.data_ptr(), D, offs.data_ptr(), B, cap, D, wt.data_ptr(),
              n_out, 1e-6, 1, xs.data_ptr(), 0, h16.data_ptr(), u16.data_ptr(), n_out,
              xn.data_ptr(), st)
    torch.cuda.synchronize()
    _eq(xs[:total], xs32[:total], "x_stats")
    _eq(h16[:total], _bf(h32[:total]), "h_pre")
    _eq(u16[:total], _bf(u32[:total]), "uvqk")
    ln = (x[:total] - xs[:total, 0:1]) * xs[:total, 1:2]
    _eq(xn[:total], _bf(ln), "xn = bf16(LN(x))")
    # statistics given (the previous layer's gate_o epilogue): the same outputs
    h2, u2, xn2 = torch.empty_like(h16), torch.empty_like(u16), torch.empty_like(xn)
    _lib.call("hstu_ln_uvqk_fwd_a16", x.data_ptr(), D, offs.data_ptr(), B, cap, D, wt.data_ptr(),
              n_out, 1e-6, 1, xs.data_ptr(), 1, h2.data_ptr(), u2.data_ptr(), n_out,
              xn2.data_ptr(), st)
    torch.cuda.synchronize()
    _eq(h2[:total], h16[:total], "h_pre (stats given)")
    _eq(u2[:total], u16[:total], "uvqk (stats given)")
    _eq(xn2[:total], xn[:total], "xn (stats given)")


def _attn_case(seed, lengths, N, d, H=1):
    offs, total = _offsets(lengths)
    g = torch.Generator(device="cuda").manual_seed(seed)
    n_out = 4 * H * d
    u16 = _bf(torch.randn(total + 5, n_out, device=DEV, generator=g))
    h16 = _bf(torch.randn(total + 5, n_out, device=DEV, generator=g))
    B = offs.numel() - 1
    start = torch.randint(950_000_000, 1_050_000_000, (B, 1), device=DEV, generator=g)
    ts = start + torch.cumsum((torch.rand(B, N, device=DEV, generator=g) * 3e5).long(), 1)
    bmap = ops.bucket_map(ts, offs, N)
    pos_w = torch.randn(2 * N - 1, device=DEV, generator=g) * 0.5
    ts_w = torch.randn(129, device=DEV, generator=g) * 0.5
    return offs, total, u16, h16, bmap, pos_w, ts_w, max(lengths)


@pytest.mark.parametrize("d,H,lengths,N", [(256, 1, [300, 1, 517, 64], 600),
                                           (192, 2, [129, 250, 7], 260),
                                           (256, 1, [2048, 1000], 2059)])
def test_attn_a16_bitexact(d, H, lengths, N):
    offs, total, u16, h16, bmap, pos_w, ts_w, max_len = _attn_case(d + N, lengths, N, d, H)
    B = offs.numel() - 1
    hv = H * d
    n_out = 4 * hv
    u32, h32 = u16.float(), h16.float()
    st = _lib.stream_handle()
    L = _lib.lib()
    # forward: the copies path on float(bf16) inputs vs the a16 path on the bf16 rows
    cb = L.hstu_attn_bf16_copies_bytes(B, N, H, d, d)
    cp = torch.empty(cb, dtype=torch.uint8, device=DEV)
    _lib.call("hstu_attn_bf16_copies", u32[:, 2 * hv:].data_ptr(), u32[:, 3 * hv:].data_ptr(),
              u32[:, hv:].data_ptr(), n_out, n_out, offs.data_ptr(), B, N, H, d, d, cp.data_ptr(), st)
    o32 = torch.full((total, hv), float("nan"), device=DEV)
    _lib.call("hstu_attn_fwd_bf16", u32[:, 2 * hv:].data_ptr(), u32[:, 3 * hv:].data_ptr(),
              u32[:, hv:].data_ptr(), n_out, n_out, offs.data_ptr(), B, N, max_len, H, d, d,
              bmap.data_ptr(), pos_w.data_ptr(), ts_w.data_ptr(), 128, o32.data_ptr(), hv,
              cp.data_ptr(), st)
    o16 = torch.full((total, hv), float("nan"), device=DEV)
    _lib.call("hstu_attn_fwd_a16", u16[:, 2 * hv:].data_ptr(), u16[:, 3 * hv:].data_ptr(),
              u16[:, hv:].data_ptr(), n_out, offs.data_ptr(), B, N, max_len, H, d,
              bmap.data_ptr(), pos_w.data_ptr(), ts_w.data_ptr(), 128,
              ops._zero_row(DEV).data_ptr(), o16.data_ptr(), hv, st)
    torch.cuda.synchronize()
    _eq(o16, o32, "attn out")
    # backward
    g = torch.Generator(device="cuda").manual_seed(7)
    dout16 = _bf(torch.randn(total, hv, device=DEV, generator=g))
    dout = dout16.float()
    ws_n = L.hstu_attn_bwd_bf16_workspace_size_copies(B, N, max_len, H, d, d, 128)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=DEV)
    d32 = torch.full((total + 5, n_out), float("nan"), device=DEV)
    dp32 = torch.empty(2 * N - 1, device=DEV)
    dt32 = torch.empty(129, device=DEV)
    _lib.call("hstu_attn_bwd_bf16", u32[:, 2 * hv:].data_ptr(), u32[:, 3 * hv:].data_ptr(),
              u32[:, hv:].data_ptr(), n_out, n_out, dout.data_ptr(), hv, offs.data_ptr(), B, N,
              max_len, H, d, d, bmap.data_ptr(), pos_w.data_ptr(), ts_w.data_ptr(), 128,
              h32[:, 2 * hv:].data_ptr(), h32[:, 3 * hv:].data_ptr(), h32[:, hv:].data_ptr(), n_out,
              d32[:, 2 * hv:].data_ptr(), d32[:, 3 * hv:].data_ptr(), d32[:, hv:].data_ptr(), n_out,
              dp32.data_ptr(), dt32.data_ptr(), cp.data_ptr(), ws.data_ptr(), ws_n, st)
    ws_a = L.hstu_attn_bwd_a16_workspace_size(B, N, max_len, H, d, 128)
    assert 0 < ws_a < ws_n
    wsa = torch.empty(ws_a, dtype=torch.uint8, device=DEV)
    d16 = torch.zeros(total + 5, n_out, dtype=torch.bfloat16, device=DEV)
    dp = torch.empty(2 * N - 1, device=DEV)
    dt = torch.empty(129, device=DEV)
    _lib.call("hstu_attn_bwd_a16", u16[:, 2 * hv:].data_ptr(), u16[:, 3 * hv:].data_ptr(),
              u16[:, hv:].data_ptr(), n_out, dout16.data_ptr(), hv, offs.data_ptr(), B, N, max_len,
              H, d, bmap.data_ptr(), pos_w.data_ptr(), ts_w.data_ptr(), 128,
              h16[:, 2 * hv:].data_ptr(), h16[:, 3 * hv:].data_ptr(), h16[:, hv:].data_ptr(), n_out,
              d16[:, 2 * hv:].data_ptr(), d16[:, 3 * hv:].data_ptr(), d16[:, hv:].data_ptr(), n_out,
              dp.data_ptr(), dt.data_ptr(), ops._zero_row(DEV).data_ptr(), wsa.data_ptr(), ws_a, st)
    torch.cuda.synchronize()
    _eq(d16[:total, hv:], _bf(d32[:total, hv:]), "dq / dk / dv")
    _eq(dp, dp32, "d pos_w")
    _eq(dt, dt32, "d ts_w")


@pytest.mark.parametrize("D,hv", [(256, 256), (192, 192), (256, 160)])
def test_gate_o_a16_bitexact(D, hv):
    offs, total = _offsets([700, 1, 333, 2048])
    cap = total + 9
    B = offs.numel() - 1
    g = torch.Generator(device="cuda").manual_seed(D + hv)
    n_out = 4 * hv
    uvqk16 = _bf(torch.randn(cap, n_out, device=DEV, generator=g))
    h16 = _bf(torch.randn(cap, n_out, device=DEV, generator=g))
    attn = torch.randn(cap, hv, device=DEV, generator=g)
    w_o = torch.randn(D, hv, device=DEV, generator=g) * 0.05
    b_o = torch.randn(D, device=DEV, generator=g)
    x = torch.randn(cap, D, device=DEV, generator=g)
    st = _lib.stream_handle()
    uvqk32, h32 = uvqk16.float(), h16.float()
    seed_off = torch.zeros(1, dtype=torch.int64, device=DEV)
    w_o16, wt_o16 = _img(w_o, False), _img(w_o, True)
    outs = {}
    for a16 in (False, True):
        ast = torch.empty(cap, 2, device=DEV)
        o_in = torch.empty(cap, hv, dtype=torch.bfloat16 if a16 else torch.float32, device=DEV)
        y = torch.empty(cap, D, device=DEV)
        u = uvqk16 if a16 else uvqk32
        ys = torch.full((cap, 2), float("nan"), device=DEV) if a16 and D == 256 else None
        _lib.call("hstu_gate_o_fwd_a16" if a16 else "hstu_gate_o_fwd_bf16", u.data_ptr(), n_out,
                  attn.data_ptr(), hv, offs.data_ptr(), B, cap, hv, D,
                  (w_o16 if a16 else w_o).data_ptr(), b_o.data_ptr(),
                  x.data_ptr(), D, 1e-6, 0.2, 1234, seed_off.data_ptr(), ast.data_ptr(),
                  o_in.data_ptr(), y.data_ptr(), D, *((_lib.ptr(ys),) if a16 else ()), st)
        if ys is not None:  # y's LN statistics = what the next LN + UVQK computes from y
            xs = torch.empty(cap, 2, device=DEV)
            wt = _img(torch.randn(D, 1024, device=DEV) * 0.05, True)
            hh = torch.empty(cap, 1024, dtype=torch.bfloat16, device=DEV)
            _lib.call("hstu_ln_uvqk_fwd_a16", y.data_ptr(), D, offs.data_ptr(), B, cap, D,
                      wt.data_ptr(), 1024, 1e-6, 1, xs.data_ptr(), 0, None, hh.data_ptr(), 1024,
                      None, st)
            torch.cuda.synchronize()
            _eq(ys[:total], xs[:total], "y_stats = LN statistics of y")
        dy = torch.randn(cap, D, device=DEV, generator=torch.Generator(device="cuda").manual_seed(3))
        du = torch.empty(cap, n_out, dtype=torch.bfloat16 if a16 else torch.float32, device=DEV)
        da = torch.empty(cap, hv, dtype=torch.bfloat16 if a16 else torch.float32, device=DEV)
        h = h16 if a16 else h32
        _lib.call("hstu_gate_o_bwd_a16" if a16 else "hstu_gate_o_bwd_bf16", dy.data_ptr(), D,
                  offs.data_ptr(), B, cap, hv, D, (wt_o16 if a16 else w_o).data_ptr(), u.data_ptr(), n_out,
                  attn.data_ptr(), hv, ast.data_ptr(), h.data_ptr(), n_out, 0.2, 1234,
                  seed_off.data_ptr(), du.data_ptr(), n_out, da.data_ptr(), hv, st)
        outs[a16] = (ast, o_in, y, du, da)
    torch.cuda.synchronize()
    (ast32, oin32, y32, du32, da32), (ast, oin, y, du, da) = outs[False], outs[True]
    n = total
    _eq(ast[:n], ast32[:n], "attn_stats")
    _eq(y[:n], y32[:n], "y")
    _eq(oin[:n], _bf(oin32[:n]), "o_in")
    _eq(du[:n, :hv], _bf(du32[:n, :hv]), "du")
    _eq(da[:n], _bf(da32[:n]), "d_attn")


@pytest.mark.parametrize("D,n_out", [(256, 1024), (192, 768)])
def test_ln_uvqk_bwd_a16_bitexact(D, n_out):
    offs, total = _offsets([700, 1, 333, 2048])
    cap = total + 9
    B = offs.numel() - 1
    g = torch.Generator(device="cuda").manual_seed(D)
    dh16 = _bf(torch.randn(cap, n_out, device=DEV, generator=g))
    w = torch.randn(D, n_out, device=DEV, generator=g) * 0.05
    x = torch.randn(cap, D, device=DEV, generator=g)
    xs = torch.stack([x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-6)], 1).contiguous()
    dy = torch.randn(cap, D, device=DEV, generator=g)
    st = _lib.stream_handle()
    dx32 = torch.empty(cap, D, device=DEV)
    dx16 = torch.empty(cap, D, device=DEV)
    dh32 = dh16.float()
    _lib.call("hstu_ln_uvqk_bwd_bf16", dh32.data_ptr(), n_out, offs.data_ptr(), B, cap, D, n_out,
              w.data_ptr(), x.data_ptr(), D, xs.data_ptr(), dy.data_ptr(), D, dx32.data_ptr(), D, st)
    _lib.call("hstu_ln_uvqk_bwd_a16", dh16.data_ptr(), n_out, offs.data_ptr(), B, cap, D, n_out,
              _img(w, False).data_ptr(), x.data_ptr(), D, xs.data_ptr(), dy.data_ptr(), D, dx16.data_ptr(), D, st)
    torch.cuda.synchronize()
    _eq(dx16[:total], dx32[:total], "dx")


def test_wgrad_multi_a16_bitexact():
    """The layer's two problems in the a16 layout (_uvqk: bf16 LN(x) x bf16 d_uvqk; _o:
    fp32 dy x bf16 o_in with the bias column sum) against gr_wgrad_multi(bf16=1) on the
    same values in fp32 (which rounds them to the same bf16 operands)."""
    offs, total = _offsets([2048] * 6 + [1000, 1])
    cap = total + 13
    B = offs.numel() - 1
    D, n_out, hv = 256, 1024, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    xn16 = _bf(torch.randn(cap, D, device=DEV, generator=g))
    du16 = _bf(torch.randn(cap, n_out, device=DEV, generator=g))
    dy = torch.randn(cap, D, device=DEV, generator=g)
    oin16 = _bf(torch.randn(cap, hv, device=DEV, generator=g))
    L = _lib.lib()
    res = {}
    for a16 in (False, True):
        c0 = torch.full((D, n_out), float("nan"), device=DEV)
        c1 = torch.full((D, hv), float("nan"), device=DEV)
        cs = torch.full((D,), float("nan"), device=DEV)
        if a16:
            keep = (xn16, du16, oin16)
            desc = np.array([[xn16.data_ptr(), D, 0, du16.data_ptr(), n_out, D, n_out, c0.data_ptr(), 0, 3],
                             [dy.data_ptr(), D, 0, oin16.data_ptr(), hv, D, hv, c1.data_ptr(), cs.data_ptr(), 2]],
                            dtype=np.int64)
            ws_n = L.gr_wgrad_multi_a16_workspace_size(desc.ctypes.data, 2, cap)
            ws = torch.empty(ws_n, dtype=torch.uint8, device=DEV)
            _lib.call("gr_wgrad_multi_a16", desc.ctypes.data, 2, offs.data_ptr(), B, cap,
                      ws.data_ptr(), ws_n, _lib.stream_handle())
        else:
            keep = (xn16.float(), du16.float(), oin16.float())
            desc = np.array([[keep[0].data_ptr(), D, 0, keep[1].data_ptr(), n_out, D, n_out, c0.data_ptr(), 0],
                             [dy.data_ptr(), D, 0, keep[2].data_ptr(), hv, D, hv, c1.data_ptr(), cs.data_ptr()]],
                            dtype=np.int64)
            ws_n = L.gr_wgrad_multi_workspace_size(desc.ctypes.data, 2, cap)
            ws = torch.empty(ws_n, dtype=torch.uint8, device=DEV)
            _lib.call("gr_wgrad_multi", desc.ctypes.data, 2, offs.data_ptr(), B, cap, 1,
                      ws.data_ptr(), ws_n, _lib.stream_handle())
        torch.cuda.synchronize()
        res[a16] = (c0, c1, cs)
        del keep
    for i, what in enumerate(("dW_uvqk", "dW_o", "db_o")):
        _eq(res[True][i], res[False][i], what)
    # and against fp64 on the bf16 operands
    ref = xn16[:total].double().t() @ du16[:total].double()
    err = (res[True][0].double() - ref).abs().max().item()
    assert err <= 1e-5 * (1 + ref.abs().max().item())


@pytest.mark.parametrize("shape", ["c3", "d192"])
def test_hstu_a16_vs_fp32_activation_bf16_mode(shape):
    """The whole encoder in bf16 mode with bf16 activations against the fp32-activation bf16
    path (ops.A16 = False): both round the MFMA operands to bf16; a16 also rounds uvqk,
    h_pre, o_in and d_uvqk where autocast would.  Tolerance (stated): output 2e-2, input
    and parameter gradients 5e-2, relative to 1 + max|ref| (the bf16 mode's bar against
    the fp32 oracle, test_hstu_bf16_mode_vs_oracle)."""
    from mygenerativerecommenders_amd.hstu import HSTU
    if shape == "c3":
        D, H, d, blocks, lengths = 256, 1, 256, 2, [300, 1, 517, 64]
    else:
        D, H, d, blocks, lengths = 192, 1, 192, 2, [129, 250, 7]
    N0, out_len = max(lengths) + 3, 0
    N = N0 + out_len
    B = len(lengths)
    torch.manual_seed(0)
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=H, linear_dim=d,
               attention_dim=d, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.0, attn_dropout_rate=0.0).to(DEV)
    enc._hstu._autocast_dtype = torch.bfloat16
    for layer in enc._hstu._attention_layers:
        layer._bf16 = True
    g = torch.Generator().manual_seed(1)
    lens = torch.tensor(lengths)
    x = torch.randn(B, N, D, generator=g).to(DEV)
    ts = (10**9 + torch.cumsum((torch.rand(B, N, generator=g) * 1e5).long(), 1)).to(DEV)
    dy = torch.randn(B, N, D, generator=g).to(DEV)
    res = {}
    for a16 in (True, False):
        ops.A16 = a16
        try:
            enc.zero_grad()
            xg = x.clone().requires_grad_(True)
            y, _ = enc(lens.to(DEV), xg, None, {"timestamps": ts})
            (y * dy).sum().backward()
            torch.cuda.synchronize()
            res[a16] = (y.detach(), xg.grad, {n: p.grad.clone() for n, p in enc.named_parameters()})
        finally:
            ops.A16 = True
    (ya, ga, pa), (yb, gb, pb) = res[True], res[False]
    mask = torch.arange(N, device=DEV)[None, :] < lens.to(DEV)[:, None]

    def rel(a, b):
        return (a - b).abs().max().item() / (1 + b.abs().max().item())
    assert rel(ya[mask], yb[mask]) <= 2e-2
    assert rel(ga[mask], gb[mask]) <= 5e-2
    for n in pb:
        assert rel(pa[n], pb[n]) <= 5e-2, n
