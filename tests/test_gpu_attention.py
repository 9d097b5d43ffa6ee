"""GPU parity: HIP jagged HSTU attention vs the CPU oracle (oracle/hstu_oracle.py,
itself pinned to the reference's golden fixtures).  Tolerance: fp32 — max abs error
<= 2e-5 * (1 + max|ref|) on outputs; the kernel is f32 MFMA (exact fp32 products,
different summation order from MKL)."""
import numpy as np
import pytest
import torch

from oracle import hstu_oracle as O

pytestmark = pytest.mark.gpu

THR = None


def _thr():
    from mygenerativerecommenders_amd.bucket_table import BUCKET_THRESHOLDS
    return np.asarray(BUCKET_THRESHOLDS, dtype=np.int64)


def _case(seed, B, N, H, dqk, dv, lengths=None, with_ts=True, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    if lengths is None:
        lengths = torch.randint(1, N + 1, (B,), generator=g)
    lengths = torch.as_tensor(lengths, dtype=torch.int64)
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lengths, 0)])
    T = int(offsets[-1])
    uvqk = torch.randn(T, 2 * H * dv + 2 * H * dqk, generator=g) * scale
    ts = None
    if with_ts:
        start = torch.randint(950_000_000, 1_050_000_000, (B, 1), generator=g)
        inc = (torch.rand(B, N, generator=g) * 3e5).to(torch.int64)
        ts = start + torch.cumsum(inc, 1)
    pos_w = torch.randn(2 * N - 1, generator=g) * 0.5
    ts_w = torch.randn(129, generator=g) * 0.5
    return lengths, offsets, uvqk, ts, pos_w, ts_w


def _make_copies(u, offs, B, N, H, dqk, dv):
    """bf16 Q, K, V copies for the wide bf16 kernels (None where they do not apply)."""
    from mygenerativerecommenders_amd import _lib
    hv, hq = H * dv, H * dqk
    cb = _lib.lib().hstu_attn_bf16_copies_bytes(B, N, H, dqk, dv)
    if not cb or u.stride(0) % 2:
        return None
    c = torch.empty(cb, dtype=torch.uint8, device=u.device)
    _lib.call("hstu_attn_bf16_copies", u[:, 2 * hv:].data_ptr(), u[:, 2 * hv + hq:].data_ptr(),
              u[:, hv:].data_ptr(), u.stride(0), u.stride(0), offs.data_ptr(), B, N, H, dqk, dv,
              c.data_ptr(), _lib.stream_handle())
    return c


def _run_gpu_fwd(offsets, uvqk, ts, pos_w, ts_w, B, N, H, dqk, dv, entry="hstu_attn_fwd",
                 copies=False):
    from mygenerativerecommenders_amd import _lib
    dev = torch.device("cuda")
    u = uvqk.to(dev)
    hv, hq = H * dv, H * dqk
    q = u[:, 2 * hv:2 * hv + hq]
    k = u[:, 2 * hv + hq:]
    v = u[:, hv:2 * hv]
    out = torch.full((u.shape[0], hv), float("nan"), device=dev)
    offs = offsets.to(dev)
    thr = torch.tensor(_thr(), device=dev)
    tsd = ts.to(dev) if ts is not None else None
    pw = pos_w.to(dev)
    tw = ts_w.to(dev)
    max_len = int((offsets[1:] - offsets[:-1]).max()) if B else 0
    from mygenerativerecommenders_amd import ops
    bmap = ops.bucket_map(tsd, offs, N) if tsd is not None else None
    extra = ()
    if entry == "hstu_attn_fwd_bf16":
        extra = (_lib.ptr(_make_copies(u, offs, B, N, H, dqk, dv) if copies else None),)
    _lib.call(entry, q.data_ptr(), k.data_ptr(), v.data_ptr(), u.stride(0), u.stride(0),
              offs.data_ptr(), B, N, max_len, H, dqk, dv, _lib.ptr(bmap), pw.data_ptr(),
              tw.data_ptr(), 128, out.data_ptr(), out.stride(0), *extra, _lib.stream_handle())
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize("B,N,H,dqk,dv,with_ts", [
    (4, 43, 1, 16, 16, True),
    (4, 43, 1, 50, 50, True),
    (3, 75, 2, 25, 25, True),
    (2, 211, 1, 50, 50, True),
    (3, 130, 2, 8, 8, False),
    (2, 150, 1, 64, 64, True),
    (2, 100, 1, 128, 96, True),
    (2, 150, 1, 256, 256, True),   # wide (C3 head dim): 16-key LDS tiles
    (2, 90, 1, 200, 136, True),
    (2, 70, 2, 160, 160, False),
])
def test_attn_fwd_vs_oracle(B, N, H, dqk, dv, with_ts):
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(B * 7 + N, B, N, H, dqk, dv,
                                                      with_ts=with_ts)
    hv, hq = H * dv, H * dqk
    q = uvqk[:, 2 * hv:2 * hv + hq]
    k = uvqk[:, 2 * hv + hq:]
    v = uvqk[:, hv:2 * hv]
    cfg = O.HSTUConfig(N=N, D=1, H=H, dqk=dqk, dv=dv)
    ref = O.hstu_attention_jagged(q, k, v, offsets, ts, cfg, pos_w, ts_w, _thr())
    got = _run_gpu_fwd(offsets, uvqk, ts, pos_w, ts_w, B, N, H, dqk, dv)
    tol = 2e-5 * (1 + ref.abs().max().item())
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() <= tol


def test_attn_fwd_full_length_and_len1():
    B, N, H, d = 3, 64, 1, 16
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(5, B, N, H, d, d, lengths=[64, 1, 63])
    q, k, v = uvqk[:, 2 * d:3 * d], uvqk[:, 3 * d:], uvqk[:, d:2 * d]
    cfg = O.HSTUConfig(N=N, D=1, H=H, dqk=d, dv=d)
    ref = O.hstu_attention_jagged(q, k, v, offsets, ts, cfg, pos_w, ts_w, _thr())
    got = _run_gpu_fwd(offsets, uvqk, ts, pos_w, ts_w, B, N, H, d, d)
    assert (got - ref).abs().max().item() <= 2e-5 * (1 + ref.abs().max().item())


def _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, dqk, dv, hpre=None, bf16=False,
                 copies=False):
    from mygenerativerecommenders_amd import _lib
    dev = torch.device("cuda")
    u = uvqk.to(dev)
    hv, hq = H * dv, H * dqk
    q, k, v = u[:, 2 * hv:2 * hv + hq], u[:, 2 * hv + hq:], u[:, hv:2 * hv]
    do = dout.to(dev).contiguous()
    T = u.shape[0]
    d = torch.full((T, u.shape[1]), float("nan"), device=dev)
    dq, dk, dvv = d[:, 2 * hv:2 * hv + hq], d[:, 2 * hv + hq:], d[:, hv:2 * hv]
    offs = offsets.to(dev)
    thr = torch.tensor(_thr(), device=dev)
    tsd = ts.to(dev) if ts is not None else None
    pw, tw = pos_w.to(dev), ts_w.to(dev)
    dpw = torch.full_like(pw, float("nan"))
    dtw = torch.full_like(tw, float("nan"))
    max_len = int((offsets[1:] - offsets[:-1]).max()) if B else 0
    L = _lib.lib()
    ws_bytes = (L.hstu_attn_bwd_bf16_workspace_size(B, N, max_len, H, dqk, dv, 128) if bf16
                else L.hstu_attn_bwd_workspace_size_d(B, N, max_len, H, dqk, dv, 128))
    del thr
    ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device=dev)
    hd = hpre.to(dev) if hpre is not None else None
    hq_p = hd[:, 2 * hv:2 * hv + hq].data_ptr() if hd is not None else None
    hk_p = hd[:, 2 * hv + hq:].data_ptr() if hd is not None else None
    hv_p = hd[:, hv:2 * hv].data_ptr() if hd is not None else None
    from mygenerativerecommenders_amd import ops
    bmap = ops.bucket_map(tsd, offs, N) if tsd is not None else None
    _lib.call("hstu_attn_bwd_bf16" if bf16 else "hstu_attn_bwd", q.data_ptr(), k.data_ptr(),
              v.data_ptr(), u.stride(0), u.stride(0), do.data_ptr(), do.stride(0), offs.data_ptr(), B, N, max_len, H, dqk, dv,
              _lib.ptr(bmap), pw.data_ptr(), tw.data_ptr(), 128,
              hq_p, hk_p, hv_p, u.stride(0) if hd is not None else 0,
              dq.data_ptr(), dk.data_ptr(), dvv.data_ptr(), d.stride(0),
              dpw.data_ptr(), dtw.data_ptr(),
              *((_lib.ptr(_make_copies(u, offs, B, N, H, dqk, dv) if copies else None),) if bf16 else ()),
              ws.data_ptr(), ws_bytes, _lib.stream_handle())
    torch.cuda.synchronize()
    return dq.cpu(), dk.cpu(), dvv.cpu(), dpw.cpu(), dtw.cpu()


def _close(got, ref, rel=3e-5):
    tol = rel * (1 + ref.abs().max().item())
    err = (got - ref).abs().max().item()
    assert torch.isfinite(got).all(), "non-finite"
    assert err <= tol, f"max abs err {err:.3e} > tol {tol:.3e}"


@pytest.mark.parametrize("B,N,H,dqk,dv,with_ts", [
    (4, 43, 1, 16, 16, True),
    (4, 43, 1, 50, 50, True),
    (3, 75, 2, 25, 25, True),
    (2, 211, 1, 50, 50, True),
    (3, 130, 2, 8, 8, False),
    (2, 150, 1, 64, 64, True),
    (2, 100, 1, 128, 96, True),
    (2, 150, 1, 256, 256, True),
    (2, 90, 1, 200, 136, True),
    (2, 70, 2, 160, 160, False),
])
def test_attn_bwd_vs_oracle(B, N, H, dqk, dv, with_ts):
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(B * 11 + N, B, N, H, dqk, dv,
                                                      with_ts=with_ts)
    hv, hq = H * dv, H * dqk
    uv = uvqk.clone().requires_grad_(True)
    pw = pos_w.clone().requires_grad_(True)
    tw = ts_w.clone().requires_grad_(True)
    q, k, v = uv[:, 2 * hv:2 * hv + hq], uv[:, 2 * hv + hq:], uv[:, hv:2 * hv]
    cfg = O.HSTUConfig(N=N, D=1, H=H, dqk=dqk, dv=dv)
    ref = O.hstu_attention_jagged(q, k, v, offsets, ts, cfg, pw, tw, _thr())
    g = torch.Generator().manual_seed(99)
    dout = torch.randn(ref.shape, generator=g)
    (ref * dout).sum().backward()
    gq, gk, gv = (uv.grad[:, 2 * hv:2 * hv + hq], uv.grad[:, 2 * hv + hq:],
                  uv.grad[:, hv:2 * hv])
    dq, dk, dvv, dpw, dtw = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, dqk, dv)
    _close(dq, gq)
    _close(dk, gk)
    _close(dvv, gv)
    if with_ts:
        _close(dpw, pw.grad, rel=1e-4)
        _close(dtw, tw.grad, rel=1e-4)


def test_attn_c3_full_length():
    """C3 geometry: one full-length ml-20m sequence (N = 2059, d = 256) plus a short one,
    forward and backward against the oracle."""
    B, N, H, d = 2, 2059, 1, 256
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(23, B, N, H, d, d, lengths=[2059, 777],
                                                    scale=0.5)
    hv = H * d
    uv = uvqk.clone().requires_grad_(True)
    pw = pos_w.clone().requires_grad_(True)
    tw = ts_w.clone().requires_grad_(True)
    q, k, v = uv[:, 2 * hv:3 * hv], uv[:, 3 * hv:], uv[:, hv:2 * hv]
    cfg = O.HSTUConfig(N=N, D=1, H=H, dqk=d, dv=d)
    ref = O.hstu_attention_jagged(q, k, v, offsets, ts, cfg, pw, tw, _thr())
    got = _run_gpu_fwd(offsets, uvqk, ts, pos_w, ts_w, B, N, H, d, d)
    _close(got, ref.detach())
    g = torch.Generator().manual_seed(7)
    dout = torch.randn(ref.shape, generator=g)
    (ref * dout).sum().backward()
    dq, dk, dvv, dpw, dtw = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d)
    _close(dq, uv.grad[:, 2 * hv:3 * hv])
    _close(dk, uv.grad[:, 3 * hv:])
    _close(dvv, uv.grad[:, hv:2 * hv])
    _close(dpw, pw.grad, rel=1e-4)
    _close(dtw, tw.grad, rel=1e-4)


def test_attn_bwd_fused_silu_grad():
    B, N, H, d = 3, 75, 1, 32
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(17, B, N, H, d, d)
    g = torch.Generator().manual_seed(5)
    hpre = torch.randn(uvqk.shape, generator=g)
    dout = torch.randn(uvqk.shape[0], H * d, generator=g)
    a = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d)
    b = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d, hpre=hpre)
    s = torch.sigmoid(hpre)
    sg = s * (1 + hpre * (1 - s))
    hv = H * d
    _close(b[0], a[0] * sg[:, 2 * hv:3 * hv])
    _close(b[1], a[1] * sg[:, 3 * hv:])
    _close(b[2], a[2] * sg[:, hv:2 * hv])


@pytest.mark.parametrize("B,N,d", [(6, 211, 50), (5, 150, 64), (4, 300, 32)])
def test_attn_bwd_launch_modes_bitexact(B, N, d):
    """Every f32 backward launch form -- one fused launch (single tiles or tile pairs),
    split dK/dV + dQ launches, the two-pass form with stored dS, and the one-launch dS
    hand-off -- gives the same gradients: dK and dV bit-identical, dQ bit-identical except
    in the hand-off form (descending key tiles).  The relative-bias gradients are deterministic in
    each form, but a tile pair shares one slab (its two tiles' partials meet in LDS
    before the slab reduce), so across forms they agree to fp32 rounding."""
    from mygenerativerecommenders_amd import _lib
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(31 + N, B, N, 1, d, d)
    g = torch.Generator().manual_seed(3)
    dout = torch.randn(uvqk.shape[0], d, generator=g)
    hpre = torch.randn(uvqk.shape, generator=g)
    modes = [{}, {"ATTN_BWD_DS": 0}, {"ATTN_BWD_DS": 0, "ATTN_BWD_PAIRS": 2},
             {"ATTN_BWD_DS": 0, "ATTN_BWD_PAIRS": 0}, {"ATTN_BWD_DS": 0, "ATTN_BWD_SPLIT": 1},
             {"ATTN_BWD_DS": 1, "ATTN_BWD_PAIRS": 2},
             {"ATTN_BWD_DS": 2}, {"ATTN_BWD_DS": 2, "ATTN_BWD_PAIRS": 2}]
    outs = []
    for m in modes:
        old = {k: _lib.set_option(k, v) for k, v in m.items()}
        try:
            outs.append(_run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, 1, d, d,
                                     hpre=hpre))
        finally:
            for k, v in old.items():
                _lib.set_option(k, v)
    for m, o in zip(modes[1:], outs[1:]):
        for i, (x, y) in enumerate(zip(outs[0], o)):
            assert torch.isfinite(x).all() and torch.isfinite(y).all()
            if i < 3 and not (i == 0 and m.get("ATTN_BWD_DS") == 2):
                assert torch.equal(x, y), (m, i, (x - y).abs().max().item())
            else:  # bias grads across slab layouts; dQ of the in-launch hand-off (its key
                # tiles are summed in descending order, as they are published)
                _close(y, x, rel=1e-6)


@pytest.mark.parametrize("B,N,dqk,dv,with_ts", [(2, 300, 256, 256, True), (3, 140, 160, 160, True),
                                                (2, 90, 200, 136, False)])
def test_attn_bwd_wide_stored_ds_bitexact(B, N, dqk, dv, with_ts):
    """Wide heads (d > 128): dQ from the dS tiles the dK/dV pass stores
    (GR_OPT_ATTN_BWD_WIDE_DS, default) against the recomputing dQ pass (option 0), and
    the dK/dV forms (GR_OPT_ATTN_BWD_WIDE_SPLIT: one workgroup for both, the default; dV
    and dK as workgroups of one launch; as two launches): every gradient bit-identical (the
    same S, dS values, summed in the same order), with and without a bucket map, silu'(h)
    epilogue on."""
    from mygenerativerecommenders_amd import _lib
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(41 + N, B, N, 1, dqk, dv, with_ts=with_ts)
    g = torch.Generator().manual_seed(4)
    dout = torch.randn(uvqk.shape[0], dv, generator=g)
    hpre = torch.randn(uvqk.shape, generator=g)
    a = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, 1, dqk, dv, hpre=hpre)
    others = []
    with _lib.option("ATTN_BWD_WIDE_DS", 0):  # recomputing dQ pass (combined dK/dV)
        others.append(_run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, 1, dqk, dv, hpre=hpre))
    for sp in (1, 2):  # dV and dK workgroups in one launch; dV and dK launches
        with _lib.option("ATTN_BWD_WIDE_SPLIT", sp):
            others.append(_run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, 1, dqk, dv,
                                       hpre=hpre))
    for b in others:
        for i, (x, y) in enumerate(zip(a, b)):
            if i >= 3 and not with_ts:
                break  # no bias gradients without a bucket map
            assert torch.isfinite(x).all(), i
            assert torch.equal(x, y), (i, (x - y).abs().max().item())


def test_bucket_map_vs_reference_semantics():
    """Every causal (i, j) bucket of the device map equals the reference bucket fn
    (hstu.py:579-581 on ts_next(i) - ts(j)), including full-length rows (ts[N-1] wrap)
    and huge deltas near the clamp."""
    from mygenerativerecommenders_amd import ops
    B, N = 3, 130
    g = torch.Generator().manual_seed(3)
    lengths = torch.tensor([130, 1, 77])
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lengths, 0)])
    ts = torch.randint(0, 2**40, (B, N), generator=g)
    ts[0, :64] = torch.cumsum(torch.randint(0, 50, (64,), generator=g), 0)
    ts[2, 5] = 2**62
    dev = torch.device("cuda")
    bmap = ops.bucket_map(ts.to(dev), offsets.to(dev), N).cpu().numpy()
    T = (N + 63) // 64
    tpb = T * (T + 1) // 2
    qk = bmap[: B * tpb * 4096].reshape(B, tpb, 64, 64)
    kq = bmap[B * tpb * 4096:].reshape(B, tpb, 64, 64)
    for b in range(B):
        L = int(lengths[b])
        ext = torch.cat([ts[b], ts[b, N - 1:N]])
        for i in range(L):
            j = torch.arange(i + 1)
            ref = O.bucket_reference_semantics(ext[i + 1] - ts[b, :i + 1])
            qt = i // 64
            for jj in range(i + 1):
                kt = jj // 64
                t = qt * (qt + 1) // 2 + kt
                assert qk[b, t, i % 64, jj % 64] == int(ref[jj]), (b, i, jj)
                assert kq[b, t, jj % 64, i % 64] == int(ref[jj]), (b, i, jj)
            del j


# ---------------------------------------------------------------- bf16 compute mode
# hstu_attn_fwd_bf16: Q, K, V and P rounded to bf16 (MFMA operands), fp32 accumulation,
# fp32 bias / silu / output.  Tolerance: max abs error <= 1.5e-2 * (1 + max|ref|) against
# the fp32 oracle (bf16 keeps 8 mantissa bits: ~2^-9 relative per operand, and the
# output sums up to N of them).

BF16_FWD_TOL = 1.5e-2


@pytest.mark.parametrize("B,N,H,dqk,dv,with_ts", [
    (4, 43, 1, 16, 16, True),
    (4, 43, 1, 50, 50, True),
    (3, 75, 2, 25, 25, True),
    (2, 211, 1, 50, 50, True),      # C2 head
    (3, 130, 2, 8, 8, False),
    (2, 150, 1, 64, 64, True),
    (2, 100, 1, 128, 96, True),
    (2, 150, 1, 256, 256, True),    # C3 head
    (2, 90, 1, 200, 136, True),
    (2, 70, 2, 160, 160, False),
    (2, 2059, 1, 256, 256, True),   # C3 length
])
def test_attn_fwd_bf16_vs_oracle(B, N, H, dqk, dv, with_ts):
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(B * 7 + N, B, N, H, dqk, dv,
                                                      with_ts=with_ts)
    hv, hq = H * dv, H * dqk
    q = uvqk[:, 2 * hv:2 * hv + hq]
    k = uvqk[:, 2 * hv + hq:]
    v = uvqk[:, hv:2 * hv]
    cfg = O.HSTUConfig(N=N, D=1, H=H, dqk=dqk, dv=dv)
    ref = O.hstu_attention_jagged(q, k, v, offsets, ts, cfg, pos_w, ts_w, _thr())
    from mygenerativerecommenders_amd import _lib
    modes = [False]
    if _lib.lib().hstu_attn_bf16_copies_bytes(B, N, H, dqk, dv):
        modes.append(True)  # wide heads: the DMA-staged kernel on the bf16 copies
    for copies in modes:
        got = _run_gpu_fwd(offsets, uvqk, ts, pos_w, ts_w, B, N, H, dqk, dv,
                           entry="hstu_attn_fwd_bf16", copies=copies)
        assert torch.isfinite(got).all()
        err = (got - ref).abs().max().item()
        scale = 1 + ref.abs().max().item()
        print(f"bf16 fwd (copies={copies}) rel err {err / scale:.3e}")
        assert err <= BF16_FWD_TOL * scale
        # and it is genuinely the reduced-precision path (not the fp32 kernel)
        assert err > 0


# hstu_attn_bwd_bf16: bf16 MFMA operands (Q, K, V, dO, P, dS), fp32 accumulation and
# elementwise; the bias gradients sum fp32 dS.  Tolerance: max abs error
# <= 2e-2 * (1 + max|ref|) per gradient against the fp32 oracle.
BF16_BWD_TOL = 2e-2


@pytest.mark.parametrize("B,N,H,dqk,dv,with_ts", [
    (4, 43, 1, 16, 16, True),
    (4, 43, 1, 50, 50, True),
    (3, 75, 2, 25, 25, True),
    (2, 211, 1, 50, 50, True),      # C2 head
    (3, 130, 2, 8, 8, False),
    (2, 150, 1, 64, 64, True),
    (2, 100, 1, 128, 96, True),
    (2, 150, 1, 256, 256, True),    # C3 head (wide 32x32x16 path, hstu_attn_bf16w.hip)
    (2, 90, 1, 200, 136, True),     # dqk != dv: split dV / dK passes
    (2, 70, 2, 160, 160, False),
    (2, 300, 2, 192, 192, True),    # wide path, two heads, ragged 128-key tiles
    (3, 100, 1, 130, 130, True),    # wide path, 130 of 160 padded dims
    (2, 2059, 1, 256, 256, True),   # C3 length
])
def test_attn_bwd_bf16_vs_oracle(B, N, H, dqk, dv, with_ts):
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(B * 11 + N, B, N, H, dqk, dv,
                                                      with_ts=with_ts)
    hv, hq = H * dv, H * dqk
    uv = uvqk.clone().requires_grad_(True)
    pw = pos_w.clone().requires_grad_(True)
    tw = ts_w.clone().requires_grad_(True)
    q, k, v = uv[:, 2 * hv:2 * hv + hq], uv[:, 2 * hv + hq:], uv[:, hv:2 * hv]
    cfg = O.HSTUConfig(N=N, D=1, H=H, dqk=dqk, dv=dv)
    ref = O.hstu_attention_jagged(q, k, v, offsets, ts, cfg, pw, tw, _thr())
    g = torch.Generator().manual_seed(99)
    dout = torch.randn(ref.shape, generator=g)
    (ref * dout).sum().backward()
    gq, gk, gv = (uv.grad[:, 2 * hv:2 * hv + hq], uv.grad[:, 2 * hv + hq:],
                  uv.grad[:, hv:2 * hv])
    dq, dk, dvv, dpw, dtw = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, dqk, dv,
                                         bf16=True)
    pairs = [("dq", dq, gq), ("dk", dk, gk), ("dv", dvv, gv)]
    if with_ts:
        pairs += [("dpos", dpw, pw.grad), ("dts", dtw, tw.grad)]
    for name, got, want in pairs:
        err = (got - want).abs().max().item() / (1 + want.abs().max().item())
        print(f"bf16 bwd {name} rel err {err:.3e}")
        _close(got, want, rel=BF16_BWD_TOL)


@pytest.mark.parametrize("B,N,H,d,with_ts", [(2, 300, 2, 192, True), (2, 150, 1, 256, False)])
def test_attn_bwd_bf16_forward_copies_bitexact(B, N, H, d, with_ts):
    """The backward on the forward's bf16 copies equals the backward that converts its own
    operands, bit for bit (same rounding, same kernels)."""
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(B * 5 + N, B, N, H, d, d, with_ts=with_ts)
    g = torch.Generator().manual_seed(3)
    dout = torch.randn(uvqk.shape[0], H * d, generator=g)
    a = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d, bf16=True)
    b = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d, bf16=True, copies=True)
    for x, y in zip(a[:3] if not with_ts else a, b):  # no bias: dpos / dts are not written
        assert torch.equal(x, y)


@pytest.mark.parametrize("d", [32, 256])
def test_attn_bwd_bf16_fused_silu_grad(d):
    B, N, H = 3, 75, 1
    lengths, offsets, uvqk, ts, pos_w, ts_w = _case(17, B, N, H, d, d)
    g = torch.Generator().manual_seed(5)
    hpre = torch.randn(uvqk.shape, generator=g)
    dout = torch.randn(uvqk.shape[0], H * d, generator=g)
    a = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d, bf16=True)
    b = _run_gpu_bwd(offsets, uvqk, dout, ts, pos_w, ts_w, B, N, H, d, d, hpre=hpre, bf16=True)
    s = torch.sigmoid(hpre)
    sg = s * (1 + hpre * (1 - s))
    hv = H * d
    for x, y, sl in ((a[0], b[0], slice(2 * hv, 3 * hv)), (a[1], b[1], slice(3 * hv, 4 * hv)),
                     (a[2], b[2], slice(hv, 2 * hv))):
        assert torch.allclose(y, x * sg[:, sl], rtol=1e-5, atol=1e-6)
