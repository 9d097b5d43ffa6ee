"""GPU parity of the drop-in HSTU encoder against the reference's own outputs
(tests/golden/hstu_*.npz, recorded from the reference by oracle/gen_golden.py) and
against the CPU oracle at larger sizes.

Tolerances (fp32 path, f32 MFMA): outputs max-abs <= 3e-5 * (1 + max|ref|); input and
parameter gradients <= 2e-4 * (1 + max|ref|) (sums over up to ~10^4 terms)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import hstu_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _build(d):
    from mygenerativerecommenders_amd.hstu import HSTU
    N0, out_len = int(d["N0"]), int(d["out_len"])
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=int(d["D"]),
               item_embedding_dim=int(d["D"]), num_blocks=int(d["blocks"]), num_heads=int(d["H"]),
               linear_dim=int(d["dv"]), attention_dim=int(d["dqk"]), normalization="rel_bias",
               linear_config="uvqk", linear_activation="silu", linear_dropout_rate=0.2,
               attn_dropout_rate=0.0, concat_ua=bool(d["concat_ua"]))
    state = {k[6:]: torch.tensor(d[k]) for k in d.files if k.startswith("param:")}
    missing, unexpected = enc.load_state_dict(state, strict=False)
    assert not unexpected, unexpected
    assert missing == ["_attn_mask"], missing
    return enc


def _close(got, ref, rel, what):
    got = got.detach().float().cpu()
    ref = torch.as_tensor(ref).float()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    assert torch.isfinite(got).all(), what
    err = (got - ref).abs().max().item()
    tol = rel * (1 + ref.abs().max().item())
    assert err <= tol, f"{what}: max abs err {err:.3e} > {tol:.3e}"


CASES = sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, "hstu_*.npz")))


@pytest.mark.parametrize("name", CASES)
def test_hstu_vs_reference_golden(name):
    d = np.load(os.path.join(GOLDEN, f"hstu_{name}.npz"))
    enc = _build(d).cuda().eval()  # concat_ua cases run the concatenated-gate kernels
    x = torch.tensor(d["x"]).cuda().requires_grad_(True)
    lengths = torch.tensor(d["lengths"]).cuda()
    payload = {"timestamps": torch.tensor(d["ts"]).cuda()} if int(d["with_ts"]) else {}
    y, _ = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None, past_payloads=payload)
    _close(y, d["y"], 3e-5, "y")
    (y * torch.tensor(d["dy"]).cuda()).sum().backward()
    # the reference's x.grad is zero on padded rows as well
    _close(x.grad, d["dx"], 2e-4, "dx")
    for pname, p in enc.named_parameters():
        ref = d["grad:" + pname]
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        _close(g, ref, 2e-4, "grad " + pname)


@pytest.mark.parametrize("B,N0,out_len,D,blocks,H,dh,min_len", [
    (8, 200, 11, 50, 4, 1, 50, 20),     # ml-1m geometry (C2), jagged lengths U[20, 200]
    (2, 500, 11, 256, 2, 1, 256, 200),  # ml-20m-like width (C3: D = d = 256), 8 key tiles
    (2, 300, 11, 256, 1, 2, 128, 100),  # C3 variant h = 2, d = 128
    (2, 2048, 11, 256, 2, 1, 256, 2048),  # C3 geometry: N = 2059, a full 2048-token row
    (3, 2048, 11, 256, 2, 1, 256, 700),   # C3 ragged rows
])
def test_hstu_shapes_vs_oracle(B, N0, out_len, D, blocks, H, dh, min_len):
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=H, linear_dim=dh,
               attention_dim=dh, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for layer in enc._hstu._attention_layers:
            layer._rel_attn_bias._ts_w.normal_(0, 0.3, generator=g)
            layer._rel_attn_bias._pos_w.normal_(0, 0.3, generator=g)
    enc.eval()
    lengths = torch.randint(min_len, N0 + 1, (B,), generator=g)
    x = torch.randn(B, N, D, generator=g)
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    thr = np.asarray(__import__("mygenerativerecommenders_amd.bucket_table",
                                fromlist=["x"]).BUCKET_THRESHOLDS)
    cfg = O.HSTUConfig(N=N, D=D, H=H, dqk=dh, dv=dh)
    st = {k: v.detach().clone().requires_grad_(True) for k, v in enc.state_dict().items()
          if k != "_attn_mask"}
    layers = [O.layer_params_from_state(st, i) for i in range(blocks)]
    xr = x.clone().requires_grad_(True)
    yr = O.hstu_forward(lengths, xr, ts, cfg, layers, thr)
    dy = torch.randn(yr.shape, generator=g)
    (yr * dy).sum().backward()

    enc = enc.cuda()
    xg = x.cuda().requires_grad_(True)
    y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
    _close(y, yr, 3e-5, "y")
    (y * dy.cuda()).sum().backward()
    _close(xg.grad, xr.grad, 2e-4, "dx")
    for pname, p in enc.named_parameters():
        _close(p.grad, st[pname].grad, 2e-4, "grad " + pname)


def test_hstu_train_mode_dropout_statistics():
    """Training-mode dropout cannot match torch's RNG; check its statistics instead:
    the fraction of dropped o_in entries ~ p, kept ones scaled by 1/(1-p), and the
    backward regenerates the same mask (finite-difference check of dy . y)."""
    from mygenerativerecommenders_amd import ops
    torch.manual_seed(3)
    rows, D, hv = 4096, 32, 32
    dev = torch.device("cuda")
    offsets = torch.tensor([0, rows], device=dev)
    u = torch.randn(rows, 4 * hv, device=dev)
    attn = torch.randn(rows, hv, device=dev)
    w = torch.randn(D, hv, device=dev)
    b = torch.zeros(D, device=dev)
    from mygenerativerecommenders_amd import _lib
    stats = torch.empty(rows, 2, device=dev)
    o_in = torch.empty(rows, hv, device=dev)
    y = torch.empty(rows, D, device=dev)
    _lib.call("hstu_gate_o_fwd", u.data_ptr(), u.stride(0), attn.data_ptr(), hv,
              offsets.data_ptr(), 1, rows, hv, D, w.data_ptr(), b.data_ptr(), None, 0, 1e-6,
              0.2, 1234, None, stats.data_ptr(), o_in.data_ptr(), y.data_ptr(), D,
              _lib.stream_handle())
    torch.cuda.synchronize()
    ln = torch.nn.functional.layer_norm(attn, [hv], eps=1e-6)
    full = u[:, :hv] * ln
    kept = o_in != 0
    frac_drop = 1 - kept.float().mean().item()
    assert abs(frac_drop - 0.2) < 0.01
    assert torch.allclose(o_in[kept], full[kept] / 0.8, rtol=1e-4, atol=1e-5)
    assert torch.allclose(y, o_in @ w.t(), rtol=1e-4, atol=1e-4)
    # the backward regenerates the same mask from (seed, element)
    dy = torch.randn(rows, D, device=dev)
    du = torch.empty(rows, hv, device=dev)
    da = torch.empty(rows, hv, device=dev)
    _lib.call("hstu_gate_o_bwd", dy.data_ptr(), D, offsets.data_ptr(), 1, rows, hv, D,
              w.data_ptr(), u.data_ptr(), u.stride(0), attn.data_ptr(), hv, stats.data_ptr(),
              None, 0, 0.2, 1234, None, du.data_ptr(), hv, da.data_ptr(), hv,
              _lib.stream_handle())
    torch.cuda.synchronize()
    g = (dy @ w) * kept.float() / 0.8
    assert torch.allclose(du, g * ln, rtol=1e-4, atol=1e-5)
    # a device seed offset changes the mask
    off = torch.tensor([7], dtype=torch.int64, device=dev)
    o_in2 = torch.empty_like(o_in)
    _lib.call("hstu_gate_o_fwd", u.data_ptr(), u.stride(0), attn.data_ptr(), hv,
              offsets.data_ptr(), 1, rows, hv, D, w.data_ptr(), b.data_ptr(), None, 0, 1e-6,
              0.2, 1234, off.data_ptr(), stats.data_ptr(), o_in2.data_ptr(), y.data_ptr(), D,
              _lib.stream_handle())
    torch.cuda.synchronize()
    assert ((o_in2 != 0) != kept).float().mean().item() > 0.2
    del ops


@pytest.mark.parametrize("B,N0,out_len,D,blocks,min_len", [
    (8, 200, 11, 50, 4, 20),       # C2 geometry
    (2, 2048, 11, 256, 2, 700),    # C3 geometry
])
def test_hstu_bf16_mode_vs_oracle(B, N0, out_len, D, blocks, min_len):
    """autocast_dtype=torch.bfloat16: attention operands in bf16 (fp32 accumulation),
    projections / LN / parameters fp32.  Stated tolerance against the fp32 oracle:
    outputs max abs err <= 2e-2 * (1 + max|ref|), input and parameter gradients
    <= 5e-2 * (1 + max|ref|)."""
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
               autocast_dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for layer in enc._hstu._attention_layers:
            layer._rel_attn_bias._ts_w.normal_(0, 0.3, generator=g)
            layer._rel_attn_bias._pos_w.normal_(0, 0.3, generator=g)
    enc.eval()
    lengths = torch.randint(min_len, N0 + 1, (B,), generator=g)
    x = torch.randn(B, N, D, generator=g)
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    thr = np.asarray(__import__("mygenerativerecommenders_amd.bucket_table",
                                fromlist=["x"]).BUCKET_THRESHOLDS)
    cfg = O.HSTUConfig(N=N, D=D, H=1, dqk=D, dv=D)
    st = {k: v.detach().clone().requires_grad_(True) for k, v in enc.state_dict().items()
          if k != "_attn_mask"}
    layers = [O.layer_params_from_state(st, i) for i in range(blocks)]
    xr = x.clone().requires_grad_(True)
    yr = O.hstu_forward(lengths, xr, ts, cfg, layers, thr)
    dy = torch.randn(yr.shape, generator=g)
    (yr * dy).sum().backward()
    enc = enc.cuda()
    xg = x.cuda().requires_grad_(True)
    y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
    (y * dy.cuda()).sum().backward()

    def rel(got, ref):
        return (got.detach().cpu() - ref).abs().max().item() / (1 + ref.abs().max().item())

    ey = rel(y, yr)
    print(f"bf16 encoder y rel err {ey:.3e}")
    assert 0 < ey <= 2e-2
    assert rel(xg.grad, xr.grad) <= 5e-2
    for pname, p in enc.named_parameters():
        e = rel(p.grad, st[pname].grad)
        print(f"bf16 encoder grad {pname} rel err {e:.3e}")
        assert e <= 5e-2, pname


@pytest.mark.parametrize("D,H,N0", [(256, 1, 700), (192, 2, 300)])
def test_hstu_bf16_panel_vec_bitexact(D, H, N0):
    """The float4-staged bf16 row panel (GR_OPT_PANEL_VEC=1, K % 32 == 0) stages the same
    bf16 operands in the same k order as the scalar-staged one: encoder output and every
    gradient bit-identical between the two (ragged rows, partial last row tile; D = 192,
    H = 2 has a half-filled second UVQK column panel)."""
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    B, out_len = 3, 11
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=2, num_heads=H, linear_dim=D // H,
               attention_dim=D // H, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
               autocast_dtype=torch.bfloat16).cuda()
    g = torch.Generator().manual_seed(3)
    lengths = torch.tensor([N0 - 37, 19, N0 // 2])
    x = torch.randn(B, N, D, generator=g)
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(B, N, D, generator=g).cuda()

    from mygenerativerecommenders_amd import _lib

    def run(vec):
        prev = _lib.set_option("PANEL_VEC", vec)
        try:
            enc.zero_grad(set_to_none=True)
            enc._hstu._dropout_step.zero_()  # same dropout masks in both runs
            xg = x.cuda().requires_grad_(True)
            y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
            (y * dy).sum().backward()
            torch.cuda.synchronize()
        finally:
            _lib.set_option("PANEL_VEC", prev)
        return [y.detach().clone(), xg.grad.clone()] + [p.grad.clone() for p in enc.parameters()]

    a, b = run(1), run(0)
    assert torch.isfinite(a[0]).all()
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), i


@pytest.mark.parametrize("D,dh,H", [(50, 50, 1), (32, 16, 2), (64, 64, 1),
                                    (256, 256, 1), (192, 48, 2), (160, 40, 1)])
def test_hstu_concat_ua_vs_oracle(D, dh, H):
    """concat_ua=True at ml-1m-like widths (ragged lengths, relative bias) against the
    oracle (fp32 tolerances as above)."""
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    B, N0, out_len, blocks = 6, 120, 11, 2
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=H, linear_dim=dh,
               attention_dim=dh, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
               concat_ua=True).eval()
    g = torch.Generator().manual_seed(1)
    lengths = torch.randint(10, N0 + 1, (B,), generator=g)
    x = torch.randn(B, N, D, generator=g)
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    thr = np.asarray(__import__("mygenerativerecommenders_amd.bucket_table",
                                fromlist=["x"]).BUCKET_THRESHOLDS)
    cfg = O.HSTUConfig(N=N, D=D, H=H, dqk=dh, dv=dh, concat_ua=True)
    st = {k: v.detach().clone().requires_grad_(True) for k, v in enc.state_dict().items()
          if k != "_attn_mask"}
    layers = [O.layer_params_from_state(st, i) for i in range(blocks)]
    xr = x.clone().requires_grad_(True)
    yr = O.hstu_forward(lengths, xr, ts, cfg, layers, thr)
    dy = torch.randn(yr.shape, generator=g)
    (yr * dy).sum().backward()
    enc = enc.cuda()
    xg = x.cuda().requires_grad_(True)
    y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
    _close(y, yr, 3e-5, "y")
    (y * dy.cuda()).sum().backward()
    _close(xg.grad, xr.grad, 2e-4, "dx")
    for pname, p in enc.named_parameters():
        _close(p.grad, st[pname].grad, 2e-4, "grad " + pname)


def test_hstu_concat_ua_train_dropout_regenerates_mask():
    """Train mode with dropout: d(sum(y * dy)) / dx from the kernels equals a finite
    difference along a random direction (the backward regenerates the forward's
    3 hdv-wide o_in mask from the same counter)."""
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(4)
    B, N0, out_len, D = 3, 40, 5, 32
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=1, num_heads=1, linear_dim=D, attention_dim=D,
               normalization="rel_bias", linear_config="uvqk", linear_activation="silu",
               linear_dropout_rate=0.3, attn_dropout_rate=0.0, concat_ua=True).cuda().train()
    lengths = torch.tensor([40, 13, 27]).cuda()
    x = torch.randn(B, N, D, device="cuda", dtype=torch.float64).float()
    dy = torch.randn(B, N, D, device="cuda")
    direction = torch.randn(B, N, D, device="cuda")
    counter = enc._hstu._dropout_step  # one device counter per encoder forward
    step = counter.clone()

    def f(xx):
        counter.copy_(step)  # the forward bumps it: same mask every evaluation
        y, _ = enc(lengths, xx, None, {})
        return (y * dy).sum()

    xg = x.clone().requires_grad_(True)
    f(xg).backward()
    eps = 1e-2
    with torch.no_grad():
        fd = (f(x + eps * direction) - f(x - eps * direction)) / (2 * eps)
    an = (xg.grad * direction).sum()
    assert abs(fd.item() - an.item()) <= 2e-2 * (1 + abs(an.item())), (fd.item(), an.item())


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("B,N0,D,blocks,freeze", [(8, 200, 50, 4, None), (2, 500, 256, 2, None),
                                                 (4, 200, 50, 3, "_o"), (4, 200, 50, 2, "_uvqk")])
def test_hstu_stack_node_matches_per_layer_nodes(bf16, B, N0, D, blocks, freeze):
    """The encoder as one autograd node (ops.stu_stack: every layer's weight gradients in
    one gr_wgrad_multi launch pair) against one node per layer (ops.stu_layer), train
    mode with dropout: the forward and the input gradient are bit-identical (same
    kernels, same masks), the weight gradients agree to fp32 summation order
    (1e-5 relative), frozen parameters get no gradient."""
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    out_len = 11
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
               autocast_dtype=torch.bfloat16 if bf16 else None).cuda().train()
    if freeze:
        for name, p in enc.named_parameters():
            if freeze in name:
                p.requires_grad_(False)
    g = torch.Generator().manual_seed(5)
    lengths = torch.randint(N0 // 3, N0 + 1, (B,), generator=g)
    x = torch.randn(B, N, D, generator=g).cuda()
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(B, N, D, generator=g).cuda()
    from mygenerativerecommenders_amd import ops
    outs = []
    ops.FUSE_BOUNDARIES = False  # the fused boundaries: test_hstu_stack_boundaries_*
    for use_stack in (True, False):
        enc._hstu._use_stack = use_stack
        enc._hstu._dropout_step.zero_()  # same dropout masks in both runs
        enc.zero_grad(set_to_none=True)
        xg = x.clone().requires_grad_(True)
        y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
        (y * dy).sum().backward()
        outs.append((y.detach(), xg.grad, {n: (p.grad.clone() if p.grad is not None else None)
                                           for n, p in enc.named_parameters()}))
    enc._hstu._use_stack = True
    ops.FUSE_BOUNDARIES = True
    (y0, dx0, g0), (y1, dx1, g1) = outs
    assert torch.equal(y0, y1)
    assert torch.equal(dx0, dx1)
    for n in g0:
        if g1[n] is None:
            assert g0[n] is None, n
            continue
        assert g0[n] is not None, n
        err = (g0[n] - g1[n]).abs().max().item()
        # bf16 mode with one weight frozen: the per-layer node's single GEMM (gr_wgrad)
        # has fp32 operands, the stack's gr_wgrad_multi bf16 ones (the mode's operand type)
        tol = 5e-3 if (bf16 and freeze) else 1e-5
        assert err <= tol * (1 + g1[n].abs().max().item()), (n, err)


@pytest.mark.parametrize("B,N0,D,hdv,blocks,act,dropout", [
    (8, 200, 50, 50, 4, "silu", 0.2), (4, 100, 16, 16, 3, "silu", 0.0),
    (4, 120, 32, 64, 2, "none", 0.1), (3, 90, 64, 32, 3, "silu", 0.0),
    (2, 300, 256, 256, 2, "silu", 0.0)])
def test_hstu_stack_boundaries_match_unfused(B, N0, D, hdv, blocks, act, dropout):
    """Layer boundaries as one launch (hstu_boundary_fwd: gate_o(l) + LN/UVQK(l+1);
    hstu_boundary_bwd: ln_uvqk_bwd(l) + gate_o_bwd(l-1)) against the two launches each
    replaces, train mode (same dropout masks).  The fused launch runs the UVQK product as
    a row-wave MFMA chain where the separate launch may take the row panel (n_out > 128),
    so the two agree to fp32 summation order: 2e-5 relative to each tensor's largest
    entry.  Shapes outside the fused set (D = 256 here) run the two launches inside the
    entry point and must be bit-identical."""
    from mygenerativerecommenders_amd import ops
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(1)
    out_len = 11
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=hdv,
               attention_dim=hdv, normalization="rel_bias", linear_config="uvqk",
               linear_activation=act, linear_dropout_rate=dropout,
               attn_dropout_rate=0.0).cuda().train()
    g = torch.Generator().manual_seed(7)
    lengths = torch.randint(N0 // 3, N0 + 1, (B,), generator=g)
    x = torch.randn(B, N, D, generator=g).cuda()
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(B, N, D, generator=g).cuda()
    outs = []
    try:
        for fuse in (True, False):
            ops.FUSE_BOUNDARIES = fuse
            enc._hstu._dropout_step.zero_()
            enc.zero_grad(set_to_none=True)
            xg = x.clone().requires_grad_(True)
            y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
            (y * dy).sum().backward()
            outs.append((y.detach(), xg.grad, {n: p.grad.clone() for n, p in enc.named_parameters()}))
    finally:
        ops.FUSE_BOUNDARIES = True
    (y0, dx0, g0), (y1, dx1, g1) = outs

    def close(a, b, what):
        if D > 64 or hdv > 64:
            assert torch.equal(a, b), what
            return
        err = (a - b).abs().max().item()
        assert err <= 2e-5 * (1 + b.abs().max().item()), (what, err)
    close(y0, y1, "y")
    close(dx0, dx1, "dx")
    for n in g0:
        close(g0[n], g1[n], n)


@pytest.mark.parametrize("B,N0,D,hdv,blocks,rab", [(16, 200, 50, 50, 3, True), (6, 70, 64, 64, 2, True),
                                                    (5, 40, 48, 40, 2, True), (4, 96, 256, 256, 2, True),
                                                    (8, 64, 50, 20, 2, True), (16, 200, 50, 50, 3, False),
                                                    (6, 70, 64, 64, 2, False)])
def test_hstu_boundary_as_dq_epilogue_matches_separate(B, N0, D, hdv, blocks, rab):
    """hstu_attn_bwd_bnd runs the layer boundary (ln_uvqk_bwd(l) + gate_o_bwd(l - 1), or
    ln_uvqk_bwd(0) alone) as the epilogue of the attention dQ launch at narrow single-head
    shapes (GR_OPT_BOUNDARY_FUSE, default on), against the attention backward and the
    boundary as separate launches (option 0), train mode with dropout and ragged lengths.
    The epilogues are the row-wave units of hstu_boundary_fwd / _bwd (same operation
    order; hipcc may contract multiply-adds differently inside another kernel: the forward
    agrees to 1e-6 relative), and the first layer's ln_uvqk_bwd alone may take the row
    panel when separate (n_out > 128), so gradients agree to fp32 summation order: 2e-5
    relative.  Also the forward epilogue (hstu_attn_fwd_bnd) is exercised here, with and
    without the relative bias (rab = False: the no-bucket-map instantiations), n_out = 4 h dv
    up to 256 (h dv = 64).  Shapes the epilogue does not cover (D = 256; h dv = 20) run the
    separate launches inside the call and are bit-identical."""
    from mygenerativerecommenders_amd import _lib
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(3)
    out_len = 11
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=hdv,
               attention_dim=hdv, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2,
               attn_dropout_rate=0.0, enable_relative_attention_bias=rab).cuda().train()
    g = torch.Generator().manual_seed(11)
    lengths = torch.randint(1, N0 + 1, (B,), generator=g)
    lengths[0] = N0
    x = torch.randn(B, N, D, generator=g).cuda()
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(B, N, D, generator=g).cuda()
    outs = []
    for fuse in (1, 0):
        with _lib.option("BOUNDARY_FUSE", fuse):
            enc._hstu._dropout_step.zero_()
            enc.zero_grad(set_to_none=True)
            xg = x.clone().requires_grad_(True)
            y, _ = enc(lengths.cuda(), xg, None, {"timestamps": ts.cuda()})
            (y * dy).sum().backward()
            torch.cuda.synchronize()
            outs.append((y.detach(), xg.grad, {n: p.grad.clone() for n, p in enc.named_parameters()}))
    (y0, dx0, g0), (y1, dx1, g1) = outs
    exact = D > 64 or hdv <= 32

    def close(a, b, what, rel=2e-5):
        if exact:
            assert torch.equal(a, b), what
            return
        assert torch.isfinite(a).all(), what
        err = (a - b).abs().max().item()
        assert err <= rel * (1 + b.abs().max().item()), (what, err)
    # the epilogue is the same row-wave unit, but hipcc may contract its multiply-adds
    # differently inside another kernel: the forward agrees to a few ulp
    close(y0, y1, "y", 1e-6)
    close(dx0, dx1, "dx")
    for n in g0:
        close(g0[n], g1[n], n)


@pytest.mark.parametrize("bf16", [False, True])
def test_hstu_stack_wgrad_overlap(bf16):
    """Weight gradients on the side stream (ops.OVERLAP_WGRAD: layer l's launched beside
    the later layers' backward, layer 0's on the main stream) against all layers' in one
    launch at the end, eager and under HIP-graph capture: output and input gradient
    bit-identical, weight gradients equal to fp32 split-K order (1e-5 relative)."""
    from mygenerativerecommenders_amd import ops
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(2)
    B, N0, out_len, D, blocks = 8, 200, 11, 50, 4
    N = N0 + out_len
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
               autocast_dtype=torch.bfloat16 if bf16 else None).cuda().train()
    g = torch.Generator().manual_seed(9)
    lengths = torch.randint(N0 // 3, N0 + 1, (B,), generator=g).cuda()
    x = torch.randn(B, N, D, generator=g).cuda()
    ts = (1_000_000_000 + torch.cumsum(torch.randint(0, 200_000, (B, N), generator=g), 1)).cuda()
    dy = torch.randn(B, N, D, generator=g).cuda()

    def run():
        enc._hstu._dropout_step.zero_()
        enc.zero_grad(set_to_none=False)
        xg = x.clone().requires_grad_(True)
        y, _ = enc(lengths, xg, None, {"timestamps": ts})
        (y * dy).sum().backward()
        return y.detach().clone(), xg.grad.clone(), {n: p.grad.clone() for n, p in enc.named_parameters()}

    outs = []
    try:
        for ov in (True, False):
            ops.OVERLAP_WGRAD = ov
            outs.append(run())
        # the overlapped form captured in a graph and replayed
        ops.OVERLAP_WGRAD = True
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            run()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        enc._hstu._dropout_step.zero_()
        xg = x.clone().requires_grad_(True)
        with torch.cuda.graph(graph):
            y, _ = enc(lengths, xg, None, {"timestamps": ts})
            (y * dy).sum().backward()
        enc._hstu._dropout_step.zero_()
        for p in enc.parameters():
            p.grad.zero_()
        xg.grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
        outs.append((y.detach().clone(), xg.grad.clone(), {n: p.grad.clone() for n, p in enc.named_parameters()}))
    finally:
        ops.OVERLAP_WGRAD = False
    (y0, dx0, g0) = outs[1]
    for y1, dx1, g1 in (outs[0], outs[2]):
        assert torch.equal(y0, y1)
        assert torch.equal(dx0, dx1)
        for n in g0:
            err = (g0[n] - g1[n]).abs().max().item()
            assert err <= 1e-5 * (1 + g0[n].abs().max().item()), (n, err)
