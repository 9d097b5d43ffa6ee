"""GPU parity of the jagged data-movement kernels (utils/ops.py:18-114):
``asynchronous_complete_cumsum``, ``dense_to_jagged`` and ``jagged_to_padded_dense``
through the C-ABI, against the reference's own known answers (tests/golden/jagged_ops.npz,
restating reference tests/test_ops.py:7-53) and a numpy restatement on seeded ragged
inputs.  Pure copies: bit-exact."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _np_dense_to_jagged(dense, offs):
    return np.concatenate([dense[b, : offs[b + 1] - offs[b]] for b in range(len(offs) - 1)])


def _np_jagged_to_padded(values, offs, N):
    out = np.zeros((len(offs) - 1, N, values.shape[1]), values.dtype)
    for b in range(len(offs) - 1):
        L = min(int(offs[b + 1] - offs[b]), N)
        out[b, :L] = values[offs[b]:offs[b] + L]
    return out


def test_jagged_ops_reference_known_answers():
    from mygenerativerecommenders_amd import ops
    d = np.load(os.path.join(GOLDEN, "jagged_ops.npz"))
    offs = ops.asynchronous_complete_cumsum(torch.from_numpy(d["lengths"]).long().cuda())
    assert np.array_equal(offs.cpu().numpy(), d["offsets"])
    jag = ops.dense_to_jagged(torch.from_numpy(d["dense"]).cuda(), offs,
                              total_rows=int(d["offsets"][-1]))
    assert np.array_equal(jag.cpu().numpy(), d["jagged"])
    pad = ops.jagged_to_padded_dense(torch.from_numpy(d["values"]).cuda(),
                                     torch.from_numpy(d["offsets2"]).cuda(), 3)
    assert np.array_equal(pad.cpu().numpy(), d["padded"].astype(np.float32))


# D even -> float2 stream, D odd -> float stream; lengths include empty and full rows
@pytest.mark.parametrize("B,N,D", [(128, 211, 50), (5, 17, 7), (3, 1, 1), (9, 300, 256), (2, 2059, 256)])
def test_jagged_roundtrip_ragged(B, N, D):
    from mygenerativerecommenders_amd import ops
    g = torch.Generator().manual_seed(B * 1000 + N + D)
    lengths = torch.randint(0, N + 1, (B,), generator=g)
    lengths[0] = 0
    lengths[-1] = N
    dense = torch.randn(B, N, D, generator=g)
    offs_np = np.concatenate([[0], np.cumsum(lengths.numpy())]).astype(np.int64)
    offs = ops.asynchronous_complete_cumsum(lengths.cuda())
    assert np.array_equal(offs.cpu().numpy(), offs_np)
    total = int(offs_np[-1])
    jag = ops.dense_to_jagged(dense.cuda(), offs, total_rows=total)
    ref = _np_dense_to_jagged(dense.numpy(), offs_np)
    assert np.array_equal(jag.cpu().numpy(), ref)
    # the output is allocated uninitialised: padded rows must be written as exact zeros
    pad = ops.jagged_to_padded_dense(jag, offs, N)
    assert np.array_equal(pad.cpu().numpy(), _np_jagged_to_padded(ref, offs_np, N))


def test_jagged_unaligned_views_take_scalar_path():
    """A dense view starting 4 bytes into its storage cannot use 8-byte vectors; the
    result must still be exact."""
    from mygenerativerecommenders_amd import ops
    g = torch.Generator().manual_seed(7)
    B, N, D = 6, 40, 50
    storage = torch.randn(B * N * D + 1, generator=g).cuda()
    dense = storage[1:].view(B, N, D)
    lengths = torch.tensor([0, 40, 3, 17, 39, 1])
    offs_np = np.concatenate([[0], np.cumsum(lengths.numpy())]).astype(np.int64)
    offs = ops.asynchronous_complete_cumsum(lengths.cuda())
    jag = ops.dense_to_jagged(dense, offs, total_rows=int(offs_np[-1]))
    assert np.array_equal(jag.cpu().numpy(), _np_dense_to_jagged(dense.cpu().numpy(), offs_np))


def test_jagged_ops_autograd():
    """dense_to_jagged's backward is jagged_to_padded and vice versa (padding rows get 0)."""
    from mygenerativerecommenders_amd import ops
    g = torch.Generator().manual_seed(3)
    B, N, D = 4, 23, 50
    lengths = torch.tensor([23, 0, 11, 5])
    offs = ops.asynchronous_complete_cumsum(lengths.cuda())
    dense = torch.randn(B, N, D, generator=g).cuda().requires_grad_(True)
    jag = ops.dense_to_jagged(dense, offs, total_rows=int(lengths.sum()))
    w = torch.randn(jag.shape, generator=g).cuda()
    (jag * w).sum().backward()
    offs_np = np.concatenate([[0], np.cumsum(lengths.numpy())]).astype(np.int64)
    assert np.array_equal(dense.grad.cpu().numpy(), _np_jagged_to_padded(w.cpu().numpy(), offs_np, N))


@pytest.mark.parametrize("B", [0, 1, 63, 64, 65, 256, 257, 1000, 70000])
def test_complete_cumsum_sizes(B):
    """Scan edges: single lane, wave and workgroup boundaries, several rows per thread."""
    from mygenerativerecommenders_amd import ops
    g = torch.Generator().manual_seed(B)
    lengths = torch.randint(0, 3000, (B,), generator=g)
    offs = ops.asynchronous_complete_cumsum(lengths.cuda())
    ref = np.concatenate([[0], np.cumsum(lengths.numpy())]).astype(np.int64)
    assert np.array_equal(offs.cpu().numpy(), ref)


@pytest.mark.parametrize("D", [16, 7])
def test_dense_to_jagged_bounded_by_max_rows(D):
    """max_rows smaller than offsets[B]: nothing at or past it is written (canary tail),
    and the rows inside keep their values; with zero_fill the truncated tails and the
    rows past offsets[B] are zero."""
    from mygenerativerecommenders_amd import _lib
    dev = torch.device("cuda")
    B, N = 5, 12
    lengths = torch.tensor([12, 3, 15, 0, 9])  # 15 > N: truncated to N on copy
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lengths, 0)])
    dense = torch.randn(B, N, D)
    total = int(offs[-1])
    dense_d, offs_d = dense.to(dev), offs.to(dev)
    for max_rows, zero_fill in ((20, 0), (20, 1), (total + 6, 1)):
        buf = torch.full((total + 10, D), 7.0, device=dev)
        _lib.call("gr_dense_to_jagged", dense_d.data_ptr(), offs_d.data_ptr(), B, N,
                  D, max_rows, zero_fill, buf.data_ptr(), _lib.stream_handle())
        torch.cuda.synchronize()
        got = buf.cpu()
        assert torch.all(got[max_rows:] == 7.0), "wrote at or past max_rows"
        for b in range(B):
            s0, s1 = int(offs[b]), int(offs[b + 1])
            L = min(s1 - s0, N)
            for r in range(s0, min(s1, max_rows)):
                if r - s0 < L:
                    assert torch.equal(got[r], dense[b, r - s0])
                elif zero_fill:
                    assert torch.all(got[r] == 0)
        if zero_fill and max_rows > total:
            assert torch.all(got[total:max_rows] == 0)


def test_jagged_to_padded_grad_truncated_rows_are_zero():
    """Autograd through jagged_to_padded_dense with a length above N: the gradient of
    the rows no padded position reads is 0 (fbgemm semantics), not uninitialised."""
    from mygenerativerecommenders_amd import ops
    dev = torch.device("cuda")
    lengths = torch.tensor([4, 9, 2], device=dev)
    offs = ops.asynchronous_complete_cumsum(lengths)
    N, D = 6, 8
    values = torch.randn(15 + 3, D, device=dev, requires_grad=True)  # 3 rows past offsets[B]
    out = ops.jagged_to_padded_dense(values, offs, N)
    g = torch.randn_like(out)
    out.backward(g)
    grad = values.grad.cpu()
    ref = torch.zeros(18, D)
    o = offs.cpu()
    for b in range(3):
        s0, L = int(o[b]), min(int(lengths[b]), N)
        ref[s0:s0 + L] = g[b, :L].cpu()
    assert torch.equal(grad, ref)


# ------------------------------------------------------------------ encoder prologue
def _prologue_vs_separate(B, N, D, lengths, with_ts=True, with_step=True, dense=None):
    """hstu_encoder_prologue against the separate calls it replaces (cumsum, dense_to_jagged
    with zero_fill = 0, hstu_bucket_map, step += 1): offsets, the copied rows and the whole
    bucket map bit-identical, the counter advanced by one."""
    from mygenerativerecommenders_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(B * 7 + N + D)
    if dense is None:
        dense = torch.randn(B, N, D, generator=g).to(dev)
    ts = None
    if with_ts:
        inc = (-torch.log(torch.rand(B, N, generator=g).clamp_min(1e-12)) * 1e5).long()
        ts = (torch.randint(0, 10**9, (B, 1), generator=g) + torch.cumsum(inc, 1)).to(dev)
    step = torch.full((1,), 41, dtype=torch.int64, device=dev) if with_step else None
    lengths_d = lengths.to(dev)
    xj, offs, bmap = ops.encoder_prologue(lengths_d, dense, ts, step)
    offs_ref = ops.asynchronous_complete_cumsum(lengths_d)
    assert torch.equal(offs.cpu(), offs_ref.cpu())
    ref = ops.dense_to_jagged(dense, offs_ref, zero_fill=False)
    o = offs_ref.cpu()
    for b in range(B):
        s0, L = int(o[b]), min(int(lengths[b]), N)
        if s0 < B * N:
            L = min(L, B * N - s0)
            assert torch.equal(xj[s0:s0 + L].cpu(), ref[s0:s0 + L].cpu()), b
    if with_ts:
        assert torch.equal(bmap.cpu(), ops.bucket_map(ts, offs_ref, N).cpu())
    else:
        assert bmap is None
    if with_step:
        assert int(step.item()) == 42
    return dense, xj, offs


@pytest.mark.parametrize("B,N,D", [(128, 201, 50), (5, 17, 7), (3, 1, 1), (9, 300, 256),
                                   (2, 2059, 256), (70, 130, 64)])
def test_encoder_prologue_matches_separate_calls(B, N, D):
    g = torch.Generator().manual_seed(B + N)
    lengths = torch.randint(0, N + 1, (B,), generator=g)
    lengths[0] = 0
    lengths[-1] = N
    _prologue_vs_separate(B, N, D, lengths)


def test_encoder_prologue_edges():
    # no bucket map / no counter; lengths above N (truncated copies, offsets keep them)
    _prologue_vs_separate(6, 40, 50, torch.tensor([40, 0, 55, 3, 40, 1]), with_ts=False)
    _prologue_vs_separate(4, 64, 50, torch.tensor([64, 64, 64, 64]), with_step=False)
    # an unaligned view takes the 4-byte stream
    storage = torch.randn(6 * 40 * 50 + 1).cuda()
    _prologue_vs_separate(6, 40, 50, torch.tensor([0, 40, 3, 17, 39, 1]),
                          dense=storage[1:].view(6, 40, 50))
    # B = 0: offsets = [0] only
    from mygenerativerecommenders_amd import ops
    xj, offs, bmap = ops.encoder_prologue(torch.zeros(0, dtype=torch.int64, device="cuda"),
                                          torch.zeros(0, 5, 8, device="cuda"), None)
    assert offs.cpu().tolist() == [0] and xj.shape == (0, 8)


def test_encoder_prologue_autograd_and_hstu_forward():
    """dense gradient = jagged_to_padded of the jagged gradient; HSTU.forward through the
    prologue equals the separate-call path (same output, same input gradient)."""
    from mygenerativerecommenders_amd import ops
    from mygenerativerecommenders_amd.hstu import HSTU
    B, N, D = 4, 23, 50
    lengths = torch.tensor([23, 0, 11, 5])
    dense = torch.randn(B, N, D).cuda().requires_grad_(True)
    xj, offs, _ = ops.encoder_prologue(lengths.cuda(), dense, None)
    w = torch.randn(xj.shape).cuda()
    (xj[:39] * w[:39]).sum().backward()
    offs_np = np.concatenate([[0], np.cumsum(lengths.numpy())]).astype(np.int64)
    wz = w.cpu().numpy().copy()
    wz[39:] = 0
    assert np.array_equal(dense.grad.cpu().numpy(), _np_jagged_to_padded(wz, offs_np, N))

    torch.manual_seed(0)
    enc = HSTU(max_sequence_len=20, max_output_len=3, embedding_dim=D, item_embedding_dim=D,
               num_blocks=2, num_heads=1, linear_dim=D, attention_dim=D,
               normalization="rel_bias", linear_config="uvqk", linear_activation="silu",
               linear_dropout_rate=0.2, attn_dropout_rate=0.0).cuda()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, N, D, generator=g).cuda()
    inc = (-torch.log(torch.rand(B, N, generator=g).clamp_min(1e-12)) * 1e5).long()
    ts = (10**9 + torch.cumsum(inc, 1)).cuda()
    dy = torch.randn(B, N, D, generator=g).cuda()
    outs = []
    for use in (True, False):
        enc.use_prologue = use
        enc._hstu._dropout_step.zero_()
        xr = x.clone().requires_grad_(True)
        y, _ = enc(past_lengths=lengths.cuda(), user_embeddings=xr, valid_mask=None,
                   past_payloads={"timestamps": ts})
        y.backward(dy)
        outs.append((y.detach().cpu(), xr.grad.cpu(), int(enc._hstu._dropout_step.item())))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2] == 1
