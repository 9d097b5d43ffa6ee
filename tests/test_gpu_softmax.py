"""GPU parity of normalization="softmax_rel_bias" (sequential_encoders/hstu.py:341-389) —
the layer of ops.stu_softmax_layer over hstu_softmax_attn_fwd / _bwd — against the
reference's own record (tests/golden/softmax_*.npz, oracle/gen_golden.py) and the CPU
oracle (oracle/hstu_oracle.py::softmax_attention_jagged) at larger sizes.

Tolerances (fp32, FMA): outputs max-abs <= 3e-5 * (1 + max|ref|); input and parameter
gradients <= 2e-4 * (1 + max|ref|), as the encoder's golden tests."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import hstu_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(glob.glob(os.path.join(GOLDEN, "softmax_*.npz")))


def _build(d, rab=True, dropout=0.2):
    from mygenerativerecommenders_amd.hstu import HSTU
    enc = HSTU(max_sequence_len=int(d["N0"]), max_output_len=int(d["out_len"]),
               embedding_dim=int(d["D"]), item_embedding_dim=int(d["D"]),
               num_blocks=int(d["blocks"]), num_heads=int(d["H"]), linear_dim=int(d["dv"]),
               attention_dim=int(d["dqk"]), normalization="softmax_rel_bias",
               linear_config="uvqk", linear_activation="silu", linear_dropout_rate=dropout,
               attn_dropout_rate=0.0, concat_ua=bool(d["concat_ua"]),
               enable_relative_attention_bias=rab)
    state = {k[6:]: torch.tensor(np.asarray(d[k])) for k in d if k.startswith("param:")}
    missing, unexpected = enc.load_state_dict(state, strict=False)
    assert not unexpected and missing == ["_attn_mask"], (missing, unexpected)
    return enc.cuda().eval()


def _close(got, ref, rel, what):
    got = got.detach().float().cpu()
    ref = (ref.detach() if torch.is_tensor(ref) else torch.as_tensor(np.asarray(ref))).float()
    assert got.shape == ref.shape, (what, tuple(got.shape), tuple(ref.shape))
    assert torch.isfinite(got).all(), what
    err = (got - ref).abs().max().item() if got.numel() else 0.0
    assert err <= rel * (1 + ref.abs().max().item()), (what, err)


def _fwd_bwd(enc, d):
    x = torch.tensor(np.asarray(d["x"])).cuda().requires_grad_(True)
    y, _ = enc(past_lengths=torch.tensor(np.asarray(d["lengths"])).cuda(), user_embeddings=x,
               valid_mask=None, past_payloads={"timestamps": torch.tensor(np.asarray(d["ts"])).cuda()})
    (y * torch.tensor(np.asarray(d["dy"])).cuda()).sum().backward()
    return y, x.grad


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p) for p in CASES])
def test_softmax_matches_reference_golden(path):
    d = dict(np.load(path))
    enc = _build(d, rab=bool(int(d["rab"])))
    y, dx = _fwd_bwd(enc, d)
    _close(y, d["y"], 3e-5, "y")
    _close(dx, d["dx"], 2e-4, "dx")
    for name, p in enc.named_parameters():
        _close(p.grad if p.grad is not None else torch.zeros_like(p), d["grad:" + name], 2e-4, name)


def _random(B, N, D, H, dqk, dv, blocks, seed, rab=True, concat_ua=False):
    g = torch.Generator().manual_seed(seed)
    lengths = torch.randint(1, N + 1, (B,), generator=g)
    lengths[0] = N
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        ts[b] = 10**9 + torch.cumsum(torch.randint(1, 300000, (N,), generator=g), 0)
    from mygenerativerecommenders_amd.hstu import HSTU
    enc = HSTU(max_sequence_len=N - 1, max_output_len=1, embedding_dim=D, item_embedding_dim=D,
               num_blocks=blocks, num_heads=H, linear_dim=dv, attention_dim=dqk,
               normalization="softmax_rel_bias", linear_config="uvqk", linear_activation="silu",
               linear_dropout_rate=0.0, attn_dropout_rate=0.0, concat_ua=concat_ua,
               enable_relative_attention_bias=rab)
    with torch.no_grad():
        for name, p in enc.named_parameters():
            if "_pos_w" in name or "_ts_w" in name:
                p.normal_(0, 0.5, generator=g)
            if "_uvqk" in name:
                p.normal_(0, 0.2, generator=g)  # O(1) scores: the softmax is not flat
    d = {"N0": N - 1, "out_len": 1, "D": D, "H": H, "dqk": dqk, "dv": dv, "blocks": blocks,
         "concat_ua": int(concat_ua), "lengths": lengths.numpy(), "ts": ts.numpy(),
         "x": torch.randn(B, N, D, generator=g).numpy(),
         "dy": torch.randn(B, N, D, generator=g).numpy()}
    for name, p in enc.state_dict().items():
        if name != "_attn_mask":
            d["param:" + name] = p.numpy()
    return d


def _oracle(d, rab=True):
    cfg = O.HSTUConfig(N=int(d["N0"]) + 1, D=int(d["D"]), H=int(d["H"]), dqk=int(d["dqk"]),
                       dv=int(d["dv"]), concat_ua=bool(d["concat_ua"]), softmax=True)
    st = {k[6:]: torch.tensor(np.asarray(d[k]), requires_grad=True)
          for k in d if k.startswith("param:")}
    layers = [O.layer_params_from_state(st, i) for i in range(int(d["blocks"]))]
    x = torch.tensor(d["x"], requires_grad=True)
    thr = np.load(os.path.join(GOLDEN, "bucket_thresholds.npz"))["thresholds"]
    y = O.hstu_forward(torch.tensor(d["lengths"]), x, torch.tensor(d["ts"]), cfg, layers, thr)
    (y * torch.tensor(d["dy"])).sum().backward()
    return y, x.grad, {k: (p.grad if p.grad is not None else torch.zeros_like(p))
                       for k, p in st.items()}


@pytest.mark.parametrize("shape", [(16, 211, 50, 1, 50, 50, 2, True, False),
                                   (6, 80, 48, 2, 16, 24, 2, True, False),
                                   (5, 64, 32, 1, 32, 32, 1, False, False),
                                   (4, 40, 32, 1, 16, 16, 1, True, True)],
                         ids=["c2", "h2", "norab", "concat_ua"])
def test_softmax_matches_oracle(shape):
    B, N, D, H, dqk, dv, blocks, rab, cua = shape
    d = _random(B, N, D, H, dqk, dv, blocks, seed=N + B, rab=rab, concat_ua=cua)
    enc = _build(d, rab=rab, dropout=0.0)
    y, dx = _fwd_bwd(enc, d)
    y_ref, dx_ref, grads = _oracle(d, rab)
    _close(y, y_ref, 1e-4, "y")
    _close(dx, dx_ref, 3e-4, "dx")
    for name, p in enc.named_parameters():
        _close(p.grad, grads[name], 3e-4, name)


def test_softmax_cache_states_and_train_mode():
    """return_cache_states gives the reference's (v, padded q, padded k, outputs); train
    mode (dropout 0.2 before the O projection) runs forward and backward with finite
    gradients; the cached step raises as the reference's branch cannot run."""
    d = _random(3, 24, 16, 1, 16, 16, 1, seed=9)
    enc = _build(d, dropout=0.2)
    lengths = torch.tensor(d["lengths"]).cuda()
    ts = torch.tensor(d["ts"]).cuda()
    x = torch.tensor(d["x"]).cuda()
    with torch.no_grad():
        y, states = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
                        past_payloads={"timestamps": ts}, return_cache_states=True)
    rows = int(lengths.sum())
    v, pq, pk, out = states[0]
    assert v.shape == (rows, 16) and pq.shape == (3, 24, 16) and pk.shape == (3, 24, 16)
    assert out.shape == (rows, 16)
    assert torch.equal(y[0, :24], out[:24])  # sequence 0 has the full length
    with torch.no_grad(), pytest.raises(NotImplementedError, match="softmax_rel_bias"):
        off = torch.cat([torch.zeros(1, dtype=torch.int64, device="cuda"), lengths.cumsum(0)])
        enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
            past_payloads={"timestamps": ts}, delta_x_offsets=(off[:-1], off[:-1] * 0),
            cache=states)
    enc.train()
    xg = x.clone().requires_grad_(True)
    y, _ = enc(past_lengths=lengths, user_embeddings=xg, valid_mask=None,
               past_payloads={"timestamps": ts})
    y.square().sum().backward()
    assert torch.isfinite(xg.grad).all()
    assert all(torch.isfinite(p.grad).all() for p in enc.parameters())


def test_softmax_native_entry_points():
    from mygenerativerecommenders_amd import _lib
    d = _random(4, 32, 16, 1, 16, 16, 1, seed=4)
    enc = _build(d, dropout=0.0)
    _lib.timing_enable(True)
    try:
        _lib.kernel_times()
        _fwd_bwd(enc, d)
        t = _lib.kernel_times(("softmax_attn_fwd", "softmax_attn_bwd"))
    finally:
        _lib.timing_enable(False)
    assert t["softmax_attn_fwd"][1] == 1 and t["softmax_attn_bwd"][1] == 2, t
