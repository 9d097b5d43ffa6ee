"""GPU parity of cached (incremental) HSTU decoding — the delta_x_offsets / cache branch of
sequential_encoders/hstu.py (:151-177, :293-298, :321-322, :393-423) — against the
reference's own record (tests/golden/decode_*.npz, oracle/gen_golden.py) and the CPU
oracle (oracle/hstu_oracle.py: hstu_forward_cached / stu_layer_cached).

Tolerances (fp32): outputs and caches max-abs <= 3e-5 * (1 + max|ref|), as the encoder's
golden tests."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import hstu_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(glob.glob(os.path.join(GOLDEN, "decode_*.npz")))
NAMES = ("v", "q", "k", "out")


def _build(d, bf16=False):
    from mygenerativerecommenders_amd.hstu import HSTU
    enc = HSTU(max_sequence_len=int(d["N0"]), max_output_len=int(d["out_len"]),
               embedding_dim=int(d["D"]), item_embedding_dim=int(d["D"]),
               num_blocks=int(d["blocks"]), num_heads=int(d["H"]), linear_dim=int(d["dv"]),
               attention_dim=int(d["dqk"]), normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
               concat_ua=bool(d["concat_ua"]),
               autocast_dtype=torch.bfloat16 if bf16 else None)
    state = {k[6:]: torch.tensor(np.asarray(d[k])) for k in d if k.startswith("param:")}
    missing, unexpected = enc.load_state_dict(state, strict=False)
    assert not unexpected and missing == ["_attn_mask"], (missing, unexpected)
    return enc.cuda().eval()


def _close(got, ref, what, rel=3e-5):
    got = got.detach().float().cpu()
    ref = torch.as_tensor(np.asarray(ref)).float()
    assert got.shape == ref.shape, (what, tuple(got.shape), tuple(ref.shape))
    err = (got - ref).abs().max().item() if got.numel() else 0.0
    assert err <= rel * (1 + ref.abs().max().item()), (what, err)


def _run(enc, d, key, states=None, delta=None):
    dev = "cuda"
    payload = {"timestamps": torch.tensor(d["ts" + key]).to(dev)} if int(d["with_ts"]) else {}
    B, N, D = d["x" + key].shape
    return enc(past_lengths=torch.tensor(d["lengths"]).to(dev),
               user_embeddings=torch.tensor(d["x" + key]).to(dev),
               valid_mask=torch.ones(B, N, 1, device=dev), past_payloads=payload,
               delta_x_offsets=delta, cache=states, return_cache_states=True)


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p) for p in CASES])
def test_decode_matches_reference_golden(path):
    d = dict(np.load(path))
    enc = _build(d)
    with torch.no_grad():
        y0, states = _run(enc, d, "0")
        _close(y0, d["y0"], "y0")
        for l, st in enumerate(states):
            for nm, t in zip(NAMES, st):
                _close(t, d[f"s0:{l}:{nm}"], f"s0:{l}:{nm}")
        held = [tuple(st) for st in states]
        delta = (torch.tensor(d["delta0"]).cuda(), torch.tensor(d["delta1"]).cuda())
        y1, states1 = _run(enc, d, "1", states, delta)
    _close(y1, d["y1"], "y1")
    for l, st in enumerate(states1):
        for i, (nm, t) in enumerate(zip(NAMES, st)):
            assert t is held[l][i], (l, nm)  # updated in place, as index_copy_ does
            _close(t, d[f"s1:{l}:{nm}"], f"s1:{l}:{nm}")


def _random_case(B, N, D, H, d, blocks, seed, with_ts=True, concat_ua=False, positions=None):
    g = torch.Generator().manual_seed(seed)
    lengths = torch.randint(1, N + 1, (B,), generator=g)
    lengths[0] = N  # a full-length row: query N - 1 takes the ts[N - 1] wrap
    pos = (torch.rand(B, generator=g) * lengths).long().clamp(max=lengths - 1)
    pos[1 % B] = lengths[1 % B] - 1
    if positions is not None:
        lengths[:] = N
        pos = torch.tensor(positions, dtype=torch.int64)
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        ts[b, :] = 10**9 + torch.cumsum(torch.randint(1, 200000, (N,), generator=g), 0)
    rec = {"N0": N - 1, "out_len": 1, "D": D, "H": H, "dqk": d, "dv": d, "blocks": blocks,
           "concat_ua": int(concat_ua), "with_ts": int(with_ts), "lengths": lengths.numpy(),
           "x0": torch.randn(B, N, D, generator=g).numpy(), "ts0": ts.numpy()}
    x1 = torch.tensor(rec["x0"]).clone()
    for b in range(B):
        x1[b, int(pos[b])] = torch.randn(D, generator=g)
    rec["x1"] = x1.numpy()
    ts1 = ts.clone()
    ts1[:, -1] += 7  # a moved timestamp changes the bias of every query reaching it
    rec["ts1"] = ts1.numpy()
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lengths, 0)])
    rec["delta0"], rec["delta1"] = (offsets[:-1] + pos).numpy(), pos.numpy()
    from mygenerativerecommenders_amd.hstu import HSTU
    enc = HSTU(max_sequence_len=N - 1, max_output_len=1, embedding_dim=D, item_embedding_dim=D,
               num_blocks=blocks, num_heads=H, linear_dim=d, attention_dim=d,
               normalization="rel_bias", linear_config="uvqk", linear_activation="silu",
               linear_dropout_rate=0.0, attn_dropout_rate=0.0, concat_ua=concat_ua)
    with torch.no_grad():
        for name, p in enc.named_parameters():
            if "_pos_w" in name or "_ts_w" in name:
                p.normal_(0, 0.5, generator=g)
    for name, p in enc.state_dict().items():
        if name != "_attn_mask":
            rec["param:" + name] = p.numpy()
    return rec


def _oracle_layers(d):
    cfg = O.HSTUConfig(N=int(d["N0"]) + int(d["out_len"]), D=int(d["D"]), H=int(d["H"]),
                       dqk=int(d["dqk"]), dv=int(d["dv"]), concat_ua=bool(d["concat_ua"]))
    st = {k[6:]: torch.tensor(np.asarray(d[k])) for k in d if k.startswith("param:")}
    return cfg, [O.layer_params_from_state(st, i) for i in range(int(d["blocks"]))]


@pytest.mark.parametrize("shape", [(16, 211, 50, 1, 50, 2), (6, 96, 64, 2, 32, 2),
                                   (3, 2059, 256, 1, 256, 1)],
                         ids=["c2", "h2", "c3_width"])
def test_decode_matches_oracle(shape):
    """Both passes against the oracle at the ml-1m shape (N = 211), two heads and the
    ml-20m width (D = dqk = dv = 256, N = 2059); each step's oracle starts from the
    GPU's own caches, so the decode is checked on its own."""
    B, N, D, H, d, blocks = shape
    rec = _random_case(B, N, D, H, d, blocks, seed=B * 1000 + N)
    enc = _build(rec)
    cfg, layers = _oracle_layers(rec)
    lengths = torch.tensor(rec["lengths"])
    with torch.no_grad():
        y0, states = _run(enc, rec, "0")
    y0_ref, states_ref = O.hstu_forward_cached(lengths, torch.tensor(rec["x0"]),
                                               torch.tensor(rec["ts0"]), cfg, layers)
    _close(y0, y0_ref, "y0", rel=1e-4)
    for l in range(blocks):
        for nm, t, r in zip(NAMES, states[l], states_ref[l]):
            _close(t, r, f"s0:{l}:{nm}", rel=1e-4)
    cpu_states = [tuple(t.detach().cpu().clone() for t in st) for st in states]
    delta = (torch.tensor(rec["delta0"]).cuda(), torch.tensor(rec["delta1"]).cuda())
    with torch.no_grad():
        y1, states1 = _run(enc, rec, "1", states, delta)
    y1_ref, states1_ref = O.hstu_forward_cached(
        lengths, torch.tensor(rec["x1"]), torch.tensor(rec["ts1"]), cfg, layers,
        delta=(torch.tensor(rec["delta0"]), torch.tensor(rec["delta1"])), cache=cpu_states)
    _close(y1, y1_ref, "y1", rel=1e-4)
    for l in range(blocks):
        for nm, t, r in zip(NAMES, states1[l], states1_ref[l]):
            _close(t, r, f"s1:{l}:{nm}", rel=1e-4)


@pytest.mark.parametrize("d", [50, 32], ids=["scalar_d50", "vec_d32"])
def test_decode_chunk_boundaries(d):
    """Positions on both sides of the 64-key chunk boundaries of hstu_decode_attn (its
    chunk partials are summed by the reduce launch), at a head dim read by scalar loads
    (d = 50) and by float4 loads (d = 32)."""
    rec = _random_case(7, 200, d, 1, d, 2, seed=d, positions=[0, 63, 64, 127, 128, 198, 199])
    enc = _build(rec)
    cfg, layers = _oracle_layers(rec)
    with torch.no_grad():
        _, states = _run(enc, rec, "0")
        cpu_states = [tuple(t.cpu().clone() for t in st) for st in states]
        delta = (torch.tensor(rec["delta0"]).cuda(), torch.tensor(rec["delta1"]).cuda())
        y1, states1 = _run(enc, rec, "1", states, delta)
    y1_ref, states1_ref = O.hstu_forward_cached(
        torch.tensor(rec["lengths"]), torch.tensor(rec["x1"]), torch.tensor(rec["ts1"]), cfg,
        layers, delta=(torch.tensor(rec["delta0"]), torch.tensor(rec["delta1"])), cache=cpu_states)
    _close(y1, y1_ref, "y1", rel=1e-4)
    for l in range(2):
        for nm, t, r in zip(NAMES, states1[l], states1_ref[l]):
            _close(t, r, f"s1:{l}:{nm}", rel=1e-4)


def test_decode_without_bias_and_concat_ua():
    rec = _random_case(5, 40, 32, 1, 16, 2, seed=7, with_ts=False, concat_ua=True)
    enc = _build(rec)
    cfg, layers = _oracle_layers(rec)
    lengths = torch.tensor(rec["lengths"])
    with torch.no_grad():
        _, states = _run(enc, rec, "0")
        cpu_states = [tuple(t.cpu().clone() for t in st) for st in states]
        delta = (torch.tensor(rec["delta0"]).cuda(), torch.tensor(rec["delta1"]).cuda())
        y1, _ = _run(enc, rec, "1", states, delta)
    y1_ref, _ = O.hstu_forward_cached(
        lengths, torch.tensor(rec["x1"]), None, cfg, layers,
        delta=(torch.tensor(rec["delta0"]), torch.tensor(rec["delta1"])), cache=cpu_states)
    _close(y1, y1_ref, "y1", rel=1e-4)


def test_decode_from_bf16_caches():
    """bf16 mode: the full pass runs bf16 MFMA; its caches (fp32 copies) feed the fp32
    cached step, which must equal the oracle's step over the same caches."""
    rec = _random_case(4, 129, 256, 1, 256, 1, seed=11)
    enc = _build(rec, bf16=True)
    cfg, layers = _oracle_layers(rec)
    with torch.no_grad():
        _, states = _run(enc, rec, "0")
        assert all(t.dtype == torch.float32 for st in states for t in st)
        cpu_states = [tuple(t.cpu().clone() for t in st) for st in states]
        delta = (torch.tensor(rec["delta0"]).cuda(), torch.tensor(rec["delta1"]).cuda())
        y1, _ = _run(enc, rec, "1", states, delta)
    y1_ref, _ = O.hstu_forward_cached(
        torch.tensor(rec["lengths"]), torch.tensor(rec["x1"]), torch.tensor(rec["ts1"]), cfg,
        layers, delta=(torch.tensor(rec["delta0"]), torch.tensor(rec["delta1"])), cache=cpu_states)
    _close(y1, y1_ref, "y1", rel=1e-4)


def test_decode_errors():
    rec = _random_case(3, 16, 16, 1, 16, 1, seed=3)
    enc = _build(rec)
    with torch.no_grad():
        _, states = _run(enc, rec, "0")
    good = (torch.tensor(rec["delta0"]).cuda(), torch.tensor(rec["delta1"]).cuda())
    with pytest.raises(NotImplementedError, match="inference-only"):
        _run(enc, rec, "1", states, good)  # autograd on: no backward exists
    with torch.no_grad():
        with pytest.raises(ValueError, match="cache"):
            _run(enc, rec, "1", None, good)
        with pytest.raises(ValueError, match="one per sequence"):
            _run(enc, rec, "1", states, (good[0][:2], good[1][:2]))
        bad = good[0].clone()
        bad[0] = int(np.sum(rec["lengths"]))
        with pytest.raises(IndexError):
            _run(enc, rec, "1", states, (bad, good[1]))
        with pytest.raises(IndexError):
            _run(enc, rec, "1", states, (good[0], good[1] + 16))


def test_decode_native_entry_points():
    """The cached step runs the library's kernels (no torch fallback): its launches are
    recorded by the library's own timing."""
    from mygenerativerecommenders_amd import _lib
    rec = _random_case(4, 32, 16, 1, 16, 1, seed=5)
    enc = _build(rec)
    with torch.no_grad():
        _, states = _run(enc, rec, "0")
        delta = (torch.tensor(rec["delta0"]).cuda(), torch.tensor(rec["delta1"]).cuda())
        _lib.timing_enable(True)
        try:
            _lib.kernel_times()
            _run(enc, rec, "1", states, delta)
            t = _lib.kernel_times(("decode_attn", "decode_scatter", "rows_copy", "ln_uvqk_fwd",
                                   "gate_o_fwd"))
        finally:
            _lib.timing_enable(False)
    # one layer: the row gather and the output scatter; the cache scatter; the chunk and
    # reduce launches of the attention
    assert t["decode_attn"][1] == 2 and t["decode_scatter"][1] == 1, t
    assert t["rows_copy"][1] == 2, t
