"""CPU: the oracle restatement against the reference's own recorded outputs
(tests/golden/*.npz, written by oracle/gen_golden.py from /root/reference).

This pins the oracle: every GPU parity test compares against it (or against the
goldens directly)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import hstu_oracle as O
from oracle import topk_oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
HSTU_CASES = sorted(glob.glob(os.path.join(GOLDEN, "hstu_*.npz")))
DECODE_CASES = sorted(glob.glob(os.path.join(GOLDEN, "decode_*.npz")))
SOFTMAX_CASES = sorted(glob.glob(os.path.join(GOLDEN, "softmax_*.npz")))


def _thr():
    return np.load(os.path.join(GOLDEN, "bucket_thresholds.npz"))["thresholds"]


def test_package_bucket_table_matches_reference_golden():
    from mygenerativerecommenders_amd.bucket_table import BUCKET_THRESHOLDS, NUM_BUCKETS
    assert NUM_BUCKETS == 128
    assert np.array_equal(np.asarray(BUCKET_THRESHOLDS, dtype=np.int64), _thr())


def test_bucket_threshold_form_equals_reference_semantics():
    d = np.load(os.path.join(GOLDEN, "bucket_thresholds.npz"))
    x = torch.from_numpy(d["probe_x"])
    ref = torch.from_numpy(d["probe_bucket"])
    assert torch.equal(O.bucket_via_thresholds(x, d["thresholds"]), ref)
    assert torch.equal(O.bucket_via_thresholds(-x, d["thresholds"]), ref)
    assert torch.equal(O.bucket_reference_semantics(x), ref)
    # random int64 deltas over the whole clamp range
    g = torch.Generator().manual_seed(0)
    r = torch.randint(-(2**62), 2**62, (200_000,), generator=g)
    assert torch.equal(O.bucket_via_thresholds(r, d["thresholds"]),
                       O.bucket_reference_semantics(r))


@pytest.mark.parametrize("path", HSTU_CASES, ids=[os.path.basename(p) for p in HSTU_CASES])
@pytest.mark.parametrize("variant", ["jagged", "padded"])
def test_hstu_oracle_vs_reference(path, variant):
    d = np.load(path)
    cfg = O.HSTUConfig(N=int(d["N"]), D=int(d["D"]), H=int(d["H"]), dqk=int(d["dqk"]),
                       dv=int(d["dv"]), concat_ua=bool(d["concat_ua"]))
    st = {k[6:]: torch.tensor(d[k], requires_grad=True) for k in d.files if k.startswith("param:")}
    layers = [O.layer_params_from_state(st, i) for i in range(int(d["blocks"]))]
    x = torch.tensor(d["x"], requires_grad=True)
    ts = torch.tensor(d["ts"]) if int(d["with_ts"]) else None
    fn = O.hstu_forward if variant == "jagged" else O.hstu_forward_padded
    y = fn(torch.tensor(d["lengths"]), x, ts, cfg, layers, _thr())
    (y * torch.tensor(d["dy"])).sum().backward()
    assert (y - torch.tensor(d["y"])).abs().max().item() <= 1e-5
    assert (x.grad - torch.tensor(d["dx"])).abs().max().item() <= 1e-5
    for k, p in st.items():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        ref = torch.tensor(d["grad:" + k])
        assert (g - ref).abs().max().item() <= 2e-5 * (1 + ref.abs().max().item()), k


@pytest.mark.parametrize("path", SOFTMAX_CASES, ids=[os.path.basename(p) for p in SOFTMAX_CASES])
def test_softmax_oracle_vs_reference(path):
    """normalization="softmax_rel_bias" (hstu.py:341-389): output and every gradient."""
    d = np.load(path)
    cfg = O.HSTUConfig(N=int(d["N"]), D=int(d["D"]), H=int(d["H"]), dqk=int(d["dqk"]),
                       dv=int(d["dv"]), concat_ua=bool(d["concat_ua"]), softmax=True)
    st = {k[6:]: torch.tensor(d[k], requires_grad=True) for k in d.files if k.startswith("param:")}
    layers = [O.layer_params_from_state(st, i) for i in range(int(d["blocks"]))]
    x = torch.tensor(d["x"], requires_grad=True)
    y = O.hstu_forward(torch.tensor(d["lengths"]), x, torch.tensor(d["ts"]), cfg, layers, _thr())
    (y * torch.tensor(d["dy"])).sum().backward()
    assert (y - torch.tensor(d["y"])).abs().max().item() <= 1e-5
    assert (x.grad - torch.tensor(d["dx"])).abs().max().item() <= 1e-5
    for k, p in st.items():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        ref = torch.tensor(d["grad:" + k])
        assert (g - ref).abs().max().item() <= 2e-5 * (1 + ref.abs().max().item()), k


def _decode_case(d):
    cfg = O.HSTUConfig(N=int(d["N"]), D=int(d["D"]), H=int(d["H"]), dqk=int(d["dqk"]),
                       dv=int(d["dv"]), concat_ua=bool(d["concat_ua"]))
    st = {k[6:]: torch.tensor(d[k]) for k in d.files if k.startswith("param:")}
    layers = [O.layer_params_from_state(st, i) for i in range(int(d["blocks"]))]
    return cfg, layers


@pytest.mark.parametrize("path", DECODE_CASES, ids=[os.path.basename(p) for p in DECODE_CASES])
def test_decode_oracle_vs_reference(path):
    """The cached path (hstu.py:293-298, 321-322, 151-177, 415-418): full pass with cache
    states, then one re-encoded position per sequence, against the reference's record."""
    d = np.load(path)
    cfg, layers = _decode_case(d)
    with_ts = int(d["with_ts"])
    lengths = torch.tensor(d["lengths"])
    y0, states = O.hstu_forward_cached(lengths, torch.tensor(d["x0"]),
                                       torch.tensor(d["ts0"]) if with_ts else None, cfg, layers)
    assert (y0 - torch.tensor(d["y0"])).abs().max().item() <= 1e-5
    for l, st in enumerate(states):
        for nm, t in zip(("v", "q", "k", "out"), st):
            assert t.shape == d[f"s0:{l}:{nm}"].shape, (l, nm)
            assert (t - torch.tensor(d[f"s0:{l}:{nm}"])).abs().max().item() <= 1e-5, (l, nm)
    delta = (torch.tensor(d["delta0"]), torch.tensor(d["delta1"]))
    y1, states1 = O.hstu_forward_cached(lengths, torch.tensor(d["x1"]),
                                        torch.tensor(d["ts1"]) if with_ts else None, cfg,
                                        layers, delta=delta, cache=states)
    assert (y1 - torch.tensor(d["y1"])).abs().max().item() <= 1e-5
    for l, st in enumerate(states1):
        assert st[0] is states[l][0] and st[3] is states[l][3]  # updated in place
        for nm, t in zip(("v", "q", "k", "out"), st):
            assert (t - torch.tensor(d[f"s1:{l}:{nm}"])).abs().max().item() <= 1e-5, (l, nm)


@pytest.mark.parametrize("name", ["T1", "T2", "T3_small"])
def test_topk_oracle_vs_reference(name):
    d = np.load(os.path.join(GOLDEN, f"topk_{name}.npz"))
    s, ids, idx = topk_oracle.mips_topk(d["Q"], d["E"], d["ids"], d["invalid"], int(d["k"]))
    assert np.array_equal(ids, d["top_ids"])
    if int(d["integer"]):
        assert np.array_equal(s, d["top_scores"])
    else:
        np.testing.assert_allclose(s, d["top_scores"], rtol=1e-6, atol=1e-7)
    assert np.array_equal(d["ids"][idx], ids)


def test_topk_oracle_edge_cases():
    g = np.random.default_rng(1)
    Q = g.standard_normal((3, 8), dtype=np.float32)
    E = np.ones((20, 8), np.float32)  # all ties -> index order
    s, ids, idx = topk_oracle.mips_topk(Q, E, np.arange(20), None, 5)
    assert (idx == np.arange(5)[None, :]).all()
    # fewer valid than k: padded with -inf / -1
    inv = np.tile(np.arange(18, dtype=np.int64)[None, :], (3, 1))
    s, ids, idx = topk_oracle.mips_topk(Q, E, np.arange(20), inv, 5)
    assert (idx[:, :2] == [18, 19]).all() and (idx[:, 2:] == -1).all()
    assert np.isneginf(s[:, 2:]).all()


def test_jagged_ops_golden():
    """Reference tests/test_ops.py:7-53 known answers, restated in numpy."""
    d = np.load(os.path.join(GOLDEN, "jagged_ops.npz"))
    assert np.array_equal(np.concatenate([[0], np.cumsum(d["lengths"])]), d["offsets"])
    offs = d["offsets"]
    jag = np.concatenate([d["dense"][b, : offs[b + 1] - offs[b]] for b in range(len(offs) - 1)])
    assert np.array_equal(jag, d["jagged"])
    o2 = d["offsets2"]
    pad = np.zeros((len(o2) - 1, 3, 1), np.float32)
    for b in range(len(o2) - 1):
        pad[b, : o2[b + 1] - o2[b]] = d["values"][o2[b]:o2[b + 1]]
    assert np.array_equal(pad, d["padded"])


# ---------------------------------------------------------------- sampled-softmax loss (N1)

SSM_CASES = sorted(glob.glob(os.path.join(GOLDEN, "ssm_*.npz")))


@pytest.mark.parametrize("path", SSM_CASES, ids=lambda p: os.path.basename(p))
def test_loss_oracle_matches_reference_golden(path):
    from oracle import loss_oracle
    z = np.load(path)
    r = loss_oracle.from_golden(z)
    assert abs(float(r["loss"]) - float(z["loss"])) <= 1e-6 * max(1.0, abs(float(z["loss"])))
    for key in ("d_out", "d_sup_emb", "d_weight"):
        ref = z[key].astype(np.float64)
        err = np.abs(r[key] - ref).max() / max(np.abs(ref).max(), 1e-30)
        assert err < 1e-5, (key, err)


@pytest.mark.parametrize("path", SSM_CASES, ids=lambda p: os.path.basename(p))
def test_sampler_draw_matches_reference(path):
    """LocalNegativesSampler.sample_offsets consumes the generator exactly as the
    reference's forward (negative_sampler.py:110-118): same seed, same sampled ids."""
    from mygenerativerecommenders_amd.negatives_sampler import LocalNegativesSampler
    z = np.load(path)
    M, R = z["offsets"].shape
    if bool(z["use_all_ids"]):
        s = LocalNegativesSampler(True, 1e-6, all_item_ids=z["all_ids"].tolist())
    else:
        s = LocalNegativesSampler(True, 1e-6, num_items=len(z["all_ids"]))
    torch.manual_seed(int(z["rng_seed"]))
    offs = s.sample_offsets(torch.from_numpy(z["sup_ids"]), R)
    assert np.array_equal(offs.numpy(), z["offsets"])
    assert np.array_equal(s.all_item_ids[offs].numpy(), z["sampled_ids"].reshape(M, R))


def test_sampler_argument_validation():
    from mygenerativerecommenders_amd.negatives_sampler import LocalNegativesSampler
    with pytest.raises(ValueError):
        LocalNegativesSampler(True, 1e-6)
    with pytest.raises(ValueError):
        LocalNegativesSampler(True, 1e-6, num_items=3, all_item_ids=[1, 2])
    s = LocalNegativesSampler(False, 1e-6, num_items=5)
    assert s.all_item_ids.tolist() == [0, 1, 2, 3, 4]
    assert s.debug_str() == "local"
    with pytest.raises(RuntimeError):
        s.item_table()


# ---------------------------------------------------------------- input preprocessor (N2)

def test_preproc_oracle_matches_reference_golden():
    from oracle import preproc_oracle
    z = np.load(os.path.join(GOLDEN, "preproc.npz"))
    D = z["x"].shape[-1]
    y, valid = preproc_oracle.preprocess(z["x"], z["ids"], z["pos_w"], D ** 0.5)
    assert np.allclose(y, z["y"], rtol=1e-6, atol=1e-6)
    assert np.array_equal(valid, z["valid"])
    dx, dpos = preproc_oracle.preprocess_bwd(z["dy"], z["ids"], D ** 0.5, z["pos_w"].shape[0])
    assert np.allclose(dx, z["dx"], rtol=1e-6, atol=1e-6)
    assert np.allclose(dpos, z["dpos"], rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------- item embeddings (N2)

def test_embedding_oracle_matches_reference_golden():
    from oracle import embedding_oracle as EO
    z = np.load(os.path.join(GOLDEN, "embeddings.npz"))
    out = EO.get_item_embeddings(z["ids"], z["item_w"], z["year_w"], z["year_table"])
    assert np.array_equal(out, z["out"])  # a gather: bit-exact
    dw0, dw1 = EO.get_item_embeddings_bwd(z["ids"], z["dout"], z["item_w"].shape[0],
                                          z["year_w"].shape[0], z["year_table"])
    assert np.allclose(dw0, z["d_item_w"], rtol=1e-5, atol=1e-6)
    assert np.allclose(dw1, z["d_year_w"], rtol=1e-5, atol=1e-6)
