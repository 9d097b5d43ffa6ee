"""CPU: host-side logic of the drop-in modules (construction, parameter / state-dict
contract with the reference, error behaviour, no silent CPU path)."""
import os

import numpy as np
import pytest
import torch

from mygenerativerecommenders_amd import _lib

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _hstu(**kw):
    from mygenerativerecommenders_amd.hstu import HSTU
    args = dict(max_sequence_len=200, max_output_len=11, embedding_dim=50, item_embedding_dim=50,
                num_blocks=2, num_heads=1, linear_dim=50, attention_dim=50,
                normalization="rel_bias", linear_config="uvqk", linear_activation="silu",
                linear_dropout_rate=0.2, attn_dropout_rate=0.0)
    args.update(kw)
    return HSTU(**args)


def test_state_dict_keys_and_shapes_match_reference():
    d = np.load(os.path.join(GOLDEN, "hstu_b4_n32_d50_h1.npz"))
    ref = {k[6:]: d[k].shape for k in d.files if k.startswith("param:")}
    enc = _hstu(max_sequence_len=32, num_blocks=2)
    ours = {k: tuple(v.shape) for k, v in enc.state_dict().items() if k != "_attn_mask"}
    assert ours == {k: tuple(v) for k, v in ref.items()}
    mask = enc.state_dict()["_attn_mask"]
    assert mask.dtype == torch.bool and mask.shape == (43, 43)
    assert torch.equal(mask, torch.triu(torch.ones(43, 43, dtype=torch.bool), 1))


def test_parameter_init_statistics_match_reference():
    torch.manual_seed(0)
    enc = _hstu(num_blocks=1)
    layer = enc._hstu._attention_layers[0]
    assert abs(layer._uvqk.std().item() - 0.02) < 0.002
    assert abs(layer._rel_attn_bias._ts_w.std().item() - 0.02) < 0.01
    assert layer._o.weight.shape == (50, 50)
    # xavier_uniform bound sqrt(6/(50+50))
    assert layer._o.weight.abs().max().item() <= (6 / 100) ** 0.5 + 1e-6
    assert layer._rel_attn_bias._pos_w.numel() == 2 * 211 - 1


def test_unsupported_configurations_raise():
    with pytest.raises(ValueError):
        _hstu(linear_config="uv")
    enc = _hstu(concat_ua=True)  # supported: the geometry carries the flag
    assert enc._hstu._attention_layers[0]._geometry(211, 211).concat_ua
    enc = _hstu(concat_ua=True, linear_dim=96, attention_dim=96)  # o_in wider than 3 x 64
    from mygenerativerecommenders_amd import ops
    with pytest.raises(NotImplementedError):
        ops._pad_cat_weight(enc._hstu._attention_layers[0]._o.weight, 96)
    with pytest.raises(ValueError):
        _hstu(autocast_dtype=torch.float16)
    assert _hstu(autocast_dtype=torch.bfloat16)._hstu._attention_layers[0]._geometry(211, 211).bf16
    enc = _hstu(normalization="softmax_rel_bias")  # supported since round 6: fp32 layer
    geo = enc._hstu._attention_layers[0]._geometry(211, 211)
    assert geo.softmax and not geo.a16
    assert enc._hstu._stack_params(211, 211, None, False) is None  # per-layer nodes
    enc = _hstu(normalization="softmax_rel_bias", autocast_dtype=torch.bfloat16)
    assert not enc._hstu._attention_layers[0]._geometry(211, 211).bf16
    with pytest.raises(ValueError):
        _hstu(normalization="softmax")._hstu._attention_layers[0]._geometry(211, 211)


def test_cpu_tensors_are_rejected_no_silent_fallback():
    enc = _hstu(max_sequence_len=8, max_output_len=0, embedding_dim=8, item_embedding_dim=8,
                linear_dim=8, attention_dim=8)
    x = torch.randn(2, 8, 8)
    with pytest.raises((_lib.GrError, RuntimeError)):
        enc(torch.tensor([8, 3]), x, None, {})


def test_bias_module_materialises_on_gpu_only():
    from mygenerativerecommenders_amd._lib import GrError
    from mygenerativerecommenders_amd.hstu import RelativeBucketedTimeAndPositionBasedBias
    from mygenerativerecommenders_amd.hstu import _default_bucketization_fn
    m = RelativeBucketedTimeAndPositionBasedBias(10, 128, _default_bucketization_fn)
    assert m._ts_w.shape == (129,) and m._pos_w.shape == (19,)
    with pytest.raises(GrError):  # no CPU path: the GPU test checks the values
        m(torch.zeros(1, 10, dtype=torch.int64))
    with pytest.raises(ValueError):
        RelativeBucketedTimeAndPositionBasedBias(10, 64, _default_bucketization_fn)


def test_custom_bucketization_fn_checked_against_the_kernel_table():
    """hstu.py:71-95 honours any bucketization_fn; the kernels implement the default
    one only, so a different function must raise instead of being silently replaced."""
    from mygenerativerecommenders_amd.hstu import RelativeBucketedTimeAndPositionBasedBias
    # the reference builds its default as a lambda (hstu.py:579-581): accepted
    ref_fn = lambda x: (torch.log(torch.abs(x).clamp(min=1)) / 0.301).long()  # noqa: E731
    m = RelativeBucketedTimeAndPositionBasedBias(10, 128, ref_fn)
    assert m._bucketization_fn is ref_fn
    for bad in (lambda x: (torch.log(torch.abs(x).clamp(min=1)) / 0.302).long(),
                lambda x: torch.log2(torch.abs(x).clamp(min=1)).long(),
                lambda x: torch.zeros_like(x),
                lambda x: (torch.log(torch.abs(x).clamp(min=1)) / 0.301).long() + (x > 10**6)):
        with pytest.raises(ValueError, match="bucketization_fn"):
            RelativeBucketedTimeAndPositionBasedBias(10, 128, bad)
    with pytest.raises(ValueError, match="bucketization_fn"):
        RelativeBucketedTimeAndPositionBasedBias(10, 128, lambda x: x.nonexistent())


def test_cached_decoding_host_checks():
    """delta_x_offsets / cache (hstu.py:293-298, 151-177): the checks that run before any
    device work — a cache per layer, one delta entry per sequence, entries in range, and
    no autograd (the cached step has no backward) — then the product path refuses CPU
    tensors (no CPU fallback)."""
    from mygenerativerecommenders_amd._lib import GrError
    enc = _hstu(max_sequence_len=8, max_output_len=0, embedding_dim=8, item_embedding_dim=8,
                linear_dim=8, attention_dim=8)
    x = torch.randn(16, 8)
    off = torch.tensor([0, 8, 16])
    mask = enc._attn_mask
    delta = (torch.tensor([7, 15]), torch.tensor([7, 7]))
    n_layers = len(enc._hstu._attention_layers)
    with pytest.raises(ValueError, match="cache"):
        enc._hstu.jagged_forward(x, off, None, mask, delta_x_offsets=delta)
    with pytest.raises(ValueError, match="cache"):
        enc._hstu.jagged_forward(x, off, None, mask, delta_x_offsets=delta,
                                 cache=[None] * (n_layers + 1))
    states = (torch.zeros(16, 8), torch.zeros(2, 8, 8), torch.zeros(2, 8, 8), torch.zeros(16, 8))
    cache = [states] * n_layers
    with pytest.raises(ValueError, match="one per sequence"):
        enc._hstu.jagged_forward(x, off, None, mask, delta_x_offsets=(delta[0][:1], delta[1][:1]),
                                 cache=cache)
    with pytest.raises(IndexError):
        enc._hstu.jagged_forward(x, off, None, mask, delta_x_offsets=(delta[0] + 1, delta[1]),
                                 cache=cache)
    with pytest.raises(IndexError):
        enc._hstu.jagged_forward(x, off, None, mask, delta_x_offsets=(delta[0], delta[1] + 1),
                                 cache=cache)
    with pytest.raises(NotImplementedError, match="inference-only"):
        enc._hstu.jagged_forward(x, off, None, mask, delta_x_offsets=delta, cache=cache)
    layer = enc._hstu._attention_layers[0]
    with pytest.raises(ValueError, match="cache"):
        layer(x, off, None, mask, delta_x_offsets=delta, cache=None)
    with torch.no_grad(), pytest.raises(GrError, match="CPU"):
        layer(x, off, None, mask, delta_x_offsets=delta, cache=states)


def test_candidate_index_contract():
    from mygenerativerecommenders_amd.candidate_index import CandidateIndex
    from mygenerativerecommenders_amd.top_k import MIPSBruteForceTopK
    E = torch.randn(1, 30, 8)
    idx = CandidateIndex(k=500, ids=torch.arange(1, 31), top_k_module=MIPSBruteForceTopK(),
                         embeddings=E)
    assert idx._k == 30 and idx.num_objects == 30
    assert idx.ids.shape == (1, 30)
    assert torch.equal(idx.embeddings, E)
    assert idx._embeddings_t.shape == (8, 30)
    with pytest.raises(TypeError):
        CandidateIndex(k=5, ids=torch.arange(3), top_k_module=torch.nn.Identity())
    with pytest.raises(NotImplementedError):
        idx.filter_invalid_ids(torch.zeros(2, 3, dtype=torch.int64))
    with pytest.raises((_lib.GrError, RuntimeError)):
        idx.get_top_k_outputs(torch.randn(2, 8))  # CPU tensors: no CPU path


def test_bench_flop_accounting():
    import bench
    fwd, dkv, dq = bench.attn_flops(torch.tensor([200, 200]), 1, 50, 50, 4)
    T = 2 * 200 * 201 / 2
    assert fwd == 2 * T * 100 and dkv == 2 * T * 150 and dq == 2 * T * 50
    lengths, x, ts, past_ids, dy = bench.make_batch(4, 200, 11, 50, 0, "cpu")
    assert x.shape == (4, 211, 50) and ts.shape == (4, 211)
    # target timestamp sits at index L (features.py:53-57) and padding is 0
    assert (ts[:, 200] > 0).all() and (ts[:, 201:] == 0).all()
    assert (past_ids[:, 200:] == 0).all()


def test_local_embedding_module_layout_and_year_table(tmp_path):
    """embeddings.py:40-101 layout: half-width item and year tables, the item -> year
    lookup buffer (empty mapping -> zeros of num_items + 1), CSV loading, clamping."""
    import torch

    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    m = LocalEmbeddingModule(100, 50)
    assert m._item_emb.weight.shape == (101, 25) and m._year_emb.weight.shape == (101, 25)
    assert m.year_lookup_table.shape == (101,) and not m.year_lookup_table.any()
    assert m.item_embedding_dim == 50 and m.debug_str() == "local_emb_d50"
    assert m._item_emb.weight[0].abs().sum() > 0  # reset_params re-inits the padding row too
    csv_path = tmp_path / "movies.csv"
    csv_path.write_text("movie_id,title,year\n1,a,1995\n7,b,2000\n")
    m2 = LocalEmbeddingModule(100, 50, movies_csv=str(csv_path))
    assert m2.year_lookup_table.shape == (8,)
    assert m2.year_lookup_table[1] == 1995 and m2.year_lookup_table[7] == 2000
    ids = torch.tensor([0, 1, 7, 50, -3])
    assert m2.lookup_year_ids(ids).tolist() == [0, 1995, 2000, 2000, 0]
