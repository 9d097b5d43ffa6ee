"""GPU: item-embedding gather through the C-ABI (gr_item_embedding_fwd/bwd)
against the reference golden (tests/golden/embeddings.npz, LocalEmbeddingModule with an
item -> year mapping), a torch fp32 reference at ml-1m size, the padding-row rule, the
categorical module, and HIP-graph replays."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _module_from_golden(z):
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    num_items = z["item_w"].shape[0] - 1
    m = LocalEmbeddingModule(num_items, 2 * z["item_w"].shape[1])
    with torch.no_grad():
        m._item_emb.weight.copy_(torch.from_numpy(z["item_w"]))
        m._year_emb.weight.copy_(torch.from_numpy(z["year_w"]))
    m.year_lookup_table = torch.from_numpy(z["year_table"]).clone()
    return m.cuda()


def test_local_embedding_matches_reference_golden():
    z = np.load(os.path.join(GOLDEN, "embeddings.npz"))
    m = _module_from_golden(z)
    ids = torch.from_numpy(z["ids"]).cuda()
    out = m.get_item_embeddings(ids)
    assert np.array_equal(out.detach().cpu().numpy(), z["out"])
    (out * torch.from_numpy(z["dout"]).cuda()).sum().backward()
    np.testing.assert_allclose(m._item_emb.weight.grad.cpu().numpy(), z["d_item_w"],
                               rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(m._year_emb.weight.grad.cpu().numpy(), z["d_year_w"],
                               rtol=1e-5, atol=1e-6)


def test_local_embedding_ml1m_vs_torch_fp32():
    """ml-1m shape: 128 x 211 ids over 3,952 items, a real-looking year map."""
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    g = torch.Generator().manual_seed(3)
    years = torch.randint(1919, 2001, (3952,), generator=g)
    m = LocalEmbeddingModule(3952, 50, item2year={i + 1: int(years[i]) for i in range(3952)}).cuda()
    ids = torch.randint(0, 3953, (128, 211), generator=g)
    ids[:, 200:] = 0
    ids = ids.cuda()
    out = m.get_item_embeddings(ids)
    w0 = m._item_emb.weight.detach().clone().requires_grad_(True)
    w1 = m._year_emb.weight.detach().clone().requires_grad_(True)
    ref = torch.cat([torch.nn.functional.embedding(ids, w0, padding_idx=0),
                     torch.nn.functional.embedding(m.lookup_year_ids(ids), w1, padding_idx=0)],
                    -1)
    assert torch.equal(out, ref)
    dy = torch.randn(out.shape, generator=g).cuda()
    (out * dy).sum().backward()
    (ref * dy).sum().backward()
    torch.testing.assert_close(m._item_emb.weight.grad, w0.grad, rtol=1e-5, atol=1e-6)
    # ~330 rows share each year: fp32 sums in another order (atomics vs sorted segments)
    torch.testing.assert_close(m._year_emb.weight.grad, w1.grad, rtol=1e-4, atol=1e-4)
    assert not m._item_emb.weight.grad[0].any() and not m._year_emb.weight.grad[0].any()


def test_categorical_embedding_vs_torch():
    from mygenerativerecommenders_amd.embeddings import CategoricalEmbeddingModule
    g = torch.Generator().manual_seed(4)
    cat = torch.randint(0, 30, (500,), generator=g)
    m = CategoricalEmbeddingModule(500, 24, cat).cuda()
    ids = torch.randint(0, 501, (7, 33), generator=g).cuda()
    out = m.get_item_embeddings(ids)
    w = m._item_emb.weight.detach().clone().requires_grad_(True)
    cid = m._item_id_to_category_id[(ids - 1).clamp(min=0)] + 1
    ref = torch.nn.functional.embedding(cid, w, padding_idx=0)
    assert torch.equal(out, ref)
    dy = torch.randn(out.shape, generator=g).cuda()
    (out * dy).sum().backward()
    (ref * dy).sum().backward()
    torch.testing.assert_close(m._item_emb.weight.grad, w.grad, rtol=1e-5, atol=1e-6)


def test_embedding_backward_deterministic_mode():
    """GR_OPT_DETERMINISTIC: the owner-computes backward sums every table row's
    contributions in id order -- equal to the reference golden, to the atomic backward
    within fp32 rounding, and bit-identical from run to run (ml-1m-sized batch with a
    year mapping, so both tables have heavily shared rows)."""
    from mygenerativerecommenders_amd import _lib
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    z = np.load(os.path.join(GOLDEN, "embeddings.npz"))

    def grads(m, ids, dout):
        m.zero_grad(set_to_none=True)
        (m.get_item_embeddings(ids) * dout).sum().backward()
        return m._item_emb.weight.grad.clone(), m._year_emb.weight.grad.clone()
    m = _module_from_golden(z)
    ids = torch.from_numpy(z["ids"]).cuda()
    dout = torch.from_numpy(z["dout"]).cuda()
    with _lib.option("DETERMINISTIC", 1):
        gi, gy = grads(m, ids, dout)
    np.testing.assert_allclose(gi.cpu().numpy(), z["d_item_w"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(gy.cpu().numpy(), z["d_year_w"], rtol=1e-5, atol=1e-6)
    g = torch.Generator().manual_seed(4)
    V, D, B, N = 3953, 50, 128, 211
    m2 = LocalEmbeddingModule(V, D, item2year={i: 1919 + i % 81 for i in range(1, V + 1)}).cuda()
    ids2 = torch.randint(0, V + 1, (B, N), generator=g).cuda()
    dout2 = torch.randn(B, N, D, generator=g).cuda()
    ref = grads(m2, ids2, dout2)
    with _lib.option("DETERMINISTIC", 1):
        a = grads(m2, ids2, dout2)
        b = grads(m2, ids2, dout2)
    for x, y, r in zip(a, b, ref):
        assert torch.equal(x, y)
        assert (x - r).abs().max().item() <= 1e-5 * (1 + r.abs().max().item())
        assert not x[0].any()  # padding row


def test_embedding_graph_replay():
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    m = LocalEmbeddingModule(3952, 50).cuda()
    ids = torch.randint(0, 3953, (64, 50), device="cuda")
    dy = torch.randn(64, 50, 50, device="cuda")

    def step():
        (m.get_item_embeddings(ids) * dy).sum().backward()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    ref = m._item_emb.weight.grad.clone()
    m._item_emb.weight.grad = None
    m._year_emb.weight.grad = None
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        step()
    for _ in range(3):
        gr.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(m._item_emb.weight.grad, ref, rtol=1e-5, atol=1e-6)


def test_embedding_rejects_cpu_tensors():
    from mygenerativerecommenders_amd import _lib
    from mygenerativerecommenders_amd.embeddings import item_embedding
    with pytest.raises(_lib.GrError):
        item_embedding(torch.zeros(3, dtype=torch.int64), torch.zeros(4, 2))
