"""GPU parity of the fused MIPS top-k (mips_topk / mips_merge_topk).

Bar: BIT-EXACT ids, catalog indices and scores against the C oracle
(oracle/topk_oracle.c: fp32 fmaf chain, canonical order score desc / index asc) on
every input, and exact ids against the reference's own outputs
(tests/golden/topk_*.npz, recorded from reference CandidateIndex + MIPSBruteForceTopK).
"""
import os

import numpy as np
import pytest
import torch

from oracle import topk_oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _gpu(Q, E, ids, invalid, k, index_base=0):
    from mygenerativerecommenders_amd.top_k import PackedItems, mips_topk
    dev = torch.device("cuda")
    packed = PackedItems(torch.as_tensor(E).to(dev))
    s, i, x = mips_topk(torch.as_tensor(Q).to(dev), packed, k,
                        item_ids=None if ids is None else torch.as_tensor(ids).to(dev),
                        invalid_ids=None if invalid is None else torch.as_tensor(invalid).to(dev),
                        index_base=index_base, return_index=True)
    torch.cuda.synchronize()
    return s.cpu().numpy(), i.cpu().numpy(), x.cpu().numpy()


def _check_exact(Q, E, ids, invalid, k):
    s, i, x = _gpu(Q, E, ids, invalid, k)
    rs, ri, rx = topk_oracle.mips_topk(Q, E, ids, invalid, k)
    assert np.array_equal(x, rx), f"index mismatch rows {np.where((x != rx).any(1))[0][:8]}"
    assert np.array_equal(i, ri)
    assert np.array_equal(s.view(np.uint32), rs.view(np.uint32)) or np.array_equal(s, rs)


@pytest.mark.parametrize("name", ["T1", "T2", "T3_small"])
def test_candidate_index_vs_reference_golden(name):
    from mygenerativerecommenders_amd.candidate_index import CandidateIndex
    from mygenerativerecommenders_amd.top_k import MIPSBruteForceTopK
    d = np.load(os.path.join(GOLDEN, f"topk_{name}.npz"))
    dev = torch.device("cuda")
    idx = CandidateIndex(k=int(d["k"]), ids=torch.tensor(d["ids"]),
                         top_k_module=MIPSBruteForceTopK(),
                         embeddings=torch.tensor(d["E"]).unsqueeze(0).to(dev)).to(dev)
    ids, scores = idx.get_top_k_outputs(torch.tensor(d["Q"]).to(dev),
                                        invalid_ids=torch.tensor(d["invalid"]).to(dev))
    ids, scores = ids.cpu().numpy(), scores.cpu().numpy()
    assert np.array_equal(ids, d["top_ids"])
    if int(d["integer"]):
        assert np.array_equal(scores, d["top_scores"])  # exact in any summation order
    else:
        np.testing.assert_allclose(scores, d["top_scores"], rtol=2e-6, atol=1e-6)
    # and bit-exact against the fmaf-chain oracle
    _check_exact(d["Q"], d["E"], d["ids"], d["invalid"], int(d["k"]))


@pytest.mark.parametrize("B,X,D,k,N0", [
    (128, 3953, 50, 200, 211),      # ml-1m retrieval shape
    (128, 200_000, 50, 200, 211),
    (37, 50_000, 16, 100, 0),
    (20, 30_000, 64, 256, 256),
    (5, 777, 8, 10, 3),
    (64, 100_000, 256, 200, 211),
])
def test_mips_topk_bitexact_vs_oracle(B, X, D, k, N0):
    g = np.random.default_rng(B * 1000 + D)
    E = g.standard_normal((X, D), dtype=np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    Q = g.standard_normal((B, D), dtype=np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    ids = np.arange(1, X + 1, dtype=np.int64)
    inv = None
    if N0:
        inv = np.zeros((B, N0), np.int64)
        for b in range(B):
            n = g.integers(N0 // 2, N0 + 1)
            inv[b, :n] = g.integers(1, X + 1, n)
    _check_exact(Q, E, ids, inv, k)


@pytest.mark.parametrize("X", [3953, 40_000])
def test_mips_topk_explicit_ids_bitexact(X):
    """Non-arange item ids (explicit id table): the small-catalog path searches each item
    in the sorted invalid list, the large path filters during compaction."""
    g = np.random.default_rng(X)
    B, D, k, N0 = 96, 50, 200, 211
    E = g.standard_normal((X, D), dtype=np.float32)
    Q = g.standard_normal((B, D), dtype=np.float32)
    ids = g.permutation(np.arange(10, 10 + 3 * X, 3, dtype=np.int64))
    inv = np.zeros((B, N0), np.int64)
    for b in range(B):
        inv[b] = g.choice(ids, N0)
    inv[:, -5:] = 0  # padding ids that match nothing
    _check_exact(Q, E, ids, inv, k)


def test_mips_topk_adversarial_orderings():
    """Sorted catalog (every item beats the running threshold: maximum compactions),
    all-equal scores (ties resolved by index), duplicated / zero invalid ids, and
    too few valid items (rows padded with -inf / -1)."""
    g = np.random.default_rng(7)
    B, X, D, k = 16, 20_000, 16, 200
    Q = np.abs(g.standard_normal((B, D), dtype=np.float32))
    base = np.linspace(0.0, 1.0, X, dtype=np.float32)[:, None]
    E = (base * np.ones((1, D), np.float32)).astype(np.float32)  # scores increase with index
    _check_exact(Q, E, np.arange(X, dtype=np.int64), None, k)
    E2 = np.ones((X, D), np.float32)  # all equal
    inv = np.zeros((B, 50), np.int64)
    inv[:, :10] = 5
    inv[:, 10:20] = np.arange(10)[None, :]
    _check_exact(Q, E2, np.arange(X, dtype=np.int64), inv, k)
    # fewer valid than k
    E3 = g.standard_normal((150, D), dtype=np.float32)
    inv3 = np.tile(np.arange(0, 40, dtype=np.int64)[None, :], (B, 1))
    _check_exact(Q, E3, np.arange(150, dtype=np.int64), inv3, k)


def test_sharded_merge_equals_full():
    from mygenerativerecommenders_amd.top_k import PackedItems, merge_topk, mips_topk
    g = np.random.default_rng(11)
    B, X, D, k, N0, P = 64, 90_001, 50, 200, 211, 4
    E = g.standard_normal((X, D), dtype=np.float32)
    Q = g.standard_normal((B, D), dtype=np.float32)
    ids = np.arange(1, X + 1, dtype=np.int64)
    inv = g.integers(1, X + 1, (B, N0)).astype(np.int64)
    dev = torch.device("cuda")
    bounds = np.linspace(0, X, P + 1).astype(int)
    parts = []
    for r in range(P):
        a, b = bounds[r], bounds[r + 1]
        pk = PackedItems(torch.tensor(E[a:b]).to(dev))
        parts.append(mips_topk(torch.tensor(Q).to(dev), pk, k, item_ids=torch.tensor(ids[a:b]).to(dev),
                               invalid_ids=torch.tensor(inv).to(dev), index_base=int(a),
                               return_index=True))
    cs = torch.stack([p[0] for p in parts])
    ci = torch.stack([p[2] for p in parts])
    cd = torch.stack([p[1] for p in parts])
    s, i, x = merge_topk(cs, ci, cd, k, return_index=True)
    rs, ri, rx = topk_oracle.mips_topk(Q, E, ids, inv, k)
    assert np.array_equal(x.cpu().numpy(), rx)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)
