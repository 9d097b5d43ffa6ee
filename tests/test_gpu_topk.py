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


def test_mips_topk_small_path_edges():
    """The one-kernel small-catalog path (X <= 8192, D <= 64, k <= 256) at its edges:
    X = 8192 exactly, k = 256, all-equal scores (ties by index), sorted scores, -0.0 vs
    +0.0 ties, explicit ids with a long sorted invalid list (N0 = 2059), every item
    invalid, and X < k."""
    g = np.random.default_rng(17)
    B, D = 9, 64
    X = 8192
    Q = g.standard_normal((B, D), dtype=np.float32)
    E = g.standard_normal((X, D), dtype=np.float32)
    _check_exact(Q, E, np.arange(1, X + 1, dtype=np.int64), None, 256)
    E2 = np.ones((X, D), np.float32)
    inv = np.zeros((B, 40), np.int64)
    inv[:, :20] = np.arange(1, 21)[None, :]
    _check_exact(np.abs(Q), E2, np.arange(1, X + 1, dtype=np.int64), inv, 200)
    base = np.linspace(-1.0, 1.0, X, dtype=np.float32)[:, None]
    _check_exact(np.abs(Q), (base * np.ones((1, D), np.float32)).astype(np.float32),
                 np.arange(X, dtype=np.int64), None, 256)
    E0 = np.zeros((777, D), np.float32)  # every score +-0: ties resolved by index
    E0[::3, 0] = -0.0
    _check_exact(Q, E0, np.arange(777, dtype=np.int64), None, 100)
    ids = g.permutation(np.arange(7, 7 + 2 * 3953, 2, dtype=np.int64))
    inv2 = np.stack([g.choice(ids, 2059) for _ in range(B)])
    _check_exact(Q[:, :50].copy(), E[:3953, :50].copy(), ids, inv2, 200)
    inv3 = np.tile(np.arange(300, dtype=np.int64)[None, :], (B, 1))  # all invalid
    _check_exact(Q[:, :16].copy(), E[:300, :16].copy(), np.arange(300, dtype=np.int64), inv3, 50)
    _check_exact(Q[:, :8].copy(), E[:37, :8].copy(), np.arange(37, dtype=np.int64), None, 200)


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


# ---------------------------------------------------------------- large-catalog filter path
# X >= 262,144 and D <= 64 take the sample -> tau -> filter -> merge path; its result must
# be bit-identical to the oracle whether the fast path held (flag 0) or the exact
# fallback ran (flag 1).  The flag is the first int32 of the workspace.

def _gpu_flag(Q, E, ids, invalid, k, index_base=0):
    from mygenerativerecommenders_amd.top_k import PackedItems, mips_topk, topk_workspace_bytes
    dev = torch.device("cuda")
    packed = PackedItems(torch.as_tensor(E).to(dev))
    N0 = 0 if invalid is None else invalid.shape[1]
    ws = torch.full((topk_workspace_bytes(Q.shape[0], E.shape[0], E.shape[1], k, N0),), 7,
                    dtype=torch.uint8, device=dev)
    s, i, x = mips_topk(torch.as_tensor(Q).to(dev), packed, k,
                        item_ids=None if ids is None else torch.as_tensor(ids).to(dev),
                        invalid_ids=None if invalid is None else torch.as_tensor(invalid).to(dev),
                        index_base=index_base, return_index=True, workspace=ws)
    torch.cuda.synchronize()
    flag = int(ws[:4].view(torch.int32).item())
    return s.cpu().numpy(), i.cpu().numpy(), x.cpu().numpy(), flag


def _check_filter(Q, E, ids, invalid, k, expect_flag):
    s, i, x, flag = _gpu_flag(Q, E, ids, invalid, k)
    rs, ri, rx = topk_oracle.mips_topk(Q, E, ids, invalid, k)
    if expect_flag is not None:
        assert flag == expect_flag, f"fallback flag {flag}, expected {expect_flag}"
    assert np.array_equal(x, rx), f"index mismatch rows {np.where((x != rx).any(1))[0][:8]}"
    assert np.array_equal(i, ri)
    assert np.array_equal(s.view(np.uint32), rs.view(np.uint32))


def _normal_catalog(g, B, X, D, N0):
    E = g.standard_normal((X, D), dtype=np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    Q = g.standard_normal((B, D), dtype=np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    inv = None
    if N0:
        inv = np.zeros((B, N0), np.int64)
        for b in range(B):
            n = g.integers(N0 // 2, N0 + 1)
            inv[b, :n] = g.integers(1, X + 1, n)
    return Q, E, inv


@pytest.mark.parametrize("B,X,D,k,N0", [
    (128, 600_001, 50, 200, 211),   # C4 shape per 16 shards-ish, ragged last block
    (200, 300_000, 50, 200, 211),   # two query chunks (128 + 72)
    (8, 262_144, 16, 100, 0),       # narrow chunk (NQG 2), no invalid ids
    (64, 400_000, 64, 256, 256),    # D = 64, k = N0 = 256
])
def test_mips_filter_path_bitexact(B, X, D, k, N0):
    g = np.random.default_rng(B + X + D)
    Q, E, inv = _normal_catalog(g, B, X, D, N0)
    _check_filter(Q, E, np.arange(1, X + 1, dtype=np.int64), inv, k, expect_flag=0)


@pytest.mark.parametrize("D", [5, 8, 17, 20, 40, 47, 49, 58])
def test_mips_filter_bf16_layouts_bitexact(D):
    """Every bf16 block layout of the filter copy (16x16x32 chunks, a 16x16x16 chunk and a
    tail of 1-3 stored k-groups; dims padded to 4, not 32) is bit-exact end to end."""
    g = np.random.default_rng(D)
    B, X, k, N0 = 40, 262_144 + 77, 64, 33
    Q, E, inv = _normal_catalog(g, B, X, D, N0)
    _check_filter(Q, E, np.arange(1, X + 1, dtype=np.int64), inv, k, expect_flag=0)


@pytest.mark.parametrize("D,B,X", [(256, 32, 1_000_000), (256, 128, 1_000_000), (256, 64, 300_001),
                                   (96, 40, 262_144 + 77), (130, 24, 300_001)])
def test_mips_filter_wide_d_bitexact(D, B, X):
    """The bf16 filter beyond D = 64 (k-chunks of 32 dims, 4 or 2 query tiles per
    workgroup, exact f32 rescoring in 64-dim rounds): bit-exact against the oracle,
    including the SURVEY C4 variant D = 256 at X = 1 M with its B = 128 (no fallback:
    the measured-norm error bound keeps the candidate sub-lists from overflowing)."""
    g = np.random.default_rng(D + B)
    k, N0 = (200, 211) if D == 256 else (64, 33)
    Q, E, inv = _normal_catalog(g, B, X, D, N0)
    _check_filter(Q, E, np.arange(1, X + 1, dtype=np.int64), inv, k, expect_flag=0)


def test_mips_filter_path_explicit_ids():
    g = np.random.default_rng(5)
    B, X, D, k, N0 = 96, 300_000, 50, 200, 211
    Q, E, _ = _normal_catalog(g, B, X, D, 0)
    ids = g.permutation(np.arange(10, 10 + 3 * X, 3, dtype=np.int64))
    # invalid ids drawn from each query's own top-500, so the exclusion really bites
    sc = Q @ E.T
    inv = np.zeros((B, N0), np.int64)
    for b in range(B):
        top = np.argpartition(-sc[b], 500)[:500]
        inv[b, :200] = ids[g.choice(top, 200, replace=False)]
    _check_filter(Q, E, ids, inv, k, expect_flag=0)


def test_mips_filter_path_fallbacks():
    """Inputs that defeat the sampled threshold must still give the exact answer through
    the gated fallback: the best items all inside sampled blocks (too few candidates),
    scores increasing with the index (list overflow), all-equal scores (overflow, ties
    by index)."""
    g = np.random.default_rng(3)
    B, X, D, k = 32, 300_000, 16, 200
    Q = np.abs(g.standard_normal((B, D), dtype=np.float32)) + 0.1
    ids = np.arange(X, dtype=np.int64)
    E = (0.01 * g.standard_normal((X, D))).astype(np.float32)
    blk = np.arange(X) // 16
    E[blk % 16 == 0] += 1.0  # every sampled block beats every other item
    _check_filter(Q, E, ids, None, k, expect_flag=1)
    base = np.linspace(0.0, 1.0, X, dtype=np.float32)[:, None]
    _check_filter(Q, (base * np.ones((1, D), np.float32)).astype(np.float32), ids, None, k,
                  expect_flag=1)
    inv = np.tile(np.arange(0, 40, dtype=np.int64)[None, :], (B, 1))
    _check_filter(Q, np.ones((X, D), np.float32), ids, inv, k, expect_flag=1)


def test_sharded_merge_equals_full_filter_path():
    """Two 300K-row shards through the filter path, then the cross-shard merge."""
    from mygenerativerecommenders_amd.top_k import PackedItems, merge_topk, mips_topk
    g = np.random.default_rng(12)
    B, X, D, k, N0 = 128, 600_000, 50, 200, 211
    Q, E, inv = _normal_catalog(g, B, X, D, N0)
    ids = np.arange(1, X + 1, dtype=np.int64)
    dev = torch.device("cuda")
    parts = []
    for a, b in ((0, 300_000), (300_000, X)):
        pk = PackedItems(torch.tensor(E[a:b]).to(dev))
        parts.append(mips_topk(torch.tensor(Q).to(dev), pk, k, item_ids=None,
                               invalid_ids=torch.tensor(inv).to(dev), index_base=int(a) + 1,
                               return_index=True))
    s, i, x = merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[2] for p in parts]),
                         torch.stack([p[1] for p in parts]), k, return_index=True)
    rs, ri, rx = topk_oracle.mips_topk(Q, E, ids, inv, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(x.cpu().numpy() - 1, rx)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), rs.view(np.uint32))


# ---------------------------------------------------------------- bf16 filter scores
# The filter pass scores a bf16 copy of the table; the merge rescores every candidate
# with the exact f32 chain and only trusts those >= tau_e (mips_tau_kernel's bound), so
# the result stays bit-identical to the oracle.  The launch option GR_OPT_MIPS_FILTER_FP32
# keeps the f32 filter (exact filter scores) reachable.

@pytest.mark.parametrize("fp32", [False, True], ids=["bf16-filter", "f32-filter"])
def test_mips_filter_score_type_bitexact(fp32):
    from mygenerativerecommenders_amd import _lib
    g = np.random.default_rng(31)
    B, X, D, k, N0 = 128, 400_000, 50, 200, 211
    Q, E, inv = _normal_catalog(g, B, X, D, N0)
    with _lib.option("MIPS_FILTER_FP32", int(fp32)):
        _check_filter(Q, E, np.arange(1, X + 1, dtype=np.int64), inv, k, expect_flag=0)


def test_mips_filter_bf16_rescoring_orders_near_ties():
    """400 items every query scores within ~1e-5 of each other (far below bf16
    resolution) and well above the rest: only the exact rescoring can order them."""
    g = np.random.default_rng(21)
    B, X, D, k = 64, 300_000, 50, 200
    _, E, _ = _normal_catalog(g, B, X, D, 0)
    u = g.standard_normal(D).astype(np.float32)
    u /= np.linalg.norm(u)
    Q = (u[None, :] + 0.3 * g.standard_normal((B, D)) / np.sqrt(D)).astype(np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    idx = g.choice(X, 400, replace=False)
    E[idx] = (u[None, :] + 1e-5 * g.standard_normal((400, D))).astype(np.float32)
    _check_filter(Q, E, np.arange(X, dtype=np.int64), None, k, expect_flag=0)


def test_mips_filter_bf16_unnormalised_norms():
    """Item norms spread over 0.5 .. 20 and large queries: the error bound scales with
    ||q|| max||x||; whichever path runs, the answer is exact."""
    g = np.random.default_rng(41)
    B, X, D, k, N0 = 48, 300_000, 32, 150, 64
    Q, E, inv = _normal_catalog(g, B, X, D, N0)
    E *= g.uniform(0.5, 20.0, (X, 1)).astype(np.float32)
    Q *= np.float32(100.0)
    _check_filter(Q, E, np.arange(1, X + 1, dtype=np.int64), inv, k, expect_flag=None)


def test_mips_filter_bf16_nan_row_takes_exact_path():
    """A NaN item makes the bf16 bound NaN: no candidate is trusted and the exact path
    runs; every finite item keeps its exact rank (the NaN item itself is outside the
    reference's contract: torch.topk would rank it first)."""
    g = np.random.default_rng(43)
    B, X, D, k = 16, 262_144, 16, 50
    Q, E, _ = _normal_catalog(g, B, X, D, 0)
    E[12345, 3] = np.nan
    s, i, x, flag = _gpu_flag(Q, E, np.arange(X, dtype=np.int64), None, k)
    assert flag == 1
    E0 = E.copy()
    E0[12345] = 0.0  # score 0: far below every query's top-50
    rs, ri, rx = topk_oracle.mips_topk(Q, E0, np.arange(X, dtype=np.int64), None, k)
    for b in range(B):
        keep = i[b] != 12345
        n = int(keep.sum())
        assert np.array_equal(i[b][keep], ri[b][:n])
        assert np.array_equal(s[b][keep].view(np.uint32), rs[b][:n].view(np.uint32))


# ---------------------------------------------------------------- reference caller sequence
# Retrieval.retrieve (retrieval.py:19-47) runs under @torch.inference_mode: the candidate
# table is an inference tensor (no version counter), update_embeddings() is called on
# first use with the L2-normalised item embeddings, and invalid_ids = past_ids (B, N)
# with zero padding -- N0 = 211 at ml-1m and 2059 at ml-20m.

def _past_ids(g, B, N0, ids):
    inv = np.zeros((B, N0), np.int64)
    for b in range(B):
        L = int(g.integers(N0 // 4, N0 + 1))
        inv[b, :L] = g.choice(ids, L)
    return inv


def _retrieve_like_reference(E, Q, ids, inv, k, second_epoch=True):
    from mygenerativerecommenders_amd.candidate_index import CandidateIndex
    from mygenerativerecommenders_amd.top_k import MIPSBruteForceTopK
    dev = torch.device("cuda")
    out = []
    with torch.inference_mode():
        table = torch.tensor(E, device=dev)
        index = CandidateIndex(k=k, ids=torch.tensor(ids), top_k_module=MIPSBruteForceTopK()).to(dev)
        assert index.embeddings is None
        index.update_embeddings(table.unsqueeze(0))
        q = torch.tensor(Q, device=dev)
        past = torch.tensor(inv, device=dev)
        out.append([t.cpu().numpy() for t in index.get_top_k_outputs(q, invalid_ids=past)])
        if second_epoch:
            # next validation epoch: the same storage rewritten in place (inference tensors
            # carry no version counter), then update_embeddings() as on_validation_epoch_start
            table.mul_(-1.0)
            index.update_embeddings(table.unsqueeze(0))
            out.append([t.cpu().numpy() for t in index.get_top_k_outputs(q, invalid_ids=past)])
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("X,N0,explicit", [
    (3953, 211, False),      # ml-1m: small-catalog path
    (3953, 2059, True),      # small-catalog path, explicit ids, list in dynamic LDS
    (27_278, 211, False),    # ml-20m catalog: range-select path, LDS lists
    (27_278, 2059, False),   # ml-20m validation: N0 = 2059, pre-sorted workspace lists
    (27_278, 2059, True),
    (300_000, 2059, False),  # filter path, N0 = 2059 (list in dynamic LDS of the merge)
])
def test_retrieve_inference_mode_bitexact(X, N0, explicit):
    g = np.random.default_rng(X + N0)
    B, D, k = 128, 50, 200
    Q, E, _ = _normal_catalog(g, B, X, D, 0)
    ids = (g.permutation(np.arange(7, 7 + 2 * X, 2, dtype=np.int64)) if explicit
           else np.arange(1, X + 1, dtype=np.int64))
    inv = _past_ids(g, B, N0, ids)
    got = _retrieve_like_reference(E, Q, ids, inv, k)
    for (top_ids, top_scores), sign in zip(got, (1.0, -1.0)):
        rs, ri, _ = topk_oracle.mips_topk(Q, (sign * E).astype(np.float32), ids, inv, k)
        assert np.array_equal(top_ids, ri), f"ids differ in rows {np.where((top_ids != ri).any(1))[0][:8]}"
        assert np.array_equal(top_scores.view(np.uint32), rs.view(np.uint32))


def _reference_filter(scores, ids, invalid, k):
    """candidate_index.py:141-158 restated in torch: drop the row's invalid ids from the
    top-k' list, keep the first k (nonzero + view(-1, k): needs >= k valid per row)."""
    valid = ~(ids.unsqueeze(2) == invalid.unsqueeze(1)).max(2)[0]
    valid = torch.logical_and(valid, torch.cumsum(valid.int(), dim=1) <= k)
    off = torch.nonzero(valid, as_tuple=True)[1].view(-1, k)
    return torch.gather(ids, 1, off), torch.gather(scores, 1, off)


@pytest.mark.parametrize("X,N0,explicit", [(3953, 211, False), (27_278, 2059, False),
                                           (27_278, 2059, True), (1000, 600, False)])
def test_reference_k_prime_sequence_equals_fused(X, N0, explicit):
    """The reference's CandidateIndex asks its top-k module for k' = min(k + N0, X) and
    filters (candidate_index.py:125-158); with our MIPSBruteForceTopK that takes the
    wide-k path (k' = 411 / 2259).  Same ids and scores as the fused exclusion."""
    from mygenerativerecommenders_amd.candidate_index import CandidateIndex
    from mygenerativerecommenders_amd.top_k import MIPSBruteForceTopK
    g = np.random.default_rng(X + 3 * N0)
    B, D, k = 64, 50, 200
    Q, E, _ = _normal_catalog(g, B, X, D, 0)
    ids = (g.permutation(np.arange(7, 7 + 2 * X, 2, dtype=np.int64)) if explicit
           else np.arange(1, X + 1, dtype=np.int64))
    inv = _past_ids(g, B, N0, ids)
    inv[:, -1] = 0
    dev = torch.device("cuda")
    with torch.inference_mode():
        table = torch.tensor(E, device=dev).unsqueeze(0)
        mod = MIPSBruteForceTopK()
        index = CandidateIndex(k=k, ids=torch.tensor(ids), top_k_module=mod, embeddings=table).to(dev)
        q, past = torch.tensor(Q, device=dev), torch.tensor(inv, device=dev)
        k_prime = min(k + N0, X)
        s_p, i_p = mod(query_embeddings=q, item_embeddings_t=index._embeddings_t,
                       item_ids=index.ids, k=k_prime, sorted=True)
        ref_ids, ref_scores = _reference_filter(s_p, i_p, past, k)
        fused_ids, fused_scores = index.get_top_k_outputs(q, invalid_ids=past)
    assert torch.equal(ref_ids, fused_ids)
    assert torch.equal(ref_scores, fused_scores)
    rs, ri, _ = topk_oracle.mips_topk(Q, E, ids, None, k_prime)
    assert np.array_equal(i_p.cpu().numpy(), ri)
    assert np.array_equal(s_p.cpu().numpy().view(np.uint32), rs.view(np.uint32))


@pytest.mark.parametrize("B,X,D,k,N0,explicit", [
    (128, 3953, 50, 411, 0, False),
    (32, 27_278, 256, 2259, 0, False),      # D = 256
    (1024, 150_001, 16, 300, 40, False),    # 3 chunks of 65,536 (ragged last), exclusion
    (1024, 150_001, 16, 300, 40, True),
    (16, 500, 8, 700, 20, False),           # k > X: rows padded with -inf / -1
])
def test_mips_topk_wide_k_bitexact(B, X, D, k, N0, explicit):
    g = np.random.default_rng(B + X + k)
    Q, E, _ = _normal_catalog(g, B, X, D, 0)
    ids = (g.permutation(np.arange(7, 7 + 2 * X, 2, dtype=np.int64)) if explicit
           else np.arange(1, X + 1, dtype=np.int64))
    inv = _past_ids(g, B, N0, ids) if N0 else None
    _check_exact(Q, E, ids, inv, k)


def test_mips_topk_wide_k_ties_across_chunks():
    """All-equal scores over 3 chunks: the k smallest catalog indices, in index order."""
    B, X, D, k = 1024, 140_000, 8, 333
    Q = np.ones((B, D), np.float32)
    E = np.full((X, D), 0.5, np.float32)
    inv = np.tile(np.array([1, 5, 65_540, 0], np.int64)[None, :], (B, 1))
    _check_exact(Q, E, np.arange(X, dtype=np.int64), inv, k)


# ---------------------------------------------------------------- C4 at full size
def test_c4_10m_single_and_8_shards_bitexact():
    """10M items, B = 128, k = 200, 211 invalid ids; one shard, and 8 row
    shards of 1.25M merged by mips_merge_topk (the all-gather's device merge)."""
    from mygenerativerecommenders_amd.top_k import PackedItems, merge_topk, mips_topk
    g = np.random.default_rng(2024)
    B, X, D, k, N0, P = 128, 10_000_000, 50, 200, 211, 8
    E = g.standard_normal((X, D), dtype=np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    Q = g.standard_normal((B, D), dtype=np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    inv = _past_ids(g, B, N0, np.arange(1, X + 1, dtype=np.int64))
    rs, ri, rx = topk_oracle.mips_topk(Q, E, np.arange(1, X + 1, dtype=np.int64), inv, k)
    dev = torch.device("cuda")
    q, past = torch.tensor(Q, device=dev), torch.tensor(inv, device=dev)
    Et = torch.tensor(E, device=dev)
    pk = PackedItems(Et)
    s, i, x = mips_topk(q, pk, k, invalid_ids=past, index_base=1, return_index=True)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), rs.view(np.uint32))
    del pk
    parts = []
    for r in range(P):
        a, b = r * X // P, (r + 1) * X // P
        pk = PackedItems(Et[a:b])
        parts.append(mips_topk(q, pk, k, invalid_ids=past, index_base=a + 1, return_index=True))
        del pk
    s, i, x = merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[2] for p in parts]),
                         torch.stack([p[1] for p in parts]), k, return_index=True)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), rs.view(np.uint32))
