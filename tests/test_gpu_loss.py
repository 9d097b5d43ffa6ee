"""GPU parity of the fused sampled-softmax loss:
``SampledSoftmaxLoss.jagged_forward`` (autoregressive_losses.py:259-306) with
``LocalNegativesSampler`` (negative_sampler.py:66-131) and ``DotProductSimilarity``
(dot_product.py:31-64), forward and backward, against

  * the reference's own recorded outputs (tests/golden/ssm_*.npz), given the sampled
    offsets the reference drew (the device RNG differs from the CPU one; the draw itself
    is pinned on CPU by tests/test_oracle_golden.py::test_sampler_draw_matches_reference);
  * the float64 oracle (oracle/loss_oracle.py) on random cases with edge shapes;
  * a plain PyTorch fp32 restatement at the ml-1m C2 size.

Tolerances (fp32 kernel, fp64 / fp32 checkers): loss and per-token loss 1e-5 relative
(+1e-4 absolute per token); gradients 2e-4 of the largest gradient entry.  The table
gradient is accumulated with fp32 atomics, so only its summation order differs.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import loss_oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SSM_CASES = sorted(glob.glob(os.path.join(GOLDEN, "ssm_*.npz")))


class _Emb(torch.nn.Module):
    def __init__(self, weight):
        super().__init__()
        self.weight = torch.nn.Parameter(weight)

    def get_item_embeddings(self, ids):
        return torch.nn.functional.embedding(ids, self.weight)


class _IselEmb(_Emb):
    """Row gather by index_select (backward: index_add_)."""

    def get_item_embeddings(self, ids):
        return self.weight.index_select(0, ids.reshape(-1)).view(*ids.shape, self.weight.shape[1])


def _sampler(l2_norm, all_ids, offsets, emb):
    from mygenerativerecommenders_amd.negatives_sampler import LocalNegativesSampler

    class _Fixed(LocalNegativesSampler):
        def sample_offsets(self, positive_ids, num_to_sample):
            assert offsets.shape == positive_ids.shape + (num_to_sample,)
            return offsets

    s = _Fixed(l2_norm, 1e-6, all_item_ids=all_ids.tolist()).cuda()
    s._embeddings_module = emb
    return s


def _run(out, sup_ids, sup_emb, weights, weight, all_ids, offsets, T, l2_norm):
    from mygenerativerecommenders_amd.losses import SampledSoftmaxLoss
    from mygenerativerecommenders_amd.similarity import DotProductSimilarity
    dev = torch.device("cuda")
    emb = _Emb(torch.as_tensor(weight, dtype=torch.float32).to(dev))
    offs = torch.as_tensor(offsets, dtype=torch.int64).to(dev)
    s = _sampler(l2_norm, torch.as_tensor(all_ids), offs, emb)
    o = torch.as_tensor(out, dtype=torch.float32).to(dev).requires_grad_(True)
    p = torch.as_tensor(sup_emb, dtype=torch.float32).to(dev).requires_grad_(True)
    loss = SampledSoftmaxLoss(offs.shape[1], T).jagged_forward(
        output_embeddings=o, supervision_ids=torch.as_tensor(sup_ids).to(dev),
        supervision_embeddings=p, supervision_weights=torch.as_tensor(weights).to(dev),
        negatives_sampler=s, similarity=DotProductSimilarity())
    loss.backward()
    return (loss.item(), o.grad.cpu().double().numpy(), p.grad.cpu().double().numpy(),
            emb.weight.grad.cpu().double().numpy())


def _close(got, ref, tol, what):
    ref = np.asarray(ref, dtype=np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    err = np.abs(got - ref).max() / scale
    assert err < tol, f"{what}: max err {err:.3g} of scale {scale:.3g}"


@pytest.mark.parametrize("path", SSM_CASES, ids=lambda p: os.path.basename(p))
def test_loss_matches_reference_golden(path):
    z = np.load(path)
    loss, d_out, d_sup, d_w = _run(z["out"], z["sup_ids"], z["sup_emb"], z["weights"],
                                   z["weight"], z["all_ids"], z["offsets"], float(z["T"]),
                                   bool(z["l2_norm"]))
    ref = float(z["loss"])
    assert abs(loss - ref) <= 1e-5 * max(1.0, abs(ref)), (loss, ref)
    _close(d_out, z["d_out"], 2e-4, "d_out")
    _close(d_sup, z["d_sup_emb"], 2e-4, "d_sup_emb")
    _close(d_w, z["d_weight"], 2e-4, "d_weight")


def _random_case(M, D, V, R, T, seed, unit_out=True, zero_frac=0.15):
    g = torch.Generator().manual_seed(seed)
    ids = (torch.randperm(V, generator=g) + 1).numpy().astype(np.int64)
    weight = (torch.randn(V + 1, D, generator=g) * 0.3).numpy()
    weight[ids[0]] = 0.0                       # eps-clamp row of the table
    out = torch.randn(M, D, generator=g)
    if unit_out:
        out = out / out.norm(dim=-1, keepdim=True)
    sup_emb = torch.randn(M, D, generator=g).numpy()
    sup_ids = ids[torch.randint(0, V, (M,), generator=g).numpy()]
    sup_ids[torch.rand(M, generator=g).numpy() < zero_frac] = 0
    weights = (sup_ids != 0).astype(np.float32)
    offsets = torch.randint(0, V, (M, R), generator=g).numpy()
    return out.numpy(), sup_ids, sup_emb, weights, weight, ids, offsets


@pytest.mark.parametrize("M,D,V,R,T", [
    (3000, 50, 3953, 128, 0.05),   # ml-1m shapes
    (400, 256, 1000, 128, 0.05),   # ml-20m embedding width (E = 16 lanes-elements)
    (700, 64, 50, 100, 0.05),      # R not a multiple of 64, heavy id collisions
    (300, 32, 7, 1, 0.1),          # one negative, tiny catalog
    (200, 16, 30, 0, 0.05),        # no negatives: loss 0, gradients 0
    (129, 100, 500, 65, 0.2),      # D between lane-element buckets, R = 64 + 1
    (600, 50, 6000, 128, 0.05),    # V > 4096: counting-sort table-gradient path
    (150, 256, 40000, 128, 0.05),  # V > LDS histogram bins: global-atomic count path
])
def test_loss_random_vs_oracle(M, D, V, R, T):
    out, sup_ids, sup_emb, weights, weight, ids, offsets = _random_case(M, D, V, R, T, M + D + R)
    loss, d_out, d_sup, d_w = _run(out, sup_ids, sup_emb, weights, weight, ids, offsets, T, True)
    r = loss_oracle.sampled_softmax(out, sup_ids, sup_emb, weights, weight[ids], ids, offsets,
                                    T, True, 1e-6)
    assert abs(loss - float(r["loss"])) <= 1e-5 * max(1.0, abs(float(r["loss"])))
    d_weight = np.zeros_like(weight, dtype=np.float64)
    d_weight[ids] = r["d_table"]
    if R == 0:
        assert loss == 0.0 and not d_w.any()
    else:
        _close(d_w, d_weight, 2e-4, "d_weight")
    for got, key in ((d_out, "d_out"), (d_sup, "d_sup_emb")):
        if np.abs(r[key]).max() > 0:
            _close(got, r[key], 2e-4, key)
        else:
            assert not got.any(), key


@pytest.mark.parametrize("M,D,V,R", [(3000, 50, 3953, 128), (700, 64, 50, 100),
                                     (150, 256, 40000, 128)])
def test_table_gradient_deterministic_mode(M, D, V, R):
    """GR_OPT_DETERMINISTIC: the table gradient from a stable radix sort of the samples
    by row and one in-order sum per row -- equal to the oracle, bit-identical across runs
    (the default counting-sort path flushes rows with fp32 atomics in arbitrary order)."""
    from mygenerativerecommenders_amd import _lib, ops
    out, sup_ids, sup_emb, weights, weight, ids, offsets = _random_case(M, D, V, R, 0.05, 7 * M + D)
    dev = torch.device("cuda")
    tab = torch.as_tensor(weight[ids], dtype=torch.float32).to(dev)
    tab_n = tab / tab.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    sup = torch.as_tensor(sup_emb, dtype=torch.float32).to(dev)
    sup_n = sup / sup.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    o = torch.as_tensor(out, dtype=torch.float32).to(dev)
    offs = torch.as_tensor(offsets, dtype=torch.int64).to(dev)
    sid = torch.as_tensor(sup_ids).to(dev)
    all_ids = torch.as_tensor(ids).to(dev)
    w = torch.as_tensor(weights).to(dev)

    def grad_table():
        t = tab_n.detach().clone().requires_grad_(True)
        lt = ops.sampled_softmax_loss(o, sup_n, t, sid, offs, all_ids, 0.05)
        ((lt * w).sum() / w.sum()).backward()
        return t.grad
    with _lib.option("DETERMINISTIC", 1):
        g1 = grad_table()
        g2 = grad_table()
    g0 = grad_table()
    assert torch.equal(g1, g2)
    r = loss_oracle.sampled_softmax(out, sup_ids, sup_emb, weights, weight[ids], ids, offsets,
                                    0.05, True, 1e-6)
    _close(g1.cpu().double().numpy(), r["d_tab_norm"], 2e-4, "d_table (deterministic)")
    _close(g0.cpu().double().numpy(), r["d_tab_norm"], 2e-4, "d_table (atomic)")


def test_per_token_loss_vs_oracle():
    from mygenerativerecommenders_amd import ops
    out, sup_ids, sup_emb, weights, weight, ids, offsets = _random_case(2000, 50, 3953, 128,
                                                                        0.05, 5)
    r = loss_oracle.sampled_softmax(out, sup_ids, sup_emb, weights, weight[ids], ids, offsets,
                                    0.05, True, 1e-6, grads=False)
    pos = torch.from_numpy(sup_emb)
    pos = pos / pos.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    tab = torch.from_numpy(weight[ids])
    tab = tab / tab.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    lt = ops.sampled_softmax_loss(torch.from_numpy(out).cuda(), pos.cuda(), tab.cuda(),
                                  torch.from_numpy(sup_ids).cuda(),
                                  torch.from_numpy(offsets).cuda(), torch.from_numpy(ids).cuda(),
                                  0.05).cpu().double().numpy()
    assert np.all(np.abs(lt - r["loss_t"]) <= 1e-4 + 1e-5 * np.abs(r["loss_t"]))


def _torch_reference_loss(out, sup_ids, sup_emb, weights, table_raw, ids, offsets, T):
    """autoregressive_losses.py:259-306 restated in PyTorch fp32 (materialising path)."""
    def l2(x):
        return x / torch.clamp(torch.linalg.norm(x, ord=2, dim=-1, keepdim=True), min=1e-6)
    neg_ids = ids[offsets]
    neg = l2(table_raw[offsets])
    pos = l2(sup_emb)
    pos_logits = torch.bmm(pos.unsqueeze(1), out.unsqueeze(2)).squeeze(2) / T
    neg_logits = torch.bmm(neg, out.unsqueeze(2)).squeeze(2)
    neg_logits = torch.where(sup_ids.unsqueeze(1) == neg_ids, -5e4, neg_logits / T)
    jl = -torch.nn.functional.log_softmax(torch.cat([pos_logits, neg_logits], dim=1), dim=1)[:, 0]
    return (jl * weights).sum() / weights.sum()


def test_loss_c2_size_vs_torch_fp32():
    """ml-1m C2: 128 sequences x 199 supervised positions, R = 128, 3953-row catalog."""
    M, D, V, R, T = 128 * 199, 50, 3953, 128, 0.05
    out, sup_ids, sup_emb, weights, weight, ids, offsets = _random_case(M, D, V, R, T, 77)
    loss, d_out, d_sup, d_w = _run(out, sup_ids, sup_emb, weights, weight, ids, offsets, T, True)
    dev = torch.device("cuda")
    o = torch.from_numpy(out).to(dev).requires_grad_(True)
    p = torch.from_numpy(sup_emb).to(dev).requires_grad_(True)
    w = torch.from_numpy(weight).to(dev).requires_grad_(True)
    idt = torch.from_numpy(ids).to(dev)
    ref = _torch_reference_loss(o, torch.from_numpy(sup_ids).to(dev), p,
                                torch.from_numpy(weights).to(dev), w[idt], idt,
                                torch.from_numpy(offsets).to(dev), T)
    ref.backward()
    assert abs(loss - ref.item()) <= 1e-5 * abs(ref.item())
    _close(d_out, o.grad.cpu().double().numpy(), 2e-4, "d_out")
    _close(d_sup, p.grad.cpu().double().numpy(), 2e-4, "d_sup_emb")
    _close(d_w, w.grad.cpu().double().numpy(), 2e-4, "d_weight")


def test_sampler_forward_contract():
    from mygenerativerecommenders_amd.negatives_sampler import LocalNegativesSampler
    dev = torch.device("cuda")
    s = LocalNegativesSampler(True, 1e-6, all_item_ids=list(range(1, 101))).to(dev)
    s._embeddings_module = _Emb(torch.randn(101, 24, device=dev))
    pos_ids = torch.randint(1, 101, (17,), device=dev)
    ids, emb = s(pos_ids, 9)
    assert ids.shape == (17, 9) and emb.shape == (17, 9, 24)
    assert int(ids.min()) >= 1 and int(ids.max()) <= 100
    ref = s._embeddings_module.get_item_embeddings(ids)
    ref = ref / ref.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    assert torch.allclose(emb, ref, rtol=1e-6, atol=1e-6)


def test_empty_batch_is_nan_like_reference():
    out, sup_ids, sup_emb, weights, weight, ids, offsets = _random_case(0, 16, 10, 4, 0.05, 1)
    from mygenerativerecommenders_amd.losses import SampledSoftmaxLoss
    from mygenerativerecommenders_amd.similarity import DotProductSimilarity
    dev = torch.device("cuda")
    emb = _Emb(torch.from_numpy(weight).to(dev))
    s = _sampler(True, torch.from_numpy(ids), torch.from_numpy(offsets).to(dev), emb)
    loss = SampledSoftmaxLoss(4, 0.05).jagged_forward(
        torch.from_numpy(out).to(dev), torch.from_numpy(sup_ids).to(dev),
        torch.from_numpy(sup_emb).to(dev), torch.from_numpy(weights).to(dev), s,
        DotProductSimilarity())
    assert torch.isnan(loss).item()


def test_loss_graph_replays_match_eager():
    """The loss forward + backward captured into one HIP graph and replayed 3 times gives
    the eager result every time (the table-gradient counting sort keeps per-step counters
    that must be re-zeroed inside the graph)."""
    M, D, V, R, T = 4000, 50, 3953, 128, 0.05
    out, sup_ids, sup_emb, weights, weight, ids, offsets = _random_case(M, D, V, R, T, 9)
    ref = _run(out, sup_ids, sup_emb, weights, weight, ids, offsets, T, True)
    from mygenerativerecommenders_amd.losses import SampledSoftmaxLoss
    from mygenerativerecommenders_amd.similarity import DotProductSimilarity
    dev = torch.device("cuda")
    emb = _IselEmb(torch.as_tensor(weight).to(dev))
    s = _sampler(True, torch.as_tensor(ids), torch.as_tensor(offsets).to(dev), emb)
    o = torch.as_tensor(out).to(dev).requires_grad_(True)
    p = torch.as_tensor(sup_emb).to(dev).requires_grad_(True)
    sid = torch.as_tensor(sup_ids).to(dev)
    wt = torch.as_tensor(weights).to(dev)
    mod, sim = SampledSoftmaxLoss(R, T), DotProductSimilarity()

    def step():
        loss = mod.jagged_forward(o, sid, p, wt, s, sim)
        loss.backward()
        return loss

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    for t in (o, p, emb.weight):
        t.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss_static = step()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert abs(loss_static.item() - ref[0]) <= 1e-5 * max(1.0, abs(ref[0]))
        _close(o.grad.cpu().double().numpy(), ref[1], 1e-5, "d_out")
        _close(emb.weight.grad.cpu().double().numpy(), ref[3], 1e-5, "d_weight")
        # the counting sort's bound checks dropped nothing
        from mygenerativerecommenders_amd.ops import last_sampled_softmax_status
        assert last_sampled_softmax_status() == 0


@pytest.mark.parametrize("dedup", [False, True])
def test_in_batch_negatives_vs_oracle(dedup):
    """InBatchNegativesSampler (negative_sampler.py:135-211) under the fused loss: the
    batch's present rows (de-duplicated by id with the reference's own torch.unique call)
    are the table, offsets are the reference's draw over it (same generator state), and
    loss, d_out and the embedding-weight gradient (through the cache, the positives and
    the normalisation) match the float64 oracle run on that table."""
    from mygenerativerecommenders_amd.losses import SampledSoftmaxLoss
    from mygenerativerecommenders_amd.negatives_sampler import InBatchNegativesSampler
    from mygenerativerecommenders_amd.similarity import DotProductSimilarity
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(31 + int(dedup))
    B, N, D, V, R, T = 6, 40, 48, 90, 64, 0.05
    weight = torch.randn(V, D, generator=g)
    ids = torch.randint(1, V, (B, N), generator=g)
    presences = torch.rand(B, N, generator=g) > 0.25
    out = torch.randn(int(presences.sum()), D, generator=g)
    w_p = weight.clone().to(dev).requires_grad_(True)
    out_p = out.clone().to(dev).requires_grad_(True)
    ids_d, pres_d = ids.to(dev), presences.to(dev)
    emb = w_p[ids_d]                                  # (B, N, D): a function of the id
    sampler = InBatchNegativesSampler(True, 1e-6, dedup)
    sampler.process_batch(ids_d, pres_d, emb)
    sup_ids = ids_d[pres_d]
    sup_emb = emb[pres_d]
    weights = torch.ones(sup_ids.shape, device=dev)
    torch.manual_seed(123)
    loss = SampledSoftmaxLoss(R, T).jagged_forward(out_p, sup_ids, sup_emb, weights, sampler,
                                                   DotProductSimilarity())
    loss.backward()
    torch.manual_seed(123)
    offsets = sampler.sample_offsets(sup_ids, R)
    cache_ids = sampler.get_all_ids_and_embeddings()[0].cpu().numpy()
    table = weight.numpy()[cache_ids]               # the cache rows before normalisation
    r = loss_oracle.sampled_softmax(out.numpy(), sup_ids.cpu().numpy(), sup_emb.detach().cpu().numpy(),
                                    weights.cpu().numpy(), table, cache_ids,
                                    offsets.cpu().numpy(), T, True, 1e-6)
    assert abs(loss.item() - float(r["loss"])) <= 1e-5 * max(1.0, abs(float(r["loss"])))
    d_weight = np.zeros((V, D), dtype=np.float64)
    np.add.at(d_weight, sup_ids.cpu().numpy(), r["d_sup_emb"])
    np.add.at(d_weight, cache_ids, r["d_table"])
    _close(out_p.grad.cpu().double().numpy(), r["d_out"], 2e-4, "d_out")
    _close(w_p.grad.cpu().double().numpy(), d_weight, 2e-4, "d_weight")
    if dedup:
        assert len(set(cache_ids.tolist())) == len(cache_ids)
