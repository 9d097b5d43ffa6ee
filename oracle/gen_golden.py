"""Golden-fixture generator (TEST INFRASTRUCTURE — runs only in the survey/build
container, never on the GPU box, never on the product path).

It imports the REFERENCE implementation from ``/root/reference/src`` and records
input -> output pairs as small ``.npz`` files under ``tests/golden/``.  Only these
data files travel; the reference itself does not.

Fixtures written:
  * ``bucket_thresholds.npz``  -- for b in [0, 128], the smallest integer |dt| whose
    reference bucket (``hstu.py:579-581`` lambda, clamped as at ``hstu.py:117-123``)
    is >= b.  Found by binary search over the reference's own bucketization fn.
  * ``hstu_*.npz``             -- ``HSTU.forward`` (``hstu.py:633-672``) output and
    the gradients of the input embeddings and of every encoder parameter, eval mode
    (dropout off), fp32, jagged lengths, seeded.
  * ``topk_T1.npz`` / ``topk_T2.npz`` -- ``CandidateIndex.get_top_k_outputs``
    (``candidate_index.py:107-164``) over ``MIPSBruteForceTopK`` (``top_k.py:44-70``)
    with invalid ids. T1: random normal; T2: integer-valued, tie-free (exact in any
    summation order).
  * ``jagged_ops.npz``         -- the known-answer cases of the reference's
    ``tests/test_ops.py:7-53`` (cumsum / dense_to_jagged / jagged_to_padded_dense).
  * ``preproc.npz``            -- ``LearnablePositionalEmbeddingInputFeaturesPreprocessor``
    (``learnable_positional_embedding.py:42-58``), eval mode, with input / table grads.
  * ``decode_*.npz``           -- the cached (incremental) ``HSTU.forward`` path: a full
    pass with ``return_cache_states=True`` (``hstu.py:420-423``), then one step with
    ``delta_x_offsets`` / ``cache`` (``hstu.py:293-298, 321-322, 151-177, 415-418``) that
    re-encodes one position per sequence; outputs and every layer's cache states.
  * ``softmax_*.npz``          -- ``HSTU.forward`` with ``normalization="softmax_rel_bias"``
    (``hstu.py:341-389``): output and every gradient, as the ``hstu_*`` cases.
  * ``muon.npz``               -- two ``Muon.step`` (``optimizers/muon.py:46-86``) on CPU.
  * ``embeddings.npz``         -- ``LocalEmbeddingModule.get_item_embeddings``
    (``embeddings/embeddings.py:94-97``) with an installed item -> year mapping, and the
    gradients of both tables.
  * ``ssm_*.npz``              -- ``SampledSoftmaxLoss.jagged_forward``
    (``autoregressive_losses.py:259-306``) with ``LocalNegativesSampler``
    (``negative_sampler.py:66-131``) and ``DotProductSimilarity``: inputs, the seed of
    the sampling draw, the sampled ids / offsets it produced, the loss and the
    gradients of the query rows, the supervision embeddings and the embedding table.

Usage:  python oracle/gen_golden.py [--only loss|preproc|muon|embeddings|decode|softmax]   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _import_reference():
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    from generative_recommenders_pl.models.indexing.candidate_index import (  # noqa
        CandidateIndex,
    )
    from generative_recommenders_pl.models.indexing.top_k import (  # noqa
        MIPSBruteForceTopK,
    )
    from generative_recommenders_pl.models.sequential_encoders.hstu import HSTU  # noqa
    from generative_recommenders_pl.models.utils import ops  # noqa

    return HSTU, CandidateIndex, MIPSBruteForceTopK, ops


def synth_timestamps(gen: torch.Generator, B: int, N: int, lengths: torch.Tensor):
    """SURVEY.md §8d timestamps: start U[9.5e8, 1.05e9], Exp(1e5 s) increments,
    sorted, padded positions 0, the target timestamp sits at index L_b
    (``features.py:53-57``)."""
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        start = 9.5e8 + float(torch.rand(1, generator=gen)) * 1e8
        inc = -torch.log(torch.rand(L + 1, generator=gen).clamp_min(1e-12)) * 1e5
        seq = (start + torch.cumsum(inc, 0)).to(torch.int64)
        n_fill = min(L + 1, N)
        ts[b, :n_fill] = seq[:n_fill]
    return ts


def gen_bucket_thresholds(HSTU):
    enc = HSTU(
        max_sequence_len=4, max_output_len=1, embedding_dim=8, item_embedding_dim=8,
        num_blocks=1, num_heads=1, linear_dim=8, attention_dim=8,
        normalization="rel_bias", linear_config="uvqk", linear_activation="silu",
        linear_dropout_rate=0.0, attn_dropout_rate=0.0,
    )
    rab = enc._hstu._attention_layers[0]._rel_attn_bias
    fn = rab._bucketization_fn
    nb = rab._num_buckets

    def bucket(x: int) -> int:
        t = torch.tensor([x], dtype=torch.int64)
        return int(torch.clamp(fn(t), min=0, max=nb)[0])

    thr = np.zeros(nb + 1, dtype=np.int64)
    hi_limit = (1 << 62)
    for b in range(1, nb + 1):
        lo, hi = 1, hi_limit
        assert bucket(hi) >= b, b
        while lo < hi:
            mid = (lo + hi) // 2
            if bucket(mid) >= b:
                hi = mid
            else:
                lo = mid + 1
        thr[b] = lo
    # monotonicity spot check on a dense + log-spaced sweep
    xs = np.unique(np.concatenate([
        np.arange(0, 5000, dtype=np.int64),
        np.logspace(0, 18, 20000).astype(np.int64),
        thr, np.maximum(thr - 1, 0), thr + 1,
    ]))
    t = torch.from_numpy(xs)
    ref = torch.clamp(fn(t), min=0, max=nb).numpy()
    via_table = np.searchsorted(thr, xs, side="right") - 1
    assert np.array_equal(ref, via_table), "bucket fn is not monotone / table wrong"
    # negative deltas: reference takes abs()
    ref_neg = torch.clamp(fn(-t), min=0, max=nb).numpy()
    assert np.array_equal(ref_neg, via_table)
    np.savez_compressed(os.path.join(OUT, "bucket_thresholds.npz"), thresholds=thr,
             probe_x=xs, probe_bucket=ref.astype(np.int64))
    print("bucket thresholds:", thr[:16].tolist(), "... max", thr[-1])
    return thr


def gen_hstu_case(HSTU, name, B, N0, out_len, D, H, dqk, dv, blocks, seed,
                  lengths=None, with_ts=True, concat_ua=False, normalization="rel_bias",
                  rab=True, prefix="hstu"):
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)
    N = N0 + out_len
    enc = HSTU(
        max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
        item_embedding_dim=D, num_blocks=blocks, num_heads=H, linear_dim=dv,
        attention_dim=dqk, normalization=normalization, linear_config="uvqk",
        linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
        concat_ua=concat_ua, enable_relative_attention_bias=rab,
    )
    # the reference zero-inits nothing; pos/ts weights are N(0, 0.02).  Scale them up
    # so the bias path is exercised with O(1) magnitudes.
    with torch.no_grad():
        for layer in enc._hstu._attention_layers:
            if rab:
                layer._rel_attn_bias._ts_w.normal_(0, 0.5, generator=gen)
                layer._rel_attn_bias._pos_w.normal_(0, 0.5, generator=gen)
            layer._o.bias.normal_(0, 0.1, generator=gen)
    enc.eval()
    if lengths is None:
        lengths = torch.randint(1, N0 + 1, (B,), generator=gen)
    lengths = torch.as_tensor(lengths, dtype=torch.int64)
    x = torch.randn(B, N, D, generator=gen)
    # padded rows are ignored by the reference (dense_to_jagged drops them)
    ts = synth_timestamps(gen, B, N, lengths)
    payload = {"timestamps": ts} if with_ts else {}
    x.requires_grad_(True)
    y, _ = enc(past_lengths=lengths, user_embeddings=x,
               valid_mask=torch.ones(B, N, 1), past_payloads=payload)
    dy = torch.randn(y.shape, generator=gen)
    (y * dy).sum().backward()
    rec = {
        "B": B, "N0": N0, "out_len": out_len, "N": N, "D": D, "H": H, "dqk": dqk,
        "dv": dv, "blocks": blocks, "with_ts": int(with_ts), "concat_ua": int(concat_ua),
        "normalization": normalization, "rab": int(rab),
        "lengths": lengths.numpy(), "x": x.detach().numpy(), "ts": ts.numpy(),
        "y": y.detach().numpy(), "dy": dy.numpy(), "dx": x.grad.numpy(),
    }
    for pname, p in enc.named_parameters():
        rec["param:" + pname] = p.detach().numpy()
        rec["grad:" + pname] = (p.grad if p.grad is not None
                                else torch.zeros_like(p)).numpy()
    np.savez_compressed(os.path.join(OUT, f"{prefix}_{name}.npz"), **rec)
    print(f"{prefix}_{name}: y {tuple(y.shape)} |y|max {y.abs().max():.3f}")


def gen_hstu_decode_case(HSTU, name, B, N0, out_len, D, H, dqk, dv, blocks, seed, lengths,
                         positions, with_ts=True, concat_ua=False):
    """Full pass with cache states, then one cached step: sequence b's row at position
    positions[b] (delta_x_offsets = (offsets[b] + p, p)) gets a new embedding and a new
    timestamp.  The reference mutates the cache tensors in place, so the first pass's
    states are copied before the step."""
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)
    N = N0 + out_len
    enc = HSTU(
        max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
        item_embedding_dim=D, num_blocks=blocks, num_heads=H, linear_dim=dv,
        attention_dim=dqk, normalization="rel_bias", linear_config="uvqk",
        linear_activation="silu", linear_dropout_rate=0.2, attn_dropout_rate=0.0,
        concat_ua=concat_ua,
    )
    with torch.no_grad():
        for layer in enc._hstu._attention_layers:
            layer._rel_attn_bias._ts_w.normal_(0, 0.5, generator=gen)
            layer._rel_attn_bias._pos_w.normal_(0, 0.5, generator=gen)
            layer._o.bias.normal_(0, 0.1, generator=gen)
    enc.eval()
    lengths = torch.as_tensor(lengths, dtype=torch.int64)
    pos = torch.as_tensor(positions, dtype=torch.int64)
    assert bool((pos < lengths).all())
    x0 = torch.randn(B, N, D, generator=gen)
    ts0 = synth_timestamps(gen, B, N, lengths)
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lengths, 0)])
    rec = {
        "B": B, "N0": N0, "out_len": out_len, "N": N, "D": D, "H": H, "dqk": dqk,
        "dv": dv, "blocks": blocks, "with_ts": int(with_ts), "concat_ua": int(concat_ua),
        "lengths": lengths.numpy(), "positions": pos.numpy(), "x0": x0.numpy(),
        "ts0": ts0.numpy(),
    }
    with torch.no_grad():
        y0, states = enc(past_lengths=lengths, user_embeddings=x0,
                         valid_mask=torch.ones(B, N, 1),
                         past_payloads={"timestamps": ts0} if with_ts else {},
                         return_cache_states=True)
        rec["y0"] = y0.numpy()
        for l, st in enumerate(states):
            for nm, t in zip(("v", "q", "k", "out"), st):
                rec[f"s0:{l}:{nm}"] = t.detach().clone().numpy()
        x1 = x0.clone()
        ts1 = ts0.clone()
        for b in range(B):
            p = int(pos[b])
            x1[b, p] = torch.randn(D, generator=gen)
            # a new timestamp between the neighbours' (or past the last one)
            lo = int(ts0[b, p - 1]) if p > 0 else int(ts0[b, p]) - 500000
            ts1[b, p] = lo + int(torch.randint(1, 400000, (1,), generator=gen))
        delta = (offsets[:-1] + pos, pos.clone())
        y1, states1 = enc(past_lengths=lengths, user_embeddings=x1,
                          valid_mask=torch.ones(B, N, 1),
                          past_payloads={"timestamps": ts1} if with_ts else {},
                          delta_x_offsets=delta, cache=states, return_cache_states=True)
    rec["x1"] = x1.numpy()
    rec["ts1"] = ts1.numpy()
    rec["delta0"] = delta[0].numpy()
    rec["delta1"] = delta[1].numpy()
    rec["y1"] = y1.numpy()
    for l, st in enumerate(states1):
        for nm, t in zip(("v", "q", "k", "out"), st):
            rec[f"s1:{l}:{nm}"] = t.detach().numpy()
    for pname, p in enc.named_parameters():
        rec["param:" + pname] = p.detach().numpy()
    np.savez_compressed(os.path.join(OUT, f"decode_{name}.npz"), **rec)
    print(f"decode_{name}: y1 {tuple(y1.shape)} |y1 - y0|max {(y1 - y0).abs().max():.3f}")


def gen_decode():
    HSTU = _import_reference()[0]
    gen_hstu_decode_case(HSTU, "b3_n16_d16_h1", 3, 16, 5, 16, 1, 16, 16, 2, seed=61,
                         lengths=[21, 9, 1], positions=[20, 4, 0])
    gen_hstu_decode_case(HSTU, "b4_n24_d24_h2", 4, 24, 3, 24, 2, 12, 12, 2, seed=62,
                         lengths=[27, 13, 5, 20], positions=[26, 12, 2, 0])
    gen_hstu_decode_case(HSTU, "b2_n12_d16_nots", 2, 12, 2, 16, 1, 16, 8, 1, seed=63,
                         lengths=[14, 6], positions=[13, 5], with_ts=False)
    gen_hstu_decode_case(HSTU, "b2_n12_d16_cua", 2, 12, 2, 16, 1, 16, 16, 2, seed=64,
                         lengths=[10, 14], positions=[9, 7], concat_ua=True)


def gen_softmax():
    """normalization="softmax_rel_bias" (hstu.py:341-389, non-cached branch): padded q / k
    over all heads' columns at once, softmax over every one of the n keys (padding and
    future keys included) of (qk + bias) / sqrt(attention_dim), then the causal mask."""
    HSTU = _import_reference()[0]
    gen_hstu_case(HSTU, "b4_n16_d16_h1", 4, 16, 5, 16, 1, 16, 16, 2, seed=71,
                  normalization="softmax_rel_bias", prefix="softmax")
    gen_hstu_case(HSTU, "b3_n24_d24_h2", 3, 24, 5, 24, 2, 8, 12, 2, seed=72,
                  lengths=[29, 1, 13], normalization="softmax_rel_bias", prefix="softmax")
    gen_hstu_case(HSTU, "b3_n16_d16_norab", 3, 16, 3, 16, 1, 16, 16, 1, seed=73,
                  normalization="softmax_rel_bias", rab=False, prefix="softmax")
    gen_hstu_case(HSTU, "b2_n12_d16_cua", 2, 12, 2, 16, 1, 16, 16, 1, seed=74,
                  lengths=[14, 6], normalization="softmax_rel_bias", concat_ua=True,
                  prefix="softmax")


def gen_topk_case(CandidateIndex, MIPSBruteForceTopK, name, B, X, D, k, N0, seed,
                  integer=False):
    gen = torch.Generator().manual_seed(seed)
    ids = torch.arange(1, X + 1, dtype=torch.int64)
    if integer:
        # T2: integer-valued so fp32 sums are exact in ANY order; tie-free via the
        # last component e_last = j (item index), q_last = 1, other dims scaled 2^12.
        assert X <= 4096
        E = torch.randint(-8, 9, (X, D), generator=gen).float() * 4096.0
        E[:, -1] = torch.arange(X).float()
        Q = torch.randint(-8, 9, (B, D), generator=gen).float()
        Q[:, -1] = 1.0
    else:
        E = torch.randn(X, D, generator=gen)
        E = E / E.norm(dim=-1, keepdim=True).clamp_min(1e-6)
        Q = torch.randn(B, D, generator=gen)
        Q = Q / Q.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    # invalid ids: mostly drawn from the top of each row's ranking (so exclusion
    # matters), tail zero-padded like past_ids padding.
    logits = Q @ E.T
    order = torch.argsort(logits, dim=1, descending=True)
    invalid = torch.zeros(B, N0, dtype=torch.int64)
    for b in range(B):
        n_valid = int(torch.randint(N0 // 2, N0 + 1, (1,), generator=gen))
        pick = order[b, : 2 * N0][torch.randperm(2 * N0, generator=gen)[:n_valid]]
        invalid[b, :n_valid] = ids[pick]
    index = CandidateIndex(k=k, ids=ids, top_k_module=MIPSBruteForceTopK(),
                           embeddings=E.unsqueeze(0))
    top_ids, top_scores = index.get_top_k_outputs(query_embeddings=Q, invalid_ids=invalid)
    np.savez_compressed(
        os.path.join(OUT, f"topk_{name}.npz"), Q=Q.numpy(), E=E.numpy(), ids=ids.numpy(),
        invalid=invalid.numpy(), k=k, top_ids=top_ids.numpy(),
        top_scores=top_scores.numpy(), integer=int(integer))
    print(f"topk_{name}: B={B} X={X} D={D} k={k} N0={N0}")


def gen_jagged_ops(ops):
    lengths = torch.tensor([1, 2], dtype=torch.int32)
    offs = ops.asynchronous_complete_cumsum(lengths)
    dense = torch.tensor([[1.0, 2, 3], [4, 5, 6]]).unsqueeze(-1)
    jag = ops.dense_to_jagged(dense, offs)
    values = torch.tensor([1.0, 4, 5]).unsqueeze(-1)
    offs2 = torch.tensor([0, 1, 3])
    pad = ops.jagged_to_padded_dense(values, offs2, 3, 0)
    np.savez(os.path.join(OUT, "jagged_ops.npz"), lengths=lengths.numpy(),
             offsets=offs.numpy(), dense=dense.numpy(), jagged=jag.numpy(),
             values=values.numpy(), offsets2=offs2.numpy(), padded=pad.numpy())


def _import_reference_loss():
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    from generative_recommenders_pl.models.losses.autoregressive_losses import (  # noqa
        SampledSoftmaxLoss,
    )
    from generative_recommenders_pl.models.negatives_samples.negative_sampler import (  # noqa
        LocalNegativesSampler,
    )
    from generative_recommenders_pl.models.similarity.dot_product import (  # noqa
        DotProductSimilarity,
    )

    return SampledSoftmaxLoss, LocalNegativesSampler, DotProductSimilarity


def gen_sampled_softmax_case(name, M, D, n_catalog, R, T, l2_norm, seed, use_all_ids=True,
                             zero_rows=False, unit_out=False):
    SampledSoftmaxLoss, LocalNegativesSampler, DotProductSimilarity = _import_reference_loss()

    class _Capture(LocalNegativesSampler):
        def forward(self, positive_ids, num_to_sample):
            ids, emb = super().forward(positive_ids, num_to_sample)
            self.captured = ids.detach().clone()
            return ids, emb

    class _Emb(torch.nn.Module):
        def __init__(self, weight):
            super().__init__()
            self.emb = torch.nn.Embedding.from_pretrained(weight, freeze=False)

        def get_item_embeddings(self, ids):
            return self.emb(ids)

    g = torch.Generator().manual_seed(seed)
    if use_all_ids:
        all_ids = (torch.randperm(n_catalog, generator=g) + 1).tolist()
        sampler = _Capture(l2_norm=l2_norm, l2_norm_eps=1e-6, all_item_ids=all_ids)
    else:
        all_ids = list(range(n_catalog))
        sampler = _Capture(l2_norm=l2_norm, l2_norm_eps=1e-6, num_items=n_catalog)
    weight = torch.randn(max(all_ids) + 1, D, generator=g) * 0.5
    out = torch.randn(M, D, generator=g)
    if unit_out:  # as the training step's L2-normalised encoder output
        out = out / out.norm(dim=-1, keepdim=True)
    sup_emb = torch.randn(M, D, generator=g)
    if zero_rows:
        weight[all_ids[0]] = 0.0
        weight[all_ids[1]] *= 1e-8
        sup_emb[0] = 0.0
    cat = torch.tensor(all_ids)
    sup_ids = cat[torch.randint(0, n_catalog, (M,), generator=g)]
    sup_ids[torch.rand(M, generator=g) < 0.15] = 0
    weights = (sup_ids != 0).float()
    emb = _Emb(weight.clone())
    sampler._embeddings_module = emb
    out.requires_grad_(True)
    sup_emb.requires_grad_(True)
    rng_seed = seed + 1000
    torch.manual_seed(rng_seed)
    loss = SampledSoftmaxLoss(num_to_sample=R, softmax_temperature=T).jagged_forward(
        output_embeddings=out, supervision_ids=sup_ids, supervision_embeddings=sup_emb,
        supervision_weights=weights, negatives_sampler=sampler,
        similarity=DotProductSimilarity())
    loss.backward()
    sampled = sampler.captured
    inv = {int(v): i for i, v in enumerate(all_ids)}
    offsets = torch.tensor([[inv[int(v)] for v in row] for row in sampled.reshape(M, R)],
                           dtype=torch.int64).reshape(M, R)
    rec = dict(out=out.detach().numpy(), sup_ids=sup_ids.numpy(),
               sup_emb=sup_emb.detach().numpy(), weights=weights.numpy(),
               weight=weight.numpy(), all_ids=np.array(all_ids, dtype=np.int64),
               use_all_ids=np.array(use_all_ids), sampled_ids=sampled.numpy(),
               offsets=offsets.numpy(), rng_seed=np.array(rng_seed), R=np.array(R),
               T=np.array(T, dtype=np.float64), l2_norm=np.array(l2_norm),
               eps=np.array(1e-6), loss=np.array(loss.item(), dtype=np.float32),
               d_out=out.grad.numpy(), d_sup_emb=sup_emb.grad.numpy(),
               d_weight=emb.emb.weight.grad.numpy())
    np.savez_compressed(os.path.join(OUT, f"ssm_{name}.npz"), **rec)
    n_coll = int((sampled.reshape(M, R) == sup_ids[:, None]).sum())
    print(f"ssm_{name}: loss {loss.item():.6f} collisions {n_coll}")


def gen_preprocessor():
    """LearnablePositionalEmbeddingInputFeaturesPreprocessor.forward (eval: dropout off)
    and the gradients of its input and positional table."""
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    from generative_recommenders_pl.models.preprocessors.learnable_positional_embedding import (  # noqa
        LearnablePositionalEmbeddingInputFeaturesPreprocessor as Pre,
    )
    torch.manual_seed(31)
    B, N, D = 3, 13, 24
    m = Pre(max_sequence_len=20, embedding_dim=D, dropout_rate=0.2).eval()
    g = torch.Generator().manual_seed(32)
    x = torch.randn(B, N, D, generator=g, requires_grad=True)
    ids = torch.randint(1, 50, (B, N), generator=g)
    ids[0, 9:] = 0
    ids[2, 4:] = 0
    lengths = (ids != 0).sum(1)
    _, y, valid, _ = m(lengths, ids, x, {})
    dy = torch.randn(B, N, D, generator=g)
    (y * dy).sum().backward()
    np.savez_compressed(os.path.join(OUT, "preproc.npz"), x=x.detach().numpy(), ids=ids.numpy(),
                        pos_w=m._pos_emb.weight.detach().numpy(), y=y.detach().numpy(),
                        valid=valid.numpy(), dy=dy.numpy(), dx=x.grad.numpy(),
                        dpos=m._pos_emb.weight.grad.numpy())
    print(f"preproc: y {tuple(y.shape)}")


def gen_embeddings():
    """LocalEmbeddingModule.get_item_embeddings (embeddings/embeddings.py:94-97) and the
    gradients of its two tables, with an item -> year mapping installed in the module's
    ``item2year`` global (the reference fills it from a CSV that does not exist here)."""
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    import generative_recommenders_pl.models.embeddings.embeddings as E  # noqa
    torch.manual_seed(51)
    num_items, dim = 2100, 50
    g = torch.Generator().manual_seed(52)
    years = torch.randint(1919, 2001, (num_items,), generator=g)
    E.item2year = {i + 1: int(years[i]) for i in range(0, num_items - 300)}  # ids > 1800 unmapped
    m = E.LocalEmbeddingModule(num_items=num_items, item_embedding_dim=dim)
    ids = torch.randint(0, num_items + 1, (5, 37), generator=g)
    ids[1, 20:] = 0
    ids[3, :5] = 1799
    out = m.get_item_embeddings(ids)
    dout = torch.randn(out.shape, generator=g)
    (out * dout).sum().backward()
    np.savez_compressed(os.path.join(OUT, "embeddings.npz"), ids=ids.numpy(),
                        item_w=m._item_emb.weight.detach().numpy(),
                        year_w=m._year_emb.weight.detach().numpy(),
                        year_table=m.year_lookup_table.numpy(), out=out.detach().numpy(),
                        dout=dout.numpy(), d_item_w=m._item_emb.weight.grad.numpy(),
                        d_year_w=m._year_emb.weight.grad.numpy())
    print(f"embeddings: out {tuple(out.shape)}")


def gen_muon():
    """Two steps of the reference Muon (optimizers/muon.py:46-86) on CPU over parameters of
    three shape classes (wide, tall, two square of one shape) with fixed gradients."""
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    from generative_recommenders_pl.models.optimizers.muon import Muon  # noqa
    g = torch.Generator().manual_seed(41)
    shapes = [(8, 24), (24, 8), (12, 12), (12, 12)]
    params = [torch.nn.Parameter(torch.randn(s, generator=g)) for s in shapes]
    p0 = [p.detach().clone() for p in params]
    opt = Muon(params, lr=0.02, weight_decay=0.01, momentum=0.95)
    rec = {f"p0_{i}": p.numpy() for i, p in enumerate(p0)}
    for step in range(2):
        for i, p in enumerate(params):
            gr = torch.randn(p.shape, generator=g)
            rec[f"g{step}_{i}"] = gr.numpy()
            p.grad = gr.clone()
        opt.step()
        for i, p in enumerate(params):
            rec[f"p{step + 1}_{i}"] = p.detach().numpy().copy()
    np.savez_compressed(os.path.join(OUT, "muon.npz"), **rec)
    print("muon: 2 steps over", shapes)


def gen_sampled_softmax():
    gen_sampled_softmax_case("small", 37, 16, 40, 24, 0.05, True, seed=21)
    gen_sampled_softmax_case("d50", 64, 50, 300, 128, 0.05, True, seed=22, unit_out=True)
    gen_sampled_softmax_case("nol2", 29, 24, 20, 70, 0.1, False, seed=23, use_all_ids=False)
    gen_sampled_softmax_case("zero", 16, 8, 12, 5, 0.05, True, seed=24, zero_rows=True)


def main():
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if only == "loss":
        gen_sampled_softmax()
        return
    if only == "preproc":
        gen_preprocessor()
        return
    if only == "muon":
        gen_muon()
        return
    if only == "embeddings":
        gen_embeddings()
        return
    if only == "decode":
        gen_decode()
        return
    if only == "softmax":
        gen_softmax()
        return
    gen_sampled_softmax()
    gen_preprocessor()
    gen_muon()
    gen_embeddings()
    gen_decode()
    gen_softmax()
    HSTU, CandidateIndex, MIPSBruteForceTopK, ops = _import_reference()
    gen_bucket_thresholds(HSTU)
    gen_jagged_ops(ops)
    # HSTU goldens: B=4, N0 in {16, 32}, D in {16, 50},
    # h in {1, 2}, 2 blocks, jagged lengths.
    gen_hstu_case(HSTU, "b4_n16_d16_h1", 4, 16, 11, 16, 1, 16, 16, 2, seed=1)
    gen_hstu_case(HSTU, "b4_n32_d50_h1", 4, 32, 11, 50, 1, 50, 50, 2, seed=2)
    gen_hstu_case(HSTU, "b4_n32_d16_h2", 4, 32, 11, 16, 2, 8, 8, 2, seed=3)
    gen_hstu_case(HSTU, "b3_n64_d50_h2", 3, 64, 11, 50, 2, 25, 25, 2, seed=4,
                  lengths=[64, 1, 37])
    # full-length row (L_b = N0 so query N-1 ... uses ts[N-1] wrap) and no-timestamp
    gen_hstu_case(HSTU, "b2_n8_d16_full", 2, 8, 0, 16, 1, 16, 16, 2, seed=5,
                  lengths=[8, 5])
    gen_hstu_case(HSTU, "b3_n16_d16_nots", 3, 16, 11, 16, 1, 16, 16, 2, seed=6,
                  with_ts=False)
    gen_hstu_case(HSTU, "b2_n16_d16_cua", 2, 16, 11, 16, 1, 16, 16, 1, seed=7,
                  concat_ua=True)
    gen_topk_case(CandidateIndex, MIPSBruteForceTopK, "T1", 16, 3000, 50, 200, 211,
                  seed=11)
    gen_topk_case(CandidateIndex, MIPSBruteForceTopK, "T2", 16, 4000, 50, 200, 211,
                  seed=12, integer=True)
    gen_topk_case(CandidateIndex, MIPSBruteForceTopK, "T3_small", 5, 300, 16, 10, 7,
                  seed=13)


if __name__ == "__main__":
    main()
