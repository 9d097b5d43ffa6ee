"""GPU: the reference's calling sequence around the hot path (retrieval.py:19-210,
generative_recommenders.py:355-430, utils/features.py:20-84), driven through
``runner.RetrievalRunner`` over the drop-in modules, against a CPU restatement of the
same sequence built from the oracles (HSTU: ``hstu_oracle``, loss: ``loss_oracle`` /
its torch form, top-k: the C oracle, metrics: ``metrics_oracle``).

Covered contracts: the target timestamp scattered at ``length`` (features.py:53-57), the
target id scattered into ``past_ids`` (retrieval.py:85-89), the ``[:, :-1]`` /
``[:, 1:]`` supervision shift and ar mask (retrieval.py:118-124), ids through float in
``dense_to_jagged`` (generative_recommenders.py:410-417), local negatives drawn from the
live embedding module, then validation: ``update_embeddings`` under inference mode,
``retrieve`` with ``past_ids`` as invalid ids, metrics."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import hstu_oracle as O
from oracle import loss_oracle, metrics_oracle, topk_oracle

pytestmark = pytest.mark.gpu

V, D, N0, OUT_LEN, BLOCKS, B, R, T, K = 400, 32, 48, 10, 2, 6, 16, 0.05, 20


def _modules(dev):
    from mygenerativerecommenders_amd.candidate_index import CandidateIndex
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    from mygenerativerecommenders_amd.hstu import HSTU
    from mygenerativerecommenders_amd.losses import SampledSoftmaxLoss
    from mygenerativerecommenders_amd.metrics import RetrievalMetrics
    from mygenerativerecommenders_amd.negatives_sampler import LocalNegativesSampler
    from mygenerativerecommenders_amd.postprocessors import L2NormEmbeddingPostprocessor
    from mygenerativerecommenders_amd.preprocessors import (
        LearnablePositionalEmbeddingInputFeaturesPreprocessor as Pre)
    from mygenerativerecommenders_amd.runner import RetrievalRunner
    from mygenerativerecommenders_amd.similarity import DotProductSimilarity
    from mygenerativerecommenders_amd.top_k import MIPSBruteForceTopK
    torch.manual_seed(0)
    N = N0 + OUT_LEN + 1
    emb = LocalEmbeddingModule(V, D).to(dev)
    pre = Pre(N, D, 0.0).to(dev).train()
    enc = HSTU(max_sequence_len=N0, max_output_len=OUT_LEN + 1, embedding_dim=D,
               item_embedding_dim=D, num_blocks=BLOCKS, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.0,
               attn_dropout_rate=0.0).to(dev).train()
    with torch.no_grad():  # visible relative-bias terms
        for layer in enc._hstu._attention_layers:
            layer._rel_attn_bias._ts_w.normal_(0, 0.3)
            layer._rel_attn_bias._pos_w.normal_(0, 0.3)
    post = L2NormEmbeddingPostprocessor(D, 1e-6)
    sampler = LocalNegativesSampler(True, 1e-6, all_item_ids=list(range(1, V + 1))).to(dev)
    ci = CandidateIndex(k=K, ids=torch.arange(1, V + 1), top_k_module=MIPSBruteForceTopK()).to(dev)
    metrics = RetrievalMetrics(k=K, at_k_list=[1, 5, 10, 20])
    runner = RetrievalRunner(emb, pre, enc, post, DotProductSimilarity(), sampler, ci,
                             SampledSoftmaxLoss(R, T), metrics, gr_output_length=OUT_LEN)
    return runner


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    lengths = torch.randint(5, N0 + 1, (B,), generator=g)
    lengths[0] = N0  # one full-length row
    ids = torch.zeros(B, N0, dtype=torch.int64)
    ts = torch.zeros(B, N0, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ids[b, :L] = torch.randint(1, V + 1, (L,), generator=g)
        ts[b, :L] = 1_000_000_000 + torch.cumsum(torch.randint(1, 200_000, (L,), generator=g), 0)
    return {
        "history_lengths": lengths, "historical_ids": ids,
        "historical_ratings": torch.randint(1, 6, (B, N0), generator=g),
        "historical_timestamps": ts, "historical_years": torch.zeros(B, N0, dtype=torch.int64),
        "target_ids": torch.randint(1, V + 1, (B,), generator=g),
        "target_ratings": torch.randint(1, 6, (B,), generator=g),
        "target_timestamps": ts.max(1).values + 1000,
        "target_years": torch.zeros(B, dtype=torch.int64),
    }


def _cpu_forward(runner, batch, scatter_target: bool):
    """The reference sequence on CPU (fp32 torch autograd over the oracle HSTU)."""
    N = N0 + OUT_LEN + 1
    emb, pre, enc = runner.embeddings, runner.preprocessor, runner.sequence_encoder
    w_item = emb._item_emb.weight.detach().cpu().clone().requires_grad_(True)
    w_year = emb._year_emb.weight.detach().cpu().clone().requires_grad_(True)
    pos_w = pre._pos_emb.weight.detach().cpu().clone().requires_grad_(True)
    st = {k: v.detach().cpu().clone().requires_grad_(True)
          for k, v in enc.state_dict().items() if k != "_attn_mask"}
    layers = [O.layer_params_from_state(st, i) for i in range(BLOCKS)]
    lengths = batch["history_lengths"]
    pad = OUT_LEN + 1
    ids = torch.cat([batch["historical_ids"], torch.zeros(B, pad, dtype=torch.int64)], 1)
    ts = torch.cat([batch["historical_timestamps"], torch.zeros(B, pad, dtype=torch.int64)], 1)
    ts.scatter_(1, lengths.view(-1, 1), batch["target_timestamps"].view(-1, 1))
    if scatter_target:
        ids.scatter_(1, lengths.view(-1, 1), batch["target_ids"].view(-1, 1))
    year_tab = emb.year_lookup_table.cpu()
    yid = year_tab[ids.clamp(0, year_tab.numel() - 1)]
    x_emb = torch.cat([F.embedding(ids, w_item, padding_idx=0),
                       F.embedding(yid, w_year, padding_idx=0)], -1)
    u = (x_emb * D ** 0.5 + pos_w[:N][None]) * (ids != 0)[..., None].float()
    cfg = O.HSTUConfig(N=N, D=D, H=1, dqk=D, dv=D)
    thr = np.asarray(__import__("mygenerativerecommenders_amd.bucket_table",
                                fromlist=["x"]).BUCKET_THRESHOLDS)
    y = O.hstu_forward(lengths, u, ts, cfg, layers, thr)
    y = y / y.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    leaves = {"emb._item_emb.weight": w_item, "emb._year_emb.weight": w_year,
              "pre._pos_emb.weight": pos_w, **{"enc." + k: v for k, v in st.items()}}
    return ids, x_emb, y, leaves


def _jag(x, lengths):
    return torch.cat([x[b, :int(lengths[b])] for b in range(x.shape[0])], 0)


def test_runner_training_step_matches_reference_sequence():
    dev = torch.device("cuda")
    runner = _modules(dev)
    batch = _batch(3)
    drawn = []
    real = runner.negatives_sampler.sample_offsets

    def record(pos_ids, n):
        o = real(pos_ids, n)
        drawn.append(o.detach().cpu())
        return o
    runner.negatives_sampler.sample_offsets = record
    loss = runner.training_step(batch)
    torch.cuda.synchronize()
    assert len(drawn) == 1

    ids, x_emb, y, leaves = _cpu_forward(runner, batch, scatter_target=True)
    lengths = batch["history_lengths"]
    sup_ids = _jag(ids[:, 1:], lengths)
    out = _jag(y[:, :-1], lengths)
    sup = _jag(x_emb[:, 1:], lengths)
    w = (sup_ids != 0).float()
    offs = drawn[0]
    assert offs.shape == (sup_ids.numel(), R)
    # the supervision shift: row b's last supervised id is the scattered target
    last = torch.cumsum(lengths, 0) - 1
    assert torch.equal(sup_ids[last], batch["target_ids"])
    # loss in torch (autograd to the leaves), pinned to loss_oracle's float64 value
    all_ids = torch.arange(1, V + 1)
    tab = torch.cat([F.embedding(all_ids, leaves["emb._item_emb.weight"], padding_idx=0),
                     F.embedding(emb_year(runner, all_ids), leaves["emb._year_emb.weight"],
                                 padding_idx=0)], -1)
    tab_n = tab / tab.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    pos_n = sup / sup.norm(dim=-1, keepdim=True).clamp_min(1e-6)
    pos_logit = (out * pos_n).sum(-1) / T
    neg_logit = torch.einsum("mrd,md->mr", tab_n[offs], out) / T
    neg_logit = torch.where(all_ids[offs] == sup_ids[:, None],
                            torch.full_like(neg_logit, loss_oracle.COLLISION_LOGIT), neg_logit)
    lse = torch.logsumexp(torch.cat([pos_logit[:, None], neg_logit], 1), 1)
    ref_loss = ((lse - pos_logit) * w).sum() / w.sum()
    ref64 = loss_oracle.sampled_softmax(out.detach().numpy(), sup_ids.numpy(),
                                        sup.detach().numpy(), w.numpy(), tab.detach().numpy(),
                                        all_ids.numpy(), offs.numpy(), T, grads=False)["loss"]
    assert abs(ref_loss.item() - float(ref64)) <= 1e-5 * (1 + abs(float(ref64)))
    assert abs(loss.item() - ref_loss.item()) <= 1e-4 * (1 + abs(ref_loss.item())), \
        (loss.item(), ref_loss.item())
    ref_loss.backward()
    named = {"emb." + n: p for n, p in runner.embeddings.named_parameters()}
    named.update({"pre." + n: p for n, p in runner.preprocessor.named_parameters()})
    named.update({"enc." + n: p for n, p in runner.sequence_encoder.named_parameters()})
    for name, p in named.items():
        ref = leaves[name].grad
        got = p.grad.detach().cpu()
        err = (got - ref).abs().max().item() / (1 + ref.abs().max().item())
        assert err <= 2e-4, (name, err)


def emb_year(runner, ids):
    tab = runner.embeddings.year_lookup_table.cpu()
    return tab[ids.clamp(0, tab.numel() - 1)]


def test_runner_validation_epoch_matches_oracle_topk_and_metrics():
    dev = torch.device("cuda")
    runner = _modules(dev)
    runner.sequence_encoder.eval()
    runner.preprocessor.eval()
    batches = [_batch(5), _batch(6)]
    runner.on_validation_epoch_start()
    got_ids = []
    for bt in batches:
        ids, scores = runner.validation_step(bt)
        got_ids.append(ids.cpu())
    res = runner.on_validation_epoch_end()
    # CPU: the same sequence (no target scatter), exact top-k over the normalised table
    # from the GPU's own query rows (bit-exact selection), queries checked to tolerance
    with torch.no_grad():
        emb = runner.embeddings
        all_ids = torch.arange(1, V + 1, device=dev)
        table = runner.negatives_sampler.normalize_embeddings(emb.get_item_embeddings(all_ids))
        E = table.cpu().numpy().astype(np.float32)
    tops, targets = [], []
    for bt, gids in zip(batches, got_ids):
        ids, _, y, _ = _cpu_forward(runner, bt, scatter_target=False)
        lengths = bt["history_lengths"]
        q_ref = y.detach()[torch.arange(B), lengths - 1]
        from mygenerativerecommenders_amd.runner import seq_features_from_row
        with torch.inference_mode():
            feats, _, _ = seq_features_from_row(bt, dev, OUT_LEN + 1)
            feats = feats._replace(past_embeddings=emb.get_item_embeddings(feats.past_ids))
            yg, _ = runner.forward(feats)
            from mygenerativerecommenders_amd import ops
            q = ops.get_current_embeddings(feats.past_lengths, yg).cpu()
        assert (q - q_ref).abs().max().item() <= 2e-4
        inv = feats.past_ids.cpu().numpy()
        _, want, _ = topk_oracle.mips_topk(q.numpy().astype(np.float32), E,
                                           np.arange(1, V + 1, dtype=np.int64), inv, K)
        assert np.array_equal(gids.numpy(), want)
        tops.append(want)
        targets.append(bt["target_ids"].numpy())
    ref = metrics_oracle.retrieval_metrics(np.concatenate(tops), np.concatenate(targets),
                                           [1, 5, 10, 20])
    for k, v in ref.items():
        assert abs(float(res[k]) - v) <= 1e-6, (k, float(res[k]), v)
