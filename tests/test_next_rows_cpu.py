"""CPU: the §8 "next" rows whose host logic runs anywhere —
N3 RetrievalMetrics (metrics/retrieval.py:40-68) against the oracle restatement, with a
2-rank gloo all-gather of uneven shards; N4 Muon (optimizers/muon.py:3-86) against two
steps recorded from the reference (tests/golden/muon.npz).  Tolerances: metrics 1e-6;
Muon parameters 2e-3 of the step size (bf16 Newton-Schulz)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import metrics_oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
AT_K = [10, 50, 100, 200]


def _case(B, k, seed, n_items=4000):
    g = torch.Generator().manual_seed(seed)
    top = torch.stack([torch.randperm(n_items, generator=g)[:k] + 1 for _ in range(B)])
    tgt = torch.randint(1, n_items + 1, (B,), generator=g)
    # force hits at chosen ranks (incl. rank 1 and rank k) and leave the rest to chance
    for b in range(0, B, 3):
        top[b, (b * 7) % k] = tgt[b]
    return top, tgt


def test_metrics_match_oracle():
    from mygenerativerecommenders_amd.metrics import RetrievalMetrics
    m = RetrievalMetrics(k=200, at_k_list=AT_K)
    tops, tgts = [], []
    for s in range(3):
        top, tgt = _case(50 + s, 200, s)
        m.update(top_k_ids=top, target_ids=tgt.view(-1, 1))
        tops.append(top)
        tgts.append(tgt)
    got = {k: float(v) for k, v in m.compute().items()}
    ref = metrics_oracle.retrieval_metrics(torch.cat(tops).numpy(), torch.cat(tgts).numpy(), AT_K)
    assert set(got) == set(ref)
    for key in ref:
        assert abs(got[key] - ref[key]) < 1e-6, key
    m.reset()
    assert m.top_k_ids == []


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from mygenerativerecommenders_amd.metrics import RetrievalMetrics
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                           world_size=world)
    top, tgt = _case(40, 200, 0)
    sl = slice(0, 17) if rank == 0 else slice(17, 40)  # uneven shards
    m = RetrievalMetrics(k=200, at_k_list=AT_K)
    m.update(top_k_ids=top[sl], target_ids=tgt[sl].view(-1, 1))
    res = {k: float(v) for k, v in m.compute().items()}
    out.put((rank, res))
    dist.destroy_process_group()


def test_metrics_gather_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    top, tgt = _case(40, 200, 0)
    ref = metrics_oracle.retrieval_metrics(top.numpy(), tgt.numpy(), AT_K)
    for r in (0, 1):
        for key in ref:
            assert abs(res[r][key] - ref[key]) < 1e-6, (r, key)


def test_muon_matches_reference_golden():
    from mygenerativerecommenders_amd.muon import Muon
    z = np.load(os.path.join(GOLDEN, "muon.npz"))
    n = len([k for k in z.files if k.startswith("p0_")])
    params = [torch.nn.Parameter(torch.from_numpy(z[f"p0_{i}"]).clone()) for i in range(n)]
    opt = Muon(params, lr=0.02, weight_decay=0.01, momentum=0.95)
    for step in range(2):
        for i, p in enumerate(params):
            p.grad = torch.from_numpy(z[f"g{step}_{i}"]).clone()
        opt.step()
        for i, p in enumerate(params):
            ref = z[f"p{step + 1}_{i}"]
            delta = np.abs(ref - z[f"p{step}_{i}"]).max()
            err = np.abs(p.detach().numpy() - ref).max()
            assert err <= 2e-3 * delta + 1e-7, (step, i, err, delta)
    assert all("momentum_buffer" in opt.state[p] for p in params)


def test_retrieval_metrics_reference_known_answers():
    """Known answers of the reference's own tests/test_metrics.py:36-47 (inputs and
    expected values as data): targets at rank 2, 3 and absent (rank k + 1)."""
    from mygenerativerecommenders_amd.metrics import RetrievalMetrics
    top_k_ids = torch.tensor([[1, 2, 3], [4, 5, 6], [7, 8, 9]])
    target_ids = torch.tensor([[2], [6], [3]])
    m = RetrievalMetrics(k=3, at_k_list=[1, 2, 3])
    assert m.k == 3 and m.at_k_list == [1, 2, 3]
    m.update(top_k_ids, target_ids)
    m.update(top_k_ids, target_ids)
    assert len(m.top_k_ids) == 2 and len(m.target_ids) == 2
    m.reset()
    assert m.top_k_ids == [] and m.target_ids == []
    m.update(top_k_ids, target_ids)
    out = m.compute()
    expect = {"ndcg@1": 0.0, "ndcg@2": 0.2103, "ndcg@3": 0.3770, "hr@1": 0.0,
              "hr@2": 0.3333, "hr@3": 0.6667, "mrr": 0.3611}
    for key, val in expect.items():
        assert abs(float(out[key]) - val) <= 5e-5, (key, float(out[key]), val)
