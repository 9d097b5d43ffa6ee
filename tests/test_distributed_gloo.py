"""CPU, world_size 2 over gloo: the data-parallel gradient exchange and the
row-sharded retrieval merge (the N > 1 paths of bench.py), with the C oracle standing
in for the device top-k kernel on each shard."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np_merge(cand_scores, cand_index, cand_ids, k):
    """Test-side canonical merge (score desc, index asc) of (P, B, k_in) lists."""
    P, B, K = cand_scores.shape
    out_s = torch.full((B, k), float("-inf"))
    out_i = torch.full((B, k), -1, dtype=torch.int64)
    for b in range(B):
        s = cand_scores[:, b].reshape(-1).numpy()
        x = cand_index[:, b].reshape(-1).numpy()
        d = cand_ids[:, b].reshape(-1).numpy()
        keep = x >= 0
        order = np.lexsort((x[keep], -s[keep]))[:k]
        out_s[b, :len(order)] = torch.from_numpy(s[keep][order])
        out_i[b, :len(order)] = torch.from_numpy(d[keep][order])
    return out_s, out_i


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from mygenerativerecommenders_amd.distributed import (FlatGradAllReducer,
                                                              gather_and_merge,
                                                              init_from_env, shard_bounds)
        from oracle import topk_oracle
        r, w, _ = init_from_env("gloo")
        assert (r, w) == (rank, world)
        # ---- gradient averaging
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
        red = FlatGradAllReducer(list(model.parameters()), bucket_bytes=64)
        x = torch.randn(4, 7) * (rank + 1)
        model(x).sum().backward()
        local = [p.grad.clone() for p in model.parameters()]
        allg = [[torch.empty_like(g) for _ in range(world)] for g in local]
        for g, lst in zip(local, allg):
            dist.all_gather(lst, g)
        red.allreduce(world)
        for p, lst in zip(model.parameters(), allg):
            assert torch.allclose(p.grad, sum(lst) / world, atol=1e-6)
        before = [p.grad for p in model.parameters()]
        red.allreduce(world, inplace=True)  # averaging an average is idempotent
        for p, b in zip(model.parameters(), before):
            assert p.grad.data_ptr() == b.data_ptr()
        # ---- row-sharded retrieval
        g = np.random.default_rng(5)
        X, D, B, k, N0 = 1001, 8, 6, 20, 9
        E = g.standard_normal((X, D), dtype=np.float32)
        Q = g.standard_normal((B, D), dtype=np.float32)
        ids = np.arange(1, X + 1, dtype=np.int64)
        inv = g.integers(1, X + 1, (B, N0)).astype(np.int64)
        a, b = shard_bounds(X, world, rank)
        s, i, x_local = topk_oracle.mips_topk(Q, E[a:b], ids[a:b], inv, k)
        x_glob = np.where(x_local >= 0, x_local + a, -1)
        mi, ms = gather_and_merge(torch.from_numpy(s), torch.from_numpy(i),
                                  torch.from_numpy(x_glob), k, merge_fn=_np_merge)
        rs, ri, _ = topk_oracle.mips_topk(Q, E, ids, inv, k)
        assert np.array_equal(mi.numpy(), ri)
        assert np.array_equal(ms.numpy(), rs)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_dp_allreduce_and_sharded_merge_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}: {msg}"


# ---------------------------------------------------------------- C5: DP HSTU training
# The HSTU module's own parameters (same names and shapes as the drop-in), run forward on
# the CPU through the oracle's functional restatement; the bucketed, backward-overlapped
# reducer averages them over 2 gloo ranks each holding half the batch, Muon + AdamW
# step (the reference's two-optimizer split).  Must equal one process on the whole batch.

def _hstu_case():
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    N0, out_len, D, blocks = 16, 3, 16, 2
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.0, attn_dropout_rate=0.0)
    with torch.no_grad():
        for layer in enc._hstu._attention_layers:
            layer._rel_attn_bias._ts_w.normal_(0, 0.3)
            layer._rel_attn_bias._pos_w.normal_(0, 0.3)
    g = torch.Generator().manual_seed(1)
    B, N = 4, N0 + out_len
    lengths = torch.tensor([16, 5, 11, 9])
    x = torch.randn(2, B, N, D, generator=g)  # two steps
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(2, B, N, D, generator=g)
    return enc, lengths, x, ts, dy, blocks


def _hstu_loss(enc, blocks, lengths, x, ts, dy):
    import numpy as np
    from mygenerativerecommenders_amd.bucket_table import BUCKET_THRESHOLDS
    from oracle import hstu_oracle as O
    st = dict(enc.named_parameters())
    layers = [O.layer_params_from_state(st, i) for i in range(blocks)]
    N, D = x.shape[1], x.shape[2]
    cfg = O.HSTUConfig(N=N, D=D, H=1, dqk=D, dv=D)
    y = O.hstu_forward(lengths, x, ts, cfg, layers, np.asarray(BUCKET_THRESHOLDS))
    return (y * dy).sum() / x.shape[0]  # mean over this rank's sequences


def _hstu_train(enc, blocks, lengths, x, ts, dy, rows, reducer=None, halves=None):
    """Two optimizer steps.  ``halves``: single-process reference that averages the two
    half-batch gradients as 0.5 g0 + 0.5 g1 -- the same arithmetic as the reducer's
    scaled copy + 2-rank sum, so the whole run (Muon's bf16 Newton-Schulz included,
    which amplifies last-bit differences) must match bit for bit."""
    from mygenerativerecommenders_amd.distributed import muon_adamw_split
    opts = muon_adamw_split(enc.named_parameters())
    grads = []
    for step in range(2):
        if reducer is not None:
            reducer.zero_grad()
        else:
            for p in enc.parameters():
                p.grad = None
        if halves is None:
            loss = _hstu_loss(enc, blocks, lengths[rows], x[step][rows], ts[rows], dy[step][rows])
            loss.backward()
        else:
            parts = []
            for h in halves:
                for p in enc.parameters():
                    p.grad = None
                _hstu_loss(enc, blocks, lengths[h], x[step][h], ts[h], dy[step][h]).backward()
                parts.append([p.grad.clone() for p in enc.parameters()])
            for p, g0, g1 in zip(enc.parameters(), *parts):
                p.grad = torch.mul(g0, 0.5) + torch.mul(g1, 0.5)
        if reducer is not None:
            reducer.finish()
        grads.append([p.grad.clone() for p in enc.parameters()])
        for o in opts:
            o.step()
    return grads, [p.detach().clone() for p in enc.parameters()]


def _dp_hstu_worker(rank, world, port, q, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from mygenerativerecommenders_amd.distributed import BucketedGradReducer, init_from_env
        init_from_env("gloo")
        enc, lengths, x, ts, dy, blocks = _hstu_case()
        B = lengths.numel()
        copy = __import__("copy")
        half = B // world
        halves = [slice(r * half, (r + 1) * half) for r in range(world)]
        full_grads, _ = _hstu_train(copy.deepcopy(enc), blocks, lengths, x, ts, dy, slice(0, B))
        ref_grads, ref_params = _hstu_train(copy.deepcopy(enc), blocks, lengths, x, ts, dy, None,
                                            halves=halves)
        red = BucketedGradReducer(list(enc.parameters()), bucket_bytes=4096, overlap=overlap)
        assert len(red.buckets) > 2  # several buckets, last block's parameters first
        assert red.buckets[0][0] is list(enc.parameters())[-1]
        grads, params = _hstu_train(enc, blocks, lengths, x, ts, dy, halves[rank], red)
        # 2 ranks x B/2 == 1 process x B (first step, fp32 summation-order tolerance)
        for g, r in zip(grads[0], full_grads[0]):
            assert torch.allclose(g, r, rtol=1e-5, atol=1e-6), (g - r).abs().max()
        # ... and bit-identical to the same averaging done in one process, through two
        # Muon + AdamW steps
        for step in range(2):
            for g, r in zip(grads[step], ref_grads[step]):
                assert torch.equal(g, r), (step, (g - r).abs().max())
        for p, r in zip(params, ref_params):
            assert torch.equal(p, r), (p - r).abs().max()
        # .grad are views into the reducer's buckets (no copy back)
        bufs = [(b.data_ptr(), b.data_ptr() + 4 * b.numel()) for b in red.buffers]
        for p in enc.parameters():
            assert any(lo <= p.grad.data_ptr() < hi for lo, hi in bufs)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


import pytest  # noqa: E402


@pytest.mark.parametrize("overlap", [True, False])
def test_dp_hstu_bucketed_overlap_world2_equals_full_batch(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_hstu_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}: {msg}"


# ---------------------------------------------------------------- C5 with item tables
# LocalEmbeddingModule's two (num_items + 1, D/2) tables join the exchange (reference DDP
# all-reduces every parameter, configs/trainer/ddp.yaml).  The year table goes through
# the reducer's row_support (only the rows the item -> year map can reach travel).  The
# table gathers run test-side with torch ops on the CPU (the module's own gather is a
# HIP kernel); a second gather of random "negative" rows touches most item rows.

def _tables_case():
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    enc, lengths, x, ts, dy, blocks = _hstu_case()
    V, D = 97, x.shape[-1]
    torch.manual_seed(3)
    item2year = {i: 1990 + (i % 7) for i in range(1, V + 1)}  # years index the year table
    emb = LocalEmbeddingModule(2100, D, item2year=item2year)
    g = torch.Generator().manual_seed(4)
    B, N = x.shape[1], x.shape[2]
    ids = torch.randint(1, V + 1, (2, B, N), generator=g)
    ids[:, :, -2:] = 0  # padding ids: no table gradient (padding_idx 0)
    neg = torch.randint(0, V + 1, (2, B, 64), generator=g)
    wneg = torch.randn(2, B, 64, D // 2, generator=g)
    return enc, emb, lengths, ids, neg, wneg, ts, dy, blocks


def _tables_loss(enc, emb, blocks, lengths, ids, neg, wneg, ts, dy, x_noise):
    item_w, year_w = emb._item_emb.weight, emb._year_emb.weight
    yid = emb.year_lookup_table[ids.clamp(0, emb.year_lookup_table.numel() - 1)]
    xe = torch.cat([torch.nn.functional.embedding(ids, item_w, padding_idx=0),
                    torch.nn.functional.embedding(yid, year_w, padding_idx=0)], -1)
    loss = _hstu_loss(enc, blocks, lengths, xe + x_noise, ts, dy)
    negs = torch.nn.functional.embedding(neg, item_w, padding_idx=0)
    return loss + (negs * wneg).sum() / ids.shape[0]


def _tables_train(enc, emb, blocks, case, rows, reducer=None, halves=None):
    from mygenerativerecommenders_amd.distributed import muon_adamw_split
    lengths, ids, neg, wneg, ts, dy, x_noise = case
    named = list(emb.named_parameters(prefix="_embedding_module")) + list(enc.named_parameters())
    params = [p for _, p in named]
    opts = muon_adamw_split(named)
    grads = []
    for step in range(2):
        for p in params:
            p.grad = None
        if halves is None:
            _tables_loss(enc, emb, blocks, lengths[rows], ids[step][rows], neg[step][rows],
                         wneg[step][rows], ts[rows], dy[step][rows], x_noise[step][rows]).backward()
        else:
            parts = []
            for h in halves:
                for p in params:
                    p.grad = None
                _tables_loss(enc, emb, blocks, lengths[h], ids[step][h], neg[step][h],
                             wneg[step][h], ts[h], dy[step][h], x_noise[step][h]).backward()
                parts.append([p.grad.clone() for p in params])
            for p, g0, g1 in zip(params, *parts):
                p.grad = torch.mul(g0, 0.5) + torch.mul(g1, 0.5)
        if reducer is not None:
            reducer.finish()
        grads.append([p.grad.clone() for p in params])
        for o in opts:
            o.step()
    return grads, [p.detach().clone() for p in params]


def _dp_tables_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import copy
        from mygenerativerecommenders_amd.distributed import BucketedGradReducer, init_from_env
        init_from_env("gloo")
        enc, emb, lengths, ids, neg, wneg, ts, dy, blocks = _tables_case()
        x_noise = torch.randn(2, *ids.shape[1:], enc._embedding_dim,
                              generator=torch.Generator().manual_seed(9)) * 0.01
        case = (lengths, ids, neg, wneg, ts, dy, x_noise)
        B = lengths.numel()
        halves = [slice(r * B // world, (r + 1) * B // world) for r in range(world)]
        full_g, _ = _tables_train(copy.deepcopy(enc), copy.deepcopy(emb), blocks, case, slice(0, B))
        ref_g, ref_p = _tables_train(copy.deepcopy(enc), copy.deepcopy(emb), blocks, case, None,
                                     halves=halves)
        params = list(emb.parameters()) + list(enc.parameters())
        support = emb.grad_row_support()
        yrows = support[emb._year_emb.weight]
        assert yrows.tolist() == list(range(1990, 1997))
        red = BucketedGradReducer(params, bucket_bytes=16 << 10, overlap=True,
                                  row_support=support)
        dense_bytes = 4 * sum(p.numel() for p in params)
        assert red.exchange_bytes == dense_bytes - 4 * (emb._year_emb.weight.numel()
                                                        - yrows.numel() * emb._year_emb.weight.shape[1])
        got_g, got_p = _tables_train(enc, emb, blocks, case, halves[rank], red)
        # 2 ranks x B/2 == 1 process x B, tables included (fp32 summation tolerance)
        for g, r in zip(got_g[0], full_g[0]):
            assert torch.allclose(g, r, rtol=1e-5, atol=1e-6), (g - r).abs().max()
        # the item table gradient touches most rows; the year table only the mapped years
        assert (got_g[0][0].abs().sum(1) > 0).sum() > 80
        ynz = (got_g[0][1].abs().sum(1) > 0).nonzero().reshape(-1)
        assert set(ynz.tolist()) <= set(yrows.tolist()) and ynz.numel() > 0
        # bit-identical to the same 0.5 g0 + 0.5 g1 averaging in one process, 2 steps
        for step in range(2):
            for g, r in zip(got_g[step], ref_g[step]):
                assert torch.equal(g, r), (step, (g - r).abs().max())
        for p, r in zip(got_p, ref_p):
            assert torch.equal(p, r), (p - r).abs().max()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def _spawn(target, world=2, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=timeout) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}: {msg}"


def test_dp_with_item_tables_world2_equals_full_batch():
    _spawn(_dp_tables_worker)


def _unused_worker(rank, world, port, q):
    """A parameter that only rank 0 uses sits in the FIRST bucket; on rank 1 the later
    buckets complete first.  Launching in bucket order keeps the collectives paired;
    find_unused_parameters leaves a parameter no rank used at grad None."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from mygenerativerecommenders_amd.distributed import BucketedGradReducer, init_from_env
        init_from_env("gloo")
        torch.manual_seed(0)
        a = torch.nn.Parameter(torch.randn(6, 5))
        b = torch.nn.Parameter(torch.randn(5, 4))
        c = torch.nn.Parameter(torch.randn(40))   # used by rank 0 only
        never = torch.nn.Parameter(torch.randn(3))
        for find_unused in (True, False):
            red = BucketedGradReducer([a, b, never, c], bucket_bytes=64, overlap=True,
                                      find_unused_parameters=find_unused)
            assert red.buckets[0] == [c]
            x = torch.randn(3, 6, generator=torch.Generator().manual_seed(rank))
            red.zero_grad()
            loss = (x @ a @ b).square().sum()
            if rank == 0:
                loss = loss + c.sin().sum()
            loss.backward()
            red.finish()
            ga = [torch.empty_like(a) for _ in range(world)]
            xa = (x @ a @ b)
            ref_a = torch.autograd.grad(xa.square().sum(), a)[0]
            dist.all_gather(ga, ref_a)
            assert torch.allclose(a.grad, sum(ga) / world, atol=1e-5)
            assert torch.allclose(c.grad, c.detach().cos() / world, atol=1e-6)
            if find_unused:
                assert never.grad is None
            else:
                assert torch.equal(never.grad, torch.zeros(3))
            red.remove_hooks()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_bucket_order_with_rank_dependent_unused_parameter_world2():
    _spawn(_unused_worker, timeout=120)
