"""C5 rehearsal on one GPU: two processes, both on cuda:0, gloo over 127.0.0.1, train the
real drop-in HSTU module (HIP kernels) with the bucketed, backward-overlapped gradient
reducer and the reference's Muon + AdamW split.  The kernels are deterministic, so two
ranks x B/2 must equal -- bit for bit -- one process that averages the same two
half-batch gradients as 0.5 g0 + 0.5 g1, through two optimizer steps; and equal the
whole-batch gradient within fp32 summation tolerance."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(dev):
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    N0, out_len, D, blocks = 200, 11, 64, 3
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.0, attn_dropout_rate=0.0).to(dev)
    g = torch.Generator().manual_seed(1)
    B, N = 8, N0 + out_len
    lengths = torch.randint(30, N0 + 1, (B,), generator=g)
    x = torch.randn(2, B, N, D, generator=g)
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(2, B, N, D, generator=g)
    return enc, lengths.to(dev), x.to(dev), ts.to(dev), dy.to(dev)


def _loss(enc, lengths, x, ts, dy):
    y, _ = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
               past_payloads={"timestamps": ts})
    return (y * dy).sum() / x.shape[0]


def _train(enc, lengths, x, ts, dy, rows=None, halves=None, reducer=None):
    from mygenerativerecommenders_amd.distributed import muon_adamw_split
    opts = muon_adamw_split(enc.named_parameters())
    grads = []
    for step in range(2):
        for p in enc.parameters():
            p.grad = None
        if halves is None:
            _loss(enc, lengths[rows], x[step][rows], ts[rows], dy[step][rows]).backward()
        else:
            parts = []
            for h in halves:
                for p in enc.parameters():
                    p.grad = None
                _loss(enc, lengths[h], x[step][h], ts[h], dy[step][h]).backward()
                parts.append([p.grad.clone() for p in enc.parameters()])
            for p, g0, g1 in zip(enc.parameters(), *parts):
                p.grad = torch.mul(g0, 0.5) + torch.mul(g1, 0.5)
        if reducer is not None:
            reducer.finish()
        grads.append([p.grad.clone() for p in enc.parameters()])
        for o in opts:
            o.step()
    torch.cuda.synchronize()
    return grads, [p.detach().clone() for p in enc.parameters()]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        from mygenerativerecommenders_amd.distributed import BucketedGradReducer, init_from_env
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        init_from_env("gloo")
        enc, lengths, x, ts, dy = _case(dev)
        B = lengths.numel()
        halves = [slice(r * B // world, (r + 1) * B // world) for r in range(world)]
        full, _ = _train(copy.deepcopy(enc), lengths, x, ts, dy, rows=slice(0, B))
        ref_g, ref_p = _train(copy.deepcopy(enc), lengths, x, ts, dy, halves=halves)
        red = BucketedGradReducer(list(enc.parameters()), bucket_bytes=64 << 10, overlap=True)
        assert len(red.buckets) >= 3
        got_g, got_p = _train(enc, lengths, x, ts, dy, rows=halves[rank], reducer=red)
        for g, r in zip(got_g[0], full[0]):
            assert torch.allclose(g, r, rtol=2e-4, atol=1e-5 * (1 + r.abs().max().item())), \
                (g - r).abs().max().item()
        for step in range(2):
            for g, r in zip(got_g[step], ref_g[step]):
                assert torch.equal(g, r), (step, (g - r).abs().max().item())
        for p, r in zip(got_p, ref_p):
            assert torch.equal(p, r), (p - r).abs().max().item()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))


def test_c5_dp_hstu_two_ranks_one_gpu_bitexact():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}: {msg}"


# ------------------------------------------------------------------ C5 width with tables
def _c5_case(dev):
    """C5 geometry: D = 256, N0 = 2048 (N = 2059), h = 1, d = 256, at 2
    blocks and a small batch; LocalEmbeddingModule with the ml-20m-sized item and year
    tables (131,262 items, 128-wide halves) and a synthetic item -> year map."""
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    from mygenerativerecommenders_amd.hstu import HSTU
    torch.manual_seed(0)
    N0, out_len, D, blocks, V = 2048, 11, 256, 2, 131_262
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
               item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
               attention_dim=D, normalization="rel_bias", linear_config="uvqk",
               linear_activation="silu", linear_dropout_rate=0.0, attn_dropout_rate=0.0).to(dev)
    emb = LocalEmbeddingModule(V, D, item2year={i: 1919 + (i * 7919) % 97
                                                for i in range(1, V + 1)}).to(dev)
    g = torch.Generator().manual_seed(3)
    B, N = 4, N0 + out_len
    lengths = torch.tensor([2048, 1500, 700, 2048])
    pos = torch.arange(N)[None, :]
    ids = torch.randint(1, V + 1, (2, B, N), generator=g)
    ids = torch.where(pos < lengths[:, None], ids, torch.zeros_like(ids))
    ts = torch.zeros(B, N, dtype=torch.int64)
    for b in range(B):
        L = int(lengths[b])
        ts[b, :L + 1] = 1_000_000_000 + torch.cumsum((torch.rand(L + 1, generator=g) * 2e5).long(), 0)
    dy = torch.randn(2, B, N, D, generator=g)
    return enc, emb, lengths.to(dev), ids.to(dev), ts.to(dev), dy.to(dev)


def _c5_loss(enc, emb, lengths, ids, ts, dy):
    x = emb.get_item_embeddings(ids) * (enc._embedding_dim ** 0.5)
    y, _ = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
               past_payloads={"timestamps": ts})
    return (y * dy).sum() / ids.shape[0]


def _c5_train(enc, emb, case, rows=None, halves=None, reducer=None):
    from mygenerativerecommenders_amd.distributed import muon_adamw_split
    lengths, ids, ts, dy = case
    named = list(emb.named_parameters(prefix="_embedding_module")) + list(enc.named_parameters())
    params = [p for _, p in named]
    opts = muon_adamw_split(named)
    grads = []
    for step in range(2):
        for p in params:
            p.grad = None
        if halves is None:
            _c5_loss(enc, emb, lengths[rows], ids[step][rows], ts[rows], dy[step][rows]).backward()
        else:
            parts = []
            for h in halves:
                for p in params:
                    p.grad = None
                _c5_loss(enc, emb, lengths[h], ids[step][h], ts[h], dy[step][h]).backward()
                parts.append([p.grad.clone() for p in params])
            for p, g0, g1 in zip(params, *parts):
                p.grad = torch.mul(g0, 0.5) + torch.mul(g1, 0.5)
        if reducer is not None:
            reducer.finish()
        grads.append([p.grad.clone() for p in params])
        for o in opts:
            o.step()
    torch.cuda.synchronize()
    return grads, [p.detach().clone() for p in params]


def _c5_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        from mygenerativerecommenders_amd import _lib
        from mygenerativerecommenders_amd.distributed import BucketedGradReducer, init_from_env
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        init_from_env("gloo")
        # the item-table backward's fixed-order form (its default uses fp32 atomics)
        _lib.set_option("DETERMINISTIC", 1)
        enc, emb, lengths, ids, ts, dy = _c5_case(dev)
        case = (lengths, ids, ts, dy)
        B = lengths.numel()
        halves = [slice(r * B // world, (r + 1) * B // world) for r in range(world)]
        full_g, _ = _c5_train(copy.deepcopy(enc), copy.deepcopy(emb), case, rows=slice(0, B))
        ref_g, ref_p = _c5_train(copy.deepcopy(enc), copy.deepcopy(emb), case, halves=halves)
        params = list(emb.parameters()) + list(enc.parameters())
        support = emb.grad_row_support()
        assert support[emb._year_emb.weight].numel() == 97
        # 1 MB buckets: the encoder's 2.7 MB split over several, the 67 MB item table
        # one of its own; launched in order while the backward still runs
        red = BucketedGradReducer(params, bucket_bytes=1 << 20, overlap=True,
                                  row_support=support)
        assert len(red.buckets) >= 4 and red.buckets[-1] == [emb._item_emb.weight]
        got_g, got_p = _c5_train(enc, emb, case, rows=halves[rank], reducer=red)
        # 2 ranks x B/2 == 1 process x B within fp32 summation tolerance, tables included
        for g, r in zip(got_g[0], full_g[0]):
            assert torch.allclose(g, r, rtol=2e-4, atol=1e-5 * (1 + r.abs().max().item())), \
                (g - r).abs().max().item()
        yg = got_g[0][1]  # the year table: gradient only on the mapped rows
        nz = (yg.abs().sum(1) > 0).nonzero().reshape(-1)
        assert nz.numel() > 0 and set(nz.tolist()) <= set(support[emb._year_emb.weight].tolist())
        # bit-identical to 0.5 g0 + 0.5 g1 in one process, through two optimizer steps
        for step in range(2):
            for g, r in zip(got_g[step], ref_g[step]):
                assert torch.equal(g, r), (step, (g - r).abs().max().item())
        for p, r in zip(got_p, ref_p):
            assert torch.equal(p, r), (p - r).abs().max().item()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))


def test_c5_width_tables_two_ranks_one_gpu_bitexact():
    """C5 (D = 256, N0 = 2048, item + year tables, row-support bucketed
    reducer overlapping the backward, Muon + AdamW) on the GPU with two ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}: {msg}"
