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
