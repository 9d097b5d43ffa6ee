"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL/xGMI
("nccl" backend on ROCm) or gloo on CPU.

Reference parallelism: Lightning DDP only (configs/trainer/ddp.yaml) —
one fp32 gradient all-reduce per step — and torchmetrics' all-gather of top-k ids.
Here:
  * ``FlatGradAllReducer``: the step's gradients are flattened into ONE contiguous
    fp32 buffer and exchanged with a single all-reduce (ml-1m encoder grads are
    ~250 KB: latency-bound, one collective beats buckets); buckets of
    ``bucket_bytes`` are used when the flat buffer is large (ml-20m scale).
  * ``ShardedCandidateIndex``: the item table is row-sharded (rank r holds rows
    [r*X/P, (r+1)*X/P)); each rank runs the fused local top-k, the (B, k) score /
    index / id lists are all-gathered as one packed (B, k, 20 B) buffer and merged on
    device.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def init_from_env(backend: Optional[str] = None):
    """Initialises the default process group from torchrun's env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


class FlatGradAllReducer:
    """Gradient averaging over the data-parallel group: the step's gradients are
    flattened into ONE contiguous fp32 buffer and exchanged with a single RCCL
    all-reduce (ml-1m encoder grads are ~250 KB: latency-bound, so one collective beats
    buckets; above ``bucket_bytes`` the buffer is split into buckets issued together).
    Gradients stay ordinary tensors (autograd "steals" the backward's outputs, so no
    accumulate kernels run), which keeps the step capturable in a HIP graph."""

    def __init__(self, params: List[torch.nn.Parameter], group=None,
                 bucket_bytes: int = 64 << 20):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.bucket_bytes = bucket_bytes

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def allreduce(self, world: Optional[int] = None, inplace: bool = False):
        """inplace=True copies the averaged gradients back into the existing .grad
        tensors (static buffers of a captured graph) instead of re-pointing .grad."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        world = world or dist.get_world_size(self.group)
        if world == 1:
            return
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        flat = torch.cat([g.reshape(-1) for g in grads])
        max_el = max(1, self.bucket_bytes // 4)
        handles = [dist.all_reduce(flat[s:s + max_el], op=dist.ReduceOp.SUM, group=self.group,
                                   async_op=True) for s in range(0, flat.numel(), max_el)]
        for h in handles:
            h.wait()
        flat.div_(world)
        off = 0
        for p, g in zip(self.params, grads):
            k = g.numel()
            if inplace and p.grad is not None:
                p.grad.copy_(flat[off:off + k].view_as(p))
            else:
                p.grad = flat[off:off + k].view_as(p)
            off += k


class BucketedGradReducer:
    """Data-parallel gradient averaging overlapped with the backward (the MI355X shape
    of Lightning DDP's bucketed all-reduce, configs/trainer/ddp.yaml; SURVEY.md §8e:
    ~147 MB of gradients at C5 must overlap the backward).

    * Parameters are packed into buckets of ``bucket_bytes`` in REVERSE registration
      order -- the order the layer-by-layer backward produces their gradients (last
      block first), so the first bucket completes while earlier blocks still run.
    * Each bucket is one persistent fp32 buffer.  A post-accumulate-grad hook scales the
      fresh gradient by 1/world straight into the parameter's slice of its bucket (one
      kernel, no torch.cat, no copy back) and re-points ``p.grad`` at that slice.
    * Collectives are issued strictly in bucket order on every rank (as DDP does): a
      completed bucket is launched only once every bucket before it has been, so ranks
      whose hooks fire in different orders still pair the same buffers.
      ``overlap=True``: hooks launch the ready prefix during the backward (async; RCCL
      runs it on its own stream).  ``overlap=False``: hooks only pack (e.g. inside a
      captured HIP graph) and ``finish()`` launches every bucket.
    * ``row_support={param: rows}`` (embedding tables): the caller guarantees that the
      gradient of ``param`` is zero outside ``rows`` on every rank -- e.g. the year
      table of ``LocalEmbeddingModule``, whose gradient can only land on the years the
      item -> year map produces (``LocalEmbeddingModule.grad_row_support``).  Only those
      rows travel; the result is identical to the dense exchange.
    * ``finish()`` launches what is left, waits, and writes the averages back where
      needed.  A parameter that got no gradient on this rank contributes zeros.  With
      ``find_unused_parameters=True`` one extra small all-reduce counts, per parameter,
      the ranks that produced a gradient; parameters no rank touched get ``grad = None``
      (as DDP leaves them), so the optimizer skips them.  Without it (DDP's default,
      which would raise on such a parameter) they get a zero gradient.
    ``zero_grad()`` must run before each backward (set_to_none, so the backward's
    output is stolen, not accumulated into the bucket view)."""

    def __init__(self, params: List[torch.nn.Parameter], group=None,
                 bucket_bytes: int = 25 << 20, overlap: bool = True,
                 row_support: Optional[dict] = None, find_unused_parameters: bool = False):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.overlap = overlap
        self.find_unused = find_unused_parameters
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.scale = 1.0 / self.world
        self.rows = {}
        for p, r in (row_support or {}).items():
            if p.dim() < 1:
                raise ValueError("row_support: parameter must have a row dimension")
            r = torch.as_tensor(r, dtype=torch.int64).reshape(-1).unique()  # sorted, unique
            if r.numel() and (int(r[0]) < 0 or int(r[-1]) >= p.shape[0]):
                raise ValueError("row_support: row index outside the parameter")
            self.rows[p] = r.to(p.device)

        def exch_numel(p):
            r = self.rows.get(p)
            return p.numel() if r is None else r.numel() * (p.numel() // max(1, p.shape[0]))

        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            nb = exch_numel(p) * 4
            if cur and size + nb > bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            self.buckets.append(cur)
        self.buffers: List[torch.Tensor] = []
        self.slot = {}
        for bi, bucket in enumerate(self.buckets):
            buf = torch.zeros(sum(exch_numel(p) for p in bucket), dtype=torch.float32,
                              device=bucket[0].device)
            off = 0
            for p in bucket:
                n = exch_numel(p)
                shape = p.shape if p not in self.rows else (self.rows[p].numel(),) + tuple(p.shape[1:])
                self.slot[p] = (bi, buf[off:off + n].view(shape))
                off += n
            self.buffers.append(buf)
        self.index = {p: i for i, p in enumerate(self.params)}
        self.exchange_bytes = sum(4 * b.numel() for b in self.buffers)
        self._reset()
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _reset(self):
        self._ready = [0] * len(self.buckets)
        self._handles: List[Optional[object]] = [None] * len(self.buckets)
        self._next = 0
        self._seen = set()

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def _launch_ready(self, upto_all: bool = False):
        """Launches buckets in index order: the consecutive run of complete buckets from
        the next unlaunched one (every remaining bucket when ``upto_all``)."""
        while self._next < len(self.buckets) and (
                upto_all or self._ready[self._next] == len(self.buckets[self._next])):
            if self.world > 1:
                self._handles[self._next] = dist.all_reduce(
                    self.buffers[self._next], op=dist.ReduceOp.SUM, group=self.group,
                    async_op=True)
            self._next += 1

    def _on_grad(self, p: torch.nn.Parameter):
        bi, view = self.slot[p]
        g = p.grad
        rows = self.rows.get(p)
        if rows is not None:  # only the supported rows travel; p.grad stays dense
            torch.mul(g.index_select(0, rows), self.scale, out=view)
        elif g is not view:
            if self.scale != 1.0:
                torch.mul(g, self.scale, out=view)
            else:
                view.copy_(g)
            p.grad = view
        if p not in self._seen:
            self._seen.add(p)
            self._ready[bi] += 1
            if self.overlap and self._ready[bi] == len(self.buckets[bi]):
                self._launch_ready()

    def finish(self):
        """Completes the step's exchange: after it every .grad is the group average."""
        unseen = [p for p in self.params if p not in self._seen]
        for p in unseen:
            view = self.slot[p][1]
            view.zero_()
            if p not in self.rows:
                p.grad = view
            else:
                p.grad = torch.zeros_like(p)
        self._launch_ready(upto_all=True)
        used = None
        if self.find_unused and self.world > 1:
            used = torch.ones(len(self.params), dtype=torch.float32, device=self.buffers[0].device)
            for p in unseen:
                used[self.index[p]] = 0.0
            dist.all_reduce(used, op=dist.ReduceOp.SUM, group=self.group)
        for h in self._handles:
            if h is not None:
                h.wait()
        if self.world > 1:  # the averaged rows into an otherwise zero dense gradient:
            # rows outside the support are zero by the caller's promise, so a broken
            # promise shows as a gradient that differs from the dense exchange rather than
            # as ranks that silently keep different local rows
            for p, rows in self.rows.items():
                g = torch.zeros_like(p)
                g.index_copy_(0, rows, self.slot[p][1])
                p.grad = g
        if used is not None:
            for p, u in zip(self.params, used.tolist()):
                if u == 0.0:
                    p.grad = None
        elif self.find_unused:
            for p in unseen:
                p.grad = None
        self._reset()

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def muon_adamw_split(named_params, muon_lr=5e-3, muon_momentum=0.95, muon_wd=5e-3,
                     adam_lr=5e-4, adam_betas=(0.8, 0.95), adam_eps=1e-10, adam_wd=5e-3,
                     flat_adam: bool = False, **adam_kwargs):
    """The reference's two-optimizer split (generative_recommenders.py:297-310,
    configs/experiment/ml-1m-hstu-muon.yaml:23-36): parameters whose name contains
    "emb" and every parameter with ndim < 2 -> AdamW; the remaining matrices -> Muon.
    ``named_params``: iterable of (name, parameter).  Returns [AdamW, Muon] (the
    reference's optimizer1, optimizer2), skipping an empty group.  ``flat_adam``: the
    AdamW group as ``optim.FlatAdamW`` (the same update in one launch; ``adam_kwargs``
    such as fused / capturable are then not used)."""
    from .muon import Muon
    named = [(n, p) for n, p in named_params if p.requires_grad]
    adam = [p for n, p in named if "emb" in n or p.ndim < 2]
    ids = {id(p) for p in adam}
    mats = [p for n, p in named if id(p) not in ids]
    opts = []
    if adam and flat_adam:
        from .optim import FlatAdamW
        opts.append(FlatAdamW(adam, lr=adam_lr, betas=adam_betas, eps=adam_eps, weight_decay=adam_wd))
    elif adam:
        opts.append(torch.optim.AdamW(adam, lr=adam_lr, betas=adam_betas, eps=adam_eps,
                                      weight_decay=adam_wd, **adam_kwargs))
    if mats:
        opts.append(Muon(mats, lr=muon_lr, momentum=muon_momentum, weight_decay=muon_wd))
    return opts


class ShardedCandidateIndex:
    """Row-sharded brute-force retrieval.  Each rank owns a contiguous
    slice of the catalog; results are identical to a single-GPU CandidateIndex over
    the whole table (same canonical order: score desc, catalog index asc)."""

    def __init__(self, k: int, ids_shard: torch.Tensor, emb_shard: torch.Tensor,
                 row_offset: int, group=None):
        from .top_k import PackedItems
        self.k = k
        self.ids = ids_shard.to(torch.int64).contiguous()
        self.row_offset = int(row_offset)
        # contiguous ids (the common 1..X catalog): derive ids from the index on device
        start = int(self.ids[0].item()) if self.ids.numel() else 0
        ar = torch.arange(start, start + self.ids.numel(), device=self.ids.device)
        self.arange_base = start if bool(torch.equal(self.ids, ar)) else None
        self.group = group
        self.packed = PackedItems(emb_shard.float().contiguous())

    def local_top_k(self, query_embeddings: torch.Tensor,
                    invalid_ids: Optional[torch.Tensor] = None, k: Optional[int] = None):
        """This rank's (scores, ids, global index) (B, k): no collective, no host sync,
        so it can be captured in a HIP graph."""
        from .top_k import mips_topk
        k = k or self.k
        if self.arange_base is not None:  # global index = id (monotone in the row)
            return mips_topk(query_embeddings, self.packed, k, item_ids=None,
                             invalid_ids=invalid_ids, index_base=self.arange_base,
                             return_index=True)
        return mips_topk(query_embeddings, self.packed, k, item_ids=self.ids,
                         invalid_ids=invalid_ids, index_base=self.row_offset,
                         return_index=True)

    def get_top_k_outputs(self, query_embeddings: torch.Tensor,
                          invalid_ids: Optional[torch.Tensor] = None, k: Optional[int] = None):
        from .top_k import merge_topk
        k = k or self.k
        s, i, x = self.local_top_k(query_embeddings, invalid_ids, k)
        return gather_and_merge(s, i, x, k, self.group, merge_topk)


def gather_and_merge(scores, ids, index, k, group=None, merge_fn=None):
    """All-gathers every rank's (B, k) local top-k (score, id, global catalog index) and
    merges them into the global top-k with the canonical order (score desc, index asc).
    Returns (ids, scores).  ``merge_fn(cand_scores, cand_index, cand_ids, k)`` defaults
    to the device merge kernel (``mips_merge_topk``)."""
    if merge_fn is None:
        from .top_k import merge_topk as merge_fn
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return ids, scores
    P = dist.get_world_size(group)
    B, kk = scores.shape
    # ONE collective: (score f32 | id i64 | index i64) packed as 5 int32 words per entry
    # (20 B x B x k per rank) instead of three all-gathers of 4 + 8 + 8 B
    packed = torch.cat([scores.float().contiguous().view(torch.int32).unsqueeze(-1),
                        ids.to(torch.int64).contiguous().view(torch.int32).view(B, kk, 2),
                        index.to(torch.int64).contiguous().view(torch.int32).view(B, kk, 2)],
                       dim=-1).contiguous()
    out = torch.empty((P,) + tuple(packed.shape), dtype=torch.int32, device=packed.device)
    try:
        dist.all_gather_into_tensor(out, packed, group=group)
    except (RuntimeError, NotImplementedError, AttributeError):  # backends without it
        dist.all_gather(list(out.unbind(0)), packed, group=group)
    gs = out[..., 0].contiguous().view(torch.float32)
    gi = out[..., 1:3].contiguous().view(torch.int64).squeeze(-1)
    gx = out[..., 3:5].contiguous().view(torch.int64).squeeze(-1)
    ms, mi = merge_fn(gs, gx, gi, k)
    return mi, ms


def shard_bounds(X: int, world: int, rank: int):
    a = (X * rank) // world
    b = (X * (rank + 1)) // world
    return a, b
