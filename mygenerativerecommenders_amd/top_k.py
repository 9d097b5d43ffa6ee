"""Top-k modules — drop-in for reference ``models/indexing/top_k.py`` (Hydra
``_target_: ...indexing.top_k.MIPSBruteForceTopK``), running the fused gfx950
scorer + selector of ``libgr_hstu.so`` (``mips_topk``).

Differences from the reference, all deliberate:
  * results are always sorted, with a canonical tie order (score desc, catalog index
    asc) — ``torch.topk`` leaves ties unspecified;
  * the (B, X) logits are never materialised;
  * invalid-id exclusion can be fused (``invalid_ids=``), which
    ``CandidateIndex.get_top_k_outputs`` uses instead of top-(k+N0) + filtering;
  * limits: D <= 256, k <= 4096, N0 <= 8192, X < 2^31 (per shard).  k <= 256 runs
    the fused paths; larger k (the reference CandidateIndex asks for k + N0) runs the
    library's chunked exact path.
"""
from __future__ import annotations

import abc
from typing import Optional, Tuple

import torch

from . import _lib


class TopKModule(torch.nn.Module):
    """top_k.py:21-40."""

    @abc.abstractmethod
    def forward(self, query_embeddings: torch.Tensor, item_embeddings_t: torch.Tensor,
                item_ids: torch.Tensor, k: int, sorted: bool = True
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        pass


class PackedItems:
    """An item table in the MFMA-native blocked layout (``mips_pack_items``)."""

    def __init__(self, items: torch.Tensor):
        _lib.require_gpu(items)
        if items.dim() != 2 or items.dtype != torch.float32:
            raise TypeError("PackedItems: expected a (X, D) float32 tensor")
        items = items.contiguous()
        self.X, self.D = items.shape
        if self.D > 256:
            raise ValueError(f"mips_topk supports D <= 256 (got {self.D})")
        nbytes = _lib.lib().mips_packed_items_bytes(self.X, self.D)
        self.buf = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=items.device)
        _lib.call("mips_pack_items", items.data_ptr(), self.X, self.D, self.buf.data_ptr(),
                  _lib.stream_handle())
        self.device = items.device
        # one grow-only workspace per stream (stream-ordered reuse: calls on one stream
        # never overlap; two streams get two buffers).  A grown buffer's predecessor is
        # kept alive (a captured graph may still point at it); growth at least doubles,
        # so few are ever retired.
        self._ws = {}        # stream handle -> (bytes, workspace)
        self._retired = []
        self._need = {}      # (B, k, N0) -> bytes

    def workspace(self, B: int, k: int, N0: int):
        """(bytes needed, a workspace of at least that many bytes) for a (B, k, N0) call
        on the current stream."""
        key = (B, k, N0)
        n = self._need.get(key)
        if n is None:
            n = topk_workspace_bytes(B, self.X, self.D, k, N0)
            self._need[key] = n
        sk = _lib.stream_handle() or 0
        ent = self._ws.get(sk)
        if ent is None or ent[1].numel() < n:
            if ent is not None:
                self._retired.append(ent[1])
                n_alloc = max(n, 2 * ent[1].numel())
            else:
                n_alloc = n
            ent = (n_alloc, torch.empty(n_alloc, dtype=torch.uint8, device=self.device))
            self._ws[sk] = ent
        return n, ent[1]


K_MAX = 4096
N0_MAX = 8192


def topk_workspace_bytes(B: int, X: int, D: int, k: int, N0: int = 0) -> int:
    """Workspace ``mips_topk`` needs for a (B, D) query batch over X items with N0
    invalid ids per query."""
    return max(int(_lib.lib().mips_topk_workspace_size(B, X, D, k, N0)), 16)


def mips_topk(queries: torch.Tensor, packed: PackedItems, k: int,
              item_ids: Optional[torch.Tensor] = None, invalid_ids: Optional[torch.Tensor] = None,
              index_base: int = 0, return_index: bool = False,
              workspace: Optional[torch.Tensor] = None):
    """Fused brute-force MIPS top-k over a packed table.  Returns (scores (B,k) f32,
    ids (B,k) i64[, global index (B,k) i64]).  ``workspace`` (uint8, at least
    ``topk_workspace_bytes``) may be passed to reuse one buffer across calls; on the
    large-catalog filter path its first int32 is 1 when the exact fallback ran."""
    _lib.require_gpu(queries)
    B, D = queries.shape
    if D != packed.D:
        raise ValueError(f"query dim {D} != item dim {packed.D}")
    if not 0 < k <= K_MAX:
        raise ValueError(f"mips_topk supports 0 < k <= {K_MAX} (got {k})")
    q = queries if queries.dtype == torch.float32 and queries.is_contiguous() else \
        queries.contiguous().float()
    dev = q.device
    ids = None
    if item_ids is not None:
        ids = item_ids.reshape(-1)
        if ids.dtype != torch.int64 or ids.device != dev or not ids.is_contiguous():
            ids = ids.to(device=dev, dtype=torch.int64).contiguous()
        if ids.numel() != packed.X:
            raise ValueError(f"item_ids has {ids.numel()} entries, table has {packed.X}")
    inv = None
    N0 = 0
    if invalid_ids is not None:
        inv = invalid_ids
        if inv.dtype != torch.int64 or inv.device != dev or not inv.is_contiguous():
            inv = inv.to(device=dev, dtype=torch.int64).contiguous()
        if inv.dim() != 2 or inv.shape[0] != B:
            raise ValueError("invalid_ids must be (B, N0)")
        N0 = inv.shape[1]
        if N0 > N0_MAX:
            raise ValueError(f"mips_topk supports N0 <= {N0_MAX} invalid ids per row (got {N0})")
    scores = torch.empty(B, k, dtype=torch.float32, device=dev)
    out_ids = torch.empty(B, k, dtype=torch.int64, device=dev)
    out_idx = torch.empty(B, k, dtype=torch.int64, device=dev) if return_index else None
    if workspace is None:
        ws_n, ws = packed.workspace(B, k, N0)
    else:
        ws_n = topk_workspace_bytes(B, packed.X, D, k, N0)
        if workspace.dtype != torch.uint8 or workspace.numel() < ws_n or workspace.device != dev:
            raise ValueError(f"workspace must be a uint8 tensor of >= {ws_n} bytes on {dev}")
        ws = workspace
    _lib.call("mips_topk", q.data_ptr(), packed.buf.data_ptr(), packed.X, D, _lib.ptr(ids),
              int(index_base), _lib.ptr(inv), N0, B, k, scores.data_ptr(), out_ids.data_ptr(),
              _lib.ptr(out_idx), ws.data_ptr(), ws_n, _lib.stream_handle())
    if return_index:
        return scores, out_ids, out_idx
    return scores, out_ids


def merge_topk(cand_scores: torch.Tensor, cand_index: torch.Tensor, cand_ids: torch.Tensor,
               k: int, return_index: bool = False):
    """Merges (n_lists, B, k_in) candidate lists into the global (B, k) top-k
    (``mips_merge_topk``): the reduction step of a row-sharded catalog."""
    _lib.require_gpu(cand_scores, cand_index, cand_ids)
    n_lists, B, k_in = cand_scores.shape
    dev = cand_scores.device
    s = cand_scores.contiguous()
    i = cand_index.contiguous()
    d = cand_ids.contiguous()
    scores = torch.empty(B, k, dtype=torch.float32, device=dev)
    out_ids = torch.empty(B, k, dtype=torch.int64, device=dev)
    out_idx = torch.empty(B, k, dtype=torch.int64, device=dev) if return_index else None
    _lib.call("mips_merge_topk", s.data_ptr(), i.data_ptr(), d.data_ptr(), n_lists, B, k_in, k,
              scores.data_ptr(), out_ids.data_ptr(), _lib.ptr(out_idx), _lib.stream_handle())
    if return_index:
        return scores, out_ids, out_idx
    return scores, out_ids


class MIPSBruteForceTopK(TopKModule):
    """top_k.py:43-70 — (scores, ids) of the k best inner products.

    ``item_embeddings_t`` is the (D, X) transposed view the reference's CandidateIndex
    keeps.  The packed copy is cached so a table is re-laid out once per
    ``update_embeddings``, not once per query batch.  The cache key is the view's
    storage pointer, shape and strides plus its version counter when it has one.
    Inference tensors have none (``Retrieval.retrieve`` is ``@torch.inference_mode``,
    retrieval.py:19), so ``CandidateIndex.update_embeddings`` also calls
    ``invalidate()``; a caller that rewrites an inference tensor in place without it
    must call ``invalidate()`` itself.
    """

    def __init__(self) -> None:
        super().__init__()
        self._cache_key = None
        self._packed: Optional[PackedItems] = None
        self._ids_key = None
        self._ids_arange_start: Optional[int] = None

    @staticmethod
    def _key(t: torch.Tensor):
        version = None if t.is_inference() else t._version
        return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.device, version)

    def invalidate(self) -> None:
        """Drops the packed table and the ids check (the table or ids changed)."""
        self._cache_key = None
        self._packed = None
        self._ids_key = None
        self._ids_arange_start = None

    def packed_for(self, item_embeddings_t: torch.Tensor) -> PackedItems:
        key = self._key(item_embeddings_t)
        if self._packed is None or self._cache_key != key:
            self._packed = PackedItems(item_embeddings_t.t())
            self._cache_key = key
        return self._packed

    def _arange_start(self, item_ids: torch.Tensor) -> Optional[int]:
        """ids == arange(s, s + X)?  Checked once per ids buffer (one host sync, like
        the reference's per-epoch index refresh); then the kernel derives ids from
        the catalog index and skips the id gathers."""
        key = self._key(item_ids)
        if self._ids_key != key:
            flat = item_ids.reshape(-1)
            start = int(flat[0].item()) if flat.numel() else 0
            ar = torch.arange(start, start + flat.numel(), device=flat.device, dtype=flat.dtype)
            self._ids_arange_start = start if bool(torch.equal(flat, ar)) else None
            self._ids_key = key
        return self._ids_arange_start

    def forward(self, query_embeddings: torch.Tensor, item_embeddings_t: torch.Tensor,
                item_ids: torch.Tensor, k: int, sorted: bool = True,
                invalid_ids: Optional[torch.Tensor] = None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        packed = self.packed_for(item_embeddings_t)
        start = self._arange_start(item_ids)
        if start is not None:
            return mips_topk(query_embeddings, packed, k, item_ids=None, index_base=start,
                             invalid_ids=invalid_ids)
        return mips_topk(query_embeddings, packed, k, item_ids=item_ids, invalid_ids=invalid_ids)
