"""HSTU sequential encoder — drop-in for the reference's
``generative_recommenders_pl.models.sequential_encoders.hstu`` (Hydra ``_target_``
``...sequential_encoders.hstu.HSTU``), running the MI355X kernels of
``libgr_hstu.so``.

Same constructor arguments, parameter names / shapes / initialisation and
state-dict keys as the reference (``hstu.py:71-128, 208-672``), so checkpoints
round-trip.  The compute is the fused jagged path: per layer 3 launches forward
(LN+UVQK+SiLU GEMM, attention with in-kernel relative bias, gate+LN+O GEMM+residual)
and 5 backward; nothing of size (B, N, N) is materialised.  ``concat_ua=True``
(hstu.py:398-400) runs the concatenated gate [u, LN(a), u*LN(a)] at any width (the
row-wave kernels with W_o in LDS up to linear_dim * num_heads = 64 and D = 128, the
streamed-W_o form beyond).  ``autocast_dtype=torch.bfloat16`` (an extension
of the reference constructor, whose HSTUJagged takes it) selects bf16 MFMA operands.

Cached (incremental) decoding (hstu.py:151-177, 293-298, 321-322, 415-423):
``return_cache_states=True`` returns every layer's (v, padded q, padded k, outputs) as the
reference does; a later call with ``delta_x_offsets`` and ``cache`` re-encodes one row per
sequence against those caches, updating them in place (``ops.stu_decode``: the delta
rows' attention only, not the reference's full (B, h, n, n) pass).  The cached step is
inference-only (it raises under autograd) and computes in fp32 in either mode.

``normalization="softmax_rel_bias"`` (hstu.py:341-389, used by no config) runs as an fp32
layer (``ops.stu_softmax_layer``: the softmax attention kernels of
``hstu_softmax_attn.hip``, the materialised (B, n, n) bias of ``hstu_rel_bias_fwd``).

Not supported (raise): the cached step with ``softmax_rel_bias`` (the reference's branch
fails at hstu.py:343) and attention dropout > 0 (the reference ignores it too).
"""
from __future__ import annotations

import abc
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F  # noqa: F401  (kept for API parity of the module)

from . import ops
from .bucket_table import BUCKET_THRESHOLDS, NUM_BUCKETS

TIMESTAMPS_KEY = "timestamps"

HSTUCacheState = Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]


def _default_bucketization_fn(x: torch.Tensor) -> torch.Tensor:
    """hstu.py:579-581.  The fused kernel evaluates this function exactly through the
    integer threshold table in ``bucket_table.py``; it is kept for API parity."""
    return (torch.log(torch.abs(x).clamp(min=1)) / 0.301).long()


def _bucket_probe_deltas() -> torch.Tensor:
    """int64 time deltas probing the threshold table: each threshold, its two neighbours
    and the midpoint to the next threshold; every delta in [0, 4096]; 8,192 deltas drawn
    log-uniformly over [1, 2^62] from a fixed seed; and their negations."""
    thr = BUCKET_THRESHOLDS
    vals = set(range(4097))
    for b, t in enumerate(thr):
        vals.update((t - 1, t, t + 1))
        if b + 1 < len(thr):
            vals.add((t + thr[b + 1]) // 2)
    g = torch.Generator().manual_seed(20240)
    e = torch.rand(8192, generator=g, dtype=torch.float64) * 62.0
    vals.update(int(v) for v in torch.exp2(e).to(torch.int64).tolist())
    vals = sorted(v for v in vals if v >= 0)
    return torch.tensor(vals + [-v for v in vals], dtype=torch.int64)


def _check_bucketization_fn(fn: Callable[[torch.Tensor], torch.Tensor]) -> None:
    """The attention kernels bucket relative times through the integer threshold table
    of the reference's default function (hstu.py:579-581, clamped to [0, num_buckets] at
    hstu.py:117-123).  A caller-supplied function is accepted only if it agrees with
    that table on every probe delta (the reference builds it as a lambda, so an identity
    test would reject valid models); anything else raises instead of silently using
    the default buckets.  The check is a sampling heuristic, not a proof: ~25 K probes
    cover every threshold edge, all small deltas and a log-uniform sample of the int64
    range, so a function that agrees on all of them and differs elsewhere would pass."""
    d = _bucket_probe_deltas()
    thr = torch.tensor(BUCKET_THRESHOLDS, dtype=torch.int64)
    want = torch.searchsorted(thr, d.abs(), right=True) - 1
    try:
        got = torch.clamp(fn(d).long(), min=0, max=NUM_BUCKETS)
    except Exception as e:  # noqa: BLE001 — any failure means "not the default function"
        raise ValueError(f"bucketization_fn could not be evaluated on int64 deltas: {e}") from e
    if got.shape != want.shape or not torch.equal(got, want):
        bad = int((got != want).nonzero()[0, 0]) if got.shape == want.shape else 0
        raise ValueError(
            "bucketization_fn differs from the reference default "
            "(log(|dt|.clamp(min=1)) / 0.301).long() (hstu.py:579-581), which is the only "
            f"bucketization the fused attention kernels implement (first mismatch at "
            f"dt = {int(d[bad])})")


class RelativeAttentionBiasModule(torch.nn.Module):
    @abc.abstractmethod
    def forward(self, all_timestamps: torch.Tensor) -> torch.Tensor:
        pass


class RelativeBucketedTimeAndPositionBasedBias(RelativeAttentionBiasModule):
    """Relative position + time bias (hstu.py:71-128).

    ``_ts_w`` (num_buckets + 1) and ``_pos_w`` (2 * max_seq_len - 1), N(0, 0.02).
    Inside the encoder the bias is never materialised (the attention kernels rebuild it
    per tile); ``forward`` materialises it for callers that use the module on its own.
    """

    def __init__(self, max_seq_len: int, num_buckets: int,
                 bucketization_fn: Callable[[torch.Tensor], torch.Tensor]) -> None:
        super().__init__()
        # the kernels' threshold table encodes the reference's default function only
        if num_buckets != NUM_BUCKETS:
            raise ValueError(f"num_buckets must be {NUM_BUCKETS} (got {num_buckets})")
        if bucketization_fn is not _default_bucketization_fn:
            _check_bucketization_fn(bucketization_fn)
        self._max_seq_len: int = max_seq_len
        self._ts_w = torch.nn.Parameter(torch.empty(num_buckets + 1).normal_(mean=0, std=0.02))
        self._pos_w = torch.nn.Parameter(
            torch.empty(2 * max_seq_len - 1).normal_(mean=0, std=0.02))
        self._num_buckets: int = num_buckets
        self._bucketization_fn = bucketization_fn

    def forward(self, all_timestamps: torch.Tensor) -> torch.Tensor:
        """(B, N) int64 timestamps -> (B, N, N) bias, N = max_seq_len (hstu.py:96-128),
        materialised by ``hstu_rel_bias_fwd`` with gradients to ``_pos_w`` / ``_ts_w``.
        The encoder never calls this: its attention rebuilds the bias per tile."""
        return ops.rel_bias(all_timestamps, self._max_seq_len, self._pos_w, self._ts_w)


class SequentialTransductionUnitJagged(torch.nn.Module):
    """hstu.py:208-423, same constructor and parameters."""

    def __init__(
        self,
        embedding_dim: int,
        linear_hidden_dim: int,
        attention_dim: int,
        dropout_ratio: float,
        attn_dropout_ratio: float,
        num_heads: int,
        linear_activation: str,
        relative_attention_bias_module: Optional[RelativeAttentionBiasModule] = None,
        normalization: str = "rel_bias",
        linear_config: str = "uvqk",
        concat_ua: bool = False,
        epsilon: float = 1e-6,
        max_length: Optional[int] = None,
    ) -> None:
        super().__init__()
        self._embedding_dim = embedding_dim
        self._linear_dim = linear_hidden_dim
        self._attention_dim = attention_dim
        self._dropout_ratio = dropout_ratio
        self._attn_dropout_ratio = attn_dropout_ratio
        self._num_heads = num_heads
        self._rel_attn_bias = relative_attention_bias_module
        self._normalization = normalization
        self._linear_config = linear_config
        if self._linear_config == "uvqk":
            self._uvqk = torch.nn.Parameter(
                torch.empty((embedding_dim,
                             linear_hidden_dim * 2 * num_heads + attention_dim * num_heads * 2)
                            ).normal_(mean=0, std=0.02))
        else:
            raise ValueError(f"Unknown linear_config {self._linear_config}")
        self._linear_activation = linear_activation
        self._concat_ua = concat_ua
        self._o = torch.nn.Linear(
            in_features=linear_hidden_dim * num_heads * (3 if concat_ua else 1),
            out_features=embedding_dim)
        torch.nn.init.xavier_uniform_(self._o.weight)
        self._eps = epsilon
        # dropout: mask = hash(base seed + device step counter, element).  The counter
        # is bumped on the device each training forward, so CUDA/HIP-graph replays draw
        # fresh masks; the backward re-derives the forward's mask from the same counter.
        self._dropout_seed = int(torch.randint(0, 2**62, (1,)).item())
        self.register_buffer("_dropout_step", torch.zeros(1, dtype=torch.int64),
                             persistent=False)
        self._bf16 = False  # set by HSTUJagged from its autocast_dtype

    def _geometry(self, n: int, max_len: int) -> ops.STUGeometry:
        if self._linear_activation == "silu":
            act = 1
        elif self._linear_activation == "none":
            act = 0
        else:
            raise ValueError(f"Unknown linear_activation {self._linear_activation}")
        if self._normalization not in ("rel_bias", "hstu_rel_bias", "softmax_rel_bias"):
            raise ValueError(f"Unknown normalization method {self._normalization}")
        softmax = self._normalization == "softmax_rel_bias"
        return ops.STUGeometry(
            N=n, D=self._embedding_dim, H=self._num_heads, dqk=self._attention_dim,
            dv=self._linear_dim, eps=self._eps, activation=act,
            dropout_p=float(self._dropout_ratio) if self.training else 0.0,
            max_len=max_len, bf16=self._bf16 and not softmax, concat_ua=self._concat_ua,
            softmax=softmax)

    def forward(
        self,
        x: torch.Tensor,
        x_offsets: torch.Tensor,
        all_timestamps: Optional[torch.Tensor],
        invalid_attn_mask: torch.Tensor,
        delta_x_offsets: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
        cache: Optional[HSTUCacheState] = None,
        return_cache_states: bool = False,
        max_len: Optional[int] = None,
        bucket_map: Optional[torch.Tensor] = None,
        dropout_step: Optional[torch.Tensor] = None,
    ):
        """x: (rows, D) jagged; x_offsets (B+1,).  Returns (x', cache-state tuple): with
        ``return_cache_states`` the reference's (v, padded q, padded k, x') over the
        offsets[B] valid rows (one host sync), else (None, None, None, x').
        ``delta_x_offsets`` + ``cache``: the cached step (hstu.py:293-298), see
        ``ops.stu_decode``; the cache tensors are updated in place and returned.
        ``bucket_map`` (optional) is the batch's ``ops.bucket_map`` — pass it to share
        it across layers; otherwise it is built from ``all_timestamps``.
        ``dropout_step`` (optional) is an already-advanced device step counter shared by
        the layers of one encoder forward (one increment per forward instead of one per
        layer); by default the layer advances its own."""
        n = invalid_attn_mask.size(-1)
        geo = self._geometry(n, n if max_len is None else max_len)
        rab = self._rel_attn_bias
        if delta_x_offsets is not None:
            if geo.softmax:
                # hstu.py:342-343 evaluates x_offsets.size() - 1, which raises (TypeError)
                raise NotImplementedError("cached decoding with normalization="
                                          "'softmax_rel_bias' (the reference's branch fails)")
            return self._decode(x, x_offsets, all_timestamps, delta_x_offsets, cache, geo,
                                dropout_step)[:2]
        if geo.softmax:
            return self._softmax_forward(x, x_offsets, all_timestamps, n, geo, return_cache_states,
                                         dropout_step)
        bmap = None
        if rab is not None and all_timestamps is not None:
            bmap = bucket_map if bucket_map is not None else ops.bucket_map(
                all_timestamps, x_offsets, n)
        pos_w = rab._pos_w if bmap is not None else None
        ts_w = rab._ts_w if bmap is not None else None
        if bmap is not None and pos_w.numel() != 2 * n - 1:
            raise ValueError(f"_pos_w has {pos_w.numel()} entries, expected {2 * n - 1}")
        step = None
        if geo.dropout_p > 0:
            if dropout_step is not None:
                step = dropout_step
            else:
                self._dropout_step.add_(1)
                step = self._dropout_step
        y = ops.stu_layer(x, x_offsets, bmap, self._uvqk, self._o.weight, self._o.bias, pos_w,
                          ts_w, geo, self._dropout_seed, step, return_uvqk=return_cache_states)
        if return_cache_states:
            y, uvqk = y
            return y, ops.stu_cache_states(uvqk, y, x_offsets, int(x_offsets[-1]), geo)
        return y, (None, None, None, y)

    def _softmax_forward(self, x, x_offsets, all_timestamps, n, geo, return_cache_states,
                         dropout_step):
        """normalization="softmax_rel_bias" (hstu.py:341-389): the (B, n, n) bias of
        ``_rel_attn_bias`` (hstu_rel_bias_fwd; its backward gives _pos_w / _ts_w their
        gradients), then the softmax layer (ops.stu_softmax_layer), fp32."""
        rab = self._rel_attn_bias
        bias = None
        if rab is not None:
            if all_timestamps is None:
                raise ValueError("normalization='softmax_rel_bias' with a relative bias module "
                                 "needs timestamps (hstu.py:379-380)")
            bias = rab(all_timestamps)
        step = None
        if geo.dropout_p > 0:
            if dropout_step is not None:
                step = dropout_step
            else:
                self._dropout_step.add_(1)
                step = self._dropout_step
        y = ops.stu_softmax_layer(x, x_offsets, bias, self._uvqk, self._o.weight, self._o.bias,
                                  geo, self._dropout_seed, step, return_uvqk=return_cache_states)
        if return_cache_states:
            y, uvqk = y
            return y, ops.stu_cache_states(uvqk, y, x_offsets, int(x_offsets[-1]), geo)
        return y, (None, None, None, y)

    def _decode(self, x, x_offsets, all_timestamps, delta_x_offsets, cache, geo, dropout_step,
                xd=None):
        """hstu.py:293-298 (assert cache is not None), 321-322, 151-177, 393-418.  Returns
        (outputs, cache states, the re-encoded rows); ``xd``: this layer's x[delta] rows
        when the caller already has them."""
        if cache is None:
            raise ValueError("delta_x_offsets requires the cache states of a previous pass")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError(
                "cached HSTU decoding is inference-only (no backward): run it under "
                "torch.no_grad() or torch.inference_mode()")
        rab = self._rel_attn_bias
        step = None
        if geo.dropout_p > 0:
            if dropout_step is not None:
                step = dropout_step
            else:
                self._dropout_step.add_(1)
                step = self._dropout_step
        out, y = ops.stu_decode(x, x_offsets, all_timestamps if rab is not None else None,
                                delta_x_offsets[0], delta_x_offsets[1], cache, self._uvqk,
                                self._o.weight, self._o.bias,
                                rab._pos_w if rab is not None else None,
                                rab._ts_w if rab is not None else None, geo, self._dropout_seed,
                                step, xd=xd)
        return out, (cache[0], cache[1], cache[2], out), y


class HSTUJagged(torch.nn.Module):
    """hstu.py:426-518."""

    def __init__(self, modules: List[SequentialTransductionUnitJagged],
                 autocast_dtype: Optional[torch.dtype]) -> None:
        """autocast_dtype (hstu.py:439-480): None / float32 = the reference's fp32 path
        (HSTU hard-wires None, hstu.py:592); torch.bfloat16 = the opt-in bf16 compute mode:
        MFMA operands in bf16 (attention Q, K, V, dO, P, dS; the UVQK / O projections and
        their weight gradients, except the concat_ua gate GEMM), fp32 accumulation, LN,
        elementwise work and parameters."""
        super().__init__()
        self._attention_layers = torch.nn.ModuleList(modules=modules)
        if autocast_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError(f"autocast_dtype must be None, float32 or bfloat16 (got {autocast_dtype})")
        self._autocast_dtype = autocast_dtype
        for layer in self._attention_layers:
            layer._bf16 = autocast_dtype is torch.bfloat16
        # the layers as one autograd node (ops.stu_stack: every layer's weight gradients in
        # one launch pair); False = one node per layer (ops.stu_layer), as the reference
        self._use_stack = True
        # one device dropout counter per encoder forward (layers hash with their own seed)
        self.register_buffer("_dropout_step", torch.zeros(1, dtype=torch.int64),
                             persistent=False)

    def _needs_map(self, all_timestamps) -> bool:
        return all_timestamps is not None and any(
            layer._rel_attn_bias is not None and layer._normalization != "softmax_rel_bias"
            for layer in self._attention_layers)

    def _needs_step(self) -> bool:
        return self.training and any(layer._dropout_ratio > 0 for layer in self._attention_layers)

    def jagged_forward(self, x, x_offsets, all_timestamps, invalid_attn_mask,
                       delta_x_offsets=None, cache=None, return_cache_states=False,
                       max_len: Optional[int] = None, _prepared=None):
        """``_prepared`` (internal): (bucket map, advanced dropout step) already produced by
        ops.encoder_prologue.  ``delta_x_offsets`` + ``cache`` (one state tuple per layer):
        the cached step, layer by layer (hstu.py:467-478)."""
        cache_states: List[HSTUCacheState] = []
        n = invalid_attn_mask.size(-1)
        if delta_x_offsets is not None:
            if cache is None or len(cache) != len(self._attention_layers):
                raise ValueError("delta_x_offsets requires one cache state per layer")
            d0 = delta_x_offsets[0].to(torch.int64)
            d1 = delta_x_offsets[1].to(torch.int64)
            distinct = ops.check_decode_step(x_offsets, d0, d1, n)
            step = None
            if self._needs_step():
                self._dropout_step.add_(1)
                step = self._dropout_step
            xd = None
            for i, layer in enumerate(self._attention_layers):
                geo = layer._geometry(n, n if max_len is None else max_len)
                if geo.softmax:
                    # hstu.py:342-343 evaluates x_offsets.size() - 1, which raises (TypeError)
                    raise NotImplementedError("cached decoding with normalization="
                                              "'softmax_rel_bias' (the reference's branch fails)")
                x, cs, y = layer._decode(x, x_offsets, all_timestamps, (d0, d1), cache[i], geo,
                                         step, xd=xd)
                # distinct delta rows: the rows just re-encoded are the next layer's x[delta]
                xd = y if distinct else None
                if return_cache_states:
                    cache_states.append(cs)
            return x, cache_states
        if _prepared is not None:
            bmap, step = _prepared
        else:
            # one bucket map per batch, shared by every layer's forward and backward
            bmap = ops.bucket_map(all_timestamps, x_offsets, n) if self._needs_map(all_timestamps) else None
            step = None
            if self._needs_step():
                self._dropout_step.add_(1)
                step = self._dropout_step
        stack = self._stack_params(n, max_len, bmap, return_cache_states)
        if stack is not None:
            geo, params, seeds = stack
            x = ops.stu_stack(x, x_offsets, bmap, params, geo, seeds, step)
            return x, cache_states
        for layer in self._attention_layers:
            x, cs = layer(x=x, x_offsets=x_offsets, all_timestamps=all_timestamps,
                          invalid_attn_mask=invalid_attn_mask,
                          delta_x_offsets=delta_x_offsets, cache=None,
                          return_cache_states=return_cache_states, max_len=max_len,
                          bucket_map=bmap, dropout_step=step)
            if return_cache_states:
                cache_states.append(cs)
        return x, cache_states

    def _stack_params(self, n, max_len, bmap, return_cache_states):
        """(geometry, per-layer params, dropout seeds) when the layers can run as one
        ``ops.stu_stack`` node (same geometry, no concat_ua, no cache states), else None."""
        if return_cache_states or not self._use_stack:
            return None
        layers = list(self._attention_layers)
        geos = [layer._geometry(n, n if max_len is None else max_len) for layer in layers]
        if any(g != geos[0] for g in geos) or geos[0].concat_ua or geos[0].softmax:
            return None
        params = []
        for layer in layers:
            rab = layer._rel_attn_bias
            has_bias = bmap is not None and rab is not None
            if (bmap is not None) != has_bias:
                return None  # some layers without a bias module: per-layer path
            if has_bias and rab._pos_w.numel() != 2 * n - 1:
                raise ValueError(f"_pos_w has {rab._pos_w.numel()} entries, expected {2 * n - 1}")
            params.append((layer._uvqk, layer._o.weight, layer._o.bias,
                           rab._pos_w if has_bias else None, rab._ts_w if has_bias else None))
        return geos[0], params, [layer._dropout_seed for layer in layers]

    def forward(self, x, x_offsets, all_timestamps, invalid_attn_mask, delta_x_offsets=None,
                cache=None, return_cache_states=False, max_len: Optional[int] = None):
        n = invalid_attn_mask.size(1)
        if x.dim() == 3:
            x = ops.dense_to_jagged(x, x_offsets, zero_fill=False)  # B*N capacity rows, no sync
        jagged_x, cache_states = self.jagged_forward(
            x, x_offsets, all_timestamps, invalid_attn_mask, delta_x_offsets, cache,
            return_cache_states, max_len=max_len)
        y = ops.jagged_to_padded_dense(jagged_x, x_offsets, n, 0.0)
        return y, cache_states

    def forward_from_lengths(self, lengths, x, all_timestamps, invalid_attn_mask,
                             return_cache_states=False, max_len: Optional[int] = None):
        """HSTU.forward on padded fp32 input (B, N, D) with N = the mask size: the offsets,
        the jagged rows, the bucket map and the dropout step come from one launch
        (ops.encoder_prologue) instead of four (cumsum, dense_to_jagged, bucket map,
        counter add); results are identical."""
        n = invalid_attn_mask.size(1)
        need_map = self._needs_map(all_timestamps)
        step = self._dropout_step if self._needs_step() else None
        xj, x_offsets, bmap = ops.encoder_prologue(
            lengths, x, all_timestamps if need_map else None, step)
        jagged_x, cache_states = self.jagged_forward(
            xj, x_offsets, all_timestamps, invalid_attn_mask, None, None, return_cache_states,
            max_len=max_len, _prepared=(bmap, step))
        y = ops.jagged_to_padded_dense(jagged_x, x_offsets, n, 0.0)
        return y, cache_states


class HSTU(torch.nn.Module):
    """Drop-in for reference ``HSTU`` (hstu.py:521-672)."""

    def __init__(
        self,
        max_sequence_len: int,
        max_output_len: int,
        embedding_dim: int,
        item_embedding_dim: int,
        num_blocks: int,
        num_heads: int,
        linear_dim: int,
        attention_dim: int,
        normalization: str,
        linear_config: str,
        linear_activation: str,
        linear_dropout_rate: float,
        attn_dropout_rate: float,
        enable_relative_attention_bias: bool = True,
        concat_ua: bool = False,
        autocast_dtype: Optional[torch.dtype] = None,
    ) -> None:
        """Reference constructor (hstu.py:532-549) plus ``autocast_dtype`` (default None =
        the reference's hard-wired fp32; torch.bfloat16 = the opt-in bf16 MFMA mode,
        see HSTUJagged)."""
        super().__init__()
        self._embedding_dim = embedding_dim
        self._item_embedding_dim = item_embedding_dim
        self._max_sequence_length = max_sequence_len
        self._num_blocks = num_blocks
        self._num_heads = num_heads
        self._dqk = attention_dim
        self._dv = linear_dim
        self._linear_activation = linear_activation
        self._linear_dropout_rate = linear_dropout_rate
        self._attn_dropout_rate = attn_dropout_rate
        self._enable_relative_attention_bias = enable_relative_attention_bias
        self._hstu = HSTUJagged(
            modules=[
                SequentialTransductionUnitJagged(
                    embedding_dim=self._embedding_dim,
                    linear_hidden_dim=linear_dim,
                    attention_dim=attention_dim,
                    normalization=normalization,
                    linear_config=linear_config,
                    linear_activation=linear_activation,
                    num_heads=num_heads,
                    relative_attention_bias_module=(
                        RelativeBucketedTimeAndPositionBasedBias(
                            max_seq_len=max_sequence_len + max_output_len,
                            num_buckets=NUM_BUCKETS,
                            bucketization_fn=_default_bucketization_fn,
                        ) if enable_relative_attention_bias else None),
                    dropout_ratio=linear_dropout_rate,
                    attn_dropout_ratio=attn_dropout_rate,
                    concat_ua=concat_ua,
                )
                for _ in range(num_blocks)
            ],
            autocast_dtype=autocast_dtype,
        )
        self.register_buffer(
            "_attn_mask",
            torch.triu(torch.ones((self._max_sequence_length + max_output_len,
                                   self._max_sequence_length + max_output_len),
                                  dtype=torch.bool), diagonal=1))
        # forward on padded input: offsets, jagged rows, bucket map and dropout step in one
        # launch (ops.encoder_prologue); False = the reference's separate steps
        self.use_prologue = True
        self.reset_params()

    def reset_params(self):
        # hstu.py:609-621: every parameter of this module lives under _hstu -> skipped.
        for name, params in self.named_parameters():
            if ("_hstu" in name) or ("_embedding_module" in name):
                continue
            try:
                torch.nn.init.xavier_normal_(params.data)
            except Exception:
                pass

    def debug_str(self) -> str:
        s = (f"HSTU-b{self._num_blocks}-h{self._num_heads}-dqk{self._dqk}-dv{self._dv}"
             f"-l{self._linear_activation}d{self._linear_dropout_rate}"
             f"-ad{self._attn_dropout_rate}")
        if not self._enable_relative_attention_bias:
            s += "-norab"
        return s

    def forward(
        self,
        past_lengths: torch.Tensor,
        user_embeddings: torch.Tensor,
        valid_mask: torch.Tensor,
        past_payloads: Dict[str, torch.Tensor],
        delta_x_offsets: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
        cache: Optional[List[HSTUCacheState]] = None,
        return_cache_states: bool = False,
        max_len: Optional[int] = None,
    ) -> Tuple[torch.Tensor, List[HSTUCacheState]]:
        """past_lengths (B,), user_embeddings (B, N, D) fp32, past_payloads may hold
        "timestamps" (B, N) int64.  Returns ((B, N, D), cache_states); rows >= length
        are zero.  ``max_len`` (optional, host int) bounds the lengths to trim grids."""
        float_dtype = user_embeddings.dtype
        if float_dtype != torch.float32:
            user_embeddings = user_embeddings.float()
        ts = past_payloads[TIMESTAMPS_KEY] if TIMESTAMPS_KEY in past_payloads else None
        n = self._attn_mask.size(1)
        if (self.use_prologue and delta_x_offsets is None and cache is None
                and user_embeddings.dim() == 3 and user_embeddings.size(1) == n
                and (ts is None or tuple(ts.shape) == (user_embeddings.size(0), n))):
            y, cached_states = self._hstu.forward_from_lengths(
                past_lengths, user_embeddings, ts, self._attn_mask,
                return_cache_states=return_cache_states, max_len=max_len)
            return y.to(float_dtype), cached_states
        y, cached_states = self._hstu(
            x=user_embeddings,
            x_offsets=ops.asynchronous_complete_cumsum(past_lengths),
            all_timestamps=(past_payloads[TIMESTAMPS_KEY]
                            if TIMESTAMPS_KEY in past_payloads else None),
            invalid_attn_mask=self._attn_mask,
            delta_x_offsets=delta_x_offsets,
            cache=cache,
            return_cache_states=return_cache_states,
            max_len=max_len,
        )
        return y.to(float_dtype), cached_states
