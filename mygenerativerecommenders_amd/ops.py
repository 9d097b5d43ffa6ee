"""Host-side operators over the gfx950 C-ABI (``libgr_hstu.so``).

Python mirror of the reference's ``models/utils/ops.py`` jagged helpers plus the
autograd wrapper of one fused STU layer.  Every op runs on the MI355X through the
C-ABI; there is no CPU path (the CPU restatement in ``oracle/`` is test-only).

Reference map (``src/generative_recommenders_pl/models/``):
  * asynchronous_complete_cumsum .. utils/ops.py:18-38
  * dense_to_jagged .............. utils/ops.py:41-64
  * jagged_to_padded_dense ....... utils/ops.py:67-114
  * get_current_embeddings ....... utils/ops.py:171-187
  * sampled_softmax_loss ......... losses/autoregressive_losses.py:259-306 (+ the
                                   negatives gather of negative_sampler.py:105-131)
  * STU layer fwd/bwd ............ sequential_encoders/hstu.py:266-413 (+ autograd)
"""
from __future__ import annotations


import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib
from .bucket_table import BUCKET_THRESHOLDS, NUM_BUCKETS

_THR_CACHE: dict = {}


def bucket_thresholds(device) -> torch.Tensor:
    key = str(device)
    t = _THR_CACHE.get(key)
    if t is None:
        t = torch.tensor(BUCKET_THRESHOLDS, dtype=torch.int64, device=device)
        _THR_CACHE[key] = t
    return t


def _stream():
    return _lib.stream_handle()




# ------------------------------------------------------------------ jagged helpers

def asynchronous_complete_cumsum(lengths: torch.Tensor) -> torch.Tensor:
    """(B,) -> (B + 1,) int64 offsets [0, cumsum(lengths)] (utils/ops.py:18-38)."""
    _lib.require_gpu(lengths)
    lengths = lengths.to(torch.int64).contiguous()
    B = lengths.numel()
    out = torch.empty(B + 1, dtype=torch.int64, device=lengths.device)
    _lib.call("gr_complete_cumsum", lengths.data_ptr(), B, out.data_ptr(), _stream())
    return out


class _DenseToJagged(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dense, offsets, total_rows, zero_fill):
        B, N, D = dense.shape
        dense = dense.contiguous()
        out = torch.empty(total_rows, D, dtype=dense.dtype, device=dense.device)
        _lib.call("gr_dense_to_jagged", dense.data_ptr(), offsets.data_ptr(), B, N, D,
                  total_rows, int(zero_fill), out.data_ptr(), _stream())
        ctx.save_for_backward(offsets)
        ctx.shape = (B, N, D)
        return out

    @staticmethod
    def backward(ctx, g):
        (offsets,) = ctx.saved_tensors
        B, N, D = ctx.shape
        g = g.contiguous()
        out = torch.empty(B, N, D, dtype=g.dtype, device=g.device)
        _lib.call("gr_jagged_to_padded", g.data_ptr(), offsets.data_ptr(), B, N, D,
                  out.data_ptr(), _stream())
        return out, None, None, None


class _JaggedToPadded(torch.autograd.Function):
    @staticmethod
    def forward(ctx, values, offsets, N):
        B = offsets.numel() - 1
        D = values.shape[1]
        values = values.contiguous()
        out = torch.empty(B, N, D, dtype=values.dtype, device=values.device)
        _lib.call("gr_jagged_to_padded", values.data_ptr(), offsets.data_ptr(), B, N, D,
                  out.data_ptr(), _stream())
        ctx.save_for_backward(offsets)
        ctx.meta = (B, N, D, values.shape[0])
        return out

    @staticmethod
    def backward(ctx, g):
        (offsets,) = ctx.saved_tensors
        B, N, D, rows = ctx.meta
        g = g.contiguous()
        out = torch.empty(rows, D, dtype=g.dtype, device=g.device)
        # rows no padded position reaches (lengths above N, rows past offsets[B]) get 0
        _lib.call("gr_dense_to_jagged", g.data_ptr(), offsets.data_ptr(), B, N, D, rows, 1,
                  out.data_ptr(), _stream())
        return out, None, None


def dense_to_jagged(dense_tensor: torch.Tensor, offsets: torch.Tensor,
                    total_rows: Optional[int] = None, zero_fill: bool = True) -> torch.Tensor:
    """(B, N, D) -> (total, D) (utils/ops.py:41-64).  ``total_rows`` defaults to B*N
    capacity (sync-free) — pass the exact total to get an exact-size result.  Rows past
    offsets[B] are zero unless ``zero_fill=False`` (they are then scratch; the encoder
    uses that for its capacity-sized activations)."""
    _lib.require_gpu(dense_tensor, offsets)
    if dense_tensor.dtype != torch.float32:
        raise TypeError("dense_to_jagged: float32 only")
    B, N, _ = dense_tensor.shape
    if total_rows is None:
        total_rows = B * N
    return _DenseToJagged.apply(dense_tensor, offsets.to(torch.int64), int(total_rows),
                                bool(zero_fill))


def jagged_to_padded_dense(values: torch.Tensor, offsets: torch.Tensor, max_lengths: int,
                           padding_value: float = 0.0) -> torch.Tensor:
    """(total, D) -> (B, max_lengths, D), zero padded (utils/ops.py:67-114)."""
    if not isinstance(max_lengths, int):
        raise ValueError(f"max_lengths must be an integer, but got {type(max_lengths)}")
    if padding_value != 0.0:
        raise NotImplementedError("jagged_to_padded_dense: padding_value must be 0.0")
    _lib.require_gpu(values, offsets)
    squeeze = values.dim() == 1
    v = values.unsqueeze(-1) if squeeze else values
    if v.dtype != torch.float32:
        raise TypeError("jagged_to_padded_dense: float32 only")
    out = _JaggedToPadded.apply(v, offsets.to(torch.int64), max_lengths)
    return out.squeeze(-1) if squeeze else out


def get_current_embeddings(lengths: torch.Tensor, encoded_embeddings: torch.Tensor,
                           normalize: bool = False, eps: float = 1e-6) -> torch.Tensor:
    """(B, N, D) -> (B, D) with row lengths[b]-1 (utils/ops.py:171-187), optionally
    L2-normalised (the retrieval query, postprocessors.py:47-56).  One kernel
    (``gr_current_embeddings``); under autograd it is an index_select (+ l2_normalize)."""
    B, N, D = encoded_embeddings.shape
    if encoded_embeddings.requires_grad and torch.is_grad_enabled():
        idx = (lengths.to(torch.int64) - 1) + torch.arange(B, device=lengths.device) * N
        out = encoded_embeddings.reshape(-1, D).index_select(0, idx)
        return l2_normalize(out, eps) if normalize else out
    _lib.require_gpu(lengths, encoded_embeddings)
    enc = encoded_embeddings.contiguous()
    lens = lengths.to(torch.int64).contiguous()
    out = torch.empty(B, D, dtype=enc.dtype, device=enc.device)
    _lib.call("gr_current_embeddings", enc.data_ptr(), lens.data_ptr(), B, N, D,
              1 if normalize else 0, eps, out.data_ptr(), _stream())
    return out


class _L2Normalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        shape = x.shape
        D = shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        y = torch.empty_like(x2)
        _lib.call("gr_l2_normalize", x2.data_ptr(), D, x2.shape[0], D, eps, y.data_ptr(), D,
                  _stream())
        ctx.save_for_backward(x2)
        ctx.eps = eps
        ctx.shape = shape
        return y.reshape(shape)

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        D = x2.shape[1]
        g = dy.reshape(-1, D).contiguous()
        dx = torch.empty_like(x2)
        _lib.call("gr_l2_normalize_bwd", x2.data_ptr(), D, g.data_ptr(), D, x2.shape[0], D,
                  ctx.eps, dx.data_ptr(), D, _stream())
        return dx.reshape(ctx.shape), None


def l2_normalize(x: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    """x / clamp(||x||_2, eps) over the last dim (postprocessors.py:47-56), fwd + bwd."""
    _lib.require_gpu(x)
    if x.dtype != torch.float32:
        raise TypeError("l2_normalize: float32 only")
    return _L2Normalize.apply(x, float(eps))


# ------------------------------------------------------------------ relative-time buckets

def bucket_map(timestamps: torch.Tensor, offsets: torch.Tensor, N: int) -> torch.Tensor:
    """uint8 relative-time bucket of every causal (query, key) pair, computed once per
    batch and shared by all layers (``hstu_bucket_map``; reference hstu.py:111-123)."""
    _lib.require_gpu(timestamps, offsets)
    ts = timestamps.to(torch.int64).contiguous()
    B = offsets.numel() - 1
    if ts.shape != (B, N):
        raise ValueError(f"timestamps must be (B, N) = ({B}, {N}), got {tuple(ts.shape)}")
    nbytes = _lib.lib().hstu_bucket_map_bytes(B, N)
    out = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=ts.device)
    thr = bucket_thresholds(ts.device)
    _lib.call("hstu_bucket_map", ts.data_ptr(), offsets.data_ptr(), B, N, thr.data_ptr(),
              NUM_BUCKETS, out.data_ptr(), _stream())
    return out


class _EncoderPrologue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dense, lengths, ts, step):
        B, N, D = dense.shape
        dev = dense.device
        offsets = torch.empty(B + 1, dtype=torch.int64, device=dev)
        out = torch.empty(B * N, D, dtype=dense.dtype, device=dev)
        bmap = None
        if ts is not None:
            bmap = torch.empty(max(_lib.lib().hstu_bucket_map_bytes(B, N), 1), dtype=torch.uint8,
                               device=dev)
        thr = bucket_thresholds(dev) if ts is not None else None
        _lib.call("hstu_encoder_prologue", lengths.data_ptr(), B, N, dense.data_ptr(), D, B * N,
                  ts.data_ptr() if ts is not None else None, thr.data_ptr() if thr is not None else None,
                  NUM_BUCKETS, offsets.data_ptr(), out.data_ptr(),
                  bmap.data_ptr() if bmap is not None else None,
                  step.data_ptr() if step is not None else None, _stream())
        ctx.save_for_backward(offsets)
        ctx.shape = (B, N, D)
        if bmap is None:
            ctx.mark_non_differentiable(offsets)
            return out, offsets
        ctx.mark_non_differentiable(offsets, bmap)
        return out, offsets, bmap

    @staticmethod
    def backward(ctx, g, *_):
        (offsets,) = ctx.saved_tensors
        B, N, D = ctx.shape
        g = g.contiguous()
        dx = torch.empty(B, N, D, dtype=g.dtype, device=g.device)
        _lib.call("gr_jagged_to_padded", g.data_ptr(), offsets.data_ptr(), B, N, D, dx.data_ptr(),
                  _stream())
        return dx, None, None, None


def encoder_prologue(lengths: torch.Tensor, dense: torch.Tensor, timestamps: Optional[torch.Tensor],
                     step: Optional[torch.Tensor] = None):
    """The batch setup of an encoder forward as one launch (``hstu_encoder_prologue``):
    returns (x jagged with B*N capacity rows, offsets, bucket map or None), identical to
    ``dense_to_jagged(dense, asynchronous_complete_cumsum(lengths), zero_fill=False)`` and
    ``bucket_map(timestamps, offsets, N)``; ``step`` (an int64 device counter) is advanced by
    one.  Differentiable in ``dense`` (backward: jagged_to_padded_dense)."""
    _lib.require_gpu(lengths, dense)
    if dense.dtype != torch.float32 or dense.dim() != 3:
        raise TypeError("encoder_prologue: (B, N, D) float32 input expected")
    B, N, _ = dense.shape
    lengths = lengths.to(torch.int64).contiguous()
    if lengths.numel() != B:
        raise ValueError(f"encoder_prologue: {lengths.numel()} lengths for a batch of {B}")
    ts = None
    if timestamps is not None:
        ts = timestamps.to(torch.int64).contiguous()
        if ts.shape != (B, N):
            raise ValueError(f"timestamps must be (B, N) = ({B}, {N}), got {tuple(ts.shape)}")
    outs = _EncoderPrologue.apply(dense.contiguous(), lengths, ts, step)
    return (outs[0], outs[1], outs[2] if ts is not None else None)


class _RelBias(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ts, N, pos_w, ts_w):
        B = ts.shape[0]
        thr = bucket_thresholds(ts.device)
        out = torch.empty(B, N, N, dtype=torch.float32, device=ts.device)
        pw, tw = pos_w.detach().float().contiguous(), ts_w.detach().float().contiguous()
        _lib.call("hstu_rel_bias_fwd", ts.data_ptr(), B, N, thr.data_ptr(), NUM_BUCKETS,
                  pw.data_ptr(), tw.data_ptr(), out.data_ptr(), _stream())
        ctx.save_for_backward(ts)
        ctx.N = N
        ctx.shapes = (pos_w.shape, ts_w.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        (ts,) = ctx.saved_tensors
        N = ctx.N
        B = ts.shape[0]
        g = g.float().contiguous()
        d_pos = torch.empty(2 * N - 1, dtype=torch.float32, device=g.device)
        d_ts = torch.empty(NUM_BUCKETS + 1, dtype=torch.float32, device=g.device)
        ws_n = _lib.lib().hstu_rel_bias_bwd_workspace_size(B, N, NUM_BUCKETS)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=g.device)
        _lib.call("hstu_rel_bias_bwd", ts.data_ptr(), B, N, bucket_thresholds(g.device).data_ptr(),
                  NUM_BUCKETS, g.data_ptr(), d_pos.data_ptr(), d_ts.data_ptr(), ws.data_ptr(),
                  ws_n, _stream())
        pshape, tshape = ctx.shapes
        d_pos_full = d_pos
        if pshape[0] != 2 * N - 1:  # pos_w longer than 2N - 1: only its head is used
            d_pos_full = torch.zeros(pshape, dtype=torch.float32, device=g.device)
            d_pos_full[:2 * N - 1] = d_pos
        return None, None, d_pos_full, d_ts


def rel_bias(timestamps: torch.Tensor, N: int, pos_w: torch.Tensor,
             ts_w: torch.Tensor) -> torch.Tensor:
    """RelativeBucketedTimeAndPositionBasedBias.forward (hstu.py:96-128): (B, N) int64
    timestamps -> (B, N, N) fp32 bias over all (i, j), differentiable in pos_w / ts_w."""
    _lib.require_gpu(timestamps, pos_w, ts_w)
    ts = timestamps.to(torch.int64).contiguous()
    if ts.dim() != 2 or ts.shape[1] != N:
        raise ValueError(f"timestamps must be (B, {N}), got {tuple(ts.shape)}")
    if pos_w.numel() < 2 * N - 1 or ts_w.numel() != NUM_BUCKETS + 1:
        raise ValueError("rel_bias: pos_w needs >= 2N - 1 entries and ts_w num_buckets + 1")
    return _RelBias.apply(ts, int(N), pos_w, ts_w)


# ------------------------------------------------------------------ fused STU layer

class GrBoundaryFwd(ctypes.Structure):
    """include/gr_hstu.h GrBoundaryFwd: the layer-boundary arguments of hstu_attn_fwd_bnd
    (those of hstu_boundary_fwd; w_uvqk = NULL for the last layer: gate_o alone)."""
    _fields_ = [("u", ctypes.c_void_p), ("ld_u", ctypes.c_int64), ("max_rows", ctypes.c_int64),
                ("hdv", ctypes.c_int), ("D", ctypes.c_int), ("w_o", ctypes.c_void_p),
                ("b_o", ctypes.c_void_p), ("x_res", ctypes.c_void_p), ("ld_x", ctypes.c_int64),
                ("eps", ctypes.c_float), ("dropout_p", ctypes.c_float), ("seed", ctypes.c_uint64),
                ("seed_offset", ctypes.c_void_p), ("attn_stats", ctypes.c_void_p),
                ("o_in", ctypes.c_void_p), ("y", ctypes.c_void_p), ("ld_y", ctypes.c_int64),
                ("w_uvqk", ctypes.c_void_p), ("n_out", ctypes.c_int), ("activation", ctypes.c_int),
                ("x_stats", ctypes.c_void_p), ("h_pre", ctypes.c_void_p), ("uvqk", ctypes.c_void_p),
                ("ld_out", ctypes.c_int64)]


class GrBoundaryBwd(ctypes.Structure):
    """include/gr_hstu.h GrBoundaryBwd: the layer-boundary arguments of hstu_attn_bwd_bnd
    (those of hstu_boundary_bwd; hdv = 0 for the first layer: ln_uvqk_bwd alone)."""
    _fields_ = [("dh", ctypes.c_void_p), ("ld_dh", ctypes.c_int64), ("max_rows", ctypes.c_int64),
                ("D", ctypes.c_int), ("n_out", ctypes.c_int), ("w_uvqk", ctypes.c_void_p),
                ("x", ctypes.c_void_p), ("ld_x", ctypes.c_int64), ("x_stats", ctypes.c_void_p),
                ("dy_res", ctypes.c_void_p), ("ld_dy", ctypes.c_int64), ("dx", ctypes.c_void_p),
                ("ld_dx", ctypes.c_int64), ("hdv", ctypes.c_int), ("w_o", ctypes.c_void_p),
                ("u", ctypes.c_void_p), ("ld_u", ctypes.c_int64), ("attn", ctypes.c_void_p),
                ("ld_attn", ctypes.c_int64), ("attn_stats", ctypes.c_void_p),
                ("h_u", ctypes.c_void_p), ("ld_h", ctypes.c_int64), ("dropout_p", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("seed_offset", ctypes.c_void_p),
                ("du", ctypes.c_void_p), ("ld_du", ctypes.c_int64), ("d_attn", ctypes.c_void_p),
                ("ld_da", ctypes.c_int64)]


@dataclass
class STUGeometry:
    N: int              # padded max length (attention normaliser and bias extent)
    D: int
    H: int
    dqk: int
    dv: int
    eps: float
    activation: int     # 1 = silu, 0 = none
    dropout_p: float
    max_len: int        # host bound on sequence lengths (<= N)
    bf16: bool = False  # bf16 MFMA operands (HSTU autocast_dtype=bfloat16): attention, projections, weight grads
    concat_ua: bool = False  # o_in = [u, LN(a), u * LN(a)] (hstu.py:398-400)
    softmax: bool = False    # normalization="softmax_rel_bias" (hstu.py:341-389): fp32 layer

    @property
    def n_out(self):
        return 2 * self.H * self.dv + 2 * self.H * self.dqk

    @property
    def a16(self) -> bool:
        """bf16 activations in HBM (ABI 16, the ``*_a16`` entries): bf16 mode at wide
        heads, dqk == dv = d with d % 32 == 0 in (128, 256] (the ml-20m width)."""
        d = self.dqk
        return (A16 and self.bf16 and not self.concat_ua and not self.softmax and self.dqk == self.dv
                and 128 < d <= 256 and d % 32 == 0 and self.H * d <= 256)


# bf16 mode keeps the wide-head layer's activations (uvqk, h_pre, o_in, d_uvqk) in bf16
# (STUGeometry.a16); False = the fp32-activation bf16 path (A/B switch for tests and
# measurements)
A16 = True
# a16: each layer's gate_o epilogue computes the next layer's LayerNorm statistics
# (identical values), so LN + UVQK skips its statistics pass over x (A/B switch)
STATS_IN_EPILOGUE = True
_ZROWS: dict = {}


def _zero_row(device) -> torch.Tensor:
    """256 zero bf16 values (hstu_attn_fwd_a16's row for keys past a sequence)."""
    key = (device.type, device.index)
    z = _ZROWS.get(key)
    if z is None:
        z = torch.zeros(256, dtype=torch.bfloat16, device=device)
        _ZROWS[key] = z
    return z


def _cat_wide(hv: int, D: int) -> bool:
    """concat_ua beyond the LDS-resident row-wave form (hdv <= 64, D <= 128): o_in
    materialised and W_o streamed (hstu_gate_o_cat_wide_fwd / _bwd)."""
    return hv > 64 or D > 128


def _pad_cat_weight(w_o: torch.Tensor, hv: int):
    """concat_ua: _o.weight (D, 3 hv) -> (D, 3 hvp) with the u / LN(a) / u*LN(a) column
    blocks at 16-aligned offsets 0, hvp, 2 hvp (the row-wave kernel's k groups)."""
    hvp = 16 if hv <= 16 else (32 if hv <= 32 else 64)
    if hv > 64:
        raise NotImplementedError("concat_ua=True supports linear_dim * num_heads <= 64")
    D = w_o.shape[0]
    w = w_o.detach().reshape(D, 3, hv)
    pad = torch.zeros(D, 3, hvp, dtype=w_o.dtype, device=w_o.device)
    pad[:, :, :hv] = w
    return pad.reshape(D, 3 * hvp), hvp


def _stu_forward(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo: STUGeometry, seed: int,
                 seed_offset, grad_on: bool, needs_w_grad: bool, pre=None, next_w_uvqk=None,
                 images=None):
    """One STU layer forward (hstu.py:266-413): 3 launches.  Returns (y, saved, pre_next)
    with the tensors its backward needs (``_stu_backward``).
    Layer boundaries (``_fuse_boundaries``): ``pre`` = (x_stats, uvqk, h_pre) of this layer
    already made by the previous layer's hstu_boundary_fwd (the LN + UVQK launch is
    skipped); ``next_w_uvqk`` = the next layer's _uvqk: this layer's gate_o and the next
    layer's LN + UVQK run as one hstu_boundary_fwd launch, whose (x_stats, uvqk, h_pre) are
    returned as ``pre_next``."""
    dev = x.device
    rows, D = x.shape
    B = offsets.numel() - 1
    H, dv, dqk = geo.H, geo.dv, geo.dqk
    hv, hq = H * dv, H * dqk
    n_out = geo.n_out
    st = _stream()
    x = x.contiguous()
    w_uvqk = w_uvqk.contiguous()
    w_o = w_o.contiguous()
    sfx = "_bf16" if geo.bf16 else ""  # bf16 MFMA operands in the projections too
    if geo.a16:
        return _stu_forward_a16(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo, seed,
                                seed_offset, grad_on, needs_w_grad, pre, next_w_uvqk is not None,
                                images)
    if pre is not None:
        x_stats, uvqk, h_pre = pre
    else:
        x_stats, uvqk, h_pre = _ln_uvqk_outputs(rows, n_out, geo, grad_on, dev)
        _lib.call("hstu_ln_uvqk_fwd" + sfx, x.data_ptr(), x.stride(0), offsets.data_ptr(), B,
                  rows, D, w_uvqk.data_ptr(), n_out, geo.eps, geo.activation,
                  x_stats.data_ptr(), _lib.ptr(h_pre), uvqk.data_ptr(), n_out, st)
    attn = torch.empty(rows, hv, dtype=torch.float32, device=dev)
    q = uvqk[:, 2 * hv:2 * hv + hq]
    k = uvqk[:, 2 * hv + hq:]
    v = uvqk[:, hv:2 * hv]
    pos_w_c = pos_w.contiguous() if bmap is not None else None
    ts_w_c = ts_w.contiguous() if bmap is not None else None
    # wide bf16 heads: bf16 copies of Q, K, V that the attention kernels stage into LDS
    # by DMA, made once here and kept for the backward
    copies = None
    if geo.bf16 and n_out % 2 == 0:
        cb = _lib.lib().hstu_attn_bf16_copies_bytes(B, geo.N, H, dqk, dv)
        if cb:
            copies = torch.empty(cb, dtype=torch.uint8, device=dev)
            _lib.call("hstu_attn_bf16_copies", q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out,
                      n_out, offsets.data_ptr(), B, geo.N, H, dqk, dv, copies.data_ptr(), st)
    attn_args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out, n_out, offsets.data_ptr(), B,
                 geo.N, geo.max_len, H, dqk, dv, _lib.ptr(bmap), _lib.ptr(pos_w_c),
                 _lib.ptr(ts_w_c), NUM_BUCKETS, attn.data_ptr(), hv)
    if geo.bf16:
        _lib.call("hstu_attn_fwd_bf16", *attn_args, _lib.ptr(copies), st)
    elif geo.concat_ua:
        _lib.call("hstu_attn_fwd", *attn_args, st)
    attn_stats = torch.empty(rows, 2, dtype=torch.float32, device=dev)
    needs_w_grad = grad_on and needs_w_grad
    ow = 3 * hv if geo.concat_ua else hv  # o_in width
    cat_wide = geo.concat_ua and _cat_wide(hv, D)
    o_in = (torch.empty(rows, ow, dtype=torch.float32, device=dev)
            if needs_w_grad or cat_wide else None)
    w_pad = hvp = None
    if geo.concat_ua and not cat_wide:
        w_pad, hvp = _pad_cat_weight(w_o, hv)
    y = torch.empty(rows, D, dtype=torch.float32, device=dev)
    b_o_c = b_o.contiguous()
    pre_next = None
    if next_w_uvqk is not None and (geo.concat_ua or geo.bf16):
        raise ValueError("hstu_boundary_fwd: fp32, no concat_ua")
    if not geo.bf16 and not geo.concat_ua:
        # the attention and this layer's gate_o (+ the next layer's LN + UVQK: the layer
        # boundary) in one call; at narrow shapes the boundary runs as the attention
        # launch's epilogue (hstu_attn_fwd_bnd)
        bnd = GrBoundaryFwd(u=uvqk.data_ptr(), ld_u=n_out, max_rows=rows, hdv=hv, D=D,
                            w_o=w_o.data_ptr(), b_o=b_o_c.data_ptr(), x_res=x.data_ptr(),
                            ld_x=x.stride(0), eps=geo.eps, dropout_p=geo.dropout_p, seed=seed,
                            seed_offset=_lib.ptr(seed_offset), attn_stats=attn_stats.data_ptr(),
                            o_in=_lib.ptr(o_in), y=y.data_ptr(), ld_y=D)
        if next_w_uvqk is not None:
            w_next = next_w_uvqk.contiguous()
            pre_next = _ln_uvqk_outputs(rows, n_out, geo, grad_on, dev)
            nx_stats, nx_uvqk, nx_h_pre = pre_next
            bnd.w_uvqk = w_next.data_ptr()
            bnd.n_out = n_out
            bnd.activation = geo.activation
            bnd.x_stats = nx_stats.data_ptr()
            bnd.h_pre = _lib.ptr(nx_h_pre)
            bnd.uvqk = nx_uvqk.data_ptr()
            bnd.ld_out = n_out
        _lib.call("hstu_attn_fwd_bnd", *attn_args, ctypes.addressof(bnd), st)
    elif cat_wide:
        _lib.call("hstu_gate_o_cat_wide_fwd", uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
                  offsets.data_ptr(), B, rows, hv, D, w_o.data_ptr(), b_o_c.data_ptr(),
                  x.data_ptr(), x.stride(0), geo.eps, geo.dropout_p, seed,
                  _lib.ptr(seed_offset), attn_stats.data_ptr(), o_in.data_ptr(), y.data_ptr(),
                  D, st)
        if not needs_w_grad:
            o_in = None
    elif geo.concat_ua:
        _lib.call("hstu_gate_o_cat_fwd", uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
                  offsets.data_ptr(), B, rows, hv, hvp, D, w_pad.data_ptr(), b_o_c.data_ptr(),
                  x.data_ptr(), x.stride(0), geo.eps, geo.dropout_p, seed,
                  _lib.ptr(seed_offset), attn_stats.data_ptr(), _lib.ptr(o_in), y.data_ptr(),
                  D, st)
    else:  # bf16 mode
        _lib.call("hstu_gate_o_fwd" + sfx, uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
                  offsets.data_ptr(), B, rows, hv, D, w_o.data_ptr(), b_o_c.data_ptr(),
                  x.data_ptr(), x.stride(0), geo.eps, geo.dropout_p, seed,
                  _lib.ptr(seed_offset), attn_stats.data_ptr(), _lib.ptr(o_in), y.data_ptr(),
                  D, st)
    saved = (x, offsets, bmap, w_uvqk, w_o, pos_w_c, ts_w_c, x_stats, uvqk, h_pre, attn,
             attn_stats, o_in, copies if grad_on else None)
    return y, saved, pre_next


def weight_images_bf16(specs):
    """bf16 [N][K] weight images for the a16 projections (gr_weight_images_bf16, one launch):
    specs = [(fp32 2-D tensor, transpose)], returns the images."""
    import numpy as np
    outs, rows = [], []
    for w, tr in specs:
        w = w.detach()
        if not w.is_contiguous():
            w = w.contiguous()
        R, C = w.shape
        o = torch.empty((C, R) if tr else (R, C), dtype=torch.bfloat16, device=w.device)
        outs.append(o)
        rows.append((w.data_ptr(), R, C, 1 if tr else 0, o.data_ptr()))
    for c0 in range(0, len(rows), 32):  # up to 32 images per launch
        desc = np.ascontiguousarray(np.array(rows[c0:c0 + 32], dtype=np.int64))
        _lib.call("gr_weight_images_bf16", desc.ctypes.data, len(desc), _stream())
    return outs


def _a16_images(w_uvqk, w_o, grad_on: bool):
    """A layer's weight images: forward (W_uvqk^T, W_o) and, for the backward, (W_o^T,
    W_uvqk) -- the specs of weight_images_bf16."""
    specs = [(w_uvqk, True), (w_o, False)]
    if grad_on:
        specs += [(w_o, True), (w_uvqk, False)]
    return specs


def _stu_forward_a16(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo: STUGeometry, seed: int,
                     seed_offset, grad_on: bool, needs_w_grad: bool, pre=None, has_next=False,
                     images=None):
    """One STU layer forward with bf16 activations (ABI 16): LN + UVQK writes bf16 uvqk /
    h_pre (and the weight gradient's bf16 LN(x)), the attention DMAs Q / K / V from the
    bf16 uvqk rows, gate_o reads bf16 u and writes bf16 o_in.  The saved tuple's last
    slot holds xn (the fp32 path keeps its bf16 copies there).
    ``pre``: this layer's x_stats, computed by the previous layer's gate_o epilogue (the
    LN statistics pass is skipped); ``has_next``: compute the next layer's x_stats in this
    layer's gate_o epilogue (returned as the third value).  ``images``: the layer's bf16
    weight images (``_a16_images``; made here when None); the backward's two are saved in
    the tuple's weight slots."""
    dev = x.device
    rows, D = x.shape
    B = offsets.numel() - 1
    H, d = geo.H, geo.dqk
    hv = H * d
    n_out = geo.n_out
    st = _stream()
    x = x.contiguous()
    w_uvqk = w_uvqk.contiguous()
    w_o = w_o.contiguous()
    needs_w_grad = grad_on and needs_w_grad
    if images is None:
        images = weight_images_bf16(_a16_images(w_uvqk, w_o, grad_on))
    wt_uvqk, w_o16 = images[0], images[1]
    wt_o16, w_uvqk16 = (images[2], images[3]) if grad_on else (None, None)
    stats_given = pre is not None
    x_stats = pre if stats_given else torch.empty(rows, 2, dtype=torch.float32, device=dev)
    uvqk = torch.empty(rows, n_out, dtype=torch.bfloat16, device=dev)
    h_pre = torch.empty_like(uvqk) if geo.activation and grad_on else None
    xn = torch.empty(rows, D, dtype=torch.bfloat16, device=dev) if grad_on else None
    _lib.call("hstu_ln_uvqk_fwd_a16", x.data_ptr(), x.stride(0), offsets.data_ptr(), B, rows, D,
              wt_uvqk.data_ptr(), n_out, geo.eps, geo.activation, x_stats.data_ptr(),
              1 if stats_given else 0, _lib.ptr(h_pre), uvqk.data_ptr(), n_out, _lib.ptr(xn), st)
    attn = torch.empty(rows, hv, dtype=torch.float32, device=dev)
    pos_w_c = pos_w.contiguous() if bmap is not None else None
    ts_w_c = ts_w.contiguous() if bmap is not None else None
    _lib.call("hstu_attn_fwd_a16", uvqk[:, 2 * hv:].data_ptr(), uvqk[:, 3 * hv:].data_ptr(),
              uvqk[:, hv:].data_ptr(), n_out, offsets.data_ptr(), B, geo.N, geo.max_len, H, d,
              _lib.ptr(bmap), _lib.ptr(pos_w_c), _lib.ptr(ts_w_c), NUM_BUCKETS,
              _zero_row(dev).data_ptr(), attn.data_ptr(), hv, st)
    attn_stats = torch.empty(rows, 2, dtype=torch.float32, device=dev)
    o_in = torch.empty(rows, hv, dtype=torch.bfloat16, device=dev) if needs_w_grad else None
    y = torch.empty(rows, D, dtype=torch.float32, device=dev)
    b_o_c = b_o.contiguous()
    # the next layer's LN statistics from this gate_o's epilogue (one 256-column panel)
    y_stats = (torch.empty(rows, 2, dtype=torch.float32, device=dev)
               if has_next and STATS_IN_EPILOGUE and 240 < D <= 256 else None)
    _lib.call("hstu_gate_o_fwd_a16", uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
              offsets.data_ptr(), B, rows, hv, D, w_o16.data_ptr(), b_o_c.data_ptr(), x.data_ptr(),
              x.stride(0), geo.eps, geo.dropout_p, seed, _lib.ptr(seed_offset),
              attn_stats.data_ptr(), _lib.ptr(o_in), y.data_ptr(), D, _lib.ptr(y_stats), st)
    saved = (x, offsets, bmap, w_uvqk16, wt_o16, pos_w_c, ts_w_c, x_stats, uvqk, h_pre, attn,
             attn_stats, o_in, xn)
    return y, saved, y_stats


def _stu_backward_a16(saved, dy, geo: STUGeometry, seed: int, seed_offset, want_uvqk: bool,
                      defer_wgrad: bool):
    """The backward of ``_stu_forward_a16``: gate_o_bwd writes bf16 du into a bf16 d_uvqk,
    the attention backward its bf16 dq / dk / dv, ln_uvqk_bwd reads it, and the weight
    gradients take bf16 LN(x), d_uvqk and o_in (gr_wgrad_multi_a16)."""
    (x, offsets, bmap, w_uvqk16, wt_o16, pos_w, ts_w, x_stats, uvqk, h_pre, attn, attn_stats,
     o_in, xn) = saved  # the weight slots hold the backward's bf16 images
    dev = x.device
    rows, D = x.shape
    B = offsets.numel() - 1
    H, d = geo.H, geo.dqk
    hv = H * d
    n_out = geo.n_out
    st = _stream()
    dy = dy.contiguous()
    d_uvqk = torch.empty(rows, n_out, dtype=torch.bfloat16, device=dev)
    d_attn = torch.empty(rows, hv, dtype=torch.bfloat16, device=dev)
    _lib.call("hstu_gate_o_bwd_a16", dy.data_ptr(), D, offsets.data_ptr(), B, rows, hv, D,
              wt_o16.data_ptr(), uvqk.data_ptr(), n_out, attn.data_ptr(), hv, attn_stats.data_ptr(),
              _lib.ptr(h_pre), n_out, geo.dropout_p, seed, _lib.ptr(seed_offset),
              d_uvqk.data_ptr(), n_out, d_attn.data_ptr(), hv, st)
    L = _lib.lib()
    d_pos_w = d_ts_w = None
    if bmap is not None:
        d_pos_w = torch.empty(2 * geo.N - 1, dtype=torch.float32, device=dev)
        d_ts_w = torch.empty(NUM_BUCKETS + 1, dtype=torch.float32, device=dev)
    ws_n = L.hstu_attn_bwd_a16_workspace_size(B, geo.N, geo.max_len, H, d, NUM_BUCKETS)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
    hp = (lambda c: h_pre[:, c:].data_ptr()) if h_pre is not None else (lambda c: None)
    _lib.call("hstu_attn_bwd_a16", uvqk[:, 2 * hv:].data_ptr(), uvqk[:, 3 * hv:].data_ptr(),
              uvqk[:, hv:].data_ptr(), n_out, d_attn.data_ptr(), hv, offsets.data_ptr(), B, geo.N,
              geo.max_len, H, d, _lib.ptr(bmap), _lib.ptr(pos_w), _lib.ptr(ts_w), NUM_BUCKETS,
              hp(2 * hv), hp(3 * hv), hp(hv), n_out, d_uvqk[:, 2 * hv:].data_ptr(),
              d_uvqk[:, 3 * hv:].data_ptr(), d_uvqk[:, hv:].data_ptr(), n_out,
              _lib.ptr(d_pos_w), _lib.ptr(d_ts_w), _zero_row(dev).data_ptr(), ws.data_ptr(), ws_n, st)
    dx = torch.empty(rows, D, dtype=torch.float32, device=dev)
    _lib.call("hstu_ln_uvqk_bwd_a16", d_uvqk.data_ptr(), n_out, offsets.data_ptr(), B, rows, D,
              n_out, w_uvqk16.data_ptr(), x.data_ptr(), x.stride(0), x_stats.data_ptr(),
              dy.data_ptr(), D, dx.data_ptr(), D, st)
    d_w_uvqk = torch.empty(D, n_out, dtype=torch.float32, device=dev) if want_uvqk else None
    d_w_o = d_b_o = None
    if o_in is not None:
        d_w_o = torch.empty(D, hv, dtype=torch.float32, device=dev)
        d_b_o = torch.empty(D, dtype=torch.float32, device=dev)
    # gr_wgrad_multi_a16 rows {a, lda, a_stats, b, ldb, Ka, Nb, c, colsum, flags}
    problems = []
    if want_uvqk:
        problems.append(((xn.data_ptr(), D, 0, d_uvqk.data_ptr(), n_out, D, n_out,
                          d_w_uvqk.data_ptr(), 0, 3), (xn, d_uvqk)))
    if o_in is not None:
        problems.append(((dy.data_ptr(), D, 0, o_in.data_ptr(), hv, D, hv, d_w_o.data_ptr(),
                          d_b_o.data_ptr(), 2), (dy, o_in)))
    if not defer_wgrad:
        launch_wgrad_multi(problems, offsets, rows, True, a16=True)
        problems = []
    return dx, d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w, problems, None


def _ln_uvqk_outputs(rows, n_out, geo: STUGeometry, grad_on: bool, dev):
    """(x_stats, uvqk, h_pre) of one layer's LN + UVQK.  h_pre (pre-activation, for
    silu') exists only for the backward: inference / no_grad forwards skip its write."""
    x_stats = torch.empty(rows, 2, dtype=torch.float32, device=dev)
    uvqk = torch.empty(rows, n_out, dtype=torch.float32, device=dev)
    h_pre = torch.empty_like(uvqk) if geo.activation and grad_on else None
    return x_stats, uvqk, h_pre


def _stu_backward(saved, dy, geo: STUGeometry, seed: int, seed_offset, want_uvqk: bool,
                  defer_wgrad: bool = False, pre_d=None, prev=None):
    """One STU layer backward: gate_o_bwd, attention backward (+ bias reduce), ln_uvqk_bwd,
    then the two weight-gradient GEMMs (gr_wgrad2), or -- ``defer_wgrad`` -- their
    gr_wgrad_multi problem rows, left for the caller to launch with other layers'.
    Layer boundaries: ``pre_d`` = (d_uvqk, d_attn) already made by the next layer's
    hstu_boundary_bwd (gate_o_bwd is skipped); ``prev`` = (saved, seed) of the previous
    layer: this layer's ln_uvqk_bwd and the previous layer's gate_o_bwd run as one
    hstu_boundary_bwd launch, whose (d_uvqk, d_attn) are returned as ``pre_d_prev``.
    Returns (dx, d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w, problems, pre_d_prev)."""
    if geo.a16:
        return _stu_backward_a16(saved, dy, geo, seed, seed_offset, want_uvqk, defer_wgrad)
    (x, offsets, bmap, w_uvqk, w_o, pos_w, ts_w, x_stats, uvqk, h_pre, attn, attn_stats,
     o_in, copies) = saved
    dev = x.device
    rows, D = x.shape
    B = offsets.numel() - 1
    H, dv, dqk = geo.H, geo.dv, geo.dqk
    hv, hq = H * dv, H * dqk
    n_out = geo.n_out
    st = _stream()
    dy = dy.contiguous()
    if pre_d is not None:
        d_uvqk, d_attn = pre_d  # this layer's gate_o_bwd ran in the next layer's boundary
    else:
        d_uvqk = torch.empty(rows, n_out, dtype=torch.float32, device=dev)
        d_attn = torch.empty(rows, hv, dtype=torch.float32, device=dev)
    if pre_d is not None:
        pass
    elif geo.concat_ua and _cat_wide(hv, D):
        g_cat = torch.empty(rows, 3 * hv, dtype=torch.float32, device=dev)
        _lib.call("hstu_gate_o_cat_wide_bwd", dy.data_ptr(), D, offsets.data_ptr(), B, rows, hv,
                  D, w_o.data_ptr(), uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
                  attn_stats.data_ptr(), _lib.ptr(h_pre), n_out, geo.dropout_p, seed,
                  _lib.ptr(seed_offset), g_cat.data_ptr(), d_uvqk.data_ptr(), n_out,
                  d_attn.data_ptr(), hv, st)
        del g_cat
    elif geo.concat_ua:
        w_pad, hvp = _pad_cat_weight(w_o, hv)
        _lib.call("hstu_gate_o_cat_bwd", dy.data_ptr(), D, offsets.data_ptr(), B, rows, hv, hvp,
                  D, w_pad.data_ptr(), uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
                  attn_stats.data_ptr(), _lib.ptr(h_pre), n_out, geo.dropout_p, seed,
                  _lib.ptr(seed_offset), d_uvqk.data_ptr(), n_out, d_attn.data_ptr(), hv,
                  st)
    else:
        _lib.call("hstu_gate_o_bwd" + ("_bf16" if geo.bf16 else ""), dy.data_ptr(), D,
                  offsets.data_ptr(), B, rows, hv, D,
                  w_o.data_ptr(), uvqk.data_ptr(), n_out, attn.data_ptr(), hv,
                  attn_stats.data_ptr(), _lib.ptr(h_pre), n_out, geo.dropout_p, seed,
                  _lib.ptr(seed_offset), d_uvqk.data_ptr(), n_out, d_attn.data_ptr(), hv, st)
    L = _lib.lib()
    d_pos_w = d_ts_w = None
    ws_a = None
    ws_a_n = 0
    if bmap is not None:
        d_pos_w = torch.empty(2 * geo.N - 1, dtype=torch.float32, device=dev)
        d_ts_w = torch.empty(NUM_BUCKETS + 1, dtype=torch.float32, device=dev)
    # the workspace: bias slabs (with a map), the wide bf16 form's buffers and the wide
    # f32 form's dS tiles (with or without a map)
    if geo.bf16:
        ws_fn = (L.hstu_attn_bwd_bf16_workspace_size_copies if copies is not None else
                 L.hstu_attn_bwd_bf16_workspace_size)
        ws_a_n = ws_fn(B, geo.N, geo.max_len, H, dqk, dv, NUM_BUCKETS)
    elif bmap is not None or max(dqk, dv) > 128:
        # narrow f32 heads use the workspace (slabs, dS tiles) only with a bucket map
        ws_a_n = L.hstu_attn_bwd_workspace_size_d(B, geo.N, geo.max_len, H, dqk, dv, NUM_BUCKETS)
    if ws_a_n or bmap is not None:
        ws_a = torch.empty(max(ws_a_n, 4), dtype=torch.uint8, device=dev)
    q = uvqk[:, 2 * hv:2 * hv + hq]
    k = uvqk[:, 2 * hv + hq:]
    v = uvqk[:, hv:2 * hv]
    if h_pre is not None:
        hq_p = h_pre[:, 2 * hv:2 * hv + hq].data_ptr()
        hk_p = h_pre[:, 2 * hv + hq:].data_ptr()
        hv_p = h_pre[:, hv:2 * hv].data_ptr()
    else:
        hq_p = hk_p = hv_p = None
    dq = d_uvqk[:, 2 * hv:2 * hv + hq]
    dk = d_uvqk[:, 2 * hv + hq:]
    dvv = d_uvqk[:, hv:2 * hv]
    bwd_args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out, n_out,
                d_attn.data_ptr(), hv, offsets.data_ptr(), B, geo.N, geo.max_len, H, dqk, dv,
                _lib.ptr(bmap), _lib.ptr(pos_w), _lib.ptr(ts_w), NUM_BUCKETS,
                hq_p, hk_p, hv_p, n_out, dq.data_ptr(), dk.data_ptr(), dvv.data_ptr(), n_out,
                _lib.ptr(d_pos_w), _lib.ptr(d_ts_w))
    dx = torch.empty(rows, D, dtype=torch.float32, device=dev)
    pre_d_prev = None
    if prev is not None and (geo.concat_ua or geo.bf16):
        raise ValueError("hstu_boundary_bwd: fp32, no concat_ua")
    if geo.bf16:
        _lib.call("hstu_attn_bwd_bf16", *bwd_args, _lib.ptr(copies), _lib.ptr(ws_a), ws_a_n, st)
        _lib.call("hstu_ln_uvqk_bwd_bf16", d_uvqk.data_ptr(), n_out, offsets.data_ptr(), B, rows,
                  D, n_out, w_uvqk.data_ptr(), x.data_ptr(), x.stride(0), x_stats.data_ptr(),
                  dy.data_ptr(), D, dx.data_ptr(), D, st)
    else:
        # the attention backward and this layer's ln_uvqk_bwd (+ the previous layer's
        # gate_o_bwd: the layer boundary) in one call; at narrow shapes the boundary runs as
        # the epilogue of the dQ launch (hstu_attn_bwd_bnd)
        bnd = GrBoundaryBwd(dh=d_uvqk.data_ptr(), ld_dh=n_out, max_rows=rows, D=D, n_out=n_out,
                            w_uvqk=w_uvqk.data_ptr(), x=x.data_ptr(), ld_x=x.stride(0),
                            x_stats=x_stats.data_ptr(), dy_res=dy.data_ptr(), ld_dy=D,
                            dx=dx.data_ptr(), ld_dx=D)
        if prev is not None:
            (_, _, _, _, p_w_o, _, _, _, p_uvqk, p_h_pre, p_attn, p_attn_stats, _, _), p_seed = prev
            pre_d_prev = (torch.empty(rows, n_out, dtype=torch.float32, device=dev),
                          torch.empty(rows, hv, dtype=torch.float32, device=dev))
            bnd.hdv = hv
            bnd.w_o = p_w_o.data_ptr()
            bnd.u = p_uvqk.data_ptr()
            bnd.ld_u = n_out
            bnd.attn = p_attn.data_ptr()
            bnd.ld_attn = hv
            bnd.attn_stats = p_attn_stats.data_ptr()
            bnd.h_u = _lib.ptr(p_h_pre)
            bnd.ld_h = n_out
            bnd.dropout_p = geo.dropout_p
            bnd.seed = p_seed
            bnd.seed_offset = _lib.ptr(seed_offset)
            bnd.du = pre_d_prev[0].data_ptr()
            bnd.ld_du = n_out
            bnd.d_attn = pre_d_prev[1].data_ptr()
            bnd.ld_da = hv
        _lib.call("hstu_attn_bwd_bnd", *bwd_args, _lib.ptr(ws_a), ws_a_n, ctypes.addressof(bnd), st)
    # weight gradients (off the critical path): both GEMMs of the layer in one launch
    # and one slab reduce (gr_wgrad2), or deferred to the caller's gr_wgrad_multi
    d_w_uvqk = torch.empty(D, n_out, dtype=torch.float32, device=dev) if want_uvqk else None
    d_w_o = d_b_o = None
    ow = o_in.shape[1] if o_in is not None else hv  # 3 hv with concat_ua
    if o_in is not None:
        d_w_o = torch.empty(D, ow, dtype=torch.float32, device=dev)
        d_b_o = torch.empty(D, dtype=torch.float32, device=dev)
    problems = []
    if defer_wgrad:
        # rows of gr_wgrad_multi's descriptor {a, lda, a_stats, b, ldb, Ka, Nb, c, colsum}
        # plus the tensors that must stay alive until the launch
        if want_uvqk:
            problems.append(((x.data_ptr(), x.stride(0), x_stats.data_ptr(), d_uvqk.data_ptr(),
                              n_out, D, n_out, d_w_uvqk.data_ptr(), 0), (x, x_stats, d_uvqk)))
        if o_in is not None:
            problems.append(((dy.data_ptr(), D, 0, o_in.data_ptr(), ow, D, ow, d_w_o.data_ptr(),
                              d_b_o.data_ptr()), (dy, o_in)))
    elif want_uvqk and o_in is not None:
        ws_n = L.gr_wgrad2_workspace_size(rows, D, n_out, D, ow)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
        _lib.call("gr_wgrad2_bf16" if geo.bf16 else "gr_wgrad2", x.data_ptr(), x.stride(0),
                  x_stats.data_ptr(), d_uvqk.data_ptr(),
                  n_out, D, n_out, d_w_uvqk.data_ptr(), None,
                  dy.data_ptr(), D, None, o_in.data_ptr(), ow, D, ow, d_w_o.data_ptr(),
                  d_b_o.data_ptr(), offsets.data_ptr(), B, rows, ws.data_ptr(), ws_n, st)
    elif want_uvqk:
        ws_n = L.gr_wgrad_workspace_size(rows, D, n_out)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
        _lib.call("gr_wgrad", x.data_ptr(), x.stride(0), x_stats.data_ptr(), d_uvqk.data_ptr(),
                  n_out, offsets.data_ptr(), B, rows, D, n_out, d_w_uvqk.data_ptr(), None,
                  ws.data_ptr(), ws_n, st)
    elif o_in is not None:
        ws_n = L.gr_wgrad_workspace_size(rows, D, ow)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
        _lib.call("gr_wgrad", dy.data_ptr(), D, None, o_in.data_ptr(), ow, offsets.data_ptr(),
                  B, rows, D, ow, d_w_o.data_ptr(), d_b_o.data_ptr(), ws.data_ptr(), ws_n, st)
    return dx, d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w, problems, pre_d_prev


class STULayerFunction(torch.autograd.Function):
    """One SequentialTransductionUnitJagged (hstu.py:266-413) as 3 fused launches
    forward and 6 backward.  Inputs: jagged x (rows, D), offsets (B+1), the batch's
    bucket map (``bucket_map``) or None (no relative bias); parameters _uvqk (D, n_out), _o.weight (D, hdv), _o.bias (D,),
    _pos_w (2N-1,), _ts_w (129,)."""

    @staticmethod
    def forward(ctx, x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo: STUGeometry, seed: int,
                seed_offset, grad_on: bool = True, want_uvqk: bool = False):
        y, saved, _ = _stu_forward(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo, seed,
                                   seed_offset, grad_on, w_o.requires_grad or b_o.requires_grad)
        ctx.save_for_backward(*saved)
        ctx.geo = geo
        ctx.seed = seed
        ctx.seed_offset = seed_offset
        if want_uvqk:  # the layer's silu(LN(x) W_uvqk) rows, for the cache states
            uvqk = saved[8]
            ctx.mark_non_differentiable(uvqk)
            return y, uvqk
        return y

    @staticmethod
    def backward(ctx, dy, *_unused):
        dx, d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w, _, _ = _stu_backward(
            ctx.saved_tensors, dy, ctx.geo, ctx.seed, ctx.seed_offset, ctx.needs_input_grad[3])
        return (dx, None, None, d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w, None, None, None, None,
                None)


_SAVED_PER_LAYER = 14  # entries of _stu_forward's saved tuple

# layer boundaries of the stack as one launch each (hstu_boundary_fwd / _bwd); False =
# the two launches they replace (A/B switch for tests and measurements)
FUSE_BOUNDARIES = True


def _fuse_boundaries(geo: STUGeometry) -> bool:
    return FUSE_BOUNDARIES and not geo.bf16 and not geo.concat_ua


# weight gradients of layers L-1 .. 1 on a side stream, each launched as soon as its layer's
# backward is enqueued, so they run beside the later layers' critical-path kernels; layer
# 0's runs on the main stream, which is the join.  Measured slower at C2 (0.872 vs 0.795 ms
# per step, r4h: the side-stream GEMMs take the CUs the attention backward's tail would
# free and the launches no longer batch), so off by default: all layers' weight gradients
# in one launch at the end.
OVERLAP_WGRAD = False
_SIDE_STREAMS: dict = {}


def _side_stream(device):
    key = (device.type, device.index)
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _SIDE_STREAMS[key] = s
    return s


def launch_wgrad_multi(problems, offsets, rows, bf16: bool, a16: bool = False):
    """Launches the deferred weight-gradient problems (``_stu_backward(defer_wgrad=True)``)
    through gr_wgrad_multi (gr_wgrad_multi_a16 for the bf16-activation layout's 10-word
    rows), up to 16 per launch."""
    import numpy as np
    if not problems:
        return
    L = _lib.lib()
    B = offsets.numel() - 1
    dev = offsets.device
    for c0 in range(0, len(problems), 16):
        chunk = problems[c0:c0 + 16]
        desc = np.ascontiguousarray(np.array([p[0] for p in chunk], dtype=np.int64))
        n = len(chunk)
        if a16:
            ws_n = int(L.gr_wgrad_multi_a16_workspace_size(desc.ctypes.data, n, rows))
            ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
            _lib.call("gr_wgrad_multi_a16", desc.ctypes.data, n, offsets.data_ptr(), B, rows,
                      ws.data_ptr(), ws_n, _stream())
            continue
        ws_n = int(L.gr_wgrad_multi_workspace_size(desc.ctypes.data, n, rows))
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
        _lib.call("gr_wgrad_multi", desc.ctypes.data, n, offsets.data_ptr(), B, rows,
                  1 if bf16 else 0, ws.data_ptr(), ws_n, _stream())


class STUStackFunction(torch.autograd.Function):
    """Every STU layer of an encoder (HSTUJagged.jagged_forward's loop, hstu.py:467-478)
    as ONE autograd node.  Forward: the per-layer launches of ``_stu_forward``.  Backward:
    the per-layer critical path (gate_o_bwd, attention backward, ln_uvqk_bwd) layer by
    layer; each layer's two weight-gradient GEMMs as one gr_wgrad_multi launch on a side
    stream beside the later layers (``OVERLAP_WGRAD``), or all layers' in one launch at
    the end.
    params: per layer (_uvqk, _o.weight, _o.bias, _pos_w or None, _ts_w or None)."""

    @staticmethod
    def forward(ctx, x, offsets, bmap, geo: STUGeometry, seeds, seed_offset, grad_on: bool,
                *params):
        n_layers = len(seeds)
        saved_all = []
        fuse = _fuse_boundaries(geo)
        pre = None
        images = [None] * n_layers
        if geo.a16:  # every layer's bf16 weight images in one launch per 8 layers
            specs = [sp for l in range(n_layers)
                     for sp in _a16_images(params[5 * l], params[5 * l + 1], grad_on)]
            flat = weight_images_bf16(specs)
            per = len(specs) // n_layers
            images = [flat[per * l:per * (l + 1)] for l in range(n_layers)]
        for l in range(n_layers):
            w_uvqk, w_o, b_o, pos_w, ts_w = params[5 * l:5 * l + 5]
            # the next layer's _uvqk: the fp32 layer boundary (fuse) or, in the bf16
            # activation layout, "compute the next layer's LN statistics" (a16)
            nxt = params[5 * (l + 1)] if (fuse or geo.a16) and l + 1 < n_layers else None
            x, saved, pre = _stu_forward(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo,
                                         seeds[l], seed_offset, grad_on,
                                         w_o.requires_grad or b_o.requires_grad, pre, nxt,
                                         images[l])
            if grad_on:
                saved_all.extend(saved)
        if grad_on:
            ctx.save_for_backward(*saved_all)
        ctx.geo = geo
        ctx.seeds = seeds
        ctx.seed_offset = seed_offset
        return x

    @staticmethod
    def backward(ctx, dy):
        saved = ctx.saved_tensors
        geo = ctx.geo
        n_layers = len(ctx.seeds)
        grads = [None] * (5 * n_layers)
        problems = []
        offsets = saved[1]
        rows = saved[0].shape[0]
        fuse = _fuse_boundaries(geo)
        main = torch.cuda.current_stream(offsets.device)
        side = _side_stream(offsets.device) if OVERLAP_WGRAD and n_layers > 1 else None
        pre_d = None
        for l in reversed(range(n_layers)):
            sl = saved[_SAVED_PER_LAYER * l:_SAVED_PER_LAYER * (l + 1)]
            prev = None
            if fuse and l > 0:
                prev = (saved[_SAVED_PER_LAYER * (l - 1):_SAVED_PER_LAYER * l], ctx.seeds[l - 1])
            want_uvqk = ctx.needs_input_grad[7 + 5 * l]
            dx, d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w, probs, pre_d = _stu_backward(
                sl, dy, geo, ctx.seeds[l], ctx.seed_offset, want_uvqk, defer_wgrad=True,
                pre_d=pre_d, prev=prev)
            grads[5 * l:5 * l + 5] = [d_w_uvqk, d_w_o, d_b_o, d_pos_w, d_ts_w]
            if side is not None and l > 0 and probs:
                side.wait_stream(main)  # this layer's operands are enqueued on main
                with torch.cuda.stream(side):
                    launch_wgrad_multi(probs, offsets, rows, geo.bf16, geo.a16)
                for _, keep in probs:  # no reuse of their memory before the side stream ran
                    for t in keep:
                        t.record_stream(side)
            else:
                problems.extend(probs)
            dy = dx
        launch_wgrad_multi(problems, offsets, rows, geo.bf16, geo.a16)
        if side is not None:
            main.wait_stream(side)
        return (dy, None, None, None, None, None, None, *grads)


def stu_stack(x, offsets, bmap, layer_params, geo: STUGeometry, seeds, seed_offset=None):
    """All layers at once (``STUStackFunction``).  layer_params: per layer (_uvqk,
    _o.weight, _o.bias, _pos_w, _ts_w) with the bias tables None when bmap is None.
    Not for concat_ua (the per-layer ``stu_layer`` covers it)."""
    if geo.concat_ua:
        raise ValueError("stu_stack: concat_ua layers run through stu_layer")
    flat = [t for lp in layer_params for t in lp]
    _lib.require_gpu(x, offsets, *flat)
    if x.dtype != torch.float32:
        raise TypeError("stu_stack: float32 only (the reference runs fp32, hstu.py:592)")
    grad_on = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in [x] + flat)
    return STUStackFunction.apply(x, offsets, bmap, geo, tuple(int(s) for s in seeds),
                                  seed_offset, grad_on, *flat)


def stu_layer(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo: STUGeometry, seed: int = 0,
              seed_offset: Optional[torch.Tensor] = None, return_uvqk: bool = False):
    """bmap: ``bucket_map(...)`` of the batch, or None for no relative bias.
    Dropout masks hash (seed + *seed_offset, element); seed_offset is an optional device
    int64 counter (bumped per forward so that captured graphs draw fresh masks).
    ``return_uvqk``: also return the layer's (rows, n_out) u | v | q | k activations (no
    gradient; bf16 in the a16 mode), from which ``stu_cache_states`` builds the cache."""
    _lib.require_gpu(x, offsets, w_uvqk, w_o, b_o)
    if x.dtype != torch.float32:
        raise TypeError("stu_layer: float32 only (the reference runs fp32, hstu.py:592)")
    grad_on = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in (x, w_uvqk, w_o, b_o, pos_w, ts_w))
    return STULayerFunction.apply(x, offsets, bmap, w_uvqk, w_o, b_o, pos_w, ts_w, geo, int(seed),
                                  seed_offset, grad_on, bool(return_uvqk))


# ------------------------------------------------------------------ softmax_rel_bias layer

def _gate_forward(uvqk, attn, offsets, rows, x, geo: STUGeometry, w_o, b_o, seed, seed_offset,
                  attn_stats, want_o_in: bool):
    """The fp32 gate + O projection + residual (hstu.py:393-413) of ``rows`` rows; returns
    (y, o_in or None)."""
    dev = x.device
    B = offsets.numel() - 1
    hv, D, n_out = geo.H * geo.dv, geo.D, geo.n_out
    st = _stream()
    y = torch.empty(rows, D, dtype=torch.float32, device=dev)
    cat_wide = geo.concat_ua and _cat_wide(hv, D)
    ow = 3 * hv if geo.concat_ua else hv
    o_in = (torch.empty(rows, ow, dtype=torch.float32, device=dev)
            if want_o_in or cat_wide else None)
    head = (uvqk.data_ptr(), n_out, attn.data_ptr(), hv, offsets.data_ptr(), B, rows, hv)
    tail = (x.data_ptr(), x.stride(0), geo.eps, geo.dropout_p, seed, _lib.ptr(seed_offset),
            attn_stats.data_ptr(), _lib.ptr(o_in), y.data_ptr(), D, st)
    if not geo.concat_ua:
        _lib.call("hstu_gate_o_fwd", *head, D, w_o.data_ptr(), b_o.data_ptr(), *tail)
    elif cat_wide:
        _lib.call("hstu_gate_o_cat_wide_fwd", *head, D, w_o.data_ptr(), b_o.data_ptr(), *tail)
    else:
        w_pad, hvp = _pad_cat_weight(w_o, hv)
        _lib.call("hstu_gate_o_cat_fwd", *head, hvp, D, w_pad.data_ptr(), b_o.data_ptr(), *tail)
    return y, (o_in if want_o_in else None)


class SoftmaxSTULayerFunction(torch.autograd.Function):
    """One SequentialTransductionUnitJagged with normalization="softmax_rel_bias"
    (hstu.py:266-413 with the attention of :341-389), fp32: LN + UVQK + SiLU
    (hstu_ln_uvqk_fwd), the softmax attention (hstu_softmax_attn_fwd), the gate + O
    projection + residual (hstu_gate_o_fwd / _cat_).  ``bias`` is the (B, N, N) relative
    bias (``rel_bias``: its gradient flows back to _pos_w / _ts_w through that node) or
    None.  Backward: gate_o_bwd, hstu_softmax_attn_bwd (dQ / dK / dV with silu' and the bias
    gradient), ln_uvqk_bwd, the weight gradients (gr_wgrad2)."""

    @staticmethod
    def forward(ctx, x, offsets, bias, w_uvqk, w_o, b_o, geo: STUGeometry, seed: int,
                seed_offset, grad_on: bool, want_uvqk: bool):
        dev = x.device
        rows, D = x.shape
        B = offsets.numel() - 1
        H, dv, dqk = geo.H, geo.dv, geo.dqk
        hv, hq, n_out = H * dv, H * dqk, geo.n_out
        st = _stream()
        x = x.contiguous()
        w_uvqk = w_uvqk.contiguous()
        w_o = w_o.contiguous()
        b_o = b_o.contiguous()
        x_stats, uvqk, h_pre = _ln_uvqk_outputs(rows, n_out, geo, grad_on, dev)
        _lib.call("hstu_ln_uvqk_fwd", x.data_ptr(), x.stride(0), offsets.data_ptr(), B, rows, D,
                  w_uvqk.data_ptr(), n_out, geo.eps, geo.activation, x_stats.data_ptr(),
                  _lib.ptr(h_pre), uvqk.data_ptr(), n_out, st)
        bias_c = bias.detach().contiguous() if bias is not None else None
        if bias_c is not None and tuple(bias_c.shape) != (B, geo.N, geo.N):
            raise ValueError(f"softmax attention bias must be ({B}, {geo.N}, {geo.N})")
        attn = torch.empty(rows, hv, dtype=torch.float32, device=dev)
        sm_stats = torch.empty(rows, 2, dtype=torch.float32, device=dev)
        _lib.call("hstu_softmax_attn_fwd", uvqk[:, 2 * hv:].data_ptr(),
                  uvqk[:, 2 * hv + hq:].data_ptr(), n_out, uvqk[:, hv:].data_ptr(), n_out,
                  offsets.data_ptr(), B, geo.N, hq, hv, float(dqk) ** 0.5, _lib.ptr(bias_c),
                  attn.data_ptr(), hv, sm_stats.data_ptr(), st)
        attn_stats = torch.empty(rows, 2, dtype=torch.float32, device=dev)
        y, o_in = _gate_forward(uvqk, attn, offsets, rows, x, geo, w_o, b_o, seed, seed_offset,
                                attn_stats, grad_on)
        ctx.save_for_backward(x, offsets, bias_c, w_uvqk, w_o, x_stats, uvqk, h_pre, attn,
                              attn_stats, o_in, sm_stats)
        ctx.geo, ctx.seed, ctx.seed_offset = geo, seed, seed_offset
        if want_uvqk:
            ctx.mark_non_differentiable(uvqk)
            return y, uvqk
        return y

    @staticmethod
    def backward(ctx, dy, *_unused):
        (x, offsets, bias, w_uvqk, w_o, x_stats, uvqk, h_pre, attn, attn_stats, o_in,
         sm_stats) = ctx.saved_tensors
        geo, seed, seed_offset = ctx.geo, ctx.seed, ctx.seed_offset
        dev = x.device
        rows, D = x.shape
        B = offsets.numel() - 1
        H, dv, dqk = geo.H, geo.dv, geo.dqk
        hv, hq, n_out = H * dv, H * dqk, geo.n_out
        st = _stream()
        dy = dy.contiguous()
        d_uvqk = torch.empty(rows, n_out, dtype=torch.float32, device=dev)
        d_attn = torch.empty(rows, hv, dtype=torch.float32, device=dev)
        gate = (dy.data_ptr(), D, offsets.data_ptr(), B, rows, hv)
        mid = (uvqk.data_ptr(), n_out, attn.data_ptr(), hv, attn_stats.data_ptr(),
               _lib.ptr(h_pre), n_out, geo.dropout_p, seed, _lib.ptr(seed_offset))
        if not geo.concat_ua:
            _lib.call("hstu_gate_o_bwd", *gate, D, w_o.data_ptr(), *mid, d_uvqk.data_ptr(), n_out,
                      d_attn.data_ptr(), hv, st)
        elif _cat_wide(hv, D):
            g_cat = torch.empty(rows, 3 * hv, dtype=torch.float32, device=dev)
            _lib.call("hstu_gate_o_cat_wide_bwd", *gate, D, w_o.data_ptr(), *mid, g_cat.data_ptr(),
                      d_uvqk.data_ptr(), n_out, d_attn.data_ptr(), hv, st)
        else:
            w_pad, hvp = _pad_cat_weight(w_o, hv)
            _lib.call("hstu_gate_o_cat_bwd", *gate, hvp, D, w_pad.data_ptr(), *mid,
                      d_uvqk.data_ptr(), n_out, d_attn.data_ptr(), hv, st)
        want_bias = bias is not None and ctx.needs_input_grad[2]
        d_bias = torch.empty_like(bias) if want_bias else None
        L = _lib.lib()
        ws_n = L.hstu_softmax_attn_bwd_workspace_size(B, geo.N, 1 if want_bias else 0)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
        hp = (lambda c: h_pre[:, c:].data_ptr()) if h_pre is not None else (lambda c: None)
        _lib.call("hstu_softmax_attn_bwd", uvqk[:, 2 * hv:].data_ptr(),
                  uvqk[:, 2 * hv + hq:].data_ptr(), n_out, uvqk[:, hv:].data_ptr(), n_out,
                  offsets.data_ptr(), B, geo.N, hq, hv, float(dqk) ** 0.5, _lib.ptr(bias),
                  attn.data_ptr(), hv, sm_stats.data_ptr(), d_attn.data_ptr(), hv,
                  hp(2 * hv), hp(2 * hv + hq), hp(hv), n_out, d_uvqk[:, 2 * hv:].data_ptr(),
                  d_uvqk[:, 2 * hv + hq:].data_ptr(), d_uvqk[:, hv:].data_ptr(), n_out,
                  _lib.ptr(d_bias), ws.data_ptr(), ws_n, st)
        dx = torch.empty(rows, D, dtype=torch.float32, device=dev)
        _lib.call("hstu_ln_uvqk_bwd", d_uvqk.data_ptr(), n_out, offsets.data_ptr(), B, rows, D,
                  n_out, w_uvqk.data_ptr(), x.data_ptr(), x.stride(0), x_stats.data_ptr(),
                  dy.data_ptr(), D, dx.data_ptr(), D, st)
        d_w_uvqk = torch.empty(D, n_out, dtype=torch.float32, device=dev)
        ow = o_in.shape[1]
        d_w_o = torch.empty(D, ow, dtype=torch.float32, device=dev)
        d_b_o = torch.empty(D, dtype=torch.float32, device=dev)
        ws2_n = L.gr_wgrad2_workspace_size(rows, D, n_out, D, ow)
        ws2 = torch.empty(max(ws2_n, 4), dtype=torch.uint8, device=dev)
        _lib.call("gr_wgrad2", x.data_ptr(), x.stride(0), x_stats.data_ptr(), d_uvqk.data_ptr(),
                  n_out, D, n_out, d_w_uvqk.data_ptr(), None, dy.data_ptr(), D, None,
                  o_in.data_ptr(), ow, D, ow, d_w_o.data_ptr(), d_b_o.data_ptr(),
                  offsets.data_ptr(), B, rows, ws2.data_ptr(), ws2_n, st)
        return dx, None, d_bias, d_w_uvqk, d_w_o, d_b_o, None, None, None, None, None


def stu_softmax_layer(x, offsets, bias, w_uvqk, w_o, b_o, geo: STUGeometry, seed: int = 0,
                      seed_offset=None, return_uvqk: bool = False):
    """A normalization="softmax_rel_bias" layer (hstu.py:266-413, :341-389), fp32.
    ``bias``: ``rel_bias(timestamps, N, _pos_w, _ts_w)`` (differentiable) or None."""
    _lib.require_gpu(x, offsets, w_uvqk, w_o, b_o, bias)
    if x.dtype != torch.float32:
        raise TypeError("stu_softmax_layer: float32 only")
    if not geo.softmax:
        raise ValueError("stu_softmax_layer: geometry is not a softmax_rel_bias layer")
    grad_on = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in (x, w_uvqk, w_o, b_o, bias))
    return SoftmaxSTULayerFunction.apply(x, offsets, bias, w_uvqk, w_o, b_o, geo, int(seed),
                                         seed_offset, grad_on, bool(return_uvqk))


# ------------------------------------------------------------------ cached decoding

def stu_cache_states(uvqk: torch.Tensor, y: torch.Tensor, offsets: torch.Tensor, rows: int,
                     geo: STUGeometry):
    """The layer's cache states as the reference returns them with return_cache_states
    (hstu.py:420-423): (v (rows, H dv) jagged, padded q, padded k (B, N, H dqk),
    outputs (rows, D)), fp32, ``rows`` = offsets[B]."""
    hv, hq = geo.H * geo.dv, geo.H * geo.dqk
    u = uvqk[:rows]
    v = u[:, hv:2 * hv].float().contiguous()
    q = u[:, 2 * hv:2 * hv + hq].float().contiguous()
    k = u[:, 2 * hv + hq:].float().contiguous()
    with torch.no_grad():
        pq = jagged_to_padded_dense(q, offsets, geo.N)
        pk = jagged_to_padded_dense(k, offsets, geo.N)
    return v, pq, pk, y[:rows]


def check_decode_step(offsets: torch.Tensor, delta_rows: torch.Tensor, delta_pos: torch.Tensor,
                      N: int) -> bool:
    """The reference's cached step (hstu.py:151-177, 293-298) takes one delta entry per
    sequence (its flattened padded index is delta[1][e] + e * n) and indexes rows with
    index_copy_, which raises on an index out of range: the same conditions, checked here
    with one host synchronisation per step.  Returns whether the delta rows are distinct
    (then a layer's re-encoded rows are the next layer's input rows as they are)."""
    B = offsets.numel() - 1
    if delta_rows.numel() != B or delta_pos.numel() != B:
        raise ValueError(f"delta_x_offsets: {delta_rows.numel()} / {delta_pos.numel()} entries "
                         f"for {B} sequences (one per sequence, hstu.py:153-159)")
    srt = torch.sort(delta_rows)[0]
    flags = torch.stack([(delta_rows >= 0).all(), (delta_rows < offsets[-1]).all(),
                         (delta_pos >= 0).all(), (delta_pos < N).all(),
                         (srt[1:] != srt[:-1]).all()]).cpu()
    if not bool(flags[:4].all()):
        raise IndexError("delta_x_offsets: a row outside [0, offsets[B]) or a position "
                         f"outside [0, {N})")
    return bool(flags[4])


def stu_decode(x, offsets, timestamps, delta_rows, delta_pos, cache, w_uvqk, w_o, b_o, pos_w,
               ts_w, geo: STUGeometry, seed: int = 0, seed_offset=None, xd=None):
    """One cached step of a layer (hstu.py:293-298, 321-322, 151-177, 393-418), fp32:
    x (rows, D) jagged layer input, delta_rows / delta_pos the delta_x_offsets pair
    (validated by ``check_decode_step``), cache = (v, padded q, padded k, outputs) from a
    pass with return_cache_states, UPDATED IN PLACE as the reference's index_copy_ does.
    ``xd`` (optional): the rows x[delta_rows] when the caller has them (the previous
    layer's re-encoded rows, for distinct delta rows).  Launches: the row gather (unless
    ``xd``), LN + UVQK on the delta rows (hstu_decode_ln_uvqk, small-M tiles), the cache
    scatter (hstu_decode_scatter), the delta rows' attention (hstu_decode_attn: chunks +
    reduce), the gate + O projection (hstu_decode_gate_o without dropout / concat_ua,
    else the training kernels), the output scatter.  Returns (the updated outputs cache = the next layer's input,
    the re-encoded rows).  Forward only."""
    v_c, q_c, k_c, out_c = cache
    _lib.require_gpu(x, offsets, delta_rows, delta_pos, v_c, q_c, k_c, out_c, w_uvqk, w_o, b_o)
    dev = x.device
    B = offsets.numel() - 1
    E = delta_rows.numel()
    N, D, H, dqk, dv = geo.N, geo.D, geo.H, geo.dqk, geo.dv
    hv, hq, n_out = H * dv, H * dqk, geo.n_out
    for name, t, shape in (("v", v_c, (None, hv)), ("q", q_c, (B, N, hq)), ("k", k_c, (B, N, hq)),
                           ("outputs", out_c, (None, D))):
        want = tuple(t.shape[i] if s is None else s for i, s in enumerate(shape))
        if t.dtype != torch.float32 or tuple(t.shape) != want or not t.is_contiguous():
            raise ValueError(f"cache {name}: expected contiguous float32 {want}, got "
                             f"{t.dtype} {tuple(t.shape)}")
    if x.dtype != torch.float32 or x.dim() != 2 or x.shape[1] != D:
        raise ValueError(f"stu_decode: x must be (rows, {D}) float32")
    st = _stream()
    x = x.contiguous()
    rows_i = delta_rows.to(torch.int64).contiguous()
    pos_i = delta_pos.to(torch.int64).contiguous()
    if xd is None:
        xd = torch.empty(E, D, dtype=torch.float32, device=dev)
        _lib.call("gr_rows_copy", x.data_ptr(), D, rows_i.data_ptr(), 0, x.shape[0], xd.data_ptr(),
                  D, None, 0, E, E, D, st)
    off_d = torch.arange(E + 1, dtype=torch.int64, device=dev)
    uvqk = torch.empty(E, n_out, dtype=torch.float32, device=dev)
    w_uvqk = w_uvqk.detach().float().contiguous()
    if D <= 512:  # the small-M projection (16 rows x 16 columns per workgroup)
        _lib.call("hstu_decode_ln_uvqk", xd.data_ptr(), D, E, D, w_uvqk.data_ptr(), n_out, geo.eps,
                  geo.activation, uvqk.data_ptr(), n_out, st)
    else:
        x_stats = torch.empty(E, 2, dtype=torch.float32, device=dev)
        _lib.call("hstu_ln_uvqk_fwd", xd.data_ptr(), D, off_d.data_ptr(), E, E, D,
                  w_uvqk.data_ptr(), n_out, geo.eps, geo.activation, x_stats.data_ptr(), None,
                  uvqk.data_ptr(), n_out, st)
    # cache updates: v at the jagged rows, q / k at (e, delta_pos[e]) of the padded caches
    _lib.call("hstu_decode_scatter", uvqk.data_ptr(), n_out, hv, hq, rows_i.data_ptr(),
              pos_i.data_ptr(), E, N, v_c.data_ptr(), v_c.shape[0], q_c.data_ptr(), k_c.data_ptr(),
              B * N, st)
    attn = torch.empty(E, hv, dtype=torch.float32, device=dev)
    bias = timestamps is not None and pos_w is not None and ts_w is not None
    ts = pw = tw = thr = None
    if bias:
        ts = timestamps.to(torch.int64).contiguous()
        if tuple(ts.shape) != (B, N):
            raise ValueError(f"timestamps must be ({B}, {N}), got {tuple(ts.shape)}")
        pw = pos_w.detach().float().contiguous()
        tw = ts_w.detach().float().contiguous()
        thr = bucket_thresholds(dev)
    ws_n = _lib.lib().hstu_decode_attn_workspace_size(E, N, H, dv)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
    _lib.call("hstu_decode_attn", q_c.data_ptr(), k_c.data_ptr(), hq, v_c.data_ptr(), hv,
              v_c.shape[0], offsets.data_ptr(), B, rows_i.data_ptr(), E, N, H, dqk, dv,
              _lib.ptr(ts), _lib.ptr(thr), NUM_BUCKETS, _lib.ptr(pw), _lib.ptr(tw),
              attn.data_ptr(), hv, ws.data_ptr(), ws_n, st)
    y = torch.empty(E, D, dtype=torch.float32, device=dev)
    attn_stats = torch.empty(E, 2, dtype=torch.float32, device=dev)
    w_o = w_o.detach().float().contiguous()
    b_o = b_o.detach().float().contiguous()
    gate_args = (uvqk.data_ptr(), n_out, attn.data_ptr(), hv, off_d.data_ptr(), E, E, hv)
    tail = (xd.data_ptr(), D, geo.eps, geo.dropout_p, seed, _lib.ptr(seed_offset),
            attn_stats.data_ptr())
    # the small-M gate at wide rows; narrow rows (D <= 64: ml-1m) keep the row-wave kernel
    if not geo.concat_ua and geo.dropout_p == 0 and hv <= 256 and D > 64:
        _lib.call("hstu_decode_gate_o", uvqk.data_ptr(), n_out, attn.data_ptr(), hv, E, hv, D,
                  w_o.data_ptr(), b_o.data_ptr(), xd.data_ptr(), D, geo.eps, y.data_ptr(), D, st)
    elif not geo.concat_ua:
        _lib.call("hstu_gate_o_fwd", *gate_args, D, w_o.data_ptr(), b_o.data_ptr(), *tail, None,
                  y.data_ptr(), D, st)
    elif _cat_wide(hv, D):
        o_in = torch.empty(E, 3 * hv, dtype=torch.float32, device=dev)
        _lib.call("hstu_gate_o_cat_wide_fwd", *gate_args, D, w_o.data_ptr(), b_o.data_ptr(), *tail,
                  o_in.data_ptr(), y.data_ptr(), D, st)
    else:
        w_pad, hvp = _pad_cat_weight(w_o, hv)
        _lib.call("hstu_gate_o_cat_fwd", *gate_args, hvp, D, w_pad.data_ptr(), b_o.data_ptr(),
                  *tail, None, y.data_ptr(), D, st)
    _lib.call("gr_rows_copy", y.data_ptr(), D, None, 0, E, out_c.data_ptr(), D, rows_i.data_ptr(),
              0, out_c.shape[0], E, D, st)
    return out_c, y


# ------------------------------------------------------------------ sampled-softmax loss

class _SampledSoftmax(torch.autograd.Function):
    """Per-token sampled-softmax loss (``gr_sampled_softmax_fwd`` / ``_bwd``).

    Differentiable inputs: ``out`` (M, D) query rows, ``pos`` (M, D) normalised positive
    rows, ``table`` (V, D) normalised catalog rows.  ``offsets`` (M, R) index ``table``;
    ``all_ids`` (V,) maps an offset to its item id for the collision mask."""

    @staticmethod
    def forward(ctx, out, pos, table, sup_ids, offsets, all_ids, temperature):
        M, D = out.shape
        V = table.shape[0]
        R = offsets.shape[1] if offsets.dim() == 2 else 0
        out_c, pos_c, table_c = out.contiguous(), pos.contiguous(), table.contiguous()
        sup = sup_ids.to(torch.int64).contiguous()
        offs = offsets.to(torch.int64).contiguous()
        ids = all_ids.to(torch.int64).contiguous() if all_ids is not None else None
        loss = torch.empty(M, dtype=torch.float32, device=out.device)
        lse = torch.empty(M, dtype=torch.float32, device=out.device)
        _lib.call("gr_sampled_softmax_fwd", out_c.data_ptr(), D, pos_c.data_ptr(), D,
                  sup.data_ptr(), table_c.data_ptr(), D, V,
                  ids.data_ptr() if ids is not None else None, offs.data_ptr(), M, R, D,
                  float(temperature), loss.data_ptr(), lse.data_ptr(), _stream())
        ctx.save_for_backward(out_c, pos_c, table_c, sup, offs, lse)
        ctx.ids = ids
        ctx.meta = (M, R, D, V, float(temperature))
        return loss

    @staticmethod
    def backward(ctx, dloss):
        out_c, pos_c, table_c, sup, offs, lse = ctx.saved_tensors
        M, R, D, V, temperature = ctx.meta
        g = dloss.to(torch.float32).contiguous()
        d_out = torch.empty_like(out_c)
        d_pos = torch.empty_like(pos_c)
        d_table = torch.empty_like(table_c)
        ids = ctx.ids
        ws_n = _lib.lib().gr_sampled_softmax_workspace_size(M, R, V, D)
        ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=out_c.device)
        _lib.call("gr_sampled_softmax_bwd", out_c.data_ptr(), D, pos_c.data_ptr(), D,
                  sup.data_ptr(), table_c.data_ptr(), D, V,
                  ids.data_ptr() if ids is not None else None, offs.data_ptr(), M, R, D,
                  temperature, lse.data_ptr(), g.data_ptr(), d_out.data_ptr(), D,
                  d_pos.data_ptr(), D, d_table.data_ptr(), D, ws.data_ptr(), ws.numel(),
                  _stream())
        if M * R > 0:  # the backward's status word (device), read by last_sampled_softmax_status
            off = int(_lib.lib().gr_sampled_softmax_status_offset(M, R, V, D))
            global _LAST_SSM_STATUS
            _LAST_SSM_STATUS = ws[off:off + 4]
        return d_out, d_pos, d_table, None, None, None, None


_LAST_SSM_STATUS = None


def last_sampled_softmax_status() -> int:
    """Status word of the most recent sampled-softmax backward (host sync): 0 = clean;
    bit 0 / bit 1 = samples dropped by the counting sort's bound checks."""
    if _LAST_SSM_STATUS is None:
        return 0
    return int(_LAST_SSM_STATUS.view(torch.int32).item())


def sampled_softmax_loss(out: torch.Tensor, pos: torch.Tensor, table: torch.Tensor,
                         sup_ids: torch.Tensor, offsets: torch.Tensor,
                         all_ids: Optional[torch.Tensor], temperature: float) -> torch.Tensor:
    """(M,) per-token ``-log_softmax(cat[pos, neg])[:, 0]`` of
    autoregressive_losses.py:259-305, the negatives being ``table[offsets]``."""
    _lib.require_gpu(out, pos, table, sup_ids, offsets, all_ids)
    for name, t in (("out", out), ("pos", pos), ("table", table)):
        if t.dtype != torch.float32 or t.dim() != 2:
            raise TypeError(f"sampled_softmax_loss: {name} must be a 2-D float32 tensor")
    M, D = out.shape
    if pos.shape != (M, D) or table.shape[1] != D:
        raise ValueError(f"sampled_softmax_loss: shapes out {tuple(out.shape)}, pos "
                         f"{tuple(pos.shape)}, table {tuple(table.shape)} disagree")
    if D > 256:
        raise ValueError("sampled_softmax_loss: D <= 256")
    if sup_ids.shape != (M,) or offsets.dim() != 2 or offsets.shape[0] != M:
        raise ValueError("sampled_softmax_loss: sup_ids (M,) and offsets (M, R) expected")
    if all_ids is not None and all_ids.shape != (table.shape[0],):
        raise ValueError("sampled_softmax_loss: all_ids must have one id per table row")
    return _SampledSoftmax.apply(out, pos, table, sup_ids, offsets, all_ids, float(temperature))
