"""Input-features preprocessors — drop-in for reference ``models/preprocessors``
(Hydra ``_target_: ...preprocessors.LearnablePositionalEmbeddingInputFeaturesPreprocessor``),
SURVEY §8 N2.

``LearnablePositionalEmbeddingInputFeaturesPreprocessor`` (learnable_positional_embedding.py:
12-58) computes ``dropout(x * sqrt(D) + pos_emb[n]) * (past_ids != 0)`` with one fused
kernel forward (``gr_preproc_fwd``) and one pair backward (``gr_preproc_bwd``: dx and the
positional-table gradient, deterministic).  Dropout draws from the library's counter hash
(seed + a device step counter), not from PyTorch's generator: with dropout off (eval,
or p = 0) the output equals the reference's exactly; with it on, the mask has the same
distribution (keep probability 1 - p, scale 1/(1-p)).
"""
from __future__ import annotations

import abc
import math
from typing import Dict, Optional, Tuple

import torch

from . import _lib


def _stream():
    return _lib.stream_handle()


class InputFeaturesPreprocessorModule(torch.nn.Module):
    """preprocessors/__init__.py (base.py): the abstract preprocessor interface."""

    @abc.abstractmethod
    def debug_str(self) -> str:
        pass

    @abc.abstractmethod
    def forward(self, past_lengths: torch.Tensor, past_ids: torch.Tensor,
                past_embeddings: torch.Tensor, past_payloads: Dict[str, torch.Tensor]):
        pass


class _Preproc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos_w, ids, scale, p, seed, step):
        B, N, D = x.shape
        xc = x.contiguous()
        y = torch.empty_like(xc)
        _lib.call("gr_preproc_fwd", xc.data_ptr(), ids.data_ptr(), pos_w.data_ptr(), B, N, D,
                  scale, p, seed, step.data_ptr() if step is not None else None, y.data_ptr(),
                  _stream())
        ctx.save_for_backward(ids, step if step is not None else torch.empty(0))
        ctx.meta = (B, N, D, scale, p, seed, step is not None, pos_w.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, step = ctx.saved_tensors
        B, N, D, scale, p, seed, has_step, pos_shape = ctx.meta
        g = dy.contiguous()
        dx = torch.empty_like(g) if ctx.needs_input_grad[0] else None
        dpos = None
        if ctx.needs_input_grad[1]:  # the kernel writes rows < N; rows >= N get no gradient
            dpos = torch.empty(pos_shape, dtype=g.dtype, device=g.device)
            if pos_shape[0] > N:
                dpos[N:].zero_()
        _lib.call("gr_preproc_bwd", g.data_ptr(), ids.data_ptr(), B, N, D, scale, p, seed,
                  step.data_ptr() if has_step else None,
                  dx.data_ptr() if dx is not None else None,
                  dpos.data_ptr() if dpos is not None else None, _stream())
        return dx, dpos, None, None, None, None, None


def preprocess(x: torch.Tensor, pos_w: torch.Tensor, past_ids: torch.Tensor, scale: float,
               dropout_p: float = 0.0, seed: int = 0,
               step: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dropout(x * scale + pos_w[:N]) * (past_ids != 0) for x (B, N, D) fp32."""
    _lib.require_gpu(x, pos_w, past_ids)
    if x.dtype != torch.float32 or pos_w.dtype != torch.float32:
        raise TypeError("preprocess: float32 only")
    B, N, D = x.shape
    if past_ids.shape != (B, N) or pos_w.dim() != 2 or pos_w.shape[0] < N or pos_w.shape[1] != D:
        raise ValueError(f"preprocess: x {tuple(x.shape)}, past_ids {tuple(past_ids.shape)}, "
                         f"pos_w {tuple(pos_w.shape)} disagree")
    ids = past_ids.to(torch.int64).contiguous()
    return _Preproc.apply(x, pos_w, ids, float(scale), float(dropout_p), int(seed), step)


def _truncated_normal_(t: torch.Tensor, mean: float, std: float) -> None:
    """utils/initialization.py truncated_normal: N(mean, std) resampled outside 2 std."""
    with torch.no_grad():
        torch.nn.init.trunc_normal_(t, mean=mean, std=std, a=mean - 2 * std, b=mean + 2 * std)


class LearnablePositionalEmbeddingInputFeaturesPreprocessor(InputFeaturesPreprocessorModule):
    """learnable_positional_embedding.py:12-58."""

    def __init__(self, max_sequence_len: int, embedding_dim: int, dropout_rate: float) -> None:
        super().__init__()
        self._embedding_dim: int = embedding_dim
        self._pos_emb = torch.nn.Embedding(max_sequence_len, self._embedding_dim)
        self._dropout_rate: float = dropout_rate
        self._dropout_seed = int(torch.randint(0, 2**62, (1,)).item())
        self.register_buffer("_dropout_step", torch.zeros(1, dtype=torch.int64), persistent=False)
        self.reset_state()

    def debug_str(self) -> str:
        return f"posi_d{self._dropout_rate}"

    def reset_state(self) -> None:
        _truncated_normal_(self._pos_emb.weight.data, mean=0.0,
                           std=math.sqrt(1.0 / self._embedding_dim))

    def forward(self, past_lengths: torch.Tensor, past_ids: torch.Tensor,
                past_embeddings: torch.Tensor, past_payloads: Dict[str, torch.Tensor]
                ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, None]:
        p = self._dropout_rate if self.training else 0.0
        step = None
        if p > 0.0:
            with torch.no_grad():
                self._dropout_step.add_(1)
            step = self._dropout_step.clone()  # this forward's mask, whatever runs next
        user_embeddings = preprocess(past_embeddings, self._pos_emb.weight, past_ids,
                                     self._embedding_dim ** 0.5, p, self._dropout_seed, step)
        valid_mask = (past_ids != 0).unsqueeze(-1).float()
        return past_lengths, user_embeddings, valid_mask, None
