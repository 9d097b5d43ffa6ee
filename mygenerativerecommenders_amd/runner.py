"""No-Lightning runner for the retrieval model's step logic.

It restates, module for module, what the reference LightningModule does around the hot
path, so the drop-ins can be driven (and tested) in the reference's own calling order:

* ``seq_features_from_row``   utils/features.py:20-84 (padding by max_output_length,
                              target timestamp scattered at position ``length``);
* ``RetrievalRunner.forward`` generative_recommenders.py:355-393 (preprocessor ->
                              sequence encoder -> postprocessor);
* ``dense_to_jagged``         generative_recommenders.py:395-430 (ids through float);
* ``training_step``           retrieval.py:49-160 (target id scattered into past_ids,
                              the ``[:, :-1]`` / ``[:, 1:]`` shift, local negatives,
                              zero_grad / backward / step);
* ``retrieve``                retrieval.py:19-47 (``torch.inference_mode``);
* ``on_validation_epoch_start`` / ``validation_step`` / ``on_validation_epoch_end``
                              retrieval.py:162-210.

Lightning's logging, schedulers and hooks are not restated (out of scope); every
tensor op on the path runs through this package's HIP kernels.
"""
from __future__ import annotations

from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple

import torch

from . import ops

_ROW_KEYS = ("history_lengths", "historical_ids", "historical_ratings", "historical_years",
             "historical_timestamps", "target_ids", "target_ratings", "target_years",
             "target_timestamps")


class SequentialFeatures(NamedTuple):
    """utils/features.py:6-17."""
    past_lengths: torch.Tensor
    past_ids: torch.Tensor
    past_years: torch.Tensor
    past_embeddings: Optional[torch.Tensor]
    past_payloads: Dict[str, torch.Tensor]


def seq_features_from_row(row: Dict[str, torch.Tensor], device: torch.device,
                          max_output_length: int
                          ) -> Tuple[SequentialFeatures, torch.Tensor, torch.Tensor]:
    """utils/features.py:20-84: (features, target_ids (B, 1), target_ratings (B, 1))."""
    lengths = row["history_lengths"].to(device)
    ids = row["historical_ids"].to(device)
    ratings = row["historical_ratings"].to(device)
    ts = row["historical_timestamps"].to(device)
    years = row["historical_years"].to(device)
    target_ids = row["target_ids"].to(device).unsqueeze(1)
    target_ratings = row["target_ratings"].to(device).unsqueeze(1)
    target_ts = row["target_timestamps"].to(device).unsqueeze(1)
    if max_output_length > 0:
        B = lengths.size(0)

        def pad(t):
            return torch.cat([t, t.new_zeros(B, max_output_length)], dim=1)
        ids, ratings, years, ts = pad(ids), pad(ratings), pad(years), pad(ts)
        ts.scatter_(1, lengths.view(-1, 1), target_ts.view(-1, 1))
    extra = {k: v.to(device) for k, v in row.items() if k not in _ROW_KEYS}
    feats = SequentialFeatures(past_lengths=lengths, past_ids=ids, past_years=years,
                               past_embeddings=None,
                               past_payloads={"timestamps": ts, "ratings": ratings, **extra})
    return feats, target_ids, target_ratings


class RetrievalRunner:
    """The Retrieval module's steps over this package's drop-in modules.

    ``gr_output_length`` is the model's output length (configs: 10); rows are padded by
    ``gr_output_length + 1`` as retrieval.py:79-83 does.  ``optimizers`` is a list (the
    reference's Muon + AdamW pair, or one optimizer, or empty for gradients only)."""

    def __init__(self, embeddings, preprocessor, sequence_encoder, postprocessor, similarity,
                 negatives_sampler, candidate_index, loss, metrics, gr_output_length: int,
                 optimizers: Sequence[torch.optim.Optimizer] = ()) -> None:
        self.embeddings = embeddings
        self.preprocessor = preprocessor
        self.sequence_encoder = sequence_encoder
        self.postprocessor = postprocessor
        self.similarity = similarity
        self.negatives_sampler = negatives_sampler
        self.candidate_index = candidate_index
        self.loss = loss
        self.metrics = metrics
        self.gr_output_length = gr_output_length
        self.optimizers: List[torch.optim.Optimizer] = list(optimizers)

    @property
    def device(self) -> torch.device:
        return self.candidate_index.ids.device

    # ---------------------------------------------------- generative_recommenders.py
    def forward(self, seq_features: SequentialFeatures) -> Tuple[torch.Tensor, object]:
        past_lengths, user_embeddings, valid_mask, aux_mask = self.preprocessor(
            past_lengths=seq_features.past_lengths, past_ids=seq_features.past_ids,
            past_embeddings=seq_features.past_embeddings,
            past_payloads=seq_features.past_payloads)
        user_embeddings, cached = self.sequence_encoder(
            past_lengths=past_lengths, user_embeddings=user_embeddings, valid_mask=valid_mask,
            past_payloads=seq_features.past_payloads)
        if aux_mask is not None:  # no preprocessor on the path produces one
            raise NotImplementedError("aux_mask (mask_dense_by_aux_mask) is not on the path")
        return self.postprocessor(user_embeddings), cached

    @staticmethod
    def dense_to_jagged(lengths: torch.Tensor, **kwargs) -> Dict[str, torch.Tensor]:
        """generative_recommenders.py:395-430; exact-size outputs (one host read of the
        total, as the reference's op returns an exact-size tensor)."""
        offsets = ops.asynchronous_complete_cumsum(lengths)
        total = int(offsets[-1].item())
        out = {}
        if "supervision_ids" in kwargs:  # ids travel as float32, exact below 2**24
            ids = kwargs.pop("supervision_ids")
            if ids.numel() and int(ids.max().item()) >= 1 << 24:
                raise ValueError("dense_to_jagged: ids >= 2**24 are not exact in float32")
            out["supervision_ids"] = ops.dense_to_jagged(
                ids.unsqueeze(-1).float().contiguous(), offsets, total).squeeze(1).long()
        if "supervision_weights" in kwargs:
            out["supervision_weights"] = ops.dense_to_jagged(
                kwargs.pop("supervision_weights").unsqueeze(-1).contiguous(), offsets,
                total).squeeze(1)
        for key, value in kwargs.items():
            out[key] = ops.dense_to_jagged(value.contiguous(), offsets, total)
        return out

    # ---------------------------------------------------------------- retrieval.py
    @torch.inference_mode()
    def retrieve(self, seq_features: SequentialFeatures, filter_past_ids: bool = True
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
        seq_embeddings, _ = self.forward(seq_features)
        current = ops.get_current_embeddings(seq_features.past_lengths, seq_embeddings)
        if self.candidate_index.embeddings is None:
            self.candidate_index.update_embeddings(self.negatives_sampler.normalize_embeddings(
                self.embeddings.get_item_embeddings(self.candidate_index.ids)))
        return self.candidate_index.get_top_k_outputs(
            query_embeddings=current,
            invalid_ids=(seq_features.past_ids if filter_past_ids else None))

    def training_step(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        seq_features, target_ids, _ = seq_features_from_row(
            batch, device=self.device, max_output_length=self.gr_output_length + 1)
        seq_features.past_ids.scatter_(1, seq_features.past_lengths.view(-1, 1),
                                       target_ids.view(-1, 1))
        input_embeddings = self.embeddings.get_item_embeddings(seq_features.past_ids)
        seq_features = seq_features._replace(past_embeddings=input_embeddings)
        seq_embeddings, _ = self.forward(seq_features)
        supervision_ids = seq_features.past_ids
        # the local sampler draws from the live embedding module (retrieval.py:110-116)
        self.negatives_sampler._embeddings_module = self.embeddings
        jagged = self.dense_to_jagged(
            lengths=seq_features.past_lengths,
            output_embeddings=seq_embeddings[:, :-1, :],
            supervision_ids=supervision_ids[:, 1:],
            supervision_embeddings=input_embeddings[:, 1:, :],
            supervision_weights=(supervision_ids[:, 1:] != 0).float())
        loss = self.loss.jagged_forward(negatives_sampler=self.negatives_sampler,
                                        similarity=self.similarity, **jagged)
        for opt in self.optimizers:
            opt.zero_grad()
        loss.backward()
        for opt in self.optimizers:
            opt.step()
        return loss

    def on_validation_epoch_start(self) -> None:
        self.metrics.reset()
        with torch.inference_mode():  # Lightning runs validation hooks in inference mode
            self.candidate_index.update_embeddings(self.negatives_sampler.normalize_embeddings(
                self.embeddings.get_item_embeddings(self.candidate_index.ids)))

    def validation_step(self, batch: Dict[str, torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        with torch.inference_mode():
            seq_features, target_ids, _ = seq_features_from_row(
                batch, device=self.device, max_output_length=self.gr_output_length + 1)
            input_embeddings = self.embeddings.get_item_embeddings(seq_features.past_ids)
            seq_features = seq_features._replace(past_embeddings=input_embeddings)
            top_k_ids, top_k_scores = self.retrieve(seq_features)
            self.metrics.update(top_k_ids=top_k_ids, target_ids=target_ids)
        return top_k_ids, top_k_scores

    def on_validation_epoch_end(self) -> Dict[str, torch.Tensor]:
        results = self.metrics.compute()
        self.metrics.reset()
        return results
