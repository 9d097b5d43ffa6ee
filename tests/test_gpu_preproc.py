"""GPU parity of the fused input preprocessor (SURVEY §8 N2,
learnable_positional_embedding.py:42-58) against the reference's recorded outputs
(tests/golden/preproc.npz, dropout off) and the numpy oracle at ml-1m C2 shape; with
dropout on, the keep rate / scale and the forward-backward mask agreement.
Tolerance: fp32, 1e-6 relative (one fused multiply-add vs two roundings)."""
import os

import numpy as np
import pytest
import torch

from oracle import preproc_oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _module(max_len, D, p, pos_w=None):
    from mygenerativerecommenders_amd.preprocessors import (
        LearnablePositionalEmbeddingInputFeaturesPreprocessor as Pre)
    m = Pre(max_sequence_len=max_len, embedding_dim=D, dropout_rate=p).cuda()
    if pos_w is not None:
        with torch.no_grad():
            m._pos_emb.weight.copy_(torch.as_tensor(pos_w))
    return m


def test_preproc_matches_reference_golden():
    z = np.load(os.path.join(GOLDEN, "preproc.npz"))
    B, N, D = z["x"].shape
    m = _module(z["pos_w"].shape[0], D, 0.2, z["pos_w"]).eval()
    x = torch.from_numpy(z["x"]).cuda().requires_grad_(True)
    ids = torch.from_numpy(z["ids"]).cuda()
    lengths, y, valid, _ = m((ids != 0).sum(1), ids, x, {})
    (y * torch.from_numpy(z["dy"]).cuda()).sum().backward()
    assert np.allclose(y.detach().cpu().numpy(), z["y"], rtol=1e-6, atol=1e-6)
    assert np.array_equal(valid.cpu().numpy(), z["valid"])
    assert np.allclose(x.grad.cpu().numpy(), z["dx"], rtol=1e-6, atol=1e-6)
    assert np.allclose(m._pos_emb.weight.grad.cpu().numpy(), z["dpos"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B", [1, 17, 128, 150, 300])  # 16-group dpos: unrolled + tail loops
def test_preproc_c2_shape_vs_oracle(B):
    N, D = 211, 50
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, N, D, generator=g)
    lengths = torch.randint(20, 201, (B,), generator=g)
    ids = torch.randint(1, 3953, (B, N), generator=g)
    ids[torch.arange(N)[None, :] >= lengths[:, None]] = 0
    dy = torch.randn(B, N, D, generator=g)
    m = _module(N, D, 0.2).eval()
    pos = m._pos_emb.weight.detach().cpu().numpy()
    xg = x.cuda().requires_grad_(True)
    _, y, _, _ = m(lengths.cuda(), ids.cuda(), xg, {})
    (y * dy.cuda()).sum().backward()
    yr, _ = preproc_oracle.preprocess(x.numpy(), ids.numpy(), pos, D ** 0.5)
    dxr, dposr = preproc_oracle.preprocess_bwd(dy.numpy(), ids.numpy(), D ** 0.5, N)
    assert np.allclose(y.detach().cpu().numpy(), yr, rtol=1e-6, atol=1e-5)
    assert np.allclose(xg.grad.cpu().numpy(), dxr, rtol=1e-6, atol=1e-5)
    assert np.allclose(m._pos_emb.weight.grad.cpu().numpy(), dposr, rtol=1e-5, atol=1e-4)


def test_preproc_dropout_statistics_and_mask_agreement():
    B, N, D, p = 64, 211, 50, 0.2
    g = torch.Generator().manual_seed(4)
    x = torch.randn(B, N, D, generator=g)
    ids = torch.randint(1, 3953, (B, N), generator=g)
    ids[:, 190:] = 0
    dy = torch.randn(B, N, D, generator=g)
    m = _module(N, D, p).train()
    xg = x.cuda().requires_grad_(True)
    _, y, _, _ = m(None, ids.cuda(), xg, {})
    (y * dy.cuda()).sum().backward()
    pos = m._pos_emb.weight.detach().cpu().numpy()
    base, _ = preproc_oracle.preprocess(x.numpy(), ids.numpy(), pos, D ** 0.5)
    yv = y.detach().cpu().numpy().astype(np.float64)
    live = (ids != 0).numpy()[..., None] & (np.abs(base) > 1e-6)
    kept = live & (yv != 0)
    rate = kept.sum() / live.sum()
    assert abs(rate - (1 - p)) < 0.01, rate
    assert np.allclose(yv[kept], base[kept] / (1 - p), rtol=1e-5, atol=1e-5)
    mask = np.where(kept, 1 / (1 - p), 0.0)
    dxr, dposr = preproc_oracle.preprocess_bwd(dy.numpy(), ids.numpy(), D ** 0.5, N, mask=mask)
    assert np.allclose(xg.grad.cpu().numpy()[live], dxr[live], rtol=1e-5, atol=1e-5)
    # the positional gradient sums the same regenerated mask over the batch
    assert np.allclose(m._pos_emb.weight.grad.cpu().numpy(), dposr, rtol=1e-5, atol=1e-4)
    # a second forward draws a different mask
    _, y2, _, _ = m(None, ids.cuda(), xg, {})
    assert not torch.equal(y2, y)
