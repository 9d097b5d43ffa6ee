"""GPU: N3 RetrievalMetrics on device tensors (against the oracle restatement) and N4 Muon
on the MI355X (bf16 Newton-Schulz on the matrix cores) against the reference's two
recorded CPU steps.  Tolerance for Muon: 2e-2 of the step size (bf16 GEMMs accumulate
in a different order on the GPU than on the CPU that recorded the golden)."""
import os

import numpy as np
import pytest
import torch

from oracle import metrics_oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_metrics_on_device():
    from mygenerativerecommenders_amd.metrics import RetrievalMetrics
    g = torch.Generator().manual_seed(9)
    B, k = 128, 200
    top = torch.stack([torch.randperm(3953, generator=g)[:k] + 1 for _ in range(B)])
    tgt = torch.randint(1, 3954, (B,), generator=g)
    top[::2, 5] = tgt[::2]
    m = RetrievalMetrics(k=k, at_k_list=[10, 50, 100, 200])
    m.update(top_k_ids=top.cuda(), target_ids=tgt.cuda().view(-1, 1))
    got = m.compute()
    ref = metrics_oracle.retrieval_metrics(top.numpy(), tgt.numpy(), [10, 50, 100, 200])
    for key, v in ref.items():
        assert got[key].is_cuda
        assert abs(float(got[key]) - v) < 1e-6, key


def test_muon_on_gpu_matches_reference_golden():
    from mygenerativerecommenders_amd.muon import Muon
    z = np.load(os.path.join(GOLDEN, "muon.npz"))
    n = len([k for k in z.files if k.startswith("p0_")])
    params = [torch.nn.Parameter(torch.from_numpy(z[f"p0_{i}"]).cuda()) for i in range(n)]
    opt = Muon(params, lr=0.02, weight_decay=0.01, momentum=0.95)
    for step in range(2):
        for i, p in enumerate(params):
            p.grad = torch.from_numpy(z[f"g{step}_{i}"]).cuda()
        opt.step()
        for i, p in enumerate(params):
            ref = z[f"p{step + 1}_{i}"]
            delta = np.abs(ref - z[f"p{step}_{i}"]).max()
            err = np.abs(p.detach().cpu().numpy() - ref).max()
            assert err <= 2e-2 * delta, (step, i, err, delta)


def test_muon_orthogonalises_hstu_shapes():
    """Singular values of the NS output sit in the quintic's band (~0.5 .. 1.5) for the
    ml-20m HSTU weight shapes (C5).  A square Gaussian matrix has a few singular values
    near 0 (~1/n) that 5 NS steps cannot lift, so the band is checked on the bulk: at
    most 2 % of the values may sit below 0.3, none above 1.6."""
    from mygenerativerecommenders_amd.muon import zeropower_via_newtonschulz5
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    for shape in [(3, 256, 1024), (3, 256, 256), (4, 50, 200)]:
        G = torch.randn(shape, device="cuda", generator=g)
        X = zeropower_via_newtonschulz5(G, 5).float()
        s = torch.linalg.svdvals(X)
        low = float((s < 0.3).float().mean())
        assert low <= 0.02 and float(s.max()) < 1.6, (shape, low, s.max())
        assert 0.6 < float(s.median()) < 1.4, (shape, s.median())


def test_fused_adamw_graph_replay_matches_unfused():
    """bench.py's training legs step the optimizer with fused=True, capturable=True
    AdamW inside a HIP graph.  On the e2e parameter set (encoder, item table,
    positional table) three replays equal the unfused eager update within fp32
    rounding of the update."""
    import bench
    from mygenerativerecommenders_amd.embeddings import LocalEmbeddingModule
    from mygenerativerecommenders_amd.preprocessors import (
        LearnablePositionalEmbeddingInputFeaturesPreprocessor as Pre)
    dev = torch.device("cuda")

    def params():
        torch.manual_seed(0)
        enc = bench.build_model(200, 11, 50, 4, dev)
        emb = LocalEmbeddingModule(3953, 50).to(dev)
        pre = Pre(211, 50, 0.2).to(dev)
        return list(enc.parameters()) + list(emb.parameters()) + list(pre.parameters())

    pa, pb = params(), params()
    g = torch.Generator(device=dev).manual_seed(5)
    grads = [[torch.randn(p.shape, device=dev, generator=g) * 1e-2 for p in pa] for _ in range(3)]
    kw = dict(lr=1e-3, betas=(0.9, 0.98), weight_decay=1e-3)
    opt_a = torch.optim.AdamW(pa, fused=True, capturable=True, **kw)
    opt_b = torch.optim.AdamW(pb, foreach=False, **kw)
    for p in pa:
        p.grad = torch.zeros_like(p)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up step with zero grads keeps both in lockstep
        opt_a.step()
    torch.cuda.current_stream().wait_stream(side)
    for p in pb:
        p.grad = torch.zeros_like(p)
    opt_b.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        opt_a.step()
    for step in range(3):
        for p, gr in zip(pa, grads[step]):
            p.grad.copy_(gr)
        graph.replay()
        for p, gr in zip(pb, grads[step]):
            p.grad = gr.clone()
        opt_b.step()
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7), (a - b).abs().max().item()


@pytest.mark.parametrize("shape", [(8, 256, 1024), (8, 256, 256), (3, 300, 50), (2, 7, 13)])
def test_muon_ns_combine_kernel_is_bit_identical(shape):
    """The GPU chain (gr_bf16_scale_add combines) against the reference's torch ops on the
    same device: the GEMMs are the same calls, the combines keep both bf16 roundings, so
    the orthogonalised result is bit-identical (any other rounding moves it by ~5 %)."""
    from mygenerativerecommenders_amd.muon import _NS_COEFFS, zeropower_via_newtonschulz5
    a, b, c = _NS_COEFFS
    g = torch.Generator(device="cuda")
    g.manual_seed(sum(shape))
    G = torch.randn(shape, device="cuda", generator=g)
    X = G.bfloat16()
    if G.size(-2) > G.size(-1):
        X = X.mT
    X = X / (X.norm(dim=(-2, -1), keepdim=True) + 1e-7)
    for _ in range(5):
        A = X @ X.mT
        B = b * A + c * A @ A
        X = a * X + B @ X
    if G.size(-2) > G.size(-1):
        X = X.mT
    got = zeropower_via_newtonschulz5(G, 5)
    assert torch.equal(got, X)


def _adamw_params(seed):
    import bench
    torch.manual_seed(seed)
    enc = bench.build_model(200, 11, 50, 4, torch.device("cuda"))
    return [p for p in enc.parameters()]


@pytest.mark.parametrize("wd", [1e-3, 0.0])
def test_flat_adamw_matches_torch_fused_adamw(wd):
    """FlatAdamW (one gr_adamw_step launch, counter advanced inside) against
    torch.optim.AdamW(fused=True, capturable=True) on the C2 encoder's parameters over
    four steps of random gradients: parameters and both moments within 2 ulp of the
    update's scale (ATen's double / float promotion is mirrored), the counters equal."""
    from mygenerativerecommenders_amd.optim import FlatAdamW
    pa, pb = _adamw_params(0), _adamw_params(0)
    ta = torch.optim.AdamW(pa, lr=1e-3, betas=(0.9, 0.98), weight_decay=wd, fused=True, capturable=True)
    fb = FlatAdamW(pb, lr=1e-3, betas=(0.9, 0.98), weight_decay=wd)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for _ in range(4):
        for a, b in zip(pa, pb):
            gr = torch.randn(a.shape, device="cuda", generator=g)
            a.grad = gr.clone()
            b.grad = gr.clone()
        ta.step()
        fb.step()
    torch.cuda.synchronize()
    worst = 0.0
    for a, b in zip(pa, pb):
        sa, sb = ta.state[a], fb.state[b]
        for x, y in ((a, b), (sa["exp_avg"], sb["exp_avg"]), (sa["exp_avg_sq"], sb["exp_avg_sq"])):
            d = (x - y).abs().max().item()
            scale = x.abs().max().item() + 1e-30
            worst = max(worst, d / scale)
        assert float(sa["step"]) == float(sb["step"]) == 4.0
    assert worst <= 2.5e-7, worst


def test_flat_adamw_graph_replay():
    """Captured in a HIP graph, three replays equal three eager steps bit for bit (the
    step counter lives on the device)."""
    from mygenerativerecommenders_amd.optim import FlatAdamW
    pa, pb = _adamw_params(1), _adamw_params(1)
    oa = FlatAdamW(pa, lr=1e-3, betas=(0.9, 0.98), weight_decay=1e-3)
    ob = FlatAdamW(pb, lr=1e-3, betas=(0.9, 0.98), weight_decay=1e-3)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    grads = [torch.randn(p.shape, device="cuda", generator=g) for p in pa]
    for a, b, gr in zip(pa, pb, grads):
        a.grad = gr.clone()
        b.grad = gr.clone()
    oa.step()  # eager warm-up builds the chunk table
    ob.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            ob.step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        oa.step()
        graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
    assert float(oa.state[pa[0]]["step"]) == float(ob.state[pb[0]]["step"]) == 4.0
