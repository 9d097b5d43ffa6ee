"""gr_wgrad_multi (many weight-gradient problems in one partial + one reduce launch)
against an fp64 torch reference, and against gr_wgrad2 on the same problems.  Shapes: the
C2 encoder's 4 layers (8 problems: _uvqk 50 x 200 with LayerNorm stats, _o 50 x 50 with
the bias column sum) and the C3 encoder's 8 layers (16 problems at D = 256, wide plan).
Tolerance 1e-5 relative to the largest |C| (fp32 split-K over rows)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, st, total):
    a64 = a[:total].double()
    if st is not None:
        a64 = (a64 - st[:total, 0:1].double()) * st[:total, 1:2].double()
    return a64.t() @ b[:total].double(), a64.sum(0)


def _check(got, ref, what):
    scale = ref.abs().max().item() + 1.0
    err = (got.double() - ref).abs().max().item()
    assert err <= 1e-5 * scale, (what, err, scale)


@pytest.mark.parametrize("layers,D,n_out,lens", [(4, 50, 200, [200] * 40 + [37, 1, 0, 150]),
                                                 (8, 256, 1024, [2048, 700, 1500])])
def test_wgrad_multi_matches_reference(layers, D, n_out, lens):
    from mygenerativerecommenders_amd import _lib as L
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(layers)
    offs = torch.zeros(len(lens) + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(torch.tensor(lens), 0)
    total = int(offs[-1])
    cap = total + 29
    offs = offs.to(dev)
    keep, desc, outs = [], [], []
    for _ in range(layers):
        x = torch.randn(cap, D, device=dev, generator=g) * 2 + 0.3
        mean = x.mean(1)
        rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-6)
        st = torch.stack([mean, rstd], 1).contiguous()
        dh = torch.randn(cap, n_out, device=dev, generator=g)
        dy = torch.randn(cap, D, device=dev, generator=g)
        oin = torch.randn(cap, D, device=dev, generator=g)
        cu = torch.full((D, n_out), float("nan"), device=dev)
        co = torch.full((D, D), float("nan"), device=dev)
        cb = torch.full((D,), float("nan"), device=dev)
        keep += [x, st, dh, dy, oin]
        desc.append([x.data_ptr(), D, st.data_ptr(), dh.data_ptr(), n_out, D, n_out, cu.data_ptr(), 0])
        desc.append([dy.data_ptr(), D, 0, oin.data_ptr(), D, D, D, co.data_ptr(), cb.data_ptr()])
        outs.append((x, st, dh, dy, oin, cu, co, cb))
    d = np.ascontiguousarray(np.array(desc, dtype=np.int64))
    lib = L.lib()
    ws_n = lib.gr_wgrad_multi_workspace_size(d.ctypes.data, len(desc), cap)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
    L.call("gr_wgrad_multi", d.ctypes.data, len(desc), offs.data_ptr(), len(lens), cap, 0,
           ws.data_ptr(), ws_n, L.stream_handle())
    torch.cuda.synchronize()
    for x, st, dh, dy, oin, cu, co, cb in outs:
        ru, _ = _ref(x, dh, st, total)
        ro, rb = _ref(dy, oin, None, total)
        _check(cu, ru, "uvqk")
        _check(co, ro, "o")
        _check(cb, rb, "bias")
    # deterministic
    first = [o[5].clone() for o in outs]
    L.call("gr_wgrad_multi", d.ctypes.data, len(desc), offs.data_ptr(), len(lens), cap, 0,
           ws.data_ptr(), ws_n, L.stream_handle())
    torch.cuda.synchronize()
    assert all(torch.equal(f, o[5]) for f, o in zip(first, outs))
