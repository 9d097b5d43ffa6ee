"""Filter-path parity across bf16 layouts (flag and exactness), quick GPU check."""
import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
from mygenerativerecommenders_amd.top_k import PackedItems, mips_topk, topk_workspace_bytes
from oracle import topk_oracle
dev = torch.device("cuda")
for D in [4, 8, 16, 20, 32, 40, 48, 50, 64]:
    for B in (16, 128):
        g = np.random.default_rng(D + B)
        X, k = 262_144, 50
        E = g.standard_normal((X, D), dtype=np.float32); E /= np.linalg.norm(E, axis=1, keepdims=True)
        Q = g.standard_normal((B, D), dtype=np.float32); Q /= np.linalg.norm(Q, axis=1, keepdims=True)
        pk = PackedItems(torch.tensor(E).to(dev))
        ws = torch.zeros(topk_workspace_bytes(B, X, D, k, 0), dtype=torch.uint8, device=dev)
        s, i = mips_topk(torch.tensor(Q).to(dev), pk, k, workspace=ws)
        torch.cuda.synchronize()
        flag = int(ws[:4].view(torch.int32).item())
        rs, ri, rx = topk_oracle.mips_topk(Q, E, np.arange(X), None, k)
        print(D, B, "flag", flag, "exact", np.array_equal(i.cpu().numpy(), ri), flush=True)
