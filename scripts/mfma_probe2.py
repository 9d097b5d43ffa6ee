import ctypes, numpy as np, torch
L = ctypes.CDLL("scripts/libmfma_probe2.so")
dev = torch.device("cuda")
bf = lambda x: (np.asarray(x, np.float32).view(np.uint32) >> 16).astype(np.uint16)
rng = np.random.default_rng(1)
A = rng.integers(-3, 4, (32, 16)).astype(np.float32)
B = rng.integers(-3, 4, (16, 32)).astype(np.float32)
D = rng.integers(-3, 4, (32, 32)).astype(np.float32)
t = [torch.tensor(bf(x).view(np.int16)).to(dev) for x in (A, B, D)]
out = torch.zeros(2048, device=dev)
assert L.run_probe(*[ctypes.c_void_p(x.data_ptr()) for x in t], ctypes.c_void_p(out.data_ptr())) == 0
o = out.cpu().numpy().reshape(2, 64, 16)
def unpack(o):
    C = np.zeros((32, 32), np.float32)
    for l in range(64):
        for rr in range(16): C[(rr & 3) + 8 * (rr >> 2) + 4 * (l >> 5), l & 31] = o[l, rr]
    return C
X = A @ B
print("X = A.B:", np.array_equal(unpack(o[0]), X))
Z = unpack(o[1])
print("Z = X^T.D:", np.array_equal(Z, X.T @ D), "| max |diff|", np.abs(Z - X.T @ D).max())
