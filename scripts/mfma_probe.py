import ctypes, numpy as np, torch
L = ctypes.CDLL("scripts/libmfma_probe.so")
dev = torch.device("cuda")
def bf(x):  # float32 -> bf16 bits (values exactly representable)
    return (np.asarray(x, np.float32).view(np.uint32) >> 16).astype(np.uint16)
rng = np.random.default_rng(0)
A = rng.integers(-4, 5, (16, 32)).astype(np.float32)   # rows i (items), k
Bm = rng.integers(-4, 5, (32, 16)).astype(np.float32)  # k, cols j (queries)
# assumed layouts: 16x16x32: lane l: A[i=l%16][k=8(l/16)+e]; B[k=8(l/16)+e][j=l%16]
a32 = np.zeros((64, 8), np.uint16); b32 = np.zeros((64, 8), np.uint16)
a16 = np.zeros((64, 4), np.uint16); b16 = np.zeros((64, 4), np.uint16)
for l in range(64):
    i, g = l % 16, l // 16
    a32[l] = bf(A[i, 8 * g:8 * g + 8]); b32[l] = bf(Bm[8 * g:8 * g + 8, i])
    a16[l] = bf(A[i, 4 * g:4 * g + 4]); b16[l] = bf(Bm[4 * g:4 * g + 4, i])
t = [torch.tensor(x.view(np.int16)).to(dev) for x in (a32, b32, a16, b16)]
out = torch.zeros(512, device=dev)
assert L.run_probe(*[ctypes.c_void_p(x.data_ptr()) for x in t], ctypes.c_void_p(out.data_ptr())) == 0
o = out.cpu().numpy().reshape(2, 64, 4)
C32 = A @ Bm; C16 = A[:, :16] @ Bm[:16]
def unpack(o):  # C[row = 4(l/16)+r][col = l%16]
    C = np.zeros((16, 16), np.float32)
    for l in range(64):
        for r in range(4): C[4 * (l // 16) + r, l % 16] = o[l, r]
    return C
print("16x16x32 matches C=A.B:", np.array_equal(unpack(o[0]), C32), " transposed:", np.array_equal(unpack(o[0]), C32.T))
print("16x16x16 matches C=A.B:", np.array_equal(unpack(o[1]), C16), " transposed:", np.array_equal(unpack(o[1]), C16.T))
print(unpack(o[1])[:3, :6]); print(C16[:3, :6])
