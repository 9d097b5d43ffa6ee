"""Does a memset captured into a HIP graph re-run on every replay?  Captures
(a) a torch zero_() of a contiguous tensor and (b) the library's sampled-softmax
backward (whose per-step counters used to be zeroed by hipMemsetAsync), poisons the
buffers between replays and checks them.  Diagnostic only."""
import torch

dev = torch.device("cuda", 0)
for n in (1000, 3953, 1 << 20):
    a = torch.ones(n, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        a.zero_()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        a.zero_()
    bad = 0
    for r in range(3):
        a.fill_(7.0)
        g.replay()
        torch.cuda.synchronize()
        bad += int((a != 0).sum().item())
    print(f"zero_ n={n}: non-zero after replays = {bad}", flush=True)
    with torch.cuda.graph(g2 := torch.cuda.CUDAGraph()):
        z = torch.zeros(n, device=dev)
        z += 1.0
    for r in range(3):
        g2.replay()
        torch.cuda.synchronize()
        print(f"zeros+1 n={n} replay {r}: max {z.max().item()} min {z.min().item()}", flush=True)
