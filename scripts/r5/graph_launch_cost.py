"""Host cost of hipGraphLaunch vs node count and branch structure (torch.cuda.CUDAGraph on ROCm)."""
import time
import torch

dev = torch.device("cuda")
x = torch.zeros(256, device=dev)


def cap(n, branches=1):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    side = [torch.cuda.Stream() for _ in range(branches)]
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            if branches == 1:
                for _ in range(n):
                    x.add_(1.0)
            else:
                for b in side:
                    b.wait_stream(s)
                    with torch.cuda.stream(b):
                        for _ in range(n):
                            x.add_(1.0)
                for b in side:
                    s.wait_stream(b)
    torch.cuda.current_stream().wait_stream(s)
    return g


def bench(g, reps=50, streams=None):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / reps * 1e3, (t2 - t0) / reps * 1e3


for n in (1, 25, 125, 325, 1000):
    h, w = bench(cap(n))
    print(f"nodes {n:5d}: host {h:.3f} ms/launch, wall {w:.3f} ms/launch", flush=True)
for br, n in ((8, 125), (8, 25)):
    h, w = bench(cap(n, br))
    print(f"{br} branches x {n} nodes: host {h:.3f} ms/launch, wall {w:.3f} ms/launch", flush=True)
# 8 graphs of 125 nodes on 8 streams (the replica-group schedule)
gs = [cap(125) for _ in range(8)]
ss = [torch.cuda.Stream() for _ in range(8)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    for g, s in zip(gs, ss):
        with torch.cuda.stream(s):
            g.replay()
    torch.cuda.synchronize()
print(f"8 graphs x 125 nodes on 8 streams: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/round", flush=True)
