"""Host-side cost of one NeuralLDPCDecoder.forward (cfg2: WiMAX z=24, B=4096, T=20) on the GPU box: the
Python + ctypes time per call (no synchronisation inside the loop), the GPU time per call, and a cProfile
of the host path.  Development tool (r3, VERDICT r2 item 8: cfg2 step time vs kernel time)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import neural_ldpc_decoder as nd  # noqa: E402
from nldpc.channel import awgn_llr, sigma_for  # noqa: E402

dev = torch.device("cuda:0")
bg = np.loadtxt(os.path.join(ROOT, "resources", "wman_N0576_R34_z24.txt"), int, delimiter="\t")
Z, T, B = 24, 20, int(os.environ.get("B", "4096"))
M, N = bg.shape
conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(Z, bg), device=dev)
model = nd.NeuralLDPCDecoder(T, B, conn).to(dev)
xa = awgn_llr(B, N, Z, sigma_for(2.0, (N - M) / (N - 2)), seed=2042, device=dev)
with torch.no_grad():
    for _ in range(20):
        outs = model(xa)
    torch.cuda.synchronize()
    n = 300
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        outs = None
        outs = model(xa)
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host per call: median {1e6 * float(np.median(host)):.1f} us, mean {1e6 * float(np.mean(host)):.1f} us; "
          f"enqueue loop {1e3 * (t1 - t0) / n:.4f} ms/call, with drain {1e3 * (t2 - t0) / n:.4f} ms/call")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(100):
        outs = None
        outs = model(xa)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
