"""GPU A/B helper: bit-exactness of an experiment library's fused kernels (NLDPC_LIB_PATH) against the
same library's streaming kernels (hand-written, shared by every variant), BG2 z=384, T=20.

Neural with random weights and biases (negative biases exercise the ReLU, exact zeros in the channel
exercise the check node's zero path), all T posteriors and the final message state compared bit for
bit.  Prints one line; exit status 1 on a mismatch.  Usage: python tools/ab_check.py [KIND ...]
(3 = Neural, 1 = MS, 2 = QMS)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"))
from nldpc.decode import DecodeCfg, decode  # noqa: E402
from nldpc.graph import LiftedGraph  # noqa: E402

Z, T, B = 384, 20, 48
hb = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
g = LiftedGraph(hb, Z)
dev = torch.device("cuda")
gen = torch.Generator().manual_seed(7)
sigma = (1.0 / (2 * 0.2 * 10 ** 0.2)) ** 0.5
x = 2 * (-1 + sigma * torch.randn(B, g.N, Z, generator=gen)) / sigma ** 2
x[:, :2] = 0.0  # punctured columns: exact zeros in iteration 0
x[3, 10:12] = 0.0
x = x.to(dev)
bad = 0
for kind in [int(k) for k in sys.argv[1:]] or [3]:
    w = (0.3 + 0.9 * torch.rand(T, g.E, generator=gen)).to(dev)
    b = (0.3 * torch.randn(T, g.E, generator=gen)).to(dev) if kind == 3 else None
    wv = (0.6 + 0.6 * torch.rand(T, g.N, generator=gen)).to(dev) if kind != 3 else None
    res = {}
    for path in ("fused", "stream"):
        cfg = DecodeCfg(kind=kind, qbit=5, vn_cumulative=kind != 3, path=path)
        outs, st, _ = decode(g, cfg, x, T, w_cn=w, bias=b, w_vn=wv)
        res[path] = (outs.view(torch.int32).clone(), st.view(torch.int32).clone())
    torch.cuda.synchronize()
    no = int((res["fused"][0] != res["stream"][0]).sum())
    ns = int((res["fused"][1] != res["stream"][1]).sum())
    print(f"kind {kind}: fused vs streaming, {T} outputs x {B} codewords: {no} output words differ, {ns} state words differ")
    bad += no + ns
sys.exit(1 if bad else 0)
