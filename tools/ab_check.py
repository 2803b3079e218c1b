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

# AB_GRAPH=wimax: the cfg2 graph (WiMAX N=576 R=3/4 z=24) instead of BG2 z=384
WIMAX = os.environ.get("AB_GRAPH") == "wimax"
Z, T, B = (24, 20, 100) if WIMAX else (384, 20, 48)
hb = np.loadtxt(os.path.join(ROOT, "resources", "wman_N0576_R34_z24.txt" if WIMAX else "basegraph2_set0.txt"), int,
                delimiter="\t")
g = LiftedGraph(hb, Z)
dev = torch.device("cuda")
gen = torch.Generator().manual_seed(7)
sigma = (1.0 / (2 * (18 / 22 if WIMAX else 0.2) * 10 ** 0.2)) ** 0.5
x = 2 * (-1 + sigma * torch.randn(B, g.N, Z, generator=gen)) / sigma ** 2
x[:, :2] = 0.0  # (BG2: the punctured columns) exact zeros in iteration 0
x[3, 10:12] = 0.0
x = x.to(dev)
bad = 0
cases = []
for kind in [int(k) for k in sys.argv[1:]] or [3]:
    cases += [(kind, False)] + ([(kind, True)] if kind != 3 else [])  # Boosted: also with UCN
for kind, ucn in cases:
    w = (0.3 + 0.9 * torch.rand(T, g.E, generator=gen)).to(dev)
    b = (0.3 * torch.randn(T, g.E, generator=gen)).to(dev) if kind == 3 else None
    wu = (0.3 + 0.9 * torch.rand(T, g.E, generator=gen)).to(dev) if ucn else None
    wv = (0.6 + 0.6 * torch.rand(T, g.N, generator=gen)).to(dev) if kind != 3 else None
    xk = x
    if kind == 2:  # QMS: the reference datagen's quantised channel (AWGNPassedDatagen.py:106-107)
        xk = torch.clamp(torch.round(2 * x) / 2, -7.5, 7.5)
    res = {}
    for path in ("fused", "stream"):
        cfg = DecodeCfg(kind=kind, qbit=5, ucn=ucn, vn_cumulative=kind != 3, path=path)
        outs, st, _ = decode(g, cfg, xk, T, w_cn=w, bias=b, w_ucn=wu, w_vn=wv)
        res[path] = (outs.view(torch.int32).clone(), st.clone())
    torch.cuda.synchronize()
    no = int((res["fused"][0] != res["stream"][0]).sum())
    # the state as values: a zero c2v's sign may differ between the paths (Boosted: Q(0) * sign), which no
    # sum of the decoder observes; the outputs are compared bit for bit
    ns = int((res["fused"][1] != res["stream"][1]).sum())
    print(f"kind {kind}{' UCN' if ucn else ''}: fused vs streaming, {T} outputs x {B} codewords: {no} output words "
          f"differ, {ns} state words differ")
    bad += no + ns
sys.exit(1 if bad else 0)
