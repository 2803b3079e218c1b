"""GPU SP soft-value agreement with the reference fixtures: fraction within 1e-4 relative (dev tool)."""
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"))
from test_gpu_forward import DEV, _bg, _graph, boosted_params  # noqa: E402
from nldpc.decode import DecodeCfg, decode  # noqa: E402

for f in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "boosted_*_sp_*.npz"))):
    d = np.load(f)
    name = os.path.basename(f)[:-4]
    g = _graph(_bg(name), int(d["Z"]))
    T = int(d["T"])
    nw = tuple(int(v) for v in d["nw"])
    w_cn, w_ucn, w_vn, use_ucn = boosted_params(d, g, T, nw, [])
    for path in ("stream", "fused"):
        cfg = DecodeCfg(kind=0, qbit=int(d["q"]), ucn=use_ucn, vn_cumulative=w_vn is not None, path=path)
        try:
            o = decode(g, cfg, torch.from_numpy(d["x"]).to(DEV), T, w_cn=w_cn, w_ucn=w_ucn, w_vn=w_vn)[0].cpu().numpy()
        except Exception as e:  # fused not eligible (UCN)
            print(name, path, "skip", type(e).__name__)
            continue
        ref = d["outputs"][:T]
        rel = np.abs(o - ref) / np.maximum(np.abs(ref), 1e-30)
        print(name, path, "n", o.size, "exact", int((o == ref).sum()), "rel>1e-4", int((rel > 1e-4).sum()),
              "maxrel", float(rel.max()), "max|d|", float(np.abs(o - ref).max()))
