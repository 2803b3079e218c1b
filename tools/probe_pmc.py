"""HBM probe kernels with known byte counts, for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE
(run under rocprofv3 --pmc; tools/gpu_prof_r2.sh).  Each probe runs once over 1 GiB:
kind 0 copy (reads 1 GiB, writes 1 GiB), 1 write-only (1 GiB), 2 read 16 B/lane (1 GiB),
3 read 4 B/lane (1 GiB, the decoder's own load width)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"), ROOT]
import torch  # noqa: E402

from nldpc import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
n = (1 << 30) // 4
a = torch.ones(n, dtype=torch.float32, device=dev)
b = torch.empty(n, dtype=torch.float32, device=dev)
s = _lib.stream_of(dev)
for kind in (0, 1, 2, 3):
    _lib.check(L.nldpc_hbm_probe(kind, b.data_ptr(), a.data_ptr(), n, s), "nldpc_hbm_probe")
torch.cuda.synchronize()
print("probes done: 1 GiB each, kinds 0..3")
