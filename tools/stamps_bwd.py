"""Phase breakdown of the fused backward kernel from a diagnostic stamp build (make STAMPS=1
NLDPC_GEN_KINDS=<kind>, NLDPC_STAMPS_BWD=<file>).  Stamps (s_memtime, lane 0 of each wave, 16 slots per
iteration, gen_fused.py emit_bwd): 0 iteration start, then per chunk c the arrival at the barrier after
its LDS write (1+3c), check-node backward (2+3c) and read-back (3+3c); 1+3K after the variable-node step.
Iterations run T-1 .. 0.  Per phase: critical = the phase's last arrival minus the previous phase's last
arrival; mean / max busy = a wave's own arrival minus that release.  Usage: stamps_bwd.py stamps.bin K"""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
K = int(sys.argv[2])
nb, nw, T, nph = np.frombuffer(raw[:16], np.int32)
st = np.frombuffer(raw[16:], np.uint64).reshape(nb, nw, T, nph).astype(np.int64)
st = st[(st[:, :, :, 1] > 0).all(axis=(1, 2))]
last = 1 + 3 * K
names = ["start"] + [f"{n}{c}" for c in range(K) for n in ("W", "CNB", "R")] + ["VNB"]
crit = np.zeros(last + 1)
busy = np.zeros(last + 1)
bmax = np.zeros(last + 1)
cnt = 0
for it in range(T - 2, 0, -1):  # skip the first (cold) and last iterations
    s = st[:, :, it, :]
    prev_end = st[:, :, it + 1, last].max(axis=1)
    for k in range(1, last + 1):
        rel = s[:, :, k - 1].max(axis=1) if k > 1 else prev_end
        crit[k] += (s[:, :, k].max(axis=1) - rel).mean()
        b = s[:, :, k] - rel[:, None]
        busy[k] += b.mean()
        bmax[k] += b.max(axis=1).mean()
    cnt += 1
crit, busy, bmax = crit / cnt, busy / cnt, bmax / cnt
tot = crit[1:].sum()
print(f"{st.shape[0]} workgroups x {nw} waves, T={T}; cycles per iteration = {tot:.0f}")
print(f"{'phase':8s} {'critical':>9s} {'share':>6s} {'mean busy':>10s} {'max busy':>9s}")
for k in range(1, last + 1):
    print(f"{names[k]:8s} {crit[k]:9.0f} {100 * crit[k] / tot:5.1f}% {busy[k]:10.0f} {bmax[k]:9.0f}")
