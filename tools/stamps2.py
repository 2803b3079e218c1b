"""Phase breakdown of the fused forward kernel from a diagnostic stamp build (make STAMPS=1), any
chunk schedule.  Stamps (s_memtime, lane 0 of each wave, 16 slots per iteration): 0 iteration start,
1 after the VN, 2+k arrival at the barrier that ends phase k of the schedule (gen_fused.py).

Per phase: critical = the phase's last arrival minus the previous phase's last arrival (the release of
the barrier it starts from); mean / max busy = a wave's own arrival minus that release (the rest of the
critical time is barrier wait).  Per wave: busy cycles of the phase, to see imbalance between parts and
the SIMD arbitration.  Usage: python tools/stamps2.py stamps.bin [phase names...]"""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
nb, nw, T, nph = np.frombuffer(raw[:16], np.int32)
st = np.frombuffer(raw[16:], np.uint64).reshape(nb, nw, T, nph).astype(np.int64)
st = st[(st[:, :, :, 0] > 0).all(axis=(1, 2))]  # workgroups that ran
used = [k for k in range(nph) if (st[:, :, 1:, k] > 0).all()]
last = used[-1]
names = sys.argv[2:] or ["VN"] + [f"phase {k}" for k in range(last - 1)]
rows = []
for it in range(1, T):  # skip the first iteration (cold caches)
    prev_end = st[:, :, it - 1, last].max(axis=1)  # last arrival of the previous iteration
    s = st[:, :, it, :]
    r = []
    for k in range(1, last + 1):
        rel = prev_end if k <= 2 else s[:, :, k - 1].max(axis=1)
        if k == 2:  # phase 0 starts at the same release as the VN (the VN is its first part)
            rel = prev_end
        busy = s[:, :, k] - rel[:, None]
        crit = s[:, :, k].max(axis=1) - (rel if k != 2 else s[:, :, 1].max(axis=1) * 0 + rel)
        r.append((crit.mean(), busy.mean(), busy.max(axis=1).mean(), busy.mean(axis=0)))
    rows.append(r)
per_it = st[:, :, 2:, last].max(axis=1) - st[:, :, 1:-1, last].max(axis=1)
print(f"{st.shape[0]} workgroups x {nw} waves, T={T}; cycles per iteration (last arrival to last arrival) = "
      f"{per_it.mean():.0f}")
print(f"{'phase':12s} {'critical':>9s} {'share':>6s} {'mean busy':>10s} {'max busy':>9s}")
tot = per_it.mean()
for k in range(1, last + 1):
    c = np.mean([r[k - 1][0] for r in rows])
    m = np.mean([r[k - 1][1] for r in rows])
    x = np.mean([r[k - 1][2] for r in rows])
    nm = names[k - 1] if k - 1 < len(names) else f"slot {k}"
    # phase 0 includes the VN: its critical is from the release, like the VN's
    print(f"{nm:12s} {c:9.0f} {100 * c / tot if k != 1 else float('nan'):5.1f}% {m:10.0f} {x:9.0f}")
for k in range(1, last + 1):
    per = np.mean([r[k - 1][3] for r in rows], axis=0)
    nm = names[k - 1] if k - 1 < len(names) else f"slot {k}"
    print(f"{nm + ' per wave:':22s}", " ".join(f"{v:.0f}" for v in per))
