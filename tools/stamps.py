"""Phase breakdown of the fused forward kernel from a diagnostic stamp build (make STAMPS=1).

Usage: NLDPC_LIB_PATH=.../lib_stamps/libnldpc.so NLDPC_STAMPS=out.bin python bench.py ...; then
python tools/stamps.py out.bin.  Stamps (s_memtime, lane 0 of each wave) at: 0 iteration start,
1 after the VN, 2/5 after the LDS write of chunk 0/1, 3/6 after its check nodes, 4/7 after the read-back
(2..7 are barrier arrivals).  Per phase: critical = last arrival minus the previous barrier's last
arrival; mean = average wave's arrival minus that same release (the rest is barrier wait).  Shares,
not absolute time, are the meaningful output of a stamp build."""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
nb, nw, T, nph = np.frombuffer(raw[:16], np.int32)
st = np.frombuffer(raw[16:], np.uint64).reshape(nb, nw, T, nph).astype(np.int64)
st = st[(st[:, :, :, 0] > 0).all(axis=(1, 2))]  # workgroups that ran
names = ["VN", "write c0", "CN c0", "read c0", "write c1", "CN c1", "read c1"]
crit = {n: [] for n in names}
mean = {n: [] for n in names}
for it in range(1, T):  # skip the first iteration (cold)
    rel_prev = st[:, :, it - 1, 7].max(axis=1)  # release of the previous iteration's last barrier
    s = st[:, :, it, :]
    # VN: from release to the wave's own stamp 1 (no barrier between VN and write c0)
    mean["VN"].append((s[:, :, 1] - rel_prev[:, None]).mean())
    crit["VN"].append((s[:, :, 1].max(axis=1) - rel_prev).mean())
    mean["write c0"].append((s[:, :, 2] - s[:, :, 1]).mean())
    crit["write c0"].append((s[:, :, 2].max(axis=1) - s[:, :, 1].max(axis=1)).mean())
    for k, n in zip(range(3, 8), names[2:]):
        rel = s[:, :, k - 1].max(axis=1)
        mean[n].append((s[:, :, k] - rel[:, None]).mean())
        crit[n].append((s[:, :, k].max(axis=1) - rel).mean())
tot = sum(np.mean(crit[n]) for n in names)
print(f"{st.shape[0]} workgroups x {nw} waves, T={T}; cycles per iteration (critical path) = {tot:.0f}")
print(f"{'phase':10s} {'critical':>9s} {'share':>6s} {'mean wave':>10s} {'barrier wait':>13s}")
for n in names:
    c, m = np.mean(crit[n]), np.mean(mean[n])
    print(f"{n:10s} {c:9.0f} {100 * c / tot:5.1f}% {m:10.0f} {c - m:13.0f}")
# per-part VN time (waves 2p, 2p+1 form part p when parts are 2 waves)
vn = np.stack([st[:, :, it, 1] - st[:, :, it - 1, 7].max(axis=1)[:, None] for it in range(1, T)]).mean(axis=(0, 1))
print("VN cycles per wave:", " ".join(f"{v:.0f}" for v in vn))
# every phase per wave (arrival minus the release the phase started from)
for k, n in zip(range(2, 8), names[1:]):
    per = np.stack([st[:, :, it, k] - st[:, :, it, k - 1].max(axis=1)[:, None] if k > 2 else
                    st[:, :, it, k] - st[:, :, it, k - 1] for it in range(1, T)]).mean(axis=(0, 1))
    print(f"{n + ' per wave:':20s}", " ".join(f"{v:.0f}" for v in per))
