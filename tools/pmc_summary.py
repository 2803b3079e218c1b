"""Summarise rocprofv3 PMC passes (tools/gpu_prof_r2.sh) into profiles/pmc_traffic.json, the per-launch
counter figures bench.py's roofline quotes.

FETCH_SIZE / WRITE_SIZE are in KiB.  Calibration on the probe kernels with known bytes
(tools/probe_pmc.py, 1 GiB each): WRITE_SIZE reads the written bytes exactly; FETCH_SIZE reports half
the bytes of a coalesced streaming read at both 16 B and 4 B per lane (the decoder's width), so fetch
bytes = 2 x FETCH_SIZE x 1024 (MI355X_MICROARCH.md, HBM/rocprofv3 section).
Usage: python tools/pmc_summary.py gpurun_out r2 [previous.json] > profiles/pmc_traffic.json (entries of
workloads not re-measured are kept from previous.json).  (The QMS backward's namespace is fusedbq_ since r2:
the kernel is matched by its suffix.)"""
import collections
import csv
import json
import os
import sys

root, tag = sys.argv[1], sys.argv[2]


def counters(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for row in csv.DictReader(open(os.path.join(root, d, "run_counter_collection.csv"))):
        k = row["Kernel_Name"]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        dur[(k, row["Dispatch_Id"])] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    return acc, dur


def mean(v):
    return sum(v) / len(v) if v else None


out = {"_doc": __doc__.split("\n\n")[1].replace("\n", " ")}
# probe calibration
pf, _ = counters(f"{tag}_probe_fetch")
pw, _ = counters(f"{tag}_probe_write")
probe = [k for k in pf if "hbm_probe" in k][0]
fv, wv = pf[probe]["FETCH_SIZE"], pw[probe]["WRITE_SIZE"]
gib = 1 << 30
out["calibration"] = {
    "kinds": ["copy 1 GiB", "write 1 GiB", "read 1 GiB 16 B/lane", "read 1 GiB 4 B/lane"],
    "fetch_bytes_reported": [v * 1024 for v in fv], "write_bytes_reported": [v * 1024 for v in wv],
    "fetch_ratio_16B": fv[2] * 1024 / gib, "fetch_ratio_4B": fv[3] * 1024 / gib, "write_ratio": wv[1] * 1024 / gib,
}
KERNELS = {"cfg3": [("fused", "fused_bg2_z384::kernel<3, 0>", 65536)],
           "cfg2": [("fused", "fused_wimax_z24::kernel<3, 0>", 4096)],
           # (the backward's template is <KIND, TIED> since r4: the prefix matches both)
           "cfg5": [("fused", "fused_bg2_z384::kernel<2, 1>", 2048), ("fusedb", "_bg2_z384::bwd_kernel<2", 2048)],
           "cfg3ucn": [("fused", "fused_bg2_z384::kernel<1, 0>", 65536)]}
# Boosted side lines, one entry per (kind, sharing codes): bench.py --workload cfg3ucn --kind K --nw a,b,c
for _k, _kind in (("MS", 1), ("QMS", 2), ("SP", 0)):
    for _nw in ("112", "100", "102", "110"):
        KERNELS[f"cfg3ucn_{_k}_NW{_nw}"] = [("fused", f"fused_bg2_z384::kernel<{_kind}, 0>", 65536)]
for w, ks in KERNELS.items():
    if not os.path.isdir(os.path.join(root, f"{tag}_{w}_sq")):
        continue
    f, _ = counters(f"{tag}_{w}_fetch")
    wr, _ = counters(f"{tag}_{w}_write")
    sq, sqdur = counters(f"{tag}_{w}_sq")
    for short, name, B in ks:
        kf = [k for k in f if name in k][0]
        fetch = 2 * mean(f[kf]["FETCH_SIZE"]) * 1024
        write = mean(wr[[k for k in wr if name in k][0]]["WRITE_SIZE"]) * 1024
        ks_ = [k for k in sq if name in k][0]
        c = {n: mean(v) for n, v in sq[ks_].items()}
        d = mean([v for (k, _), v in sqdur.items() if k == ks_])
        rec = {"kernel": name, "bytes": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
               "valu_insts": c.get("SQ_INSTS_VALU"), "lds_insts": c.get("SQ_INSTS_LDS"),
               "salu_insts": c.get("SQ_INSTS_SALU"), "waves": c.get("SQ_WAVES"),
               "wait_any_over_wave_cycles": (c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") else None,
               "duration_ms_profiled": d,
               "effective_clock_ghz": (c["GRBM_GUI_ACTIVE"] / 8 / (d * 1e6)) if c.get("GRBM_GUI_ACTIVE") and d else None,
               "source": f"gpurun_out/{tag}_{w}_{{fetch,write,sq}} (rocprofv3 --pmc, one group per run)"}
        out[f"{short}_{w}_B{B}"] = rec
if len(sys.argv) > 3:  # keep the workloads this tag did not measure
    for k, v in json.load(open(sys.argv[3])).items():
        out.setdefault(k, v)
json.dump(out, sys.stdout, indent=1)
print()
