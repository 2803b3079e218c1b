"""Add the VALU class mix of a kernel (rocprofv3 --pmc SQ_INSTS_VALU, _ADD_F32, _MUL_F32, _FMA_F32, _INT32, _CVT:
tools/gpu_pmc.sh with GROUPS_="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 ...") to its entry of profiles/pmc_traffic.json, so
that bench.py prices the kernel's measured VALU instructions at their per-class issue costs
(roofline.valu_issue.weighted_frac_of_simd_cycles, the evidence behind roofline.bound).

Class costs (SIMD cycles per wave64 instruction at 4 waves per SIMD, tools/dev/valu_rate2.hip, profiles/r3_valu_rate2*.txt):
add / mul / fma f32 2.2; int32 3.0 (a mix of full-rate add / and / xor and half-rate shifts / med3, as r3 assumed);
cvt 4.2 (half rate assumed); other 4.3 (min / max / med3 / cndmask 4.1-4.2, v_cmp 5.2, v_mov 2.3, DPP moves).

Usage: python tools/mix_summary.py [--traffic] PMC_TRAFFIC_JSON ENTRY_KEY KERNEL_SUBSTRING SUMMARY_DIR [SOURCE_NOTE]
  (--traffic: the entry's bytes, instruction counts, wait fraction and clock too, from the same directory)
  e.g. python tools/mix_summary.py profiles/pmc_traffic.json fused_cfg2_B4096 "fused_wimax_z24::kernel<3, 0>" \\
       gpurun_out/r6b/mix_cfg2 "profiles/r6_valu_mix.txt"
"""
import collections
import csv
import glob
import json
import os
import sys

COSTS = {"add_f32": 2.2, "mul_f32": 2.2, "fma_f32": 2.2, "int32": 3.0, "cvt": 4.2, "other": 4.3}
COUNTERS = {"add_f32": "SQ_INSTS_VALU_ADD_F32", "mul_f32": "SQ_INSTS_VALU_MUL_F32", "fma_f32": "SQ_INSTS_VALU_FMA_F32",
            "int32": "SQ_INSTS_VALU_INT32", "cvt": "SQ_INSTS_VALU_CVT"}


def kernel_counters(summary_dir, kernel, durations=None):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(summary_dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
                if durations is not None:
                    durations[(f, row["Dispatch_Id"])] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    return {k: sum(v) / len(v) for k, v in acc.items()}


def traffic(e, summary, kernel, note):
    """--traffic: the entry's per-launch bytes (FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024, the calibration of
    profiles/pmc_traffic.json), instruction counts, SQ_WAIT_ANY / SQ_WAVE_CYCLES and the PMC clock from the same
    tools/gpu_pmc.sh directory (one counter group per run)."""
    dur = {}
    c = kernel_counters(summary, kernel, dur)
    d = sum(dur.values()) / len(dur)
    fetch, write = 2 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
    e.update({"bytes": fetch + write, "fetch_bytes": fetch, "write_bytes": write, "valu_insts": c.get("SQ_INSTS_VALU"),
              "lds_insts": c.get("SQ_INSTS_LDS"), "salu_insts": c.get("SQ_INSTS_SALU"), "waves": c.get("SQ_WAVES"),
              "wait_any_over_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
              "duration_ms_profiled": d,
              "effective_clock_ghz": c["GRBM_GUI_ACTIVE"] / 8 / (d * 1e6) if c.get("GRBM_GUI_ACTIVE") else None,
              "source": f"{note} (rocprofv3 --pmc, one group per run, tools/gpu_pmc.sh)"})


def main():
    args = [a for a in sys.argv[1:] if a != "--traffic"]
    path, key, kernel, summary = args[:4]
    note = args[4] if len(args) > 4 else summary
    c = kernel_counters(summary, kernel)
    total = c["SQ_INSTS_VALU"]
    fr = {cls: c.get(ctr, 0.0) / total for cls, ctr in COUNTERS.items()}
    fr["other"] = max(0.0, 1.0 - sum(fr.values()))
    d = json.load(open(path))
    e = d.setdefault(key, {"kernel": kernel})
    e["kernel"] = kernel
    if "--traffic" in sys.argv:
        traffic(e, summary, kernel, note)
    e["valu_mix"] = {"fractions": {k: round(v, 4) for k, v in fr.items()}, "issue_cycles": COSTS,
                     "valu_insts_in_mix_run": total,
                     "source": f"{note} (SQ_INSTS_VALU and its _ADD_F32 / _MUL_F32 / _FMA_F32 / _INT32 / _CVT classes of "
                               f"{kernel}); class costs: tools/mix_summary.py"}
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")
    mean = sum(fr[k] * COSTS[k] for k in fr)
    print(f"{key}: {total:.4g} VALU per launch in the mix run, mean {mean:.2f} SIMD cycles per instruction, "
          + ", ".join(f"{k} {v:.3f}" for k, v in fr.items()))


if __name__ == "__main__":
    main()
