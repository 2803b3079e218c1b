"""Benchmark: Neural BP decoding of 5G-NR BG2 z=384 at 20 iterations (BASELINE.json configs[2]/[3]).

    python bench.py [--gpus N --steps K --warmup W]            # N>1: starts N rank processes itself
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W
    python bench.py --workload cfg2|cfg5|cfg3ucn               # the other GPU configs (own lines)

Default workload cfg3: a step = one NeuralLDPCDecoder.forward over the rank's batch of B codewords
(default 65536 per GPU, weak scaling), T=20 iterations, every iteration's posterior written (the
reference API's output list).  At N=1 the default run also times the other single-GPU BASELINE configs
with the same timed() helper and reports them under `side_lines` (never as `value`): cfg5 and cfg2
(--no-side-lines skips them).  cfg2: the same decode on WiMAX N=576 R=3/4 z=24, B=4096.  cfg5: one
BoostedNeuralLDPCDecoder training step (QMS q=5, NW(3,0,3), T=50, B=2048: forward over all
iterations, LDPCDecoderLoss BCE, backward, clip_grad_norm 1.0, Adam, weight clamp), as
train/train_BoostedNeuralLDPCDecoder.py:278-294 does it.
Inputs: synthetic all-zero codewords over BPSK/AWGN at Eb/N0 = 2 dB generated on the device
(Philox, counter = global codeword index, so N GPUs decode exactly the codewords a single GPU would
decode at B*N).  Timed region: barrier + synchronize on both sides of K steps, max over ranks.
After timing: BER/FER of the last iteration summed over ranks with one RCCL all_reduce, and (cfg3)
a BER sweep over Eb/N0 = 1.0..4.0 dB; on rank 0 at N=1 the CPU oracle (oracle/ldpc_oracle.py, the
restatement pinned to the reference) is timed on a bounded sample of the same workload as the CPU
baseline.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, Chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles"), at the 2.4 GHz max clock
PEAK_VALU_INSTS = 256 * 4 * 2.4e9 / 2
METRIC = "codewords/sec + BER@Eb/N0, 5G-NR BG2 z=384, 20 iters, 1/2/4/8 MI355X"
KINDS = ("vn", "cn", "post", "fused", "vnb", "cnb", "fusedb")
KERNEL_NAMES = {"vn": "vn_kernel", "cn": "cn_kernel", "post": "vn_kernel (final posterior)",
                "fused": "fused_<graph>::kernel", "vnb": "vnb_kernel", "cnb": "cnb_kernel", "fusedb": "fusedb_<graph>::bwd_kernel"}
WORKLOADS = {
    # name: (base graph file, Z, T, default per-GPU batch)
    "cfg3": ("basegraph2_set0.txt", 384, 20, 65536),
    "cfg2": ("wman_N0576_R34_z24.txt", 24, 20, 4096),
    "cfg5": ("basegraph2_set0.txt", 384, 50, 2048),
    # side line (not a BASELINE config): cfg3's decode with the Boosted MS decoder and UCN on
    "cfg3ucn": ("basegraph2_set0.txt", 384, 20, 65536),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (test hook) gloo: the rank processes may share a GPU (cuda:rank % device_count) -- the product's
    # rank launch, sharding, counter all-reduce and max-time run on the one-GPU test box
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg3")
    ap.add_argument("--batch", type=int, default=None, help="codewords per GPU (default: the workload's)")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the HIP-event per-kernel timing")
    ap.add_argument("--no-sweep", action="store_true", help="skip the Eb/N0 1..4 dB BER sweep")
    ap.add_argument("--no-count-only", action="store_true", help="skip the count-only decode timing (F2)")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="decode steps as replays of one captured HIP graph (auto: cfg2, whose 0.1 ms kernel is "
                         "comparable to the host path of a module call)")
    ap.add_argument("--no-side-lines", action="store_true", help="default cfg3 run at N=1: skip the cfg5 / cfg2 lines")
    ap.add_argument("--side-steps-cfg2", type=int, default=200, help="timed steps of the cfg2 side line")
    ap.add_argument("--nw", default="1,1,2", help="cfg3ucn: NodeWeightSharingConfig (cn, ucn, vn) codes")
    ap.add_argument("--kind", default="MS", choices=("MS", "QMS", "SP"), help="cfg3ucn: Boosted decoding type")
    return ap.parse_args()


def kernel_bytes(B, E, N, Z, T, train=None):
    """Algorithmic HBM bytes of one decode (all launches of a kind together), DESIGN.md §4.

    fused: the bytes the register-resident kernel must move -- the channel read once and the T
    posteriors written, 4*(T+1)*N*Z per codeword (its message state never leaves the chip); with
    `train` (the cfg5 SAVE variant) also what it saves for the backward per iteration: v2c (int8
    codes for QMS: E*Z bytes), the clamp masks (N*Z bytes) and the xin chain (4*N*Z).
    fusedb: per iteration the saved v2c, masks and xin, the output gradient, and the VN-chain carry
    read + write (2*4*N*Z), plus the channel once.
    vn/cn/post: the streaming kernels' fp32 message traffic; vnb/cnb: their backward."""
    f = 4
    vn_first = B * f * (E * Z + N * Z)            # read xa, write v2c (all-zero state: no c2v read)
    vn = B * f * (2 * E * Z + 2 * N * Z)          # read c2v + xa, write v2c + previous posterior
    cn = B * f * (2 * E * Z)                      # gather v2c, scatter c2v
    post = B * f * (E * Z + 2 * N * Z)            # read c2v + xa, write the last posterior
    fused = B * f * (T + 1) * N * Z
    saved_it = 0
    if train:
        sb = 1 if train.get("qms") else 4
        saved_it = E * Z * sb + N * Z + (4 * N * Z if train.get("vn") else 0)
        fused += B * T * saved_it
    fusedb = B * (f * N * Z + T * (saved_it + f * N * Z + (2 * f * N * Z if train and train.get("vn") else 0)))
    vnb = B * f * (E * Z + N * Z)                 # per iteration: grad of the posterior in, grad v2c out
    cnb = B * f * (2 * E * Z)                     # per iteration: saved v2c + grad c2v in
    return {"vn": vn_first + (T - 1) * vn, "cn": T * cn, "post": post, "fused": fused,
            "vnb": (T + 1) * vnb, "cnb": T * cnb, "fusedb": fusedb}


class Prof:
    """HIP-event timing of every decoder launch inside the timed region (libnldpc's recorder: events
    on the launch stream itself)."""

    def __init__(self, enabled, capacity):
        from nldpc import _lib
        self.L, self.lib, self.enabled, self.capacity = _lib.lib(), _lib, enabled, capacity

    def begin(self):
        if self.enabled:
            self.lib.check(self.L.nldpc_profile_begin(self.capacity), "nldpc_profile_begin")

    def end(self):
        if not self.enabled:
            return None
        import ctypes
        n = len(KINDS)
        ms = (ctypes.c_float * n)()
        cnt = (ctypes.c_int32 * n)()
        self.lib.check(self.L.nldpc_profile_end(n, ms, cnt), "nldpc_profile_end")
        return {k: (ms[i], cnt[i]) for i, k in enumerate(KINDS)}


def load_pmc(key):
    """Counter totals per launch of `key` from profiles/pmc_traffic.json (written by
    tools/pmc_summary.py from rocprofv3 --pmc passes of this bench)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        v = json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None
    return v if isinstance(v, dict) else None


def load_isa_budget(kernel):
    """The committed ISA instruction budget of a kernel (profiles/isa_budget.json, written by
    tools/isa_budget.py from the gfx950 asm of single-part builds): SIMD issue cycles per workgroup-iteration
    on the busier SIMD set, the VALU instructions priced at their measured per-class issue costs."""
    try:
        v = json.load(open(os.path.join(ROOT, "profiles", "isa_budget.json"))).get(kernel)
    except (OSError, ValueError):
        return None
    return v if isinstance(v, dict) else None


def pmc_workload(args):
    """The key of this run's counters in profiles/pmc_traffic.json: the Boosted side lines are keyed by
    decoding type and sharing codes (their kernels differ), e.g. cfg3ucn_QMS_NW112."""
    if args.workload == "cfg3ucn":
        return f"cfg3ucn_{args.kind}_NW{args.nw.replace(',', '')}"
    return args.workload


def roofline(prof, kb, steps, B, Z, world, graph_tag, d5_bytes_per_cw, ceilings, pmc_key, T=None, cus=256):
    """Roofline of the dominant kernel: the algorithmic bytes it must move per launch over its average
    HIP-event launch time, against the 8 TB/s HBM spec (and the measured HBM ceilings); HBM traffic
    and VALU issue from the committed PMC summary of the same workload when present.  `frac` is always
    the compulsory-byte HBM fraction (the north star's quote); `bound` names the ceiling the evidence says
    binds: "valu" when the committed ISA budget's issue floor (profiles/isa_budget.json at the PMC effective
    clock) is at least half of the launch and a larger fraction than the bytes are of HBM peak; "hbm" when the
    bytes reach half of the HBM peak; "latency" when neither does and the PMC says the waves mostly wait
    (SQ_WAIT_ANY); "unknown" when no evidence names a ceiling (never "hbm" by default)."""
    per = {}
    for k in KINDS:
        ms_tot, n = prof[k]
        if n:
            byts = kb[k] * steps
            per[k] = {"avg_ms": ms_tot / n, "launches": n, "gbs": byts / (ms_tot / 1000.0) / 1e9,
                      "alg_bytes_per_launch": byts / n}
    dom = max(per, key=lambda k: prof[k][0])
    d = per[dom]
    pmc = load_pmc(f"{dom}_{pmc_key}")
    traffic = pmc.get("bytes") if pmc else None
    kname = KERNEL_NAMES[dom].replace("<graph>", graph_tag)
    r = {"bound": "unknown", "kernel": kname,
         "achieved": round(d["gbs"], 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
         "frac": round(d["gbs"] / PEAK_HBM_GBS, 4), "traffic": traffic,
         "alg_bytes_per_launch": d["alg_bytes_per_launch"], "avg_launch_ms": round(d["avg_ms"], 4),
         "per_kernel": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in per.items()}}
    if ceilings:
        r["measured_ceilings_gbs"] = ceilings
        top = ceilings.get("write") if dom.startswith("fused") else ceilings.get("copy")
        if top:
            r["frac_of_measured_ceiling"] = round(d["gbs"] / top, 4)
    if pmc:
        r["pmc"] = {k: v for k, v in pmc.items() if k != "_doc"}
        if pmc.get("valu_insts"):
            busy = pmc["valu_insts"] / (d["avg_ms"] / 1000.0) / PEAK_VALU_INSTS
            r["valu_issue"] = {"insts_per_launch": pmc["valu_insts"], "frac_of_peak": round(busy, 4),
                               "peak_insts_per_s": PEAK_VALU_INSTS,
                               "note": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x launch time)"}
            mix = pmc.get("valu_mix")
            if mix:  # the same instructions priced at their measured per-class issue cost
                cyc = sum(mix["fractions"][c] * mix["issue_cycles"][c] for c in mix["fractions"])
                clk = (pmc.get("effective_clock_ghz") or 2.4) * 1e9
                r["valu_issue"]["weighted_frac_of_simd_cycles"] = round(
                    pmc["valu_insts"] * cyc / (1024 * clk * d["avg_ms"] / 1000.0), 4)
                r["valu_issue"]["weighted_note"] = ("instructions x mean issue cycles of the kernel's PMC class mix / "
                                                    "(1024 SIMDs x effective clock x launch time): pmc.valu_mix")
    # the issue floor of the instruction stream (ISA budget), at the clock the PMC pass measured
    budget = load_isa_budget(pmc.get("kernel") if pmc and pmc.get("kernel") else kname)
    if budget and T and budget.get("G"):  # (an entry without its geometry's G is not used: ADVICE r5)
        clk = (pmc.get("effective_clock_ghz") if pmc else None) or budget.get("clock_ghz", 2.4)
        G = budget["G"]  # codewords per workgroup of the budgeted geometry
        # workgroup-iterations per CU; the budget is the busiest SIMD's issue cycles per workgroup-iteration (with
        # several workgroups per CU its waves' total over the 4 SIMDs: tools/isa_budget.py)
        wg_iters_per_cu = -(-B // G) / float(cus) * T
        floor_ms = budget["simd_issue_cycles_per_wg_iter"] * wg_iters_per_cu / (clk * 1e9) * 1e3
        r["issue_floor_ms"] = round(floor_ms, 3)
        r["issue_frac"] = round(floor_ms / d["avg_ms"], 4)
        r["issue_floor"] = {"simd_issue_cycles_per_wg_iter": budget["simd_issue_cycles_per_wg_iter"],
                            "clock_ghz": round(clk, 4), "wg_iters_per_cu": wg_iters_per_cu, "cus": cus,
                            "source": budget.get("source"),
                            "note": "VALU issue cycles of the busier SIMD set per workgroup-iteration (ISA of the "
                                    "hot loop at the measured per-class issue costs) x workgroup-iterations per CU / "
                                    "PMC effective clock: the launch time with no stall at all"}
    # the label: the ceiling the evidence puts nearest (the ISA issue floor or the PMC-weighted VALU issue, the
    # compulsory HBM bytes), a latency-bound kernel when neither is near and the waves mostly wait (PMC SQ_WAIT_ANY
    # over wave-cycles: the cfg5 backward's LDS round trips and barriers), else "unknown"
    vi = r.get("valu_issue", {})
    valu_frac = r.get("issue_frac") or vi.get("weighted_frac_of_simd_cycles") or vi.get("frac_of_peak")
    wait = pmc.get("wait_any_over_wave_cycles") if pmc else None
    if valu_frac is not None and valu_frac >= 0.5 and valu_frac > r["frac"]:
        r["bound"] = "valu"
    elif r["frac"] >= 0.5:
        r["bound"] = "hbm"
    elif wait is not None and wait >= 0.5:
        r["bound"] = "latency"
    r["bound_evidence"] = (f"HBM {r['frac']:.2f} of peak (compulsory bytes); VALU issue "
                           f"{'%.2f' % valu_frac if valu_frac is not None else 'unmeasured'} of the launch "
                           f"({'ISA issue floor' if r.get('issue_frac') else 'PMC class-weighted' if vi.get('weighted_frac_of_simd_cycles') else 'PMC at 2 cycles per instruction, a lower bound' if valu_frac is not None else 'no ISA budget / PMC'}); "
                           f"SQ_WAIT_ANY / wave-cycles {'%.2f' % wait if wait is not None else 'unmeasured'}")
    if dom == "fused" and d5_bytes_per_cw:
        # SURVEY §8(d) D5 models a flooding decoder whose E*Z message state crosses HBM every iteration;
        # the fused kernel keeps that state on chip, so this is an equivalent rate, not traffic
        eq = d5_bytes_per_cw * B / (d["avg_ms"] / 1000.0) / 1e9
        r["d5_equivalent"] = {"bytes_per_cw": d5_bytes_per_cw, "gbs": round(eq, 1),
                              "note": "equivalent rate of the D5 streamed-state model; not HBM traffic"}
    return r


def hbm_ceilings(dev, gib=4.0):
    """Measured HBM ceilings: best of 5 launches of libnldpc's 16 B/lane copy, write
    and read probes over `gib` GiB, HIP-event timed; GB/s of bytes moved."""
    from nldpc import _lib
    L = _lib.lib()
    n = int(gib * (1 << 30) // 4) // 4 * 4
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty(n, dtype=torch.float32, device=dev)
    a.fill_(1.0)
    stream = _lib.stream_of(dev)
    out = {}
    for name, kind, byts in (("copy", 0, 8 * n), ("write", 1, 4 * n), ("read", 2, 4 * n), ("read_4b_lane", 3, 4 * n)):
        best = None
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.check(L.nldpc_hbm_probe(kind, b.data_ptr(), a.data_ptr(), n, stream), "nldpc_hbm_probe")
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        out[name] = round(byts / (best / 1000.0) / 1e9, 1)
    del a, b
    torch.cuda.empty_cache()
    return out


def launch_ranks(args):
    """`--gpus N` with N > 1 outside a torchrun environment: start the N rank processes here (one per
    GPU, torch.distributed.run on 127.0.0.1) before anything touches the GPU, and return their exit
    code.  Inside a torchrun environment WORLD_SIZE must equal --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks")
        return None
    if args.gpus <= 1:
        return None
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def run_workload(args, rank, world, local, dev, cus, ceilings):
    """One workload's line (args.workload, with its default batch / iterations unless given)."""
    gfile, Z, T, B = WORKLOADS[args.workload]
    T = args.iters or T
    B = args.batch or B
    bg = np.loadtxt(os.path.join(ROOT, "resources", gfile), int, delimiter="\t")
    if args.workload == "cfg5":
        return bench_train(args, rank, world, local, dev, bg, Z, T, B, cus, ceilings)
    return bench_decode(args, rank, world, local, dev, bg, Z, T, B, cus, ceilings)


# what a side line keeps of its workload's own line
SIDE_KEYS = ("value", "unit", "ms_per_step", "ms_per_step_median", "value_from_median", "steps", "warmup", "timing",
             "dtype", "config", "loss", "ber", "roofline")


def side_lines(args, rank, world, local, dev, cus, ceilings):
    """the default N=1 run also times every other single-GPU BASELINE config with the same
    timed() helper -- cfg5 (BASELINE configs[4]: the Boosted training step, forward + BCE + backward + Adam) and
    cfg2 (configs[1]: WiMAX z=24, B=4096, HIP-graph replay with the eager timing beside) -- each at its own default
    batch and iterations.  Reported under `side_lines`, never as `value`."""
    import copy
    out = {}
    for wl, steps, warmup in (("cfg5", args.steps, args.warmup), ("cfg2", args.side_steps_cfg2, 20)):
        a = copy.copy(args)
        a.workload, a.steps, a.warmup = wl, steps, warmup
        a.batch = a.iters = None
        a.no_sweep = a.no_count_only = a.no_cpu_baseline = True
        a.graph = "auto"
        torch.cuda.empty_cache()
        r = run_workload(a, rank, world, local, dev, cus, ceilings)
        if rank == 0:
            out[wl] = {k: r[k] for k in SIDE_KEYS if k in r}
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    from nldpc import distributed as nd_dist
    rank, world, local = nd_dist.init(args.backend)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {world} rank(s) are running")
    dev = torch.device("cuda", local if args.backend == "nccl" else local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count  # (not a hard-coded 256)
    # measured HBM ceilings, once, before any workload allocates
    ceilings = hbm_ceilings(dev) if (rank == 0 and not args.no_profile) else None
    res = run_workload(args, rank, world, local, dev, cus, ceilings)
    if (args.workload == "cfg3" and world == 1 and not args.no_side_lines and args.batch is None
            and args.iters is None):
        side = side_lines(args, rank, world, local, dev, cus, ceilings)
        if rank == 0:
            res["side_lines"] = side
    if rank == 0:
        print(json.dumps(res), flush=True)
    nd_dist.barrier(local)
    nd_dist.finalize()
    return res


def timed(args, local, dev, step, prof):
    from nldpc import distributed as nd_dist
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    nd_dist.barrier(local)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    prof.begin()
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record()
        step()
        e1.record()
    torch.cuda.synchronize(dev)
    nd_dist.barrier(local)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    step_ms = [e0.elapsed_time(e1) for e0, e1 in ev]  # per step on torch's stream (the decoder's stream)
    return elapsed, prof.end(), step_ms


def bench_decode(args, rank, world, local, dev, bg, Z, T, B, cus=256, ceilings=None):
    import neural_ldpc_decoder as nd
    from nldpc import distributed as nd_dist
    from nldpc.channel import awgn_llr, ber_counts, sigma_for

    M, N = bg.shape
    ucn = args.workload == "cfg3ucn"
    if ucn:  # Boosted MS, NW(1,1,2): per-edge CN and UCN weights, per-column VN weights (fused UCN kernel)
        from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
        from boosted_neural_ldpc_decoder.ConnectingMatrix import ConnectingMatrix
        from boosted_neural_ldpc_decoder.ConnectingMatrixTorch import ConnectingMatrixTorch
        from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
        from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig
        from nldpc.channel import boosted_code_rate
        conn = ConnectingMatrixTorch(ConnectingMatrix(Z, bg), device=dev)
        nw = tuple(int(v) for v in args.nw.split(","))
        model = BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NodeWeightSharingConfig(*nw),
                                         decoding_type=getattr(DecoderType, args.kind)).to(dev)
        model.eval()
        rate = boosted_code_rate(N, M)
    else:
        conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(Z, bg), device=dev)
        model = nd.NeuralLDPCDecoder(T, B, conn).to(dev)  # reference default parameters: w = 0.5, b = 0
        rate = (N - M) / (N - 2)  # reference code-rate formula (AWGNPassedDatagen.py:47 / neural :36)
    E = int(conn.sum_edge)
    offset, _ = nd_dist.shard(world * B, rank, world)  # weak scaling: rank r holds [r*B, (r+1)*B)
    xa = awgn_llr(B, N, Z, sigma_for(args.ebn0, rate), seed=2042, b_offset=offset, device=dev)
    xa_host = xa[:min(B, 2048)].cpu()  # the CPU baseline decodes these same Philox codewords
    torch.cuda.synchronize(dev)
    state = {}

    def step():
        state["outs"] = None
        state["outs"] = model(xa)

    use_graph = args.graph == "on" or (args.graph == "auto" and args.workload == "cfg2")
    graph_info = None
    with torch.no_grad():
        elapsed, prof, step_ms = timed(args, local, dev, step, Prof(not args.no_profile, args.steps * (2 * T + 2)))
        if use_graph:
            # the same module call captured once into a HIP graph (stream capture of the library's launch on
            # torch's stream; outputs in the graph's pool), each step one replay: the host path of a module
            # call (Python, argument checks, ctypes) leaves the timed loop.  The eager timing above gives the
            # per-kernel HIP-event profile (events cannot be recorded inside the graph) and is reported beside.
            eager = {"ms_per_step": round(1000.0 * nd_dist.max_time(elapsed, device=dev) / args.steps, 3),
                     "ms_per_step_median": round(statistics.median(step_ms), 3)}
            g = torch.cuda.CUDAGraph()
            state["outs"] = None
            with torch.cuda.graph(g):
                g_outs = model(xa)

            def gstep():
                g.replay()
                state["outs"] = g_outs

            elapsed, _, step_ms = timed(args, local, dev, gstep, Prof(False, 0))
            graph_info = {"replay": True, "eager": eager}
        counts = ber_counts(state["outs"])  # BER / FER per iteration, decoder convention bit = LLR > 0
        # the reference helper itself on the same outputs (literal rule bit = LLR < 0: ~1 - BER)
        from boosted_neural_ldpc_decoder.Functions import Functions
        (lit_bits, _), (lit_frames, _) = Functions.evaluate_ber_fer(
            torch.zeros((B, N * Z), dtype=torch.uint8, device=dev), state["outs"])
        n_cpu = min(B, 2048)  # the codewords the CPU baseline may decode: their GPU outputs, kept for comparison
        gpu_last = state["outs"][-1][:n_cpu].cpu()
        state.clear()
        # count-only decode: the same decode with the counting fused into the kernel and
        # no posteriors written -- reported beside the headline, never as `value`
        count_only = None
        if not args.no_count_only:
            cnt = {}

            def cstep():
                cnt["c"] = model.count_errors(xa)

            c_elapsed, cprof, _ = timed(args, local, dev, cstep, Prof(not args.no_profile, args.steps + 2))
            c_elapsed = nd_dist.max_time(c_elapsed, device=dev)
            count_only = {"value": round(world * B * args.steps / c_elapsed, 1), "unit": "codewords/s",
                          "ms_per_step": round(1000.0 * c_elapsed / args.steps, 3),
                          "kernel_avg_ms": (round(cprof["fused"][0] / cprof["fused"][1], 4)
                                            if cprof and cprof["fused"][1] else None),
                          "counts_equal_decode_then_count": bool(torch.equal(cnt["c"], counts))}
        sweep = None
        if args.workload == "cfg3" and not args.no_sweep:
            sweep = {"ebn0_db": [], "bit_errors": [], "frame_errors": []}
            for eb in np.arange(1.0, 4.01, 0.5):
                x = awgn_llr(B, N, Z, sigma_for(float(eb), rate), seed=2042, b_offset=offset, device=dev)
                c = nd_dist.sum_counts(model.count_errors(x)).cpu().numpy()  # fused counting (F2)
                sweep["ebn0_db"].append(float(eb))
                sweep["bit_errors"].append(int(c[-1, 0]))
                sweep["frame_errors"].append(int(c[-1, 1]))
                del x
    elapsed = nd_dist.max_time(elapsed, device=dev)
    med = nd_dist.max_time(statistics.median(step_ms) / 1000.0, device=dev)
    counts = nd_dist.sum_counts(counts).cpu().numpy()  # the one RCCL exchange: BER accounting
    if rank != 0:
        return None
    bits_total = world * B * N * Z
    tag = {"cfg3": "bg2_z384", "cfg3ucn": "bg2_z384", "cfg2": "wimax_z24"}.get(args.workload, f"z{Z}")
    wl = {"cfg3": f"cfg3 Neural BG2 set0 z={Z}, T={T}, all T posteriors written",
          "cfg3ucn": f"cfg3 decode with BoostedNeuralLDPCDecoder {args.kind} NW({args.nw}) "
                     f"(UCN {'on' if args.nw.split(',')[1] != '0' else 'off'}), BG2 set0 z={Z}, T={T}, all T posteriors written",
          "cfg2": f"cfg2 Neural WiMAX N=576 R=3/4 z={Z}, T={T}, all T posteriors written"}[args.workload]
    res = {
        "metric": METRIC,
        "value": round(world * B * args.steps / elapsed, 1),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "ms_per_step_median": round(1000.0 * med, 3),
        "value_from_median": round(world * B / med, 1),
        # the timing mode of ms_per_step / value (cfg2's auto mode replays a captured HIP graph; its eager
        # module-call timing stays in config.graph.eager)
        "timing": "graph_replay" if graph_info else "eager",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: all-zero codewords, BPSK/AWGN Eb/N0={args.ebn0} dB, on-device Philox; "
                + ("reference init weights (1.0)" if ucn else "reference default weights (w=0.5, b=0)"),
        "config": {"workload": wl, "model": "BoostedNeuralLDPCDecoder" if ucn else "NeuralLDPCDecoder", "global_batch": world * B, "per_gpu_batch": B,
                   "seq_len": N * Z, "iters": T, "parallelism": f"dp{world}"},
        "ber": {"ebn0_db": args.ebn0, "ber_last_iter": float(counts[-1, 0]) / bits_total,
                "fer_last_iter": float(counts[-1, 1]) / (world * B),
                "bit_errors_last_iter": int(counts[-1, 0]), "bits": bits_total,
                "ber_per_iter": [float(c) / bits_total for c in counts[:, 0]]},
    }
    if count_only is not None:
        res["count_only"] = count_only
    if graph_info is not None:
        res["config"]["graph"] = graph_info
    if sweep is not None:
        sweep["ber"] = [b / bits_total for b in sweep["bit_errors"]]
        sweep["fer"] = [f / (world * B) for f in sweep["frame_errors"]]
        sweep["codewords_per_point"] = world * B
        sweep["iteration"] = T
        res["ber_sweep"] = sweep
    # D7: Functions.evaluate_ber_fer's literal value on the same outputs (rank 0's shard; its inverted
    # decision rule reports ~1 - BER)
    res["ber"]["evaluate_ber_fer_literal_rank0"] = {"bit_errors_last_iter": lit_bits[-1], "bits": B * N * Z,
                                                    "frame_errors_last_iter": lit_frames[-1], "frames": B}
    if prof is not None:
        res["roofline"] = roofline(prof, kernel_bytes(B, E, N, Z, T), args.steps, B, Z, world, tag,
                                   4 * (2 * T * E * Z + (T + 1) * N * Z), ceilings, pmc_workload(args) + f"_B{B}",
                                   T=T, cus=cus)
    if world == 1 and not args.no_cpu_baseline and not ucn:
        res["cpu_baseline"] = cpu_baseline(bg, Z, T, xa_host, gpu_last, args.cpu_seconds)
    return res


def bench_train(args, rank, world, local, dev, bg, Z, T, B, cus=256, ceilings=None):
    """cfg5: one training step of BoostedNeuralLDPCDecoder per step (train_BoostedNeuralLDPCDecoder.py:278-294)."""
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.ConnectingMatrix import ConnectingMatrix
    from boosted_neural_ldpc_decoder.ConnectingMatrixTorch import ConnectingMatrixTorch
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig
    from nldpc import distributed as nd_dist
    from nldpc.channel import awgn_llr, ber_counts, boosted_code_rate, sigma_for

    M, N = bg.shape
    conn = ConnectingMatrixTorch(ConnectingMatrix(Z, bg), device=dev)
    model = BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NodeWeightSharingConfig(3, 0, 3),
                                     decoding_type=DecoderType.QMS, decoder_qms_qbit=5).to(dev)
    E = int(conn.sum_edge)
    criterion = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)
    opt = torch.optim.Adam(model.get_trainable_parameters(), lr=1e-3)
    offset, _ = nd_dist.shard(world * B, rank, world)
    sigma = sigma_for(args.ebn0, boosted_code_rate(N, M))
    xa = awgn_llr(B, N, Z, sigma, seed=2042, b_offset=offset, qbit=5, device=dev)  # datagen quantises (A12)
    y = torch.zeros(B, N * Z, device=dev)
    state = {}

    def step():
        model.train()
        opt.zero_grad()
        outs = model(xa, target_iter=list(range(T)))
        loss = criterion(outs, y, coeff_param=list(range(len(outs))))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        model._apply_constraints()
        state["loss"] = loss.detach()
        state["last"] = outs[-1].detach()

    elapsed, prof, step_ms = timed(args, local, dev, step, Prof(not args.no_profile, args.steps * (6 * T + 8)))
    counts = ber_counts([state["last"]])
    elapsed = nd_dist.max_time(elapsed, device=dev)
    med = nd_dist.max_time(statistics.median(step_ms) / 1000.0, device=dev)
    counts = nd_dist.sum_counts(counts).cpu().numpy()
    if rank != 0:
        return None
    res = {
        "metric": METRIC,
        "value": round(world * B * args.steps / elapsed, 1),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "ms_per_step_median": round(1000.0 * med, 3),
        "timing": "eager",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: all-zero codewords, BPSK/AWGN Eb/N0={args.ebn0} dB quantised q=5, on-device Philox; "
                "reference init weights (1.0)",
        "config": {"workload": f"cfg5 Boosted QMS q=5 NW(3,0,3) BG2 z={Z}, T={T}: forward + BCE + backward + "
                               "clip_grad_norm + Adam + clamp", "model": "BoostedNeuralLDPCDecoder",
                   "global_batch": world * B, "per_gpu_batch": B, "seq_len": N * Z, "iters": T,
                   "parallelism": f"dp{world}"},
        "loss": float(state["loss"]),
        "ber": {"ebn0_db": args.ebn0, "ber_last_iter": float(counts[-1, 0]) / (world * B * N * Z),
                "fer_last_iter": float(counts[-1, 1]) / (world * B)},
    }
    if prof is not None:
        res["roofline"] = roofline(prof, kernel_bytes(B, E, N, Z, T, train={"qms": True, "vn": True}), args.steps, B, Z,
                                   world, "bg2_z384", None, ceilings, f"{args.workload}_B{B}", T=T, cus=cus)
    return res


def cpu_baseline(bg, Z, T, xa_host, gpu_last, target_s):
    """Time the CPU oracle (edge-list restatement of NeuralLDPCDecoder.forward, pinned bit-exact to the
    reference; the reference itself cannot build z=384) on a bounded sample of the
    same workload -- the first codewords of the GPU's own Philox batch -- on this host's cores, and
    check its last-iteration output against the GPU's for those codewords."""
    from oracle.ldpc_oracle import OracleGraph, neural_forward
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cores = min(avail, int(os.environ.get("OMP_NUM_THREADS", avail)))
    torch.set_num_threads(cores)
    g = OracleGraph(bg, Z)
    E = g.E
    res = {}

    def run(b):
        w = [torch.full((E,), 0.5) for _ in range(T)]
        bb = [torch.zeros(E) for _ in range(T)]
        t0 = time.perf_counter()
        with torch.no_grad():
            outs = neural_forward(g, xa_host[:b], w, bb)
        res["last"] = outs[-1]
        return time.perf_counter() - t0

    # scale the sample until it takes about target_s (per-call overheads make small batches slow per
    # codeword, so one extrapolation from b=2 undershoots)
    b, t = 2, run(2)
    for _ in range(3):
        if t >= 0.6 * target_s:
            break
        b2 = int(max(b + 1, min(len(xa_host), b * target_s / max(t, 1e-3))))
        if b2 <= b:
            break
        b, t = b2, run(b2)
    cpu_name = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    same = bool(torch.equal(res["last"], gpu_last[:b]))
    return {"value": round(b / t, 3), "unit": "codewords/s", "cores": cores, "kind": "port",
            "sample": f"oracle/ldpc_oracle.py neural_forward (the reference's dense path cannot build z=384), "
                      f"{g.M}x{g.N} base graph z={Z}, T={T}, the first B={b} codewords of the GPU's own Philox batch, "
                      f"{t:.1f} s, torch {torch.__version__} CPU, {cpu_name}",
            "last_iteration_equals_gpu": same}


if __name__ == "__main__":
    main()
