"""Benchmark: Neural BP decoding of 5G-NR BG2 z=384 at 20 iterations (BASELINE.json configs[2]/[3]).

    python bench.py [--gpus N --steps K --warmup W]            # N=1: one process
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W
    python bench.py --workload cfg2|cfg5                       # the other GPU configs (own lines)

Default workload cfg3: a step = one NeuralLDPCDecoder.forward over the rank's batch of B codewords
(default 65536 per GPU, weak scaling), T=20 iterations, every iteration's posterior written (the
reference API's output list).  cfg2: the same on WiMAX N=576 R=3/4 z=24, B=4096.  cfg5: one
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
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, Chip-level parameters)
METRIC = "codewords/sec + BER@Eb/N0, 5G-NR BG2 z=384, 20 iters, 1/2/4/8 MI355X"
KINDS = ("vn", "cn", "post", "fused", "vnb", "cnb", "fusedb")
KERNEL_NAMES = {"vn": "vn_kernel", "cn": "cn_kernel", "post": "vn_kernel (final posterior)",
                "fused": "fused_<graph>::kernel", "vnb": "vnb_kernel", "cnb": "cnb_kernel", "fusedb": "fusedb_<graph>::bwd_kernel"}
WORKLOADS = {
    # name: (base graph file, Z, T, default per-GPU batch)
    "cfg3": ("basegraph2_set0.txt", 384, 20, 65536),
    "cfg2": ("wman_N0576_R34_z24.txt", 24, 20, 4096),
    "cfg5": ("basegraph2_set0.txt", 384, 50, 2048),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
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
    return ap.parse_args()


def kernel_bytes(B, E, N, Z, T):
    """Algorithmic HBM bytes of one decode (all launches of a kind together), DESIGN.md §4.

    fused: SURVEY.md §8(d) D5's per-codeword figure 4*(2*T*E*Z + (T+1)*N*Z) (a flooding decoder whose
    message state is streamed once per iteration, plus the channel and the T posteriors) x B -- the
    figure the metric's roofline is defined on; the register-resident kernel moves only the
    compulsory part 4*(T+1)*N*Z itself (reported separately, and measured by PMC in profiles/).
    vn/cn/post: the streaming kernels' own fp32 message traffic; vnb/cnb: the backward kernels'
    (SURVEY D5 cfg5 model: 4*(3*E*Z + N*Z) per codeword-iteration, split VN/CN as below)."""
    f = 4
    vn_first = B * f * (E * Z + N * Z)            # read xa, write v2c (all-zero state: no c2v read)
    vn = B * f * (2 * E * Z + 2 * N * Z)          # read c2v + xa, write v2c + previous posterior
    cn = B * f * (2 * E * Z)                      # gather v2c, scatter c2v
    post = B * f * (E * Z + 2 * N * Z)            # read c2v + xa, write the last posterior
    fused = B * f * (2 * T * E * Z + (T + 1) * N * Z)
    vnb = B * f * (E * Z + N * Z)                 # per iteration: grad of the posterior in, grad v2c out
    cnb = B * f * (2 * E * Z)                     # per iteration: saved v2c + grad c2v in
    return {"vn": vn_first + (T - 1) * vn, "cn": T * cn, "post": post, "fused": fused,
            "fused_compulsory": B * f * (T + 1) * N * Z, "vnb": (T + 1) * vnb, "cnb": T * cnb,
            "fusedb": B * f * T * (3 * E * Z + N * Z)}


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


def roofline(prof, kb, steps, B, Z, elapsed, d5_bytes_per_cw, world, graph_tag):
    per = {}
    for k in KINDS:
        ms_tot, n = prof[k]
        if n:
            byts = kb[k] * steps
            per[k] = {"avg_ms": ms_tot / n, "launches": n, "gbs": byts / (ms_tot / 1000.0) / 1e9,
                      "alg_bytes_per_launch": byts / n}
            if k == "fused":
                per[k]["compulsory_gbs"] = kb["fused_compulsory"] * steps / (ms_tot / 1000.0) / 1e9
    dom = max(per, key=lambda k: prof[k][0])
    d = per[dom]
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(f"{dom}_B{B}_Z{Z}")
            if isinstance(traffic, dict):
                traffic = traffic.get("bytes")
        except Exception:
            traffic = None
    r = {"bound": "hbm", "kernel": KERNEL_NAMES[dom].replace("<graph>", graph_tag),
         "achieved": round(d["gbs"], 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
         "frac": round(d["gbs"] / PEAK_HBM_GBS, 4), "traffic": traffic,
         "alg_bytes_per_launch": d["alg_bytes_per_launch"], "avg_launch_ms": round(d["avg_ms"], 4),
         "per_kernel": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in per.items()},
         "decode_equiv_gbs_survey_formula": round(d5_bytes_per_cw * world * B * steps / elapsed / 1e9, 1)}
    if dom == "fused":
        # achieved uses SURVEY D5's per-codeword bytes (message state streamed once per iteration);
        # the fused kernel keeps that state in registers/LDS, so frac can exceed 1.  The kernel's
        # own HBM floor is the channel + T posteriors:
        cg = d["compulsory_gbs"]
        r["compulsory"] = {"bytes_per_launch": kb["fused_compulsory"], "achieved": round(cg, 1),
                           "frac": round(cg / PEAK_HBM_GBS, 4)}
        r["note"] = ("frac > 1: D5 assumes the E*Z message state streamed through HBM every iteration; "
                     "the fused kernel keeps it on chip and is VALU-issue bound (DESIGN.md 4.1)")
    return r


def main():
    args = parse()
    from nldpc import distributed as nd_dist
    rank, world, local = nd_dist.init("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    gfile, Z, T, B = WORKLOADS[args.workload]
    T = args.iters or T
    B = args.batch or B
    bg = np.loadtxt(os.path.join(ROOT, "resources", gfile), int, delimiter="\t")
    if args.workload == "cfg5":
        res = bench_train(args, rank, world, local, dev, bg, Z, T, B)
    else:
        res = bench_decode(args, rank, world, local, dev, bg, Z, T, B)
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
    prof.begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    nd_dist.barrier(local)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    return elapsed, prof.end()


def bench_decode(args, rank, world, local, dev, bg, Z, T, B):
    import neural_ldpc_decoder as nd
    from nldpc import distributed as nd_dist
    from nldpc.channel import awgn_llr, ber_counts, sigma_for

    M, N = bg.shape
    conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(Z, bg), device=dev)
    model = nd.NeuralLDPCDecoder(T, B, conn).to(dev)  # reference default parameters: w = 0.5, b = 0
    E = int(conn.sum_edge)
    rate = (N - M) / (N - 2)  # reference code-rate formula (AWGNPassedDatagen.py:47 / neural :36)
    offset, _ = nd_dist.shard(world * B, rank, world)  # weak scaling: rank r holds [r*B, (r+1)*B)
    xa = awgn_llr(B, N, Z, sigma_for(args.ebn0, rate), seed=2042, b_offset=offset, device=dev)
    torch.cuda.synchronize(dev)
    state = {}

    def step():
        state["outs"] = None
        state["outs"] = model(xa)

    with torch.no_grad():
        elapsed, prof = timed(args, local, dev, step, Prof(not args.no_profile, args.steps * (2 * T + 2)))
        counts = ber_counts(state["outs"])  # BER / FER per iteration, decoder convention bit = LLR > 0
        state.clear()
        # count-only decode: the same decode with the counting fused into the kernel and
        # no posteriors written -- reported beside the headline, never as `value`
        count_only = None
        if not args.no_count_only:
            cnt = {}

            def cstep():
                cnt["c"] = model.count_errors(xa)

            c_elapsed, cprof = timed(args, local, dev, cstep, Prof(not args.no_profile, args.steps + 2))
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
    counts = nd_dist.sum_counts(counts).cpu().numpy()  # the one RCCL exchange: BER accounting
    if rank != 0:
        return None
    bits_total = world * B * N * Z
    tag = {"cfg3": "bg2_z384", "cfg2": "wimax_z24"}.get(args.workload, f"z{Z}")
    wl = {"cfg3": f"cfg3 Neural BG2 set0 z={Z}, T={T}, all T posteriors written",
          "cfg2": f"cfg2 Neural WiMAX N=576 R=3/4 z={Z}, T={T}, all T posteriors written"}[args.workload]
    res = {
        "metric": METRIC,
        "value": round(world * B * args.steps / elapsed, 1),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: all-zero codewords, BPSK/AWGN Eb/N0={args.ebn0} dB, on-device Philox; "
                "reference default weights (w=0.5, b=0)",
        "config": {"workload": wl, "model": "NeuralLDPCDecoder", "global_batch": world * B, "per_gpu_batch": B,
                   "seq_len": N * Z, "iters": T, "parallelism": f"dp{world}"},
        "ber": {"ebn0_db": args.ebn0, "ber_last_iter": float(counts[-1, 0]) / bits_total,
                "fer_last_iter": float(counts[-1, 1]) / (world * B),
                "bit_errors_last_iter": int(counts[-1, 0]), "bits": bits_total,
                "ber_per_iter": [float(c) / bits_total for c in counts[:, 0]]},
    }
    if count_only is not None:
        res["count_only"] = count_only
    if sweep is not None:
        sweep["ber"] = [b / bits_total for b in sweep["bit_errors"]]
        sweep["fer"] = [f / (world * B) for f in sweep["frame_errors"]]
        sweep["codewords_per_point"] = world * B
        sweep["iteration"] = T
        res["ber_sweep"] = sweep
    if prof is not None:
        res["roofline"] = roofline(prof, kernel_bytes(B, E, N, Z, T), args.steps, B, Z, elapsed,
                                   4 * (2 * T * E * Z + (T + 1) * N * Z), world, tag)
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(bg, Z, T, sigma_for(args.ebn0, rate), args.cpu_seconds)
    return res


def bench_train(args, rank, world, local, dev, bg, Z, T, B):
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

    elapsed, prof = timed(args, local, dev, step, Prof(not args.no_profile, args.steps * (6 * T + 8)))
    counts = ber_counts([state["last"]])
    elapsed = nd_dist.max_time(elapsed, device=dev)
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
        res["roofline"] = roofline(prof, kernel_bytes(B, E, N, Z, T), args.steps, B, Z, elapsed,
                                   4 * (2 * T * E * Z + (T + 1) * N * Z) + 4 * T * (3 * E * Z + N * Z), world,
                                   "bg2_z384")
    return res


def cpu_baseline(bg, Z, T, sigma, target_s):
    """Time the CPU oracle (edge-list restatement of NeuralLDPCDecoder.forward, pinned bit-exact to the
    reference) on a bounded sample of the same workload, on this host's cores."""
    from oracle.ldpc_oracle import OracleGraph, neural_forward
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cores = min(avail, int(os.environ.get("OMP_NUM_THREADS", avail)))
    torch.set_num_threads(cores)
    g = OracleGraph(bg, Z)
    E = g.E

    def run(b):
        gen = torch.Generator().manual_seed(7)
        x = (2.0 * (-1.0 + sigma * torch.randn(b, g.N, Z, generator=gen, dtype=torch.float64)) / sigma ** 2).float()
        w = [torch.full((E,), 0.5) for _ in range(T)]
        bb = [torch.zeros(E) for _ in range(T)]
        t0 = time.perf_counter()
        with torch.no_grad():
            neural_forward(g, x, w, bb)
        return time.perf_counter() - t0

    # scale the sample until it takes about target_s (per-call overheads make small batches slow per
    # codeword, so one extrapolation from b=2 undershoots)
    b, t = 2, run(2)
    for _ in range(3):
        if t >= 0.6 * target_s:
            break
        b2 = int(max(b + 1, min(2048, b * target_s / max(t, 1e-3))))
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
    return {"value": round(b / t, 3), "unit": "codewords/s", "cores": cores, "kind": "port",
            "sample": f"oracle/ldpc_oracle.py neural_forward, {g.M}x{g.N} base graph z={Z}, T={T}, B={b} codewords, "
                      f"{t:.1f} s, torch {torch.__version__} CPU, {cpu_name}"}


if __name__ == "__main__":
    main()
