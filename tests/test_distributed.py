"""The multi-GPU path: one process per GPU, contiguous batch shards, the channel drawn
at the global codeword index, one SUM all_reduce of the [T, 2] error counters and a MAX of the time.

CPU (gloo, world size 2): the product's sharding and reductions (nldpc.distributed) over the channel's
counter layout (oracle/philox.py, the CPU restatement of the device generator, pinned to the Random123
known answers below), decoded by the oracle.
GPU: two rank processes on the one GPU of the box run the product end to end -- nldpc.channel.awgn_llr
at their b_offset, NeuralLDPCDecoder.count_errors / forward on their shard, the all_reduce -- and the
summed counts equal the single-process decode of the whole batch.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, SRC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_philox_known_answers():
    """Random123's philox4x32-10 known-answer vectors (kat_vectors: zero, all-ones and pi inputs)."""
    from oracle.philox import philox4x32_10
    cases = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
             ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
             ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
              (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in cases:
        got = philox4x32_10(np.array([ctr], dtype=np.uint32), key)[0]
        assert tuple(int(v) for v in got) == want


@pytest.mark.parametrize("L", [832, 19968, 6])
def test_channel_shards_draw_the_single_device_noise(L):
    """Counter = global codeword index: a shard starting at codeword b_offset draws exactly rows
    [b_offset, b_offset + B) of the single-device channel, for every split (L % 4 != 0 included)."""
    from nldpc.distributed import shard
    from oracle.philox import awgn_llr
    total = 13
    full = awgn_llr(total, L, 0.8, seed=2042)
    for world in (2, 3, 8):
        parts = []
        for r in range(world):
            off, cnt = shard(total, r, world)
            if cnt:
                parts.append(awgn_llr(cnt, L, 0.8, seed=2042, b_offset=off))
        assert np.array_equal(np.concatenate(parts), full)


def _worker(rank, world, port, total, q):
    for p in (SRC, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from nldpc import distributed as ndd
    from oracle.ldpc_oracle import OracleGraph, ber_counts, neural_forward
    from oracle.philox import awgn_llr
    r, w, _ = ndd.init("gloo")
    assert (r, w) == (rank, world)
    bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
    g = OracleGraph(bg, 16)
    off, cnt = ndd.shard(total, rank, world)
    x = torch.from_numpy(awgn_llr(cnt, 52 * 16, 0.9, seed=5, b_offset=off)).reshape(cnt, 52, 16)
    T = 3
    outs = neural_forward(g, x, [torch.full((g.E,), 0.5)] * T, [torch.zeros(g.E)] * T)
    counts = torch.tensor(ber_counts(outs, torch.zeros(cnt, 52 * 16)), dtype=torch.int64)
    ndd.sum_counts(counts)
    t = ndd.max_time(0.1 * (rank + 1))
    ndd.barrier()
    q.put((rank, counts.tolist(), t))
    ndd.finalize()


@pytest.mark.parametrize("total", [7, 8])
def test_sharded_decode_accounting_gloo(total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference of the same batch
    from oracle.ldpc_oracle import OracleGraph, ber_counts, neural_forward
    from oracle.philox import awgn_llr
    bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
    g = OracleGraph(bg, 16)
    x = torch.from_numpy(awgn_llr(total, 52 * 16, 0.9, seed=5)).reshape(total, 52, 16)
    outs = neural_forward(g, x, [torch.full((g.E,), 0.5)] * 3, [torch.zeros(g.E)] * 3)
    ref = [list(c) for c in ber_counts(outs, torch.zeros(total, 52 * 16))]
    for rank, counts, t in res:
        assert counts == ref
        assert t == pytest.approx(0.2)


def test_shard_partition():
    from nldpc.distributed import shard
    for total in (1, 7, 8, 65536 * 8 + 3):
        for world in (1, 2, 4, 8):
            spans = [shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            assert all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert sum(c for _, c in spans) == total


# ---------------------------------------------------------------- the product on the GPU, two ranks

def _gpu_worker(rank, world, port, total, T, q):
    for p in (SRC, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")  # both ranks share the box's one GPU; gloo carries the collectives
    try:
        import neural_ldpc_decoder as nd
        from nldpc import distributed as ndd
        from nldpc.channel import awgn_llr, ber_counts
        r, w, _ = ndd.init("gloo")
        dev = torch.device("cuda", 0)
        bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
        off, cnt = ndd.shard(total, r, w)
        conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(384, bg), device=dev)
        model = nd.NeuralLDPCDecoder(T, cnt, conn).to(dev)
        x = awgn_llr(cnt, 52, 384, 0.75, seed=2042, b_offset=off, device=dev)
        with torch.no_grad():
            fused = ndd.sum_counts(model.count_errors(x))            # fused count-only kernels
            decoded = ndd.sum_counts(ber_counts(model(x)))           # decode + device counter
        t = ndd.max_time(0.5 * (r + 1), device=dev)
        ndd.barrier()
        q.put((r, fused.cpu().tolist(), decoded.cpu().tolist(), t, None))
        ndd.finalize()
    except Exception as e:  # report instead of hanging the parent's queue
        q.put((rank, None, None, None, repr(e)))
        raise


def _bench_line(*args):
    """One bench.py run as a child process (the parent never touches the GPU): its JSON line."""
    import json
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--no-sweep", "--no-count-only", "--no-profile", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, f"bench.py {' '.join(args)} exited {r.returncode}:\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_bench_launches_ranks_and_sums_counts():
    """bench.py's own multi-rank path on the one-GPU box: --gpus 2 starts the two rank processes itself
    (launch_ranks -> torch.distributed.run), each decodes its shard of the global batch (b_offset), the
    error counters are summed and the time is the max over ranks; only the transport is gloo instead of
    RCCL (--backend gloo: both ranks on cuda:0).  The summed counts equal one rank decoding 2B."""
    B = 48
    two = _bench_line("--gpus", "2", "--backend", "gloo", "--batch", str(B))
    one = _bench_line("--gpus", "1", "--batch", str(2 * B))
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["global_batch"] == 2 * B and two["config"]["per_gpu_batch"] == B
    assert two["config"]["parallelism"] == "dp2" and two["scaling"] == "weak"
    assert two["ber"]["bit_errors_last_iter"] == one["ber"]["bit_errors_last_iter"] > 0
    assert two["ber"]["ber_per_iter"] == one["ber"]["ber_per_iter"]
    assert two["ber"]["fer_last_iter"] == one["ber"]["fer_last_iter"]


@pytest.mark.gpu
def test_two_rank_sharded_decode_on_gpu():
    """Two rank processes decode the two shards of a BG2 z=384 batch with the product (HIP kernels,
    on-device channel at the rank's b_offset) and all-reduce the counters: the result equals one
    process decoding the whole batch.  Started before this process touches the GPU (a process that
    has initialised the GPU must not start others)."""
    # conftest.py runs the multi-process GPU tests before any other GPU test, so this holds by construction
    assert not torch.cuda.is_initialized(), "rank processes must be started before this process touches the GPU"
    total, T, world = 9, 6, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, total, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r, fused, decoded, t, err in res:
        assert err is None, f"rank {r}: {err}"
    for p in procs:
        assert p.exitcode == 0
    import neural_ldpc_decoder as nd
    from nldpc.channel import awgn_llr, ber_counts
    dev = torch.device("cuda", 0)
    bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
    conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(384, bg), device=dev)
    model = nd.NeuralLDPCDecoder(T, total, conn).to(dev)
    x = awgn_llr(total, 52, 384, 0.75, seed=2042, device=dev)
    with torch.no_grad():
        ref = ber_counts(model(x)).cpu().tolist()
    assert sum(r[0] for r in ref) > 0  # the point has errors to count
    for r, fused, decoded, t, _ in res:
        assert fused == ref and decoded == ref, (r, fused, decoded, ref)
        assert t == pytest.approx(1.0)
