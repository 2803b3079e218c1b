"""The multi-GPU path's host logic on CPU: two gloo ranks shard a batch, each decodes its shard,
and the SUM / MAX reductions (RCCL on the GPU box) give the single-process result.  The decoder
here is the CPU oracle (no GPU in this container); the sharding and reductions are the product's
(nldpc.distributed)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, SRC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    for p in (SRC, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from nldpc import distributed as ndd
    from oracle.ldpc_oracle import OracleGraph, ber_counts, neural_forward
    r, w, _ = ndd.init("gloo")
    assert (r, w) == (rank, world)
    bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
    g = OracleGraph(bg, 16)
    off, cnt = ndd.shard(total, rank, world)
    gen = torch.Generator().manual_seed(5)
    x_all = (2.0 * (-1 + 0.9 * torch.randn(total, 52, 16, generator=gen)) / 0.81).float()
    T = 3
    outs = neural_forward(g, x_all[off:off + cnt], [torch.full((g.E,), 0.5)] * T, [torch.zeros(g.E)] * T)
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
    bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
    g = OracleGraph(bg, 16)
    gen = torch.Generator().manual_seed(5)
    x_all = (2.0 * (-1 + 0.9 * torch.randn(total, 52, 16, generator=gen)) / 0.81).float()
    outs = neural_forward(g, x_all, [torch.full((g.E,), 0.5)] * 3, [torch.zeros(g.E)] * 3)
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
