"""World-size-2 data-parallel path on CPU with the gloo backend (the multi-process harness of the
N>1 path; the GPU runs it over RCCL). Covers: rendezvous on 127.0.0.1, id broadcast used to
bootstrap the native communicator, DistributedSampler shards partitioning the train split, and the
bucketed mean all-reduce over the executor's real bucket plan matching the fp32 sum within 1e-6."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cap_mb, out):
    import sys
    sys.path.insert(0, ROOT)
    import dtc_import
    dtc = dtc_import.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1) bootstrap blob exchange (the ncclUniqueId travels this way)
        blob = [bytes(range(128)) if rank == 0 else None]
        dist.broadcast_object_list(blob, src=0)
        assert blob[0] == bytes(range(128))
        # 2) sampler shards: disjoint, covering, same as the rank-addressed restatement
        dtc.data.fix_seed(42)
        train_idx, _ = dtc.data.train_valid_split()
        ds = torch.utils.data.Subset(torch.utils.data.TensorDataset(torch.arange(50000)), train_idx)
        sampler = dtc.data.DistributedSampler(ds)
        sampler.set_epoch(1)
        mine = list(iter(sampler))
        allidx = [None] * world
        dist.all_gather_object(allidx, mine)
        flat = sorted(i for part in allidx for i in part)
        assert flat == list(range(len(train_idx)))
        # 3) bucketed mean all-reduce over the executor's bucket plan
        lay = dtc.nn.Layout(100, cap_mb)
        n = lay.flat_numel
        grads = [torch.from_numpy(np.random.default_rng(1000 + r).standard_normal(n).astype(np.float32))
                 for r in range(world)]
        mine = grads[rank].clone()
        dtc.parallel.bucketed_allreduce_mean_(mine, lay.buckets, world, lambda t: dist.all_reduce(t))
        want = (sum(g.double() for g in grads) / world).float()
        err = ((mine.double() - want.double()).norm() / want.double().norm()).item()
        out[rank] = err
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cap_mb", [5, 25])
def test_two_rank_gloo(cap_mb):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cap_mb, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert set(out.keys()) == {0, 1}
    for r, e in out.items():
        assert e < 1e-6, (r, e)


def _probe_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    import dtc_import
    dtc = dtc_import.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = dtc.parallel.allreduce_probe(lambda t: dist.all_reduce(t), 1 << 20, torch.device("cpu"), world,
                                         iters=3, warmup=1)
        out[rank] = r
    finally:
        dist.destroy_process_group()


def test_allreduce_probe_gloo():
    """The bench's busBW probe (parallel.allreduce_probe) over a 2-rank gloo group: both ranks
    report the same (max-over-ranks) time and busBW = algBW * 2(W-1)/W against (W-1) xGMI links."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_probe_worker, args=(2, _port(), out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert r0 == r1
    assert r0["bytes"] == 1 << 20
    assert abs(r0["busbw_GBps"] - r0["algbw_GBps"]) <= 0.011 + 1e-6 * r0["algbw_GBps"]  # W=2: factor 1
    assert r0["peak_GBps"] == 153.0
    import dtc_import
    dtc = dtc_import.load()
    alg, bus = dtc.parallel.busbw(8 << 20, 1e-3, 8)
    assert abs(alg - 8.388608) < 1e-9 and abs(bus - alg * 1.75) < 1e-9


def _syncbn_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import ops
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def allreduce(a):
            t = torch.from_numpy(np.ascontiguousarray(a, np.float64))
            dist.all_reduce(t)
            return t.numpy()

        rng = np.random.default_rng(7)
        M, Cc = 48, 8  # ragged per-rank batches: rank r holds rows [lo, hi)
        x = rng.standard_normal((M, Cc)) * 2 + 0.5
        dy = rng.standard_normal((M, Cc))
        gamma, beta = rng.standard_normal(Cc), rng.standard_normal(Cc)
        rm0, rv0 = np.zeros(Cc), np.ones(Cc)
        cuts = [0, 20, M]
        lo, hi = cuts[rank], cuts[rank + 1]
        y, mean, invstd, rm, rv = ops.sync_bn_train_fwd(x[lo:hi], gamma, beta, allreduce, rm0, rv0)
        dx, dg, db = ops.sync_bn_train_bwd(dy[lo:hi], x[lo:hi], gamma, mean, invstd, allreduce)
        # DDP's mean of the per-rank dgamma / dbeta (pre-divided by world, SUM all-reduced)
        dgm = allreduce(np.stack([dg, db]) / world)
        yf, meanf, invf, rmf, rvf = ops.bn_train_fwd(x, gamma, beta, rm0, rv0)
        dxf, dgf, dbf = ops.bn_train_bwd(dy, x, gamma, meanf, invf)
        out[rank] = max(np.abs(y - yf[lo:hi]).max(), np.abs(rm - rmf).max(), np.abs(rv - rvf).max(),
                        np.abs(dx - dxf[lo:hi]).max(), np.abs(dgm[0] - dgf / world).max(),
                        np.abs(dgm[1] - dbf / world).max())
    finally:
        dist.destroy_process_group()


def test_sync_batchnorm_gloo():
    """SyncBatchNorm semantics of the executor (dtc_rn18_set_sync_bn) restated in
    the oracle and run over 2 gloo ranks with ragged shards (20 / 28 rows): each rank's output,
    running statistics and input gradient equal plain BatchNorm over the concatenated batch, and
    DDP's mean of the per-rank dgamma / dbeta equals the full-batch gradient / world."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_syncbn_worker, args=(2, _port(), out), nprocs=2, join=True)
    assert set(out.keys()) == {0, 1}
    for r, e in out.items():
        assert e < 1e-12, (r, e)
