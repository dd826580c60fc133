"""W ranks with DISTINCT data through the product DDP path on one GPU.

The in-process thread-group communicator (include/dtc.h ``dtc_comm_init_thread_group``) gives W
native communicator handles whose collectives really move data between the ranks' buffers
(rank-ordered SUM into every buffer, root -> all copies), matched by call order as RCCL matches
them. Each rank runs in its own host thread with its own CUDA stream, model replica, executor and
data shard, exactly as one process per GPU would -- the DDP wrapper (C1/C2 broadcasts), the native
Reducer's bucketed all-reduces on its side stream inside the backward (C4), the barrier (C3) and
SyncBatchNorm's statistics all-reduces all go through the same C++ code as with RCCL.

Checks (north_star / SURVEY §8 a10, a11, f4; reference ddp/trainer.py:31, 156-157, README.md:40):
  * all-reduced gradients equal the fp32 sum of the ranks' no-communicator gradients within 1e-6
    relative (each rank pre-scaled by 1/W: DDP's mean), graphs on and off, bucket caps 1/5/25 MB;
  * the C1 construction broadcast gives every rank rank 0's parameters and buffers, the C2
    per-forward broadcast rank 0's BN running statistics;
  * SyncBatchNorm over W ranks with distinct shards equals plain BN over the concatenated batch:
    logits, DDP-averaged gradients, running statistics.
"""
import threading

import numpy as np
import pytest
import torch

from tests.conftest import rel_err

pytestmark = pytest.mark.gpu


def _run_ranks(fn, world):
    """fn(rank) in `world` threads, each on its own CUDA stream; re-raise the first failure."""
    out, errs = [None] * world, [None] * world
    streams = [torch.cuda.Stream() for _ in range(world)]

    def body(r):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(streams[r]):
                out[r] = fn(r)
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    for e in errs:
        if e is not None:
            raise e
    assert not any(t.is_alive() for t in ts), "a rank thread hung"
    return out


def _shard(world, batch, seed):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(batch, 3, 32, 32, generator=g) for _ in range(world)]
    ys = [torch.randint(0, 100, (batch,), generator=g) for _ in range(world)]
    return xs, ys


def _model(dtc, cuda, cap_mb, sync_bn=False):
    torch.manual_seed(42)
    m = dtc.ResNet18()
    if sync_bn:
        m = dtc.SyncBatchNorm.convert_sync_batchnorm(m)
    m = m.to(cuda)
    m.set_bucket_cap_mb(cap_mb)
    return m


@pytest.mark.parametrize("graphs,on_side", [(1, 0), (1, 1), (0, 0), (0, 1)])
@pytest.mark.parametrize("cap_mb", [1.0, 5.0, 25.0])
def test_ddp_two_ranks_distinct_data_allreduce_equals_fp32_sum(dtc, cuda, graphs, on_side, cap_mb):
    world, batch = 2, 32
    xs, ys = _shard(world, batch, seed=7 + int(cap_mb))
    _graphs_prev = dtc._native.lib.dtc_get_option(b"graphs")
    dtc._native.lib.dtc_set_option(b"graphs", graphs)
    dtc._native.lib.dtc_set_option(b"comm_on_side", on_side)
    try:
        # no-communicator reference: rank r's own gradient with the DDP pre-scale 1/W, from rank 0's
        # state (the C1 broadcast's result)
        ref = _model(dtc, cuda, cap_mb)
        crit = dtc.CrossEntropyLoss()
        ref._grad_scale = 1.0 / world
        local, bufs_after = [], []
        for r in range(world):
            bufs0 = ref.flat.bufs.clone()
            with dtc.autocast():
                crit(ref(xs[r].to(cuda)), ys[r].to(cuda)).backward()
            torch.cuda.synchronize()
            local.append(ref.flat.grads.double().cpu().numpy().copy())
            bufs_after.append(ref.flat.bufs.clone().cpu())
            ref.flat.bufs.copy_(bufs0)  # every rank's forward starts from rank 0's buffers (C2)
            ref.flat.nbt.sub_(1)
        expect = sum(local)  # the fp32 SUM of the pre-scaled per-rank gradients (exact in fp64 for W=2)

        comms = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
        models = [_model(dtc, cuda, cap_mb) for _ in range(world)]
        with torch.no_grad():  # rank 1 starts from a different state: C1 must overwrite it
            models[1].flat.params.add_(0.01)
            models[1].flat.bufs.add_(0.5)
        rank0_params = models[0].flat.params.clone()
        rank0_bufs = models[0].flat.bufs.clone()
        n_buckets = len(models[0].buckets())

        def rank(r):
            m = models[r]
            ddp = dtc.DistributedDataParallel(m, device_ids=[0], bucket_cap_mb=cap_mb, comm=comms[r])
            c1 = (m.flat.params.clone(), m.flat.bufs.clone())
            if r == 1:
                with torch.no_grad():  # C2: the forward's buffer broadcast must overwrite this
                    m.flat.bufs.mul_(3.0)
            comms[r].clear_log()
            crit_r = dtc.CrossEntropyLoss()
            x, y = xs[r].to(cuda), ys[r].to(cuda)
            for _ in range(2):  # first step (graph capture when on), then replay
                with dtc.autocast():
                    loss = crit_r(ddp(x), y)
                dtc._native.call("dtc_barrier", comms[r].handle, dtc._native.stream_ptr())  # C3
                loss.backward()
                g = m.flat.grads.double().cpu().numpy().copy()
                bufs = m.flat.bufs.clone().cpu()
                m.flat.bufs.copy_(rank0_bufs)  # rewind the running statistics for the replay step
                m.flat.nbt.sub_(1)
            return c1, g, bufs, comms[r].log()

        res = _run_ranks(rank, world)
        for r in range(world):
            c1, g, bufs, log = res[r]
            assert torch.equal(c1[0], rank0_params), "C1 parameter broadcast"
            assert torch.equal(c1[1], rank0_bufs), "C1 buffer broadcast"
            assert rel_err(g, expect) < 1e-6, (r, rel_err(g, expect))
            # C2: rank r's running statistics = rank 0's, updated by rank r's own batch
            assert torch.allclose(bufs, bufs_after[r], rtol=1e-5, atol=1e-6), r
            buckets = [(a, n) for a, n, is_bucket in log if is_bucket]
            assert len(buckets) == 2 * n_buckets, (r, len(buckets), n_buckets)  # two steps, each bucket once
        # both ranks end with identical gradients (every bucket reduced into every rank's buffer)
        assert np.array_equal(res[0][1], res[1][1])
    finally:
        dtc._native.lib.dtc_set_option(b"graphs", _graphs_prev)
        dtc._native.lib.dtc_set_option(b"comm_on_side", 1)


def test_sync_batchnorm_two_ranks_distinct_data_equals_concatenated_batch(dtc, cuda):
    world, batch = 2, 16
    xs, ys = _shard(world, batch, seed=21)
    # plain BN over the concatenated batch, mean loss over all world*batch images
    ref = _model(dtc, cuda, 25.0)
    crit = dtc.CrossEntropyLoss()
    with dtc.autocast():
        logits_ref = ref(torch.cat(xs).to(cuda))
        crit(logits_ref, torch.cat(ys).to(cuda)).backward()
    torch.cuda.synchronize()
    g_ref = ref.flat.grads.double().cpu().numpy().copy()
    bufs_ref = ref.flat.bufs.clone().cpu()
    logits_ref = logits_ref.detach().cpu()

    comms = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    syncs = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    models = [_model(dtc, cuda, 25.0, sync_bn=True) for _ in range(world)]

    def rank(r):
        m = models[r]
        ddp = dtc.DistributedDataParallel(m, device_ids=[0], comm=comms[r], sync_comm=syncs[r])
        with dtc.autocast():
            logits = ddp(xs[r].to(cuda))
            loss = dtc.CrossEntropyLoss()(logits, ys[r].to(cuda))
        loss.backward()
        return logits.detach().cpu(), m.flat.grads.double().cpu().numpy().copy(), m.flat.bufs.clone().cpu(), \
            syncs[r].log()

    res = _run_ranks(rank, world)
    for r in range(world):
        logits, g, bufs, log = res[r]
        assert rel_err(logits.numpy(), logits_ref[r * batch:(r + 1) * batch].numpy()) < 1e-2, r
        assert rel_err(g, g_ref) < 2e-2, (r, rel_err(g, g_ref))
        assert torch.allclose(bufs, bufs_ref, rtol=2e-2, atol=2e-3), (r, (bufs - bufs_ref).abs().max())
        # 20 BNs: a forward and a backward all-reduce each, plus the per-step batch-size check
        assert len(log) == 41, (r, len(log))
    # the ranks agree exactly on the all-reduced gradients
    assert np.array_equal(res[0][1], res[1][1])


def test_sync_batchnorm_unequal_shards_refused(dtc, cuda):
    """Every rank issues the same batch-size check each training forward (a per-rank cache
    could let one rank skip the collective while another enters it and hang); unequal shards raise on
    every rank instead of normalising with a wrong global count."""
    world = 2
    comms = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    syncs = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    models = [_model(dtc, cuda, 25.0, sync_bn=True) for _ in range(world)]

    def rank(r):
        ddp = dtc.DistributedDataParallel(models[r], device_ids=[0], comm=comms[r], sync_comm=syncs[r])
        x = torch.randn(8 + 4 * r, 3, 32, 32, device=cuda)
        try:
            with dtc.autocast():
                ddp(x)
        except dtc.NativeError as e:
            return str(e)
        return None

    msgs = _run_ranks(rank, world)
    assert all(m is not None and "batch sizes differ" in m for m in msgs), msgs


def test_sync_batchnorm_batch_change_on_one_rank_refused_on_every_rank(dtc, cuda):
    """equal shards (8, 8) on the first step, then only rank 1's batch changes (8, 12). The
    wait-or-defer decision is the same on every rank, so neither rank waits while the other enters the
    forward's SyncBN all-reduces (which would hang over RCCL): both ranks raise, at the same forward."""
    world = 2
    comms = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    syncs = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    models = [_model(dtc, cuda, 25.0, sync_bn=True) for _ in range(world)]

    def rank(r):
        ddp = dtc.DistributedDataParallel(models[r], device_ids=[0], comm=comms[r], sync_comm=syncs[r])
        for step, b in enumerate((8, 8 + 4 * r, 8, 8)):
            x = torch.randn(b, 3, 32, 32, device=cuda)
            try:
                with dtc.autocast():
                    ddp(x)
            except dtc.NativeError as e:
                return step, str(e)
        return None

    res = _run_ranks(rank, world)  # a hang would fail here ("a rank thread hung" / the 120 s group timeout)
    assert all(x is not None and "batch sizes differ" in x[1] for x in res), res
    assert res[0][0] == res[1][0] == 2, res  # refused one step late, on both ranks together


def test_sync_batchnorm_batch_change_refused_before_that_steps_backward(dtc, cuda):
    """with training steps (forward, loss, backward) the pending batch-size check is read before
    the native backward, so a mismatch on the LAST step is still refused -- on every rank, at that step's
    backward, before any gradient of it is written or all-reduced."""
    world = 2
    comms = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    syncs = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    models = [_model(dtc, cuda, 25.0, sync_bn=True) for _ in range(world)]

    def rank(r):
        ddp = dtc.DistributedDataParallel(models[r], device_ids=[0], comm=comms[r], sync_comm=syncs[r])
        crit = dtc.CrossEntropyLoss()
        for step, b in enumerate((8, 8 + 4 * r)):  # the mismatch is on the final step
            x = torch.randn(b, 3, 32, 32, device=cuda)
            y = torch.randint(0, 100, (b,), device=cuda)
            with dtc.autocast():
                loss = crit(ddp(x), y)
            try:
                loss.backward()
            except dtc.NativeError as e:
                return step, str(e)
        return None

    res = _run_ranks(rank, world)
    assert all(x is not None and "batch sizes differ" in x[1] for x in res), res
    assert res[0][0] == res[1][0] == 1, res


def test_thread_group_barrier_and_mismatch(dtc, cuda):
    """dtc_barrier over the thread group returns on every rank only after all ranks called it and each
    rank's own queued work finished; mismatched collectives are reported to every rank, not hung."""
    world = 2
    comms = dtc.parallel.Comm.thread_group(cuda.index or 0, world)
    order = []
    lock = threading.Lock()

    def rank(r):
        if r == 1:
            torch.cuda._sleep(20_000_000)  # rank 1 arrives with work still queued
        dtc._native.call("dtc_barrier", comms[r].handle, dtc._native.stream_ptr())
        with lock:
            order.append((r, torch.cuda.current_stream().query()))
        t = torch.ones(4 + r, device=cuda)  # mismatched counts
        try:
            comms[r].allreduce_sum_(t)
        except dtc.NativeError as e:
            return str(e)
        return None

    msgs = _run_ranks(rank, world)
    assert all(done for _, done in order), order
    assert all(m is not None and "mismatched" in m for m in msgs), msgs
