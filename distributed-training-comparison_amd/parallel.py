"""DistributedDataParallel mirror with a native RCCL Reducer.

Reference: ``DDP(model, device_ids=[rank], find_unused_parameters=True)`` (src/ddp/trainer.py:31)
on a ``dist.init_process_group('nccl', 'tcp://127.0.0.1:3456', world, rank)`` group
(src/ddp/main.py:18-23). The reference relies on torch's C++ Reducer; here:

* process model and rendezvous stay ``torch.distributed`` (one process per GPU, TCPStore);
* a native RCCL communicator (include/dtc.h ``dtc_comm_*``) is bootstrapped over that group:
  rank 0 creates the ncclUniqueId, ``broadcast_object_list`` ships it, all ranks init;
* construction broadcasts parameters and BN buffers from rank 0 (DDP's C1), each training
  forward re-broadcasts the BN buffers (``broadcast_buffers=True``, C2);
* the gradient all-reduce (C4) runs INSIDE the native backward: each bucket (contiguous range
  of the flat gradient buffer, block granularity, closed at ``bucket_cap_mb``) is SUM
  all-reduced on the communicator's side stream right after backward produced it, so it
  overlaps the remaining backward kernels; gradients are pre-divided by the world size in the
  kernels that write them (DDP's mean);
* ``find_unused_parameters`` is accepted and ignored (ResNet-18 has no unused parameters).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ._native import NativeError, call, lib, ptr, stream_ptr

DTYPE_F32, DTYPE_BF16, DTYPE_I64 = 0, 1, 2
_DTYPES = {torch.float32: DTYPE_F32, torch.bfloat16: DTYPE_BF16, torch.int64: DTYPE_I64}


class Comm:
    """Native RCCL communicator over the ranks of a torch.distributed group."""

    def __init__(self, rank: int, world: int, unique_id: bytes, device: int):
        self.rank, self.world, self.device = rank, world, device
        self.handle = C.c_void_p()
        buf = C.create_string_buffer(unique_id, len(unique_id))
        call("dtc_comm_init", C.byref(self.handle), rank, world, buf, device)

    @staticmethod
    def unique_id() -> bytes:
        n = lib.dtc_comm_unique_id_bytes()
        buf = C.create_string_buffer(n)
        call("dtc_comm_get_unique_id", buf)
        return buf.raw

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "Comm":
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(rank, world, obj[0], device)

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        call("dtc_comm_allreduce_sum", self.handle, ptr(t), t.numel(), _DTYPES[t.dtype], stream_ptr())
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        call("dtc_comm_broadcast", self.handle, ptr(t), t.numel(), _DTYPES[t.dtype], root, stream_ptr())
        return t

    def close(self):
        if self.handle:
            lib.dtc_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def bucket_plan(layout) -> List[Tuple[int, int]]:
    """[(offset, numel)] of the gradient buckets, in the order backward completes them."""
    return list(layout.buckets)


def bucketed_allreduce_mean_(flat_grads: torch.Tensor, buckets: Sequence[Tuple[int, int]], world: int,
                             allreduce_fn) -> torch.Tensor:
    """Reducer semantics on a flat buffer: pre-divide by world, SUM all-reduce bucket by bucket
    (the native backward does the same with RCCL; this form drives any transport, e.g. the gloo
    process group of the CPU multi-process tests)."""
    flat_grads.div_(world)
    for off, n in buckets:
        allreduce_fn(flat_grads.narrow(0, off, n))
    return flat_grads


XGMI_LINK_GBPS = 153.0  # per xGMI link and direction on MI355X; 7 links per GPU


def xgmi_peak_busbw(world: int) -> float:
    """Ceiling of all-reduce bus bandwidth on one fully connected 8-GPU node: each rank reaches
    every peer over its own link, so W ranks drive (W-1) links per GPU (GB/s)."""
    return XGMI_LINK_GBPS * max(0, min(world, 8) - 1)


def busbw(nbytes: int, seconds: float, world: int) -> Tuple[float, float]:
    """(algBW, busBW) in GB/s for a SUM all-reduce of nbytes taking `seconds` (nccl-tests
    convention: busBW = algBW * 2(W-1)/W, the per-link traffic of a ring)."""
    alg = nbytes / seconds / 1e9
    return alg, alg * 2.0 * (world - 1) / world


def allreduce_probe(allreduce_fn, nbytes: int, device, world: int, iters: int = 20, warmup: int = 5,
                    group=None) -> dict:
    """Time `iters` back-to-back SUM all-reduces of an fp32 buffer of nbytes on the current
    stream (device events; on CPU wall clock) and return the slowest rank's algBW / busBW
    against the xGMI ceiling. allreduce_fn(tensor) is the transport under test: the native RCCL
    communicator the Reducer uses (Comm.allreduce_sum_) on GPUs, dist.all_reduce under gloo."""
    import time

    n = max(1, nbytes // 4)
    buf = torch.ones(n, dtype=torch.float32, device=device)
    cuda = buf.is_cuda
    for _ in range(warmup):
        allreduce_fn(buf)
    if cuda:
        torch.cuda.synchronize(device)
    dist.barrier(group=group)
    if cuda:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    t0 = time.perf_counter()
    for _ in range(iters):
        allreduce_fn(buf)
    if cuda:
        e1.record()
        torch.cuda.synchronize(device)
        sec = e0.elapsed_time(e1) / 1e3 / iters
    else:
        sec = (time.perf_counter() - t0) / iters
    t = torch.tensor([sec], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    sec = float(t.item())
    alg, bus = busbw(n * 4, sec, world)
    peak = xgmi_peak_busbw(world)
    return {"bytes": n * 4, "us": round(sec * 1e6, 2), "algbw_GBps": round(alg, 2), "busbw_GBps": round(bus, 2),
            "peak_GBps": peak, "frac": round(bus / peak, 4) if peak else None}


class DistributedDataParallel(nn.Module):
    def __init__(self, module, device_ids=None, output_device=None, dim=0, broadcast_buffers=True,
                 process_group=None, bucket_cap_mb=25, find_unused_parameters=False, **_ignored):
        super().__init__()
        if not dist.is_initialized():
            raise NativeError("DistributedDataParallel requires torch.distributed.init_process_group")
        self.module = module
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.world_size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        flat = module.flat  # raises unless the module already lives on a GPU
        device = flat.device.index if flat.device.index is not None else torch.cuda.current_device()
        if device_ids:
            d = device_ids[0]
            d = d.index if isinstance(d, torch.device) else int(d)
            if d != device:
                raise NativeError(f"device_ids={device_ids} but the module lives on cuda:{device}")
        with torch.cuda.device(device):
            self.comm = Comm.from_process_group(device, process_group)
            module.set_bucket_cap_mb(float(bucket_cap_mb))
            # a one-rank all-reduce is the identity: no side-stream fork/join inside the backward
            module._comm = self.comm if self.world_size > 1 else None
            module._grad_scale = 1.0 / self.world_size
            # C1: make every replica start from rank 0's state
            self.comm.broadcast_(flat.params, 0)
            self.comm.broadcast_(flat.bufs, 0)
            self.comm.broadcast_(flat.nbt, 0)
            flat.refresh_bf16()

    def forward(self, *inputs, **kwargs):
        if self.broadcast_buffers and self.world_size > 1 and self.module.training:
            flat = self.module.flat
            self.comm.broadcast_(flat.bufs, 0)  # C2: rank-0 BN running statistics
        return self.module(*inputs, **kwargs)

    @property
    def buckets(self):
        return self.module.buckets()


DDP = DistributedDataParallel
