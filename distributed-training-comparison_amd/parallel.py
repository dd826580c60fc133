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

from ._native import NativeError, call, lib, ptr, require_cuda, stream_ptr

DTYPE_F32, DTYPE_BF16, DTYPE_I64, DTYPE_F64 = 0, 1, 2, 3
_DTYPES = {torch.float32: DTYPE_F32, torch.bfloat16: DTYPE_BF16, torch.int64: DTYPE_I64, torch.float64: DTYPE_F64}


class Comm:
    """Native RCCL communicator over the ranks of a torch.distributed group."""

    def __init__(self, rank: int, world: int, unique_id: bytes, device: int):
        self.rank, self.world, self.device = rank, world, device
        self.handle = C.c_void_p()
        buf = C.create_string_buffer(unique_id, len(unique_id))
        call("dtc_comm_init", C.byref(self.handle), rank, world, buf, device)

    @classmethod
    def loopback(cls, device: int, factor: float = 2.0, world: int = 1) -> "Comm":
        """Test communicator (include/dtc.h dtc_comm_init_loopback): no RCCL; every all-reduce
        multiplies its buffer by `factor` on the stream the collective would use and is logged, so
        a single GPU can check which ranges the Reducer reduces, how often and when. It reports
        `world` ranks (factor == world: that many ranks holding identical data)."""
        self = cls.__new__(cls)
        self.rank, self.world, self.device = 0, world, device
        self.handle = C.c_void_p()
        call("dtc_comm_init_loopback", C.byref(self.handle), device, int(world), float(factor))
        return self

    def log(self) -> List[Tuple[int, int, bool]]:
        """Loopback communicator: [(device address, element count, is_bucket)] in issue order."""
        out = []
        for i in range(lib.dtc_comm_log_size(self.handle)):
            a, n, asy = C.c_uint64(), C.c_uint64(), C.c_int()
            call("dtc_comm_log_entry", self.handle, i, C.byref(a), C.byref(n), C.byref(asy))
            out.append((a.value, n.value, bool(asy.value)))
        return out

    def clear_log(self) -> None:
        call("dtc_comm_log_clear", self.handle)

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
        self.process_group = process_group
        self._sync_checked = set()
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
            # SyncBatchNorm: a communicator of its own (BN-sum all-reduces run on the compute
            # stream while the Reducer's bucket all-reduces run on its side stream)
            self.sync_comm = None
            if getattr(module, "_sync_bn", False) and self.world_size > 1:
                self.sync_comm = Comm.from_process_group(device, getattr(module, "_sync_bn_group", None) or process_group)
                module.set_sync_bn(self.sync_comm)
            # C1: make every replica start from rank 0's state
            self.comm.broadcast_(flat.params, 0)
            self.comm.broadcast_(flat.bufs, 0)
            self.comm.broadcast_(flat.nbt, 0)
            flat.refresh_bf16()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """`module.`-prefixed load (the reference's test() on its DDP model, ddp/trainer.py:108-119);
        the wrapped module's bf16 shadow is re-derived from the loaded fp32 parameters."""
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.module.sync_weights()
        return res

    def _check_sync_bn_batch(self, x) -> None:
        """SyncBN normalises with world x local count (the executor all-reduces compact sums, not
        per-rank counts as torch's all_gather does): every rank's batch must be the same size --
        checked once per input shape over the process group (drop_last samplers guarantee it)."""
        n = int(x.shape[0])
        if n in self._sync_checked:
            return
        sizes = [None] * self.world_size
        dist.all_gather_object(sizes, n, group=self.process_group)
        if len(set(sizes)) != 1:
            raise NativeError(f"SyncBatchNorm: per-rank batch sizes differ {sizes}; use equal shards")
        self._sync_checked.add(n)

    def forward(self, *inputs, **kwargs):
        if self.sync_comm is not None and self.module.training and inputs:
            self._check_sync_bn_batch(inputs[0])
        if self.broadcast_buffers and self.world_size > 1 and self.module.training:
            flat = self.module.flat
            self.comm.broadcast_(flat.bufs, 0)  # C2: rank-0 BN running statistics
        return self.module(*inputs, **kwargs)

    @property
    def buckets(self):
        return self.module.buckets()


DDP = DistributedDataParallel


# ----------------------------------------------------------------------------- DataParallel
class _Replica:
    """A non-primary replica of a native ResNet: its own flat parameter / gradient / buffer
    copies and executors on one device. Parameters and buffers are refreshed from the primary
    (the wrapped module) by every forward, as torch's replicate() does (C5)."""

    def __init__(self, model, device: torch.device):
        from .nn import FlatState

        self.model, self.device = model, device
        with torch.cuda.device(device):
            self.flat = FlatState(model.flat.layout, device)
        self._executors = {}

    def executor(self, batch: int, height: int, width: int, precision: str):
        from .nn import Executor

        key = (batch, height, width, precision)
        exe = self._executors.get(key)
        if exe is None:
            with torch.cuda.device(self.device):
                exe = Executor(self.flat, batch, height, width, self.model.num_classes, self.model._bucket_cap_mb,
                               precision=precision)
            self._executors[key] = exe
        return exe

    def pull(self, primary) -> None:
        """Broadcast (replicate) of the primary's fp32 parameters, their bf16 shadow and the BN
        buffers into this replica (device-to-device copies over xGMI for a peer GPU)."""
        with torch.cuda.device(self.device):
            self.flat.params.copy_(primary.params, non_blocking=True)
            self.flat.params_bf16.copy_(primary.params_bf16, non_blocking=True)
            self.flat.bufs.copy_(primary.bufs, non_blocking=True)
            self.flat.nbt.copy_(primary.nbt, non_blocking=True)


class _DPFn(torch.autograd.Function):
    """scatter -> replicate -> parallel_apply -> gather (forward) and its reverse (backward:
    gather's backward scatters dlogits, replicate's backward reduce-adds the replicas' gradients
    into the primary's flat gradient buffer on device_ids[0])."""

    @staticmethod
    def forward(ctx, x, anchor, dp):
        model = dp.module
        chunks = x.chunk(len(dp.device_ids))  # torch.nn.parallel.scatter's split of dim 0
        train = model.training
        prec = model.compute_precision()  # autocast is thread-local: decided once, here
        runs = []
        for i, c in enumerate(chunks):
            dev = dp.devices[i]
            with torch.cuda.device(dev):
                if i == 0:
                    exe = model.executor(c.shape[0], c.shape[2], c.shape[3], prec)
                else:
                    rep = dp._replica(i)
                    rep.pull(model.flat)
                    exe = rep.executor(c.shape[0], c.shape[2], c.shape[3], prec)
                xi = c.to(dev, non_blocking=True).contiguous()
                logits = torch.empty(c.shape[0], model.num_classes, dtype=torch.float32, device=dev)
                gen = exe.forward(xi, logits, train)
                runs.append((exe, gen, logits, xi))
        ctx.dp, ctx.runs = dp, [(r[0], r[1]) for r in runs]
        ctx.sizes = [c.shape[0] for c in chunks]
        return torch.cat([r[2].to(dp.devices[0], non_blocking=True) for r in runs])  # gather (C7)

    @staticmethod
    def backward(ctx, dlogits):
        dp = ctx.dp
        model = dp.module
        parts = dlogits.contiguous().float().split(ctx.sizes)
        for i, ((exe, gen), d) in enumerate(zip(ctx.runs, parts)):
            if exe.generation != gen:
                raise NativeError("DataParallel backward: a replica ran another forward since this graph was built")
            dev = dp.devices[i]
            with torch.cuda.device(dev):
                exe.backward(d.to(dev, non_blocking=True).contiguous(), 1.0, None)
        g0 = model.flat.grads
        for i in range(1, len(ctx.runs)):  # ReduceAddCoalesced onto device_ids[0] (C6)
            g0.add_(dp._replica(i).flat.grads.to(g0.device, non_blocking=True))
        model._ensure_grads()
        return None, None, None


class DataParallel(nn.Module):
    """nn.DataParallel(model) (reference src/dp/trainer.py:27) over native executors: ONE
    process driving every device in ``device_ids``. Each forward splits the batch along dim 0,
    refreshes every replica's parameters and BN buffers from the wrapped module (replicate), runs
    the replicas' native forwards (kernel launches are asynchronous, so the devices run
    concurrently from one host thread) and gathers the logits on device_ids[0]; backward runs the
    replicas' native backwards on their logits-gradient slices and sums their gradients into the
    module's. BatchNorm statistics are per replica, and only replica 0 -- the module itself --
    keeps its running-statistics update, exactly as torch's replicate() leaves them.
    A device id may repeat (replicas sharing one GPU) -- the single-GPU test of this path."""

    def __init__(self, module, device_ids=None, output_device=None, dim=0):
        super().__init__()
        if dim != 0:
            raise NotImplementedError("DataParallel scatters along dim 0 only (the reference's use)")
        self.module = module
        if device_ids is None:
            device_ids = list(range(torch.cuda.device_count()))
        self.device_ids = [d.index if isinstance(d, torch.device) else int(d) for d in device_ids]
        self.devices = [torch.device("cuda", d) for d in self.device_ids]
        if output_device is not None:
            od = output_device.index if isinstance(output_device, torch.device) else int(output_device)
            if od != self.device_ids[0]:
                raise NotImplementedError("output_device must be device_ids[0]")
        flat = module.flat  # raises unless the module already lives on a GPU
        if flat.device.index != self.device_ids[0]:
            raise NativeError(f"module must live on device_ids[0] (cuda:{self.device_ids[0]}), not {flat.device}")
        module._grad_scale = 1.0
        module._comm = None
        self._replicas = {}

    def _replica(self, i: int) -> _Replica:
        rep = self._replicas.get(i)
        if rep is None:
            rep = _Replica(self.module, self.devices[i])
            self._replicas[i] = rep
        return rep

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.module.sync_weights()  # the bf16 shadow the executors read
        return res

    def forward(self, x, *args, **kwargs):
        if args or kwargs:
            raise NotImplementedError("the native ResNet takes one input tensor")
        if len(self.device_ids) == 1:
            return self.module(x)
        require_cuda(x)
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [N,3,H,W] input, got {tuple(x.shape)}")
        if x.dtype != torch.float32:
            x = x.float()
        return _DPFn.apply(x, self.module._anchor, self)
