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

    @classmethod
    def thread_group(cls, device: int, world: int) -> List["Comm"]:
        """In-process thread-group communicator (include/dtc.h dtc_comm_init_thread_group): `world`
        ranks on one device, rank r driven by its own host thread. Collectives really move data
        between the ranks' buffers (rank-ordered SUM, root -> all copies), so one GPU runs W ranks
        with distinct data through the product Reducer, broadcasts and SyncBN."""
        arr = (C.c_void_p * world)()
        call("dtc_comm_init_thread_group", arr, int(world), int(device))
        out = []
        for r in range(world):
            c = cls.__new__(cls)
            c.rank, c.world, c.device = r, world, device
            c.handle = C.c_void_p(arr[r])
            out.append(c)
        return out

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


_WORLD_COMM = [None]  # the default group's native communicator (set by DistributedDataParallel)


def barrier(group=None) -> None:
    """``torch.distributed.barrier()`` (reference ddp/trainer.py:156) on the native
    communicator (include/dtc.h ``dtc_barrier``): returns once every rank reached it and this rank's
    queued GPU work has finished -- torch's NCCL barrier does the same with a one-element all-reduce
    and a stream synchronize, plus a device fill kernel for its token. Here the token is the
    communicator's own, the all-reduce runs on the Reducer's side stream (one stream per
    communicator) and the host polls the completion event instead of a sleeping wait (the GPU
    queue is empty until the host returns). Before a DistributedDataParallel exists, or for
    another group, it is ``torch.distributed.barrier``."""
    comm = _WORLD_COMM[0]
    if group is None and comm is not None and comm.handle:
        call("dtc_barrier", comm.handle if comm.world > 1 else None, stream_ptr())
    elif dist.is_available() and dist.is_initialized():
        dist.barrier(group)
    else:
        call("dtc_barrier", None, stream_ptr())


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
    """``DDP(module, device_ids=[rank], find_unused_parameters=True)`` (reference ddp/trainer.py:31).

    The communicators are bootstrapped over ``process_group`` (torch.distributed). ``comm=`` (and
    ``sync_comm=`` for SyncBatchNorm) take native communicators directly instead -- e.g. the ranks of
    ``Comm.thread_group``, which runs W ranks on one GPU from W host threads (tests)."""

    def __init__(self, module, device_ids=None, output_device=None, dim=0, broadcast_buffers=True,
                 process_group=None, bucket_cap_mb=25, find_unused_parameters=False, comm=None, sync_comm=None,
                 **_ignored):
        super().__init__()
        if comm is None and not dist.is_initialized():
            raise NativeError("DistributedDataParallel requires torch.distributed.init_process_group")
        self.module = module
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        if comm is not None:
            self.world_size, self.rank = comm.world, comm.rank
        else:
            self.world_size = dist.get_world_size(process_group)
            self.rank = dist.get_rank(process_group)
        self.process_group = process_group
        self._cnt = None  # SyncBN batch-size check (see _check_sync_bn_batch)
        flat = module.flat  # raises unless the module already lives on a GPU
        device = flat.device.index if flat.device.index is not None else torch.cuda.current_device()
        if device_ids:
            d = device_ids[0]
            d = d.index if isinstance(d, torch.device) else int(d)
            if d != device:
                raise NativeError(f"device_ids={device_ids} but the module lives on cuda:{device}")
        with torch.cuda.device(device):
            self.comm = comm if comm is not None else Comm.from_process_group(device, process_group)
            if process_group is None and comm is None:
                _WORLD_COMM[0] = self.comm  # barrier() of the default group runs on it
            module.set_bucket_cap_mb(float(bucket_cap_mb))
            # a one-rank all-reduce is the identity: no side-stream fork/join inside the backward
            module._comm = self.comm if self.world_size > 1 else None
            module._grad_scale = 1.0 / self.world_size
            # SyncBatchNorm: a communicator of its own (BN-sum all-reduces run on the compute
            # stream while the Reducer's bucket all-reduces run on its side stream)
            self.sync_comm = None
            if getattr(module, "_sync_bn", False) and self.world_size > 1:
                self.sync_comm = sync_comm if sync_comm is not None else Comm.from_process_group(
                    device, getattr(module, "_sync_bn_group", None) or process_group)
                module.set_sync_bn(self.sync_comm)
                module._pre_backward = self._flush_sync_bn_check
            # C1: make every replica start from rank 0's state -- on the Reducer's communicator,
            # ordered after the caller's stream (the module's parameters were written there)
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
        per-rank counts as torch's all_gather does), so every rank's batch must be the same size.
        Every training forward of every rank issues the same check (one 2-double SUM all-reduce of
        (n, n^2) on the SyncBN communicator: sizes are equal iff W * sum(n^2) == sum(n)^2), so the
        ranks' collectives always match (no per-rank cache deciding who enters). Whether the
        host waits is decided the same way on every rank: the FIRST check is waited for
        (every rank is on its first training forward), every later one is read before that forward's
        backward (_flush_sync_bn_check) or, for a forward without backward, at the next training forward. A batch size that changes on one rank after the first step is therefore refused before
        that step's backward, on every rank at the same step: no rank ever waits for a result while
        another has gone on into the forward's SyncBN all-reduces."""
        n = int(x.shape[0])
        dev = self.module.flat.device
        if self._cnt is None:
            self._cnt = {"dev": torch.zeros(2, dtype=torch.float64, device=dev),
                         "host": torch.zeros(2, dtype=torch.float64, pin_memory=True),
                         "ev": None, "first": True}
        st = self._cnt
        if st["ev"] is not None:  # the previous step's check
            st["ev"].synchronize()
            st["ev"] = None
            self._assert_equal_batches(st["host"])
        st["dev"].copy_(torch.tensor([float(n), float(n) * n], dtype=torch.float64), non_blocking=False)
        self.sync_comm.allreduce_sum_(st["dev"])
        st["host"].copy_(st["dev"], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        st["ev"] = ev
        if st["first"]:
            st["first"] = False
            ev.synchronize()
            st["ev"] = None
            self._assert_equal_batches(st["host"])

    def _flush_sync_bn_check(self) -> None:
        """Before the native backward of a training step: read this step's pending batch-size
        check (its 2-double all-reduce was issued before the forward's SyncBN collectives, so it has long
        completed once the backward is issued after the reference's per-step barrier). Every rank reads it
        at the same point of the same step, so unequal shards are refused on every rank BEFORE their
        backward and optimizer step -- also on the last step of training -- instead of one forward late."""
        st = self._cnt
        if st is not None and st["ev"] is not None:
            st["ev"].synchronize()
            st["ev"] = None
            self._assert_equal_batches(st["host"])

    def _assert_equal_batches(self, h) -> None:
        s1, s2 = float(h[0]), float(h[1])
        if abs(self.world_size * s2 - s1 * s1) > 0.5:
            raise NativeError(f"SyncBatchNorm: per-rank batch sizes differ (sum {s1:.0f}, sum of squares "
                              f"{s2:.0f} over {self.world_size} ranks); use equal shards")

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
class DPGroup:
    """Native DataParallel group over `device_ids` (include/dtc.h dtc_dp_*): one grouped RCCL
    broadcast / reduce per call over distinct devices (ncclCommInitAll, one process), or on-device
    copies + a HIP reduce-add kernel when every replica shares one device."""

    def __init__(self, device_ids):
        self.device_ids = list(device_ids)
        n = len(self.device_ids)
        arr = (C.c_int * n)(*self.device_ids)
        self.handle = C.c_void_p()
        call("dtc_dp_create", C.byref(self.handle), n, arr)
        self.local = bool(lib.dtc_dp_is_local(self.handle))

    def _streams(self):
        return (C.c_void_p * len(self.device_ids))(*[stream_ptr(torch.cuda.current_stream(d))
                                                     for d in self.device_ids])

    def broadcast(self, tensors) -> None:
        """tensors[i] on device_ids[i]; tensors[0] (the module's) is the source (C5)."""
        n = tensors[0].numel()
        bufs = (C.c_void_p * len(tensors))(*[ptr(t) for t in tensors])
        call("dtc_dp_broadcast", self.handle, bufs, n, _DTYPES[tensors[0].dtype], self._streams())

    def reduce_add(self, tensors) -> None:
        """tensors[0] += sum of the others (fp32), onto device_ids[0] (C7)."""
        n = tensors[0].numel()
        bufs = (C.c_void_p * len(tensors))(*[ptr(t) for t in tensors])
        call("dtc_dp_reduce_add", self.handle, bufs, n, self._streams())

    def close(self):
        if getattr(self, "handle", None):
            lib.dtc_dp_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def _copy_peer(dst: torch.Tensor, src: torch.Tensor, stream) -> None:
    call("dtc_copy_peer", ptr(dst), dst.device.index, ptr(src), src.device.index, src.numel() * src.element_size(),
         stream_ptr(stream))


def _order_after(dst_dev: torch.device, src_dev: torch.device) -> None:
    """Make dst_dev's current stream wait for everything issued so far on src_dev's current stream."""
    if dst_dev == src_dev:
        return
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(src_dev))
    torch.cuda.current_stream(dst_dev).wait_event(ev)


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
        self._io = {}

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

    def io(self, name: str, shape, dtype=torch.float32) -> torch.Tensor:
        """Cached per-replica staging buffer (input chunk, logits, dlogits) on this replica's device."""
        t = self._io.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self._io[name] = t
        return t


class _DPFn(torch.autograd.Function):
    """scatter -> replicate -> parallel_apply -> gather (forward) and its reverse (backward:
    gather's backward scatters dlogits, replicate's backward reduce-adds the replicas' gradients
    into the primary's flat gradient buffer on device_ids[0]). Every byte moves through the native
    library: replicate / reduce-add as grouped RCCL collectives (or on-device copies + a HIP add
    kernel for replicas sharing a device), scatter / gather as peer copies, or as plain views into
    the caller's tensors where a replica shares device_ids[0] (no copy at all)."""

    @staticmethod
    def forward(ctx, x, anchor, dp):
        model = dp.module
        dev0 = dp.devices[0]
        sizes = [c.shape[0] for c in x.chunk(len(dp.device_ids))]  # torch.nn.parallel.scatter's split
        offs = [sum(sizes[:i]) for i in range(len(sizes))]
        train = model.training
        prec = model.compute_precision()  # autocast is thread-local: decided once, here
        reps = [None] + [dp._replica(i) for i in range(1, len(sizes))]
        # C5 replicate: fp32 master parameters, their bf16 shadow, BN buffers -- one call each
        flats = [model.flat] + [r.flat for r in reps[1:]]
        for i in range(1, len(flats)):
            _order_after(dp.devices[i], dev0)  # the replicas receive after the module's last update
        dp.group.broadcast([f.params for f in flats])
        dp.group.broadcast([f.params_bf16 for f in flats])
        dp.group.broadcast([f.bufs for f in flats])
        dp.group.broadcast([f.nbt for f in flats])
        out = torch.empty(x.shape[0], model.num_classes, dtype=torch.float32, device=dev0)
        runs = []
        for i, n in enumerate(sizes):
            dev = dp.devices[i]
            xi = x[offs[i]:offs[i] + n]
            with torch.cuda.device(dev):
                exe = (model if i == 0 else reps[i]).executor(n, x.shape[2], x.shape[3], prec)
                if dev == dev0:  # the chunk and the logits slice are views: no copies (C6 on one device)
                    lo = out[offs[i]:offs[i] + n]
                else:
                    xd = reps[i].io("x", xi.shape)
                    _order_after(dev, dev0)
                    _copy_peer(xd, xi, torch.cuda.current_stream(dev))
                    xi = xd
                    lo = reps[i].io("logits", (n, model.num_classes))
                gen = exe.forward(xi, lo, train)
                runs.append((exe, gen, lo))
        for i, (_, _, lo) in enumerate(runs):  # C6 gather onto device_ids[0]
            if dp.devices[i] != dev0:
                _order_after(dev0, dp.devices[i])
                _copy_peer(out[offs[i]:offs[i] + sizes[i]], lo, torch.cuda.current_stream(dev0))
        ctx.dp, ctx.runs, ctx.sizes, ctx.offs = dp, [(r[0], r[1]) for r in runs], sizes, offs
        return out

    @staticmethod
    def backward(ctx, dlogits):
        dp = ctx.dp
        model = dp.module
        dev0 = dp.devices[0]
        dl = dlogits.contiguous().float()
        for exe, gen in ctx.runs:
            exe.consume(gen)
        for i, (exe, gen) in enumerate(ctx.runs):
            dev = dp.devices[i]
            d = dl[ctx.offs[i]:ctx.offs[i] + ctx.sizes[i]]
            with torch.cuda.device(dev):
                if dev != dev0:  # gather's backward: the replica's slice of dlogits
                    dd = dp._replica(i).io("dlogits", d.shape)
                    _order_after(dev, dev0)
                    _copy_peer(dd, d, torch.cuda.current_stream(dev))
                    d = dd
                exe.backward(d, 1.0, None)
        # C7 ReduceAddCoalesced onto device_ids[0]: one call over the flat gradient buffers
        flats = [model.flat] + [dp._replica(i).flat for i in range(1, len(ctx.runs))]
        for i in range(1, len(flats)):
            _order_after(dev0, dp.devices[i])
        dp.group.reduce_add([f.grads for f in flats])
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
    Replicas on distinct devices exchange through RCCL; device ids that are all equal (replicas
    sharing one GPU) are the single-GPU test form of the same path."""

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
        self.group = DPGroup(self.device_ids) if len(self.device_ids) > 1 else None

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
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        if x.device != self.devices[0]:
            raise NativeError(f"DataParallel input must be on device_ids[0] ({self.devices[0]}), not {x.device}")
        return _DPFn.apply(x, self.module._anchor, self)
