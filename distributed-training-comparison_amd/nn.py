"""ResNet-18 and CrossEntropyLoss modules backed by the native executor.

Mirror of the reference's operator boundary (src/ddp/net.py, trainer.py:40):

* ``ResNet18()`` builds the module tree with the SAME ``nn.Conv2d`` / ``nn.BatchNorm2d`` /
  ``nn.Linear`` constructors in the SAME order as net.py:86-105 and net.py:16-38, so a given
  ``torch.manual_seed`` yields bit-identical initial parameters and ``state_dict()`` keys
  (``layer2.0.shortcut.0.weight`` ...). Construction is ordinary PyTorch on the host.
* ``.to('cuda')`` moves those parameters into one flat fp32 device buffer laid out by the
  native executor (reverse registration order, KRSC conv filters exposed as strided
  [K,C,R,S] views) plus its bf16 shadow; gradients are views into a flat grad buffer.
* ``forward`` runs the whole network through ``dtc_rn18_forward`` and ``backward`` through
  ``dtc_rn18_backward`` (one autograd node). Nothing falls back to torch compute: the module
  refuses to run on the CPU.
"""
from __future__ import annotations

import ctypes as C
import threading
import weakref
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from ._native import NativeError, call, lib, ptr, require_cuda, stream_ptr


# ----------------------------------------------------------------------------- autocast state
# torch semantics: inside `autocast()` (trainer.py:153, the --amp path) the network computes in reduced
# precision (bf16 here, fp16 in the reference), outside it in fp32 (trainer.py:160-165 without --amp).
# amp.autocast flips this thread-local flag; ResNet.forward picks the executor precision from it
# unless the module's `precision` attribute forces one ("bf16" / "fp32").
_AUTOCAST = threading.local()


def is_autocast_enabled() -> bool:
    return bool(getattr(_AUTOCAST, "enabled", False))


def set_autocast_enabled(enabled: bool) -> None:
    _AUTOCAST.enabled = bool(enabled)


PRECISIONS = ("bf16", "fp32")


# ----------------------------------------------------------------------------- layout
@dataclass
class ParamInfo:
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]
    stride: Tuple[int, ...]


@dataclass
class BNInfo:
    prefix: str
    channels: int
    mean_offset: int
    var_offset: int


class Layout:
    """Batch-independent parameter / buffer / bucket layout reported by the executor."""

    def __init__(self, num_classes: int = 100, bucket_cap_mb: float = 25.0):
        h = C.c_void_p()
        call("dtc_rn18_create", C.byref(h), 1, 32, 32, num_classes, float(bucket_cap_mb))
        try:
            self.params: List[ParamInfo] = []
            for i in range(lib.dtc_rn18_num_params(h)):
                name = C.c_char_p()
                off, numel = C.c_int64(), C.c_int64()
                nd = C.c_int()
                shp = (C.c_int64 * 4)()
                strd = (C.c_int64 * 4)()
                call("dtc_rn18_param_info", h, i, C.byref(name), C.byref(off), C.byref(numel), C.byref(nd), shp, strd)
                self.params.append(ParamInfo(name.value.decode(), off.value, numel.value,
                                             tuple(shp[: nd.value]), tuple(strd[: nd.value])))
            self.bns: List[BNInfo] = []
            for i in range(lib.dtc_rn18_num_bn(h)):
                pre = C.c_char_p()
                ch = C.c_int()
                mo, vo = C.c_int64(), C.c_int64()
                call("dtc_rn18_bn_info", h, i, C.byref(pre), C.byref(ch), C.byref(mo), C.byref(vo))
                self.bns.append(BNInfo(pre.value.decode(), ch.value, mo.value, vo.value))
            self.flat_numel = lib.dtc_rn18_flat_numel(h)
            self.bufs_numel = lib.dtc_rn18_bufs_numel(h)
            self.buckets = []
            for i in range(lib.dtc_rn18_num_buckets(h)):
                o, n = C.c_int64(), C.c_int64()
                call("dtc_rn18_bucket_info", h, i, C.byref(o), C.byref(n))
                self.buckets.append((o.value, n.value))
        finally:
            lib.dtc_rn18_destroy(h)


class FlatState:
    """Device buffers shared by every executor of one model."""

    def __init__(self, layout: Layout, device: torch.device):
        self.layout = layout
        self.device = device
        self.params = torch.zeros(layout.flat_numel, dtype=torch.float32, device=device)
        self.grads = torch.zeros(layout.flat_numel, dtype=torch.float32, device=device)
        self.params_bf16 = torch.zeros(layout.flat_numel, dtype=torch.bfloat16, device=device)
        self.bufs = torch.zeros(layout.bufs_numel, dtype=torch.float32, device=device)
        self.nbt = torch.zeros(len(layout.bns), dtype=torch.int64, device=device)

    def refresh_bf16(self):
        ops.cast_f32_bf16(self.params, self.params_bf16)


class Executor:
    """One native executor (plan + workspace) for a fixed (batch, height, width)."""

    def __init__(self, flat: FlatState, batch: int, height: int, width: int, num_classes: int, bucket_cap_mb: float,
                 capture: bool = False, precision: str = "bf16"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}, not {precision!r}")
        self.handle = C.c_void_p()
        call("dtc_rn18_create", C.byref(self.handle), batch, height, width, num_classes, float(bucket_cap_mb))
        self.precision = precision
        if precision == "fp32":
            call("dtc_rn18_set_precision", self.handle, 1)
        if capture:
            call("dtc_rn18_enable_capture", self.handle)
        nbytes = lib.dtc_rn18_workspace_bytes(self.handle)
        # 256-byte aligned workspace (the caching allocator returns 512-byte aligned blocks)
        self.workspace = torch.empty(nbytes + 256, dtype=torch.uint8, device=flat.device)
        base = self.workspace.data_ptr()
        self.ws_ptr = (base + 255) // 256 * 256
        self.flat = flat
        self.batch, self.height, self.width, self.num_classes = batch, height, width, num_classes
        self.generation = 0
        self._bwd_gen = 0  # generation whose forward a backward has consumed (one backward per forward)
        self._dlogits = None
        call("dtc_rn18_bind", self.handle, self.ws_ptr, ptr(flat.params), ptr(flat.grads), ptr(flat.params_bf16),
             ptr(flat.bufs), ptr(flat.nbt), stream_ptr())

    def forward(self, x: torch.Tensor, logits: torch.Tensor, train: bool) -> int:
        call("dtc_rn18_forward", self.handle, ptr(x), ptr(logits), int(bool(train)), stream_ptr())
        self.generation += 1
        return self.generation

    def consume(self, gen: int) -> None:
        """Claim the forward of generation `gen` for one backward. The kernels WRITE gradients, which
        equals the reference's zero_grad() + backward(); a second backward over the same forward
        (retain_graph=True) would have to ACCUMULATE into .grad in torch, so it is refused instead of
        silently returning the first backward's gradients."""
        if gen != self.generation:
            raise NativeError("ResNet backward: the executor ran another forward since this graph was built "
                              "(one forward per backward is supported)")
        if gen == self._bwd_gen:
            raise NativeError("ResNet backward: this forward was already back-propagated (a second backward "
                              "would accumulate gradients in torch; the native kernels write them): run "
                              "the forward again")
        self._bwd_gen = gen

    def backward(self, dlogits: torch.Tensor, grad_scale: float, comm) -> None:
        call("dtc_rn18_backward", self.handle, ptr(dlogits), float(grad_scale), comm.handle if comm else None,
             stream_ptr())

    def xent_backward(self, logits, labels, lse, gscale, grad_scale: float, comm) -> None:
        """CrossEntropy backward into the executor's dlogits buffer + the network backward, one call.
        Runs right after the per-step barrier, when the GPU is idle until it returns: the current
        stream is read with torch's raw-stream call (torch.cuda.current_stream() builds a Stream object
        through several Python device lookups)."""
        call("dtc_rn18_xent_backward", self.handle, logits.data_ptr(), labels.data_ptr(), lse.data_ptr(),
             None if gscale is None else gscale.data_ptr(), float(grad_scale), comm.handle if comm else None,
             _raw_stream(logits.device.index))

    def dlogits_buffer(self) -> torch.Tensor:
        """fp32 [batch, num_classes] view of the executor's own dlogits buffer: a loss gradient
        written here is consumed by backward() without the copy-in."""
        if self._dlogits is None:
            off = C.c_size_t()
            call("dtc_rn18_dlogits_buffer", self.handle, C.byref(off))
            start = self.ws_ptr - self.workspace.data_ptr() + off.value
            nbytes = self.batch * self.num_classes * 4
            self._dlogits = self.workspace[start:start + nbytes].view(torch.float32).view(self.batch,
                                                                                         self.num_classes)
        return self._dlogits

    def activations(self, captures: bool = False) -> Dict[str, torch.Tensor]:
        """Views of the per-layer activations the last forward left in the workspace (NHWC); with
        captures=True the backward intermediates recorded by a capture-enabled executor."""
        base = self.ws_ptr - self.workspace.data_ptr()
        out = {}
        count = lib.dtc_rn18_num_captures if captures else lib.dtc_rn18_num_activations
        info = "dtc_rn18_capture_info" if captures else "dtc_rn18_activation_info"
        for i in range(count(self.handle)):
            name = C.c_char_p()
            off = C.c_size_t()
            shp = (C.c_int * 4)()
            call(info, self.handle, i, C.byref(name), C.byref(off), shp)
            nm = name.value.decode()
            dt = torch.float32 if (nm.endswith("_f32") or self.precision == "fp32") else torch.bfloat16
            numel = shp[0] * shp[1] * shp[2] * shp[3]
            nbytes = numel * (4 if dt == torch.float32 else 2)
            o = base + off.value
            out[nm] = self.workspace[o:o + nbytes].view(dt).view(shp[0], shp[1], shp[2], shp[3])
        return out

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            lib.dtc_rn18_destroy(h)
            self.handle = None


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream(index) -> int:
    """Current HIP stream of device `index` (same value as stream_ptr() on that device)."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(index if index is not None else torch.cuda.current_device())
    return stream_ptr()


# ----------------------------------------------------------------------------- autograd nodes
class _NetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, model, exe):
        logits = torch.empty(x.shape[0], model.num_classes, dtype=torch.float32, device=x.device)
        ctx.gen = exe.forward(x, logits, model.training)
        ctx.model, ctx.exe = model, exe
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        model, exe = ctx.model, ctx.exe
        if model._pre_backward is not None:
            model._pre_backward()
        exe.consume(ctx.gen)
        exe.backward(dlogits.contiguous().float(), model._grad_scale, model._comm)
        model._ensure_grads()
        return None, None, None, None


class _HostWords:
    """A ring of pinned host words the loss launch writes its value into (the item() read). The ring is
    owned here, not by torch's pinned-memory cache: a word a kernel may still write is never handed to
    another tensor. Reusing a slot first waits for the event of the step that last wrote it, and bumps
    the slot's generation: a loss that still holds the slot's earlier generation (kept past N newer
    losses) sees the mismatch in item() and reads its own device value instead."""

    N = 256

    def __init__(self):
        self.buf = torch.empty(self.N, dtype=torch.float32, pin_memory=True)
        self.events = [None] * self.N
        self.gens = [0] * self.N
        self.i = 0
        self.mu = threading.Lock()  # rank threads of the thread-group communicator share the ring

    def take(self):
        with self.mu:
            k = self.i % self.N
            self.i += 1
            ev = self.events[k]
            self.events[k] = None
            self.gens[k] += 1
            gen = self.gens[k]
        if ev is not None:
            ev.synchronize()
        return k, self.buf[k], gen

    def owns(self, k, gen):
        """True while slot k still holds the value of the loss that took it as generation `gen`."""
        return self.gens[k] == gen

    def done(self, k, ev):
        self.events[k] = ev


_HOST_WORDS: List[Optional[_HostWords]] = [None]


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        loss, lse = ops.xent_fwd(logits, labels)
        ctx.save_for_backward(logits, labels, lse)
        ctx.lse = lse
        return loss

    @staticmethod
    def backward(ctx, gloss):
        logits, labels, lse = ctx.saved_tensors
        g = gloss.reshape(1).float().contiguous()
        return ops.xent_bwd(logits, labels, lse, g), None


class NativeLoss(torch.Tensor):
    """Scalar loss of ``CrossEntropyLoss`` applied directly to the native ResNet's logits (and its
    ``GradScaler.scale`` product). Its ``backward()`` runs the known chain
    xent-backward -> network backward as two native calls, without the autograd engine's thread
    hand-off and the per-node Python/elementwise launches in between (this runs right after the
    reference's per-step ``dist.barrier()``, when the GPU queue is empty, so every host
    microsecond there is GPU idle time). Gradients are identical to the autograd path, which is
    still taken for any other use (explicit ``gradient``, ``create_graph``, ``inputs``), and any
    arithmetic on the loss returns a plain autograd tensor."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    @property
    def _dtc_graph(self):
        """The autograd form of this loss (built on first use: the fast path never needs it)."""
        g = self.__dict__.get("_dtc_graph_t")
        if g is None:
            g = self._dtc_graph_fn()
            self.__dict__["_dtc_graph_t"] = g
        return g

    def backward(self, gradient=None, retain_graph=None, create_graph=False, inputs=None):
        fast = self._dtc_fast
        if fast is None or gradient is not None or create_graph or inputs is not None or not _FAST_BACKWARD[0]:
            return self._dtc_graph.backward(gradient, retain_graph, create_graph, inputs)
        node, logits, labels, lse, gscale = fast
        if isinstance(node, _NetFn._backward_cls):
            model, exe = node.model, node.exe
            if model._pre_backward is not None:
                model._pre_backward()
            exe.consume(node.gen)
            exe.xent_backward(logits, labels, lse, gscale, model._grad_scale, model._comm)
            model._ensure_grads()
        else:  # DataParallel's gathered logits: xent backward, then the replicas' backward + reduce-add
            from .parallel import _DPFn

            _DPFn.backward(node, ops.xent_bwd(logits, labels, lse, gscale))
        if not retain_graph:
            self._dtc_fast = None
        return None

    def item(self):
        """The loss value from the pinned host copy enqueued right after the loss kernel: waits
        for the loss, not for the whole stream (a plain ``Tensor.item()`` also waits for the
        backward and optimizer step issued since). Same value either way."""
        hc = getattr(self, "_dtc_host", None)
        if hc is None:
            return super().item()
        h, ev, ring = hc[0], hc[1], hc[2:]
        if ring and not ring[0].owns(ring[1], ring[2]):  # the slot went to a newer loss: own device value
            self._dtc_host = None
            return super().item()
        ev.synchronize()
        return h.item()

    def __float__(self):
        return float(self.item())


_FAST_BACKWARD = [True]  # tests flip this to compare against the autograd-engine path


def _wrap_loss(value: torch.Tensor, graph_fn, fast, host_copy: bool = False) -> torch.Tensor:
    """NativeLoss holding `value` (no autograd history of its own); graph_fn() builds the autograd
    form on demand (the fallback backward path)."""
    out = torch.Tensor._make_subclass(NativeLoss, value.detach(), False)
    out._dtc_graph_fn = graph_fn
    out._dtc_fast = fast
    if host_copy:
        h = torch.empty((), dtype=value.dtype, pin_memory=True)
        h.copy_(value.detach(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        out._dtc_host = (h, ev)
    return out


# The GradScaler most recently initialised (amp.GradScaler._lazy_init): the loss kernel's call also
# enqueues loss * scale for it, while the GPU is still busy with the forward, so the scaler.scale(loss)
# after the per-step barrier -- when the GPU queue is empty -- needs no launch of its own.
_PRESCALER = [None]


def _prescaler():
    """The live GradScaler whose scale the loss kernel's call pre-multiplies, or None."""
    ref = _PRESCALER[0]
    sc = ref() if ref is not None else None
    if sc is None or sc._scale is None or not sc._enabled:
        return None
    return sc


def prescale(loss: "NativeLoss", scaled: Optional[torch.Tensor] = None, sc=None) -> None:
    """Enqueue loss * scale AND build its NativeLoss wrapper now, while the GPU is busy with the
    forward: scaler.scale(loss) after the per-step barrier then only looks it up (the wrapper's
    Tensor._make_subclass and closures cost 10-30 us of host time, all of it GPU idle time there).
    `scaled`: the product already computed by the loss launch (dtc_xent_fwd_ex) for scaler `sc`."""
    sc = sc if scaled is not None else _prescaler()
    if sc is None:
        return
    scale = sc._scale
    f = loss._dtc_fast
    wrapped = _wrap_loss(scaled if scaled is not None else ops.amp_scale(loss.detach(), scale),
                         lambda: loss._dtc_graph * scale, None if f is None else (f[0], f[1], f[2], f[3], scale))
    loss._dtc_prescaled = (wrapped, scale, sc._version)


def scaled_loss(loss: torch.Tensor, scale: torch.Tensor, version: int = -1) -> torch.Tensor:
    """loss * scale (GradScaler.scale); keeps the direct backward chain of a NativeLoss. `version` is
    the scaler's state version: a product enqueued with the loss for this very scale tensor and state
    is reused (same value: the scale only changes in update(), which bumps the version)."""
    if isinstance(loss, NativeLoss):
        f = loss._dtc_fast
        pre = loss.__dict__.get("_dtc_prescaled")
        if pre is not None and pre[1] is scale and pre[2] == version and pre[0]._dtc_fast is not None:
            # the wrapper built by prescale() (same value, same backward chain) until a backward has
            # consumed its direct chain; after that a fresh wrapper is built below
            return pre[0]
        # the value on the native kernel (GradScaler K9: no torch elementwise launch in the step)
        return _wrap_loss(ops.amp_scale(loss.detach(), scale), lambda: loss._dtc_graph * scale,
                          None if f is None else (f[0], f[1], f[2], f[3], scale))
    return loss * scale


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss() with mean reduction (reference trainer.py:40) on the native kernel."""

    def forward(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        require_cuda(logits, labels)
        if logits.dtype != torch.float32:
            logits = logits.float()
        logits = logits.contiguous()
        labels = labels.long().contiguous()
        node = logits.grad_fn
        if torch.is_grad_enabled() and node is not None:
            from .parallel import _DPFn

            if isinstance(node, (_NetFn._backward_cls, _DPFn._backward_cls)):
                if logits.shape[0] <= 4096:
                    # loss + lse + scaled loss + host copy: one launch, called directly (no autograd node:
                    # the direct backward chain below needs none; the autograd form of the loss -- the
                    # same kernel's value -- is built only if a fallback backward asks for it)
                    sc = _prescaler()
                    if _HOST_WORDS[0] is None:
                        _HOST_WORDS[0] = _HostWords()
                    ring = _HOST_WORDS[0]
                    slot, host, gen = ring.take()
                    n, ncls = logits.shape
                    dev = logits.device
                    loss = torch.empty((), dtype=torch.float32, device=dev)
                    lse = torch.empty(n, dtype=torch.float32, device=dev)
                    scaled = torch.empty((), dtype=torch.float32, device=dev) if sc is not None else None
                    call("dtc_xent_fwd_ex", logits.data_ptr(), labels.data_ptr(), n, ncls, loss.data_ptr(),
                         lse.data_ptr(), None if sc is None else sc._scale.data_ptr(),
                         None if scaled is None else scaled.data_ptr(), host.data_ptr(), _raw_stream(dev.index))
                    ev = torch.cuda.Event()
                    ev.record()
                    ring.done(slot, ev)
                    out = _wrap_loss(loss, lambda: _XentFn.apply(logits, labels), (node, logits, labels, lse, None))
                    out._dtc_host = (host, ev, ring, slot, gen)
                    if sc is not None:
                        prescale(out, scaled, sc)
                    return out
                loss = _XentFn.apply(logits, labels)
                out = _wrap_loss(loss, lambda: loss, (node, logits, labels, loss.grad_fn.lse, None), host_copy=True)
                prescale(out)
                return out
        return _XentFn.apply(logits, labels)


# ----------------------------------------------------------------------------- modules
class BasicBlock(nn.Module):
    """Parameter container with reference net.py:13-38's construction order and names."""

    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes),
            )

    def forward(self, x):  # pragma: no cover - the network runs as a whole in ResNet.forward
        raise NativeError("BasicBlock runs inside the native ResNet executor; call the ResNet module")


class ResNet(nn.Module):
    """CIFAR ResNet (net.py:86-116) whose forward/backward run on the MI355X executor."""

    def __init__(self, block=BasicBlock, num_blocks=(2, 2, 2, 2), num_classes=100, bucket_cap_mb: float = 25.0):
        super().__init__()
        if block is not BasicBlock or tuple(num_blocks) != (2, 2, 2, 2):
            raise NotImplementedError("only ResNet18 (BasicBlock, [2,2,2,2]) is built natively (reference main.py:26)")
        self.in_planes = 64
        self.num_classes = num_classes
        self.conv1 = nn.Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], stride=1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], stride=2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], stride=2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], stride=2)
        self.linear = nn.Linear(512 * block.expansion, num_classes)
        self._flat: Optional[FlatState] = None
        self._layout: Optional[Layout] = None
        self._executors: Dict[Tuple[int, int, int], Executor] = {}
        self._anchor: Optional[torch.Tensor] = None
        self._comm = None
        self._grad_scale = 1.0
        self._pre_backward = None  # set by DistributedDataParallel: runs before every native backward
        self._bucket_cap_mb = float(bucket_cap_mb)
        self._capture = False
        self._sync_bn = False  # SyncBatchNorm.convert_sync_batchnorm marks the module
        self._sync_comm = None  # communicator the executors all-reduce BN sums over
        # None: follow autocast (bf16 inside, fp32 outside, as torch); "bf16" / "fp32": force
        self.precision: Optional[str] = None

    def _make_layer(self, block, planes, num_blocks, stride):
        strides = [stride] + [1] * (num_blocks - 1)
        layers = []
        for s in strides:
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    # ------------------------------------------------------------------ device placement
    def _apply(self, fn, recurse=True):
        if self._flat is not None:
            return self  # parameters are pinned in the flat device buffers
        out = super()._apply(fn, recurse)
        dev = self.conv1.weight.device
        if dev.type == "cuda":
            self._materialize(dev)
        return out

    def _resolve(self, dotted: str):
        parts = dotted.split(".")
        mod = self
        for p in parts[:-1]:
            mod = getattr(mod, p)
        return mod, parts[-1]

    def _materialize(self, device: torch.device):
        layout = Layout(self.num_classes, self._bucket_cap_mb)
        names = [n for n, _ in self.named_parameters()]
        if names != [p.name for p in layout.params]:
            raise NativeError("module parameters do not match the executor layout")
        flat = FlatState(layout, device)
        with torch.no_grad():
            for info in layout.params:
                mod, attr = self._resolve(info.name)
                old = getattr(mod, attr)
                view = torch.as_strided(flat.params, info.shape, info.stride, info.offset)
                view.copy_(old.detach().to(device))
                newp = nn.Parameter(view, requires_grad=old.requires_grad)
                newp._dtc_model = weakref.ref(self)
                mod._parameters[attr] = newp
            for i, bn in enumerate(layout.bns):
                mod, _ = self._resolve(bn.prefix + ".x")
                rm = flat.bufs.narrow(0, bn.mean_offset, bn.channels)
                rv = flat.bufs.narrow(0, bn.var_offset, bn.channels)
                rm.copy_(mod.running_mean.to(device))
                rv.copy_(mod.running_var.to(device))
                flat.nbt[i].copy_(mod.num_batches_tracked.to(device))
                mod._buffers["running_mean"] = rm
                mod._buffers["running_var"] = rv
                mod._buffers["num_batches_tracked"] = flat.nbt[i]
        self._layout = layout
        self._flat = flat
        self._anchor = torch.zeros(1, device=device, requires_grad=True)
        self._attach_grads()
        flat.refresh_bf16()

    def _attach_grads(self):
        for info in self._layout.params:
            mod, attr = self._resolve(info.name)
            mod._parameters[attr].grad = torch.as_strided(self._flat.grads, info.shape, info.stride, info.offset)

    def _ensure_grads(self):
        if self.linear.bias.grad is None or self.conv1.weight.grad is None:
            self._attach_grads()

    @property
    def flat(self) -> FlatState:
        if self._flat is None:
            raise NativeError("ResNet must be moved to a GPU (`.to('cuda')`) before use")
        return self._flat

    def sync_weights(self):
        """Re-derive the bf16 shadow after parameters were modified outside the native SGD."""
        self.flat.refresh_bf16()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        if assign:
            raise NotImplementedError("assign=True would detach parameters from the flat buffer")
        res = super().load_state_dict(state_dict, strict=strict)
        if self._flat is not None:
            self._flat.refresh_bf16()
        return res

    def buckets(self):
        """Gradient buckets [(flat offset, numel)] in the order backward completes them."""
        return Layout(self.num_classes, self._bucket_cap_mb).buckets

    def set_bucket_cap_mb(self, mb: float):
        self._bucket_cap_mb = float(mb)
        self._executors.clear()

    def compute_precision(self) -> str:
        """The precision the next forward runs in: `self.precision` when set ("bf16" / "fp32"),
        else torch's rule -- bf16 inside `autocast()`, fp32 outside (trainer.py:152-165)."""
        if self.precision is not None:
            if self.precision not in PRECISIONS:
                raise ValueError(f"precision must be None or one of {PRECISIONS}, not {self.precision!r}")
            return self.precision
        return "bf16" if is_autocast_enabled() else "fp32"

    def executor(self, batch: int, height: int, width: int, precision: Optional[str] = None) -> Executor:
        precision = precision or self.compute_precision()
        key = (batch, height, width, precision)
        exe = self._executors.get(key)
        if exe is None:
            exe = Executor(self.flat, batch, height, width, self.num_classes, self._bucket_cap_mb,
                           capture=self._capture, precision=precision)
            if self._sync_comm is not None:
                call("dtc_rn18_set_sync_bn", exe.handle, self._sync_comm.handle)
            self._executors[key] = exe
        return exe

    def set_sync_bn(self, comm) -> None:
        """Synchronise training-mode BN statistics over `comm` (a parallel.Comm of its own, not the
        Reducer's); None restores per-rank statistics. Applies to existing and new executors."""
        self._sync_comm = comm
        for exe in self._executors.values():
            call("dtc_rn18_set_sync_bn", exe.handle, comm.handle if comm is not None else None)

    def enable_capture(self, on: bool = True):
        """Keep backward intermediates for per-layer parity tests (new executors only)."""
        self._capture = on
        self._executors.clear()

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        flat = self.flat
        require_cuda(x)
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [N,3,H,W] input, got {tuple(x.shape)}")
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        exe = self.executor(x.shape[0], x.shape[2], x.shape[3])
        return _NetFn.apply(x, self._anchor, self, exe)


class SyncBatchNorm:
    """``nn.SyncBatchNorm.convert_sync_batchnorm`` for the native ResNet (README.md:40 recommends
    it; the reference trainers do not call it). The BN modules stay where they are (same
    state_dict keys); the model is marked, and ``DistributedDataParallel`` gives it a second RCCL
    communicator over which every training-mode BN all-reduces its per-channel sums
    (include/dtc.h ``dtc_rn18_set_sync_bn``). As in torch, a one-rank group keeps local statistics."""

    @staticmethod
    def convert_sync_batchnorm(module, process_group=None):
        if not isinstance(module, ResNet):
            raise NotImplementedError("convert_sync_batchnorm: only the native ResNet18 is supported")
        module._sync_bn = True
        module._sync_bn_group = process_group
        return module


def ResNet18(num_classes: int = 100) -> ResNet:
    """net.py:119-120."""
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes)
