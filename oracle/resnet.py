"""CPU oracle for the whole ResNet-18 training step — TEST INFRASTRUCTURE ONLY (see oracle/ops.py).

Restates reference src/ddp/net.py:40-45 (BasicBlock.forward) and net.py:107-116 (ResNet.forward)
with their backward, nn.CrossEntropyLoss (trainer.py:40,155) and optim.SGD Nesterov
(trainer.py:92-98), in numpy, NHWC.

``bf16_mode=True`` rounds to bfloat16 at the points where torch autocast keeps bf16 tensors
(conv/linear inputs and outputs, BatchNorm and ReLU outputs, the residual sum, activation
gradients) — the same points where the native executor rounds — so kernel-vs-oracle differences
reduce to summation order. ``bf16_mode=False`` is plain fp32 (the reference without --amp).

Parameters are taken and returned in torch layout (state_dict names; conv weights [K,C,R,S]).
"""
from __future__ import annotations

import numpy as np

from . import ops as O


def _blocks(params):
    out = []
    for L in range(1, 5):
        for b in range(2):
            pre = f"layer{L}.{b}"
            stride = 2 if (L > 1 and b == 0) else 1
            proj = f"{pre}.shortcut.0.weight" in params
            out.append((pre, stride, proj))
    return out


class _Rounder:
    def __init__(self, on):
        self.on = on

    def __call__(self, a):
        return O.bf16(a) if self.on else np.asarray(a, np.float32)


def _bn_forward(x, gamma, beta, R, relu, residual=None, eps=1e-5):
    """Training-mode BN over NHWC x (float32 values). Returns (y, mean, invstd, pre-relu rounded z)."""
    C = x.shape[-1]
    x2 = x.reshape(-1, C).astype(np.float64)
    mean = x2.mean(0)
    var = np.maximum((x2 * x2).mean(0) - mean * mean, 0.0)
    invstd = 1.0 / np.sqrt(var + eps)
    z = (x2 - mean) * (invstd * gamma) + beta
    z = R(z.reshape(x.shape))
    return z, mean, invstd, var


def forward_backward(params, buffers, x_nchw, labels, bf16_mode=True, train=True, want_acts=False, momentum=0.1,
                     dt=np.float64):
    """One forward (+ backward when train) of ResNet-18.

    params  : dict name -> np.ndarray (torch layout), float32
    buffers : dict with '<bn>.running_mean' / '<bn>.running_var' (updated copies are returned)
    Returns dict(loss, logits, grads, acts, buffers).
    """
    R = _Rounder(bf16_mode)
    P = params
    Wk = {k: R(O.kcrs_to_krsc(v)) for k, v in P.items() if v.ndim == 4}
    acts = {}
    newbuf = dict(buffers)
    bn_cache = {}

    def bn(name, x, relu, res=None):
        g, b = P[name + ".weight"].astype(np.float64), P[name + ".bias"].astype(np.float64)
        if train:
            z, mean, invstd, var = _bn_forward(x, g, b, R, relu)
            n = x.size // x.shape[-1]
            rm, rv = buffers[name + ".running_mean"], buffers[name + ".running_var"]
            newbuf[name + ".running_mean"] = ((1 - momentum) * rm + momentum * mean).astype(np.float32)
            newbuf[name + ".running_var"] = ((1 - momentum) * rv + momentum * var * n / max(n - 1, 1)).astype(np.float32)
        else:
            mean = buffers[name + ".running_mean"].astype(np.float64)
            invstd = 1.0 / np.sqrt(buffers[name + ".running_var"].astype(np.float64) + 1e-5)
            z = R((x.reshape(-1, x.shape[-1]) - mean) * (invstd * g) + b).reshape(x.shape)
        bn_cache[name] = (mean, invstd, g)
        return z

    def conv(x, wname, stride, pad):
        return R(O.conv2d_fwd(x, Wk[wname], stride, pad))

    # ------------------------------------------------------------------ forward
    x = R(O.nchw_to_nhwc(np.asarray(x_nchw, np.float32)))
    c0 = conv(x, "conv1.weight", 1, 1)
    a0 = R(O.relu(bn("bn1", c0, True)))
    acts.update({"stem.conv": c0, "stem.out": a0})
    cache = []
    h = a0
    for pre, stride, proj in _blocks(P):
        inp = h
        c1 = conv(inp, pre + ".conv1.weight", stride, 1)
        a1 = R(O.relu(bn(pre + ".bn1", c1, True)))
        c2 = conv(a1, pre + ".conv2.weight", 1, 1)
        z2 = bn(pre + ".bn2", c2, False)
        if proj:
            s = conv(inp, pre + ".shortcut.0.weight", stride, 0)
            zs = bn(pre + ".shortcut.1", s, False)
            out = R(O.relu(z2 + zs))
        else:
            s = None
            out = R(O.relu(z2 + inp))
        acts.update({pre + ".conv1": c1, pre + ".relu1": a1, pre + ".conv2": c2, pre + ".out": out})
        if proj:
            acts[pre + ".shortcut"] = s
        cache.append((pre, stride, proj, inp, c1, a1, c2, s, out))
        h = out
    wfc, bfc = P["linear.weight"], P["linear.bias"]
    feat, logits = O.head_fwd(h, wfc, bfc, bf16_mode=bf16_mode)
    acts["head.feat_f32"] = feat.astype(np.float32)
    loss, dlogits, _ = O.cross_entropy(logits, np.asarray(labels))
    result = {"loss": float(loss), "logits": logits.astype(np.float32), "acts": acts if want_acts else None,
              "buffers": newbuf, "grads": None, "dlogits": dlogits}
    if not train:
        return result

    # ------------------------------------------------------------------ backward
    grads = {}

    def bn_bwd(name, dz, x):
        mean, invstd, g = bn_cache[name]
        C = x.shape[-1]
        dx, dg, db = O.bn_train_bwd(dz.reshape(-1, C), x.reshape(-1, C), g, mean, invstd)
        grads[name + ".weight"] = dg.astype(np.float32)
        grads[name + ".bias"] = db.astype(np.float32)
        return R(dx.reshape(x.shape))

    def wgrad(x, dy, wname, stride, pad):
        K, C, r, s_ = P[wname].shape
        grads[wname] = O.krsc_to_kcrs(O.conv2d_wgrad(x, dy, r, s_, stride, pad)).astype(np.float32)

    wfc_used = O.bf16(wfc) if bf16_mode else wfc
    dwfc, dbfc, dact = O.head_bwd(dlogits, feat, wfc_used, h.shape[1:3])
    grads["linear.weight"] = dwfc.astype(np.float32)
    grads["linear.bias"] = dbfc.astype(np.float32)
    dh = R(dact)
    for pre, stride, proj, inp, c1, a1, c2, s, out in reversed(cache):
        dz = np.where(out > 0, dh, 0).astype(np.float32)
        dc2 = bn_bwd(pre + ".bn2", dz, c2)
        ds = bn_bwd(pre + ".shortcut.1", dz, s) if proj else None
        wgrad(a1, dc2, pre + ".conv2.weight", 1, 1)
        da1 = R(O.conv2d_dgrad(dc2, Wk[pre + ".conv2.weight"], a1.shape[1:3], 1, 1))
        dz1 = np.where(a1 > 0, da1, 0).astype(np.float32)
        dc1 = bn_bwd(pre + ".bn1", dz1, c1)
        wgrad(inp, dc1, pre + ".conv1.weight", stride, 1)
        dx = O.conv2d_dgrad(dc1, Wk[pre + ".conv1.weight"], inp.shape[1:3], stride, 1)
        if proj:
            wgrad(inp, ds, pre + ".shortcut.0.weight", stride, 0)
            dxs = R(O.conv2d_dgrad(ds, Wk[pre + ".shortcut.0.weight"], inp.shape[1:3], stride, 0))
            dh = R(dx + dxs)
        else:
            dh = R(dx + dz)
    dz0 = np.where(a0 > 0, dh, 0).astype(np.float32)
    dc0 = bn_bwd("bn1", dz0, c0)
    wgrad(x, dc0, "conv1.weight", 1, 1)
    result["grads"] = grads
    return result


# ----------------------------------------------------------------------------- training
def init_state(params, buffers=None):
    p = {k: np.asarray(v, np.float32).copy() for k, v in params.items()
         if not (k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"))}
    if buffers is None:
        buffers = {k: np.asarray(v, np.float32).copy() for k, v in params.items()
                   if k.endswith("running_mean") or k.endswith("running_var")}
    return {"p": p, "buf": buffers, "mom": {}, "step": 0}


def train_step(state, x, labels, lr=0.1, wd=1e-4, mu=0.9, bf16_mode=False):
    """Forward, backward and one Nesterov SGD step (reference single/trainer.py:131-147 semantics)."""
    r = forward_backward(state["p"], state["buf"], x, labels, bf16_mode=bf16_mode, train=True)
    first = state["step"] == 0
    for k, g in r["grads"].items():
        p, buf = O.sgd_nesterov(state["p"][k], g, state["mom"].get(k), lr, wd, mu, first)
        state["p"][k] = p
        state["mom"][k] = buf
    state["buf"] = r["buffers"]
    state["step"] += 1
    return r["loss"]
