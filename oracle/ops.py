"""CPU oracle (numpy) for the ResNet-18 / CIFAR-100 training step — TEST INFRASTRUCTURE ONLY.

This restates, from scratch, the arithmetic that the reference's PyTorch calls perform
(reference = youngerous/distributed-training-comparison; the math itself lives in third-party
torch==1.7.1 kernels, requirements.txt:3-4, absent here). Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import it, and only as a checker or a timed baseline; the
product path never routes through it.

Pinning: tests/test_oracle_golden.py checks these functions against golden vectors produced by
running the reference's own modules (src/*/net.py, utils.py, dataset.py) with torch CPU in the
build container (tests/golden/make_golden.py). AMP semantics: the reference autocasts to fp16 on
CUDA; this build runs bf16, so the "bf16" variants below mirror torch CPU bf16 autocast (convs,
linear and their outputs in bf16, BatchNorm/loss in fp32) — the same points where the native
kernels round.

Layouts: activations NHWC, conv filters KRSC (as the native library); helpers convert.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------- numerics helpers


def bf16(a) -> np.ndarray:
    """Round float32 values to the nearest bfloat16 (round-to-nearest-even), returned as float32."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32)
    return np.where(np.isnan(a), a, out).astype(np.float32)


def bf16_bits(a) -> np.ndarray:
    """uint16 bit patterns of bf16(a)."""
    return (bf16(a).view(np.uint32) >> 16).astype(np.uint16)


def from_bf16_bits(b) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def nchw_to_nhwc(x):
    return np.ascontiguousarray(np.transpose(x, (0, 2, 3, 1)))


def nhwc_to_nchw(x):
    return np.ascontiguousarray(np.transpose(x, (0, 3, 1, 2)))


def kcrs_to_krsc(w):
    return np.ascontiguousarray(np.transpose(w, (0, 2, 3, 1)))


def krsc_to_kcrs(w):
    return np.ascontiguousarray(np.transpose(w, (0, 3, 1, 2)))


# ----------------------------------------------------------------------------- convolution
# nn.Conv2d(in, out, k, stride, padding, bias=False): reference src/ddp/net.py:18-24, 29-35, 91


def _im2col(x, R, S, stride, pad):
    """x [N,H,W,C] -> cols [N,P,Q,R,S,C] (float64)."""
    N, H, W, C = x.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    xp = np.zeros((N, H + 2 * pad, W + 2 * pad, C), dtype=np.float64)
    xp[:, pad:pad + H, pad:pad + W, :] = x
    cols = np.empty((N, P, Q, R, S, C), dtype=np.float64)
    for r in range(R):
        for s in range(S):
            cols[:, :, :, r, s, :] = xp[:, r:r + stride * P:stride, s:s + stride * Q:stride, :]
    return cols


def conv2d_fwd(x, w, stride, pad):
    """y[n,p,q,k] = sum_{r,s,c} x[n, p*st-pad+r, q*st-pad+s, c] * w[k,r,s,c]  (NHWC, KRSC)."""
    K, R, S, C = w.shape
    cols = _im2col(x, R, S, stride, pad)
    N, P, Q = cols.shape[:3]
    y = cols.reshape(N * P * Q, R * S * C) @ np.asarray(w, np.float64).reshape(K, R * S * C).T
    return y.reshape(N, P, Q, K)


def conv2d_dgrad(dy, w, in_hw, stride, pad):
    """Input gradient of conv2d_fwd: dx[n,h,w,c] = sum dy[n,p,q,k] w[k,r,s,c] over h = p*st-pad+r."""
    N, P, Q, K = dy.shape
    _, R, S, C = w.shape
    H, W = in_hw
    dcols = np.asarray(dy, np.float64).reshape(N * P * Q, K) @ np.asarray(w, np.float64).reshape(K, R * S * C)
    dcols = dcols.reshape(N, P, Q, R, S, C)
    dxp = np.zeros((N, H + 2 * pad + stride, W + 2 * pad + stride, C), dtype=np.float64)
    for r in range(R):
        for s in range(S):
            dxp[:, r:r + stride * P:stride, s:s + stride * Q:stride, :] += dcols[:, :, :, r, s, :]
    return dxp[:, pad:pad + H, pad:pad + W, :]


def conv2d_wgrad(x, dy, R, S, stride, pad):
    """Weight gradient: dw[k,r,s,c] = sum_{n,p,q} dy[n,p,q,k] x[n, p*st-pad+r, q*st-pad+s, c]."""
    cols = _im2col(x, R, S, stride, pad)
    N, P, Q = cols.shape[:3]
    K = dy.shape[3]
    C = x.shape[3]
    dw = np.asarray(dy, np.float64).reshape(N * P * Q, K).T @ cols.reshape(N * P * Q, R * S * C)
    return dw.reshape(K, R, S, C)


# ----------------------------------------------------------------------------- batch norm (train)
# nn.BatchNorm2d(planes), training mode: reference net.py:21,25,37,92; eps 1e-5, momentum 0.1


def bn_train_fwd(x, gamma, beta, running_mean=None, running_var=None, eps=1e-5, momentum=0.1):
    """x [M, C] (pixels x channels). Returns y, mean, invstd, new running_mean, new running_var."""
    x = np.asarray(x, np.float64)
    n = x.shape[0]
    mean = x.mean(axis=0)
    var = ((x - mean) ** 2).mean(axis=0)
    invstd = 1.0 / np.sqrt(var + eps)
    y = (x - mean) * invstd * gamma + beta
    rm = rv = None
    if running_mean is not None:
        rm = (1 - momentum) * running_mean + momentum * mean
        rv = (1 - momentum) * running_var + momentum * var * n / max(n - 1, 1)
    return y, mean, invstd, rm, rv


def bn_train_bwd(dy, x, gamma, mean, invstd):
    """Gradients of bn_train_fwd w.r.t. x, gamma, beta (batch statistics are functions of x)."""
    dy = np.asarray(dy, np.float64)
    x = np.asarray(x, np.float64)
    n = x.shape[0]
    xhat = (x - mean) * invstd
    dbeta = dy.sum(axis=0)
    dgamma = (dy * xhat).sum(axis=0)
    dx = gamma * invstd * (dy - dbeta / n - xhat * dgamma / n)
    return dx, dgamma, dbeta


# ----------------------------------------------------------------------------- SyncBatchNorm (train)
# nn.SyncBatchNorm (torch/nn/modules/_functions.py SyncBatchNorm.forward/backward in torch 1.7.1, the
# conversion README.md:40 recommends): statistics over the union of every rank's batch. Restated as
# the executor computes it (dtc_rn18_set_sync_bn): per-channel (sum, sumsq) SUM all-reduced, global
# count; backward (sum dy, sum dy*xhat) SUM all-reduced; dgamma/dbeta are this rank's own sums.
# `allreduce(a)` returns the elementwise sum of `a` over ranks (np.ndarray in, np.ndarray out).


def sync_bn_train_fwd(x, gamma, beta, allreduce, running_mean=None, running_var=None, eps=1e-5, momentum=0.1):
    x = np.asarray(x, np.float64)
    s = allreduce(np.stack([x.sum(axis=0), (x * x).sum(axis=0), np.full(x.shape[1], float(x.shape[0]))]))
    n = s[2][0]
    mean = s[0] / n
    var = s[1] / n - mean * mean
    invstd = 1.0 / np.sqrt(var + eps)
    y = (x - mean) * invstd * gamma + beta
    rm = rv = None
    if running_mean is not None:
        rm = (1 - momentum) * running_mean + momentum * mean
        rv = (1 - momentum) * running_var + momentum * var * n / max(n - 1, 1)
    return y, mean, invstd, rm, rv


def sync_bn_train_bwd(dy, x, gamma, mean, invstd, allreduce):
    dy = np.asarray(dy, np.float64)
    x = np.asarray(x, np.float64)
    xhat = (x - mean) * invstd
    dbeta = dy.sum(axis=0)
    dgamma = (dy * xhat).sum(axis=0)
    g = allreduce(np.stack([dbeta, dgamma, np.full(x.shape[1], float(x.shape[0]))]))
    n = g[2][0]
    dx = gamma * invstd * (dy - g[0] / n - xhat * g[1] / n)
    return dx, dgamma, dbeta


def relu(x):
    return np.maximum(x, 0)


# ----------------------------------------------------------------------------- head and loss
# F.avg_pool2d(out, 4) + view + nn.Linear(512, 100): net.py:113-115 ; nn.CrossEntropyLoss: trainer.py:40


def head_fwd(act, w, b, bf16_mode=True):
    """act [N,h,w,C] -> (feat [N,C], logits [N,ncls]); global average pool (== avg_pool2d(4) at 4x4)."""
    feat = np.asarray(act, np.float64).mean(axis=(1, 2))
    if bf16_mode:
        feat = bf16(feat).astype(np.float64)
        logits = feat @ bf16(w).astype(np.float64).T + bf16(b).astype(np.float64)
        logits = bf16(logits).astype(np.float64)
    else:
        logits = feat @ np.asarray(w, np.float64).T + b
    return feat, logits


def head_bwd(dlogits, feat, w, hw):
    dl = np.asarray(dlogits, np.float64)
    dw = dl.T @ feat
    db = dl.sum(axis=0)
    dfeat = dl @ np.asarray(w, np.float64)
    N, C = feat.shape
    dact = np.broadcast_to((dfeat / (hw[0] * hw[1]))[:, None, None, :], (N, hw[0], hw[1], C))
    return dw, db, np.array(dact)


def cross_entropy(logits, labels):
    """Mean cross entropy and its gradient w.r.t. logits."""
    z = np.asarray(logits, np.float64)
    m = z.max(axis=1, keepdims=True)
    lse = m[:, 0] + np.log(np.exp(z - m).sum(axis=1))
    n = z.shape[0]
    loss = (lse - z[np.arange(n), labels]).mean()
    p = np.exp(z - lse[:, None])
    p[np.arange(n), labels] -= 1.0
    return loss, p / n, lse


# ----------------------------------------------------------------------------- optimizer / AMP
# optim.SGD(lr, weight_decay, momentum=0.9, nesterov=True): reference src/ddp/trainer.py:92-98


def sgd_nesterov(p, g, buf, lr, wd, mu, first_step):
    """One torch.optim.SGD step (dampening 0, nesterov). Returns (p, buf) in float32 arithmetic."""
    p = np.asarray(p, np.float32)
    d = (np.asarray(g, np.float32) + np.float32(wd) * p).astype(np.float32)
    buf = d.copy() if first_step else (np.float32(mu) * buf + d).astype(np.float32)
    d = (d + np.float32(mu) * buf).astype(np.float32)
    return (p - np.float32(lr) * d).astype(np.float32), buf


def grad_scaler_update(scale, tracker, found_inf, growth=2.0, backoff=0.5, interval=2000):
    """torch GradScaler.update (reference main.py:25, trainer.py:159)."""
    if found_inf:
        return scale * backoff, 0
    tracker += 1
    if tracker == interval:
        return scale * growth, 0
    return scale, tracker


# ----------------------------------------------------------------------------- input pipeline
CIFAR_MEAN = (0.4914, 0.4822, 0.4465)  # reference src/ddp/dataset.py:43-46 (train / valid)
CIFAR_STD = (0.2023, 0.1994, 0.2010)
IMAGENET_MEAN = (0.485, 0.456, 0.406)  # reference src/ddp/dataset.py:139-142 (test loader)
IMAGENET_STD = (0.229, 0.224, 0.225)


def cifar_augment(images, targets, index, crop, flip, mean, std, pad=4):
    """Per-sample host transforms of the reference's DataLoader (src/ddp/dataset.py:57-64, applied
    through Subset(train_idx) + DistributedSampler, dataset.py:95-98) for explicit crop/flip draws.

    The transforms live in third-party torchvision==0.8.2 (requirements.txt:4; absent here), whose
    published algorithm is restated: RandomCrop(32, padding=4) = constant-0 pad by `pad` on every
    side, then crop h x w at (i, j) with i, j drawn from [0, 2*pad]; RandomHorizontalFlip mirrors
    columns after the crop; ToTensor = uint8 HWC -> fp32 CHW, `img.float().div(255)`; Normalize =
    `sub_(mean).div_(std)` per channel. All arithmetic fp32 in that order (true divisions).
    images uint8 [N,H,W,3]; index int [n]; crop int [n,2] or None (centre); flip [n] or None.
    Returns (fp32 [n,3,H,W], int64 labels [n])."""
    images = np.asarray(images, np.uint8)
    n_img, h, w, _ = images.shape
    index = np.arange(n_img) if index is None else np.asarray(index, np.int64)
    n = index.shape[0]
    padded = np.zeros((n_img, h + 2 * pad, w + 2 * pad, 3), np.uint8)
    padded[:, pad:pad + h, pad:pad + w] = images
    out = np.empty((n, 3, h, w), np.float32)
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    for b in range(n):
        i, j = (pad, pad) if crop is None else (int(crop[b][0]), int(crop[b][1]))
        img = padded[index[b], i:i + h, j:j + w]  # [h, w, 3]
        if flip is not None and flip[b]:
            img = img[:, ::-1]
        t = img.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
        out[b] = (t - m) / s
    labels = None if targets is None else np.asarray(targets, np.int64)[index]
    return out, labels
