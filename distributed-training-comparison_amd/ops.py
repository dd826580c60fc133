"""Tensor-level wrappers over the per-op C ABI (include/dtc.h).

Each function takes torch tensors that already live on the GPU (torch is the allocator and
stream provider only), enqueues the native kernel on the current stream and returns output
tensors. bf16 tensors are passed as torch.bfloat16 (same bits as the ABI's uint16_t words).
Nothing here computes on the host and there is no fallback path.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._native import ConvDesc, NativeError, call, lib, ptr, require_cuda, stream_ptr



def conv_desc(n, h, w, c, k, r, s, stride, pad) -> ConvDesc:
    return ConvDesc(n, h, w, c, k, r, s, stride, pad)


def conv_out_hw(h, w, r, s, stride, pad):
    return (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1


def _ws(desc, mode, device):
    nbytes = lib.dtc_conv2d_workspace_size(desc, mode)
    if nbytes == 0:
        return None, 0
    return torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=device), nbytes


def conv2d_fwd(x, w, stride, pad, stats=None):
    """x [N,H,W,C] bf16, w [K,R,S,C] bf16 -> y [N,P,Q,K] bf16 (nn.Conv2d forward, net.py:18)."""
    require_cuda(x, w)
    N, H, W, Cc = x.shape
    K, R, S, _ = w.shape
    d = conv_desc(N, H, W, Cc, K, R, S, stride, pad)
    P, Q = conv_out_hw(H, W, R, S, stride, pad)
    y = torch.empty(N, P, Q, K, dtype=torch.bfloat16, device=x.device)
    ws, nb = _ws(d, 0, x.device)
    call("dtc_conv2d_fwd", d, ptr(x), ptr(w), ptr(y), ptr(stats), ptr(ws), nb, stream_ptr())
    return y


def conv2d_fwd_sc(x, w, wsc, stats=None, stats_sc=None):
    """3x3 stride-2 conv + the 1x1 stride-2 projection shortcut of the same x in one launch (net.py:18-19,
    29-36): x [N,H,W,C], w [K,3,3,C], wsc [K,C] bf16 -> (y, ysc) [N,H/2,W/2,K] bf16."""
    require_cuda(x, w, wsc)
    N, H, W, Cc = x.shape
    K = w.shape[0]
    d = conv_desc(N, H, W, Cc, K, 3, 3, 2, 1)
    P, Q = conv_out_hw(H, W, 3, 3, 2, 1)
    y = torch.empty(N, P, Q, K, dtype=torch.bfloat16, device=x.device)
    ysc = torch.empty_like(y)
    call("dtc_conv2d_fwd_sc", d, ptr(x), ptr(w), ptr(y), ptr(stats), ptr(wsc), ptr(ysc), ptr(stats_sc), stream_ptr())
    return y, ysc


def conv2d_dgrad(dy, w, in_hw, stride, pad, res=None):
    """dy [N,P,Q,K] bf16, w [K,R,S,C] -> dx [N,H,W,C] bf16 (+ res)."""
    require_cuda(dy, w)
    N = dy.shape[0]
    K, R, S, Cc = w.shape
    H, W = in_hw
    d = conv_desc(N, H, W, Cc, K, R, S, stride, pad)
    dx = torch.empty(N, H, W, Cc, dtype=torch.bfloat16, device=dy.device)
    ws, nb = _ws(d, 1, dy.device)
    call("dtc_conv2d_dgrad", d, ptr(dy), ptr(w), ptr(dx), ptr(res), ptr(ws), nb, stream_ptr())
    return dx


def conv2d_dgrad_bn(dy, w, in_hw, stride, pad, ymask, x1, mean1, invstd1, x2=None, mean2=None, invstd2=None,
                    res=None, out=None):
    """conv2d_dgrad fused with bn_bwd_reduce (dtc_conv2d_dgrad_bn): returns (dz, acc1, acc2) where
    dz = bf16(dx [+ res]) * [ymask > 0]; `out` may be `res` (in place)."""
    require_cuda(dy, w)
    N = dy.shape[0]
    K, R, S, Cc = w.shape
    H, W = in_hw
    d = conv_desc(N, H, W, Cc, K, R, S, stride, pad)
    dz = out if out is not None else torch.empty(N, H, W, Cc, dtype=torch.bfloat16, device=dy.device)
    acc1 = new_stats(Cc, dy.device)
    acc2 = new_stats(Cc, dy.device) if x2 is not None else None
    ws, nb = _ws(d, 1, dy.device)
    call("dtc_conv2d_dgrad_bn", d, ptr(dy), ptr(w), ptr(dz), ptr(res), ptr(ymask), ptr(x1), ptr(mean1), ptr(invstd1),
         ptr(acc1), ptr(x2), ptr(mean2), ptr(invstd2), ptr(acc2), ptr(ws), nb, stream_ptr())
    return dz, acc1, acc2


def conv2d_wgrad(x, dy, r, s, stride, pad, scale=1.0):
    """x [N,H,W,C] bf16, dy [N,P,Q,K] bf16 -> dw [K,R,S,C] fp32 (scaled)."""
    require_cuda(x, dy)
    N, H, W, Cc = x.shape
    K = dy.shape[3]
    d = conv_desc(N, H, W, Cc, K, r, s, stride, pad)
    dw = torch.empty(K, r, s, Cc, dtype=torch.float32, device=x.device)
    ws, nb = _ws(d, 2, x.device)
    call("dtc_conv2d_wgrad", d, ptr(x), ptr(dy), ptr(dw), float(scale), ptr(ws), nb, stream_ptr())
    return dw


def conv2d_dgrad_sc(dy, w, dsc, wsc, in_hw):
    """dx through a projection block's conv1 (3x3 stride 2) and its 1x1 stride-2 shortcut in one launch
    (dtc_conv2d_dgrad_sc): dy / dsc [N,P,Q,K], w [K,3,3,C], wsc [K,C] bf16 -> dx [N,H,W,C] bf16."""
    require_cuda(dy, w, dsc, wsc)
    N, _, _, K = dy.shape
    Cc = w.shape[3]
    H, W = in_hw
    d = conv_desc(N, H, W, Cc, K, 3, 3, 2, 1)
    dx = torch.empty(N, H, W, Cc, dtype=torch.bfloat16, device=dy.device)
    call("dtc_conv2d_dgrad_sc", d, ptr(dy), ptr(w), ptr(dx), ptr(dsc), ptr(wsc), stream_ptr())
    return dx


def conv2d_wgrad_sc(x, dy, dsc, scale=1.0):
    """Weight gradients of a projection block's 3x3 stride-2 conv1 and its 1x1 stride-2 shortcut in one
    launch (dtc_conv2d_wgrad_sc): x [N,H,W,C], dy / dsc [N,H/2,W/2,K] bf16 -> (dw [K,3,3,C], dw_sc [K,C])."""
    require_cuda(x, dy, dsc)
    N, H, W, Cc = x.shape
    K = dy.shape[3]
    d = conv_desc(N, H, W, Cc, K, 3, 3, 2, 1)
    nb = lib.dtc_conv2d_wgrad_sc_workspace_size(d)
    if nb == 0:
        raise ValueError(f"conv2d_wgrad_sc: no fused plan for {(N, H, W, Cc, K)}")
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=x.device)
    dw = torch.empty(K, 3, 3, Cc, dtype=torch.float32, device=x.device)
    dw_sc = torch.empty(K, Cc, dtype=torch.float32, device=x.device)
    call("dtc_conv2d_wgrad_sc", d, ptr(x), ptr(dy), ptr(dsc), ptr(dw), ptr(dw_sc), float(scale), ptr(ws), nb,
         stream_ptr())
    return dw, dw_sc


def conv2d_wgrad_batch(xs, dys, scale=1.0):
    """n (<= 4) same-shape 3x3 stride-1 weight gradients in one launch (dtc_conv2d_wgrad_batch):
    xs[i] [N,H,W,C] bf16, dys[i] [N,H,W,K] bf16 -> list of dw [K,3,3,C] fp32 (scaled)."""
    require_cuda(*xs, *dys)
    n = len(xs)
    N, H, W, Cc = xs[0].shape
    K = dys[0].shape[3]
    d = conv_desc(N, H, W, Cc, K, 3, 3, 1, 1)
    nb = lib.dtc_conv2d_wgrad_batch_workspace_size(d, n)
    if nb == 0:
        raise ValueError(f"conv2d_wgrad_batch: no batched halo plan for {(N, H, W, Cc, K)} x {n}")
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=xs[0].device)
    dws = [torch.empty(K, 3, 3, Cc, dtype=torch.float32, device=xs[0].device) for _ in range(n)]
    arr = C.c_void_p * n
    call("dtc_conv2d_wgrad_batch", d, n, arr(*[ptr(t) for t in xs]), arr(*[ptr(t) for t in dys]),
         arr(*[ptr(t) for t in dws]), float(scale), ptr(ws), nb, stream_ptr())
    return dws


def new_stats(c, device):
    """A zeroed BN statistics accumulator for c channels (dtc_bn_stat_words(c) int64 words: exact fixed-point
    sums, common.h): conv epilogues and BN-backward reductions ADD into it."""
    return torch.zeros(int(lib.dtc_bn_stat_words(c)), dtype=torch.int64, device=device)


def stat_totals(stats, c):
    """The two per-channel totals an accumulator holds, as the BN kernels form them (dtc_bn_stat_totals, host
    code): float64 [2, c] on the CPU -- row 0 sum x (sum dz), row 1 sum x^2 (sum dz * xhat)."""
    host = stats.detach().to("cpu", torch.int64).contiguous()
    if host.numel() != int(lib.dtc_bn_stat_words(c)):
        raise ValueError(f"stat_totals: {host.numel()} words is not an accumulator of {c} channels")
    out = torch.empty(2, c, dtype=torch.float64)
    call("dtc_bn_stat_totals", ptr(host), c, ptr(out))
    return out


def stat_from_totals(s, q, device):
    """An accumulator holding the given per-channel totals (float64 arrays of c values; test input for the
    finalize kernels): each total goes into slot 0 in the fixed-point format of common.h."""
    import numpy as np

    s, q = np.asarray(s, np.float64), np.asarray(q, np.float64)
    c = s.shape[0]
    words = np.zeros(int(lib.dtc_bn_stat_words(c)), np.int64)
    hdr = 2 * int(lib.dtc_bn_stat_words(1)) - int(lib.dtc_bn_stat_words(2))  # header words (common.h DTC_STAT_HDR)
    for j, v in enumerate((s, q)):
        d = v * 256.0
        if not np.all(np.abs(d) < 2.0 ** 55):
            raise ValueError("stat_from_totals: total out of range")
        h = np.floor(d)
        words[hdr + (2 * j) * c:hdr + (2 * j + 1) * c] = h.astype(np.int64)
        words[hdr + (2 * j + 1) * c:hdr + (2 * j + 2) * c] = np.floor((d - h) * 2.0 ** 44).astype(np.int64)
    return torch.from_numpy(words).to(device)


def bn_fwd_finalize(stats, count, gamma, beta, running_mean=None, running_var=None, nbt=None, momentum=0.1,
                    eps=1e-5):
    c = gamma.numel()
    dev = gamma.device
    mean, invstd, scale, shift = (torch.empty(c, dtype=torch.float32, device=dev) for _ in range(4))
    call("dtc_bn_fwd_finalize", ptr(stats), c, int(count), ptr(gamma), ptr(beta), ptr(running_mean),
         ptr(running_var), ptr(nbt), float(momentum), float(eps), ptr(mean), ptr(invstd), ptr(scale), ptr(shift),
         stream_ptr())
    return mean, invstd, scale, shift


def bn_apply_relu(x, scale, shift):
    y = torch.empty_like(x)
    m, c = x.numel() // x.shape[-1], x.shape[-1]
    call("dtc_bn_apply_relu", ptr(x), ptr(scale), ptr(shift), ptr(y), m, c, stream_ptr())
    return y


def bn_apply_add_relu(x, scale, shift, res):
    y = torch.empty_like(x)
    m, c = x.numel() // x.shape[-1], x.shape[-1]
    call("dtc_bn_apply_add_relu", ptr(x), ptr(scale), ptr(shift), ptr(res), ptr(y), m, c, stream_ptr())
    return y


def bn_apply_dual_relu(x, scale, shift, x2, scale2, shift2):
    y = torch.empty_like(x)
    m, c = x.numel() // x.shape[-1], x.shape[-1]
    call("dtc_bn_apply_dual_relu", ptr(x), ptr(scale), ptr(shift), ptr(x2), ptr(scale2), ptr(shift2), ptr(y), m, c,
         stream_ptr())
    return y


def bn_bwd_reduce(dy, ymask, x1, mean1, invstd1, x2=None, mean2=None, invstd2=None):
    c = x1.shape[-1]
    m = x1.numel() // c
    acc1 = new_stats(c, x1.device)
    acc2 = new_stats(c, x1.device) if x2 is not None else None
    dz = torch.empty_like(dy) if ymask is not None else None
    call("dtc_bn_bwd_reduce", ptr(dy), ptr(ymask), ptr(x1), ptr(mean1), ptr(invstd1), ptr(acc1), ptr(x2), ptr(mean2),
         ptr(invstd2), ptr(acc2), ptr(dz), m, c, stream_ptr())
    return (dz if dz is not None else dy), acc1, acc2


def bn_bwd_finalize(acc, count, gamma, mean, invstd, gscale=1.0):
    c = gamma.numel()
    dev = gamma.device
    dgamma = torch.empty(c, dtype=torch.float32, device=dev)
    dbeta = torch.empty(c, dtype=torch.float32, device=dev)
    coef = torch.empty(3, c, dtype=torch.float32, device=dev)
    call("dtc_bn_bwd_finalize", ptr(acc), c, int(count), ptr(gamma), ptr(mean), ptr(invstd), float(gscale),
         ptr(dgamma), ptr(dbeta), ptr(coef), stream_ptr())
    return dgamma, dbeta, coef


def bn_bwd_apply(dz, x1, coef1, x2=None, coef2=None):
    c = x1.shape[-1]
    m = x1.numel() // c
    dx1 = torch.empty_like(x1)
    dx2 = torch.empty_like(x2) if x2 is not None else None
    call("dtc_bn_bwd_apply", ptr(dz), ptr(x1), ptr(coef1), ptr(dx1), ptr(x2), ptr(coef2), ptr(dx2), m, c, stream_ptr())
    return dx1, dx2


def bn_mask_bits(y):
    """ReLU mask bits of a post-ReLU NHWC tensor as the forward BN apply writes them: one byte per 8
    channels, bit k = channel 8j+k > 0."""
    c = y.shape[-1]
    b = (y.reshape(-1, c // 8, 8) > 0).to(torch.int32)
    w = torch.tensor([1 << k for k in range(8)], dtype=torch.int32, device=y.device)
    return (b * w).sum(-1).to(torch.uint8).contiguous()


def stem_im2col(x):
    n, _, h, w = x.shape
    cols = torch.empty(n, h, w, 64, dtype=torch.bfloat16, device=x.device)
    call("dtc_stem_im2col", ptr(x), ptr(cols), n, h, w, stream_ptr())
    return cols


def stem_fwd(x, w27, stats=None):
    """Direct stem conv (dtc_stem_fwd): x [N,3,H,W] fp32, w27 [64,27] bf16 (KRSC) -> y [N,H,W,64] bf16."""
    n, _, h, w = x.shape
    y = torch.empty(n, h, w, 64, dtype=torch.bfloat16, device=x.device)
    call("dtc_stem_fwd", ptr(x), ptr(w27), ptr(y), ptr(stats), n, h, w, stream_ptr())
    return y


def stem_wgrad(x, dy, scale=1.0):
    """Direct stem weight gradient (dtc_stem_wgrad): x [N,3,H,W] fp32, dy [N,H,W,64] bf16 -> [64,27] fp32."""
    n, _, h, w = x.shape
    nb = lib.dtc_stem_wgrad_workspace_size(n, h, w)
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=x.device)
    dw = torch.empty(64, 27, dtype=torch.float32, device=x.device)
    call("dtc_stem_wgrad", ptr(x), ptr(dy), ptr(dw), float(scale), n, h, w, ptr(ws), nb, stream_ptr())
    return dw


def stem_pack_weight(w27):
    k = w27.shape[0]
    w64 = torch.empty(k, 64, dtype=torch.bfloat16, device=w27.device)
    call("dtc_stem_pack_weight", ptr(w27), ptr(w64), k, stream_ptr())
    return w64


def head_fwd(act, wfc, bfc):
    """act [N,h,w,C] bf16, wfc [ncls,C] bf16, bfc [ncls] fp32 -> (feat fp32 [N,C], logits fp32 [N,ncls])."""
    n, h, w, c = act.shape
    ncls = wfc.shape[0]
    feat = torch.empty(n, c, dtype=torch.float32, device=act.device)
    logits = torch.empty(n, ncls, dtype=torch.float32, device=act.device)
    call("dtc_head_fwd", ptr(act), n, h * w, c, ptr(wfc), ptr(bfc), ncls, ptr(feat), ptr(logits), stream_ptr())
    return feat, logits


def head_bwd(dlogits, feat, wfc, hw, scale=1.0):
    n, c = feat.shape
    ncls = wfc.shape[0]
    dw = torch.empty(ncls, c, dtype=torch.float32, device=feat.device)
    db = torch.empty(ncls, dtype=torch.float32, device=feat.device)
    h, w = hw
    dact = torch.empty(n, h, w, c, dtype=torch.bfloat16, device=feat.device)
    nb = lib.dtc_head_bwd_workspace_size(n, c, ncls)
    ws = torch.empty(nb // 4 + 1, dtype=torch.float32, device=feat.device)
    call("dtc_head_bwd", ptr(dlogits), ptr(feat), ptr(wfc), n, h * w, c, ncls, float(scale), ptr(dw), ptr(db),
         ptr(dact), ptr(ws), nb, stream_ptr())
    return dw, db, dact


def xent_fwd(logits, labels):
    n, ncls = logits.shape
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    lse = torch.empty(n, dtype=torch.float32, device=logits.device)
    call("dtc_xent_fwd", ptr(logits), ptr(labels), n, ncls, ptr(loss), ptr(lse), stream_ptr())
    return loss, lse


def xent_bwd(logits, labels, lse, gscale=None, out=None):
    n, ncls = logits.shape
    dl = torch.empty_like(logits) if out is None else out
    call("dtc_xent_bwd", ptr(logits), ptr(labels), ptr(lse), ptr(gscale), n, ncls, ptr(dl), stream_ptr())
    return dl


def sgd_nesterov_flat(p, g, mom, pb, lr, weight_decay, momentum, inv_scale=None, found_inf=None):
    call("dtc_sgd_nesterov_flat", ptr(p), ptr(g), ptr(mom), ptr(pb), p.numel(), float(lr), float(weight_decay),
         float(momentum), ptr(inv_scale), ptr(found_inf), stream_ptr())


def cast_f32_bf16(src, dst):
    call("dtc_cast_f32_bf16", ptr(src), ptr(dst), src.numel(), stream_ptr())


def amp_check_finite(g, found_inf):
    call("dtc_amp_check_finite", ptr(g), g.numel(), ptr(found_inf), stream_ptr())


def amp_scale(x, scale):
    """GradScaler.scale(x) (main.py:25, trainer.py:157) on the native kernel: x * scale, device-side."""
    out = torch.empty_like(x)
    call("dtc_amp_scale", ptr(x), ptr(scale), ptr(out), x.numel(), stream_ptr())
    return out


def amp_update_scale(scale, inv_scale, tracker, found_inf, growth, backoff, interval):
    call("dtc_amp_update_scale", ptr(scale), ptr(inv_scale), ptr(tracker), ptr(found_inf), float(growth),
         float(backoff), int(interval), stream_ptr())


def cifar_augment(images, index, crop, flip, mean, std, pad=4, targets=None, out=None, labels=None, status=None):
    """Gather + RandomCrop(pad) + RandomHorizontalFlip + ToTensor + Normalize on the GPU
    (reference src/ddp/dataset.py:43-64). images: uint8 [N,H,W,3]; index: int64 [n] (None: 0..n-1);
    crop: uint8 [n,2] (None: centre); flip: uint8 [n] (None: no flip). Returns (fp32 [n,3,H,W],
    int64 labels [n] or None)."""
    require_cuda(images, index, crop, flip, targets, out, labels, status)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[3] != 3 or not images.is_contiguous():
        raise ValueError(f"images must be contiguous uint8 [N,H,W,3], got {images.dtype} {tuple(images.shape)}")
    n_images, h, w, _ = images.shape
    n = index.numel() if index is not None else (crop.shape[0] if crop is not None else n_images)
    for t, shape, dt in ((index, (n,), torch.int64), (crop, (n, 2), torch.uint8), (flip, (n,), torch.uint8),
                         (targets, (n_images,), torch.int64)):
        if t is not None and (t.dtype != dt or tuple(t.shape) != shape or not t.is_contiguous()):
            raise ValueError(f"expected contiguous {dt} {shape}, got {t.dtype} {tuple(t.shape)}")
    if out is None:
        out = torch.empty(n, 3, h, w, dtype=torch.float32, device=images.device)
    if targets is not None and labels is None:
        labels = torch.empty(n, dtype=torch.int64, device=images.device)
    m = (C.c_float * 3)(*[float(v) for v in mean])
    s = (C.c_float * 3)(*[float(v) for v in std])
    call("dtc_cifar_augment", ptr(images), ptr(targets), n_images, ptr(index), ptr(crop), ptr(flip), n, h, w, int(pad),
         m, s, ptr(out), ptr(labels), ptr(status), stream_ptr())
    return out, labels
