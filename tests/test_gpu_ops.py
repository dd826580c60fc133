"""Per-op parity of the native HIP kernels against the numpy oracle (oracle/ops.py).

Inputs are drawn at bf16-representable values so the kernel and the oracle see identical
operands; the oracle accumulates in float64. Tolerances: bf16 outputs 1e-2 relative (north_star
"per-layer activations and gradients within 1e-2 relative (bf16)"); fp32-output kernels
(wgrad, BN statistics, SGD) tighter where the arithmetic allows.
"""
import numpy as np
import pytest
import torch

from oracle import ops as O
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu

CONV_CASES = [
    # (N, H, W, C, K, R, stride)  -> pad = 1 for 3x3, 0 for 1x1
    (2, 8, 8, 64, 64, 3, 1),      # layer1 conv
    (2, 8, 8, 64, 128, 3, 2),     # layer2.0.conv1 (stride 2)
    (2, 8, 8, 64, 128, 1, 2),     # layer2.0.shortcut (1x1 s2)
    (2, 8, 8, 128, 128, 3, 1),    # layer2 conv
    (3, 4, 4, 256, 512, 3, 2),    # layer4.0.conv1 (ragged pixel count, split-K)
    (4, 4, 4, 512, 512, 3, 1),    # layer4 conv (deep reduction, split-K)
    (2, 32, 32, 64, 64, 1, 1),    # stem GEMM over the 64-column im2col image
    (1, 5, 7, 64, 64, 3, 1),      # odd spatial size, M not a tile multiple
    (16, 16, 16, 256, 256, 3, 1),  # 64x64 tiles, no split (fused-stats epilogue)
    (26, 32, 32, 128, 256, 3, 1),  # 128x128 tiles, no split, ragged last pixel tile
    (100, 32, 32, 64, 64, 3, 1),   # 64x256 tiles (K=64 layers), no split
    (64, 16, 16, 64, 128, 3, 2),   # stride-2 class GEMMs big enough for 64x256 tiles
    (5, 8, 8, 256, 256, 3, 1),     # halo conv: 2 images per tile, ragged last tile
    (9, 4, 4, 512, 256, 3, 1),     # halo conv: 8 images per tile, C != K
]


def _rand_bf16(shape, gen, scale=1.0):
    return O.bf16(gen.standard_normal(shape).astype(np.float32) * scale)


def _to_dev_bf16(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev).to(torch.bfloat16)


# stride-2 3x3 forward on the column-split halo kernel (option halo_s2; conv_halo.hip ST = 2), alone and
# with the block's 1x1 stride-2 projection shortcut fused (dtc_conv2d_fwd_sc): ResNet-18's three stride-2
# geometries (output widths 16 / 8 / 4: one-row fragments, fragments spanning 2 rows with the padded
# pitch, 4 images per tile) plus a ragged batch, against the oracle
S2_CASES = [(8, 32, 32, 64, 128), (8, 16, 16, 128, 256), (8, 8, 8, 256, 512), (5, 16, 16, 128, 256), (2, 8, 8, 64, 128)]
# general stride-2 geometry (the 224x224 model's conv1 of layers 2-4: output rows of 112 / 56 / 28)
S2_GEN_CASES = [(2, 8, 224, 64, 128), (1, 4, 112, 128, 64), (2, 12, 56, 64, 64)]


@pytest.mark.parametrize("case,cfg", [(c, k) for c in S2_CASES for k in (1, 2, 3, 4)] +
                         [(c, k) for c in S2_GEN_CASES for k in (2, 3)])
def test_conv_fwd_stride2_halo_and_shortcut(dtc, cuda, case, cfg):
    """Option halo_s2: the stride-2 forward on the column-split halo kernel (auto / forced configurations),
    alone and with the 1x1 shortcut fused, + BN statistics, against the oracle; the general-geometry cases
    (rows of 112 / 56 / 28 output pixels: 64-bit per-tile bases, padded slots) take configuration 8's
    general instances at the forced settings (cfg >= 2; at auto they take the implicit GEMM, whose fused
    shortcut plan covers only layer4-size grids)."""
    N, H, W, C, K = case
    lib = dtc._native.lib
    g = np.random.default_rng(3)
    x = _rand_bf16((N, H, W, C), g)
    w = _rand_bf16((K, 3, 3, C), g, 0.05)
    wsc = _rand_bf16((K, 1, 1, C), g, 0.1)
    ref = O.conv2d_fwd(x, w, 2, 1)
    ref_sc = O.conv2d_fwd(x, wsc, 2, 0)
    xd, wd, wscd = _to_dev_bf16(x, cuda), _to_dev_bf16(w, cuda), _to_dev_bf16(wsc.reshape(K, C), cuda)
    prev = lib.dtc_get_option(b"halo_s2")
    try:
        lib.dtc_set_option(b"halo_s2", cfg)
        st = dtc.ops.new_stats(K, cuda)
        y = dtc.ops.conv2d_fwd(xd, wd, 2, 1, stats=st).float().cpu().numpy()
        st1, st2 = dtc.ops.new_stats(K, cuda), dtc.ops.new_stats(K, cuda)
        y2, ysc = dtc.ops.conv2d_fwd_sc(xd, wd, wscd, stats=st1, stats_sc=st2)
        torch.cuda.synchronize()
    finally:
        lib.dtc_set_option(b"halo_s2", prev)
    y2, ysc = y2.float().cpu().numpy(), ysc.float().cpu().numpy()
    assert rel_err(y, ref) < 1e-2 and rel_err(y2, ref) < 1e-2 and rel_err(ysc, ref_sc) < 1e-2
    for out, stt in ((y, st), (y2, st1), (ysc, st2)):  # BN statistics of the bf16 outputs, fp64 slots
        s_ = dtc.ops.stat_totals(stt, K).numpy()
        yb = out.reshape(-1, K).astype(np.float64)
        np.testing.assert_allclose(s_[0], yb.sum(0), rtol=1e-5, atol=1e-3)
        np.testing.assert_allclose(s_[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(dtc, cuda, case):
    N, H, W, C, K, R, st = case
    pad = 1 if R == 3 else 0
    g = np.random.default_rng(1)
    x = _rand_bf16((N, H, W, C), g)
    w = _rand_bf16((K, R, R, C), g, 0.05)
    stats = dtc.ops.new_stats(K, cuda)
    y = dtc.ops.conv2d_fwd(_to_dev_bf16(x, cuda), _to_dev_bf16(w, cuda), st, pad, stats=stats)
    ref = O.conv2d_fwd(x, w, st, pad)
    yk = y.float().cpu().numpy()
    assert yk.shape == ref.shape
    assert rel_err(yk, ref) < 1e-2
    # BN statistics of the bf16 output, accumulated in fp64 slots
    s = dtc.ops.stat_totals(stats, K).numpy()
    yb = yk.reshape(-1, K).astype(np.float64)
    np.testing.assert_allclose(s[0], yb.sum(0), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("case", CONV_CASES[:6] + CONV_CASES[7:])
@pytest.mark.parametrize("with_res", [False, True])
def test_conv_dgrad(dtc, cuda, case, with_res):
    N, H, W, C, K, R, st = case
    pad = 1 if R == 3 else 0
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    g = np.random.default_rng(2)
    dy = _rand_bf16((N, P, Q, K), g)
    w = _rand_bf16((K, R, R, C), g, 0.05)
    res = _rand_bf16((N, H, W, C), g) if with_res else None
    dx = dtc.ops.conv2d_dgrad(_to_dev_bf16(dy, cuda), _to_dev_bf16(w, cuda), (H, W), st, pad,
                              res=_to_dev_bf16(res, cuda) if with_res else None)
    ref = O.conv2d_dgrad(dy, w, (H, W), st, pad)
    if with_res:
        ref = ref + res
    assert rel_err(dx.float().cpu().numpy(), ref) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad(dtc, cuda, case):
    N, H, W, C, K, R, st = case
    pad = 1 if R == 3 else 0
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    g = np.random.default_rng(3)
    x = _rand_bf16((N, H, W, C), g)
    dy = _rand_bf16((N, P, Q, K), g)
    dw = dtc.ops.conv2d_wgrad(_to_dev_bf16(x, cuda), _to_dev_bf16(dy, cuda), R, R, st, pad, scale=0.5)
    ref = 0.5 * O.conv2d_wgrad(x, dy, R, R, st, pad)
    # fp32 accumulation of exact bf16 products: only summation-order differences remain
    assert rel_err(dw.cpu().numpy(), ref) < 1e-5


@pytest.mark.parametrize("case", S2_CASES + S2_GEN_CASES)
def test_conv_wgrad_stride2_halo_and_shortcut(dtc, cuda, case):
    """Option wgrad_s2: the 3x3 stride-2 weight gradient on the column-split halo kernel (all nine taps
    from one x halo per 64-pixel step), alone and with the 1x1 stride-2 shortcut's fused in (its centre
    tap against dsc: dtc_conv2d_wgrad_sc), against the oracle; geometries without a plan fall back."""
    N, H, W, C, K = case
    lib = dtc._native.lib
    g = np.random.default_rng(7)
    x = _rand_bf16((N, H, W, C), g)
    dy = _rand_bf16((N, H // 2, W // 2, K), g)
    dsc = _rand_bf16((N, H // 2, W // 2, K), g)
    ref = 0.5 * O.conv2d_wgrad(x, dy, 3, 3, 2, 1)
    ref_sc = 0.5 * O.conv2d_wgrad(x, dsc, 1, 1, 2, 0).reshape(K, C)
    xd, dyd, dscd = _to_dev_bf16(x, cuda), _to_dev_bf16(dy, cuda), _to_dev_bf16(dsc, cuda)
    prev = lib.dtc_get_option(b"wgrad_s2")
    try:
        lib.dtc_set_option(b"wgrad_s2", 1)
        dw = dtc.ops.conv2d_wgrad(xd, dyd, 3, 3, 2, 1, scale=0.5).cpu().numpy()
        d = dtc.ops.conv_desc(N, H, W, C, K, 3, 3, 2, 1)
        fused = lib.dtc_conv2d_wgrad_sc_workspace_size(d) > 0
        if fused:
            dw2, dwsc = dtc.ops.conv2d_wgrad_sc(xd, dyd, dscd, scale=0.5)
            dw2, dwsc = dw2.cpu().numpy(), dwsc.cpu().numpy()
    finally:
        lib.dtc_set_option(b"wgrad_s2", prev)
    assert rel_err(dw, ref) < 1e-5
    assert fused == (N * (H // 2) * (W // 2) % 64 == 0 or case in S2_GEN_CASES)
    if fused:
        assert rel_err(dw2, ref) < 1e-5 and rel_err(dwsc, ref_sc) < 1e-5


@pytest.mark.parametrize("case", S2_CASES)
def test_conv_dgrad_stride2_with_fused_shortcut(dtc, cuda, case):
    """Option dgrad_scf: dx through conv1 (3x3 stride 2) + the 1x1 stride-2 shortcut in one parity-class
    launch (dtc_conv2d_dgrad_sc; the shortcut as extra reduction steps of class (0, 0)) vs the oracle."""
    N, H, W, C, K = case
    lib = dtc._native.lib
    g = np.random.default_rng(9)
    dy = _rand_bf16((N, H // 2, W // 2, K), g)
    dsc = _rand_bf16((N, H // 2, W // 2, K), g)
    w = _rand_bf16((K, 3, 3, C), g, 0.05)
    wsc = _rand_bf16((K, 1, 1, C), g, 0.1)
    ref = O.conv2d_dgrad(dy, w, (H, W), 2, 1) + O.conv2d_dgrad(dsc, wsc, (H, W), 2, 0)
    prev = lib.dtc_get_option(b"dgrad_scf")
    try:
        lib.dtc_set_option(b"dgrad_scf", 1)
        dx = dtc.ops.conv2d_dgrad_sc(_to_dev_bf16(dy, cuda), _to_dev_bf16(w, cuda), _to_dev_bf16(dsc, cuda),
                                     _to_dev_bf16(wsc.reshape(K, C), cuda), (H, W))
        torch.cuda.synchronize()
    finally:
        lib.dtc_set_option(b"dgrad_scf", prev)
    assert rel_err(dx.float().cpu().numpy(), ref) < 1e-2


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[6] == 2])
@pytest.mark.parametrize("classes", [0, 1])
def test_conv_dgrad_stride2_paths(dtc, cuda, case, classes):
    """Stride-2 data gradient: parity-class decomposition (default) and the generic masked path."""
    N, H, W, C, K, R, st = case
    pad = 1 if R == 3 else 0
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    g = np.random.default_rng(12)
    dy = _rand_bf16((N, P, Q, K), g)
    w = _rand_bf16((K, R, R, C), g, 0.05)
    res = _rand_bf16((N, H, W, C), g)
    dtc._native.call("dtc_set_option", b"dgrad_classes", classes)
    try:
        dx = dtc.ops.conv2d_dgrad(_to_dev_bf16(dy, cuda), _to_dev_bf16(w, cuda), (H, W), st, pad,
                                  res=_to_dev_bf16(res, cuda))
    finally:
        dtc._native.call("dtc_set_option", b"dgrad_classes", 1)
    ref = O.conv2d_dgrad(dy, w, (H, W), st, pad) + res
    assert rel_err(dx.float().cpu().numpy(), ref) < 1e-2


def test_mfma_layout_identity(dtc, cuda):
    """A = I-style check with an asymmetric operand (guide §3): a 1x1 conv with the identity
    filter must reproduce x exactly, and a permutation filter must permute channels."""
    g = np.random.default_rng(4)
    x = _rand_bf16((2, 4, 4, 64), g)
    perm = g.permutation(64)
    w = np.zeros((64, 1, 1, 64), np.float32)
    w[np.arange(64), 0, 0, perm] = 1.0
    y = dtc.ops.conv2d_fwd(_to_dev_bf16(x, cuda), _to_dev_bf16(w, cuda), 1, 0).float().cpu().numpy()
    np.testing.assert_array_equal(y, x[..., perm])


@pytest.mark.parametrize("C", [64, 512])
def test_bn_forward(dtc, cuda, C):
    M = 300
    g = np.random.default_rng(5)
    x = O.bf16(_rand_bf16((M, C), g, 2.0) + 0.5)
    gamma = g.uniform(0.5, 1.5, C).astype(np.float32)
    beta = g.uniform(-0.5, 0.5, C).astype(np.float32)
    rm = np.zeros(C, np.float32)
    rv = np.ones(C, np.float32)
    dev = cuda
    xs = x.astype(np.float64)
    stats = dtc.ops.stat_from_totals(xs.sum(0), (xs * xs).sum(0), dev)
    t = lambda a: torch.from_numpy(a).to(dev)
    rm_d, rv_d = t(rm.copy()), t(rv.copy())
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    mean, invstd, scale, shift = dtc.ops.bn_fwd_finalize(stats, M, t(gamma), t(beta), rm_d, rv_d, nbt)
    y_ref, m_ref, is_ref, rm_ref, rv_ref = O.bn_train_fwd(x, gamma, beta, rm, rv)
    np.testing.assert_allclose(mean.cpu().numpy(), m_ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(invstd.cpu().numpy(), is_ref, rtol=1e-5)
    np.testing.assert_allclose(rm_d.cpu().numpy(), rm_ref, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(rv_d.cpu().numpy(), rv_ref, rtol=1e-5)
    assert int(nbt.item()) == 1
    assert float(stats.abs().sum()) == 0.0  # finalize re-zeroes the slots
    xd = _to_dev_bf16(x, dev)
    y = dtc.ops.bn_apply_relu(xd, scale, shift).float().cpu().numpy()
    assert rel_err(y, O.relu(y_ref)) < 1e-2
    r = _rand_bf16((M, C), g)
    y2 = dtc.ops.bn_apply_add_relu(xd, scale, shift, _to_dev_bf16(r, dev)).float().cpu().numpy()
    assert rel_err(y2, O.relu(O.bf16(y_ref) + r)) < 1e-2
    y3 = dtc.ops.bn_apply_dual_relu(xd, scale, shift, _to_dev_bf16(r, dev), scale, shift).float().cpu().numpy()
    y_r, *_ = O.bn_train_fwd(x, gamma, beta)
    yr2 = (r - m_ref) * is_ref * gamma + beta
    assert rel_err(y3, O.relu(O.bf16(y_ref) + O.bf16(yr2))) < 1e-2


@pytest.mark.parametrize("C,dual", [(64, False), (128, True), (512, False)])
def test_bn_backward(dtc, cuda, C, dual):
    M = 256
    g = np.random.default_rng(6)
    x = O.bf16(_rand_bf16((M, C), g, 1.5) + 0.2)
    x2 = O.bf16(_rand_bf16((M, C), g, 0.7) - 0.1)
    y = _rand_bf16((M, C), g)  # relu output stand-in (mask)
    dy = _rand_bf16((M, C), g)
    gamma = g.uniform(0.5, 1.5, C).astype(np.float32)
    gamma2 = g.uniform(0.5, 1.5, C).astype(np.float32)
    _, mean, invstd, _, _ = O.bn_train_fwd(x, gamma, np.zeros(C))
    _, mean2, invstd2, _, _ = O.bn_train_fwd(x2, gamma2, np.zeros(C))
    dev = cuda
    t = lambda a: torch.from_numpy(np.asarray(a, np.float32)).to(dev)
    b = lambda a: _to_dev_bf16(a, dev)
    dz, acc1, acc2 = dtc.ops.bn_bwd_reduce(b(dy), b(y), b(x), t(mean), t(invstd),
                                           b(x2) if dual else None, t(mean2) if dual else None,
                                           t(invstd2) if dual else None)
    dz_ref = np.where(y > 0, dy, 0)
    np.testing.assert_array_equal(dz.float().cpu().numpy(), dz_ref)
    dg, db, coef = dtc.ops.bn_bwd_finalize(acc1, M, t(gamma), t(mean), t(invstd), gscale=0.5)
    dx_ref, dg_ref, db_ref = O.bn_train_bwd(dz_ref, x, gamma, mean, invstd)
    np.testing.assert_allclose(dg.cpu().numpy(), 0.5 * dg_ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(db.cpu().numpy(), 0.5 * db_ref, rtol=1e-4, atol=1e-4)
    coef2 = None
    if dual:
        dg2, db2, coef2 = dtc.ops.bn_bwd_finalize(acc2, M, t(gamma2), t(mean2), t(invstd2))
        dx2_ref, dg2_ref, db2_ref = O.bn_train_bwd(dz_ref, x2, gamma2, mean2, invstd2)
        np.testing.assert_allclose(dg2.cpu().numpy(), dg2_ref, rtol=1e-4, atol=1e-4)
    dx1, dx2 = dtc.ops.bn_bwd_apply(dz, b(x), coef, b(x2) if dual else None, coef2)
    assert rel_err(dx1.float().cpu().numpy(), dx_ref) < 1e-2
    if dual:
        assert rel_err(dx2.float().cpu().numpy(), dx2_ref) < 1e-2


@pytest.mark.parametrize("head_fused", [1, 0])
def test_head_and_loss(dtc, cuda, head_fused):
    dtc._native.lib.dtc_set_option(b"head_fused", head_fused)
    try:
        _head_and_loss(dtc, cuda)
    finally:
        dtc._native.lib.dtc_set_option(b"head_fused", 1)


def _head_and_loss(dtc, cuda):
    N, C, ncls = 6, 512, 100
    g = np.random.default_rng(7)
    act = O.relu(_rand_bf16((N, 4, 4, C), g))
    w = _rand_bf16((ncls, C), g, 0.05)
    bias = g.standard_normal(ncls).astype(np.float32) * 0.1
    labels = g.integers(0, ncls, N)
    dev = cuda
    feat, logits = dtc.ops.head_fwd(_to_dev_bf16(act, dev), _to_dev_bf16(w, dev), torch.from_numpy(bias).to(dev))
    f_ref, l_ref = O.head_fwd(act, w, bias, bf16_mode=True)
    assert rel_err(feat.cpu().numpy(), f_ref) < 1e-5
    assert rel_err(logits.cpu().numpy(), l_ref) < 1e-2
    lab = torch.from_numpy(labels).to(dev)
    loss, lse = dtc.ops.xent_fwd(logits, lab)
    loss_ref, dl_ref, lse_ref = O.cross_entropy(logits.cpu().numpy(), labels)
    assert abs(float(loss) - loss_ref) < 1e-5 * max(1.0, abs(loss_ref))
    gs = torch.full((1,), 4.0, device=dev)
    dl = dtc.ops.xent_bwd(logits, lab, lse, gs)
    np.testing.assert_allclose(dl.cpu().numpy(), 4.0 * dl_ref, rtol=1e-4, atol=1e-6)
    dw, db, dact = dtc.ops.head_bwd(dl, feat, _to_dev_bf16(w, dev), (4, 4), scale=0.25)
    dw_ref, db_ref, dact_ref = O.head_bwd(dl.cpu().numpy(), feat.cpu().numpy(), w, (4, 4))
    assert rel_err(dw.cpu().numpy(), 0.25 * dw_ref) < 1e-5
    assert rel_err(db.cpu().numpy(), 0.25 * db_ref) < 1e-5
    assert rel_err(dact.float().cpu().numpy(), dact_ref) < 1e-2


@pytest.mark.parametrize("n,ncls", [(1, 100), (6, 100), (256, 100), (300, 100), (4096, 100), (7, 10), (256, 10),
                                    (65, 129), (300, 129), (1000, 1000), (33, 1000)])
def test_xent_fwd_one_launch(dtc, cuda, n, ncls):
    """dtc_xent_fwd_ex (the training step's loss in one launch): loss and lse bit-identical to the
    two-kernel dtc_xent_fwd, scaled = loss * scale (amp_scale's multiply), the loss in a pinned host word;
    and against the oracle. ADVICE r4: heads wider than 128 classes take the kernel's per-row branch
    (ncls 129 / 1000), and row counts that are not multiples of 64 / 256 / 1024 are covered."""
    g = torch.Generator(device=cuda).manual_seed(n * 1000 + ncls)
    logits = torch.randn(n, ncls, device=cuda, generator=g) * 3
    lab = torch.randint(0, ncls, (n,), device=cuda, generator=g)
    loss0, lse0 = dtc.ops.xent_fwd(logits, lab)
    scale = torch.full((), 65536.0, device=cuda)
    loss = torch.empty((), device=cuda)
    lse = torch.empty(n, device=cuda)
    scaled = torch.empty((), device=cuda)
    host = torch.full((4,), -1.0).pin_memory()
    P = dtc._native.ptr
    dtc._native.call("dtc_xent_fwd_ex", P(logits), P(lab), n, ncls, P(loss), P(lse), P(scale), P(scaled),
                     host[1:2].data_ptr(), dtc._native.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(loss, loss0) and torch.equal(lse, lse0)
    assert float(scaled) == float(loss) * 65536.0
    assert float(host[1]) == float(loss) and float(host[0]) == -1.0 and float(host[2]) == -1.0
    loss_ref, _, lse_ref = O.cross_entropy(logits.cpu().numpy(), lab.cpu().numpy())
    assert abs(float(loss) - loss_ref) < 1e-5 * max(1.0, abs(loss_ref))
    np.testing.assert_allclose(lse.cpu().numpy(), lse_ref, rtol=1e-5, atol=1e-5)
    # without the optional outputs
    dtc._native.call("dtc_xent_fwd_ex", P(logits), P(lab), n, ncls, P(loss), P(lse), None, None, None,
                     dtc._native.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(loss, loss0)
    # an out-of-range label makes the loss NaN on both paths (torch raises; the kernels flag it in the value)
    bad = lab.clone()
    bad[n // 2] = ncls
    loss1, _ = dtc.ops.xent_fwd(logits, bad)
    dtc._native.call("dtc_xent_fwd_ex", P(logits), P(bad), n, ncls, P(loss), P(lse), None, None, None,
                     dtc._native.stream_ptr())
    torch.cuda.synchronize()
    assert torch.isnan(loss).item() and torch.isnan(loss1).item()


def test_stem_im2col(dtc, cuda):
    g = np.random.default_rng(8)
    x = g.standard_normal((2, 3, 6, 5)).astype(np.float32)
    cols = dtc.ops.stem_im2col(torch.from_numpy(x).to(cuda)).float().cpu().numpy()
    ref = O._im2col(O.nchw_to_nhwc(x), 3, 3, 1, 1).reshape(2, 6, 5, 27)
    np.testing.assert_array_equal(cols[..., :27], O.bf16(ref))
    assert not cols[..., 27:].any()


@pytest.mark.parametrize("shape", [(2, 6, 5), (4, 32, 32), (3, 7, 9)])
def test_stem_direct_fwd_wgrad(dtc, cuda, shape):
    """Direct stem conv (stem.hip: taps gathered per 256-pixel tile, one K=32 MFMA k-step) vs the
    oracle conv on the same bf16 operands (conv1 = nn.Conv2d(3, 64, 3, 1, 1), net.py:91): forward
    (bf16 output), its BN batch sums, and the fp32 weight gradient; ragged last tiles included."""
    n, h, w = shape
    g = np.random.default_rng(12)
    x = g.standard_normal((n, 3, h, w)).astype(np.float32)
    w27 = _rand_bf16((64, 3, 3, 3), g, scale=0.2)
    dy = _rand_bf16((n, h, w, 64), g)
    xd = torch.from_numpy(x).to(cuda)
    xb = O.bf16(O.nchw_to_nhwc(x))  # the kernel rounds the gathered taps to bf16
    stats = dtc.ops.new_stats(64, cuda)
    y = dtc.ops.stem_fwd(xd, _to_dev_bf16(w27.reshape(64, 27), cuda), stats).float().cpu().numpy()
    ref = O.conv2d_fwd(xb, w27, 1, 1)
    assert rel_err(y, O.bf16(ref)) < 1e-2
    st = dtc.ops.stat_totals(stats, 64).numpy()
    yb = y.reshape(-1, 64).astype(np.float64)
    np.testing.assert_allclose(st[0], yb.sum(0), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(st[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)
    dw = dtc.ops.stem_wgrad(xd, _to_dev_bf16(dy, cuda), scale=0.5).cpu().numpy()
    ref_w = 0.5 * O.conv2d_wgrad(xb, dy, 3, 3, 1, 1).reshape(64, 27)
    assert rel_err(dw, ref_w) < 1e-5


def test_sgd_and_amp(dtc, cuda):
    n = 4096
    g = np.random.default_rng(9)
    p = g.standard_normal(n).astype(np.float32)
    dev = cuda
    P = torch.from_numpy(p.copy()).to(dev)
    M = torch.zeros(n, device=dev)
    PB = torch.empty(n, dtype=torch.bfloat16, device=dev)
    inv = torch.full((1,), 0.25, device=dev)
    found = torch.zeros(1, dtype=torch.int32, device=dev)
    pr, buf = p.copy(), None
    for step in range(3):
        grad = g.standard_normal(n).astype(np.float32)
        dtc.ops.sgd_nesterov_flat(P, torch.from_numpy(grad * 4).to(dev), M, PB, 0.1, 1e-4, 0.9, inv, found)
        pr, buf = O.sgd_nesterov(pr, grad, buf, 0.1, 1e-4, 0.9, step == 0)
    # fp32 update; FMA contraction may move the last bit
    np.testing.assert_allclose(P.cpu().numpy(), pr, rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(PB.float().cpu().numpy(), O.bf16(P.cpu().numpy()))
    # overflow: check sets found_inf, the step is skipped, the scale backs off
    bad = torch.zeros(n, device=dev)
    bad[17] = float("inf")
    dtc.ops.amp_check_finite(bad, found)
    assert int(found.item()) == 1
    before = P.clone()
    dtc.ops.sgd_nesterov_flat(P, bad, M, PB, 0.1, 1e-4, 0.9, inv, found)
    assert torch.equal(before, P)
    scale = torch.full((1,), 65536.0, device=dev)
    tracker = torch.zeros(1, dtype=torch.int32, device=dev)
    dtc.ops.amp_update_scale(scale, inv, tracker, found, 2.0, 0.5, 3)
    assert float(scale) == 32768.0 and int(found.item()) == 0
    for _ in range(3):
        dtc.ops.amp_update_scale(scale, inv, tracker, found, 2.0, 0.5, 3)
    assert float(scale) == 65536.0 and abs(float(inv) - 1 / 65536.0) < 1e-12


@pytest.mark.parametrize("n", [1, 7, 4096, 1_048_579, 11_220_000])
def test_amp_check_finite_positions(dtc, cuda, n):
    """found_inf over every region of the vectorised check: the 4-deep float4 trips, the float4
    remainder trips, the scalar tail (n % 4), an unaligned view (scalar kernel); finite input: 0."""
    found = torch.zeros(1, dtype=torch.int32, device=cuda)
    base = torch.zeros(n + 1, device=cuda)
    dtc.ops.amp_check_finite(base[:n], found)
    assert int(found.item()) == 0
    for pos in sorted({p for p in (0, n // 3, n // 2, n - 1 - (n % 4), n - 1) if 0 <= p < n}):
        for bad in (float("inf"), float("-inf"), float("nan")):
            g = base.clone()
            g[pos] = bad
            found.zero_()
            dtc.ops.amp_check_finite(g[:n], found)
            assert int(found.item()) == 1, (n, pos, bad)
            found.zero_()
            dtc.ops.amp_check_finite(g[1:n + 1] if pos > 0 else g[:n], found)  # 4-B offset: scalar kernel
            assert int(found.item()) == 1, (n, pos, bad, "unaligned")


@pytest.mark.parametrize("case", [
    (4, 32, 32, 64, 64),    # layer1 geometry: 2 output rows per 64-pixel step
    (3, 8, 8, 64, 128),     # whole 8x8 image per step, 3 steps (ragged split)
    (8, 16, 16, 128, 128),  # 4 rows per step, 2x2 output tiles
    (8, 8, 8, 256, 64),     # C > K
    (12, 4, 4, 512, 512),   # four 4x4 images per step (multi-image halo)
    (2, 2, 2, 64, 64),      # 2x2 images: halo too tall -> generic loader
    (2, 4, 4, 512, 512),    # 32 pixels: no whole 64-pixel step -> generic loader
    (3, 4, 4, 64, 64),      # 48 pixels (N not a multiple of 4 images) -> generic loader
    # general step geometry (option wgrad_gen; the 224x224 model's rows): rs rows x seg columns per step
    (2, 14, 224, 64, 64),   # 56-pixel segments, 4 per row
    (2, 12, 112, 64, 128),  # 56-pixel segments, 2 per row
    (3, 10, 56, 128, 64),   # one 56-pixel row per step
    (2, 28, 28, 256, 128),  # two 28-pixel rows per step
    (2, 6, 96, 64, 64),     # 32-pixel segments
    (1, 5, 40, 64, 64),     # one 40-pixel row per step (24 padded slots)
])
def test_conv_wgrad_halo(dtc, cuda, case):
    """Halo-tiled 3x3 weight gradient == generic loader == oracle (fp32 sums of exact products); the rows
    wider than 64 pixels or not dividing 64 run the general-geometry kernels (per-step 64-bit bases, zero-dy
    padded slots), which must match too."""
    N, H, W, C, K = case
    g = np.random.default_rng(7)
    x = _rand_bf16((N, H, W, C), g)
    dy = _rand_bf16((N, H, W, K), g)
    xd, dyd = _to_dev_bf16(x, cuda), _to_dev_bf16(dy, cuda)
    ref = O.conv2d_wgrad(x, dy, 3, 3, 1, 1)
    try:
        halo = dtc.ops.conv2d_wgrad(xd, dyd, 3, 3, 1, 1).cpu().numpy()
        dtc._native.lib.dtc_set_option(b"wgrad_halo", 0)
        generic = dtc.ops.conv2d_wgrad(xd, dyd, 3, 3, 1, 1).cpu().numpy()
    finally:
        dtc._native.lib.dtc_set_option(b"wgrad_halo", 224)
    assert rel_err(halo, ref) < 1e-5
    assert rel_err(generic, ref) < 1e-5


@pytest.mark.parametrize("case", [
    (4, 32, 32, 64, 64, 4),    # layer1 geometry, the executor's four-conv batch (64 splits each)
    (4, 32, 32, 64, 64, 2),
    (8, 16, 16, 128, 128, 3),  # 2x2 output tiles, three problems
    (12, 4, 4, 512, 512, 4),   # multi-image halo, one split per problem
    (3, 8, 8, 64, 128, 2),     # ragged split of 3 steps
    (2, 8, 224, 64, 64, 4),    # general geometry (56-pixel row segments), the 224x224 layer1 batch
    (2, 14, 28, 128, 128, 3),  # general geometry, two 28-pixel rows per step
])
def test_conv_wgrad_batch(dtc, cuda, case):
    """dtc_conv2d_wgrad_batch: n independent weight gradients in one halo launch (blockIdx.z =
    problem, 1/n of the splits each) + one reduce launch == the oracle per problem, and == the
    one-by-one dtc_conv2d_wgrad to fp32 summation order (different split counts); bit-identical when
    repeated."""
    N, H, W, C, K, n = case
    g = np.random.default_rng(11)
    xs = [_rand_bf16((N, H, W, C), g) for _ in range(n)]
    dys = [_rand_bf16((N, H, W, K), g) for _ in range(n)]
    xd = [_to_dev_bf16(a, cuda) for a in xs]
    dyd = [_to_dev_bf16(a, cuda) for a in dys]
    got = dtc.ops.conv2d_wgrad_batch(xd, dyd, scale=0.25)
    again = dtc.ops.conv2d_wgrad_batch(xd, dyd, scale=0.25)
    ones = [dtc.ops.conv2d_wgrad(xd[i], dyd[i], 3, 3, 1, 1, scale=0.25).cpu().numpy() for i in range(n)]
    assert len(got) == n
    for a, b in zip(got, again):
        assert torch.equal(a, b)
    for i in range(n):
        ref = 0.25 * O.conv2d_wgrad(xs[i], dys[i], 3, 3, 1, 1)
        one = ones[i]
        assert rel_err(got[i].cpu().numpy(), ref) < 1e-5, i
        assert rel_err(got[i].cpu().numpy(), one) < 1e-6, i


def test_conv_wgrad_batch_rejects_non_halo(dtc, cuda):
    """No batched plan for a stride-2 geometry: workspace size 0 and a clean error, no launch."""
    d = dtc.ops.conv_desc(8, 16, 16, 64, 128, 3, 3, 2, 1)
    assert dtc._native.lib.dtc_conv2d_wgrad_batch_workspace_size(d, 2) == 0


HALO_CASES = [
    # (N, H, W, C, K): 3x3 stride-1 convs for every halo configuration (conv_halo.hip)
    (2, 32, 32, 64, 64),
    (3, 16, 16, 128, 128),
    (5, 8, 8, 256, 128),
    (9, 4, 4, 128, 256),
]


@pytest.mark.parametrize("split", [0, 2])
@pytest.mark.parametrize("cfg", list(range(8)))
@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_configs(dtc, cuda, case, cfg, split):
    """Halo-tiled FWD (+BN statistics) and DGRAD (+residual) in each forced configuration
    (option halo_conv = 2 + cfg; a geometry the configuration cannot tile falls back to the
    implicit-GEMM kernel, which must agree as well), unsplit and split-K over reduction chunks
    (fp32 slab + splitk_reduce epilogue)."""
    N, H, W, C, K = case
    g = np.random.default_rng(21 + cfg)
    x = _rand_bf16((N, H, W, C), g)
    w = _rand_bf16((K, 3, 3, C), g, 0.05)
    dy = _rand_bf16((N, H, W, K), g)
    res = _rand_bf16((N, H, W, C), g)
    dtc._native.call("dtc_set_option", b"halo_conv", 2 + cfg)
    dtc._native.call("dtc_set_option", b"halo_split", split)
    try:
        stats = dtc.ops.new_stats(K, cuda)
        y = dtc.ops.conv2d_fwd(_to_dev_bf16(x, cuda), _to_dev_bf16(w, cuda), 1, 1, stats=stats)
        dx = dtc.ops.conv2d_dgrad(_to_dev_bf16(dy, cuda), _to_dev_bf16(w, cuda), (H, W), 1, 1,
                                  res=_to_dev_bf16(res, cuda))
        torch.cuda.synchronize()
    finally:
        dtc._native.call("dtc_set_option", b"halo_conv", 1)
        dtc._native.call("dtc_set_option", b"halo_split", 0)
    yk = y.float().cpu().numpy()
    assert rel_err(yk, O.conv2d_fwd(x, w, 1, 1)) < 1e-2
    s = dtc.ops.stat_totals(stats, K).numpy()
    yb = yk.reshape(-1, K).astype(np.float64)
    np.testing.assert_allclose(s[0], yb.sum(0), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)
    ref = O.conv2d_dgrad(dy, w, (H, W), 1, 1) + res
    assert rel_err(dx.float().cpu().numpy(), ref) < 1e-2


@pytest.mark.parametrize("case,split", [((256, 4, 4, 512, 512), 0), ((256, 8, 8, 256, 256), 2),
                                        ((256, 8, 8, 256, 256), 4), ((37, 4, 4, 512, 256), 2)])
def test_conv_halo_splitk_in_kernel_matches_reduce_launch(dtc, cuda, case, split):
    """Option splitk_ink: the last workgroup of each output tile sums the split-K partials
    (sc1 write-through stores, an agent-scope arrival counter, sc1 loads) instead of a splitk_reduce launch.
    Same sum order (0 + slab[0] + slab[1] + ...), so the bf16 outputs are bit-identical to the separate
    reduction -- forward (+ BN statistics: the same values, their fp32 partial sums grouped per workgroup
    instead of per reduce block), data gradient (+ residual) and with the BN-backward pass after it -- on every one of 8 repeated
    launches (the hand-off under uneven arrival; the counters must come back to zero each time). B=256 layer4
    (automatic split 2), layer3 forced to 2 / 4 splits, a ragged batch."""
    N, H, W, C, K = case
    g = np.random.default_rng(77 + split)
    x = _to_dev_bf16(_rand_bf16((N, H, W, C), g), cuda)
    w = _to_dev_bf16(_rand_bf16((K, 3, 3, C), g, 0.05), cuda)
    dy = _to_dev_bf16(_rand_bf16((N, H, W, K), g), cuda)
    res = _to_dev_bf16(_rand_bf16((N, H, W, C), g), cuda)
    ym = _to_dev_bf16(_rand_bf16((N, H, W, C), g), cuda)
    x1 = _to_dev_bf16(_rand_bf16((N, H, W, C), g), cuda)
    mean1 = torch.randn(C, device=cuda) * 0.1
    inv1 = torch.rand(C, device=cuda) + 0.5
    lib = dtc._native.lib

    def run():
        stats = dtc.ops.new_stats(K, cuda)
        y = dtc.ops.conv2d_fwd(x, w, 1, 1, stats=stats)
        dx = dtc.ops.conv2d_dgrad(dy, w, (H, W), 1, 1, res=res)
        dz, acc1, _ = dtc.ops.conv2d_dgrad_bn(dy, w, (H, W), 1, 1, ym, x1, mean1, inv1, res=res)
        torch.cuda.synchronize()
        return y, stats, dx, dz, acc1

    prev = lib.dtc_get_option(b"splitk_ink")
    dtc._native.call("dtc_set_option", b"halo_split", split)
    try:
        dtc._native.call("dtc_set_option", b"splitk_ink", 0)
        ref = run()
        dtc._native.call("dtc_set_option", b"splitk_ink", 1)
        for _ in range(8):
            out = run()
            for a, b in ((out[0], ref[0]), (out[2], ref[2]), (out[3], ref[3])):
                assert torch.equal(a, b)
            for a, b, nc in ((out[1], ref[1], K), (out[4], ref[4], C)):  # the same values, fp32 partials regrouped
                a, b = dtc.ops.stat_totals(a, nc), dtc.ops.stat_totals(b, nc)  # (sums of products cancel: the bound scales with each row's magnitude)
                assert ((a - b).abs() <= 2e-5 * b.abs().amax(1, keepdim=True) + 1e-6).all(), (a - b).abs().max()
    finally:
        dtc._native.call("dtc_set_option", b"splitk_ink", prev)
        dtc._native.call("dtc_set_option", b"halo_split", 0)
    yk = ref[0].float().cpu().numpy()
    assert rel_err(yk, O.conv2d_fwd(x.float().cpu().numpy(), w.float().cpu().numpy(), 1, 1)) < 1e-2


GEN_CASES = [
    # (N, H, W, C, K): stride-1 3x3 shapes the classic whole-row halo tiles do not fit (option halo_gen)
    (2, 8, 224, 64, 64),     # 56-pixel row segments, 2 rows per 128-slot tile
    (2, 6, 112, 128, 64),    # 2 segments per row, C > K
    (3, 4, 56, 64, 128),     # one 56-pixel row segment per row
    (2, 8, 28, 128, 128),    # 4 rows of 28 per 128-slot tile
    (32, 8, 224, 64, 128),   # >= 512 tiles: the 64 x 256 configuration (4 rows of a segment)
]


@pytest.mark.parametrize("case", GEN_CASES)
def test_conv_halo_general_geometry(dtc, cuda, case):
    """conv_halo's general tile geometry (rows of 56- / 28-pixel segments, padded slots, 64-bit per-tile
    bases; the 224x224 model's layers): FWD (+BN statistics: padded slots must not count) and DGRAD
    (+residual) against the oracle, and against the implicit GEMM (option halo_gen=0) on the same operands."""
    N, H, W, C, K = case
    g = np.random.default_rng(41)
    x = _rand_bf16((N, H, W, C), g)
    w = _rand_bf16((K, 3, 3, C), g, 0.05)
    dy = _rand_bf16((N, H, W, K), g)
    res = _rand_bf16((N, H, W, C), g)
    xd, wd, dyd, rd = (_to_dev_bf16(a, cuda) for a in (x, w, dy, res))

    def run():
        stats = dtc.ops.new_stats(K, cuda)
        y = dtc.ops.conv2d_fwd(xd, wd, 1, 1, stats=stats)
        dx = dtc.ops.conv2d_dgrad(dyd, wd, (H, W), 1, 1, res=rd)
        torch.cuda.synchronize()
        return y.float().cpu().numpy(), dtc.ops.stat_totals(stats, K).numpy(), dx.float().cpu().numpy()

    yk, s, dxk = run()
    dtc._native.call("dtc_set_option", b"halo_gen", 0)
    try:
        yi, si, dxi = run()
    finally:
        dtc._native.call("dtc_set_option", b"halo_gen", 1)
    assert rel_err(yk, O.conv2d_fwd(x, w, 1, 1)) < 1e-2
    yb = yk.reshape(-1, K).astype(np.float64)
    np.testing.assert_allclose(s[0], yb.sum(0), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)
    assert rel_err(dxk, O.conv2d_dgrad(dy, w, (H, W), 1, 1) + res) < 1e-2
    assert rel_err(yk, yi) < 1e-2 and rel_err(dxk, dxi) < 1e-2


C64_CASES = [(2, 32, 32), (3, 16, 16), (5, 32, 32)]


@pytest.fixture
def c64_forced(dtc):
    """conv_c64=2: the persistent layer1 kernel even where its automatic rule (at least one 256-pixel tile per
    workgroup) would leave these small test batches to conv_halo."""
    prev = dtc._native.lib.dtc_get_option(b"conv_c64")
    dtc._native.call("dtc_set_option", b"conv_c64", 2)
    yield
    dtc._native.call("dtc_set_option", b"conv_c64", prev)


@pytest.mark.parametrize("case", C64_CASES)
def test_conv_c64(dtc, cuda, case, c64_forced):
    """Persistent 64->64 3x3 kernel (conv_c64.hip, layer1): FWD (+BN statistics accumulated per
    workgroup across tiles) and DGRAD (+residual), with more tiles than workgroups for case 3."""
    N, H, W = case
    g = np.random.default_rng(31)
    x = _rand_bf16((N, H, W, 64), g)
    w = _rand_bf16((64, 3, 3, 64), g, 0.05)
    dy = _rand_bf16((N, H, W, 64), g)
    res = _rand_bf16((N, H, W, 64), g)
    stats = dtc.ops.new_stats(64, cuda)
    y = dtc.ops.conv2d_fwd(_to_dev_bf16(x, cuda), _to_dev_bf16(w, cuda), 1, 1, stats=stats)
    dx = dtc.ops.conv2d_dgrad(_to_dev_bf16(dy, cuda), _to_dev_bf16(w, cuda), (H, W), 1, 1, res=_to_dev_bf16(res, cuda))
    yk = y.float().cpu().numpy()
    assert rel_err(yk, O.conv2d_fwd(x, w, 1, 1)) < 1e-2
    s = dtc.ops.stat_totals(stats, 64).numpy()
    yb = yk.reshape(-1, 64).astype(np.float64)
    np.testing.assert_allclose(s[0], yb.sum(0), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)
    assert rel_err(dx.float().cpu().numpy(), O.conv2d_dgrad(dy, w, (H, W), 1, 1) + res) < 1e-2


C64_GEN_CASES = [(2, 16, 224), (3, 8, 64), (2, 40, 96)]


@pytest.mark.parametrize("case", C64_GEN_CASES)
def test_conv_c64_general_geometry(dtc, cuda, case, c64_forced):
    """conv_c64's general geometry (8-row x 32-column tiles, 64-bit per-tile bases; rows of 224 / 64 / 96
    pixels that the classic whole-row tiles do not fit -- the 224x224 model's layer1): FWD (+BN statistics)
    and DGRAD (+residual) against the oracle, and against conv_halo (option c64_gen=0) on the same operands:
    the same nine taps x two k-steps per pixel in the same order, so the bf16 outputs are bit-identical."""
    N, H, W = case
    g = np.random.default_rng(33)
    x = _rand_bf16((N, H, W, 64), g)
    w = _rand_bf16((64, 3, 3, 64), g, 0.05)
    dy = _rand_bf16((N, H, W, 64), g)
    res = _rand_bf16((N, H, W, 64), g)
    xd, wd, dyd, rd = (_to_dev_bf16(a, cuda) for a in (x, w, dy, res))

    def run():
        stats = dtc.ops.new_stats(64, cuda)
        y = dtc.ops.conv2d_fwd(xd, wd, 1, 1, stats=stats)
        dx = dtc.ops.conv2d_dgrad(dyd, wd, (H, W), 1, 1, res=rd)
        dx0 = dtc.ops.conv2d_dgrad(dyd, wd, (H, W), 1, 1)
        torch.cuda.synchronize()
        return y.float().cpu().numpy(), dtc.ops.stat_totals(stats, 64).numpy(), dx.float().cpu().numpy(), dx0.float().cpu().numpy()

    yk, s, dxk, dx0k = run()
    dtc._native.call("dtc_set_option", b"c64_gen", 0)
    try:
        yh, sh, dxh, dx0h = run()
    finally:
        dtc._native.call("dtc_set_option", b"c64_gen", 1)
    assert rel_err(yk, O.conv2d_fwd(x, w, 1, 1)) < 1e-2
    yb = yk.reshape(-1, 64).astype(np.float64)
    np.testing.assert_allclose(s[0], yb.sum(0), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[1], (yb * yb).sum(0), rtol=1e-5, atol=1e-3)
    ref = O.conv2d_dgrad(dy, w, (H, W), 1, 1)
    assert rel_err(dxk, ref + res) < 1e-2 and rel_err(dx0k, ref) < 1e-2
    np.testing.assert_array_equal(yk, yh)
    np.testing.assert_array_equal(dx0k, dx0h)
    assert rel_err(dxk, dxh) < 1e-2  # + residual: conv_halo rounds the same sum (fp32 order may differ)


def test_conv_c64_large_grid(dtc, cuda):
    """More tiles than resident workgroups (1024 tiles / 256 workgroups at the bench shape's
    layer1 geometry, batch 64 here): every tile of every workgroup's walk is computed, against
    the implicit-GEMM kernel on the same operands (option conv_c64=0)."""
    g = np.random.default_rng(32)
    x = torch.from_numpy(_rand_bf16((300, 32, 32, 64), g)).to(cuda).bfloat16()
    w = torch.from_numpy(_rand_bf16((64, 3, 3, 64), g, 0.05)).to(cuda).bfloat16()
    y1 = dtc.ops.conv2d_fwd(x, w, 1, 1)
    d1 = dtc.ops.conv2d_dgrad(x, w, (32, 32), 1, 1)
    dtc._native.call("dtc_set_option", b"conv_c64", 0)
    dtc._native.call("dtc_set_option", b"halo_conv", 0)
    try:
        y0 = dtc.ops.conv2d_fwd(x, w, 1, 1)
        d0 = dtc.ops.conv2d_dgrad(x, w, (32, 32), 1, 1)
    finally:
        dtc._native.call("dtc_set_option", b"conv_c64", 1)
        dtc._native.call("dtc_set_option", b"halo_conv", 1)
    torch.cuda.synchronize()
    assert rel_err(y1.float().cpu().numpy(), y0.float().cpu().numpy()) < 1e-2
    assert rel_err(d1.float().cpu().numpy(), d0.float().cpu().numpy()) < 1e-2


BNB_CASES = [
    # (N, H, W, C, K, R, stride, res, dual): dgrad output [N,H,W,C] feeding a BN backward
    (3, 32, 32, 64, 64, 3, 1, False, False),   # conv_c64 mode 3
    (3, 32, 32, 64, 64, 3, 1, True, False),    # conv_c64 mode 4 (in place on the residual)
    (2, 16, 16, 128, 128, 3, 1, True, True),   # conv_halo, second BN (projection shortcut)
    (5, 8, 8, 256, 256, 3, 1, True, False),    # conv_halo
    (9, 4, 4, 512, 512, 3, 1, True, True),     # layer4 geometry (split-K reduce or implicit GEMM)
    (4, 16, 16, 64, 128, 3, 2, True, True),    # stride-2 parity classes: separate reduction pass
    (2, 8, 224, 64, 64, 3, 1, True, False),    # conv_c64 general geometry (224-wide rows), mode 4
    (2, 8, 96, 64, 64, 3, 1, False, False),    # conv_c64 general geometry, mode 3
]


@pytest.mark.parametrize("split", [0, 2])
@pytest.mark.parametrize("case", BNB_CASES)
def test_conv_dgrad_bn_fused(dtc, cuda, case, split):
    """dtc_conv2d_dgrad_bn (BN-backward reduction in the dgrad epilogue) against the unfused pair
    dtc_conv2d_dgrad -> dtc_bn_bwd_reduce on the same operands: dz bit-exact (both round the same
    fp32 accumulator to bf16 and mask it), the fp64 sums equal up to summation order."""
    N, H, W, C, K, R, st, with_res, dual = case
    pad = 1
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    g = np.random.default_rng(41)
    b = lambda a: _to_dev_bf16(a, cuda)
    t = lambda a: torch.from_numpy(np.asarray(a, np.float32)).to(cuda)
    dy = b(_rand_bf16((N, P, Q, K), g))
    w = b(_rand_bf16((K, R, R, C), g, 0.05))
    res = _rand_bf16((N, H, W, C), g) if with_res else None
    ym = b(_rand_bf16((N, H, W, C), g))
    x1n = O.bf16(_rand_bf16((N, H, W, C), g, 1.5) + 0.3)
    x2n = O.bf16(_rand_bf16((N, H, W, C), g, 0.7) - 0.1)
    _, m1, i1, _, _ = O.bn_train_fwd(x1n.reshape(-1, C), np.ones(C, np.float32), np.zeros(C))
    _, m2, i2, _, _ = O.bn_train_fwd(x2n.reshape(-1, C), np.ones(C, np.float32), np.zeros(C))
    x1, x2 = b(x1n), b(x2n) if dual else None
    mean2, inv2 = (t(m2), t(i2)) if dual else (None, None)
    dtc._native.call("dtc_set_option", b"halo_split", split)
    try:
        dx = dtc.ops.conv2d_dgrad(dy, w, (H, W), st, pad, res=b(res) if with_res else None)
        dz0, a10, a20 = dtc.ops.bn_bwd_reduce(dx, ym, x1, t(m1), t(i1), x2, mean2, inv2)
        resd = b(res) if with_res else None
        dz1, a11, a21 = dtc.ops.conv2d_dgrad_bn(dy, w, (H, W), st, pad, ym, x1, t(m1), t(i1), x2, mean2, inv2,
                                                res=resd, out=resd)
        torch.cuda.synchronize()
    finally:
        dtc._native.call("dtc_set_option", b"halo_split", 0)
    np.testing.assert_array_equal(dz1.float().cpu().numpy(), dz0.float().cpu().numpy())
    if with_res:
        assert dz1.data_ptr() == resd.data_ptr()
    for a1, a0 in [(a11, a10)] + ([(a21, a20)] if dual else []):
        s1, s0 = dtc.ops.stat_totals(a1, C).numpy(), dtc.ops.stat_totals(a0, C).numpy()
        np.testing.assert_allclose(s1, s0, rtol=1e-5, atol=1e-3 * np.abs(s0).max())


S2D_CASES = [(256, 32, 32, 64, 128), (256, 16, 16, 128, 256), (256, 8, 8, 256, 512), (8, 32, 32, 64, 128),
             (3, 16, 16, 128, 256), (5, 8, 8, 256, 512), (2, 8, 8, 64, 128), (64, 16, 16, 64, 128)]


@pytest.mark.parametrize("case", S2D_CASES)
@pytest.mark.parametrize("sc", [True, False])
def test_conv_dgrad_stride2_halo_subpixel(dtc, cuda, case, sc):
    """Option dgrad_s2h (dgrad_s2.hip): the stride-2 3x3 data gradient as a halo-tiled
    sub-pixel convolution (nine (dy offset, parity class, tap) steps over one dy halo per 64-channel chunk),
    with the 1x1 stride-2 shortcut's dgrad fused as a tenth step of class (0, 0) -- ResNet-18's three
    projection blocks at B=256 (128- / 64-position tiles, multi-image tiles), small and ragged batches (the
    last tile past the tensor) -- against the oracle, and against the implicit-GEMM parity classes
    (dgrad_s2h=0) on the same operands (same products, other summation order: 1e-2)."""
    N, H, W, C, K = case
    lib = dtc._native.lib
    g = np.random.default_rng(31 + N)
    dy = _rand_bf16((N, H // 2, W // 2, K), g)
    dsc = _rand_bf16((N, H // 2, W // 2, K), g)
    w = _rand_bf16((K, 3, 3, C), g, 0.05)
    wsc = _rand_bf16((K, 1, 1, C), g, 0.1)
    dyd, dscd, wd, wscd = (_to_dev_bf16(a, cuda) for a in (dy, dsc, w, wsc.reshape(K, C)))

    def run():
        if sc:
            return dtc.ops.conv2d_dgrad_sc(dyd, wd, dscd, wscd, (H, W))
        return dtc.ops.conv2d_dgrad(dyd, wd, (H, W), 2, 1)

    prev = lib.dtc_get_option(b"dgrad_s2h")
    try:
        lib.dtc_set_option(b"dgrad_s2h", 2)  # every geometry (the default 1 leaves K = 512 to the classes)
        dx = run().float()
        lib.dtc_set_option(b"dgrad_s2h", 0)
        dx_gemm = run().float()
        torch.cuda.synchronize()
    finally:
        lib.dtc_set_option(b"dgrad_s2h", prev)
    ref = O.conv2d_dgrad(dy, w, (H, W), 2, 1)
    if sc:
        ref = ref + O.conv2d_dgrad(dsc, wsc, (H, W), 2, 0)
    got = dx.cpu().numpy()
    assert rel_err(got, ref) < 1e-2
    assert rel_err(got, dx_gemm.cpu().numpy()) < 1e-2
    assert np.isfinite(got).all()


@pytest.mark.parametrize("case", [(4, 32, 32, 64, 64), (12, 4, 4, 512, 512), (8, 16, 16, 128, 128),
                                  (2, 14, 224, 64, 64), (3, 8, 8, 64, 128)])
def test_conv_wgrad_halo_trim_bit_identical(dtc, cuda, case):
    """Option wgrad_trim (round 6, default on): a wave whose rows of the last halo DMA round lie past the step's
    halo issues no zero-filling DMA for them (those LDS rows are never read) and waits on one instruction fewer
    per stage. The same products in the same order: the weight gradient must be bit-identical to the untrimmed
    kernel's (layer1's 136-row halos, layer4's four-image 144-row halos, the general geometry), and match the
    oracle."""
    N, H, W, C, K = case
    g = np.random.default_rng(21 + N)
    x = _rand_bf16((N, H, W, C), g)
    dy = _rand_bf16((N, H, W, K), g)
    xd, dyd = _to_dev_bf16(x, cuda), _to_dev_bf16(dy, cuda)
    lib = dtc._native.lib
    prev = lib.dtc_get_option(b"wgrad_trim")
    try:
        lib.dtc_set_option(b"wgrad_trim", 0)
        a = dtc.ops.conv2d_wgrad(xd, dyd, 3, 3, 1, 1).cpu().numpy()
        lib.dtc_set_option(b"wgrad_trim", 1)
        b = dtc.ops.conv2d_wgrad(xd, dyd, 3, 3, 1, 1).cpu().numpy()
    finally:
        lib.dtc_set_option(b"wgrad_trim", prev)
    np.testing.assert_array_equal(a, b)
    assert rel_err(b, O.conv2d_wgrad(x, dy, 3, 3, 1, 1)) < 1e-5
