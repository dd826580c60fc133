"""Whole-network parity of the native executor against the numpy oracle.

Per-layer ("teacher-forced") checks — the north_star criterion "per-layer activations and
gradients within 1e-2 relative (bf16)": every layer's oracle evaluation takes THAT LAYER'S INPUTS
from the executor (forward activations, and backward intermediates kept by a capture-enabled
executor), so each comparison isolates one layer. bf16-valued outputs: 1e-2; fp32 parameter
gradients computed from identical bf16 operands: 1e-4 (summation order only).

End-to-end checks compare free-running forward/backward. Two CORRECT bf16 implementations drift
apart with depth: the oracle run twice with fp32 vs fp64 conv accumulation differs by 1.8% at
layer4 and 0.6% on logits (batch 2), and by 21% on the concatenated parameter gradient (batch 2
and 8 alike; the stem/layer1 weight gradients of a freshly initialised BN network are dominated
by amplified rounding noise). The free-running bounds below are set from those measurements.
"""
import numpy as np
import pytest
import torch

from oracle import ops as O
from oracle import resnet as R
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu

BF = 1e-2     # bf16-valued tensors, teacher-forced
F32 = 1e-4    # fp32 gradients from identical bf16 operands


@pytest.fixture(autouse=True)
def _autocast_bf16(dtc):
    """Every test here is about the AMP (bf16) executor: run it with autocast on, as the reference's
    --amp loop does (trainer.py:153). The fp32 executor has its own tests (test_gpu_fp32.py)."""
    prev = dtc.nn.is_autocast_enabled()
    dtc.nn.set_autocast_enabled(True)
    yield
    dtc.nn.set_autocast_enabled(prev)


def _setup(dtc, cuda, batch, seed=0, capture=False, hw=32):
    torch.manual_seed(42)
    model = dtc.ResNet18()
    sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    model = model.to(cuda)
    if capture:
        model.enable_capture()
    g = np.random.default_rng(seed)
    x = g.standard_normal((batch, 3, hw, hw)).astype(np.float32)
    y = g.integers(0, 100, batch)
    return model, sd, x, y


def _split_state(sd):
    params = {k: v for k, v in sd.items() if not (k.endswith("running_mean") or k.endswith("running_var")
                                                  or k.endswith("num_batches_tracked"))}
    bufs = {k: v for k, v in sd.items() if k.endswith("running_mean") or k.endswith("running_var")}
    return params, bufs


def _np(t):
    return t.detach().float().cpu().numpy()


def _f32(a):
    return np.asarray(a, np.float32)


def _bn_fwd(x, g, b, rnd=O.bf16):
    """Oracle BN (train) on an NHWC tensor -> output rounded like the executor's (bf16 under
    autocast, fp32 otherwise), mean, invstd."""
    C = x.shape[-1]
    y, mean, invstd, _, _ = O.bn_train_fwd(x.reshape(-1, C), g, b)
    return rnd(y.reshape(x.shape)), mean, invstd


def _bn_bwd(dz, x, g, rnd=O.bf16):
    C = x.shape[-1]
    _, mean, invstd, _, _ = O.bn_train_fwd(x.reshape(-1, C), g, np.zeros(C))
    dx, dg, db = O.bn_train_bwd(dz.reshape(-1, C), x.reshape(-1, C), g, mean, invstd)
    return rnd(dx.reshape(x.shape)), dg, db


def _teacher_forced(dtc, cuda, batch, hw=32, stages=(0, 1, 2, 3, 4), imgs=None, seed=0, precision="bf16"):
    """Run one capture-enabled training forward/backward of the executor at (batch, hw x hw) and
    check every layer of the listed stages (0 = stem + head, 1..4 = layer1..4) against the oracle
    evaluated on THAT layer's executor inputs. `imgs` (index array) restricts the per-image ops
    (conv forward / dgrad, the ReLU masks) to those images -- BN statistics and weight gradients,
    which reduce over the whole batch, are always checked at full size, so every batch-dependent
    kernel plan (split-K factors, wgrad splits, persistent-tile walks) is the one under test.
    precision "bf16": the AMP executor at the north_star's 1e-2 (bf16 outputs; fp32 weight gradients
    from identical bf16 operands 1e-4); "fp32": the non-AMP executor at the north_star's 1e-5
    everywhere, against the fp32 (unrounded) oracle."""
    model, sd, x, y = _setup(dtc, cuda, batch, seed=seed, capture=True, hw=hw)
    model.precision = precision
    bf = precision == "bf16"
    rnd = O.bf16 if bf else _f32
    crit = dtc.CrossEntropyLoss()
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    logits = model(xd)
    loss = crit(logits, yd)
    loss.backward()
    torch.cuda.synchronize()
    exe = model.executor(batch, hw, hw, precision)
    A = {k: _np(v) for k, v in exe.activations().items()}
    G = {k: _np(v) for k, v in exe.activations(captures=True).items()}
    P = {k: v for k, v in _split_state(sd)[0].items()}
    W = {k: rnd(O.kcrs_to_krsc(v)) for k, v in P.items() if v.ndim == 4}
    grads = {k: _np(p.grad) for k, p in model.named_parameters()}
    del model, exe
    torch.cuda.empty_cache()
    sel = slice(None) if imgs is None else np.asarray(imgs)
    errs = {}

    def chk(name, got, ref, tol=BF):
        errs[name] = (rel_err(got, ref), tol if bf else 1e-5)  # fp32 mode: 1e-5 for everything

    def conv_f(inp, w, st, pad):
        return O.conv2d_fwd(inp[sel], w, st, pad)

    def conv_d(dy, w, shape_hw, st, pad):
        return O.conv2d_dgrad(dy[sel], w, shape_hw, st, pad)

    # ---------------- forward, layer by layer
    xb = rnd(O.nchw_to_nhwc(x))
    if 0 in stages:
        chk("stem.conv", A["stem.conv"][sel], conv_f(xb, W["conv1.weight"], 1, 1))
        a0, _, _ = _bn_fwd(A["stem.conv"], P["bn1.weight"], P["bn1.bias"], rnd)
        chk("stem.out", A["stem.out"], O.relu(a0))
    inp = A["stem.out"]
    blocks = []
    for L in range(1, 5):
        for bi in range(2):
            pre = f"layer{L}.{bi}"
            st = 2 if (L > 1 and bi == 0) else 1
            proj = f"{pre}.shortcut.0.weight" in P
            blocks.append((L, pre, st, proj, inp))
            if L in stages:
                chk(pre + ".conv1", A[pre + ".conv1"][sel], conv_f(inp, W[pre + ".conv1.weight"], st, 1))
                z1, _, _ = _bn_fwd(A[pre + ".conv1"], P[pre + ".bn1.weight"], P[pre + ".bn1.bias"], rnd)
                chk(pre + ".relu1", A[pre + ".relu1"], O.relu(z1))
                chk(pre + ".conv2", A[pre + ".conv2"][sel], conv_f(A[pre + ".relu1"], W[pre + ".conv2.weight"], 1, 1))
                z2, _, _ = _bn_fwd(A[pre + ".conv2"], P[pre + ".bn2.weight"], P[pre + ".bn2.bias"], rnd)
                if proj:
                    chk(pre + ".shortcut", A[pre + ".shortcut"][sel], conv_f(inp, W[pre + ".shortcut.0.weight"], st, 0))
                    zs, _, _ = _bn_fwd(A[pre + ".shortcut"], P[pre + ".shortcut.1.weight"],
                                       P[pre + ".shortcut.1.bias"], rnd)
                    chk(pre + ".out", A[pre + ".out"], O.relu(z2 + zs))
                else:
                    chk(pre + ".out", A[pre + ".out"], O.relu(z2 + inp))
            inp = A[pre + ".out"]
    feat, lg = O.head_fwd(inp, P["linear.weight"], P["linear.bias"], bf16_mode=bf)
    if 0 in stages:
        chk("head.feat", A["head.feat_f32"].reshape(feat.shape), feat, 1e-5)
        chk("logits", _np(logits), lg)

    # ---------------- backward, layer by layer (inputs = the executor's own intermediates)
    _, dl, _ = O.cross_entropy(_np(logits), y)
    if 0 in stages:
        dw, db, dact = O.head_bwd(dl, A["head.feat_f32"].reshape(feat.shape), rnd(P["linear.weight"]),
                                  inp.shape[1:3])
        chk("linear.weight.grad", grads["linear.weight"], dw, F32)
        chk("linear.bias.grad", grads["linear.bias"], db, F32)
        chk("grad.layer4.1.dy", G["grad.layer4.1.dy"], dact)
    for L, pre, st, proj, inp in reversed(blocks):
        if L not in stages:
            continue
        gp = "grad." + pre
        np.testing.assert_array_equal(G[gp + ".dz"][sel], np.where(A[pre + ".out"] > 0, G[gp + ".dy"], 0)[sel])
        dc2, dg2, db2 = _bn_bwd(G[gp + ".dz"], A[pre + ".conv2"], P[pre + ".bn2.weight"], rnd)
        chk(gp + ".dc2", G[gp + ".dc2"], dc2)
        chk(pre + ".bn2.weight.grad", grads[pre + ".bn2.weight"], dg2, 1e-3)
        chk(pre + ".bn2.bias.grad", grads[pre + ".bn2.bias"], db2, 1e-3)
        chk(pre + ".conv2.weight.grad", O.kcrs_to_krsc(grads[pre + ".conv2.weight"]),
            O.conv2d_wgrad(A[pre + ".relu1"], G[gp + ".dc2"], 3, 3, 1, 1), F32)
        chk(gp + ".da1", G[gp + ".da1"][sel], conv_d(G[gp + ".dc2"], W[pre + ".conv2.weight"],
                                                     A[pre + ".relu1"].shape[1:3], 1, 1))
        np.testing.assert_array_equal(G[gp + ".dz1"][sel], np.where(A[pre + ".relu1"] > 0, G[gp + ".da1"], 0)[sel])
        dc1, dg1, db1 = _bn_bwd(G[gp + ".dz1"], A[pre + ".conv1"], P[pre + ".bn1.weight"], rnd)
        chk(gp + ".dc1", G[gp + ".dc1"], dc1)
        chk(pre + ".bn1.weight.grad", grads[pre + ".bn1.weight"], dg1, 1e-3)
        chk(pre + ".conv1.weight.grad", O.kcrs_to_krsc(grads[pre + ".conv1.weight"]),
            O.conv2d_wgrad(inp, G[gp + ".dc1"], 3, 3, st, 1), F32)
        dx = conv_d(G[gp + ".dc1"], W[pre + ".conv1.weight"], inp.shape[1:3], st, 1)
        if proj:
            ds, dgs, dbs = _bn_bwd(G[gp + ".dz"], A[pre + ".shortcut"], P[pre + ".shortcut.1.weight"], rnd)
            chk(gp + ".ds", G[gp + ".ds"], ds)
            chk(pre + ".shortcut.1.weight.grad", grads[pre + ".shortcut.1.weight"], dgs, 1e-3)
            chk(pre + ".shortcut.0.weight.grad", O.kcrs_to_krsc(grads[pre + ".shortcut.0.weight"]),
                O.conv2d_wgrad(inp, G[gp + ".ds"], 1, 1, st, 0), F32)
            chk(gp + ".dxs", G[gp + ".dxs"][sel], conv_d(G[gp + ".ds"], W[pre + ".shortcut.0.weight"],
                                                         inp.shape[1:3], st, 0))
            chk(gp + ".dx", G[gp + ".dx"][sel], dx + G[gp + ".dxs"][sel])
        else:
            chk(gp + ".dx", G[gp + ".dx"][sel], dx + G[gp + ".dz"][sel])
    if 0 in stages:
        np.testing.assert_array_equal(G["grad.stem.dz"], np.where(A["stem.out"] > 0, G["grad.layer1.0.dx"], 0))
        dc0, dg0, db0 = _bn_bwd(G["grad.stem.dz"], A["stem.conv"], P["bn1.weight"], rnd)
        chk("grad.stem.dc", G["grad.stem.dc"], dc0)
        chk("bn1.weight.grad", grads["bn1.weight"], dg0, 1e-3)
        chk("conv1.weight.grad", O.kcrs_to_krsc(grads["conv1.weight"]),
            O.conv2d_wgrad(xb, G["grad.stem.dc"], 3, 3, 1, 1), F32)
    bad = {k: v for k, v in errs.items() if v[0] > v[1]}
    worst = max(errs.items(), key=lambda kv: kv[1][0] / kv[1][1])
    print(f"teacher-forced {precision} B={batch} {hw}x{hw} stages={stages}: {len(errs)} checks, worst {worst[0]} "
          f"{worst[1][0]:.2e} (tol {worst[1][1]:.0e})")
    assert not bad, f"per-layer parity failures: {bad}"
    return errs


@pytest.mark.parametrize("batch", [2, 8])
def test_per_layer_teacher_forced(dtc, cuda, batch):
    errs = _teacher_forced(dtc, cuda, batch)
    assert len(errs) > 90


# BASELINE config 2 at its own size (B=256, 32x32): the launches bench.py times -- conv_c64's
# multi-tile persistent walk, the batched wgrad_halo split plan on layer1, the halo layer2 tiles, split-K
# layer3/4 fwd/dgrad/wgrad, the stride-2 parity classes -- against the oracle. Split by stage so each
# test's numpy work stays well inside the per-test time limit; conv forward / dgrad compared on a
# sample of 24 images spread over the batch (first, last, tile boundaries), everything that reduces
# over the batch (BN, weight gradients) on all 256.
_B256_IMGS = np.unique(np.concatenate([np.arange(4), np.arange(60, 68), np.arange(124, 132), np.arange(252, 256)]))


@pytest.mark.parametrize("stages", [(0, 1), (2,), (3, 4)])
def test_per_layer_teacher_forced_config2_b256(dtc, cuda, stages):
    errs = _teacher_forced(dtc, cuda, 256, stages=stages, imgs=_B256_IMGS, seed=21)
    assert len(errs) >= 20


# BASELINE config 3's per-rank shapes: global batch 256 over W = 2 / 4 / 8 ranks (ddp/trainer.py:34) gives
# 128 / 64 / 32 images per GPU, where the tile plans, split-K factors and wgrad splits differ from B = 256
# (small-GEMM regime: layer4 at B=32 is 512 x 512 x 4608, SURVEY §7 iii). Default options, every stage
# (the stem and layer1 included: conv_c64's tile walk at 64 / 128 images; at 32 layer1 takes conv_halo).
@pytest.mark.parametrize("batch", [32, 64, 128])
def test_per_layer_teacher_forced_config3_per_rank(dtc, cuda, batch):
    imgs = None if batch <= 32 else np.unique(np.concatenate([np.arange(4), np.arange(28, 36), np.arange(batch - 4, batch)]))
    errs = _teacher_forced(dtc, cuda, batch, imgs=imgs, seed=23 + batch)
    assert len(errs) > 90


@pytest.mark.parametrize("batch,stages", [(8, (0, 1, 2, 3, 4)), (64, (2, 3, 4))])
@pytest.mark.parametrize("opts", [{"halo_s2": 1}, {"wgrad_s2": 1}, {"halo_s2": 2, "wgrad_s2": 1}, {"dgrad_scf": 1}])
def test_per_layer_teacher_forced_halo_s2(dtc, cuda, batch, stages, opts):
    """The stride-2 convs on the column-split halo kernels with the shortcut fused (options halo_s2:
    forward, wgrad_s2: weight gradients; halo_s2=2 forces the halo forward on layer2.0.conv1 too):
    every layer against the oracle."""
    lib = dtc._native.lib
    prev = {k: lib.dtc_get_option(k.encode()) for k in opts}
    try:
        for k, v in opts.items():
            lib.dtc_set_option(k.encode(), v)
        errs = _teacher_forced(dtc, cuda, batch, stages=stages, seed=31)
    finally:
        for k, v in prev.items():
            lib.dtc_set_option(k.encode(), v)
    assert len(errs) >= 20


def test_per_layer_teacher_forced_224(dtc, cuda):
    """BASELINE config 5's geometry (224x224, global pool; SURVEY §7 viii) at batch 2: every layer,
    through the 64-bit-addressed implicit-GEMM path the 224x224 shapes take."""
    errs = _teacher_forced(dtc, cuda, 2, hw=224, seed=22)
    assert len(errs) > 90


def test_config5_b512_224_step_properties(dtc, cuda):
    """BASELINE config 5 at its full per-GPU size: batch 512 at 224x224 (activations > 2 GiB: the
    largest is 512x224x224x64 bf16 = 3.3 GB). One AMP training step + SGD step must run and give a
    finite loss near ln(100) for a fresh network, finite non-zero gradients in every parameter,
    running statistics that moved, and a second step whose loss is finite too."""
    torch.manual_seed(42)
    model = dtc.ResNet18().to(cuda)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    scaler = dtc.GradScaler()
    g = torch.Generator(device=cuda).manual_seed(9)
    x = torch.randn(512, 3, 224, 224, device=cuda, generator=g)
    y = torch.randint(0, 100, (512,), device=cuda, generator=g)
    rm0 = model.flat.bufs.clone()
    losses = []
    for _ in range(2):
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(model(x), y)
        scaler.scale(loss).backward()
        if not losses:
            gr = model.flat.grads.clone()
        scaler.step(opt)
        scaler.update()
        losses.append(float(loss))
    torch.cuda.synchronize()
    assert np.isfinite(losses).all() and 3.0 < losses[0] < 8.0, losses
    assert bool(torch.isfinite(gr).all())  # the first step's (loss-scaled) gradients
    lay = model.flat.layout
    grn = gr.cpu().numpy()
    for p in lay.params:
        assert np.abs(grn[p.offset:p.offset + p.numel]).sum() > 0, p.name
    assert float((model.flat.bufs - rm0).abs().sum()) > 0
    assert int(model.state_dict()["bn1.num_batches_tracked"]) == 2


@pytest.mark.parametrize("batch", [2, 8])
def test_end_to_end_drift_bounded(dtc, cuda, batch):
    """Free-running forward/backward vs the oracle. Bounds: logits/loss 3e-2 / 1e-2, every
    activation 5e-2, concatenated gradient 0.35 (oracle-vs-oracle: 1.8%, 0.6%, 21%)."""
    model, sd, x, y = _setup(dtc, cuda, batch)
    crit = dtc.CrossEntropyLoss()
    logits = model(torch.from_numpy(x).to(cuda))
    loss = crit(logits, torch.from_numpy(y).to(cuda))
    loss.backward()
    torch.cuda.synchronize()
    params, bufs = _split_state(sd)
    ref = R.forward_backward(params, bufs, x, y, bf16_mode=True, train=True, want_acts=True)
    assert rel_err(_np(logits), ref["logits"]) < 3e-2
    assert abs(float(loss) - ref["loss"]) < 1e-2 * max(1.0, abs(ref["loss"]))
    acts = model.executor(batch, 32, 32).activations()
    worst = max(rel_err(_np(acts[k]).reshape(v.shape), v) for k, v in ref["acts"].items())
    assert worst < 5e-2
    g_exe = np.concatenate([_np(p.grad).ravel() for _, p in model.named_parameters()])
    g_ref = np.concatenate([ref["grads"][k].ravel() for k, _ in model.named_parameters()])
    assert rel_err(g_exe, g_ref) < 0.35
    # only the head gradients sit above the rounding-noise floor (oracle-vs-oracle: linear.weight
    # 0.6%, linear.bias 0.03%, but layer4.1.conv2.weight already 13-14%): hold those to 2e-2
    for k in ("linear.weight", "linear.bias"):
        assert rel_err(_np(dict(model.named_parameters())[k].grad), ref["grads"][k]) < 2e-2, k
    sd2 = model.state_dict()
    for k, v in ref["buffers"].items():  # running statistics after one training forward
        assert rel_err(sd2[k].cpu().numpy(), v) < 2e-2, k
    assert int(sd2["bn1.num_batches_tracked"]) == 1


def test_eval_mode_matches_oracle(dtc, cuda):
    model, sd, x, y = _setup(dtc, cuda, 4, seed=1)
    g = np.random.default_rng(2)
    with torch.no_grad():
        for name, buf in model.named_buffers():
            if name.endswith("running_mean"):
                buf.copy_(torch.from_numpy(g.standard_normal(buf.shape).astype(np.float32) * 0.1))
            elif name.endswith("running_var"):
                buf.copy_(torch.from_numpy(g.uniform(0.5, 2.0, buf.shape).astype(np.float32)))
    sd = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    model.eval()
    with torch.no_grad():
        logits = model(torch.from_numpy(x).to(cuda))
    params, bufs = _split_state(sd)
    ref = R.forward_backward(params, bufs, x, y, bf16_mode=True, train=False)
    assert rel_err(_np(logits), ref["logits"]) < 3e-2
    sd2 = model.state_dict()
    for k in bufs:  # eval never touches the running statistics
        np.testing.assert_array_equal(sd2[k].cpu().numpy(), sd[k])


def test_sgd_step_in_situ(dtc, cuda):
    """After a real backward, the fused step equals torch.optim.SGD(nesterov) math on the
    executor's own gradients (oracle.ops.sgd_nesterov), two consecutive steps."""
    model, sd, x, y = _setup(dtc, cuda, 4, seed=3)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    bufs = {}
    for step in range(2):
        opt.zero_grad()
        crit(model(xd), yd).backward()
        before = {k: _np(p) for k, p in model.named_parameters()}
        grads = {k: _np(p.grad) for k, p in model.named_parameters()}
        opt.step()
        for k, p in model.named_parameters():
            ref, bufs[k] = O.sgd_nesterov(before[k], grads[k], bufs.get(k), 0.1, 1e-4, 0.9, step == 0)
            np.testing.assert_allclose(_np(p), ref, rtol=1e-6, atol=1e-6, err_msg=k)
    flat = model.flat
    np.testing.assert_array_equal(_np(flat.params_bf16), _np(flat.params.bfloat16()))


def _train_steps(dtc, cuda, steps, graphs, batch=8, seed=5):
    _graphs_prev = dtc._native.lib.dtc_get_option(b"graphs")
    dtc._native.lib.dtc_set_option(b"graphs", int(graphs))
    try:
        model, _, x, y = _setup(dtc, cuda, batch, seed=seed)
        crit = dtc.CrossEntropyLoss()
        opt = dtc.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
        xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
        losses, grads = [], None
        for _ in range(steps):
            opt.zero_grad()
            loss = crit(model(xd), yd)
            loss.backward()
            grads = _np(model.flat.grads)
            opt.step()
            losses.append(float(loss))
        return np.array(losses), grads, _np(model.flat.params), {k: _np(v) for k, v in model.named_buffers()}
    finally:
        dtc._native.lib.dtc_set_option(b"graphs", _graphs_prev)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_graph_replay_matches_eager(dtc, cuda, mode):
    """hipGraph replay (option graphs: 1 forward and backward, 2 forward only, 3 backward only) vs eager
    launches of the same step: identical kernels and arguments, and a deterministic step (exact BN sums,
    fixed split-K orders), so three training steps give identical losses, gradients, parameters and
    running statistics."""
    lg, gg, pg, bg = _train_steps(dtc, cuda, 3, graphs=mode)
    le, ge, pe, be = _train_steps(dtc, cuda, 3, graphs=False)
    np.testing.assert_array_equal(lg, le)
    np.testing.assert_array_equal(gg, ge)
    np.testing.assert_array_equal(pg, pe)
    for k in bg:
        np.testing.assert_array_equal(bg[k], be[k], err_msg=k)


@pytest.mark.parametrize("graphs", [True, False])
def test_side_stream_wgrad_matches_serial(dtc, cuda, graphs):
    """Weight gradients on the side stream (option bwd_streams=1, the default), forked/joined by
    events inside the (captured) backward, vs everything on one stream: the same kernels on the
    same operands in a deterministic step, so three training steps give identical results."""
    la, ga, pa, _ = _train_steps(dtc, cuda, 3, graphs=graphs)
    dtc._native.lib.dtc_set_option(b"bwd_streams", 0)
    try:
        lb, gb, pb, _ = _train_steps(dtc, cuda, 3, graphs=graphs)
    finally:
        dtc._native.lib.dtc_set_option(b"bwd_streams", 1)
    np.testing.assert_array_equal(la, lb)
    np.testing.assert_array_equal(ga, gb)
    np.testing.assert_array_equal(pa, pb)


@pytest.mark.parametrize("graphs", [True, False])
def test_fused_bn_finalize_matches_separate(dtc, cuda, graphs):
    """BN coefficients computed inside the apply kernels (option bn_fused_fin=1, default) vs the
    separate finalize launches: the same exact slot totals and the same coefficient expressions, but the
    separate path's BN-backward reduction stores dz and groups its partials per its own grid, so losses,
    gradients, parameters and running statistics agree to rounding. The projection shortcut's
    dgrad is computed separately in both arms (dgrad_scf=0): the fused-finalize executor would otherwise
    fold it into conv1's class-(0, 0) dgrad as one fp32 sum (one bf16 rounding of dx instead of two), a
    legitimate 1-ulp difference that 3 steps at lr 0.1 on 8 images amplify past rtol 1e-4. For the same
    reason both arms use the two-pass BN backward (bn_cg=0: the one-launch kernel, which needs the fused
    finalize, groups the sums differently; see test_bn_one_launch_matches_two_pass)."""
    lib = dtc._native.lib
    lib.dtc_set_option(b"dgrad_scf", 0)
    lib.dtc_set_option(b"bn_cg", 0)
    lib.dtc_set_option(b"wgrad_s2", 0)  # (the older executor has no fused conv1 + shortcut weight gradient)
    try:
        la, ga, pa, ba = _train_steps(dtc, cuda, 3, graphs=graphs)
        lib.dtc_set_option(b"bn_fused_fin", 0)
        try:
            lb, gb, pb, bb = _train_steps(dtc, cuda, 3, graphs=graphs)
        finally:
            lib.dtc_set_option(b"bn_fused_fin", 1)
    finally:
        lib.dtc_set_option(b"dgrad_scf", 1)
        lib.dtc_set_option(b"bn_cg", 1)
        lib.dtc_set_option(b"wgrad_s2", 1)
    np.testing.assert_allclose(la, lb, rtol=1e-4)
    assert rel_err(ga, gb) < 1e-3
    assert rel_err(pa, pb) < 1e-5
    for k in ba:
        assert rel_err(ba[k], bb[k]) < 1e-4, k


DEFAULT_STEM_BN_FUSE = 1
DEFAULT_SC_FUSE = 1
DEFAULT_STEM_WLDS = 1


def _grads_repeated(dtc, cuda, graphs, reps=2, batch=8, seed=5, hw=32):
    _graphs_prev = dtc._native.lib.dtc_get_option(b"graphs")
    dtc._native.lib.dtc_set_option(b"graphs", int(graphs))
    try:
        model, _, x, y = _setup(dtc, cuda, batch, seed=seed, hw=hw)
        crit = dtc.CrossEntropyLoss()
        xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
        out = []
        for _ in range(reps):  # graphs: capture, then replay
            loss = crit(model(xd), yd)
            loss.backward()
            out.append(_np(model.flat.grads).copy())
        return out
    finally:
        dtc._native.lib.dtc_set_option(b"graphs", _graphs_prev)


def _assert_same_grads(dtc, a, b, what, close=None):
    """Two flat gradient vectors that must be identical, checked per parameter (the message names the first
    that differs). The step is deterministic (BN sums are exact integer fixed point, common.h; every split-K
    sum has a fixed order), so any difference is a real one. close: {parameter name: rtol} for parameters a
    compared option computes with a different, legitimate fp32 grouping."""
    close = close or {}
    for pe in dtc.nn.Layout(100, 25.0).params:
        x = a[pe.offset:pe.offset + pe.numel]
        y = b[pe.offset:pe.offset + pe.numel]
        if pe.name in close:
            assert rel_err(y, x) < close[pe.name], (what, pe.name, rel_err(y, x))
        else:
            np.testing.assert_array_equal(x, y, err_msg=f"{what}: {pe.name}")


@pytest.mark.parametrize("batch", [256, 32])
def test_backward_repeatable_across_steps(dtc, cuda, batch):
    """Run-to-run bit-reproducibility of the default training step (the reference trains with
    cudnn.deterministic = True, src/ddp/utils.py:12-13): the same forward + backward twice on the same weights
    and data -- eager, and graph capture then replay -- at config 2's batch and config 3's per-rank batch must
    give identical gradients, bit for bit. Every split-K sum (in-kernel hand-off and reduce launches) runs in a
    fixed split order, and the BN batch statistics and backward sums are exact integer fixed-point sums
    (common.h), so the order in which workgroups' atomic adds arrive changes nothing. (Rounds 1-5 summed the BN
    partials with fp64 atomics: r05k / r05o saw two identical B=256 steps differ in the stem and layer1
    gradients, one fp32 coefficient rounded the other way.) Four repetitions per mode."""
    for graphs in (0, 1):
        g = _grads_repeated(dtc, cuda, graphs, reps=4, batch=batch)
        for r in range(1, len(g)):
            _assert_same_grads(dtc, g[0], g[r], f"graphs={graphs} B={batch} rep {r}")


@pytest.mark.parametrize("batch,hw", [(8, 32), (3, 32), (5, 8)])
def test_bn_reduce_unrolled_loads_bit_identical(dtc, cuda, batch, hw):
    """Option bn_red_unroll (default 4): the mask-bit BN-backward reduction issues the loads of 4 (or 2) rows
    per thread before their math instead of a load-use loop (1). Each thread adds its rows in the same order,
    so every gradient is bit-identical -- including ragged row counts that leave a remainder loop (batch 3 / 5)."""
    lib = dtc._native.lib
    try:
        lib.dtc_set_option(b"bn_red_unroll", 1)
        ga = _grads_repeated(dtc, cuda, 1, batch=batch, hw=hw)
        for ru in (2, 4):
            lib.dtc_set_option(b"bn_red_unroll", ru)
            gb = _grads_repeated(dtc, cuda, 1, batch=batch, hw=hw)
            for rep in range(2):
                assert np.isfinite(gb[rep]).all()
                assert np.array_equal(gb[rep], ga[rep]), (ru, rep, rel_err(gb[rep], ga[rep]))
    finally:
        lib.dtc_set_option(b"bn_red_unroll", 4)


@pytest.mark.parametrize("graphs", [True, False])
def test_wgrad_batch_matches_unbatched(dtc, cuda, graphs):
    """Deferred, batched 3x3 weight gradients (option wgrad_batch=4, default: one halo launch per
    geometry within a DDP bucket, 1/P of the split-K slab each) vs one launch per conv, on the same
    parameters and batch (capture and replay): only the fp32 split-K summation order differs."""
    ga = _grads_repeated(dtc, cuda, graphs)
    dtc._native.lib.dtc_set_option(b"wgrad_batch", 1)
    try:
        gb = _grads_repeated(dtc, cuda, graphs)
    finally:
        dtc._native.lib.dtc_set_option(b"wgrad_batch", 4)
    lay = dtc.nn.Layout(100, 25.0)
    for rep in range(2):
        for pe in lay.params:
            a = ga[rep][pe.offset:pe.offset + pe.numel]
            b = gb[rep][pe.offset:pe.offset + pe.numel]
            assert rel_err(a, b) < 1e-5, (rep, pe.name, rel_err(a, b))


@pytest.mark.parametrize("graphs", [True, False])
def test_bn_mask_bits_match_bf16_mask(dtc, cuda, graphs):
    """Mask-bit BN backward (option bn_mask=1, default: the forward BN apply writes the ReLU mask as
    bits, the reduction stores no dz, the apply forms dz from dy and the bits) vs masking with the
    bf16 outputs and a stored dz: masking is exact and the sums are the same partials (exact integer
    totals), so gradients are identical (capture and replay), and so are three training steps. The
    shortcut's dgrad stays a separate launch in both arms (dgrad_scf=0: the bn_mask=0 executor has no
    fused form; see test_fused_bn_finalize_matches_separate)."""
    lib = dtc._native.lib
    lib.dtc_set_option(b"dgrad_scf", 0)
    lib.dtc_set_option(b"bn_cg", 0)  # the two-pass kernels: the same summation order as bn_mask=0
    lib.dtc_set_option(b"wgrad_s2", 0)  # the bn_mask=0 executor has no fused conv1 + shortcut weight gradient
    try:
        ga = _grads_repeated(dtc, cuda, graphs)
        la, _, pa, ba = _train_steps(dtc, cuda, 3, graphs=graphs)
        lib.dtc_set_option(b"bn_mask", 0)
        try:
            gb = _grads_repeated(dtc, cuda, graphs)
            lb, _, pb, bb = _train_steps(dtc, cuda, 3, graphs=graphs)
        finally:
            lib.dtc_set_option(b"bn_mask", 1)
    finally:
        lib.dtc_set_option(b"dgrad_scf", 1)
        lib.dtc_set_option(b"bn_cg", 1)
        lib.dtc_set_option(b"wgrad_s2", 1)
    for rep in range(2):
        _assert_same_grads(dtc, ga[rep], gb[rep], f"bn_mask rep {rep}")
    np.testing.assert_array_equal(la, lb)
    np.testing.assert_array_equal(pa, pb)
    for k in ba:
        np.testing.assert_array_equal(ba[k], bb[k], err_msg=k)


@pytest.mark.parametrize("batch", [8, 32, 64])
def test_bn_one_launch_matches_two_pass(dtc, cuda, batch):
    """Option bn_cg (default): the mask-bit BN backward of tensors of at most 4096 pixels (2048 with the
    projection's second BN) as ONE launch per BN -- a workgroup per 8 channels holds the whole batch's slice,
    reduces sum(dz), sum(dz * xhat) in a fixed order and applies -- vs the reduce + apply pair. The sums are
    grouped differently (fp32 per thread, then fp64 over the waves, instead of per-block fp32 partials folded
    in fp64), so some bf16 outputs round the other way; one step's concatenated gradient agrees far inside the
    21% two correct bf16 implementations differ by, the first loss exactly. Exactness is
    the teacher-forced per-layer tests' job (the one-launch path is the default there at these batches)."""
    lib = dtc._native.lib
    try:
        lib.dtc_set_option(b"bn_cg", 0)
        ga = _grads_repeated(dtc, cuda, 1, batch=batch)
        la, _, _, ba = _train_steps(dtc, cuda, 1, graphs=1)
        lib.dtc_set_option(b"bn_cg", 1)
        gb = _grads_repeated(dtc, cuda, 1, batch=batch)
        lb, _, _, bb = _train_steps(dtc, cuda, 1, graphs=1)
    finally:
        lib.dtc_set_option(b"bn_cg", 1)
    for rep in range(2):
        assert np.isfinite(gb[rep]).all()
        assert rel_err(gb[rep], ga[rep]) < 2e-2, (rep, rel_err(gb[rep], ga[rep]))
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    for k in ba:
        assert rel_err(ba[k], bb[k]) < 1e-6, k


@pytest.mark.parametrize("batch", [8, 64])
def test_shortcut_compact_dx_matches_full(dtc, cuda, batch):
    """Option sc_compact (default): the projection shortcut's dx is computed at its stride-2 grid only
    (a 1x1 dgrad over the Hout x Wout pixels) and conv1's parity-class dgrad adds it at the (even, even)
    pixels; the full-resolution path writes the same values plus zeros at the other parities. Same
    reduction order, no split-K: the gradients agree exactly (graphs on and off)."""
    lib = dtc._native.lib
    for graphs in (0, 1):
        ga = _grads_repeated(dtc, cuda, graphs, batch=batch)
        lib.dtc_set_option(b"sc_compact", 0)
        try:
            gb = _grads_repeated(dtc, cuda, graphs, batch=batch)
        finally:
            lib.dtc_set_option(b"sc_compact", 1)
        for rep in range(2):
            np.testing.assert_array_equal(ga[rep], gb[rep])


@pytest.mark.parametrize("batch,hw", [(8, 32), (256, 32), (8, 8)])
def test_stem_bn_fused_wgrad_matches_separate(dtc, cuda, batch, hw):
    """Option stem_bn_fuse: the stem BN's backward apply inside the stem weight gradient (dc formed per
    tile in LDS, never stored) vs bn_bwd_fin_apply + stem_wgrad. Same coefficients, same fp32 expression
    and bf16 rounding: every gradient but the stem conv's is identical; the stem conv's differs only by
    the fp32 grouping of its per-workgroup partials (two tiles per workgroup instead of four at B=256;
    the same grouping -- so identical -- at small batches). 8x8 images take the global-gather path."""
    lib = dtc._native.lib
    for graphs in (1, 0):
        ga = _grads_repeated(dtc, cuda, graphs, batch=batch, hw=hw)
        lib.dtc_set_option(b"stem_bn_fuse", 1 - DEFAULT_STEM_BN_FUSE)
        try:
            gb = _grads_repeated(dtc, cuda, graphs, batch=batch, hw=hw)
        finally:
            lib.dtc_set_option(b"stem_bn_fuse", DEFAULT_STEM_BN_FUSE)
        for rep in range(2):
            _assert_same_grads(dtc, ga[rep], gb[rep], f"stem_bn_fuse rep {rep} graphs {graphs}",
                               close={"conv1.weight": 1e-5} if batch > 64 else None)


@pytest.mark.parametrize("level", [1, 2, 3])
def test_shortcut_fused_forward_matches_separate(dtc, cuda, level):
    """Option sc_fuse: the projection shortcut (1x1 stride 2) computed inside conv1's launch from the
    centre-tap im2col tiles (level 1: layer4's plan at B=64 and 256; 2: every 64x64-tile plan; 3: also
    layer2's 128x128) vs its own launch. With the implicit-GEMM fusion (halo_s2=0) neither path splits K and
    both tile the shortcut identically, so every output element sees the same MFMA sequence and every BN
    statistic the same fp32 partials: the gradients are identical. With the column-split halo forward
    (halo_s2=1, default: layer3/4 fused in conv_halo) the shortcut's MFMA sequence per element is the same
    but its BN statistics are reduced over the halo tiles instead of the 1x1 GEMM's (other fp32 partials):
    the gradients then agree to the bf16 propagation of last-bit statistic differences (1e-2)."""
    lib = dtc._native.lib
    for s2 in (0, 1):
        for graphs in (1, 0):
            try:
                lib.dtc_set_option(b"halo_s2", s2)
                lib.dtc_set_option(b"sc_fuse", 0)
                ga = _grads_repeated(dtc, cuda, graphs, batch=64)
                lib.dtc_set_option(b"sc_fuse", level)
                gb = _grads_repeated(dtc, cuda, graphs, batch=64)
            finally:
                lib.dtc_set_option(b"sc_fuse", DEFAULT_SC_FUSE)
                lib.dtc_set_option(b"halo_s2", 1)
            for rep in range(2):
                if s2 == 0:
                    _assert_same_grads(dtc, ga[rep], gb[rep], f"sc_fuse={level} rep {rep}")
                else:
                    assert np.isfinite(gb[rep]).all() and rel_err(gb[rep], ga[rep]) < 1e-2, rel_err(gb[rep], ga[rep])


@pytest.mark.parametrize("batch", [8, 64])
def test_fused_shortcut_dgrad_and_wgrad_match_separate(dtc, cuda, batch):
    """Options wgrad_s2 (conv1's and the projection shortcut's weight gradients in one column-split halo
    launch) and dgrad_scf (the shortcut's dgrad as extra reduction steps of conv1's class-(0,0) dgrad) vs
    the separate launches, graphs on and off. wgrad_s2 changes only the fp32 summation order of those
    weight gradients: every parameter gradient within 1e-5. dgrad_scf changes the bf16 rounding of the
    data gradient entering layer3 (one fp32 sum instead of two bf16-rounded ones added): everything the
    backward computes before it (layer4, linear) is bit-identical, the first BN behind it (layer3.1.bn2)
    within 1e-2, and the rest finite (further down, rounding differences are amplified as in any two
    correct bf16 implementations -- DESIGN.md §4)."""
    lib = dtc._native.lib
    lay = dtc.nn.Layout(100, 25.0)

    def run(opts, graphs):
        prev = {k: lib.dtc_get_option(k) for k in opts}
        try:
            for k, v in opts.items():
                lib.dtc_set_option(k, v)
            return _grads_repeated(dtc, cuda, graphs, batch=batch)
        finally:
            for k, v in prev.items():
                lib.dtc_set_option(k, v)

    for graphs in (1, 0):
        base = run({b"dgrad_scf": 0, b"wgrad_s2": 0}, graphs)
        ws2 = run({b"dgrad_scf": 0, b"wgrad_s2": 1}, graphs)
        dsf = run({b"dgrad_scf": 1, b"wgrad_s2": 0}, graphs)
        for rep in range(2):
            for pe in lay.params:
                a = base[rep][pe.offset:pe.offset + pe.numel]
                assert rel_err(ws2[rep][pe.offset:pe.offset + pe.numel], a) < 1e-5, (graphs, rep, pe.name)
                b = dsf[rep][pe.offset:pe.offset + pe.numel]
                if pe.name.startswith(("layer4", "linear")):
                    assert np.array_equal(a, b), (graphs, rep, pe.name)
                elif pe.name.startswith("layer3.1.bn2"):
                    assert rel_err(b, a) < 1e-2, (graphs, rep, pe.name, rel_err(b, a))
                assert np.isfinite(b).all()


@pytest.mark.parametrize("batch,hw", [(8, 32), (256, 32), (8, 8)])
def test_stem_weight_lds_matches_gather(dtc, cuda, batch, hw):
    """Option stem_wlds: the stem forward's weight fragments gathered from an LDS copy (coalesced loads)
    instead of per-lane global gathers; the input rows capped at 8 KB of LDS (wider tiles take the
    global-gather path). The same values reach the same MFMAs: identical gradients."""
    lib = dtc._native.lib
    try:
        lib.dtc_set_option(b"stem_wlds", 0)
        ga = _grads_repeated(dtc, cuda, 1, batch=batch, hw=hw)
        lib.dtc_set_option(b"stem_wlds", 1)
        gb = _grads_repeated(dtc, cuda, 1, batch=batch, hw=hw)
    finally:
        lib.dtc_set_option(b"stem_wlds", DEFAULT_STEM_WLDS)
    for rep in range(2):
        _assert_same_grads(dtc, ga[rep], gb[rep], f"stem_wlds rep {rep}")


def test_head_after_forward_graph_matches_eager(dtc, cuda):
    """The replayed forward's head is launched after the graph straight into each call's own logits
    tensor (the graph cannot bake in a per-call pointer): identical logits and gradients to the eager
    forward (train and eval), and the logits of consecutive forwards into different tensors stay distinct."""
    lib = dtc._native.lib
    prev = lib.dtc_get_option(b"graphs")
    res = {}
    try:
        for graphs in (0, 2):
            lib.dtc_set_option(b"graphs", graphs)
            g = _grads_repeated(dtc, cuda, graphs, batch=16)
            model, _, x, _ = _setup(dtc, cuda, 16, seed=3)
            xd = torch.from_numpy(x).to(cuda)
            with torch.no_grad():
                model.eval()
                e1 = model(xd)
                e2 = model(xd * 0.5)  # a second output tensor: must not overwrite e1
                res[graphs] = (g, _np(e1), _np(e2))
    finally:
        lib.dtc_set_option(b"graphs", prev)
    for rep in range(2):
        np.testing.assert_array_equal(res[0][0][rep], res[2][0][rep])
    np.testing.assert_array_equal(res[0][1], res[2][1])
    np.testing.assert_array_equal(res[0][2], res[2][2])
    assert not np.array_equal(res[2][1], res[2][2])


def test_graph_recapture_on_option_change(dtc, cuda):
    """Options are baked into captured launches: changing one re-captures (results unchanged)."""
    model, _, x, y = _setup(dtc, cuda, 4, seed=6)
    xd = torch.from_numpy(x).to(cuda)
    with torch.no_grad():
        a = _np(model(xd))
        dtc._native.lib.dtc_set_option(b"dgrad_classes", 0)
        try:
            b = _np(model(xd))
        finally:
            dtc._native.lib.dtc_set_option(b"dgrad_classes", 1)
        c = _np(model(xd))
    assert rel_err(a, b) < 1e-2 and rel_err(a, c) < 1e-2


def test_live_conv_profile(dtc, cuda):
    """dtc_rn18_profile_*: per-call device timestamps, folded once per training step."""
    import ctypes as C

    model, _, x, y = _setup(dtc, cuda, 8, seed=7)
    crit = dtc.CrossEntropyLoss()
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    dtc._native.lib.dtc_set_option(b"sc_fuse", 0)  # one launch per conv (sc_fuse merges conv1 + shortcut)
    dtc._native.lib.dtc_set_option(b"dgrad_scf", 0)  # (and dgrad_scf their dgrads,
    dtc._native.lib.dtc_set_option(b"wgrad_s2", 0)  # wgrad_s2 their weight gradients)
    try:
        crit(model(xd), yd).backward()
        exe = model.executor(8, 32, 32)
        dtc._native.call("dtc_rn18_profile_begin", exe.handle, 1)
        steps = 3
        for _ in range(steps):
            crit(model(xd), yd).backward()
        ms, fl, cnt = (C.c_double * 3)(), (C.c_double * 3)(), (C.c_int * 3)()
        dtc._native.call("dtc_rn18_profile_end", exe.handle, ms, fl, cnt)
    finally:
        dtc._native.lib.dtc_set_option(b"sc_fuse", DEFAULT_SC_FUSE)
        dtc._native.lib.dtc_set_option(b"dgrad_scf", 1)
        dtc._native.lib.dtc_set_option(b"wgrad_s2", 1)
    # 20 convs; the stem has no dgrad; the 13 stride-1 3x3 weight gradients run batched per geometry
    # within a DDP bucket (layer4 3, layer3 3, layer2 3, layer1 4: four launches) beside the 7 others
    assert list(cnt) == [20 * steps, 19 * steps, 11 * steps]
    fwd_flops = 8 * 1.1108e9  # per image: stem 3.5 MFLOP + layer1 302 + 3 x 268.4 (layers 2-4)
    assert abs(fl[0] / steps / fwd_flops - 1) < 0.01
    assert abs(fl[2] / steps / fwd_flops - 1) < 0.01  # every weight gradient counted exactly once
    for k in range(3):
        assert 0 < ms[k] / cnt[k] < 5.0  # ms per call: positive, sane


def _perturb_ulp(model, seed):
    """1-ulp init perturbation, identical to tests/golden/make_golden.py::_perturb_ulp."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for prm in model.parameters():
            sign = torch.randint(0, 2, prm.shape, generator=g).float() * 2 - 1
            prm.mul_(1 + sign * 2.0 ** -23)


_LC_BATCHES = {}


def _lc_batches(lc, cuda):
    """The 200 seeded synthetic batches of the loss-curve fixture (tests/golden/make_golden.py::
    synthetic_stream: labels randint(1234 + step), x = 0.5 * T[y] + randn), generated once on the host in
    the fixture's order and kept on the GPU for every curve of the ensemble."""
    key = (lc["batch"], lc["steps"])
    if key not in _LC_BATCHES:
        batch, steps = key
        templates = torch.randn(100, 3, 32, 32, generator=torch.Generator().manual_seed(1234))
        out = []
        for s in range(steps):
            gen = torch.Generator().manual_seed(1234 + s)
            y = torch.randint(0, 100, (batch,), generator=gen)
            x = 0.5 * templates[y] + torch.randn(batch, 3, 32, 32, generator=gen)
            out.append((x.to(cuda), y.to(cuda)))
        _LC_BATCHES[key] = out
    return _LC_BATCHES[key]


def _loss_curve(dtc, cuda, lc, ulp_seed=0):
    batches = _lc_batches(lc, cuda)
    torch.manual_seed(42)
    model = dtc.ResNet18()
    if ulp_seed:
        _perturb_ulp(model, ulp_seed)
    model = model.to(cuda)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=lc["lr"], weight_decay=lc["wd"], momentum=lc["momentum"], nesterov=True)
    losses = []
    for x, y in batches:
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(model(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.detach())
    return np.array([float(v) for v in torch.stack(losses).cpu()])


def test_loss_curve_200_steps(dtc, cuda):
    """north_star: 200-step loss curve within 1% of the reference.

    Fixture (tests/golden/make_golden.py loss, loss_chaos): the REFERENCE net + SGD recipe
    (src/single/net.py, utils.fix_seed(42), SGD nesterov lr 0.1 wd 1e-4; single/trainer.py:131-147) on
    the seeded synthetic stream, batch 128, bf16 autocast: once from the seed-42 init and once from each
    of 99 inits perturbed by 1 ulp (100 curves). Training is chaotic: the reference's OWN 1-ulp reruns
    spread the 200-step mean loss by ~1.8% (s.d.), so one curve cannot be held to 1%; the ensemble of 100
    resolves it (3 standard errors of the difference of the two ensemble means ~0.75%). Criterion: our
    ensemble over the same 100 inits has a 200-step mean loss within 1% of the reference's, with the 3-s.e.
    resolution printed beside it (and required < 1%, i.e. the check really resolves 1%); and the
    per-step ensemble means within 1% over the leading steps where the reference ensemble itself resolves
    1% (before the trajectories decorrelate)."""
    import json
    import os

    lc = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "loss_curve.json")))
    ref_curves = [np.array(lc["bf16"])] + [np.array(c) for c in lc.get("bf16_ulp", [])]
    ours = [_loss_curve(dtc, cuda, lc, u) for u in range(len(ref_curves))]
    assert all(np.all(np.isfinite(c)) for c in ours)
    first = np.abs(ours[0][:5] - ref_curves[0][:5]) / ref_curves[0][:5]
    assert np.all(first < 1e-2), first
    mo = np.array([c.mean() for c in ours])
    mr = np.array([c.mean() for c in ref_curves])
    n = len(mr)
    se = np.sqrt(mo.var(ddof=1) / n + mr.var(ddof=1) / n) / mr.mean()
    rel = (mo.mean() - mr.mean()) / mr.mean()
    O_ = np.stack(ours)
    R_ = np.stack(ref_curves)
    step_rel = (O_.mean(0) - R_.mean(0)) / R_.mean(0)
    step_se = np.sqrt(O_.var(0, ddof=1) / n + R_.var(0, ddof=1) / n) / R_.mean(0)
    resolvable = 3.0 * step_se < 1e-2
    K = int(np.argmin(resolvable)) if not resolvable.all() else len(resolvable)
    worst_k = float(np.abs(step_rel[:K]).max()) if K else 0.0
    report = (f"loss-curve parity (n={n} curves per side x {O_.shape[1]} steps): 200-step ensemble mean ours "
              f"{mo.mean():.4f} ref {mr.mean():.4f} rel {rel:+.4f} (bound 0.01; resolution 3 s.e. = {3 * se:.4f}); "
              f"per-step ensemble means over the first {K} resolvable steps: max |rel| {worst_k:.4f} (bound 0.01)")
    print(report)
    import warnings

    warnings.warn(report, UserWarning)  # lands in the pytest warnings summary of the GPU test log
    assert K >= 5 and worst_k < 1e-2, report
    if n >= 100:  # the full ensemble: north_star's 1% itself, and the check resolves it
        assert 3 * se < 1e-2 and abs(rel) < 1e-2, report
    else:  # a partial fixture (ensemble still being generated): the statistical bound of round 2
        assert abs(rel) < max(1e-2, 3.0 * se), report


def test_native_loss_backward_matches_autograd(dtc, cuda):
    """NativeLoss.backward (direct xent-backward -> network-backward chain, plain and
    GradScaler-scaled) writes the same gradients as the autograd-engine path."""
    from importlib import import_module

    nnmod = import_module(dtc.__name__ + ".nn")
    model, _, x, y = _setup(dtc, cuda, 8, seed=11)
    crit = dtc.CrossEntropyLoss()
    scaler = dtc.GradScaler()
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    out = {}
    for fast in (True, False):
        nnmod._FAST_BACKWARD[0] = fast
        try:
            loss = crit(model(xd), yd)
            assert isinstance(loss, nnmod.NativeLoss)
            loss.backward()
            g_plain = model.flat.grads.clone()
            loss = crit(model(xd), yd)
            scaled = scaler.scale(loss)
            assert isinstance(scaled, nnmod.NativeLoss)
            assert abs(float(scaled) - float(loss) * 65536.0) < 1e-3 * float(scaled)
            scaled.backward()
            g_scaled = model.flat.grads.clone()
        finally:
            nnmod._FAST_BACKWARD[0] = True
        torch.cuda.synchronize()
        out[fast] = (g_plain, g_scaled)
    assert rel_err(out[True][0].cpu().numpy(), out[False][0].cpu().numpy()) < 1e-5
    assert rel_err(out[True][1].cpu().numpy(), out[False][1].cpu().numpy()) < 1e-5
    ratio = (out[True][1].norm() / out[True][0].norm()).item()
    assert abs(ratio - 65536.0) < 1e-2 * 65536.0
    # arithmetic on the loss leaves the fast path: a plain autograd tensor
    loss = crit(model(xd), yd)
    assert type(loss * 2.0) is torch.Tensor


@pytest.mark.parametrize("head_fused", [1, 0])
@pytest.mark.parametrize("precision,batch", [("bf16", 8), ("bf16", 64), ("fp32", 8)])
def test_xent_fused_into_head_backward_bit_identical(dtc, cuda, head_fused, precision, batch):
    """Option xent_fuse (default on): the CrossEntropyLoss backward is computed inside the head backward
    kernel instead of a launch of its own. Every gradient and the executor's dlogits buffer are
    bit-identical to the separate xent_bwd launch, for the one-launch head backward and the three-kernel
    one (head_fused 0, where the fused call falls back to xent_bwd first), bf16 and fp32 executors."""
    lib = dtc._native.lib
    prev_hf = lib.dtc_get_option(b"head_fused")
    lib.dtc_set_option(b"head_fused", head_fused)
    try:
        model, _, x, y = _setup(dtc, cuda, batch, seed=16)
        crit = dtc.CrossEntropyLoss()
        scaler = dtc.GradScaler(init_scale=256.0)
        xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
        out = {}
        for fuse in (1, 0):
            lib.dtc_set_option(b"xent_fuse", fuse)
            with dtc.autocast(enabled=precision == "bf16"):
                loss = crit(model(xd), yd)
            scaler.scale(loss).backward()
            exe = model.executor(batch, 32, 32, precision)
            torch.cuda.synchronize()
            out[fuse] = (model.flat.grads.clone(), exe.dlogits_buffer().clone())
        assert torch.equal(out[1][1], out[0][1])
        assert torch.equal(out[1][0], out[0][0])
        assert float(out[1][1].abs().sum()) > 0
    finally:
        lib.dtc_set_option(b"xent_fuse", 1)
        lib.dtc_set_option(b"head_fused", prev_hf)


def test_second_backward_refused_and_sums_rezeroed(dtc, cuda):
    """the BN backward sums are zeroed by the training forward only. (1) The Python layer
    refuses a second backward over one forward (torch would ACCUMULATE into .grad; the kernels write);
    (2) a second backward issued straight through the C ABI re-zeroes the sums first, so it writes the
    same gradients as the first instead of adding onto the first backward's sums."""
    import ctypes as C

    model, _, x, y = _setup(dtc, cuda, 8, seed=5)
    crit = dtc.CrossEntropyLoss()
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    loss = crit(model(xd), yd)
    loss.backward(retain_graph=True)
    g1 = model.flat.grads.clone()
    with pytest.raises(dtc.NativeError, match="already back-propagated"):
        loss.backward()
    exe = model.executor(8, 32, 32)
    dl = exe.dlogits_buffer()
    for graphs in (1, 0):
        _graphs_prev = dtc._native.lib.dtc_get_option(b"graphs")
        dtc._native.lib.dtc_set_option(b"graphs", graphs)
        try:
            crit(model(xd), yd).backward()
            g_a = model.flat.grads.clone()
            dtc._native.call("dtc_rn18_backward", exe.handle, C.c_void_p(dl.data_ptr()), C.c_float(1.0), None,
                             dtc._native.stream_ptr())
            torch.cuda.synchronize()
            g_b = model.flat.grads.clone()
        finally:
            dtc._native.lib.dtc_set_option(b"graphs", _graphs_prev)
        assert torch.equal(g_a, g_b), (graphs, (g_a - g_b).abs().max().item())
    assert rel_err(g1.cpu().numpy(), g_a.cpu().numpy()) < 1e-5


def test_native_barrier_waits_for_queued_work(dtc, cuda):
    """dtc.barrier() (dtc_barrier; the reference's per-step dist.barrier(), trainer.py:156) returns only
    after the work queued on the current stream before it finished -- torch's NCCL barrier semantics
    -- with no communicator (world 1) and through a one-rank RCCL communicator registered as the
    default group's."""
    s = torch.cuda.current_stream()
    torch.cuda._sleep(50_000_000)  # a long spin kernel (~20+ ms)
    assert not s.query()
    dtc.barrier()
    assert s.query()
    comm = dtc.parallel.Comm(0, 1, dtc.parallel.Comm.unique_id(), cuda.index or 0)
    prev = dtc.parallel._WORLD_COMM[0]
    dtc.parallel._WORLD_COMM[0] = comm
    try:
        torch.cuda._sleep(50_000_000)
        assert not s.query()
        dtc.barrier()
        assert s.query()
        dtc._native.call("dtc_barrier", comm.handle, dtc._native.stream_ptr())  # the RCCL form itself
        assert s.query()
    finally:
        dtc.parallel._WORLD_COMM[0] = prev
        comm.close()


def test_scaled_loss_prescaled_with_the_loss(dtc, cuda):
    """The loss call also enqueues loss * scale for the last initialised GradScaler (before the per-step
    barrier); scaler.scale(loss) reuses it only for the same scale tensor and scaler state: the value
    is loss * current scale before and after update() changes the scale, and a loss taken before an
    update is scaled by the new scale when scale() is called after it."""
    from importlib import import_module

    nnmod = import_module(dtc.__name__ + ".nn")
    model, _, x, y = _setup(dtc, cuda, 8, seed=13)
    crit = dtc.CrossEntropyLoss()
    scaler = dtc.GradScaler(init_scale=1024.0)
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    scaler.scale(crit(model(xd), yd))  # initialises the scaler (registers it for prescaling)
    loss = crit(model(xd), yd)
    assert loss.__dict__.get("_dtc_prescaled") is not None
    s1 = scaler.scale(loss)
    assert s1.data_ptr() == loss._dtc_prescaled[0].data_ptr()  # no new launch: the prescaled product
    assert float(s1) == float(loss) * 1024.0
    stale = crit(model(xd), yd)
    scaler.update(new_scale=4.0)  # changes the scale after `stale` was prescaled with 1024
    s2 = scaler.scale(stale)
    assert s2.data_ptr() != stale._dtc_prescaled[0].data_ptr()
    assert float(s2) == float(stale) * 4.0
    s2.backward()  # the direct backward chain still applies
    assert isinstance(s2, nnmod.NativeLoss)


def test_native_loss_item_and_dlogits_buffer(dtc, cuda):
    """NativeLoss.item() reads the pinned host copy taken right after the loss kernel: equal to the
    device value even when read after the backward and the optimizer step have been issued; the
    fused xent backward writes the executor's own dlogits buffer (graph path skips the copy-in)."""
    model, _, x, y = _setup(dtc, cuda, 8, seed=12)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    vals = []
    for _ in range(3):
        opt.zero_grad()
        loss = crit(model(xd), yd)
        ref = loss.detach().clone()
        loss.backward()
        opt.step()
        v = loss.item()
        assert v == float(ref.cpu()), (v, float(ref.cpu()))
        assert float(loss) == v
        vals.append(v)
    exe = model.executor(8, 32, 32)
    dl = exe.dlogits_buffer()
    assert dl.shape == (8, 100) and dl.dtype == torch.float32
    # the last backward's dlogits: rows are softmax - onehot over the batch, so each row sums to ~0
    assert float(dl.sum(1).abs().max()) < 1e-5
    assert np.isfinite(vals).all()


def test_native_loss_item_after_host_ring_wraps(dtc, cuda):
    """a loss kept past the pinned host-word ring's N newer losses must not read the value a
    later launch wrote into its reused slot: item() falls back to the loss's own device value."""
    from importlib import import_module

    nnmod = import_module(type(dtc.CrossEntropyLoss()).__module__)
    model, _, x, y = _setup(dtc, cuda, 2, seed=5)
    crit = dtc.CrossEntropyLoss()
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    first = crit(model(xd), yd)
    v0 = float(first.detach().cpu())
    n = nnmod._HostWords.N
    held = [first]
    with dtc.autocast():  # a different value in every later slot (bf16 logits)
        for i in range(n + 4):
            held.append(crit(model(xd * (1.0 + 0.01 * (i + 1))), yd))
    torch.cuda.synchronize()
    assert first.item() == v0
    for ls in held[-4:]:  # the newest losses still read their own slots
        assert ls.item() == float(ls.detach().cpu())


def test_data_parallel_replicas_match_chunked_single(dtc, cuda):
    """DataParallel (reference src/dp/trainer.py:27) with two replicas on cuda:0 (device_ids=[0, 0]:
    the one-GPU form of scatter / replicate / parallel_apply / gather / reduce-add) against the
    same module run on each half-batch separately:
      * gathered logits == the concatenated per-chunk logits (bit-exact: same kernels, same inputs);
      * module gradient == 0.5 * (grad of chunk 0 + grad of chunk 1) under the mean loss over the
        whole batch (the scaling by 1/2 is exact in binary floating point);
      * BN running statistics == the update from chunk 0 alone (replica 0 is the module).
    A second step checks that replica 1 picks up the module's updated parameters (replicate)."""
    B = 16
    g = np.random.default_rng(7)
    x = torch.from_numpy(g.standard_normal((2 * B, 3, 32, 32)).astype(np.float32)).to(cuda)
    y = torch.from_numpy(g.integers(0, 100, 2 * B)).to(cuda)

    torch.manual_seed(42)
    ref = dtc.ResNet18().to(cuda)
    crit = dtc.CrossEntropyLoss()
    logits_ref, grads = [], []
    bufs0 = None
    for c in range(2):
        ref.zero_grad()
        lo = ref(x[c * B:(c + 1) * B])
        crit(lo, y[c * B:(c + 1) * B]).backward()
        logits_ref.append(lo.detach().clone())
        grads.append(ref.flat.grads.clone())
        if c == 0:
            bufs0 = ref.flat.bufs.clone()
    g_ref = 0.5 * (grads[0] + grads[1])

    torch.manual_seed(42)
    m = dtc.ResNet18().to(cuda)
    dp = dtc.DataParallel(m, device_ids=[0, 0])
    dp.zero_grad()
    lo = dp(x)
    crit(lo, y).backward()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(lo), _np(torch.cat(logits_ref)))
    np.testing.assert_allclose(_np(m.flat.grads), _np(g_ref), rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(_np(m.flat.bufs), _np(bufs0))
    assert sorted(dp.state_dict())[0].startswith("module.")

    # step 2: an SGD update on the module, then replica 1 must run with the new parameters
    opt = dtc.SGD(dp.parameters(), lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-4)
    opt.step()
    torch.cuda.synchronize()
    lo2 = dp(x)
    ref2 = dtc.ResNet18()
    torch.manual_seed(0)
    ref2 = ref2.to(cuda)
    ref2.load_state_dict(m.state_dict())
    with torch.no_grad():
        l1 = ref2(x[B:])
    # replica 1's half was produced from the module's updated parameters and buffers
    torch.cuda.synchronize()
    assert rel_err(_np(lo2[B:]), _np(l1)) < 1e-6


def test_dp_trainer_runs(dtc, cuda, tmp_path):
    """`train.py dp` (src/dp/main.py flow: fit -> validate -> checkpoint -> test) through the native
    DataParallel with two replicas on cuda:0, AMP on, a few steps of synthetic data: the
    checkpoint holds `module.`-prefixed keys (DataParallel.state_dict) and test() reloads it."""
    import glob
    import json
    import os

    t = dtc.trainer.main(["--epoch", "1", "--batch-size", "64", "--max-steps", "3", "--amp", "--contain-test",
                          "--workers", "0", "--synthetic-train", "640", "--synthetic-test", "128",
                          "--eval-step", "1", "--device-ids", "0,0", "--ckpt-path", str(tmp_path)], "dp")
    assert isinstance(t.model, dtc.DataParallel)
    ck = glob.glob(os.path.join(str(tmp_path), "version-0", "best_model_*.pt"))
    log = open(os.path.join(str(tmp_path), "version-0", "experiment.log")).read()
    assert "[DP Version 0 Epoch 0] global step: 3" in log
    if not ck:  # validation accuracy stayed 0 (no improvement to save): save through the same method
        t.save_checkpoint(0, 0.5, t.model)
        ck = glob.glob(os.path.join(str(tmp_path), "version-0", "best_model_*.pt"))
    assert len(ck) == 1
    sd = torch.load(ck[0], weights_only=True)
    assert sd and all(k.startswith("module.") for k in sd)
    res = t.test(sd)  # dp/main.py:33-39: reload the best checkpoint into the DataParallel model and test
    assert np.isfinite(res["test_loss"]) and 0.0 <= res["top_1_acc"] <= 100.0


def _native_kernels_only(dtc, cuda, fn):
    """Run fn under the torch profiler and return the GPU kernels it launched that are not this
    library's (names outside the dtc:: namespace): torch elementwise / copy kernels on the hot path."""
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if e.device_type.name == "CUDA"}
    native = sorted(n for n in names if "dtc::" in n)
    assert len(native) >= 20, f"profiler saw too few native kernels to judge: {sorted(names)}"
    return sorted(n for n in names if "dtc::" not in n and not n.startswith(("Memcpy", "Memset", "hipMemcpy",
                                                                             "hipMemset", "__amd_rocclr")))


def test_data_parallel_step_launches_only_native_kernels(dtc, cuda):
    """Config 4's step (dp/trainer.py:132-148: forward, CE, scaled backward, step, update) through
    the native DataParallel: replicate / reduce-add / scatter / gather run in this library (RCCL or
    its on-device copies + HIP reduce-add), so no torch compute kernel appears in the step."""
    torch.manual_seed(42)
    dp = dtc.DataParallel(dtc.ResNet18().to(cuda), device_ids=[0, 0])
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(dp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    scaler = dtc.GradScaler()
    g = torch.Generator(device=cuda).manual_seed(1)
    x = torch.randn(64, 3, 32, 32, device=cuda, generator=g)
    y = torch.randint(0, 100, (64,), device=cuda, generator=g)

    def step():
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(dp(x), y)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        return loss

    step()  # warm: executors, replicas, graphs
    foreign = _native_kernels_only(dtc, cuda, step)
    assert not foreign, foreign


def _grads_with(model, crit, x, y, comm):
    model._comm = comm
    loss = crit(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return model.flat.grads.detach().cpu().numpy().copy()


@pytest.mark.parametrize("graphs,on_side", [(1, 0), (1, 1), (0, 0), (0, 1)])
@pytest.mark.parametrize("cap_mb", [1.0, 5.0, 25.0])
def test_reducer_reduces_every_bucket_once_after_its_producers(dtc, cuda, graphs, on_side, cap_mb):
    """The N>1 DDP backward (ddp/trainer.py:157) on one GPU, made observable: a loopback
    communicator (dtc_comm_init_loopback) replaces each bucket's ncclAllReduce with `bucket *= 2` on
    the communicator's side stream and logs (address, count). Then, on capture AND on replay:
      * the logged ranges are exactly the bucket plan, in backward-completion order, each once, and
        together tile the flat gradient buffer [0, numel) with no gap or overlap;
      * every bucket's gradients are exactly 2x the no-communicator gradients -- a bucket skipped
        (1x), reduced twice (4x) or reduced before its producing kernels finished (they WRITE the
        gradient, so the doubling would be overwritten: 1x) fails;
      * with the DDP mean pre-scale of 1/2 (module._grad_scale, W=2) the result equals the local
        gradient (the mean over two identical ranks).
    The last bucket of the plan is only layer1 + the stem (the unavoidable exposed tail). on_side: the eager
    backward's bucket collectives on the weight-gradient stream itself (option comm_on_side)."""
    _graphs_prev = dtc._native.lib.dtc_get_option(b"graphs")
    dtc._native.lib.dtc_set_option(b"graphs", graphs)
    dtc._native.lib.dtc_set_option(b"comm_on_side", on_side)
    comm = dtc.parallel.Comm.loopback(cuda.index or 0, 2.0)
    try:
        torch.manual_seed(42)
        model = dtc.ResNet18().to(cuda)
        model.set_bucket_cap_mb(cap_mb)
        buckets = model.buckets()
        numel = model.flat.grads.numel()
        assert buckets[0][0] == 0 and sum(n for _, n in buckets) == numel
        assert all(o1 + n1 == o2 for (o1, n1), (o2, _) in zip(buckets, buckets[1:]))
        assert buckets[-1][1] * 4 <= 2 * 2**20, buckets[-1]  # tail <= 2 MB (layer1 + stem: 0.57 MB)
        crit = dtc.CrossEntropyLoss()
        g = torch.Generator().manual_seed(3)
        x = torch.randn(32, 3, 32, 32, generator=g).to(cuda)
        y = torch.randint(0, 100, (32,), generator=g).to(cuda)
        g0 = _grads_with(model, crit, x, y, None)
        assert np.isfinite(g0).all() and np.abs(g0).sum() > 0
        base = model.flat.grads.data_ptr()
        for rep in range(2):  # first use (capture when graphs are on), then replay
            comm.clear_log()
            g1 = _grads_with(model, crit, x, y, comm)
            log = comm.log()
            assert all(is_bucket for _, _, is_bucket in log)
            assert [((a - base) // 4, n) for a, n, _ in log] == buckets, (rep, log)
            for off, n in buckets:
                assert rel_err(g1[off:off + n], 2.0 * g0[off:off + n]) < 1e-3, (rep, off, n)
        model._grad_scale = 0.5  # DDP over W=2 identical ranks: pre-divide by 2, SUM (x2) -> local grad
        g2 = _grads_with(model, crit, x, y, comm)
        assert rel_err(g2, g0) < 1e-3
        model._comm, model._grad_scale = None, 1.0
    finally:
        comm.close()
        dtc._native.lib.dtc_set_option(b"graphs", _graphs_prev)
        dtc._native.lib.dtc_set_option(b"comm_on_side", 1)


@pytest.mark.parametrize("graphs", [1, 0])
def test_bucketed_allreduce_backward_one_rank_rccl(dtc, cuda, graphs):
    """The same backward through a real one-rank RCCL communicator (the production transport; a
    one-rank SUM is the identity): gradients equal the no-communicator backward, capture and replay."""
    _graphs_prev = dtc._native.lib.dtc_get_option(b"graphs")
    dtc._native.lib.dtc_set_option(b"graphs", graphs)
    comm = dtc.parallel.Comm(0, 1, dtc.parallel.Comm.unique_id(), cuda.index or 0)
    try:
        torch.manual_seed(42)
        model = dtc.ResNet18().to(cuda)
        model.set_bucket_cap_mb(1.0)
        assert len(model.buckets()) >= 5  # block-granular buckets
        crit = dtc.CrossEntropyLoss()
        g = torch.Generator().manual_seed(3)
        x = torch.randn(32, 3, 32, 32, generator=g).to(cuda)
        y = torch.randint(0, 100, (32,), generator=g).to(cuda)
        g0 = _grads_with(model, crit, x, y, None)
        g1 = _grads_with(model, crit, x, y, comm)
        g2 = _grads_with(model, crit, x, y, comm)
        assert rel_err(g1, g0) < 1e-3 and rel_err(g2, g0) < 1e-3
        model._comm = None
    finally:
        comm.close()
        dtc._native.lib.dtc_set_option(b"graphs", _graphs_prev)


def test_sync_batchnorm_two_identical_ranks_loopback(dtc, cuda):
    """SyncBatchNorm at W=2 on one GPU: a loopback communicator reporting 2 ranks doubles every BN
    sum the executor all-reduces (= two ranks holding the same batch). Global statistics then equal
    the local ones (sums x2, count x2), so logits, every gradient and the running statistics must equal
    plain BN (dgamma/dbeta = (1/W) x the all-reduced sums = this rank's share, which DDP's mean then
    averages -- torch SyncBN + DDP). A path that skipped a collective would halve that BN's mean / its
    backward sums (sums x1, count x2) and fail. The BN sums are exact integers (common.h), doubled sums over
    a doubled count give the same fp64 quotients, so logits and gradients are bit-identical to plain BN.
    Every forward and backward BN all-reduce is logged: 20 BNs -> 20 forward + 20 backward in-stream
    collectives of hdr + 4*C int64 words each (the 16-word header and the compacted slot 0, not all 8 slots).
    """
    comm = dtc.parallel.Comm.loopback(cuda.index or 0, 2.0, world=2)
    dtc._native.lib.dtc_set_option(b"bn_cg", 0)  # the SyncBN executor's two-pass BN backward in both arms
    try:
        g = torch.Generator().manual_seed(5)
        x = torch.randn(32, 3, 32, 32, generator=g).to(cuda)
        y = torch.randint(0, 100, (32,), generator=g).to(cuda)
        res = []
        for sync in (False, True):
            torch.manual_seed(42)
            model = dtc.ResNet18().to(cuda)
            if sync:
                model = dtc.SyncBatchNorm.convert_sync_batchnorm(model)
                model.set_sync_bn(comm)
                comm.clear_log()
            logits = model(x)
            dtc.CrossEntropyLoss()(logits, y).backward()
            torch.cuda.synchronize()
            res.append((logits.detach().cpu().numpy(), model.flat.grads.detach().cpu().numpy().copy(),
                        model.flat.bufs.detach().cpu().numpy().copy(), model))
        (l0, g0, b0, m0), (l1, g1, b1, m1) = res
        log = comm.log()
        assert len(log) == 40 and not any(a for _, _, a in log)
        chans = sorted(n for _, n, _ in log)
        hdr = 2 * dtc._native.lib.dtc_bn_stat_words(1) - dtc._native.lib.dtc_bn_stat_words(2)
        assert chans[0] == hdr + 4 * 64 and chans[-1] == hdr + 4 * 512
        # running_var's unbiased factor uses the GLOBAL count (2M/(2M-1) vs M/(M-1): up to 1e-4 on
        # layer4 at M=512), as torch SyncBatchNorm does; running_mean is unaffected
        np.testing.assert_array_equal(l1, l0)
        np.testing.assert_array_equal(g1, g0)
        assert rel_err(b1, b0) < 2e-4
        m1.set_sync_bn(None)
    finally:
        dtc._native.lib.dtc_set_option(b"bn_cg", 1)
        comm.close()


def test_sync_batchnorm_one_rank(dtc, cuda):
    """SyncBatchNorm path (dtc_rn18_set_sync_bn) with a one-rank RCCL
    communicator: every BN's statistic slots are compacted into slot 0 and go through an in-stream int64
    all-reduce (the identity over one rank) and the executor runs eagerly; logits, gradients and running
    statistics must equal the per-rank BatchNorm path bit for bit (the sums are exact integers: compaction
    and the collective change no bit). The two-rank statistics semantics are covered by
    tests/test_ddp_gloo.py::test_sync_batchnorm_gloo."""
    comm = dtc.parallel.Comm(0, 1, dtc.parallel.Comm.unique_id(), cuda.index or 0)
    dtc._native.lib.dtc_set_option(b"bn_cg", 0)  # the SyncBN executor's two-pass BN backward in both arms
    try:
        t = torch.arange(6, dtype=torch.float64, device=cuda)
        comm.allreduce_sum_(t)
        torch.cuda.synchronize()
        assert t.cpu().tolist() == [0.0, 1.0, 2.0, 3.0, 4.0, 5.0]
        g = torch.Generator().manual_seed(5)
        x = torch.randn(32, 3, 32, 32, generator=g).to(cuda)
        y = torch.randint(0, 100, (32,), generator=g).to(cuda)
        res = []
        for sync in (False, True):
            torch.manual_seed(42)
            model = dtc.ResNet18().to(cuda)
            if sync:
                model = dtc.SyncBatchNorm.convert_sync_batchnorm(model)
                model.set_sync_bn(comm)
            logits = model(x)
            dtc.CrossEntropyLoss()(logits, y).backward()
            torch.cuda.synchronize()
            res.append((logits.detach().cpu().numpy(), model.flat.grads.detach().cpu().numpy().copy(),
                        model.flat.bufs.detach().cpu().numpy().copy()))
            model.set_sync_bn(None)
        (l0, g0, b0), (l1, g1, b1) = res
        assert np.isfinite(g1).all() and np.abs(g1).sum() > 0
        np.testing.assert_array_equal(l1, l0)
        np.testing.assert_array_equal(g1, g0)
        np.testing.assert_array_equal(b1, b0)
    finally:
        dtc._native.lib.dtc_set_option(b"bn_cg", 1)
        comm.close()


@pytest.mark.parametrize("graphs", [1, 4])
def test_graph_exec_churn(dtc, cuda, graphs):
    """Graph-exec lifecycle under churn (the round-2 worker-thread crash must show up as a test
    failure if it recurs): every cycle changes an option (the next step drops and destroys the step graphs
    and re-captures them) and arms / disarms the live conv profile (the profiled graph set, the device
    drains under the capture lock), forward and backward replayed (graphs=1) or the default mode; every
    loss stays finite and every profiled pass records its conv launches."""
    import ctypes as C
    lib = dtc._native.lib
    torch.manual_seed(42)
    model = dtc.ResNet18().to(cuda)
    crit = dtc.CrossEntropyLoss()
    x = torch.randn(8, 3, 32, 32, device=cuda)
    y = torch.randint(0, 100, (8,), device=cuda)
    lib.dtc_set_option(b"graphs", graphs)
    try:
        crit(model(x), y).backward()
        exe = model.executor(8, 32, 32)
        for i in range(12):
            lib.dtc_set_option(b"sc_fuse", i % 2)
            loss = crit(model(x), y)
            loss.backward()
            assert np.isfinite(loss.item())
            dtc._native.call("dtc_rn18_profile_begin", exe.handle, 1)
            for _ in range(2):
                crit(model(x), y).backward()
            ms, fl, cnt = (C.c_double * 3)(), (C.c_double * 3)(), (C.c_int * 3)()
            dtc._native.call("dtc_rn18_profile_end", exe.handle, ms, fl, cnt)
            assert cnt[0] > 0 and cnt[1] > 0 and cnt[2] > 0, list(cnt)
        torch.cuda.synchronize()
    finally:
        lib.dtc_set_option(b"sc_fuse", 1)
        lib.dtc_set_option(b"graphs", 4)
