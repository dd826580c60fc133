"""Whole-network parity: the native executor vs the numpy oracle (oracle/resnet.py) on identical
seeded inputs and seed-42 parameters (north_star tolerances: per-layer activations and gradients
within 1e-2 relative in bf16)."""
import numpy as np
import pytest
import torch

from oracle import resnet as R
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu


def _setup(dtc, cuda, batch, seed=0):
    torch.manual_seed(42)
    model = dtc.ResNet18()
    sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    model = model.to(cuda)
    g = np.random.default_rng(seed)
    x = g.standard_normal((batch, 3, 32, 32)).astype(np.float32)
    y = g.integers(0, 100, batch)
    return model, sd, x, y


def _oracle_state(sd):
    params = {k: v for k, v in sd.items() if not (k.endswith("running_mean") or k.endswith("running_var")
                                                  or k.endswith("num_batches_tracked"))}
    bufs = {k: v for k, v in sd.items() if k.endswith("running_mean") or k.endswith("running_var")}
    return params, bufs


@pytest.mark.parametrize("batch", [2, 5])
def test_forward_backward_matches_oracle(dtc, cuda, batch):
    model, sd, x, y = _setup(dtc, cuda, batch)
    crit = dtc.CrossEntropyLoss()
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    logits = model(xd)
    loss = crit(logits, yd)
    loss.backward()
    torch.cuda.synchronize()
    params, bufs = _oracle_state(sd)
    ref = R.forward_backward(params, bufs, x, y, bf16_mode=True, train=True, want_acts=True)
    assert rel_err(logits.detach().cpu().numpy(), ref["logits"]) < 1e-2
    assert abs(float(loss) - ref["loss"]) < 1e-2 * max(1.0, abs(ref["loss"]))
    acts = model.executor(batch, 32, 32).activations()
    worst = {}
    for name, ra in ref["acts"].items():
        ka = acts[name].float().cpu().numpy()
        if name.startswith("stem.im2col"):
            continue
        worst[name] = rel_err(ka.reshape(ra.shape), ra)
    bad = {k: v for k, v in worst.items() if v > 1e-2}
    assert not bad, f"activations off: {bad}"
    gworst = {}
    for name, p in model.named_parameters():
        gworst[name] = rel_err(p.grad.detach().cpu().numpy(), ref["grads"][name])
    bad = {k: v for k, v in gworst.items() if v > 1e-2}
    assert not bad, f"gradients off: {sorted(bad.items(), key=lambda kv: -kv[1])[:10]}"
    # running statistics after one training forward
    sd2 = model.state_dict()
    for k, v in ref["buffers"].items():
        assert rel_err(sd2[k].cpu().numpy(), v) < 1e-3, k
    assert int(sd2["bn1.num_batches_tracked"]) == 1


def test_eval_mode_matches_oracle(dtc, cuda):
    model, sd, x, y = _setup(dtc, cuda, 4, seed=1)
    # give the running statistics non-trivial values
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
    params, bufs = _oracle_state(sd)
    ref = R.forward_backward(params, bufs, x, y, bf16_mode=True, train=False)
    assert rel_err(logits.cpu().numpy(), ref["logits"]) < 1e-2
    # eval must not touch the running statistics
    sd2 = model.state_dict()
    for k in bufs:
        np.testing.assert_array_equal(sd2[k].cpu().numpy(), sd[k])


def test_sgd_steps_track_oracle(dtc, cuda):
    """Three full training steps (forward, backward, Nesterov SGD) stay within bf16 tolerance."""
    model, sd, x, y = _setup(dtc, cuda, 4, seed=3)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    params, bufs = _oracle_state(sd)
    state = R.init_state(params, bufs)
    xd, yd = torch.from_numpy(x).to(cuda), torch.from_numpy(y).to(cuda)
    losses, ref_losses = [], []
    for _ in range(3):
        opt.zero_grad()
        loss = crit(model(xd), yd)
        loss.backward()
        opt.step()
        losses.append(float(loss))
        ref_losses.append(R.train_step(state, x, y, lr=0.1, bf16_mode=True))
    np.testing.assert_allclose(losses, ref_losses, rtol=2e-2)
    for name, p in model.named_parameters():
        assert rel_err(p.detach().cpu().numpy(), state["p"][name]) < 1e-2, name
    # the bf16 shadow equals the rounded master weights
    flat = model.flat
    np.testing.assert_array_equal(flat.params_bf16.float().cpu().numpy(),
                                  flat.params.bfloat16().float().cpu().numpy())
