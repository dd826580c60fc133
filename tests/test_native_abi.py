"""The C-ABI library loads and exports every symbol include/dtc.h declares; host-side planning
(layout, buckets, workspaces, conv plans) is consistent. No GPU compute here."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    text = open(os.path.join(ROOT, "include", "dtc.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dtc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(dtc):
    lib = dtc._native.lib
    names = _header_functions()
    assert len(names) >= 50
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding covers exactly the header
    assert sorted(dtc._native.SYMBOLS) == names


def test_abi_version_and_error_channel(dtc):
    lib = dtc._native.lib
    assert lib.dtc_abi_version() == 1
    rc = lib.dtc_rn18_create(None, 1, 32, 32, 100, 25.0)
    assert rc < 0
    assert "null" in dtc._native.last_error()
    h = C.c_void_p()
    assert lib.dtc_rn18_create(C.byref(h), 0, 32, 32, 100, 25.0) < 0  # bad batch -> invalid argument
    assert "bad shape" in dtc._native.last_error()


def test_layout_matches_module_tree(dtc):
    import torch
    torch.manual_seed(0)
    m = dtc.ResNet18()
    lay = dtc.nn.Layout()
    assert [p.name for p in lay.params] == [n for n, _ in m.named_parameters()]
    assert sum(p.numel for p in lay.params) == 11_220_132
    # reverse registration order, 64-element aligned, non-overlapping
    offs = [p.offset for p in lay.params]
    assert offs == sorted(offs, reverse=True)
    for p in lay.params:
        assert p.offset % 64 == 0
    spans = sorted((p.offset, p.offset + p.numel) for p in lay.params)
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    assert lay.flat_numel >= spans[-1][1] and lay.flat_numel % 64 == 0
    conv = {p.name: p for p in lay.params}["layer2.0.conv1.weight"]
    assert conv.shape == (128, 64, 3, 3) and conv.stride == (576, 1, 192, 64)  # KRSC storage
    assert [b.prefix for b in lay.bns][:3] == ["bn1", "layer1.0.bn1", "layer1.0.bn2"]
    assert len(lay.bns) == 20 and sum(b.channels for b in lay.bns) * 2 == 9600


@pytest.mark.parametrize("cap_mb", [1, 5, 25, 100, 1000])
def test_buckets_tile_the_gradient_buffer(dtc, cap_mb):
    lay = dtc.nn.Layout(100, cap_mb)
    pos = 0
    for off, n in lay.buckets:
        assert off == pos and n > 0
        pos += n
    assert pos == lay.flat_numel
    # every bucket closes at a block boundary at or above the cap, except the one open when layer2's
    # backward ends (option bucket_tail: closed there when >= 1 MB) and the last: at most layer1 + stem,
    # the unavoidable tail
    tail_start = min(p.offset for p in lay.params if p.name.startswith("layer1.") or p.name in
                     ("conv1.weight", "bn1.weight", "bn1.bias"))
    for off, n in lay.buckets[:-1]:
        assert n * 4 >= cap_mb * 2 ** 20 or off + n == tail_start
    assert lay.buckets[-1][0] >= tail_start and lay.buckets[-1][1] * 4 < 0.6 * 2 ** 20


def test_bucket_tail_option_restores_torch_cap_rule(dtc):
    """Option bucket_tail=0: buckets close only at the cap (torch DDP's rule); the last one is then
    whatever remains (100 MB cap: one 42.8 MB bucket, all of it issued after the stem)."""
    lib = dtc._native.lib
    try:
        lib.dtc_set_option(b"bucket_tail", 0)
        lay = dtc.nn.Layout(100, 100)
        assert len(lay.buckets) == 1 and lay.buckets[0][1] == lay.flat_numel
        lay = dtc.nn.Layout(100, 25)
        assert all(n * 4 >= 25 * 2 ** 20 for _, n in lay.buckets[:-1])
    finally:
        lib.dtc_set_option(b"bucket_tail", 1)
    # the first bucket starts with the head (linear.bias at offset 0): it is ready first
    names_at_0 = [p.name for p in lay.params if p.offset == 0]
    assert names_at_0 == ["linear.bias"]


def test_workspace_and_conv_plans(dtc):
    lib = dtc._native.lib
    h = C.c_void_p()
    dtc._native.call("dtc_rn18_create", C.byref(h), 256, 32, 32, 100, 25.0)
    ws = lib.dtc_rn18_workspace_bytes(h)
    assert 0.3e9 < ws < 3e9, ws
    assert lib.dtc_rn18_num_activations(h) == 2 + 8 * 4 + 3 + 1  # direct stem: no im2col image
    lib.dtc_rn18_destroy(h)
    d = dtc._native.ConvDesc(256, 4, 4, 512, 512, 3, 3, 1, 1)
    assert lib.dtc_conv2d_workspace_size(d, 2) > 0  # wgrad always wants split-K slabs
    d = dtc._native.ConvDesc(256, 32, 32, 64, 64, 3, 3, 1, 1)
    assert lib.dtc_conv2d_workspace_size(d, 0) == 0  # big layer: no split in forward
    # 224x224 (BASELINE config 5) plans too
    dtc._native.call("dtc_rn18_create", C.byref(h), 8, 224, 224, 100, 25.0)
    lib.dtc_rn18_destroy(h)
    # config 5 at its full per-GPU batch: 512 x 224 x 224 (activations > 2 GiB) plans and fits HBM
    dtc._native.call("dtc_rn18_create", C.byref(h), 512, 224, 224, 100, 25.0)
    ws = lib.dtc_rn18_workspace_bytes(h)
    assert 30e9 < ws < 200e9, ws  # well inside 288 GB
    lib.dtc_rn18_destroy(h)
    assert lib.dtc_rn18_create(C.byref(h), 700, 224, 224, 100, 25.0) < 0  # int32 element-index guard


@pytest.mark.parametrize("desc", [(8, 32, 32, 3, 64, 3, 3, 1, 1), (8, 32, 32, 64, 100, 3, 3, 1, 1),
                                  (8, 32, 32, 64, 64, 5, 5, 1, 2), (8, 32, 32, 64, 64, 3, 3, 3, 1),
                                  (0, 32, 32, 64, 64, 3, 3, 1, 1), (8, 1, 1, 64, 64, 3, 3, 1, 0)])
def test_conv_abi_rejects_unsupported_descriptors(dtc, desc):
    """Descriptors outside what the kernels implement (C or K not a multiple of 64, 5x5, stride 3, empty batch
    or output) are refused at the boundary: workspace queries return 0 and every conv entry point returns an
    error code with a message -- before any planning arithmetic (a C = 3 descriptor used to divide by C / 64 = 0
    in the workspace query: SIGFPE) and before any device call."""
    lib = dtc._native.lib
    d = dtc._native.ConvDesc(*desc)
    for p in range(3):
        assert lib.dtc_conv2d_workspace_size(d, p) == 0
    assert lib.dtc_conv2d_wgrad_sc_workspace_size(d) == 0
    assert lib.dtc_conv2d_wgrad_batch_workspace_size(d, 2) == 0
    one = C.c_void_p(16)
    assert lib.dtc_conv2d_fwd(d, one, one, one, None, None, 0, None) != 0
    assert b"unsupported convolution descriptor" in lib.dtc_last_error()
    assert lib.dtc_conv2d_dgrad(d, one, one, one, None, None, 0, None) != 0
    assert lib.dtc_conv2d_wgrad(d, one, one, one, C.c_float(1.0), one, 0, None) != 0


# executor / kernel options added by the round-2 performance work, with their defaults (kernels.h)
_OPTION_DEFAULTS = {
    "stem_bn_fuse": 1, "fork_lazy": 1, "side_prio": 1, "sc_fuse": 1, "stem_wlds": 1,
    "bn_red_elems": 16384, "bn_red_blocks": 256, "bn_fa_blocks": 1024,
    "sc_compact": 1, "stem_prologue": 1, "dgrad_class_order": 1, "wgrad_direct": 1, "wgrad_xcd": 1,
    # round 3
    "halo_s2": 1, "wgrad_s2": 1, "dgrad_scf": 1, "bucket_tail": 1, "wgrad_gen": 1,
    "halo_gen": 1, "bn_red_unroll": 4, "c64_gen": 1, "graphs": 4, "head_fused": 1,
    # round 4
    "bn_cg": 1, "bn_cg_elems": 262144, "wgrad_s2_wgs": 128, "comm_on_side": 1, "c64_wgs": 256, "wgrad_halo_l1": 0,
    # round 5
    "splitk_ink": 1, "comm_prio": 0, "comm_tail_inline": 1, "dgrad_s2h": 1, "halo_small": 1,
    # round 6
    "xent_fuse": 1, "wgrad_trim": 1,
}
# measured-negative variants deleted in rounds 4-6 with their code paths (DESIGN.md keeps their numbers)
_REMOVED_OPTIONS = ("bn_onepass", "sc_stream", "wgrad_defer", "stem_recompute", "wgrad_pmap", "wgrad_prio",
                    "halo_nhb2", "wgrad_kernel", "head_direct", "halo_nosplit", "graph_ev", "wgrad_tail",
                    "wgrad_stages", "wgrad_pf", "wgrad_diag",
                    # round 5
                    "bnb_mask", "bnb_fuse", "halo_stage_epi", "igemm_stages", "halo_l2pf", "dgrad_first", "wgrad_s2_ps", "c64_waves", "wgrad_early",
                    # round 6
                    "wgrad_ink", "wgrad_ink_max", "wgrad_ring", "wgrad_ksplit", "bn_in_conv", "amp_in_bwd",
                    "s2d_split", "s2d_wgs", "fork_ev", "wgrad_stagger",
                    "wgrad_setprio", "halo_setprio", "halo_xcd_cg", "c64_pf", "halo_wstages")


def test_options_registered_with_defaults(dtc):
    """dtc_set_option / dtc_get_option (host only): every option has its documented default, a set is
    read back, an unknown name is an error, and restoring leaves the default."""
    lib = dtc._native.lib
    for name, default in _OPTION_DEFAULTS.items():
        key = name.encode()
        assert lib.dtc_get_option(key) == default, name
        assert lib.dtc_set_option(key, default + 1) == 0
        assert lib.dtc_get_option(key) == default + 1
        assert lib.dtc_set_option(key, default) == 0
        assert lib.dtc_get_option(key) == default
    assert lib.dtc_set_option(b"no_such_option", 1) != 0
    for name in _REMOVED_OPTIONS:
        assert lib.dtc_set_option(name.encode(), 1) != 0, name


def test_kernels_keep_accumulators_out_of_scratch(dtc):
    """Every gfx950 kernel in the built library (tools/scratch_check.py reads the code objects' note
    metadata): at most a few spilled dwords of private segment. A runtime-indexed register array (e.g. an
    MFMA accumulator picked by a wave-dependent index) is placed in scratch instead -- hundreds of bytes per
    lane and an order of magnitude slower (the first wgrad_ksplit build: 608 B/lane, 10x) -- and is not
    reported as a spill by the compiler. Exempt: the 128 x 256 halo tile (a forced-option tuning
    configuration, 1 workgroup per CU, never planned by default)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scratch_check
    lib = os.path.join(ROOT, "distributed-training-comparison_amd", "_lib", "libdtc_amd.so")
    res = scratch_check.kernel_resources(lib)
    assert len(res) > 100
    bad = {k: v for k, v in res.items() if v[0] > 64 and "ELi128ELi256E" not in k}
    assert not bad, bad
    assert all(v[0] == 0 for k, v in res.items() if "wgrad_halo_kernel" in k)


def test_bn_stat_accumulator_host_decode(dtc):
    """The BN statistics accumulator format (common.h: exact int64 fixed point, 8 slots x (hi, lo), a
    header flag) read by the host decoder dtc_bn_stat_totals (pure host code, no GPU): totals encoded into
    slot 0 come back exactly when they have no bits below 2^-52; spreading a total over the slots (as the
    producers' atomic adds do, in any order) gives the same bits; the flag word makes every total NaN."""
    import numpy as np
    import torch

    c = 24
    rng = np.random.default_rng(3)
    s = np.round(rng.normal(0, 1e4, c) * 2.0 ** 20) / 2.0 ** 20  # multiples of 2^-20
    q = np.round(np.abs(rng.normal(0, 1e7, c)) * 2.0 ** 10) / 2.0 ** 10
    w = dtc.ops.stat_from_totals(s, q, "cpu")
    hdr = 2 * dtc._native.lib.dtc_bn_stat_words(1) - dtc._native.lib.dtc_bn_stat_words(2)
    slots = (dtc._native.lib.dtc_bn_stat_words(1) - hdr) // 4
    assert w.dtype == torch.int64 and w.numel() == dtc._native.lib.dtc_bn_stat_words(c) == hdr + slots * 4 * c
    assert hdr % 16 == 0 and slots == 8  # line-aligned rows (common.h)
    tot = dtc.ops.stat_totals(w, c).numpy()
    np.testing.assert_array_equal(tot[0], s)
    np.testing.assert_array_equal(tot[1], q)
    # split each total's integer words over the slots (hi and lo words add independently): same totals
    a = w.numpy().copy()
    spread = np.zeros_like(a)
    for j in range(4):  # (statistic, word) rows of slot 0
        row = a[hdr + j * c:hdr + (j + 1) * c]
        parts = [row // slots] * (slots - 1)
        parts.append(row - (slots - 1) * (row // slots))
        for k, part in enumerate(parts):
            spread[hdr + (k * 4 + j) * c:hdr + (k * 4 + j + 1) * c] = part
    tot2 = dtc.ops.stat_totals(torch.from_numpy(spread), c).numpy()
    np.testing.assert_array_equal(tot2, tot)
    spread[0] = 1  # a non-finite partial was seen
    assert np.isnan(dtc.ops.stat_totals(torch.from_numpy(spread), c).numpy()).all()
