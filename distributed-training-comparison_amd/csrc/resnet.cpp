// ResNet-18 (CIFAR variant) training-step executor.
//
// Mirrors the module structure of the reference (src/ddp/net.py:13-45 BasicBlock,
// net.py:86-116 ResNet, net.py:119-120 ResNet18) and runs its forward and backward as two
// calls that enqueue hand-written kernels on one stream:
//
//   forward : stem im2col -> conv(+BN stats) -> BN finalize -> BN+ReLU -> 8 BasicBlocks
//             [conv1 -> bn1+relu -> conv2 -> (shortcut conv) -> bn2 (+bn_sc) + add + relu]
//             -> global avg pool + Linear
//   backward: head -> blocks in reverse [BN2 reduce/finalize/apply -> conv2 wgrad/dgrad ->
//             BN1 ... -> conv1 wgrad/dgrad (+shortcut) with the residual gradient fused into
//             the dgrad epilogue] -> stem BN -> stem wgrad, issuing each gradient bucket's
//             RCCL all-reduce on the communicator's side stream as soon as it is complete.
//
// Parameter memory: one flat fp32 buffer in REVERSE registration order, 64-element aligned.
// Backward visits layers from the head to the stem, i.e. it finishes gradients in increasing
// address order, so every DDP bucket is a contiguous prefix-extension of the buffer.
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include "comm.h"
#include "kernels.h"

namespace dtc {

static inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

struct ParamEntry {
  std::string name;
  int64_t offset = 0, numel = 0;
  int ndim = 0;
  int64_t shape[4] = {0, 0, 0, 0};
  int64_t stride[4] = {0, 0, 0, 0};
};

struct ConvL {
  ConvShape s{};
  int P = 0, Q = 0;
  int pidx = -1;  // param index of the weight
};

struct BNL {
  std::string prefix;
  int C = 0;
  int gidx = -1, bidx = -1;  // param indices of weight (gamma) and bias (beta)
  int64_t rm_off = 0, rv_off = 0;
  int nbt = 0;
  size_t stats = 0, acc = 0, mean = 0, invstd = 0, scale = 0, shift = 0, coef = 0;  // workspace byte offsets
};

struct BlockL {
  ConvL c1, c2, sc;
  BNL b1, b2, bsc;
  bool proj = false;
  int Cin = 0, Cout = 0, Hin = 0, Win = 0, Hout = 0, Wout = 0;
  size_t C1 = 0, A1 = 0, C2 = 0, S = 0, OUT = 0;  // activation buffers (workspace byte offsets)
  size_t MA1 = 0, MOUT = 0;  // ReLU mask bits of A1 / OUT (bf16 executor, option bn_mask)
  size_t DC2 = 0, DC1 = 0, DSC = 0;  // backward: conv-output gradients read by the (side-stream) wgrads
  int64_t grad_hi = 0;  // end of this block's flat region: after its backward, [0, grad_hi) is complete
};

struct Net {
  int B = 0, H = 0, W = 0, ncls = 100;
  // fp32 mode (dtc_rn18_set_precision): fp32 activations, f32-MFMA convs, fp32 BN / head -- the
  // reference without --amp (ddp/trainer.py:160-165). Default: bf16 activations (autocast).
  bool f32 = false;
  size_t esz() const { return f32 ? 4 : 2; }
  std::vector<ParamEntry> params;
  int64_t flat_numel = 0;
  int64_t bufs_numel = 0;
  ConvL stem;
  BNL bn0;
  std::vector<BlockL> blocks;
  std::vector<BNL*> bns;  // registration order
  int fc_w = -1, fc_b = -1;
  // workspace
  size_t ws_bytes = 0;
  size_t X0 = 0, WSTEM = 0, C0 = 0, A0 = 0, FEAT = 0, G[6] = {0, 0, 0, 0, 0, 0}, SLAB = 0;
  size_t MA0 = 0;  // ReLU mask bits of A0
  size_t XIN = 0;  // executor-owned copy of the fp32 NCHW input (direct stem conv, bf16 mode)
  bool stem_direct = false;  // planned with option stem_direct (bf16): stem.hip instead of im2col + GEMM
  size_t HEADWS = 0, HEADWS_bytes = 0;
  size_t DC0 = 0, SLABW = 0;  // stem conv-output gradient; split-K slab of the side-stream wgrads
  size_t TICK = 0;            // split-K arrival counters of the compute stream's convs (the only in-kernel split-K)
  unsigned* tick(int i) { return (unsigned*)(ws + TICK) + (size_t)i * DTC_TICKS; }
  size_t BNERR = 0;           // int: set by a one-pass BN backward whose grid barrier timed out
  // backward weight gradients run on a side stream (option bwd_streams), overlapped with the
  // data-gradient / BN chain; forked after the conv-output gradient exists, joined at bucket points
  hipStream_t side_st = nullptr;
  hipStream_t sc_st = nullptr;  // the projection shortcut's conv (fwd) / dgrad branch (option sc_stream)
  bool sc_pending = false;
  std::vector<hipEvent_t> evs;
  int ev_next = 0;
  bool side_pending = false;
  size_t slab_bytes = 0;
  size_t stats_lo = 0, acc_lo = 0, stats_hi = 0;  // BN slot regions [stats_lo, acc_lo), [acc_lo, stats_hi)
  // the backward sums [acc_lo, stats_hi) are zeroed by every training forward; a backward that finds
  // them already used (a second backward over one forward) zeroes them first instead of adding onto
  // the previous backward's sums
  bool sums_fresh = false;
  // buckets: [offset, numel) in flat elements, and the block index after whose backward it fires
  std::vector<int64_t> bucket_off, bucket_len;
  std::vector<int> bucket_after_block;  // -1 = after the stem (last)
  // dtc_rn18_xent_backward with option xent_fuse: the CrossEntropyLoss backward's inputs, consumed by the
  // head backward kernel (one launch fewer after the per-step barrier); set only for that call
  XentArgs xent;
  // live conv timing (bench roofline): each conv call stamps min(start)/max(end) of its workgroups
  // (s_memrealtime) into its own slot; one kernel per step folds the slots into running totals.
  // Graph-safe: the slot pointers are baked at capture, nothing happens on the host per call.
  static constexpr int PROF_SLOTS = 256, PROF_BWD0 = 96;  // forward calls use [0,96), backward [96,256)
  bool profiling = false;
  // both in the caller-owned workspace (planned by plan_workspace): the slot pointers baked into the
  // profiled graphs stay valid for the executor's lifetime, so arming / disarming profiling neither
  // frees memory nor destroys graphs (it switches between the two graph sets below)
  size_t PROF_TS = 0, PROF_ACC = 0;
  u64* prof_ts = nullptr;   // [PROF_SLOTS][DTC_PROF_SLOT_U64] device
  u64* prof_acc = nullptr;  // [PROF_SLOTS][2] device: (sum ticks, calls)
  int prof_next = 0;
  int prof_kind[PROF_SLOTS] = {};
  double prof_flops[PROF_SLOTS] = {};
  int prof_khz = 100000;
  // event timing (dtc_rn18_profile_events; bench.py's roofline, the serialized eager step): every timed
  // launcher call is bracketed by two timing events on the compute stream -- its launch duration as a
  // rocprofv3 kernel trace of the same step sees it (dispatch to completion), summed per kind at the end
  bool prof_events = false;
  hipStream_t prof_st = nullptr;
  std::vector<hipEvent_t> prof_evpool;  // 2 per bracketed call, created up front
  size_t prof_evn = 0;                  // pairs used
  long long prof_evdropped = 0;         // calls that found the pool used up (not bracketed: reported)
  std::vector<std::pair<int, double>> prof_evwork;  // (kind, work) per pair
  // communication timing (dtc_rn18_comm_timing; bench.py's comm_exposed_us / buckets_us at N > 1): for the
  // next ct_left backward calls with a communicator, timing events on the streams the work runs on -- the
  // backward's start (compute stream), each bucket collective's start / end (its own stream), the compute
  // stream's wait for the weight-gradient stream before the stem weight gradient (join_c -> join_d), and the
  // tail from the last backward kernel to the Reducer's join (tail_a -> tail_b)
  struct CommTimes {
    hipEvent_t bwd0 = nullptr, join_c = nullptr, join_d = nullptr, tail_a = nullptr, tail_b = nullptr;
    std::vector<hipEvent_t> b0, b1;  // per bucket
    bool join = false, tail = false;  // join_c / join_d, tail_a recorded (eager backward)
    bool ok = false;                  // the backward succeeded and recorded tail_b (only these steps count)
    std::vector<bool> bucket;        // bucket i recorded
  };
  std::vector<CommTimes> ct;  // one per armed step
  int ct_left = 0, ct_used = 0;
  CommTimes* ct_cur = nullptr;  // the set of the backward in progress (null: not timed)
  // hipGraph replay (option "graphs"): the forward per train flag, the backward as segments split
  // at bucket boundaries (the all-reduces stay eager on the communicator's side stream)
  struct Seg { hipGraphExec_t exec = nullptr; std::vector<int> buckets; };
  hipStream_t cap_st = nullptr;
  bool cap_locked = false;  // this executor holds g_graph_mu (between begin_capture and end_capture)
  int graph_epoch = -1;
  // graph sets indexed [profiling]: the profiled set carries the timing stamps and the per-step fold
  hipGraphExec_t fwd_exec[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [profiling][train]
  std::vector<Seg> bwd_segs[2];
  float bwd_gs[2] = {0.f, 0.f};
  bool bwd_comm[2] = {false, false};
  // recorded on the launch stream after every graph launch: drop_graphs waits for it before destroying
  hipEvent_t launch_ev = nullptr;
  bool launched = false;
  size_t LOGITS = 0, DLOGITS = 0;  // graph-owned copies of the caller's logits / dlogits
  // activation registry (per-layer parity): name, workspace byte offset, N,H,W,C
  struct Act { std::string name; size_t off; int n, h, w, c; };
  std::vector<Act> acts;
  // optional capture of backward intermediates (parity tests): name -> slot in the workspace
  bool capture = false;
  // SyncBatchNorm: per-channel BN sums all-reduced over this communicator
  // (its own, never the Reducer's, so the two collective streams cannot interleave on one comm)
  Comm* sync = nullptr;
  int sync_world = 1;
  std::vector<Act> caps;
  // bound memory
  char* ws = nullptr;
  float* p = nullptr;
  float* g = nullptr;
  u16* pb = nullptr;
  float* bufs = nullptr;
  int64_t* nbt = nullptr;

  template <typename T>
  T* at(size_t off) const { return (T*)(ws + off); }
  const u16* wbf(int pidx) const { return pb + params[pidx].offset; }
  float* pf(int pidx) const { return p + params[pidx].offset; }
  float* gf(int pidx) const { return g + params[pidx].offset; }
};

// ------------------------------------------------------------------ construction
static int add_param(Net& n, const std::string& name, std::vector<int64_t> shape, bool conv_krsc) {
  ParamEntry e;
  e.name = name;
  e.ndim = (int)shape.size();
  e.numel = 1;
  for (int i = 0; i < e.ndim; ++i) {
    e.shape[i] = shape[i];
    e.numel *= shape[i];
  }
  if (conv_krsc) {  // logical [K][C][R][S] stored as K R S C
    const int64_t K = shape[0], C = shape[1], R = shape[2], S = shape[3];
    (void)K;
    e.stride[0] = R * S * C;
    e.stride[1] = 1;
    e.stride[2] = S * C;
    e.stride[3] = C;
  } else {
    int64_t s = 1;
    for (int i = e.ndim - 1; i >= 0; --i) {
      e.stride[i] = s;
      s *= shape[i];
    }
  }
  n.params.push_back(e);
  return (int)n.params.size() - 1;
}

static void make_conv(Net& n, ConvL& c, const std::string& name, int N, int H, int W, int Cin, int Cout, int k,
                      int stride) {
  c.s = ConvShape{N, H, W, Cin, Cout, k, k, stride, k == 3 ? 1 : 0};
  c.P = (H + 2 * c.s.pad - k) / stride + 1;
  c.Q = (W + 2 * c.s.pad - k) / stride + 1;
  c.pidx = add_param(n, name, {Cout, Cin, k, k}, true);
}

static void make_bn(Net& n, BNL& b, const std::string& prefix, int C) {
  b.prefix = prefix;
  b.C = C;
  b.gidx = add_param(n, prefix + ".weight", {C}, false);
  b.bidx = add_param(n, prefix + ".bias", {C}, false);
}

static int build(Net& n) {
  const int B = n.B;
  // stem: registered as conv1.weight [64,3,3,3], bn1.{weight,bias}   (net.py:91-92)
  n.stem.s = ConvShape{B, n.H, n.W, 64, 64, 1, 1, 1, 0};  // GEMM over the 64-column im2col image
  n.stem.P = n.H;
  n.stem.Q = n.W;
  n.stem.pidx = add_param(n, "conv1.weight", {64, 3, 3, 3}, true);
  make_bn(n, n.bn0, "bn1", 64);
  // layers (net.py:93-96, _make_layer net.py:99-105)
  int in_planes = 64, H = n.H, W = n.W;
  const int planes[4] = {64, 128, 256, 512};
  const int strides[4] = {1, 2, 2, 2};
  for (int L = 0; L < 4; ++L) {
    for (int bi = 0; bi < 2; ++bi) {
      const int stride = bi == 0 ? strides[L] : 1;
      BlockL blk;
      const std::string pre = "layer" + std::to_string(L + 1) + "." + std::to_string(bi);
      blk.Cin = in_planes;
      blk.Cout = planes[L];
      blk.Hin = H;
      blk.Win = W;
      make_conv(n, blk.c1, pre + ".conv1.weight", B, H, W, in_planes, planes[L], 3, stride);
      make_bn(n, blk.b1, pre + ".bn1", planes[L]);
      blk.Hout = blk.c1.P;
      blk.Wout = blk.c1.Q;
      make_conv(n, blk.c2, pre + ".conv2.weight", B, blk.Hout, blk.Wout, planes[L], planes[L], 3, 1);
      make_bn(n, blk.b2, pre + ".bn2", planes[L]);
      blk.proj = (stride != 1 || in_planes != planes[L]);  // net.py:28
      if (blk.proj) {
        make_conv(n, blk.sc, pre + ".shortcut.0.weight", B, H, W, in_planes, planes[L], 1, stride);
        make_bn(n, blk.bsc, pre + ".shortcut.1", planes[L]);
      }
      n.blocks.push_back(blk);
      in_planes = planes[L];
      H = blk.Hout;
      W = blk.Wout;
    }
  }
  n.fc_w = add_param(n, "linear.weight", {n.ncls, 512}, false);  // net.py:97
  n.fc_b = add_param(n, "linear.bias", {n.ncls}, false);
  if (H < 1 || W < 1) return set_error(DTC_EINVAL, "rn18: input %dx%d too small", n.H, n.W);

  // flat layout: reverse registration order, 64-element alignment
  int64_t off = 0;
  for (int i = (int)n.params.size() - 1; i >= 0; --i) {
    n.params[i].offset = off;
    off = align_up(off + n.params[i].numel, 64);
  }
  n.flat_numel = off;

  // BN registry in registration order and buffer layout
  n.bns.push_back(&n.bn0);
  for (auto& b : n.blocks) {
    n.bns.push_back(&b.b1);
    n.bns.push_back(&b.b2);
    if (b.proj) n.bns.push_back(&b.bsc);
  }
  int64_t boff = 0;
  for (size_t i = 0; i < n.bns.size(); ++i) {
    BNL* b = n.bns[i];
    b->rm_off = boff;
    boff = align_up(boff + b->C, 64);
    b->rv_off = boff;
    boff = align_up(boff + b->C, 64);
    b->nbt = (int)i;
  }
  n.bufs_numel = boff;
  for (auto& b : n.blocks)  // conv1.weight is the block's first-registered, hence highest, param
    b.grad_hi = align_up(n.params[b.c1.pidx].offset + n.params[b.c1.pidx].numel, 64);
  return 0;
}

// fp32 stem: a 1x1 "conv" over the 32-column fp32 im2col image (27 taps + 5 zero columns)
static ConvShape f32_stem_shape(const Net& n) { return ConvShape{n.B, n.H, n.W, 32, 64, 1, 1, 1, 0}; }

static void plan_workspace(Net& n, float bucket_cap_mb) {
  n.acts.clear();
  n.caps.clear();
  n.bucket_off.clear();
  n.bucket_len.clear();
  n.bucket_after_block.clear();
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = (size_t)align_up((int64_t)(off + bytes), 256);
    return o;
  };
  const int64_t B = n.B;
  const int64_t M0 = B * n.H * n.W;
  const size_t E = n.esz();
  n.stem_direct = !n.f32 && option_get(OPT_STEM_DIRECT) != 0;
  n.XIN = n.stem_direct ? take(M0 * 3 * 4) : 0;
  n.X0 = n.stem_direct ? 0 : take(M0 * 64 * 2);  // im2col: [M0][64] bf16 or [M0][32] fp32
  n.WSTEM = take(64 * 64 * 2);
  n.C0 = take(M0 * 64 * E);
  n.A0 = take(M0 * 64 * E);
  n.MA0 = take(M0 * 64 / 8);
  int64_t gmax = M0 * 64;
  for (auto& b : n.blocks) {
    const int64_t M = B * b.Hout * b.Wout;
    const size_t bytes = M * b.Cout * E;
    b.C1 = take(bytes);
    b.A1 = take(bytes);
    b.C2 = take(bytes);
    if (b.proj) b.S = take(bytes);
    b.OUT = take(bytes);
    b.MA1 = take(M * b.Cout / 8);
    b.MOUT = take(M * b.Cout / 8);
    gmax = std::max<int64_t>(gmax, std::max<int64_t>(M * b.Cout, B * b.Hin * b.Win * b.Cin));
  }
  if (!n.stem_direct) n.acts.push_back({"stem.im2col", n.X0, (int)B, n.H, n.W, 64});
  n.acts.push_back({"stem.conv", n.C0, (int)B, n.H, n.W, 64});
  n.acts.push_back({"stem.out", n.A0, (int)B, n.H, n.W, 64});
  for (size_t i = 0; i < n.blocks.size(); ++i) {
    const BlockL& b = n.blocks[i];
    const std::string pre = "layer" + std::to_string(i / 2 + 1) + "." + std::to_string(i % 2);
    n.acts.push_back({pre + ".conv1", b.C1, (int)B, b.Hout, b.Wout, b.Cout});
    n.acts.push_back({pre + ".relu1", b.A1, (int)B, b.Hout, b.Wout, b.Cout});
    n.acts.push_back({pre + ".conv2", b.C2, (int)B, b.Hout, b.Wout, b.Cout});
    if (b.proj) n.acts.push_back({pre + ".shortcut", b.S, (int)B, b.Hout, b.Wout, b.Cout});
    n.acts.push_back({pre + ".out", b.OUT, (int)B, b.Hout, b.Wout, b.Cout});
  }
  n.FEAT = take(B * 512 * 4);
  n.LOGITS = take(B * n.ncls * 4);
  n.DLOGITS = take(B * n.ncls * 4);
  n.HEADWS_bytes = head_bwd_workspace((int)B, 512, n.ncls);
  n.HEADWS = take(n.HEADWS_bytes);
  n.acts.push_back({"head.feat_f32", n.FEAT, (int)B, 1, 1, 512});
  for (int i = 0; i < 6; ++i) n.G[i] = take(gmax * E);
  for (auto& b : n.blocks) {  // per-block, so a pending side-stream wgrad never sees them overwritten
    const size_t bytes = (size_t)B * b.Hout * b.Wout * b.Cout * E;
    b.DC2 = take(bytes);
    b.DC1 = take(bytes);
    if (b.proj) b.DSC = take(bytes);
  }
  n.DC0 = take(M0 * 64 * E);
  // BN per-layer state
  n.PROF_TS = take((size_t)Net::PROF_SLOTS * DTC_PROF_SLOT_U64 * sizeof(u64));
  n.PROF_ACC = take((size_t)Net::PROF_SLOTS * 2 * sizeof(u64));
  n.stats_lo = off;  // forward statistics of every BN, then backward sums: both zeroed by the training forward
  for (BNL* b : n.bns) b->stats = take(DTC_STAT_WORDS(b->C) * 8);
  n.acc_lo = off;
  for (BNL* b : n.bns) b->acc = take(DTC_STAT_WORDS(b->C) * 8);
  n.BNERR = take(256);
  n.stats_hi = off;
  for (BNL* b : n.bns) {
    b->mean = take(b->C * 4);
    b->invstd = take(b->C * 4);
    b->scale = take(b->C * 4);
    b->shift = take(b->C * 4);
    b->coef = take(3 * b->C * 4);
  }
  // split-K slabs: max over every conv pass
  size_t slab = (size_t)64 * 64 * 4;
  auto consider = [&](const ConvShape& s) {
    for (int m = 0; m < 3; ++m)
      slab = std::max(slab, n.f32 ? f32_conv_workspace(s, m) : plan_conv(s, m).slab_bytes);
  };
  consider(n.f32 ? f32_stem_shape(n) : n.stem.s);
  for (auto& b : n.blocks) {
    consider(b.c1.s);
    consider(b.c2.s);
    if (b.proj) consider(b.sc.s);
    if (!n.f32)
      for (int np = 2; np <= DTC_WG_BATCH; ++np) {
        slab = std::max(slab, conv_wgrad_batch_slab_bytes(b.c1.s, np));
        slab = std::max(slab, conv_wgrad_batch_slab_bytes(b.c2.s, np));
      }
    if (!n.f32 && b.proj) slab = std::max(slab, conv_wgrad_s2_slab_bytes(b.c1.s));  // conv1 + shortcut wgrad (wgrad_s2)
  }
  if (n.stem_direct) slab = std::max(slab, stem_wgrad_slab_bytes(M0));
  n.slab_bytes = slab;
  n.SLAB = take(slab);
  n.SLABW = take(slab);
  n.TICK = take((size_t)DTC_TICKS * 4);  // zeroed at bind; every in-kernel split-K leaves its counters zero
  if (n.capture) {
    auto cap = [&](const std::string& nm, int h, int w, int c) {
      n.caps.push_back({nm, take((size_t)B * h * w * c * E), (int)B, h, w, c});
    };
    for (size_t i = 0; i < n.blocks.size(); ++i) {
      const BlockL& b = n.blocks[i];
      const std::string pre = "grad.layer" + std::to_string(i / 2 + 1) + "." + std::to_string(i % 2);
      for (const char* k : {".dy", ".dz", ".dc2", ".da1", ".dz1", ".dc1"}) cap(pre + k, b.Hout, b.Wout, b.Cout);
      if (b.proj) {
        cap(pre + ".ds", b.Hout, b.Wout, b.Cout);
        cap(pre + ".dxs", b.Hin, b.Win, b.Cin);
      }
      cap(pre + ".dx", b.Hin, b.Win, b.Cin);
    }
    cap("grad.stem.dz", n.H, n.W, 64);
    cap("grad.stem.dc", n.H, n.W, 64);
  }
  n.ws_bytes = off;

  // gradient buckets at block granularity in backward order (head + layer4.1 first); a bucket
  // closes once it holds >= bucket_cap_mb (torch DDP's rule). Option bucket_tail (default 1; a
  // deviation from torch's cap semantics, reported in the bench line's buckets_mb): whatever is open
  // when layer2's backward ends also closes there if it is >= 1 MB, so the last bucket -- issued after
  // the stem, overlapping nothing -- is only layer1 + the stem (0.6 MB, the unavoidable tail of SURVEY
  // A.2) instead of up to the whole cap
  const int64_t cap = (int64_t)(bucket_cap_mb * 1024.0 * 1024.0 / 4.0);
  const bool tail_split = option_get(OPT_BUCKET_TAIL) != 0;
  int64_t start = 0;
  for (int bi = (int)n.blocks.size() - 1; bi >= 0 && cap > 0; --bi) {
    const int64_t hi = n.blocks[bi].grad_hi;
    const bool tail_edge = tail_split && bi == 2 && n.blocks.size() == 8;  // layer2.0: next come layer1 and the stem
    if (hi - start >= cap || (tail_edge && (hi - start) * 4 >= (1 << 20))) {
      n.bucket_off.push_back(start);
      n.bucket_len.push_back(hi - start);
      n.bucket_after_block.push_back(bi);
      start = hi;
    }
  }
  n.bucket_off.push_back(start);
  n.bucket_len.push_back(n.flat_numel - start);
  n.bucket_after_block.push_back(-1);
}

// ------------------------------------------------------------------ profiling helpers
static double conv_flops(const ConvShape& s) {
  const int P = (s.H + 2 * s.pad - s.R) / s.stride + 1, Q = (s.W + 2 * s.pad - s.S) / s.stride + 1;
  return 2.0 * s.N * P * Q * (double)s.K * s.R * s.S * s.C;
}
// kinds: 0 conv forward, 1 conv dgrad, 2 conv wgrad (work = algorithmic FLOPs), 3 BN family (work =
// algorithmic HBM bytes: the tensors each BN kernel must read / write once)
static u64* prof_slot(Net& n, int kind, double flops) {
  if (!n.profiling || n.prof_next >= Net::PROF_SLOTS) return nullptr;
  const int i = n.prof_next++;
  n.prof_kind[i] = kind;
  n.prof_flops[i] = flops;
  return n.prof_ts + (size_t)i * DTC_PROF_SLOT_U64;
}
static bool side_on(const Net& n);
// event bracket of one launcher call (-1: not recorded -- events off, a capture in progress, the weight
// gradients on a side stream the compute-stream events would not cover, or the pool used up)
static int prof_ev_open(Net& n, int kind, double work) {
  // (prof_st may be the null stream: the caller's default stream)
  if (!n.profiling || !n.prof_events || n.cap_locked || side_on(n)) return -1;
  if (n.prof_evn * 2 + 1 >= n.prof_evpool.size()) {  // pool used up: counted, so the caller can refuse the total
    ++n.prof_evdropped;
    return -1;
  }
  const int i = (int)n.prof_evn++;
  if (n.prof_evwork.size() < n.prof_evn) n.prof_evwork.resize(n.prof_evn);
  n.prof_evwork[i] = {kind, work};
  if (hipEventRecord(n.prof_evpool[2 * i], n.prof_st) != hipSuccess) return -1;
  return i;
}
static void prof_ev_close(Net& n, int i) {
  if (i >= 0) (void)hipEventRecord(n.prof_evpool[2 * i + 1], n.prof_st);
}
#define PROF(kind, flops, call)                        \
  do {                                                 \
    u64* ts = prof_slot(n, (kind), (flops));           \
    const int pev_ = prof_ev_open(n, (kind), (flops)); \
    const int prc_ = (call);                           \
    prof_ev_close(n, pev_);                            \
    DTC_TRY(prc_);                                     \
  } while (0)

// ------------------------------------------------------------------ graph capture helpers
// Process-wide: graph capture (begin_capture .. end_capture) and graph destruction (drop_graphs: a device
// drain + hipGraphExecDestroy) are serialised across host threads. Several executors driven by one thread
// each (the thread-group communicator's W ranks in one process) otherwise capture and drain at the same
// time: a device drain while another thread's stream is capturing crashed the HIP runtime (segfault in
// the first backward of test_gpu_ddp_group's graphs-on case). Capture happens once per executor and
// option epoch, so the lock costs nothing per step; no collective is issued inside a captured region
// (bucket all-reduces run between the replayed segments), so a rank holding it never waits on another.
static std::recursive_mutex g_graph_mu;

static void drop_graphs(Net& n) {
  std::lock_guard<std::recursive_mutex> lk(g_graph_mu);
  // An exec may still be running (the caller's previous step is asynchronous). Round 2 saw a rare
  // crash in a HIP runtime thread (no Python frame) when execs were destroyed right after a device
  // drain and the profiling slots their kernels stamp were freed next (dtc_rn18_profile_end). The
  // slots now live in the workspace (never freed while an exec exists) and an exec is destroyed only
  // after (1) the event recorded behind its LAST launch on the launch stream has completed -- the
  // runtime has retired every command of that launch, in stream order -- and (2) a device drain.
  bool any = false;
  for (auto& set : n.fwd_exec)
    for (auto e : set) any = any || e != nullptr;
  for (auto& v : n.bwd_segs) any = any || !v.empty();
  if (!any) return;
  if (n.launched && n.launch_ev) (void)hipEventSynchronize(n.launch_ev);
  (void)hipDeviceSynchronize();
  for (auto& set : n.fwd_exec)
    for (auto& e : set)
      if (e) {
        (void)hipGraphExecDestroy(e);
        e = nullptr;
      }
  for (auto& v : n.bwd_segs) {
    for (auto& sg : v)
      if (sg.exec) (void)hipGraphExecDestroy(sg.exec);
    v.clear();
  }
  n.launched = false;
}
static int graph_launch(Net& n, hipGraphExec_t ex, hipStream_t st) {
  DTC_HIP(hipGraphLaunch(ex, st));
  // drop_graphs waits on this event (the exec's last launch retired) before destroying an exec
  if (!n.launch_ev) DTC_HIP(hipEventCreateWithFlags(&n.launch_ev, hipEventDisableTiming));
  DTC_HIP(hipEventRecord(n.launch_ev, st));
  n.launched = true;
  return 0;
}
// option graphs: 0 = eager launches, 1 = forward and backward replayed from hipGraphs, 2 = forward only,
// 3 = backward only, 4 (default) = eager launches -- except the backward with a communicator whose bucket
// collectives run on a stream of their own (comm_on_side=0: segment graphs, host-issued collectives between
// them). Measured (tools/bench_ab.sh, one MI355X, images/s): the replayed backward is slower than eager at
// every batch (no communicator: B=256 +4-5% eager (r03), B=64 52.8k -> 59.9k (r04j); with a communicator on
// the weight-gradient stream, loopback r04g / r04h: B=256 116.1k -> 125.9k, 128 78.3k -> 87.7k, 64 49.5k ->
// 57.0k, 32 27.0k -> 31.1k), and since the round-4 host-path changes the replayed forward is no faster
// either (r04s, 3 rounds: B=256 132.5k -> 133.9k eager, B=128 93.0k / 93.2k, B=64 59.9k / 60.2k; r04r: B=32
// 33.9k -> 34.3k, with a communicator 32.3k -> 32.8k): a graph launch's host cost and the ~14 us completion
// gap behind it outweigh the launches it saves (`bwd`: which segment asks; `comm`: it has a communicator)
static bool graphs_on(Net& n, bool bwd, bool comm = false) {
  const int g = option_get(OPT_GRAPHS);
  if (n.capture || n.sync || g == 0 || (g == 2 && bwd) || (g == 3 && !bwd)) return false;
  if (g == 4 && (!bwd || !(comm && option_get(OPT_COMM_ON_SIDE) == 0))) return false;
  if (n.graph_epoch != option_epoch()) {  // options are baked into captured launches
    drop_graphs(n);
    n.graph_epoch = option_epoch();
  }
  return true;
}
static int begin_capture(Net& n) {
  g_graph_mu.lock();  // released by the matching end_capture (or here on failure)
  n.cap_locked = true;
  hipError_t e = hipSuccess;
  if (!n.cap_st) e = hipStreamCreateWithFlags(&n.cap_st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamBeginCapture(n.cap_st, hipStreamCaptureModeRelaxed);
  if (e != hipSuccess) {
    n.cap_locked = false;
    g_graph_mu.unlock();
    return set_error((int)e, "begin capture: %s", hipGetErrorString(e));
  }
  return 0;
}
// Ends the capture on n.cap_st (always, also when the captured body failed); *out stays null
// for an empty capture.
static int end_capture_locked(Net& n, int body_rc, hipGraphExec_t* out) {
  *out = nullptr;
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(n.cap_st, &g);
  if (body_rc != 0 || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    return body_rc != 0 ? body_rc : set_error((int)e, "hipStreamEndCapture: %s", hipGetErrorString(e));
  }
  size_t nodes = 0;
  e = hipGraphGetNodes(g, nullptr, &nodes);
  if (e == hipSuccess && nodes > 0) e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return set_error((int)e, "graph instantiate: %s", hipGetErrorString(e));
  return 0;
}
static int end_capture(Net& n, int body_rc, hipGraphExec_t* out) {
  if (!n.cap_locked) {  // begin_capture failed (a segment boundary inside the backward): nothing open
    *out = nullptr;
    return body_rc != 0 ? body_rc : set_error(DTC_EINVAL, "end_capture without an open capture");
  }
  const int rc = end_capture_locked(n, body_rc, out);
  n.cap_locked = false;
  g_graph_mu.unlock();  // taken by begin_capture
  return rc;
}

// ------------------------------------------------------------------ forward / backward
static int bn_finalize_fwd(Net& n, BNL& b, int64_t count, bool train, hipStream_t st) {
  if (train) {
    return bn_fwd_finalize(n.at<int64_t>(b.stats), b.C, count, n.pf(b.gidx), n.pf(b.bidx), n.bufs + b.rm_off,
                           n.bufs + b.rv_off, n.nbt ? n.nbt + b.nbt : nullptr, 0.1f, 1e-5f, n.at<float>(b.mean),
                           n.at<float>(b.invstd), n.at<float>(b.scale), n.at<float>(b.shift), st);
  }
  return bn_eval_coef(b.C, n.pf(b.gidx), n.pf(b.bidx), n.bufs + b.rm_off, n.bufs + b.rv_off, 1e-5f,
                      n.at<float>(b.mean), n.at<float>(b.invstd), n.at<float>(b.scale), n.at<float>(b.shift), st);
}

static bool bn_fused() { return option_get(OPT_BN_FUSED_FIN) != 0; }
// Mask-bit BN backward (option bn_mask, default on): the training forward's fused BN apply also
// writes the ReLU mask of its output as bits, and the backward forms dz = dy * bit where it needs it
// instead of reading the bf16 output (2 B) and storing / re-reading dz (4 B) per element.
static bool bn_mask_on(const Net& n) {
  return !n.f32 && option_get(OPT_BN_MASK) != 0 && bn_fused();
}

// SUM all-reduce of one BN's statistic accumulator (exact int64 fixed point, common.h) on the compute
// stream: the slots are first folded into slot 0 (the others zeroed), so the collective carries the
// header (the non-finite flag) and slot 0, DTC_STAT_HDR + 4*C words, not every slot; integer sums make
// the global totals independent of the ranks' order too. Every apply kernel folds the slots, so after
// this each rank folds the global sums (torch SyncBatchNorm's all-gather of per-rank mean/invstd/count,
// as one reduction; every rank's batch is the same size -- checked by the Python DDP wrapper).
static int sync_bn_sums(Net& n, size_t off, int C, hipStream_t st) {
  DTC_TRY(bn_fold_slots(n.at<int64_t>(off), C, st));
  return comm_allreduce(n.sync, n.ws + off, (size_t)DTC_STAT_HDR + (size_t)4 * C, 2, st);
}

static BnFwdArgs fwd_args(Net& n, BNL& b, int64_t count) {
  BnFwdArgs a;
  a.stats = n.at<int64_t>(b.stats);
  a.count = count;
  a.gamma = n.pf(b.gidx);
  a.beta = n.pf(b.bidx);
  a.rmean = n.bufs + b.rm_off;
  a.rvar = n.bufs + b.rv_off;
  a.nbt = n.nbt ? n.nbt + b.nbt : nullptr;
  a.mean = n.at<float>(b.mean);
  a.invstd = n.at<float>(b.invstd);
  return a;
}

// BN (+ residual / second BN) + ReLU after the producing conv(s): y = relu(bn(x) [+ x2 | + bn2(x2)])
static int bn_act(Net& n, int mode, BNL& b, const u16* x, BNL* b2, const u16* x2, u16* y, int64_t M, bool train,
                  hipStream_t st, size_t mask_off = 0) {
  if (train && n.sync) {  // SyncBN: global per-channel (sum, sumsq) slots, global element count
    DTC_TRY(sync_bn_sums(n, b.stats, b.C, st));
    if (b2) DTC_TRY(sync_bn_sums(n, b2->stats, b2->C, st));
  }
  const int64_t cnt = train && n.sync ? M * n.sync_world : M;  // elements behind each channel's stats
  if (train && bn_fused()) {
    const BnFwdArgs a1 = fwd_args(n, b, cnt);
    const BnFwdArgs a2 = b2 ? fwd_args(n, *b2, cnt) : BnFwdArgs{};
    uint8_t* mask = bn_mask_on(n) && mask_off ? n.at<uint8_t>(mask_off) : nullptr;
    const double work = (double)M * b.C * (4.0 + (mode != 1 ? 2.0 : 0.0) + (mask ? 0.125 : 0.0));
    u64* ts = prof_slot(n, 3, work);
    const int ev = prof_ev_open(n, 3, work);
    const int rc = bn_fin_apply(mode, x, a1, x2, b2 ? &a2 : nullptr, y, M, b.C, st, mask, ts);
    prof_ev_close(n, ev);
    return rc;
  }
  DTC_TRY(bn_finalize_fwd(n, b, cnt, train, st));
  if (b2) DTC_TRY(bn_finalize_fwd(n, *b2, cnt, train, st));
  const float* s1 = n.at<float>(b.scale);
  const float* h1 = n.at<float>(b.shift);
  if (mode == 1) return bn_apply_relu(x, s1, h1, y, M, b.C, st);
  if (mode == 2) return bn_apply_add_relu(x, s1, h1, x2, y, M, b.C, st);
  return bn_apply_dual_relu(x, s1, h1, x2, n.at<float>(b2->scale), n.at<float>(b2->shift), y, M, b.C, st);
}

static ConvShape f32_stem_shape(const Net& n);
static int forward_body_f32(Net& n, float* logits, bool train, hipStream_t st);

// everything after the input im2col (reads only executor-owned memory: capturable)
static int forward_head(Net& n, float* logits, hipStream_t st) {
  const BlockL& last = n.blocks.back();
  return head_fwd(n.at<u16>(last.OUT), n.B, last.Hout * last.Wout, 512, n.wbf(n.fc_w), n.pf(n.fc_b), n.ncls,
                  n.at<float>(n.FEAT), logits, st);
}

static int forward_body(Net& n, float* logits, bool train, hipStream_t st) {
  if (n.f32) return forward_body_f32(n, logits, train, st);
  const int64_t M0 = (int64_t)n.B * n.H * n.W;
  n.prof_next = train ? 0 : Net::PROF_SLOTS;  // eval passes are not timed
  // the forward statistics AND the backward sums of every BN (the backward that follows this training
  // forward accumulates into zeroed slots; its graph then starts with real work, no memset node) --
  // done by forward()'s input-copy launch on the direct-stem path
  if (train && !n.stem_direct) DTC_TRY(zero_bytes(n.ws + n.stats_lo, n.stats_hi - n.stats_lo, st));
  if (n.stem_direct) {  // stem.hip: taps gathered per tile from the fp32 input, one K=32 k-step
    PROF(0, 2.0 * M0 * 64 * 27,
         stem_fwd(n.at<float>(n.XIN), n.wbf(n.stem.pidx), n.at<u16>(n.C0), train ? n.at<int64_t>(n.bn0.stats) : nullptr,
                  n.B, n.H, n.W, st, ts));
  } else {
    DTC_TRY(stem_pack_weight(n.wbf(n.stem.pidx), n.at<u16>(n.WSTEM), 64, st));
    PROF(0, 2.0 * M0 * 64 * 27,
         conv_fwd(n.stem.s, n.at<u16>(n.X0), n.at<u16>(n.WSTEM), n.at<u16>(n.C0),
                  train ? n.at<int64_t>(n.bn0.stats) : nullptr, n.at<float>(n.SLAB), n.slab_bytes, st, ts));
  }
  DTC_TRY(bn_act(n, 1, n.bn0, n.at<u16>(n.C0), nullptr, nullptr, n.at<u16>(n.A0), M0, train, st, n.MA0));
  const u16* in = n.at<u16>(n.A0);
  n.ev_next = 0;
  for (auto& b : n.blocks) {
    const int64_t M = (int64_t)n.B * b.Hout * b.Wout;
    float* slab = n.at<float>(n.SLAB);
    // option sc_fuse: the projection shortcut inside conv1's launch (its centre-tap im2col tiles)
    const bool scf = b.proj && option_get(OPT_SC_FUSE) != 0 && conv_fwd_sc_ok(b.c1.s, b.sc.s);
    if (b.proj && !scf)  // the shortcut conv first
      PROF(0, conv_flops(b.sc.s),
           conv_fwd(b.sc.s, in, n.wbf(b.sc.pidx), n.at<u16>(b.S), train ? n.at<int64_t>(b.bsc.stats) : nullptr, slab,
                    n.slab_bytes, st, ts, n.tick(0)));
    if (scf) {
      PROF(0, conv_flops(b.c1.s) + conv_flops(b.sc.s),
           conv_fwd_sc(b.c1.s, b.sc.s, in, n.wbf(b.c1.pidx), n.at<u16>(b.C1), train ? n.at<int64_t>(b.b1.stats) : nullptr,
                       n.wbf(b.sc.pidx), n.at<u16>(b.S), train ? n.at<int64_t>(b.bsc.stats) : nullptr, st, ts));
    } else {
      PROF(0, conv_flops(b.c1.s),
           conv_fwd(b.c1.s, in, n.wbf(b.c1.pidx), n.at<u16>(b.C1), train ? n.at<int64_t>(b.b1.stats) : nullptr, slab,
                    n.slab_bytes, st, ts, n.tick(0)));
    }
    DTC_TRY(bn_act(n, 1, b.b1, n.at<u16>(b.C1), nullptr, nullptr, n.at<u16>(b.A1), M, train, st, b.MA1));
    PROF(0, conv_flops(b.c2.s),
         conv_fwd(b.c2.s, n.at<u16>(b.A1), n.wbf(b.c2.pidx), n.at<u16>(b.C2),
                  train ? n.at<int64_t>(b.b2.stats) : nullptr, slab, n.slab_bytes, st, ts, n.tick(0)));
    if (b.proj) {
      DTC_TRY(bn_act(n, 3, b.b2, n.at<u16>(b.C2), &b.bsc, n.at<u16>(b.S), n.at<u16>(b.OUT), M, train, st, b.MOUT));
    } else {
      DTC_TRY(bn_act(n, 2, b.b2, n.at<u16>(b.C2), nullptr, in, n.at<u16>(b.OUT), M, train, st, b.MOUT));
    }
    in = n.at<u16>(b.OUT);
  }
  // graphed forward: the head is launched by forward() after the graph, into the caller's logits
  if (logits == nullptr) return 0;
  return forward_head(n, logits, st);
}

// ------------------------------------------------------------------ fp32 mode (no autocast)
// Same structure as forward_body / backward_body with fp32 activations: f32-MFMA convs
// (conv_f32.hip, BN statistics in the forward epilogue), the fused BN apply kernels on fp32
// tensors (no autocast rounding points), a separate masked BN-backward reduction after each dgrad,
// fp32 head with the fp32 master Linear weights.
static int bn_act_f32(Net& n, int mode, BNL& b, const float* x, BNL* b2, const float* x2, float* y, int64_t M,
                      bool train, hipStream_t st) {
  if (train && n.sync) {
    DTC_TRY(sync_bn_sums(n, b.stats, b.C, st));
    if (b2) DTC_TRY(sync_bn_sums(n, b2->stats, b2->C, st));
  }
  const int64_t cnt = train && n.sync ? M * n.sync_world : M;
  if (train) {
    const BnFwdArgs a1 = fwd_args(n, b, cnt);
    const BnFwdArgs a2 = b2 ? fwd_args(n, *b2, cnt) : BnFwdArgs{};
    return bn_fin_apply(mode, x, a1, x2, b2 ? &a2 : nullptr, y, M, b.C, st);
  }
  DTC_TRY(bn_finalize_fwd(n, b, cnt, false, st));
  if (b2) DTC_TRY(bn_finalize_fwd(n, *b2, cnt, false, st));
  const float* s1 = n.at<float>(b.scale);
  const float* h1 = n.at<float>(b.shift);
  if (mode == 1) return bn_apply_relu(x, s1, h1, y, M, b.C, st);
  if (mode == 2) return bn_apply_add_relu(x, s1, h1, x2, y, M, b.C, st);
  return bn_apply_dual_relu(x, s1, h1, x2, n.at<float>(b2->scale), n.at<float>(b2->shift), y, M, b.C, st);
}

static int forward_body_f32(Net& n, float* logits, bool train, hipStream_t st) {
  const int64_t M0 = (int64_t)n.B * n.H * n.W;
  float* slab = n.at<float>(n.SLAB);
  n.prof_next = train ? 0 : Net::PROF_SLOTS;
  DTC_TRY(f32_stem_pack_weight(n.pf(n.stem.pidx), n.at<float>(n.WSTEM), 64, st));
  if (train) DTC_TRY(zero_bytes(n.ws + n.stats_lo, n.stats_hi - n.stats_lo, st));  // + the backward sums
  PROF(0, 2.0 * M0 * 64 * 27,
       conv_f32(f32_stem_shape(n), CONV_FWD, n.at<float>(n.X0), n.at<float>(n.WSTEM), n.at<float>(n.C0), nullptr,
                train ? n.at<int64_t>(n.bn0.stats) : nullptr, nullptr, 0, 0, 0.f, slab, n.slab_bytes, st, ts));
  DTC_TRY(bn_act_f32(n, 1, n.bn0, n.at<float>(n.C0), nullptr, nullptr, n.at<float>(n.A0), M0, train, st));
  const float* in = n.at<float>(n.A0);
  for (auto& b : n.blocks) {
    const int64_t M = (int64_t)n.B * b.Hout * b.Wout;
    PROF(0, conv_flops(b.c1.s),
         conv_f32(b.c1.s, CONV_FWD, in, n.pf(b.c1.pidx), n.at<float>(b.C1), nullptr,
                  train ? n.at<int64_t>(b.b1.stats) : nullptr, nullptr, 0, 0, 0.f, slab, n.slab_bytes, st, ts));
    DTC_TRY(bn_act_f32(n, 1, b.b1, n.at<float>(b.C1), nullptr, nullptr, n.at<float>(b.A1), M, train, st));
    PROF(0, conv_flops(b.c2.s),
         conv_f32(b.c2.s, CONV_FWD, n.at<float>(b.A1), n.pf(b.c2.pidx), n.at<float>(b.C2), nullptr,
                  train ? n.at<int64_t>(b.b2.stats) : nullptr, nullptr, 0, 0, 0.f, slab, n.slab_bytes, st, ts));
    if (b.proj) {
      PROF(0, conv_flops(b.sc.s),
           conv_f32(b.sc.s, CONV_FWD, in, n.pf(b.sc.pidx), n.at<float>(b.S), nullptr,
                    train ? n.at<int64_t>(b.bsc.stats) : nullptr, nullptr, 0, 0, 0.f, slab, n.slab_bytes, st, ts));
      DTC_TRY(bn_act_f32(n, 3, b.b2, n.at<float>(b.C2), &b.bsc, n.at<float>(b.S), n.at<float>(b.OUT), M, train, st));
    } else {
      DTC_TRY(bn_act_f32(n, 2, b.b2, n.at<float>(b.C2), nullptr, in, n.at<float>(b.OUT), M, train, st));
    }
    in = n.at<float>(b.OUT);
  }
  const BlockL& last = n.blocks.back();
  return head_fwd(in, n.B, last.Hout * last.Wout, 512, n.pf(n.fc_w), n.pf(n.fc_b), n.ncls, n.at<float>(n.FEAT),
                  logits, st);
}

struct BwdCtx;
static int maybe_bucket(Net& n, int after_block, const BwdCtx& cx, hipStream_t st);
static int cap(Net& n, const std::string& name, const void* src, hipStream_t st);
static BnBwdArgs bwd_args(Net& n, BNL& b, int64_t count, float gs);

static int backward_body_f32(Net& n, const float* dlogits, float gs, const BwdCtx& cx, hipStream_t st) {
  n.prof_next = Net::PROF_BWD0;
  n.ev_next = 0;
  float* G[6];
  for (int i = 0; i < 6; ++i) G[i] = n.at<float>(n.G[i]);
  float* slab = n.at<float>(n.SLAB);
  const BlockL& last = n.blocks.back();
  // the BN backward sums were zeroed by the training forward (forward_body)
  DTC_TRY(head_bwd(dlogits, n.at<float>(n.FEAT), n.pf(n.fc_w), n.B, last.Hout * last.Wout, 512, n.ncls, gs,
                   n.gf(n.fc_w), n.gf(n.fc_b), G[0], n.at<float>(n.HEADWS), n.HEADWS_bytes, st, n.xent.logits ? &n.xent : nullptr));
  for (int bi = (int)n.blocks.size() - 1; bi >= 0; --bi) {
    BlockL& b = n.blocks[bi];
    const int64_t M = (int64_t)n.B * b.Hout * b.Wout;
    const float* in = bi > 0 ? n.at<float>(n.blocks[bi - 1].OUT) : n.at<float>(n.A0);
    float* dc2 = n.at<float>(b.DC2);
    float* dc1 = n.at<float>(b.DC1);
    float* dsc = b.proj ? n.at<float>(b.DSC) : nullptr;
    const std::string cp = n.capture ? "grad.layer" + std::to_string(bi / 2 + 1) + "." + std::to_string(bi % 2) : "";
    DTC_TRY(cap(n, cp + ".dy", G[0], st));
    // out = relu(bn2(c2) + shortcut): dz = dy * [out > 0] and the BN-backward sums of bn2 (+ bn_sc)
    DTC_TRY(bn_bwd_reduce(G[0], n.at<float>(b.OUT), n.at<float>(b.C2), n.at<float>(b.b2.mean),
                          n.at<float>(b.b2.invstd), n.at<int64_t>(b.b2.acc), b.proj ? n.at<float>(b.S) : nullptr,
                          b.proj ? n.at<float>(b.bsc.mean) : nullptr, b.proj ? n.at<float>(b.bsc.invstd) : nullptr,
                          b.proj ? n.at<int64_t>(b.bsc.acc) : nullptr, G[1], M, b.Cout, st));
    float* dz2 = G[1];
    {
      if (n.sync) {
        DTC_TRY(sync_bn_sums(n, b.b2.acc, b.b2.C, st));
        if (b.proj) DTC_TRY(sync_bn_sums(n, b.bsc.acc, b.bsc.C, st));
      }
      const float g2 = n.sync ? gs / (float)n.sync_world : gs;
      const int64_t cnt = n.sync ? M * n.sync_world : M;
      const BnBwdArgs a1 = bwd_args(n, b.b2, cnt, g2);
      const BnBwdArgs a2 = b.proj ? bwd_args(n, b.bsc, cnt, g2) : BnBwdArgs{};
      DTC_TRY(bn_bwd_fin_apply(dz2, n.at<float>(b.C2), a1, dc2, b.proj ? n.at<float>(b.S) : nullptr,
                               b.proj ? &a2 : nullptr, dsc, M, b.Cout, st));
    }
    DTC_TRY(cap(n, cp + ".dz", dz2, st));
    DTC_TRY(cap(n, cp + ".dc2", dc2, st));
    if (b.proj) DTC_TRY(cap(n, cp + ".ds", dsc, st));
    PROF(2, conv_flops(b.c2.s),
         conv_f32(b.c2.s, CONV_WGRAD, n.at<float>(b.A1), dc2, nullptr, nullptr, nullptr, n.gf(b.c2.pidx), 0, 0, gs,
                  slab, n.slab_bytes, st, ts));
    PROF(1, conv_flops(b.c2.s),
         conv_f32(b.c2.s, CONV_DGRAD, dc2, n.pf(b.c2.pidx), G[4], nullptr, nullptr, nullptr, 0, 0, 0.f, slab,
                  n.slab_bytes, st, ts));
    DTC_TRY(cap(n, cp + ".da1", G[4], st));
    // a1 = relu(bn1(c1)): dz1 = da1 * [a1 > 0] (in place) and bn1's sums
    DTC_TRY(bn_bwd_reduce(G[4], n.at<float>(b.A1), n.at<float>(b.C1), n.at<float>(b.b1.mean),
                          n.at<float>(b.b1.invstd), n.at<int64_t>(b.b1.acc), nullptr, nullptr, nullptr, nullptr, G[4],
                          M, b.Cout, st));
    DTC_TRY(cap(n, cp + ".dz1", G[4], st));
    {
      if (n.sync) DTC_TRY(sync_bn_sums(n, b.b1.acc, b.b1.C, st));
      const float g1 = n.sync ? gs / (float)n.sync_world : gs;
      const BnBwdArgs a1 = bwd_args(n, b.b1, n.sync ? M * n.sync_world : M, g1);
      DTC_TRY(bn_bwd_fin_apply(G[4], n.at<float>(b.C1), a1, dc1, (const float*)nullptr, nullptr, nullptr, M, b.Cout,
                               st));
    }
    DTC_TRY(cap(n, cp + ".dc1", dc1, st));
    PROF(2, conv_flops(b.c1.s),
         conv_f32(b.c1.s, CONV_WGRAD, in, dc1, nullptr, nullptr, nullptr, n.gf(b.c1.pidx), 0, 0, gs, slab,
                  n.slab_bytes, st, ts));
    if (b.proj) {
      PROF(2, conv_flops(b.sc.s),
           conv_f32(b.sc.s, CONV_WGRAD, in, dsc, nullptr, nullptr, nullptr, n.gf(b.sc.pidx), 0, 0, gs, slab,
                    n.slab_bytes, st, ts));
      PROF(1, conv_flops(b.sc.s),
           conv_f32(b.sc.s, CONV_DGRAD, dsc, n.pf(b.sc.pidx), G[5], nullptr, nullptr, nullptr, 0, 0, 0.f, slab,
                    n.slab_bytes, st, ts));
      DTC_TRY(cap(n, cp + ".dxs", G[5], st));
      PROF(1, conv_flops(b.c1.s),
           conv_f32(b.c1.s, CONV_DGRAD, dc1, n.pf(b.c1.pidx), G[0], G[5], nullptr, nullptr, 0, 0, 0.f, slab,
                    n.slab_bytes, st, ts));
    } else {  // dx = dgrad + dz2 (the identity shortcut's gradient)
      PROF(1, conv_flops(b.c1.s),
           conv_f32(b.c1.s, CONV_DGRAD, dc1, n.pf(b.c1.pidx), G[0], dz2, nullptr, nullptr, 0, 0, 0.f, slab,
                    n.slab_bytes, st, ts));
    }
    DTC_TRY(cap(n, cp + ".dx", G[0], st));
    DTC_TRY(maybe_bucket(n, bi, cx, st));
  }
  const int64_t M0 = (int64_t)n.B * n.H * n.W;
  float* dc0 = n.at<float>(n.DC0);
  DTC_TRY(bn_bwd_reduce(G[0], n.at<float>(n.A0), n.at<float>(n.C0), n.at<float>(n.bn0.mean), n.at<float>(n.bn0.invstd),
                        n.at<int64_t>(n.bn0.acc), nullptr, nullptr, nullptr, nullptr, G[1], M0, 64, st));
  {
    if (n.sync) DTC_TRY(sync_bn_sums(n, n.bn0.acc, n.bn0.C, st));
    const float g0 = n.sync ? gs / (float)n.sync_world : gs;
    const BnBwdArgs a0 = bwd_args(n, n.bn0, n.sync ? M0 * n.sync_world : M0, g0);
    DTC_TRY(bn_bwd_fin_apply(G[1], n.at<float>(n.C0), a0, dc0, (const float*)nullptr, nullptr, nullptr, M0, 64, st));
  }
  DTC_TRY(cap(n, "grad.stem.dz", G[1], st));
  DTC_TRY(cap(n, "grad.stem.dc", dc0, st));
  PROF(2, 2.0 * M0 * 64 * 27,
       conv_f32(f32_stem_shape(n), CONV_WGRAD, n.at<float>(n.X0), dc0, nullptr, nullptr, nullptr, n.gf(n.stem.pidx),
                27, 27, gs, slab, n.slab_bytes, st, ts));
  DTC_TRY(maybe_bucket(n, -1, cx, st));
  if (n.profiling) DTC_TRY(prof_accumulate(n.prof_ts, Net::PROF_SLOTS, n.prof_acc, st));
  return 0;
}

static int forward_impl(Net& n, const float* x, float* logits, bool train, hipStream_t st);
static int forward(Net& n, const float* x, float* logits, bool train, hipStream_t st) {
  DTC_TRY(forward_impl(n, x, logits, train, st));
  if (train) n.sums_fresh = true;
  return 0;
}
static int forward_impl(Net& n, const float* x, float* logits, bool train, hipStream_t st) {
  n.prof_st = st;
  // graphed bf16 forward: the pool + FC head is launched after the graph straight into the caller's logits
  // (the graph cannot bake in a per-call pointer); the fp32 executor's graph writes a graph-owned buffer
  // that is copied out after the replay
  if (n.f32) DTC_TRY(f32_stem_im2col(x, n.at<float>(n.X0), n.B, n.H, n.W, st));
  else if (n.stem_direct) {  // the graph reads only executor memory: a copy of the 12 B/pixel input (+ the
    // training step's BN slots zeroed in the same launch)
    const size_t xb = (size_t)n.B * 3 * n.H * n.W * 4;
    if (xb % 16 == 0 && ((uintptr_t)x & 15) == 0 && option_get(OPT_STEM_PROLOGUE) != 0) {
      DTC_TRY(copy_and_zero(x, n.at<float>(n.XIN), xb, n.ws + n.stats_lo, train ? n.stats_hi - n.stats_lo : 0, st));
    } else {
      DTC_HIP(hipMemcpyAsync(n.at<float>(n.XIN), x, xb, hipMemcpyDeviceToDevice, st));
      if (train) DTC_TRY(zero_bytes(n.ws + n.stats_lo, n.stats_hi - n.stats_lo, st));
    }
  } else {
    DTC_TRY(stem_im2col(x, n.at<u16>(n.X0), n.B, n.H, n.W, st));
  }
  if (!graphs_on(n, false)) return forward_body(n, logits, train, st);
  hipGraphExec_t& ex = n.fwd_exec[n.profiling ? 1 : 0][train ? 1 : 0];
  if (!ex) {
    DTC_TRY(begin_capture(n));
    const int rc = forward_body(n, n.f32 ? n.at<float>(n.LOGITS) : nullptr, train, n.cap_st);
    DTC_TRY(end_capture(n, rc, &ex));
  }
  DTC_TRY(graph_launch(n, ex, st));
  if (!n.f32) return forward_head(n, logits, st);
  DTC_HIP(hipMemcpyAsync(logits, n.at<float>(n.LOGITS), (size_t)n.B * n.ncls * 4, hipMemcpyDeviceToDevice, st));
  return 0;
}

// Bucket point after block `after_block` (-1: after the stem). Eager: all-reduce the buckets that
// are complete now. Capturing: close the current graph segment there and open the next one; the
// replay issues the all-reduces between segments.
struct BwdCtx {
  Comm* comm = nullptr;
  bool capturing = false;
  std::vector<Net::Seg>* segs = nullptr;
};
static int join_side(Net& n, hipStream_t st);
static int next_event(Net& n, hipEvent_t* ev);
static bool side_covers(hipStream_t st);
static int stop_or_record(Net& n, hipStream_t st, hipEvent_t* ev);
static int maybe_bucket(Net& n, int after_block, const BwdCtx& cx, hipStream_t st) {
  if (!cx.comm) return 0;
  std::vector<int> ids;
  for (size_t i = 0; i < n.bucket_off.size(); ++i)
    if (n.bucket_after_block[i] == after_block) ids.push_back((int)i);
  if (ids.empty()) return 0;
  if (!cx.capturing) {
    // The bucket's producers are the compute stream (BN dgamma / dbeta, the head) and the weight-gradient
    // side stream. The compute stream does NOT wait for the side stream here (that join would stall the
    // dgrad / BN chain behind the queued weight gradients at every bucket point): the side stream is
    // forked from the compute stream instead, so it holds both producers, and the collective is ordered
    // after it. The side stream is joined into the compute stream once, at the end of the backward.
    hipStream_t prod = st;
    if (n.side_pending) {
      if (!side_covers(st)) {  // (a flush's fork right before this point already ordered it: no second marker)
        hipEvent_t ev;
        DTC_TRY(stop_or_record(n, st, &ev));
        DTC_HIP(hipStreamWaitEvent(n.side_st, ev, 0));
        g_fork_watch = ForkWatch{st, false};
      }
      prod = n.side_st;
    }
    // option comm_on_side: the collective on the weight-gradient stream itself (it holds both producers
    // now; the stream is joined into the compute stream at the end of the backward) -- one HIP stream
    // fewer competing for the process's hardware queues (GPU_MAX_HW_QUEUES); the weight gradients of
    // later buckets then queue behind it on that stream
    const bool on_side = option_get(OPT_COMM_ON_SIDE) != 0 && prod == n.side_st;
    // option comm_tail_inline: the last bucket (after the stem, nothing left to overlap) is all-reduced on the
    // compute stream itself when every earlier collective is already ordered before that stream (none
    // pending on the communicator's stream): the fork to the communicator's stream and the join back cost
    // two cross-stream hand-offs, ~15 us each (bench --sim-world 2 buckets_us / comm_exposed_us, round 5)
    const bool inline_tail = after_block == -1 && prod == st && option_get(OPT_COMM_TAIL_INLINE) != 0 &&
                             !comm_pending(cx.comm);
    for (int i : ids) {
      hipEvent_t t0 = nullptr, t1 = nullptr;
      if (n.ct_cur && i < (int)n.ct_cur->b0.size()) {
        t0 = n.ct_cur->b0[i];
        t1 = n.ct_cur->b1[i];
        n.ct_cur->bucket[i] = true;
      }
      if (on_side || inline_tail)
        DTC_TRY(comm_allreduce_on(cx.comm, n.g + n.bucket_off[i], (size_t)n.bucket_len[i], prod, t0, t1));
      else DTC_TRY(comm_allreduce_async(cx.comm, n.g + n.bucket_off[i], (size_t)n.bucket_len[i], prod, t0, t1));
    }
    return 0;
  }
  DTC_TRY(join_side(n, st));  // a graph segment ends here: every stream forked in it joins back
  Net::Seg sg;
  sg.buckets = ids;
  DTC_TRY(end_capture(n, 0, &sg.exec));
  cx.segs->push_back(sg);
  return begin_capture(n);
}

static int cap(Net& n, const std::string& name, const void* src, hipStream_t st) {
  if (!n.capture) return 0;
  for (const auto& a : n.caps)
    if (a.name == name) {
      DTC_HIP(hipMemcpyAsync(n.ws + a.off, src, (size_t)a.n * a.h * a.w * a.c * n.esz(), hipMemcpyDeviceToDevice, st));
      return 0;
    }
  return set_error(DTC_EINVAL, "capture slot %s missing", name.c_str());
}

static BnBwdArgs bwd_args(Net& n, BNL& b, int64_t count, float gs) {
  BnBwdArgs a;
  a.acc = n.at<int64_t>(b.acc);
  a.count = count;
  a.gamma = n.pf(b.gidx);
  a.mean = n.at<float>(b.mean);
  a.invstd = n.at<float>(b.invstd);
  a.gscale = gs;
  a.dgamma = n.gf(b.gidx);
  a.dbeta = n.gf(b.bidx);
  return a;
}

// dx1 = BN-backward apply of b1 on (dz, x1) [; dx2 of b2 on (dz, x2)], coefficients from the sums
// bn_bwd_reduce accumulated; dgamma / dbeta into the flat gradient buffer.
// Small tensors (option bn_cg, bn_bwd_cg_ok): the mask-bit BN backward -- reduction, coefficients, apply --
// as ONE launch (bn.hip bn_bwd_cg: one workgroup per 8 channels over the whole batch, no fp64 slots); not
// with SyncBN (its sums are all-reduced between the two passes)
// Measured (kernel trace r04e, batch 256): at layer4's 4096 x 512 the one launch took 26-30 us against
// 11 us for the pair -- 64 workgroups of 16-B pieces strided by the channel count -- so it is used only
// for tensors of at most 256K elements (layer4 at the per-rank batch 32 of config 3)
static bool bn_cg_on(const Net& n, int64_t M, int C, bool dual) {
  return option_get(OPT_BN_CG) != 0 && !n.sync && !n.f32 && bn_fused() && M * C <= (int64_t)option_get(OPT_BN_CG_ELEMS) &&
         bn_bwd_cg_ok(M, C, dual);
}
static int bn_bwd_one_launch(Net& n, BNL& b1, const u16* dy, const uint8_t* mbits, u16* dzo, const u16* x1, u16* dx1,
                             BNL* b2, const u16* x2, u16* dx2, int64_t M, float gs, hipStream_t st) {
  const BnBwdArgs a1 = bwd_args(n, b1, M, gs);
  const BnBwdArgs a2 = b2 ? bwd_args(n, *b2, M, gs) : BnBwdArgs{};
  const double work = (double)M * b1.C * (6.125 + (x2 ? 4.0 : 0.0) + (dzo ? 2.0 : 0.0));
  u64* ts = prof_slot(n, 3, work);
  const int ev = prof_ev_open(n, 3, work);
  const int rc = bn_bwd_cg(dy, mbits, dzo, x1, a1, dx1, x2, b2 ? &a2 : nullptr, dx2, M, b1.C, st, ts);
  prof_ev_close(n, ev);
  return rc;
}

static int bn_bwd_coef_apply(Net& n, BNL& b1, const u16* dz, const u16* x1, u16* dx1, BNL* b2, const u16* x2, u16* dx2,
                             int64_t M, float gs, hipStream_t st, const uint8_t* mbits = nullptr,
                             u16* dzo = nullptr) {
  if (n.sync) {  // SyncBN backward: global sum(dz), sum(dz*xhat); dgamma/dbeta stay this rank's share
    DTC_TRY(sync_bn_sums(n, b1.acc, b1.C, st));
    if (b2) DTC_TRY(sync_bn_sums(n, b2->acc, b2->C, st));
    gs /= (float)n.sync_world;
  }
  const int64_t cnt = n.sync ? M * n.sync_world : M;
  if (bn_fused()) {
    const BnBwdArgs a1 = bwd_args(n, b1, cnt, gs);
    const BnBwdArgs a2 = b2 ? bwd_args(n, *b2, cnt, gs) : BnBwdArgs{};
    if (mbits) {
      const double work = (double)M * b1.C * (6.125 + (x2 ? 4.0 : 0.0) + (dzo ? 2.0 : 0.0));
      u64* ts = prof_slot(n, 3, work);
      const int ev = prof_ev_open(n, 3, work);
      const int rc = bn_bwd_fin_apply_mask(dz, mbits, dzo, x1, a1, dx1, x2, b2 ? &a2 : nullptr, dx2, M, b1.C, st, ts);
      prof_ev_close(n, ev);
      return rc;
    }
    return bn_bwd_fin_apply(dz, x1, a1, dx1, x2, b2 ? &a2 : nullptr, dx2, M, b1.C, st);
  }
  DTC_CHECK_ARG(mbits == nullptr, "mask-bit BN backward needs the fused finalize");
  DTC_TRY(bn_bwd_finalize(n.at<int64_t>(b1.acc), b1.C, cnt, n.pf(b1.gidx), n.at<float>(b1.mean), n.at<float>(b1.invstd),
                          gs, n.gf(b1.gidx), n.gf(b1.bidx), n.at<float>(b1.coef), st));
  if (b2)
    DTC_TRY(bn_bwd_finalize(n.at<int64_t>(b2->acc), b2->C, cnt, n.pf(b2->gidx), n.at<float>(b2->mean),
                            n.at<float>(b2->invstd), gs, n.gf(b2->gidx), n.gf(b2->bidx), n.at<float>(b2->coef), st));
  return bn_bwd_apply(dz, x1, n.at<float>(b1.coef), dx1, x2, b2 ? n.at<float>(b2->coef) : nullptr, dx2, M, b1.C, st);
}

// Side stream for the weight gradients (fork after their input gradient exists, join before
// anything reads the weight gradients: bucket all-reduces and the end of backward).
static bool side_on(const Net& n) { return option_get(OPT_BWD_STREAMS) != 0; }
static int next_event(Net& n, hipEvent_t* ev) {
  if (n.evs.empty()) {
    n.evs.resize(64);
    for (auto& e : n.evs) DTC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  *ev = n.evs[n.ev_next];
  n.ev_next = (n.ev_next + 1) % (int)n.evs.size();
  return 0;
}
// A marker recorded on `st` (the fork / join points of the weight-gradient stream). Round 6 measured the
// alternative -- waiting on the producing kernel's own stop event (hipExtLaunchKernelGGL) instead of a recorded
// marker, which removes the marker's ~2.7 us bubble in isolation (tools/probes/fork_gap.hip) -- and removed it:
// on a busy stream each such launch cost the host ~4 us and left a ~4.7 us gap after the kernel (B=256 -2.7%,
// 24 of 24 in-process A/B rounds; backward host issue 189 -> 321 us; profiles/r06w_fork_ev.txt)
static int stop_or_record(Net& n, hipStream_t st, hipEvent_t* ev) {
  DTC_TRY(next_event(n, ev));
  DTC_HIP(hipEventRecord(*ev, st));
  return 0;
}
static int fork_side(Net& n, hipStream_t st, hipStream_t* out) {
  if (!side_on(n)) {
    *out = st;
    return 0;
  }
  if (!n.side_st) {
    // option side_prio: the weight-gradient stream at the lowest priority, so the dispatcher prefers the
    // dgrad / BN chain (the critical path) when both have workgroups ready
    if (option_get(OPT_SIDE_PRIO) != 0) {
      int lo = 0, hi = 0;
      DTC_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));  // lo = least urgent
      DTC_HIP(hipStreamCreateWithPriority(&n.side_st, hipStreamNonBlocking, lo));
    } else {
      DTC_HIP(hipStreamCreateWithFlags(&n.side_st, hipStreamNonBlocking));
    }
  }
  hipEvent_t ev;
  DTC_TRY(stop_or_record(n, st, &ev));
  DTC_HIP(hipStreamWaitEvent(n.side_st, ev, 0));
  g_fork_watch = ForkWatch{st, false};
  n.side_pending = true;
  *out = n.side_st;
  return 0;
}
// the side stream already waits for everything issued on st (forked from it, nothing launched on st since)
static bool side_covers(hipStream_t st) { return g_fork_watch.st == st && !g_fork_watch.dirty; }
static int join_side(Net& n, hipStream_t st) {
  if (!n.side_pending) return 0;
  hipEvent_t ev;
  DTC_TRY(stop_or_record(n, n.side_st, &ev));
  DTC_HIP(hipStreamWaitEvent(st, ev, 0));
  n.side_pending = false;
  return 0;
}

// BN-backward reduction of the BN(s) whose post-ReLU output is `y`, for a dgrad epilogue (bnb_epi.h):
// the conv producing dy stores dz = dy * [y > 0] and accumulates the sums bn_bwd_reduce would.
static BnbArgs bnb_of(Net& n, size_t y, size_t x1, BNL& b1, size_t x2 = 0, BNL* b2 = nullptr) {
  BnbArgs a;
  a.ym = n.at<u16>(y);
  a.x1 = n.at<u16>(x1);
  a.mean1 = n.at<float>(b1.mean);
  a.invstd1 = n.at<float>(b1.invstd);
  a.acc1 = n.at<int64_t>(b1.acc);
  if (b2 != nullptr) {
    a.x2 = n.at<u16>(x2);
    a.mean2 = n.at<float>(b2->mean);
    a.invstd2 = n.at<float>(b2->invstd);
    a.acc2 = n.at<int64_t>(b2->acc);
  }
  return a;
}

// Deferred 3x3 stride-1 weight gradients (option wgrad_batch): every wgrad of the halo geometry is
// queued and issued together with the others of its geometry -- at most wgrad_batch per launch --
// when the geometry changes, before a DDP bucket that needs them is all-reduced, and at the end of
// backward. The inputs stay valid while queued (per-block conv-output gradient buffers, forward
// activations). One batched launch of P problems writes the split-K slab of ONE (conv_wgrad_batch).
struct WgQueue {
  ConvShape s{};
  int count = 0;
  const u16* x[DTC_WG_BATCH] = {};
  const u16* dy[DTC_WG_BATCH] = {};
  float* dw[DTC_WG_BATCH] = {};
};
static int wgrad_batch_max() { return std::min(std::max(option_get(OPT_WGRAD_BATCH), 1), DTC_WG_BATCH); }
static bool same_shape(const ConvShape& a, const ConvShape& b) {
  return a.N == b.N && a.H == b.H && a.W == b.W && a.C == b.C && a.K == b.K && a.R == b.R && a.S == b.S &&
         a.stride == b.stride && a.pad == b.pad;
}
static int wg_flush(Net& n, WgQueue& q, float gs, float* slabw, hipStream_t sd) {
  if (q.count == 0) return 0;
  const int np = q.count;
  q.count = 0;
  if (np == 1) {
    PROF(2, conv_flops(q.s),
         conv_wgrad(q.s, q.x[0], q.dy[0], q.dw[0], 0, 0, gs, slabw, n.slab_bytes, sd, ts));
    return 0;
  }
  PROF(2, conv_flops(q.s) * np,
       conv_wgrad_batch(q.s, np, q.x, q.dy, q.dw, gs, slabw, n.slab_bytes, sd, ts));
  return 0;
}
static int fork_side(Net& n, hipStream_t st, hipStream_t* out);
// lazy (option fork_lazy): the side stream is forked from `st` here, only when something is launched,
// instead of by the caller before every wgrad (a queued-only wgrad needs no fork: the launch's fork
// is later on the main stream, so it covers the queued inputs too)
static int wg_issue(Net& n, WgQueue& q, const ConvShape& s, const u16* x, const u16* dy, float* dw, float gs,
                    float* slabw, hipStream_t& sd, hipStream_t st = nullptr, bool lazy = false) {
  const int bmax = wgrad_batch_max();
  if (bmax <= 1 || wgrad_halo_splits(s, 2) <= 0) {
    if (lazy) DTC_TRY(fork_side(n, st, &sd));
    PROF(2, conv_flops(s), conv_wgrad(s, x, dy, dw, 0, 0, gs, slabw, n.slab_bytes, sd, ts));
    return 0;
  }
  if (q.count > 0 && !same_shape(q.s, s)) {
    if (lazy) DTC_TRY(fork_side(n, st, &sd));
    DTC_TRY(wg_flush(n, q, gs, slabw, sd));
  }
  q.s = s;
  q.x[q.count] = x;
  q.dy[q.count] = dy;
  q.dw[q.count] = dw;
  if (++q.count >= bmax) {
    if (lazy) DTC_TRY(fork_side(n, st, &sd));
    DTC_TRY(wg_flush(n, q, gs, slabw, sd));
  }
  return 0;
}
// (the plan's bucket points, with or without a communicator: the batches -- and so the split-K
// summation order -- are the same whether or not the gradients are all-reduced)
static bool bucket_fires(const Net& n, int after_block) {
  for (int a : n.bucket_after_block)
    if (a == after_block) return true;
  return false;
}

// Backward with the mask-bit BN path (bn_mask_on): G[0] carries the RAW gradient of a block output
// (never masked in place by a reduction), each BN reduction reads (dy, mask bits, x) and stores
// nothing, and each BN apply forms dz = dy * bit again. The identity shortcut needs dz itself (the
// residual of conv1's dgrad): bn2's apply writes it over dy in place (same lane reads then writes).
// Parity captures (n.capture) materialise dz with bn_mask_apply into their slots.
static int cap_masked(Net& n, const std::string& name, const u16* dy, size_t mask_off, int64_t M, int C, hipStream_t st) {
  if (!n.capture) return 0;
  for (const auto& a : n.caps)
    if (a.name == name) return bn_mask_apply(dy, n.at<uint8_t>(mask_off), (u16*)(n.ws + a.off), M, C, st);
  return set_error(DTC_EINVAL, "capture slot %s missing", name.c_str());
}

// BN-backward sums of the BN(s) whose post-ReLU output gradient a dgrad writes, from the mask bits

static int backward_body_mask(Net& n, const float* dlogits, float gs, const BwdCtx& cx, hipStream_t st) {
  n.prof_next = Net::PROF_BWD0;
  n.ev_next = 0;
  // (Every BN's backward sums come from a reduction pass of its own -- or the one-launch small-tensor kernel;
  // the round-3/4 option that accumulated them in the producing dgrad's epilogue measured slower and was
  // removed in round 5: DESIGN.md.)
  u16* G[6];
  for (int i = 0; i < 6; ++i) G[i] = n.at<u16>(n.G[i]);
  float* slab = n.at<float>(n.SLAB);
  float* slabw = n.at<float>(n.SLABW);
  hipStream_t sd = st;  // weight-gradient stream
  const BlockL& last = n.blocks.back();
  // the BN backward sums were zeroed by the training forward (forward_body)
  DTC_TRY(head_bwd(dlogits, n.at<float>(n.FEAT), n.wbf(n.fc_w), n.B, last.Hout * last.Wout, 512, n.ncls, gs,
                   n.gf(n.fc_w), n.gf(n.fc_b), G[0], n.at<float>(n.HEADWS), n.HEADWS_bytes, st, n.xent.logits ? &n.xent : nullptr));
  WgQueue wq;
  for (int bi = (int)n.blocks.size() - 1; bi >= 0; --bi) {
    BlockL& b = n.blocks[bi];
    const int64_t M = (int64_t)n.B * b.Hout * b.Wout;
    const u16* in = bi > 0 ? n.at<u16>(n.blocks[bi - 1].OUT) : n.at<u16>(n.A0);
    u16* dc2 = n.at<u16>(b.DC2);
    u16* dc1 = n.at<u16>(b.DC1);
    u16* dsc = b.proj ? n.at<u16>(b.DSC) : nullptr;
    const uint8_t* mout = n.at<uint8_t>(b.MOUT);
    const uint8_t* ma1 = n.at<uint8_t>(b.MA1);
    const std::string cp = n.capture ? "grad.layer" + std::to_string(bi / 2 + 1) + "." + std::to_string(bi % 2) : "";
    DTC_TRY(cap(n, cp + ".dy", G[0], st));
    DTC_TRY(cap_masked(n, cp + ".dz", G[0], b.MOUT, M, b.Cout, st));
    // out = relu(bn2(c2) + shortcut): sums of dz = dy * [out > 0] (and of the projection BN), then
    // dc2 (and dsc); an identity block also needs dz itself as conv1's dgrad residual: in place in G[0]
    if (bn_cg_on(n, M, b.Cout, b.proj)) {
      DTC_TRY(bn_bwd_one_launch(n, b.b2, G[0], mout, b.proj ? nullptr : G[0], n.at<u16>(b.C2), dc2,
                                b.proj ? &b.bsc : nullptr, b.proj ? n.at<u16>(b.S) : nullptr, dsc, M, gs, st));
    } else {
      PROF(3, (double)M * b.Cout * (b.proj ? 6.125 : 4.125),
           bn_bwd_reduce_mask(G[0], mout, n.at<u16>(b.C2), n.at<float>(b.b2.mean), n.at<float>(b.b2.invstd),
                              n.at<int64_t>(b.b2.acc), b.proj ? n.at<u16>(b.S) : nullptr,
                              b.proj ? n.at<float>(b.bsc.mean) : nullptr, b.proj ? n.at<float>(b.bsc.invstd) : nullptr,
                              b.proj ? n.at<int64_t>(b.bsc.acc) : nullptr, M, b.Cout, st, ts));
      DTC_TRY(bn_bwd_coef_apply(n, b.b2, G[0], n.at<u16>(b.C2), dc2, b.proj ? &b.bsc : nullptr,
                                b.proj ? n.at<u16>(b.S) : nullptr, dsc, M, gs, st, mout, b.proj ? nullptr : G[0]));
    }
    DTC_TRY(cap(n, cp + ".dc2", dc2, st));
    if (b.proj) DTC_TRY(cap(n, cp + ".ds", dsc, st));
    // the shortcut's dx at its stride-2 grid only (option sc_compact): the 1x1 stride-2 conv's dgrad
    // is zero at three of four parities; conv1's parity-class dgrad adds it at the fourth
    const bool sc_cmp = b.proj && !n.capture && option_get(OPT_SC_COMPACT) != 0 && dgrad_class_ok(b.c1.s);
    const ConvShape sc_dg = sc_cmp ? ConvShape{b.sc.s.N, b.Hout, b.Wout, b.sc.s.C, b.sc.s.K, 1, 1, 1, 0} : b.sc.s;
    // option dgrad_scf: the shortcut's dgrad as extra reduction steps of conv1's class-(0, 0) dgrad (one launch)
    const bool dscf = b.proj && !n.capture && conv_dgrad_sc_ok(b.c1.s);
    const bool lazy = option_get(OPT_FORK_LAZY) != 0;
    if (!lazy) DTC_TRY(fork_side(n, st, &sd));
    DTC_TRY(wg_issue(n, wq, b.c2.s, n.at<u16>(b.A1), dc2, n.gf(b.c2.pidx), gs, slabw, sd, st, lazy));
    PROF(1, conv_flops(b.c2.s),
         conv_dgrad(b.c2.s, dc2, n.wbf(b.c2.pidx), G[4], nullptr, slab, n.slab_bytes, st, ts, nullptr, 0, n.tick(0)));
    DTC_TRY(cap(n, cp + ".da1", G[4], st));
    DTC_TRY(cap_masked(n, cp + ".dz1", G[4], b.MA1, M, b.Cout, st));
    if (bn_cg_on(n, M, b.Cout, false)) {
      DTC_TRY(bn_bwd_one_launch(n, b.b1, G[4], ma1, nullptr, n.at<u16>(b.C1), dc1, nullptr, nullptr, nullptr, M, gs, st));
    } else {
      PROF(3, (double)M * b.Cout * 4.125,
           bn_bwd_reduce_mask(G[4], ma1, n.at<u16>(b.C1), n.at<float>(b.b1.mean), n.at<float>(b.b1.invstd),
                              n.at<int64_t>(b.b1.acc), nullptr, nullptr, nullptr, nullptr, M, b.Cout, st, ts));
      DTC_TRY(bn_bwd_coef_apply(n, b.b1, G[4], n.at<u16>(b.C1), dc1, nullptr, nullptr, nullptr, M, gs, st, ma1));
    }
    DTC_TRY(cap(n, cp + ".dc1", dc1, st));
    if (!lazy || b.proj) DTC_TRY(fork_side(n, st, &sd));  // (the shortcut's wgrad below launches)
    // option wgrad_s2: conv1 (3x3 stride 2) and the shortcut (1x1 stride 2) weight gradients in one
    // column-split halo launch (x read once; the shortcut is conv1's centre tap against dsc)
    const bool wsc = b.proj && wgrad_s2_splits(b.c1.s) > 0 && n.slab_bytes >= conv_wgrad_s2_slab_bytes(b.c1.s) &&
                     b.sc.s.R == 1 && b.sc.s.stride == 2 && b.sc.s.C == b.c1.s.C && b.sc.s.K == b.c1.s.K;
    if (wsc) {
      PROF(2, conv_flops(b.c1.s) + conv_flops(b.sc.s),
           conv_wgrad_s2(b.c1.s, in, dc1, dsc, n.gf(b.c1.pidx), n.gf(b.sc.pidx), gs, slabw, n.slab_bytes, sd, ts));
    } else {
      DTC_TRY(wg_issue(n, wq, b.c1.s, in, dc1, n.gf(b.c1.pidx), gs, slabw, sd, st, lazy && !b.proj));
    }
    if (b.proj) {
      if (!wsc)
        PROF(2, conv_flops(b.sc.s),
             conv_wgrad(b.sc.s, in, dsc, n.gf(b.sc.pidx), 0, 0, gs, slabw, n.slab_bytes, sd, ts));
      if (dscf) {
        PROF(1, conv_flops(b.c1.s) + conv_flops(b.sc.s),
             conv_dgrad_sc(b.c1.s, dc1, n.wbf(b.c1.pidx), G[0], dsc, n.wbf(b.sc.pidx), st, ts));
      } else {
        PROF(1, conv_flops(b.sc.s),
             conv_dgrad(sc_dg, dsc, n.wbf(b.sc.pidx), G[5], nullptr, slab, n.slab_bytes, st, ts, nullptr, 0, n.tick(0)));
        PROF(1, conv_flops(b.c1.s),
             conv_dgrad(b.c1.s, dc1, n.wbf(b.c1.pidx), G[0], G[5], slab, n.slab_bytes, st, ts, nullptr, sc_cmp ? 1 : 0,
                        n.tick(0)));
      }
      DTC_TRY(cap(n, cp + ".dxs", G[5], st));
    } else {  // residual = dz of this block's output (G[0], written by bn2's apply); dx over it in place
      PROF(1, conv_flops(b.c1.s),
           conv_dgrad(b.c1.s, dc1, n.wbf(b.c1.pidx), G[0], G[0], slab, n.slab_bytes, st, ts, nullptr, 0, n.tick(0)));
    }
    DTC_TRY(cap(n, cp + ".dx", G[0], st));
    if (bucket_fires(n, bi)) {
      if (lazy && wq.count > 0) DTC_TRY(fork_side(n, st, &sd));
      DTC_TRY(wg_flush(n, wq, gs, slabw, sd));
    }
    DTC_TRY(maybe_bucket(n, bi, cx, st));
  }
  // stem: a0 = relu(bn1(conv1(x)))
  const int64_t M0 = (int64_t)n.B * n.H * n.W;
  u16* dc0 = n.at<u16>(n.DC0);
  const uint8_t* m0 = n.at<uint8_t>(n.MA0);
  // option stem_bn_fuse: the stem BN's apply runs inside the stem weight gradient (dc0 never stored;
  // not with parity captures, which want dc0, or SyncBN, whose sums are all-reduced first)
  if (n.stem_direct && !n.capture && !n.sync && bn_fused() && option_get(OPT_STEM_BN_FUSE) != 0) {
    PROF(3, (double)M0 * 64 * 4.125,
           bn_bwd_reduce_mask(G[0], m0, n.at<u16>(n.C0), n.at<float>(n.bn0.mean), n.at<float>(n.bn0.invstd),
                              n.at<int64_t>(n.bn0.acc), nullptr, nullptr, nullptr, nullptr, M0, 64, st, ts));
    if (option_get(OPT_FORK_LAZY) && wq.count > 0) DTC_TRY(fork_side(n, st, &sd));
    DTC_TRY(wg_flush(n, wq, gs, slabw, sd));
    const BnBwdArgs a0 = bwd_args(n, n.bn0, M0, gs);
    PROF(2, 2.0 * M0 * 64 * 27,
         stem_wgrad_bn(n.at<float>(n.XIN), G[0], m0, n.at<u16>(n.C0), a0, n.gf(n.stem.pidx), gs, n.B, n.H, n.W, slab,
                       n.slab_bytes, st, ts));
    const bool ctj = n.ct_cur && !cx.capturing;
    if (ctj) DTC_HIP(hipEventRecord(n.ct_cur->join_c, st));
    DTC_TRY(join_side(n, st));  // after the stem kernel: it depends on nothing the side stream computes
    if (ctj) {  // every backward kernel of either stream is behind join_d: the tail starts there
      DTC_HIP(hipEventRecord(n.ct_cur->join_d, st));
      DTC_HIP(hipEventRecord(n.ct_cur->tail_a, st));
      n.ct_cur->join = n.ct_cur->tail = true;
    }
    DTC_TRY(maybe_bucket(n, -1, cx, st));
    if (n.profiling) DTC_TRY(prof_accumulate(n.prof_ts, Net::PROF_SLOTS, n.prof_acc, st));
    return 0;
  }
  PROF(3, (double)M0 * 64 * 4.125,
       bn_bwd_reduce_mask(G[0], m0, n.at<u16>(n.C0), n.at<float>(n.bn0.mean), n.at<float>(n.bn0.invstd),
                          n.at<int64_t>(n.bn0.acc), nullptr, nullptr, nullptr, nullptr, M0, 64, st, ts));
  DTC_TRY(bn_bwd_coef_apply(n, n.bn0, G[0], n.at<u16>(n.C0), dc0, nullptr, nullptr, nullptr, M0, gs, st, m0));
  DTC_TRY(cap_masked(n, "grad.stem.dz", G[0], n.MA0, M0, 64, st));
  DTC_TRY(cap(n, "grad.stem.dc", dc0, st));
  if (option_get(OPT_FORK_LAZY) && wq.count > 0) DTC_TRY(fork_side(n, st, &sd));
  DTC_TRY(wg_flush(n, wq, gs, slabw, sd));
  const bool ctj = n.ct_cur && !cx.capturing;
  if (ctj) DTC_HIP(hipEventRecord(n.ct_cur->join_c, st));
  DTC_TRY(join_side(n, st));  // the stem wgrad is the last kernel: run it on the main stream
  if (ctj) {
    DTC_HIP(hipEventRecord(n.ct_cur->join_d, st));
    n.ct_cur->join = true;
  }
  PROF(2, 2.0 * M0 * 64 * 27,
       n.stem_direct ? stem_wgrad(n.at<float>(n.XIN), dc0, n.gf(n.stem.pidx), gs, n.B, n.H, n.W, slab, n.slab_bytes, st, ts)
                     : conv_wgrad(n.stem.s, n.at<u16>(n.X0), dc0, n.gf(n.stem.pidx), 27, 27, gs, slab, n.slab_bytes, st, ts));
  if (ctj) {  // the last backward kernel has been issued
    DTC_HIP(hipEventRecord(n.ct_cur->tail_a, st));
    n.ct_cur->tail = true;
  }
  DTC_TRY(maybe_bucket(n, -1, cx, st));
  if (n.profiling) DTC_TRY(prof_accumulate(n.prof_ts, Net::PROF_SLOTS, n.prof_acc, st));
  return 0;
}

static int backward_body(Net& n, const float* dlogits, float gs, const BwdCtx& cx, hipStream_t st) {
  if (n.f32) return backward_body_f32(n, dlogits, gs, cx, st);
  if (bn_mask_on(n)) return backward_body_mask(n, dlogits, gs, cx, st);
  n.prof_next = Net::PROF_BWD0;
  n.ev_next = 0;
  u16* G[6];
  for (int i = 0; i < 6; ++i) G[i] = n.at<u16>(n.G[i]);
  float* slab = n.at<float>(n.SLAB);
  float* slabw = n.at<float>(n.SLABW);
  hipStream_t sd = st;  // weight-gradient stream
  const BlockL& last = n.blocks.back();
  // the BN backward sums were zeroed by the training forward (forward_body)
  DTC_TRY(head_bwd(dlogits, n.at<float>(n.FEAT), n.wbf(n.fc_w), n.B, last.Hout * last.Wout, 512, n.ncls, gs,
                   n.gf(n.fc_w), n.gf(n.fc_b), G[0], n.at<float>(n.HEADWS), n.HEADWS_bytes, st, n.xent.logits ? &n.xent : nullptr));
  // fuse: the dgrad producing a BN output's gradient also does that BN's backward reduction
  // (captures keep the unfused order: they record dy and dz separately)
  const bool fuse = !n.capture;
  bool dz_ready = false;  // G[0] already holds the next BN's dz (the previous dgrad's fused epilogue)
  WgQueue wq;
  for (int bi = (int)n.blocks.size() - 1; bi >= 0; --bi) {
    BlockL& b = n.blocks[bi];
    const int64_t M = (int64_t)n.B * b.Hout * b.Wout;
    const u16* in = bi > 0 ? n.at<u16>(n.blocks[bi - 1].OUT) : n.at<u16>(n.A0);
    u16* dc2 = n.at<u16>(b.DC2);
    u16* dc1 = n.at<u16>(b.DC1);
    u16* dsc = b.proj ? n.at<u16>(b.DSC) : nullptr;
    const std::string cp = n.capture ? "grad.layer" + std::to_string(bi / 2 + 1) + "." + std::to_string(bi % 2) : "";
    DTC_TRY(cap(n, cp + ".dy", G[0], st));
    // out = relu(bn2(c2) + shortcut): dz = dy * [out > 0]
    u16* dz2 = G[0];
    if (!dz_ready) {
      dz2 = G[1];
      DTC_TRY(bn_bwd_reduce(G[0], n.at<u16>(b.OUT), n.at<u16>(b.C2), n.at<float>(b.b2.mean),
                            n.at<float>(b.b2.invstd), n.at<int64_t>(b.b2.acc), b.proj ? n.at<u16>(b.S) : nullptr,
                            b.proj ? n.at<float>(b.bsc.mean) : nullptr, b.proj ? n.at<float>(b.bsc.invstd) : nullptr,
                            b.proj ? n.at<int64_t>(b.bsc.acc) : nullptr, G[1], M, b.Cout, st));
    }
    DTC_TRY(bn_bwd_coef_apply(n, b.b2, dz2, n.at<u16>(b.C2), dc2, b.proj ? &b.bsc : nullptr,
                              b.proj ? n.at<u16>(b.S) : nullptr, dsc, M, gs, st));
    DTC_TRY(cap(n, cp + ".dz", dz2, st));
    DTC_TRY(cap(n, cp + ".dc2", dc2, st));
    if (b.proj) DTC_TRY(cap(n, cp + ".ds", dsc, st));
    // conv2: dW2 (side stream) and da1
    DTC_TRY(fork_side(n, st, &sd));
    DTC_TRY(wg_issue(n, wq, b.c2.s, n.at<u16>(b.A1), dc2, n.gf(b.c2.pidx), gs, slabw, sd));
    // a1 = relu(bn1(c1)): da1 -> dz1 (fused into the dgrad, or a separate reduction)
    {
      const BnbArgs bz = bnb_of(n, b.A1, b.C1, b.b1);
      PROF(1, conv_flops(b.c2.s),
           conv_dgrad(b.c2.s, dc2, n.wbf(b.c2.pidx), G[4], nullptr, slab, n.slab_bytes, st, ts, fuse ? &bz : nullptr));
    }
    if (!fuse) {
      DTC_TRY(cap(n, cp + ".da1", G[4], st));
      DTC_TRY(bn_bwd_reduce(G[4], n.at<u16>(b.A1), n.at<u16>(b.C1), n.at<float>(b.b1.mean),
                            n.at<float>(b.b1.invstd), n.at<int64_t>(b.b1.acc), nullptr, nullptr, nullptr, nullptr,
                            G[4], M, b.Cout, st));
    }
    DTC_TRY(cap(n, cp + ".dz1", G[4], st));
    DTC_TRY(bn_bwd_coef_apply(n, b.b1, G[4], n.at<u16>(b.C1), dc1, nullptr, nullptr, nullptr, M, gs, st));
    DTC_TRY(cap(n, cp + ".dc1", dc1, st));
    // conv1 (+ shortcut): weight grads (side stream), then the block-input gradient with the residual fused
    DTC_TRY(fork_side(n, st, &sd));
    DTC_TRY(wg_issue(n, wq, b.c1.s, in, dc1, n.gf(b.c1.pidx), gs, slabw, sd));
    // the block input's gradient feeds the previous block's bn2 (+ its projection BN) or the stem BN
    BnbArgs bp;
    if (bi > 0) {
      BlockL& pb = n.blocks[bi - 1];
      bp = bnb_of(n, pb.OUT, pb.C2, pb.b2, pb.proj ? pb.S : 0, pb.proj ? &pb.bsc : nullptr);
    } else {
      bp = bnb_of(n, n.A0, n.C0, n.bn0);
    }
    const BnbArgs* bpp = fuse ? &bp : nullptr;
    if (b.proj) {
      PROF(2, conv_flops(b.sc.s), conv_wgrad(b.sc.s, in, dsc, n.gf(b.sc.pidx), 0, 0, gs, slabw, n.slab_bytes, sd, ts));
      PROF(1, conv_flops(b.sc.s), conv_dgrad(b.sc.s, dsc, n.wbf(b.sc.pidx), G[5], nullptr, slab, n.slab_bytes, st, ts));
      PROF(1, conv_flops(b.c1.s), conv_dgrad(b.c1.s, dc1, n.wbf(b.c1.pidx), G[0], G[5], slab, n.slab_bytes, st, ts, bpp));
    } else {  // fused: dz2 is G[0] and the dgrad updates it in place (residual read, dz written per element)
      PROF(1, conv_flops(b.c1.s), conv_dgrad(b.c1.s, dc1, n.wbf(b.c1.pidx), G[0], dz2, slab, n.slab_bytes, st, ts, bpp));
    }
    dz_ready = fuse;
    if (b.proj) DTC_TRY(cap(n, cp + ".dxs", G[5], st));
    DTC_TRY(cap(n, cp + ".dx", G[0], st));
    if (bucket_fires(n, bi)) DTC_TRY(wg_flush(n, wq, gs, slabw, sd));
    DTC_TRY(maybe_bucket(n, bi, cx, st));
  }
  // stem: a0 = relu(bn1(conv1(x)))
  const int64_t M0 = (int64_t)n.B * n.H * n.W;
  u16* dc0 = n.at<u16>(n.DC0);
  u16* dz0 = G[0];
  if (!dz_ready) {
    dz0 = G[1];
    DTC_TRY(bn_bwd_reduce(G[0], n.at<u16>(n.A0), n.at<u16>(n.C0), n.at<float>(n.bn0.mean),
                          n.at<float>(n.bn0.invstd), n.at<int64_t>(n.bn0.acc), nullptr, nullptr, nullptr, nullptr, G[1],
                          M0, 64, st));
  }
  DTC_TRY(bn_bwd_coef_apply(n, n.bn0, dz0, n.at<u16>(n.C0), dc0, nullptr, nullptr, nullptr, M0, gs, st));
  DTC_TRY(cap(n, "grad.stem.dz", dz0, st));
  DTC_TRY(cap(n, "grad.stem.dc", dc0, st));
  DTC_TRY(wg_flush(n, wq, gs, slabw, sd));
  DTC_TRY(join_side(n, st));  // the stem wgrad is the last kernel: run it on the main stream
  PROF(2, 2.0 * M0 * 64 * 27,
       n.stem_direct ? stem_wgrad(n.at<float>(n.XIN), dc0, n.gf(n.stem.pidx), gs, n.B, n.H, n.W, slab, n.slab_bytes, st, ts)
                     : conv_wgrad(n.stem.s, n.at<u16>(n.X0), dc0, n.gf(n.stem.pidx), 27, 27, gs, slab, n.slab_bytes, st, ts));
  DTC_TRY(maybe_bucket(n, -1, cx, st));
  if (n.profiling) DTC_TRY(prof_accumulate(n.prof_ts, Net::PROF_SLOTS, n.prof_acc, st));
  return 0;
}

static int backward_impl(Net& n, const float* dlogits, float gs, Comm* comm, hipStream_t st);
static int backward(Net& n, const float* dlogits, float gs, Comm* comm, hipStream_t st) {
  n.ct_cur = nullptr;
  if (comm && n.ct_left > 0 && n.ct_used < (int)n.ct.size()) {
    n.ct_cur = &n.ct[n.ct_used++];
    --n.ct_left;
    n.ct_cur->join = n.ct_cur->tail = n.ct_cur->ok = false;
    n.ct_cur->bucket.assign(n.ct_cur->b0.size(), false);
    DTC_HIP(hipEventRecord(n.ct_cur->bwd0, st));
  }
  const int rc = backward_impl(n, dlogits, gs, comm, st);
  if (rc == 0 && n.ct_cur) {
    DTC_HIP(hipEventRecord(n.ct_cur->tail_b, st));  // after the Reducer's join
    n.ct_cur->ok = true;
  }
  n.ct_cur = nullptr;
  return rc;
}
static int backward_impl(Net& n, const float* dlogits, float gs, Comm* comm, hipStream_t st) {
  n.prof_st = st;
  if (!n.sums_fresh) DTC_TRY(zero_bytes(n.ws + n.acc_lo, n.stats_hi - n.acc_lo, st));
  n.sums_fresh = false;
  if (!graphs_on(n, true, comm != nullptr)) {
    BwdCtx cx;
    cx.comm = comm;
    const int rc = backward_body(n, dlogits, gs, cx, st);
    g_fork_watch = ForkWatch{};
    DTC_TRY(rc);
  } else {
    const int pi = n.profiling ? 1 : 0;
    if (!n.bwd_segs[pi].empty() && (n.bwd_gs[pi] != gs || n.bwd_comm[pi] != (comm != nullptr))) drop_graphs(n);
    if (n.bwd_segs[pi].empty()) {
      std::vector<Net::Seg> segs;
      BwdCtx cx;
      cx.comm = comm;
      cx.capturing = true;
      cx.segs = &segs;
      Net::Seg tail;
      int rc = begin_capture(n);
      if (rc == 0) rc = end_capture(n, backward_body(n, n.at<float>(n.DLOGITS), gs, cx, n.cap_st), &tail.exec);
      if (rc != 0) {
        for (auto& sg : segs)
          if (sg.exec) (void)hipGraphExecDestroy(sg.exec);
        return rc;
      }
      segs.push_back(tail);
      n.bwd_segs[pi] = segs;
      n.bwd_gs[pi] = gs;
      n.bwd_comm[pi] = comm != nullptr;
    }
    if (dlogits != n.at<float>(n.DLOGITS))
      DTC_HIP(hipMemcpyAsync(n.at<float>(n.DLOGITS), dlogits, (size_t)n.B * n.ncls * 4, hipMemcpyDeviceToDevice, st));
    // option comm_on_side: each bucket's collective on the weight-gradient stream forked from the compute
    // stream after its segment (that stream is idle between the replayed segments), joined once at the end:
    // no stream of the communicator's own in the backward
    const bool on_side = option_get(OPT_COMM_ON_SIDE) != 0 && comm != nullptr;
    for (const auto& sg : n.bwd_segs[pi]) {
      if (sg.exec) DTC_TRY(graph_launch(n, sg.exec, st));
      for (int i : sg.buckets) {
        hipEvent_t t0 = nullptr, t1 = nullptr;
        if (n.ct_cur && i < (int)n.ct_cur->b0.size()) {
          t0 = n.ct_cur->b0[i];
          t1 = n.ct_cur->b1[i];
          n.ct_cur->bucket[i] = true;
        }
        if (on_side) {
          hipStream_t sd = st;
          DTC_TRY(fork_side(n, st, &sd));
          DTC_TRY(comm_allreduce_on(comm, n.g + n.bucket_off[i], (size_t)n.bucket_len[i], sd, t0, t1));
        } else {
          DTC_TRY(comm_allreduce_async(comm, n.g + n.bucket_off[i], (size_t)n.bucket_len[i], st, t0, t1));
        }
      }
    }
    if (on_side) DTC_TRY(join_side(n, st));
  }
  if (comm) DTC_TRY(comm_join(comm, st));
  return 0;
}

}  // namespace dtc

// ------------------------------------------------------------------ C ABI (executor part)
#include "../../include/dtc.h"

struct dtc_net {
  dtc::Net n;
  float bucket_cap_mb = 25.f;
};

using namespace dtc;

extern "C" {

int dtc_rn18_create(dtc_net** out, int batch, int height, int width, int num_classes, float bucket_cap_mb) {
  DTC_CHECK_ARG(out != nullptr, "dtc_rn18_create: null out");
  DTC_CHECK_ARG(batch > 0 && height >= 8 && width >= 8 && num_classes > 0, "dtc_rn18_create: bad shape");
  // Kernels whose buffer descriptors take 32-bit byte offsets (conv_c64, conv_halo, wgrad_halo, the
  // igemm fast wgrad loader) gate themselves on tensors < 2 GiB and the executor falls back to the
  // 64-bit-addressed implicit-GEMM loaders above that (224x224 at batch > 333). What remains is the
  // element index of the largest activation, [batch, height, width, 64]: it must fit an int32
  // (224x224: batch <= 684; BASELINE config 5 is 512).
  DTC_CHECK_ARG((int64_t)batch * height * width * 64 < (1ll << 31),
                "dtc_rn18_create: activation too large (batch*height*width*64 elements >= 2^31)");
  dtc_net* h = new dtc_net();
  h->n.B = batch;
  h->n.H = height;
  h->n.W = width;
  h->n.ncls = num_classes;
  int r = build(h->n);
  if (r) {
    delete h;
    return r;
  }
  h->bucket_cap_mb = bucket_cap_mb;
  plan_workspace(h->n, bucket_cap_mb);
  *out = h;
  return 0;
}

static void ct_free(Net& n);
int dtc_rn18_destroy(dtc_net* net) {
  if (net) {
    drop_graphs(net->n);
    ct_free(net->n);
    if (net->n.cap_st) (void)hipStreamDestroy(net->n.cap_st);
    if (net->n.side_st) (void)hipStreamDestroy(net->n.side_st);
    if (net->n.sc_st) (void)hipStreamDestroy(net->n.sc_st);
    for (auto& e : net->n.evs)
      if (e) (void)hipEventDestroy(e);
    if (net->n.launch_ev) (void)hipEventDestroy(net->n.launch_ev);
  }
  delete net;
  return 0;
}

int dtc_rn18_num_params(const dtc_net* net) { return net ? (int)net->n.params.size() : DTC_EINVAL; }

int dtc_rn18_param_info(const dtc_net* net, int idx, const char** name, int64_t* offset, int64_t* numel, int* ndim,
                        int64_t* shape4, int64_t* stride4) {
  DTC_CHECK_ARG(net && idx >= 0 && idx < (int)net->n.params.size(), "dtc_rn18_param_info: bad index");
  const ParamEntry& e = net->n.params[idx];
  if (name) *name = e.name.c_str();
  if (offset) *offset = e.offset;
  if (numel) *numel = e.numel;
  if (ndim) *ndim = e.ndim;
  for (int i = 0; i < 4; ++i) {
    if (shape4) shape4[i] = e.shape[i];
    if (stride4) stride4[i] = e.stride[i];
  }
  return 0;
}

int64_t dtc_rn18_flat_numel(const dtc_net* net) { return net ? net->n.flat_numel : DTC_EINVAL; }
int dtc_rn18_num_bn(const dtc_net* net) { return net ? (int)net->n.bns.size() : DTC_EINVAL; }

int dtc_rn18_bn_info(const dtc_net* net, int idx, const char** prefix, int* channels, int64_t* mean_offset,
                     int64_t* var_offset) {
  DTC_CHECK_ARG(net && idx >= 0 && idx < (int)net->n.bns.size(), "dtc_rn18_bn_info: bad index");
  const BNL* b = net->n.bns[idx];
  if (prefix) *prefix = b->prefix.c_str();
  if (channels) *channels = b->C;
  if (mean_offset) *mean_offset = b->rm_off;
  if (var_offset) *var_offset = b->rv_off;
  return 0;
}

int64_t dtc_rn18_bufs_numel(const dtc_net* net) { return net ? net->n.bufs_numel : DTC_EINVAL; }
size_t dtc_rn18_workspace_bytes(const dtc_net* net) { return net ? net->n.ws_bytes : 0; }
int dtc_rn18_num_buckets(const dtc_net* net) { return net ? (int)net->n.bucket_off.size() : DTC_EINVAL; }

int dtc_rn18_bucket_info(const dtc_net* net, int idx, int64_t* offset, int64_t* numel) {
  DTC_CHECK_ARG(net && idx >= 0 && idx < (int)net->n.bucket_off.size(), "dtc_rn18_bucket_info: bad index");
  if (offset) *offset = net->n.bucket_off[idx];
  if (numel) *numel = net->n.bucket_len[idx];
  return 0;
}

int dtc_rn18_bind(dtc_net* net, void* workspace, float* params, float* grads, uint16_t* params_bf16, float* bufs,
                  int64_t* num_batches_tracked, void* stream) {
  DTC_CHECK_ARG(net && workspace && params && grads && params_bf16 && bufs, "dtc_rn18_bind: null pointer");
  DTC_CHECK_ARG(((uintptr_t)workspace & 255) == 0, "dtc_rn18_bind: workspace must be 256-byte aligned");
  DTC_CHECK_ARG(((uintptr_t)params_bf16 & 15) == 0 && ((uintptr_t)params & 15) == 0 && ((uintptr_t)grads & 15) == 0,
                "dtc_rn18_bind: parameter buffers must be 16-byte aligned");
  Net& n = net->n;
  n.ws = (char*)workspace;
  n.p = params;
  n.g = grads;
  n.pb = params_bf16;
  n.bufs = bufs;
  n.nbt = num_batches_tracked;
  n.prof_ts = n.at<u64>(n.PROF_TS);
  n.prof_acc = n.at<u64>(n.PROF_ACC);
  drop_graphs(n);  // captured launches hold the previous pointers
  DTC_HIP(hipMemsetAsync(n.ws + n.stats_lo, 0, n.stats_hi - n.stats_lo, (hipStream_t)stream));
  DTC_HIP(hipMemsetAsync(n.ws + n.TICK, 0, (size_t)DTC_TICKS * 4, (hipStream_t)stream));
  return 0;
}

int dtc_rn18_enable_capture(dtc_net* net) {
  DTC_CHECK_ARG(net && net->n.ws == nullptr, "dtc_rn18_enable_capture: call before dtc_rn18_bind");
  net->n.capture = true;
  plan_workspace(net->n, net->bucket_cap_mb);
  return 0;
}

int dtc_rn18_set_precision(dtc_net* net, int fp32) {
  DTC_CHECK_ARG(net && net->n.ws == nullptr, "dtc_rn18_set_precision: call before dtc_rn18_bind");
  net->n.f32 = fp32 != 0;
  plan_workspace(net->n, net->bucket_cap_mb);
  return 0;
}

int dtc_rn18_precision(const dtc_net* net) { return net ? (net->n.f32 ? 1 : 0) : DTC_EINVAL; }

int dtc_rn18_num_captures(const dtc_net* net) { return net ? (int)net->n.caps.size() : DTC_EINVAL; }

int dtc_rn18_capture_info(const dtc_net* net, int idx, const char** name, size_t* ws_offset, int* shape4) {
  DTC_CHECK_ARG(net && idx >= 0 && idx < (int)net->n.caps.size(), "dtc_rn18_capture_info: bad index");
  const auto& a = net->n.caps[idx];
  if (name) *name = a.name.c_str();
  if (ws_offset) *ws_offset = a.off;
  if (shape4) {
    shape4[0] = a.n; shape4[1] = a.h; shape4[2] = a.w; shape4[3] = a.c;
  }
  return 0;
}

int dtc_rn18_num_activations(const dtc_net* net) { return net ? (int)net->n.acts.size() : DTC_EINVAL; }

int dtc_rn18_activation_info(const dtc_net* net, int idx, const char** name, size_t* ws_offset, int* shape4) {
  DTC_CHECK_ARG(net && idx >= 0 && idx < (int)net->n.acts.size(), "dtc_rn18_activation_info: bad index");
  const auto& a = net->n.acts[idx];
  if (name) *name = a.name.c_str();
  if (ws_offset) *ws_offset = a.off;
  if (shape4) {
    shape4[0] = a.n; shape4[1] = a.h; shape4[2] = a.w; shape4[3] = a.c;
  }
  return 0;
}

int dtc_rn18_dlogits_buffer(const dtc_net* net, size_t* ws_offset) {
  DTC_CHECK_ARG(net && ws_offset, "dtc_rn18_dlogits_buffer: bad args");
  *ws_offset = net->n.DLOGITS;
  return 0;
}

int dtc_rn18_profile_begin(dtc_net* net, int capacity) {
  DTC_CHECK_ARG(net && capacity > 0 && net->n.ws, "dtc_rn18_profile_begin: bad args or unbound net");
  Net& n = net->n;
  const size_t bytes = (size_t)Net::PROF_SLOTS * 2 * sizeof(u64);
  const size_t ts_bytes = (size_t)Net::PROF_SLOTS * DTC_PROF_SLOT_U64 * sizeof(u64);
  int dev = 0;
  DTC_HIP(hipGetDevice(&dev));
  DTC_HIP(hipDeviceGetAttribute(&n.prof_khz, hipDeviceAttributeWallClockRate, dev));
  DTC_CHECK_ARG(n.prof_khz > 0, "dtc_rn18_profile_begin: no wall clock rate");
  // the previous step may still run (its profiled graphs stamp these slots): drain, then reset.
  // slots -> (~0, 0) (folding all-zero slots adds nothing and resets them), then totals -> 0.
  // The drains hold g_graph_mu like drop_graphs: no device drain while another host
  // thread's stream is capturing.
  std::lock_guard<std::recursive_mutex> lk(g_graph_mu);
  DTC_HIP(hipDeviceSynchronize());
  DTC_HIP(hipMemset(n.prof_ts, 0, ts_bytes));
  DTC_TRY(prof_accumulate(n.prof_ts, Net::PROF_SLOTS, n.prof_acc, nullptr));
  DTC_HIP(hipMemset(n.prof_acc, 0, bytes));
  DTC_HIP(hipDeviceSynchronize());
  n.profiling = true;  // the next calls launch (capturing on first use) the profiled graph set
  return 0;
}

int dtc_rn18_profile_events(dtc_net* net, int pairs) {
  DTC_CHECK_ARG(net && pairs >= 0, "dtc_rn18_profile_events: bad args");
  Net& n = net->n;
  n.prof_events = pairs > 0;
  n.prof_evn = 0;
  n.prof_evdropped = 0;
  const size_t want = (size_t)pairs * 2;
  while (n.prof_evpool.size() < want) {
    hipEvent_t e;
    // timing events without the system-scope release fence at completion (no L2 write-back between the
    // bracketed launches: the kernels see the caches the unbracketed step gives them)
    DTC_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    n.prof_evpool.push_back(e);
  }
  return 0;
}

int dtc_rn18_profile_events_result(dtc_net* net, int nkinds, double* ms_by_kind, double* work_by_kind,
                                   int* count_by_kind) {
  DTC_CHECK_ARG(net != nullptr && nkinds >= 1 && nkinds <= 4, "dtc_rn18_profile_events_result: bad args");
  Net& n = net->n;
  for (int k = 0; k < nkinds; ++k) {
    if (ms_by_kind) ms_by_kind[k] = 0;
    if (work_by_kind) work_by_kind[k] = 0;
    if (count_by_kind) count_by_kind[k] = 0;
  }
  for (size_t i = 0; i < n.prof_evn; ++i) {
    const int k = n.prof_evwork[i].first;
    if (k >= nkinds) continue;
    DTC_HIP(hipEventSynchronize(n.prof_evpool[2 * i + 1]));
    float ms = 0.f;
    DTC_HIP(hipEventElapsedTime(&ms, n.prof_evpool[2 * i], n.prof_evpool[2 * i + 1]));
    if (ms_by_kind) ms_by_kind[k] += ms;
    if (work_by_kind) work_by_kind[k] += n.prof_evwork[i].second;
    if (count_by_kind) count_by_kind[k] += 1;
  }
  n.prof_evn = 0;
  n.prof_events = false;
  return 0;
}

static void ct_free(Net& n) {
  for (auto& c : n.ct) {
    for (hipEvent_t e : {c.bwd0, c.join_c, c.join_d, c.tail_a, c.tail_b})
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c.b0) (void)hipEventDestroy(e);
    for (hipEvent_t e : c.b1) (void)hipEventDestroy(e);
  }
  n.ct.clear();
  n.ct_left = n.ct_used = 0;
}

int dtc_rn18_comm_timing(dtc_net* net, int steps) {
  DTC_CHECK_ARG(net && steps >= 0 && steps <= 100000, "dtc_rn18_comm_timing: bad args");
  Net& n = net->n;
  ct_free(n);
  const size_t nb = n.bucket_off.size();
  n.ct.resize(steps);
  for (auto& c : n.ct) {
    for (hipEvent_t* e : {&c.bwd0, &c.join_c, &c.join_d, &c.tail_a, &c.tail_b}) DTC_HIP(hipEventCreate(e));
    c.b0.resize(nb);
    c.b1.resize(nb);
    for (size_t i = 0; i < nb; ++i) {
      DTC_HIP(hipEventCreate(&c.b0[i]));
      DTC_HIP(hipEventCreate(&c.b1[i]));
    }
  }
  n.ct_left = steps;
  return 0;
}

int dtc_rn18_comm_timing_result(dtc_net* net, int max_buckets, double* bucket_us, double* exposed_us, int* steps) {
  DTC_CHECK_ARG(net && max_buckets >= 0 && (max_buckets == 0 || bucket_us) && exposed_us && steps,
                "dtc_rn18_comm_timing_result: bad args");
  Net& n = net->n;
  const int nb = std::min<int>(max_buckets, (int)n.bucket_off.size());
  for (int i = 0; i < 3 * max_buckets; ++i) bucket_us[i] = 0.0;
  for (int i = 0; i < 5; ++i) exposed_us[i] = 0.0;
  auto us = [](hipEvent_t a, hipEvent_t b, double& out) -> int {
    float ms = 0.f;
    DTC_HIP(hipEventSynchronize(b));
    DTC_HIP(hipEventElapsedTime(&ms, a, b));
    out = 1e3 * (double)ms;
    return 0;
  };
  int recorded = 0, joined = 0, tailed = 0;
  std::vector<int> bcount(nb, 0);
  for (int k = 0; k < n.ct_used; ++k) {
    Net::CommTimes& c = n.ct[k];
    if (!c.ok) continue;  // a backward that failed recorded no end event
    double bwd = 0;
    if (c.tail) {  // (a replayed backward records no tail / join events)
      double tail = 0;
      DTC_TRY(us(c.tail_a, c.tail_b, tail));
      exposed_us[0] += tail;
      ++tailed;
    }
    DTC_TRY(us(c.bwd0, c.tail_b, bwd));
    exposed_us[3] += bwd;
    if (c.join) {
      double j = 0;
      DTC_TRY(us(c.join_c, c.join_d, j));
      exposed_us[1] += j;
      ++joined;
    }
    for (int i = 0; i < nb; ++i) {
      if (!c.bucket[i]) continue;
      double a = 0, b = 0;
      DTC_TRY(us(c.bwd0, c.b0[i], a));
      DTC_TRY(us(c.bwd0, c.b1[i], b));
      bucket_us[3 * i] += a;
      bucket_us[3 * i + 1] += b;
      bucket_us[3 * i + 2] += b - a;
      ++bcount[i];
    }
    ++recorded;
  }
  // tail: the mean over the steps that recorded one, -1 when none did (replayed backwards: unavailable)
  exposed_us[0] = tailed ? exposed_us[0] / tailed : -1.0;
  if (recorded) exposed_us[3] /= recorded;
  if (joined) exposed_us[1] /= joined;
  exposed_us[2] = tailed ? exposed_us[0] + exposed_us[1] : -1.0;
  exposed_us[4] = joined;
  for (int i = 0; i < nb; ++i)
    if (bcount[i])
      for (int j = 0; j < 3; ++j) bucket_us[3 * i + j] /= bcount[i];
  *steps = recorded;
  ct_free(n);
  return 0;
}

int dtc_rn18_profile_events_dropped(dtc_net* net, long long* dropped) {
  DTC_CHECK_ARG(net != nullptr && dropped != nullptr, "dtc_rn18_profile_events_dropped: bad args");
  *dropped = net->n.prof_evdropped;
  return 0;
}

int dtc_rn18_profile_end(dtc_net* net, double* ms_by_kind, double* flops_by_kind, int* count_by_kind) {
  return dtc_rn18_profile_end_ex(net, 3, ms_by_kind, flops_by_kind, count_by_kind);
}

int dtc_rn18_profile_end_ex(dtc_net* net, int nkinds, double* ms_by_kind, double* work_by_kind, int* count_by_kind) {
  DTC_CHECK_ARG(net != nullptr && nkinds >= 1 && nkinds <= 4, "dtc_rn18_profile_end_ex: bad args");
  double* flops_by_kind = work_by_kind;
  Net& n = net->n;
  for (int k = 0; k < nkinds; ++k) {
    if (ms_by_kind) ms_by_kind[k] = 0;
    if (flops_by_kind) flops_by_kind[k] = 0;
    if (count_by_kind) count_by_kind[k] = 0;
  }
  if (!n.profiling) return 0;
  std::vector<u64> acc((size_t)Net::PROF_SLOTS * 2);
  std::lock_guard<std::recursive_mutex> lk(g_graph_mu);  // as profile_begin
  DTC_HIP(hipDeviceSynchronize());
  DTC_HIP(hipMemcpy(acc.data(), n.prof_acc, acc.size() * sizeof(u64), hipMemcpyDeviceToHost));
  for (int i = 0; i < Net::PROF_SLOTS; ++i) {
    const u64 calls = acc[2 * i + 1];
    if (calls == 0) continue;
    const int k = n.prof_kind[i];
    if (k >= nkinds) continue;
    if (ms_by_kind) ms_by_kind[k] += (double)acc[2 * i] / (double)n.prof_khz;
    if (flops_by_kind) flops_by_kind[k] += n.prof_flops[i] * (double)calls;
    if (count_by_kind) count_by_kind[k] += (int)calls;
  }
  n.profiling = false;  // back to the plain graph set; both sets stay captured
  return 0;
}

int dtc_rn18_set_sync_bn(dtc_net* net, dtc_comm* comm) {
  DTC_CHECK_ARG(net != nullptr, "dtc_rn18_set_sync_bn: null net");
  Net& n = net->n;
  n.sync = (Comm*)comm;
  n.sync_world = comm ? comm_world((Comm*)comm) : 1;
  drop_graphs(n);
  return 0;
}

int dtc_rn18_forward(dtc_net* net, const float* x, float* logits, int train, void* stream) {
  DTC_CHECK_ARG(net && net->n.ws && x && logits, "dtc_rn18_forward: unbound net or null pointer");
  return forward(net->n, x, logits, train != 0, (hipStream_t)stream);
}

int dtc_rn18_backward(dtc_net* net, const float* dlogits, float grad_scale, dtc_comm* comm, void* stream) {
  DTC_CHECK_ARG(net && net->n.ws && dlogits, "dtc_rn18_backward: unbound net or null pointer");
  return backward(net->n, dlogits, grad_scale, (Comm*)comm, (hipStream_t)stream);
}

int dtc_rn18_xent_backward(dtc_net* net, const float* logits, const int64_t* labels, const float* lse,
                           const float* gscale, float grad_scale, dtc_comm* comm, void* stream) {
  DTC_CHECK_ARG(net && net->n.ws && logits && labels && lse, "dtc_rn18_xent_backward: unbound net or null pointer");
  Net& n = net->n;
  float* dl = n.at<float>(n.DLOGITS);
  // option xent_fuse: the eager backward's head kernel computes dlogits itself (and still stores it into
  // the dlogits buffer); a graph-replayed backward keeps the separate launch (its head reads the buffer)
  if (option_get(OPT_XENT_FUSE) != 0 && !n.capture && !graphs_on(n, true, comm != nullptr)) {
    n.xent.logits = logits;
    n.xent.labels = labels;
    n.xent.lse = lse;
    n.xent.gscale = gscale;
    const int rc = backward(n, dl, grad_scale, (Comm*)comm, (hipStream_t)stream);
    n.xent = XentArgs();
    return rc;
  }
  DTC_TRY(xent_bwd(logits, labels, lse, gscale, n.B, n.ncls, dl, (hipStream_t)stream));
  return backward(n, dl, grad_scale, (Comm*)comm, (hipStream_t)stream);
}

}  // extern "C"
