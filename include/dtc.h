/*
 * dtc.h — C ABI of libdtc_amd.so: the MI355X-native (gfx950) kernels and executor for the
 * ResNet-18 / CIFAR-100 data-parallel training step of youngerous/distributed-training-comparison.
 *
 * The reference has no FFI of its own: its operator boundary is the PyTorch module API that
 * src/{single,dp,ddp}/net.py and trainer.py call (nn.Conv2d, nn.BatchNorm2d, F.relu,
 * F.avg_pool2d, nn.Linear, nn.CrossEntropyLoss, optim.SGD, GradScaler, DDP). Every entry
 * point below names the reference call it replaces (file:line under the reference tree).
 *
 * Conventions
 *   - plain C types only; bf16 tensors are uint16_t words (IEEE bfloat16 bit patterns);
 *   - activations are NHWC; conv filters are KRSC ([out][kh][kw][in], in innermost);
 *   - every compute call takes `stream` = a hipStream_t (void* here) and only enqueues work;
 *   - the CALLER owns every device buffer, workspaces included; the library never allocates
 *     or frees caller memory inside a call. Handles (dtc_comm, dtc_net) are library-owned and
 *     released by their destroy function;
 *   - return value: 0 = ok, > 0 = hipError_t / ncclResult_t passed through, < 0 = invalid
 *     argument. dtc_last_error() gives the message (thread-local). Nothing throws or exits;
 *   - reentrant: no unguarded global mutable state; calls for different devices may be made
 *     from different threads (the device is the one current on the calling thread).
 */
#ifndef DTC_AMD_H
#define DTC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DTC_ABI_VERSION 1

/* ------------------------------------------------------------------ library */
int dtc_abi_version(void);
const char* dtc_last_error(void);
/* Diagnostics: on SIGSEGV/SIGBUS/SIGFPE/SIGABRT print the faulting native thread (tid, name) and its
 * frames to stderr, then chain to the previous handler (e.g. Python's faulthandler). Idempotent. */
int dtc_install_crash_handler(void);
/* Process-wide kernel tuning knobs (atomic; for benchmarking and A/B measurement). The full list, with
 * defaults and one line each, is the DTC_OPTIONS table in csrc/kernels.h; unknown names return DTC_EINVAL.
 * Examples: "graphs" (0 eager, 1 forward + backward hipGraphs, 2 forward only, 3 backward only,
 * default 4 = auto: the executor captures on first use and replays; any option change invalidates
 * captured graphs), "splitk_ink" (split-K slabs summed in-kernel by the last workgroup of each tile,
 * default 1), "dgrad_s2h" (stride-2 data gradient as a halo sub-pixel conv, default 1), "stem_direct"
 * (plan time: direct 3x3 stem conv, default 1; 0 = im2col + GEMM). */
int dtc_set_option(const char* name, int value);
int dtc_get_option(const char* name);

/* ------------------------------------------------------------------ convolution
 * Replaces nn.Conv2d(bias=False) forward / backward (reference src/ddp/net.py:18-24,
 * net.py:29-35, net.py:91) as launched by autocast (cuDNN in the reference).
 * Requirements: c % 64 == 0, k % 64 == 0, stride in {1, 2} (the 3-channel stem has its own direct
 * kernels, dtc_stem_*; dtc_stem_im2col + a 1x1 "conv" over 64 im2col channels is kept as the
 * stem_direct=0 variant). */
typedef struct {
  int n, h, w, c; /* input  [n][h][w][c]  bf16 */
  int k, r, s;    /* filter [k][r][s][c]  bf16 */
  int stride, pad;
} dtc_conv_desc;

enum { DTC_CONV_FWD = 0, DTC_CONV_DGRAD = 1, DTC_CONV_WGRAD = 2 };

/* bytes of workspace the given pass wants: split-K partial slabs (fp32), and for FWD / DGRAD split-K also
 * the arrival counters of the in-kernel reduction (the last workgroup of each output tile sums the slab;
 * option splitk_ink). 0 is valid for FWD/DGRAD; a workspace with room for the slab only reduces the slab in
 * a separate launch. */
size_t dtc_conv2d_workspace_size(const dtc_conv_desc* d, int pass);
/* y[n][p][q][k] = conv(x, w); if stats != NULL, per-channel (sum, sum^2) of the bf16 output are
 * ADDED into stats — the batch statistics BatchNorm2d needs (net.py:21). A statistics accumulator is
 * dtc_bn_stat_words(k) int64 words, zeroed before its first producer: exact fixed-point sums, so the
 * totals do not depend on the order of the producers' atomic adds (the step is bit-reproducible, as the
 * reference's cudnn.deterministic asks, src/ddp/utils.py:12-13); dtc_bn_stat_totals reads them. */
int dtc_conv2d_fwd(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t* stats,
                   void* ws, size_t ws_bytes, void* stream);
/* dx = conv^T(dy, w) (+ res if non-NULL): the input gradient of Conv2d */
/* 3x3 stride-2 conv (desc) and its BasicBlock's 1x1 stride-2 projection shortcut (net.py:18-19, 29-36) of
 * the same input in one launch: y = conv(x, w), ysc = conv1x1_s2(x, wsc [K][C]); optional BN statistics of
 * each. The shortcut reads exactly the 3x3's centre-tap pixels, so x is read once. Returns
 * DTC_EINVAL for geometries without a fused plan (callers then run the two convs separately). */
int dtc_conv2d_fwd_sc(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t* stats,
                      const uint16_t* wsc, uint16_t* ysc, int64_t* stats_sc, void* stream);
int dtc_conv2d_dgrad(const dtc_conv_desc* d, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                     const uint16_t* res, void* ws, size_t ws_bytes, void* stream);
/* The same dgrad when dx is the gradient of a post-ReLU BatchNorm output y = relu(bn(x1) [+ bn2(x2)])
 * (net.py:41-44, 108): stores dz = bf16(dx) * [ymask > 0] in dx and ADDS the BN-backward sums into
 * acc1 (and acc2 if x2) exactly as dtc_bn_bwd_reduce would on that dz -- in the conv's epilogue where
 * the kernel has one (3x3 stride 1 and split-K paths), else as a second pass. dx may alias res. */
int dtc_conv2d_dgrad_bn(const dtc_conv_desc* d, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                        const uint16_t* res, const uint16_t* ymask, const uint16_t* x1, const float* mean1,
                        const float* invstd1, int64_t* acc1, const uint16_t* x2, const float* mean2,
                        const float* invstd2, int64_t* acc2, void* ws, size_t ws_bytes, void* stream);
/* dx of a projection block's input through conv1 (3x3 stride 2, desc) AND the 1x1 stride-2 shortcut
 * (net.py:18-19, 29-36) in one launch: dx = dgrad(dy, w) + dgrad(dsc, wsc [K][C]); the shortcut's term is
 * nonzero only at the (even, even) pixels and runs as extra reduction steps of that parity class. */
int dtc_conv2d_dgrad_sc(const dtc_conv_desc* d, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                        const uint16_t* dsc, const uint16_t* wsc, void* stream);
/* dw[k][r][s][c] (fp32) = scale * sum over pixels of dy (x) im2col(x): the weight gradient */
int dtc_conv2d_wgrad(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* dy, float* dw, float scale,
                     void* ws, size_t ws_bytes, void* stream);
/* n (1..4) independent weight gradients of one 3x3 / stride-1 / pad-1 geometry (64-multiple
 * channels) in one halo launch + one reduce launch: dw[i] = scale * wgrad(x[i], dy[i]). The chip is
 * filled by n x splits workgroups, so each gradient's fp32 split-K slab is 1/n the size of a single
 * dtc_conv2d_wgrad's. Replaces the weight-gradient halves of n `nn.Conv2d` backward passes
 * (net.py:18-24, 29-35) that autograd would run one by one. Workspace: ..._batch_workspace_size
 * (0 = no halo plan for this geometry: use dtc_conv2d_wgrad per problem). */
/* The weight gradients of a projection block's 3x3 stride-2 conv1 (desc) and its 1x1 stride-2 shortcut
 * (net.py:18-19, 29-36) in one launch (+ two fixed-order reduces): dw [K][3][3][C] from (x, dy), dw_sc [K][C]
 * from (x, dsc); the shortcut is the centre tap of conv1's operand, so x is read once. Workspace size 0:
 * no fused plan for the geometry (callers then run dtc_conv2d_wgrad for each). */
size_t dtc_conv2d_wgrad_sc_workspace_size(const dtc_conv_desc* d);
int dtc_conv2d_wgrad_sc(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* dy, const uint16_t* dsc, float* dw,
                        float* dw_sc, float scale, void* ws, size_t ws_bytes, void* stream);
size_t dtc_conv2d_wgrad_batch_workspace_size(const dtc_conv_desc* d, int n);
int dtc_conv2d_wgrad_batch(const dtc_conv_desc* d, int n, const uint16_t* const* x, const uint16_t* const* dy,
                           float* const* dw, float scale, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ batch norm (training)
 * Replaces nn.BatchNorm2d train-mode forward/backward (net.py:21,25,37,92) with the F.relu and
 * residual add of BasicBlock.forward (net.py:41-44) and ResNet.forward (net.py:108) fused.
 * x is NHWC bf16 with m = n*h*w pixels and c channels (c % 8 == 0). */
/* Size of one statistics accumulator for c channels, in int64 words (a header word holding the
 * non-finite flag, then 8 slots x 2 statistics x (hi, lo) x c). Zero it before its first producer. */
size_t dtc_bn_stat_words(int c);
/* Host-side read of an accumulator copied to host memory: totals[0][c] = first statistic (sum x / sum dz),
 * totals[1][c] = second (sum x^2 / sum dz*xhat), exactly as the BN kernels form them (NaN if flagged).
 * Pure host code, no device call. */
int dtc_bn_stat_totals(const int64_t* host_words, int c, double* totals);
int dtc_bn_fwd_finalize(int64_t* stats, int c, int64_t count, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum,
                        float eps, float* mean, float* invstd, float* scale, float* shift, void* stream);
int dtc_bn_apply_relu(const uint16_t* x, const float* scale, const float* shift, uint16_t* y, int64_t m, int c,
                      void* stream);
int dtc_bn_apply_add_relu(const uint16_t* x, const float* scale, const float* shift, const uint16_t* res,
                          uint16_t* y, int64_t m, int c, void* stream);
int dtc_bn_apply_dual_relu(const uint16_t* x, const float* scale, const float* shift, const uint16_t* x2,
                           const float* scale2, const float* shift2, uint16_t* y, int64_t m, int c, void* stream);
/* dz = dy * [ymask > 0] (ymask may be NULL: no ReLU); acc1 += (sum dz, sum dz*xhat1) and, if x2,
 * acc2 += (sum dz, sum dz*xhat2); acc* are statistics accumulators (dtc_bn_stat_words(c) int64) */
int dtc_bn_bwd_reduce(const uint16_t* dy, const uint16_t* ymask, const uint16_t* x1, const float* mean1,
                      const float* invstd1, int64_t* acc1, const uint16_t* x2, const float* mean2,
                      const float* invstd2, int64_t* acc2, uint16_t* dz, int64_t m, int c, void* stream);
/* dgamma = gscale*sum dz*xhat, dbeta = gscale*sum dz; coef[3][c] for dtc_bn_bwd_apply; acc re-zeroed */
int dtc_bn_bwd_finalize(int64_t* acc, int c, int64_t count, const float* gamma, const float* mean,
                        const float* invstd, float gscale, float* dgamma, float* dbeta, float* coef, void* stream);
int dtc_bn_bwd_apply(const uint16_t* dz, const uint16_t* x1, const float* coef1, uint16_t* dx1, const uint16_t* x2,
                     const float* coef2, uint16_t* dx2, int64_t m, int c, void* stream);

/* ------------------------------------------------------------------ stem, head, loss
 * stem: self.conv1 = nn.Conv2d(3, 64, 3, 1, 1) (net.py:91) as im2col [n*h*w][64] + GEMM.
 * head: F.avg_pool2d(out, 4) + view + self.linear (net.py:113-115), global pool.
 * loss: nn.CrossEntropyLoss() (trainer.py:40, 155), mean reduction. */
int dtc_stem_im2col(const float* x_nchw, uint16_t* cols, int n, int h, int w, void* stream);
int dtc_stem_pack_weight(const uint16_t* w27, uint16_t* w64, int k, void* stream);
/* Direct stem conv (the executor's default): y [n*h*w][64] bf16 = conv1(x) from fp32 NCHW x and the
 * bf16 KRSC weight [64][27], the 27 taps gathered per 256-pixel tile into LDS (no im2col matrix in
 * HBM); stats (optional, dtc_bn_stat_words(64) int64, accumulated) = BN batch sums of the bf16 outputs. The
 * weight gradient dw27 [64][27] fp32 = scale * sum_pixels dy (x) taps(x), workspace from
 * dtc_stem_wgrad_workspace_size. */
int dtc_stem_fwd(const float* x_nchw, const uint16_t* w27, uint16_t* y, int64_t* stats, int n, int h, int w,
                 void* stream);
size_t dtc_stem_wgrad_workspace_size(int n, int h, int w);
int dtc_stem_wgrad(const float* x_nchw, const uint16_t* dy, float* dw27, float scale, int n, int h, int w, void* ws,
                   size_t ws_bytes, void* stream);
int dtc_head_fwd(const uint16_t* act, int n, int hw, int c, const uint16_t* wfc, const float* bfc, int ncls,
                 float* feat, float* logits, void* stream);
size_t dtc_head_bwd_workspace_size(int n, int c, int ncls);
int dtc_head_bwd(const float* dlogits, const float* feat, const uint16_t* wfc, int n, int hw, int c, int ncls,
                 float scale, float* dw, float* db, uint16_t* dact, void* ws, size_t ws_bytes, void* stream);
int dtc_xent_fwd(const float* logits, const int64_t* labels, int n, int ncls, float* loss, float* lse,
                 void* stream);
/* The training step's loss in one launch (n <= 4096): loss and lse as dtc_xent_fwd (bit-identical), plus
 * scaled = loss * (*scale) when scaled != NULL (GradScaler.scale) and the loss stored into host_loss (a
 * pinned, device-accessible host word; NULL = none) -- read after an event recorded behind the launch. */
int dtc_xent_fwd_ex(const float* logits, const int64_t* labels, int n, int ncls, float* loss, float* lse,
                    const float* scale, float* scaled, float* host_loss, void* stream);
int dtc_xent_bwd(const float* logits, const int64_t* labels, const float* lse, const float* gscale, int n, int ncls,
                 float* dlogits, void* stream);

/* ------------------------------------------------------------------ optimizer / AMP
 * sgd: optim.SGD(lr, weight_decay, momentum, nesterov=True).step() (trainer.py:92-98, 158) over a
 * flat fp32 buffer; grads are multiplied by *inv_scale (GradScaler.unscale_) and the step is skipped
 * when *found_inf != 0 (GradScaler.step); p_bf16 receives the bf16 shadow of the new parameters.
 * amp: GradScaler's _amp_foreach_non_finite_check_and_unscale_ / _amp_update_scale_ (main.py:25). */
int dtc_sgd_nesterov_flat(float* p, const float* g, float* momentum_buf, uint16_t* p_bf16, int64_t n, float lr,
                          float weight_decay, float momentum, const float* inv_scale, const int* found_inf,
                          void* stream);
int dtc_cast_f32_bf16(const float* src, uint16_t* dst, int64_t n, void* stream);
int dtc_amp_check_finite(const float* g, int64_t n, int* found_inf, void* stream);
/* GradScaler.scale(loss): out = x * (*scale) with the scale device-resident (no host sync) */
int dtc_amp_scale(const float* x, const float* scale, float* out, int64_t n, void* stream);
int dtc_amp_update_scale(float* scale, float* inv_scale, int* growth_tracker, int* found_inf, float growth_factor,
                         float backoff_factor, int growth_interval, void* stream);

/* ------------------------------------------------------------------ input pipeline
 * Replaces the host DataLoader workers' per-sample transforms (src/ddp/dataset.py:43-64:
 * RandomCrop(32, padding=4) -> RandomHorizontalFlip -> ToTensor -> Normalize) and the
 * Subset/DistributedSampler gather (dataset.py:95-98) with one launch per batch.
 * images: uint8 [n_images][h][w][3] in device memory; targets: int64 [n_images] (may be NULL when
 * labels is NULL); index: int64 [n] dataset rows (NULL: 0..n-1); crop: uint8 [n][2] (row, col)
 * offsets into the zero-padded image, each in [0, 2*pad] (NULL: pad, pad = no crop shift);
 * flip: uint8 [n], non-zero = mirror (NULL: none); mean/std: HOST pointers to 3 floats;
 * out: fp32 [n][3][h][w]; labels: int64 [n] (NULL: skip); status: device int set to 1 when an index
 * is out of range or an offset exceeds 2*pad (that image is written as zeros before normalize,
 * label 0); never cleared by the call (NULL: skip). Requires w % 4 == 0 and h*w*3 <= 12 KiB. */
int dtc_cifar_augment(const uint8_t* images, const int64_t* targets, int64_t n_images, const int64_t* index,
                      const uint8_t* crop, const uint8_t* flip, int n, int h, int w, int pad, const float* mean,
                      const float* std, float* out, int64_t* labels, int* status, void* stream);

/* ------------------------------------------------------------------ RCCL communicator
 * Replaces the NCCL traffic of DistributedDataParallel (trainer.py:31): the construction-time
 * parameter broadcast, the per-forward buffer broadcast and the bucketed gradient all-reduce.
 * Bootstrap: rank 0 calls dtc_comm_get_unique_id, the id travels over the existing
 * torch.distributed rendezvous (init_process_group, ddp/main.py:18-23), every rank calls
 * dtc_comm_init. dtype: 0 = fp32, 1 = bf16, 2 = int64, 3 = fp64. */
typedef struct dtc_comm dtc_comm;
size_t dtc_comm_unique_id_bytes(void);
int dtc_comm_get_unique_id(void* out);
int dtc_comm_init(dtc_comm** out, int rank, int world, const void* unique_id, int device);
int dtc_comm_allreduce_sum(dtc_comm* comm, void* buf, size_t count, int dtype, void* stream);
int dtc_comm_broadcast(dtc_comm* comm, void* buf, size_t count, int dtype, int root, void* stream);
int dtc_comm_destroy(dtc_comm* comm);
/* torch.distributed.barrier() (reference ddp/trainer.py:156, dp/single variants have none): returns
 * once every rank called it and this rank's work enqueued on `stream` before the call has finished
 * (torch's NCCL barrier = a one-element all-reduce + a stream synchronize). One float is SUM
 * all-reduced on the communicator's side stream; the host polls the completion event (no sleeping
 * driver wait: the GPU is idle until the host returns). comm == NULL or a loopback communicator:
 * the stream drain alone. */
int dtc_barrier(dtc_comm* comm, void* stream);
/* Test communicator (no RCCL): every all-reduce through it -- dtc_comm_allreduce_sum, the Reducer's
 * bucket all-reduces inside dtc_rn18_backward and SyncBN's statistics all-reduces -- multiplies the
 * buffer by `factor` on the stream the collective would run on (the side stream for buckets) and
 * appends (address, count, is_async) to a host log; broadcast is the identity; the communicator
 * reports `world` ranks. With factor == world it is `world` ranks holding identical data. Lets a
 * one-GPU test prove that every gradient bucket is reduced exactly once and only after its producers,
 * and that SyncBN's sums really go through the collective (a one-rank RCCL SUM is the identity and
 * proves neither). fp32 / int64 / fp64 buffers only (int64 x the integer factor). */
int dtc_comm_init_loopback(dtc_comm** out, int device, int world, float factor);
int dtc_comm_log_size(dtc_comm* comm);
int dtc_comm_log_entry(dtc_comm* comm, int idx, uint64_t* addr, uint64_t* count, int* is_async);
int dtc_comm_log_clear(dtc_comm* comm);
/* In-process thread-group communicator (test transport, no RCCL): `world` handles outs[0..world-1] =
 * ranks 0..world-1 on one device, each driven by its own host thread with its own streams and buffers.
 * Collectives are matched by call order (as RCCL's): the calling thread blocks until every rank issued
 * the same collective (kind, count, dtype, root; a mismatch or a 120 s wait is an error for all ranks),
 * then the data really moves between the ranks' buffers on a group stream that waits for every rank's
 * producers -- SUM all-reduce as the rank-ordered fp32/int64/fp64 sum written into every buffer, broadcast as
 * root -> all copies, barrier as a host rendezvous + stream drain -- and each rank's consumer stream
 * (the Reducer's side stream for buckets) waits for the result. Lets one GPU run W ranks with DISTINCT
 * data through the product Reducer, broadcasts and SyncBN (max 8 ranks). Every all-reduce is logged
 * as for the loopback communicator. Destroy each handle with dtc_comm_destroy. */
int dtc_comm_init_thread_group(dtc_comm** outs, int world, int device);
int dtc_comm_rank(const dtc_comm* comm);
int dtc_comm_world(const dtc_comm* comm);

/* ------------------------------------------------------------------ DataParallel group
 * Replaces the per-step traffic of nn.DataParallel (reference src/dp/trainer.py:27):
 * replicate = broadcast of the module's flat buffers from device_ids[0] to every replica (C5),
 * backward = reduce-add of the replicas' flat gradient buffers onto device_ids[0] (C7), input scatter
 * / logits gather as peer copies (C6). One process drives all devices: distinct devices get one RCCL
 * rank each (ncclCommInitAll) and every call is one grouped RCCL collective over all replicas;
 * replicas that all share ONE device (device_ids=[0, 0], the single-GPU test form) run the same
 * calls as on-device copies and a fixed-order HIP reduce-add kernel. bufs[i] / streams[i] belong to
 * replica i (its device), bufs[0] is the root. dtype as for dtc_comm_*. */
typedef struct dtc_dp dtc_dp;
int dtc_dp_create(dtc_dp** out, int n, const int* devices);
int dtc_dp_destroy(dtc_dp* group);
int dtc_dp_is_local(const dtc_dp* group);
int dtc_dp_broadcast(dtc_dp* group, void* const* bufs, size_t count, int dtype, void* const* streams);
int dtc_dp_reduce_add(dtc_dp* group, float* const* bufs, size_t count, void* const* streams);
/* dst (on dst_device) <- src (on src_device), `bytes`, ordered on `stream` (hipMemcpyPeerAsync; a plain
 * device-to-device copy when the devices are equal) */
int dtc_copy_peer(void* dst, int dst_device, const void* src, int src_device, size_t bytes, void* stream);

/* ------------------------------------------------------------------ ResNet-18 executor
 * The whole forward (ResNet.forward, net.py:107-116) and backward of ResNet18() (net.py:119-120)
 * as one call each, for a fixed per-rank batch and input size. Parameters live in ONE flat fp32
 * buffer laid out in reverse registration order (so backward produces gradients in increasing
 * address order and DDP buckets are contiguous); conv weights are stored KRSC and exposed to
 * Python as strided [k][c][r][s] views. dtc_rn18_param_info lists the 62 parameters in
 * registration order (net.py:86-105) with names identical to ResNet18().state_dict() keys. */
typedef struct dtc_net dtc_net;
int dtc_rn18_create(dtc_net** out, int batch, int height, int width, int num_classes, float bucket_cap_mb);
int dtc_rn18_destroy(dtc_net* net);
int dtc_rn18_num_params(const dtc_net* net);
int dtc_rn18_param_info(const dtc_net* net, int idx, const char** name, int64_t* offset, int64_t* numel, int* ndim,
                        int64_t* shape4, int64_t* stride4);
int64_t dtc_rn18_flat_numel(const dtc_net* net);
/* BN buffers: running_mean/running_var in one fp32 flat buffer; num_batches_tracked in an int64 array */
int dtc_rn18_num_bn(const dtc_net* net);
int dtc_rn18_bn_info(const dtc_net* net, int idx, const char** prefix, int* channels, int64_t* mean_offset,
                     int64_t* var_offset);
int64_t dtc_rn18_bufs_numel(const dtc_net* net);
size_t dtc_rn18_workspace_bytes(const dtc_net* net);
int dtc_rn18_num_buckets(const dtc_net* net);
int dtc_rn18_bucket_info(const dtc_net* net, int idx, int64_t* offset, int64_t* numel);
/* Precision of the executor (call before dtc_rn18_bind; re-plans the workspace): 0 = bf16 activations
 * with fp32 accumulation and master weights (the reference under --amp, autocast, trainer.py:152-159),
 * 1 = fp32 throughout (the reference without --amp, ddp/trainer.py:160-165): fp32 activations in the
 * workspace, f32-input MFMA convolutions, BN / pool / Linear on fp32 tensors with the fp32 master
 * weights (no bf16 shadow), no autocast rounding points. */
int dtc_rn18_set_precision(dtc_net* net, int fp32);
int dtc_rn18_precision(const dtc_net* net);
/* Attach caller-owned device memory. Zeroes the workspace statistics areas (enqueued on stream). */
int dtc_rn18_bind(dtc_net* net, void* workspace, float* params, float* grads, uint16_t* params_bf16, float* bufs,
                  int64_t* num_batches_tracked, void* stream);
/* x: NCHW fp32 [batch][3][h][w]; logits fp32 [batch][ncls]. train != 0: batch statistics +
 * running-stat update; train == 0: running statistics (eval mode).
 * Graph mode (option "graphs"): everything after the input im2col is captured once per train flag
 * (on an internal stream) and replayed into `stream`; logits are copied out of the workspace. The
 * backward is captured as segments split at bucket boundaries, with the all-reduces issued eagerly
 * between segment replays; re-captured when grad_scale or the presence of comm changes, and after
 * dtc_rn18_bind. Capture mode (dtc_rn18_enable_capture) runs eagerly. */
int dtc_rn18_forward(dtc_net* net, const float* x, float* logits, int train, void* stream);
/* Gradients of every parameter, scaled by grad_scale (1/world for DDP's mean), written (not
 * accumulated) into the bound flat grad buffer. If comm != NULL each bucket is all-reduced (sum)
 * on the communicator's side stream as soon as backward has produced it; the call returns with
 * `stream` ordered after the last all-reduce. Must follow a training-mode dtc_rn18_forward (one
 * backward per forward: the forward saves the activations and zeroes the BN backward sums). */
int dtc_rn18_backward(dtc_net* net, const float* dlogits, float grad_scale, dtc_comm* comm, void* stream);
/* SyncBatchNorm (replaces nn.SyncBatchNorm.convert_sync_batchnorm(model), torch/nn/modules/
 * batchnorm.py, the conversion README.md:40 recommends; not called by the reference trainers).
 * comm != NULL: every training-mode BN all-reduces its per-channel partial sums (exact int64) over `comm`
 * (forward: sum x, sum x^2; backward: sum dz, sum dz*xhat) on the compute stream and normalises
 * with the global element count (running_var's unbiased factor too); dgamma/dbeta keep this
 * rank's share (x 1/world) so the Reducer's mean matches DDP over SyncBatchNorm. Use a
 * communicator of its own, not the one passed to dtc_rn18_backward. Disables graph replay.
 * comm == NULL: per-rank statistics (the reference's BatchNorm2d). */
int dtc_rn18_set_sync_bn(dtc_net* net, dtc_comm* comm);
/* CrossEntropyLoss backward fused with the network backward (the reference's
 * `scaler.scale(loss).backward()`, ddp/trainer.py:157, when the loss is nn.CrossEntropyLoss of the
 * network's logits, trainer.py:40,155): dlogits = (softmax(logits) - onehot(labels)) * (*gscale) / N
 * written into the executor's own dlogits buffer, then dtc_rn18_backward on it -- one call, so the
 * two launches reach the GPU back to back (this runs right after the per-step barrier, when the GPU
 * queue is empty). logits [batch][num_classes] fp32, labels int64 [batch], lse = the per-row
 * log-sum-exp dtc_xent_fwd wrote, gscale: device fp32 scalar or NULL (1). */
int dtc_rn18_xent_backward(dtc_net* net, const float* logits, const int64_t* labels, const float* lse,
                           const float* gscale, float grad_scale, dtc_comm* comm, void* stream);
/* Byte offset into the workspace of the executor's own fp32 [batch][num_classes] dlogits buffer.
 * A caller that writes the loss gradient there (e.g. the fused cross-entropy backward) and passes
 * that pointer to dtc_rn18_backward saves the graph path's copy-in. */
int dtc_rn18_dlogits_buffer(const dtc_net* net, size_t* ws_offset);

/* Per-layer activations held in the workspace after dtc_rn18_forward (NHWC bf16 except the
 * fp32 "head.feat_f32"): name, byte offset into the workspace, {n, h, w, c}. For parity tests. */
int dtc_rn18_num_activations(const dtc_net* net);
int dtc_rn18_activation_info(const dtc_net* net, int idx, const char** name, size_t* ws_offset, int* shape4);
/* Opt-in (before dtc_rn18_bind): keep copies of the backward's activation gradients per block
 * ("grad.layer2.0.dz", ".dc2", ".ds", ".da1", ".dz1", ".dc1", ".dxs", ".dx", "grad.stem.dz/dc") in
 * extra workspace, for teacher-forced per-layer parity tests. */
int dtc_rn18_enable_capture(dtc_net* net);
int dtc_rn18_num_captures(const dtc_net* net);
int dtc_rn18_capture_info(const dtc_net* net, int idx, const char** name, size_t* ws_offset, int* shape4);
/* Live timing of every convolution call of training steps (forward, dgrad, wgrad incl. split-K
 * reductions) between begin and end. Each call's kernels stamp the first workgroup start and the
 * last workgroup end (s_memrealtime, converted with hipDeviceAttributeWallClockRate) into a device
 * slot; the backward folds the slots into device totals once per step (graph-safe, no host work
 * per call). begin() arms it (first call: allocation + graph re-capture; later calls: totals
 * re-zeroed; `capacity` > 0 is unused), end() synchronizes the device, returns per-pass totals
 * (index 0 = forward, 1 = dgrad, 2 = wgrad: ms, algorithmic FLOPs, calls) and disarms. */
int dtc_rn18_profile_begin(dtc_net* net, int capacity);
int dtc_rn18_profile_end(dtc_net* net, double* ms_by_kind, double* flops_by_kind, int* count_by_kind);
/* The same with nkinds (1..4) entries per array; kind 3 = the BatchNorm family of the mask-bit path
 * (forward finalize+apply, backward reduce, backward finalize+apply), work = algorithmic HBM bytes
 * (every tensor the kernel must touch, read or written once: the in-step BN HBM roofline). */
int dtc_rn18_profile_end_ex(dtc_net* net, int nkinds, double* ms_by_kind, double* work_by_kind, int* count_by_kind);
/* Event timing of the same launcher calls (bench.py's roofline): while profiling is armed and `pairs` > 0,
 * every timed launcher call of an EAGER step whose weight gradients run on the compute stream (options
 * graphs = 0, bwd_streams = 0) is bracketed by two timing events on the compute stream (at most `pairs`
 * calls; `pairs` = 0 switches it off). _result synchronises, sums the elapsed times (ms) and algorithmic
 * work per kind as profile_end_ex does, and resets. */
int dtc_rn18_profile_events(dtc_net* net, int pairs);
int dtc_rn18_profile_events_result(dtc_net* net, int nkinds, double* ms_by_kind, double* work_by_kind,
                                   int* count_by_kind);
/* Timed launcher calls since the last dtc_rn18_profile_events() that were NOT bracketed because the event
 * pool was used up (`pairs` too small for the region): their durations are missing from _result's totals,
 * so a caller reporting a roofline from them must refuse it when this is non-zero. */
int dtc_rn18_profile_events_dropped(dtc_net* net, long long* dropped);
/* Communication timing of the DDP backward (the first multi-GPU run must be diagnosable by
 * itself): the next `steps` backward calls that carry a communicator record timing events -- the backward's
 * start and the Reducer's join on the compute stream, each bucket collective's start / end on the stream it
 * runs on, the compute stream's wait for the weight-gradient stream (collectives of the earlier buckets and
 * the remaining weight gradients) before the stem weight gradient, and the tail from the last backward kernel
 * to the join (the last bucket's collective). steps = 0 disarms. _result synchronises and returns means over
 * the recorded steps: bucket_us[3 * i + 0 / 1 / 2] = start / end offset from the backward's start and the
 * collective's duration for bucket i < max_buckets (issue order); exposed_us[0] = tail (last kernel -> join),
 * [1] = the weight-gradient join wait, [2] = [0] + [1], [3] = the backward's duration, [4] = steps with a
 * join recorded (eager backward); *steps = steps recorded. Then disarms and frees the events. */
int dtc_rn18_comm_timing(dtc_net* net, int steps);
int dtc_rn18_comm_timing_result(dtc_net* net, int max_buckets, double* bucket_us, double* exposed_us, int* steps);

#ifdef __cplusplus
}
#endif
#endif /* DTC_AMD_H */
