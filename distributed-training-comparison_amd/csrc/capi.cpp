// extern "C" entry points of libdtc_amd.so (declared in include/dtc.h) and the thread-local
// error channel. Each wrapper validates arguments, forwards to the C++ launcher and returns
// its status; no exception or exit() crosses this boundary.
#include <cstdarg>
#include <cstdio>
#include <string>
#include "../../include/dtc.h"
#include "comm.h"
#include "kernels.h"

#include <atomic>
#include <cstring>
#include <cstdlib>
#include <dlfcn.h>
#include <fcntl.h>
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace dtc {
static std::atomic<int> g_opts[OPT_COUNT] = {
#define DTC_OPT_DEF(id, name, def) {def},
    DTC_OPTION_LIST(DTC_OPT_DEF)
#undef DTC_OPT_DEF
};
static const char* g_opt_names[OPT_COUNT] = {
#define DTC_OPT_NAME(id, name, def) #name,
    DTC_OPTION_LIST(DTC_OPT_NAME)
#undef DTC_OPT_NAME
};
static std::atomic<int> g_epoch{0};
// DTC_OPTIONS="name=value,name=value" in the environment overrides defaults at library load (A/B and
// bisection runs of whole test suites without code changes)
static int apply_env_options() {
  const char* e = getenv("DTC_OPTIONS");
  if (!e) return 0;
  std::string s(e);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    const std::string kv = s.substr(pos, end - pos);
    const size_t eq = kv.find('=');
    if (eq != std::string::npos) {
      const std::string k = kv.substr(0, eq);
      const int v = atoi(kv.c_str() + eq + 1);
      for (int i = 0; i < OPT_COUNT; ++i)
        if (k == g_opt_names[i]) g_opts[i].store(v);
    }
    pos = end + 1;
  }
  return 1;
}
static const int g_env_applied = apply_env_options();
int option_get(int id) { return g_opts[id].load(std::memory_order_relaxed); }
int option_epoch() { return g_epoch.load(std::memory_order_relaxed); }
int option_set(const char* name, int value) {
  for (int i = 0; i < OPT_COUNT; ++i)
    if (name && strcmp(name, g_opt_names[i]) == 0) {
      g_opts[i].store(value, std::memory_order_relaxed);
      g_epoch.fetch_add(1, std::memory_order_relaxed);
      return 0;
    }
  return set_error(DTC_EINVAL, "unknown option %s", name ? name : "(null)");
}

static thread_local std::string g_err;
int set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
const char* last_error() { return g_err.c_str(); }
}  // namespace dtc

using namespace dtc;

// ------------------------------------------------------------------ native crash report (diagnostics)
// dtc_install_crash_handler(): on SIGSEGV / SIGBUS / SIGFPE / SIGABRT print the faulting THREAD (tid,
// name) and its native frames (library + nearest exported symbol + offset) to stderr, then hand the
// signal to the previous handler (Python's faulthandler prints the Python threads). faulthandler alone
// cannot say in which native thread -- ours or a runtime worker -- a fault happened.
static struct sigaction g_prev_sa[32];
// the report also goes to the file DTC_CRASH_LOG names (opened at install): under pytest's fd capture, fd 2 of a
// test is a temporary file that is lost with the process (r06s: a SIGSEGV left only faulthandler's frames)
static int g_crash_fd = -1;
static void put(const char* s) {
  (void)!write(2, s, strlen(s));
  if (g_crash_fd >= 0) (void)!write(g_crash_fd, s, strlen(s));
}
static void put_hex(uintptr_t v) {
  char b[19] = "0x";
  for (int i = 0; i < 16; ++i) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
  b[18] = 0;
  put(b);
}
static void crash_report(int sig, siginfo_t* si, void* uc) {
  char name[32] = {0};
  (void)pthread_getname_np(pthread_self(), name, sizeof(name));
  put("\n=== dtc crash report: signal ");
  put(sig == SIGSEGV ? "SIGSEGV" : sig == SIGBUS ? "SIGBUS" : sig == SIGFPE ? "SIGFPE" : "SIGABRT");
  put(" addr ");
  put_hex((uintptr_t)(si ? si->si_addr : nullptr));
  put(" tid ");
  put_hex((uintptr_t)syscall(SYS_gettid));
  put(" pid ");
  put_hex((uintptr_t)getpid());
  put(" thread '");
  put(name);
  put("'\n");
  void* fr[48];
  const int nf = backtrace(fr, 48);
  for (int i = 0; i < nf; ++i) {
    Dl_info d;
    put("  #");
    put_hex((uintptr_t)i);
    put(" ");
    if (dladdr(fr[i], &d) && d.dli_fname) {
      put(d.dli_fname);
      put(" +");
      put_hex((uintptr_t)fr[i] - (uintptr_t)d.dli_fbase);
      if (d.dli_sname) {
        put(" ");
        put(d.dli_sname);
        put(" +");
        put_hex((uintptr_t)fr[i] - (uintptr_t)d.dli_saddr);
      }
    } else {
      put_hex((uintptr_t)fr[i]);
    }
    put("\n");
  }
  put("=== end dtc crash report\n");
  // our own disposition goes first (a re-entry ends in the default action, never a loop), and
  // the previous handler is called only when it is not this one -- if Python's faulthandler was enabled
  // again after us, each records the other as "previous" and chaining both ways would recurse
  signal(sig, SIG_DFL);
  const struct sigaction& p = g_prev_sa[sig];
  if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction && p.sa_sigaction != crash_report) {
    p.sa_sigaction(sig, si, uc);
  } else if (!(p.sa_flags & SA_SIGINFO) && p.sa_handler != SIG_IGN && p.sa_handler != SIG_DFL && p.sa_handler) {
    p.sa_handler(sig);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

static inline hipStream_t S(void* s) { return (hipStream_t)s; }
static inline ConvShape shape_of(const dtc_conv_desc* d) {
  return ConvShape{d->n, d->h, d->w, d->c, d->k, d->r, d->s, d->stride, d->pad};
}
// The convolutions the kernels implement: 1x1 / 3x3, stride 1 / 2, pad 0 / 1, C and K multiples of 64,
// a non-empty output. Checked at the boundary, before any planning arithmetic (which divides by C / 64).
static bool desc_ok(const dtc_conv_desc* d) {
  if (!d || d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0 || d->k <= 0) return false;
  if (d->c % 64 != 0 || d->k % 64 != 0 || d->r != d->s || (d->r != 1 && d->r != 3)) return false;
  if ((d->stride != 1 && d->stride != 2) || d->pad < 0 || d->pad > 1) return false;
  const int64_t p = (d->h + 2 * d->pad - d->r) / d->stride + 1, q = (d->w + 2 * d->pad - d->s) / d->stride + 1;
  return p > 0 && q > 0 && (int64_t)d->n * d->h * d->w * std::max(d->c, d->k) < (1ll << 40);
}

#define GUARD(body)                                                          \
  try {                                                                      \
    body                                                                     \
  } catch (...) {                                                            \
    return set_error(DTC_EINVAL, "%s: unexpected C++ exception", __func__); \
  }

extern "C" {

int dtc_abi_version(void) { return DTC_ABI_VERSION; }
int dtc_set_option(const char* name, int value) { return option_set(name, value); }
int dtc_get_option(const char* name) {
  for (int i = 0; i < OPT_COUNT; ++i)
    if (name && strcmp(name, g_opt_names[i]) == 0) return option_get(i);
  return set_error(DTC_EINVAL, "unknown option %s", name ? name : "(null)");
}
const char* dtc_last_error(void) { return last_error(); }

int dtc_install_crash_handler(void) {
  static std::atomic<int> once{0};
  if (once.exchange(1)) return 0;
  void* warm[2];
  (void)backtrace(warm, 2);  // loads the unwinder now, not inside the handler
  if (const char* path = getenv("DTC_CRASH_LOG")) g_crash_fd = open(path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  static char altstack[1 << 16];
  stack_t ss;
  ss.ss_sp = altstack;
  ss.ss_size = sizeof(altstack);
  ss.ss_flags = 0;
  (void)sigaltstack(&ss, nullptr);
  for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGABRT}) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = crash_report;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(sig, &sa, &g_prev_sa[sig]) != 0) return set_error(DTC_EINVAL, "sigaction failed");
  }
  return 0;
}

size_t dtc_conv2d_workspace_size(const dtc_conv_desc* d, int pass) {
  if (!desc_ok(d) || pass < 0 || pass > 2) return 0;
  const size_t slab = plan_conv(shape_of(d), pass).slab_bytes;
  // FWD / DGRAD split-K: + the arrival counters of the in-kernel reduction at the workspace's end (+ room to
  // align them to 256 B, so a workspace of exactly this size always holds both)
  return slab > 0 && pass != 2 ? slab + (size_t)DTC_TICKS * 4 + 256 : slab;
}

// FWD / DGRAD workspace: [split-K slab][DTC_TICKS u32 arrival counters] when it holds both (the counters of
// the in-kernel reduction are zeroed on the call's stream first; the workspace is scratch between calls),
// else the whole of it is slab and a split-K plan reduces in a separate launch. Nothing is carved out (and
// nothing zeroed) when the plan has no slab or the in-kernel reduction is off (option splitk_ink).
static unsigned* ws_ticks(size_t slab, void* ws, size_t& ws_bytes, hipStream_t st) {
  const size_t tb = (size_t)DTC_TICKS * 4;
  if (ws == nullptr || slab == 0 || ws_bytes < slab + tb || option_get(OPT_SPLITK_INK) == 0) return nullptr;
  const uintptr_t end = ((uintptr_t)ws + ws_bytes - tb) & ~(uintptr_t)255;
  if (end < (uintptr_t)ws + slab) return nullptr;
  if (hipMemsetAsync((void*)end, 0, tb, st) != hipSuccess) return nullptr;
  ws_bytes = end - (uintptr_t)ws;
  return (unsigned*)end;
}
static unsigned* op_ticks(const dtc_conv_desc* d, int pass, void* ws, size_t& ws_bytes, hipStream_t st) {
  return ws_ticks(plan_conv(shape_of(d), pass).slab_bytes, ws, ws_bytes, st);
}

int dtc_conv2d_fwd(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t* stats, void* ws,
                   size_t ws_bytes, void* stream) {
  DTC_CHECK_ARG(d && x && w && y, "dtc_conv2d_fwd: null argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_fwd: unsupported convolution descriptor");
  unsigned* tick = op_ticks(d, CONV_FWD, ws, ws_bytes, S(stream));
  GUARD(return conv_fwd(shape_of(d), x, w, y, stats, (float*)ws, ws ? ws_bytes : 0, S(stream), nullptr, tick);)
}

int dtc_conv2d_fwd_sc(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t* stats,
                      const uint16_t* wsc, uint16_t* ysc, int64_t* stats_sc, void* stream) {
  DTC_CHECK_ARG(d && x && w && y && wsc && ysc, "dtc_conv2d_fwd_sc: null argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_fwd_sc: unsupported convolution descriptor");
  const ConvShape s = shape_of(d);
  const ConvShape sc{s.N, s.H, s.W, s.C, s.K, 1, 1, 2, 0};
  DTC_CHECK_ARG(conv_fwd_sc_ok(s, sc), "dtc_conv2d_fwd_sc: no fused plan for this geometry");
  GUARD(return conv_fwd_sc(s, sc, x, w, y, stats, wsc, ysc, stats_sc, S(stream));)
}

int dtc_conv2d_dgrad(const dtc_conv_desc* d, const uint16_t* dy, const uint16_t* w, uint16_t* dx, const uint16_t* res,
                     void* ws, size_t ws_bytes, void* stream) {
  DTC_CHECK_ARG(d && dy && w && dx, "dtc_conv2d_dgrad: null argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_dgrad: unsupported convolution descriptor");
  unsigned* tick = op_ticks(d, CONV_DGRAD, ws, ws_bytes, S(stream));
  GUARD(return conv_dgrad(shape_of(d), dy, w, dx, res, (float*)ws, ws ? ws_bytes : 0, S(stream), nullptr, nullptr, 0,
                          tick);)
}

int dtc_conv2d_dgrad_bn(const dtc_conv_desc* d, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                        const uint16_t* res, const uint16_t* ymask, const uint16_t* x1, const float* mean1,
                        const float* invstd1, int64_t* acc1, const uint16_t* x2, const float* mean2,
                        const float* invstd2, int64_t* acc2, void* ws, size_t ws_bytes, void* stream) {
  DTC_CHECK_ARG(d && dy && w && dx && ymask && x1 && mean1 && invstd1 && acc1, "dtc_conv2d_dgrad_bn: null argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_dgrad_bn: unsupported convolution descriptor");
  DTC_CHECK_ARG(!x2 || (mean2 && invstd2 && acc2), "dtc_conv2d_dgrad_bn: second BN arguments");
  BnbArgs a;
  a.ym = ymask; a.x1 = x1; a.mean1 = mean1; a.invstd1 = invstd1; a.acc1 = acc1;
  a.x2 = x2; a.mean2 = mean2; a.invstd2 = invstd2; a.acc2 = acc2;
  unsigned* tick = op_ticks(d, CONV_DGRAD, ws, ws_bytes, S(stream));
  GUARD(return conv_dgrad(shape_of(d), dy, w, dx, res, (float*)ws, ws ? ws_bytes : 0, S(stream), nullptr, &a, 0,
                          tick);)
}

int dtc_conv2d_dgrad_sc(const dtc_conv_desc* d, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                        const uint16_t* dsc, const uint16_t* wsc, void* stream) {
  DTC_CHECK_ARG(d && dy && w && dx && dsc && wsc, "dtc_conv2d_dgrad_sc: null argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_dgrad_sc: unsupported convolution descriptor");
  DTC_CHECK_ARG(conv_dgrad_sc_ok(shape_of(d)), "dtc_conv2d_dgrad_sc: no fused plan for this geometry");
  GUARD(return conv_dgrad_sc(shape_of(d), dy, w, dx, dsc, wsc, S(stream));)
}

int dtc_conv2d_wgrad(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* dy, float* dw, float scale, void* ws,
                     size_t ws_bytes, void* stream) {
  DTC_CHECK_ARG(d && x && dy && dw && ws, "dtc_conv2d_wgrad: null argument (workspace is required)");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_wgrad: unsupported convolution descriptor");
  GUARD(return conv_wgrad(shape_of(d), x, dy, dw, 0, 0, scale, (float*)ws, ws_bytes, S(stream));)
}

size_t dtc_conv2d_wgrad_sc_workspace_size(const dtc_conv_desc* d) {
  if (!desc_ok(d)) return 0;
  const ConvShape s = shape_of(d);
  return wgrad_s2_splits(s) > 0 ? conv_wgrad_s2_slab_bytes(s) + (size_t)DTC_TICKS * 4 : 0;
}

int dtc_conv2d_wgrad_sc(const dtc_conv_desc* d, const uint16_t* x, const uint16_t* dy, const uint16_t* dsc, float* dw,
                        float* dw_sc, float scale, void* ws, size_t ws_bytes, void* stream) {
  DTC_CHECK_ARG(d && x && dy && dsc && dw && dw_sc, "dtc_conv2d_wgrad_sc: null argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_wgrad_sc: unsupported convolution descriptor");
  GUARD(return conv_wgrad_s2(shape_of(d), x, dy, dsc, dw, dw_sc, scale, (float*)ws, ws ? ws_bytes : 0, S(stream));)
}

size_t dtc_conv2d_wgrad_batch_workspace_size(const dtc_conv_desc* d, int n) {
  if (!desc_ok(d) || n < 1 || n > DTC_WG_BATCH) return 0;
  const ConvShape s = shape_of(d);
  return wgrad_halo_splits(s, n) > 0 ? conv_wgrad_batch_slab_bytes(s, n) : 0;
}

int dtc_conv2d_wgrad_batch(const dtc_conv_desc* d, int n, const uint16_t* const* x, const uint16_t* const* dy,
                           float* const* dw, float scale, void* ws, size_t ws_bytes, void* stream) {
  DTC_CHECK_ARG(d && x && dy && dw && ws && n >= 1 && n <= DTC_WG_BATCH, "dtc_conv2d_wgrad_batch: bad argument");
  DTC_CHECK_ARG(desc_ok(d), "dtc_conv2d_wgrad_batch: unsupported convolution descriptor");
  for (int i = 0; i < n; ++i) DTC_CHECK_ARG(x[i] && dy[i] && dw[i], "dtc_conv2d_wgrad_batch: null problem %d", i);
  GUARD(return conv_wgrad_batch(shape_of(d), n, x, dy, dw, scale, (float*)ws, ws_bytes, S(stream));)
}

size_t dtc_bn_stat_words(int c) { return c > 0 ? DTC_STAT_WORDS(c) : 0; }

int dtc_bn_stat_totals(const int64_t* w, int c, double* totals) {
  DTC_CHECK_ARG(w && totals && c > 0, "dtc_bn_stat_totals: bad args");
  for (int j = 0; j < 2; ++j)
    for (int ch = 0; ch < c; ++ch) {
      int64_t hi = 0, lo = 0;
      for (int k = 0; k < DTC_STAT_SLOTS; ++k) {
        hi += w[stat_word(k, j, 0, c) + ch];
        lo += w[stat_word(k, j, 1, c) + ch];
      }
      totals[(size_t)j * c + ch] = stat_total(hi, lo, w[0]);
    }
  return 0;
}

int dtc_bn_fwd_finalize(int64_t* stats, int c, int64_t count, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, float* mean,
                        float* invstd, float* scale, float* shift, void* stream) {
  return bn_fwd_finalize(stats, c, count, gamma, beta, running_mean, running_var, nbt, momentum, eps, mean, invstd,
                         scale, shift, S(stream));
}
int dtc_bn_apply_relu(const uint16_t* x, const float* scale, const float* shift, uint16_t* y, int64_t m, int c,
                      void* stream) {
  return bn_apply_relu(x, scale, shift, y, m, c, S(stream));
}
int dtc_bn_apply_add_relu(const uint16_t* x, const float* scale, const float* shift, const uint16_t* res, uint16_t* y,
                          int64_t m, int c, void* stream) {
  return bn_apply_add_relu(x, scale, shift, res, y, m, c, S(stream));
}
int dtc_bn_apply_dual_relu(const uint16_t* x, const float* scale, const float* shift, const uint16_t* x2,
                           const float* scale2, const float* shift2, uint16_t* y, int64_t m, int c, void* stream) {
  return bn_apply_dual_relu(x, scale, shift, x2, scale2, shift2, y, m, c, S(stream));
}
int dtc_bn_bwd_reduce(const uint16_t* dy, const uint16_t* ymask, const uint16_t* x1, const float* mean1,
                      const float* invstd1, int64_t* acc1, const uint16_t* x2, const float* mean2, const float* invstd2,
                      int64_t* acc2, uint16_t* dz, int64_t m, int c, void* stream) {
  return bn_bwd_reduce(dy, ymask, x1, mean1, invstd1, acc1, x2, mean2, invstd2, acc2, dz, m, c, S(stream));
}
int dtc_bn_bwd_finalize(int64_t* acc, int c, int64_t count, const float* gamma, const float* mean, const float* invstd,
                        float gscale, float* dgamma, float* dbeta, float* coef, void* stream) {
  return bn_bwd_finalize(acc, c, count, gamma, mean, invstd, gscale, dgamma, dbeta, coef, S(stream));
}
int dtc_bn_bwd_apply(const uint16_t* dz, const uint16_t* x1, const float* coef1, uint16_t* dx1, const uint16_t* x2,
                     const float* coef2, uint16_t* dx2, int64_t m, int c, void* stream) {
  return bn_bwd_apply(dz, x1, coef1, dx1, x2, coef2, dx2, m, c, S(stream));
}

int dtc_stem_im2col(const float* x, uint16_t* cols, int n, int h, int w, void* stream) {
  return stem_im2col(x, cols, n, h, w, S(stream));
}
int dtc_stem_pack_weight(const uint16_t* w27, uint16_t* w64, int k, void* stream) {
  return stem_pack_weight(w27, w64, k, S(stream));
}
int dtc_stem_fwd(const float* x_nchw, const uint16_t* w27, uint16_t* y, int64_t* stats, int n, int h, int w,
                 void* stream) {
  GUARD(return stem_fwd(x_nchw, w27, y, stats, n, h, w, S(stream));)
}
size_t dtc_stem_wgrad_workspace_size(int n, int h, int w) {
  return n > 0 && h > 0 && w > 0 ? stem_wgrad_slab_bytes((int64_t)n * h * w) : 0;
}
int dtc_stem_wgrad(const float* x_nchw, const uint16_t* dy, float* dw27, float scale, int n, int h, int w, void* ws,
                   size_t ws_bytes, void* stream) {
  GUARD(return stem_wgrad(x_nchw, dy, dw27, scale, n, h, w, (float*)ws, ws_bytes, S(stream));)
}
int dtc_head_fwd(const uint16_t* act, int n, int hw, int c, const uint16_t* wfc, const float* bfc, int ncls,
                 float* feat, float* logits, void* stream) {
  return head_fwd(act, n, hw, c, wfc, bfc, ncls, feat, logits, S(stream));
}
size_t dtc_head_bwd_workspace_size(int n, int c, int ncls) { return head_bwd_workspace(n, c, ncls); }
int dtc_head_bwd(const float* dlogits, const float* feat, const uint16_t* wfc, int n, int hw, int c, int ncls,
                 float scale, float* dw, float* db, uint16_t* dact, void* ws, size_t ws_bytes, void* stream) {
  return head_bwd(dlogits, feat, wfc, n, hw, c, ncls, scale, dw, db, dact, (float*)ws, ws_bytes, S(stream));
}
int dtc_xent_fwd(const float* logits, const int64_t* labels, int n, int ncls, float* loss, float* lse, void* stream) {
  return xent_fwd(logits, labels, n, ncls, loss, lse, S(stream));
}
int dtc_xent_fwd_ex(const float* logits, const int64_t* labels, int n, int ncls, float* loss, float* lse,
                    const float* scale, float* scaled, float* host_loss, void* stream) {
  GUARD(return xent_fwd_fused(logits, labels, n, ncls, loss, lse, scale, scaled, host_loss, S(stream));)
}
int dtc_xent_bwd(const float* logits, const int64_t* labels, const float* lse, const float* gscale, int n, int ncls,
                 float* dlogits, void* stream) {
  return xent_bwd(logits, labels, lse, gscale, n, ncls, dlogits, S(stream));
}

int dtc_sgd_nesterov_flat(float* p, const float* g, float* mom, uint16_t* pb, int64_t n, float lr, float wd, float mu,
                          const float* inv_scale, const int* found_inf, void* stream) {
  return sgd_nesterov(p, g, mom, pb, n, lr, wd, mu, inv_scale, found_inf, S(stream));
}
int dtc_cast_f32_bf16(const float* src, uint16_t* dst, int64_t n, void* stream) {
  return cast_f32_bf16(src, dst, n, S(stream));
}
int dtc_amp_scale(const float* x, const float* scale, float* out, int64_t n, void* stream) {
  return amp_scale(x, scale, out, n, S(stream));
}
int dtc_amp_check_finite(const float* g, int64_t n, int* found_inf, void* stream) {
  return amp_check_finite(g, n, found_inf, S(stream));
}
int dtc_amp_update_scale(float* scale, float* inv_scale, int* growth_tracker, int* found_inf, float growth,
                         float backoff, int interval, void* stream) {
  return amp_update_scale(scale, inv_scale, growth_tracker, found_inf, growth, backoff, interval, S(stream));
}

int dtc_cifar_augment(const uint8_t* images, const int64_t* targets, int64_t n_images, const int64_t* index,
                      const uint8_t* crop, const uint8_t* flip, int n, int h, int w, int pad, const float* mean,
                      const float* stdv, float* out, int64_t* labels, int* status, void* stream) {
  return cifar_augment(images, targets, n_images, index, crop, flip, n, h, w, pad, mean, stdv, out, labels, status,
                       S(stream));
}

size_t dtc_comm_unique_id_bytes(void) { return comm_unique_id_bytes(); }
int dtc_comm_get_unique_id(void* out) { GUARD(return comm_get_unique_id(out);) }
int dtc_comm_init(dtc_comm** out, int rank, int world, const void* id, int device) {
  GUARD(return comm_init((Comm**)out, rank, world, id, device);)
}
int dtc_comm_allreduce_sum(dtc_comm* comm, void* buf, size_t count, int dtype, void* stream) {
  return comm_allreduce((Comm*)comm, buf, count, dtype, S(stream));
}
int dtc_comm_broadcast(dtc_comm* comm, void* buf, size_t count, int dtype, int root, void* stream) {
  return comm_broadcast((Comm*)comm, buf, count, dtype, root, S(stream));
}
int dtc_comm_destroy(dtc_comm* comm) { return comm_destroy((Comm*)comm); }
int dtc_barrier(dtc_comm* comm, void* stream) { GUARD(return comm_barrier((Comm*)comm, S(stream));) }
int dtc_comm_init_loopback(dtc_comm** out, int device, int world, float factor) {
  GUARD(return comm_init_loopback((Comm**)out, device, world, factor);)
}
int dtc_comm_init_thread_group(dtc_comm** outs, int world, int device) {
  GUARD(return comm_init_thread_group((Comm**)outs, world, device);)
}
int dtc_comm_rank(const dtc_comm* comm) { return comm_rank((const Comm*)comm); }
int dtc_comm_world(const dtc_comm* comm) { return comm_world((const Comm*)comm); }
int dtc_comm_log_size(dtc_comm* comm) {
  const auto* l = comm_log((Comm*)comm);
  return l ? (int)l->size() : DTC_EINVAL;
}
int dtc_comm_log_entry(dtc_comm* comm, int idx, uint64_t* addr, uint64_t* count, int* is_async) {
  const auto* l = comm_log((Comm*)comm);
  DTC_CHECK_ARG(l && idx >= 0 && idx < (int)l->size(), "dtc_comm_log_entry: bad index");
  if (addr) *addr = (*l)[idx].addr;
  if (count) *count = (*l)[idx].count;
  if (is_async) *is_async = (*l)[idx].async;
  return 0;
}
int dtc_dp_create(dtc_dp** out, int n, const int* devices) { GUARD(return dp_create((DPGroup**)out, n, devices);) }
int dtc_dp_destroy(dtc_dp* g) { return dp_destroy((DPGroup*)g); }
int dtc_dp_is_local(const dtc_dp* g) { return dp_local((const DPGroup*)g); }
int dtc_dp_broadcast(dtc_dp* g, void* const* bufs, size_t count, int dtype, void* const* streams) {
  GUARD(return dp_broadcast((DPGroup*)g, bufs, count, dtype, streams);)
}
int dtc_dp_reduce_add(dtc_dp* g, float* const* bufs, size_t count, void* const* streams) {
  GUARD(return dp_reduce_add((DPGroup*)g, bufs, count, streams);)
}
int dtc_copy_peer(void* dst, int dst_device, const void* src, int src_device, size_t bytes, void* stream) {
  return copy_peer(dst, dst_device, src, src_device, bytes, S(stream));
}
int dtc_comm_log_clear(dtc_comm* comm) {
  DTC_CHECK_ARG(comm != nullptr, "dtc_comm_log_clear: null comm");
  comm_log_clear((Comm*)comm);
  return 0;
}

}  // extern "C"
