// Implicit-GEMM convolution on bf16 MFMA (v_mfma_f32_16x16x32_bf16) for gfx950.
//
// Replaces the cuDNN kernels that `nn.Conv2d` (reference src/*/net.py:18-24, 29-35, 91)
// launches for forward, data-gradient and weight-gradient. One kernel template serves
// all three; only the tile LOADERS differ:
//
//   mode   D (MFMA rows x cols)     A-side operand (rows)           B-side operand (cols)        reduction
//   FWD    y[kout][pixel]           W  (KRSC rows)   row image      im2col(x)        row image   (r,s,c)
//   DGRAD  dx[c][pixel]             W^T (k rows,c)   tr image       im2col^T(dy)     row image   (r,s,k)
//   WGRAD  dW[(r,s,c)][kout]        im2col(x) (m,c)  tr image       dy (m,kout)      tr image    pixels m
//
// LDS images: 128-byte rows (64 bf16). A "row image" holds one GEMM row per LDS row with
// the reduction index contiguous; fragments are read with ds_read_b128. A "tr image"
// holds the REDUCTION index as the LDS row (64 rows x 64 columns per 8 KiB image);
// fragments are read with ds_read_b64_tr_b16 (gfx950 transposing LDS read), so NHWC
// tensors are staged exactly as they lie in HBM and never transposed in memory.
// Tiles are filled by global_load_lds (LDS-DMA, 16 B per lane, lane-linear destination);
// bank-conflict swizzles are applied on the per-lane SOURCE address and the matching
// XOR on the read (guide §5.4 rule 21). Padding rows read a 1 KiB zero page.
#include "common.h"
#include "kernels.h"
#include "tile_common.h"

static __device__ __attribute__((aligned(1024))) uint4 g_zero_page[64];

namespace dtc {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct IGemmParams {
  const u16* src0;  // FWD: x (NHWC)   DGRAD: dy (NPQK)   WGRAD: x (NHWC)
  const u16* src1;  // FWD: W (KRSC)   DGRAD: W (KRSC)    WGRAD: dy (NPQK)
  u16* out;         // bf16 output (non-slab epilogue): FWD y (NPQK), DGRAD dx (NHWC)
  float* slab;      // fp32 split-K partials
  const u16* res;   // DGRAD: optional residual added in the epilogue
  int64_t* stats;    // FWD: optional per-channel (sum, sumsq) accumulators [SLOTS][2][K]
  int N, H, W, C, K, R, S, P, Q, stride, pad;
  int M;            // GEMM pixel extent: FWD/WGRAD N*P*Q, DGRAD N*H*W
  int RSC;
  FastDiv fd_q, fd_pq;  // FWD/WGRAD: Q, P*Q ; DGRAD: W, H*W
  FastDiv fd_cc;        // reduction chunks per tap: FWD C/64, DGRAD K/64
  int num_kt, kt_per_split, tiles_a;
  int xcd_remap;
  int cls;  // DGRAD, stride 2: blockIdx.z = output parity class (h%2, w%2); M counts class pixels
  int cls_order;  // 1: blockIdx.z runs the classes heaviest first (option dgrad_class_order)
  int res_compact;  // DGRAD classes: res is [N][H/2][W/2][C], added to class (0, 0) only (a 1x1 stride-2
                    // shortcut's dx, which is zero at the other three parities)
  // WGRAD fast path: each 64-pixel reduction step covers whole rows of one image (PQ % 64 == 0,
  // 64 % Q == 0) or whole images (64 % PQ == 0); tensors < 4 GiB so 32-bit buffer offsets work.
  int wg_fast;
  uint32_t src0_bytes, src1_bytes;
  u64* ts;  // optional call timing slot: atomicMin(start), atomicMax(end), s_memrealtime ticks
  // FWD, SC kernels: the projection shortcut (1x1, stride 2, pad 0) of the same input in the same
  // launch. Its reduction is exactly the 3x3 conv's centre tap: reduction steps [kt_c0, kt_c1) stage
  // W_sc's chunk beside W's and run a second set of MFMAs on the same im2col fragments.
  const u16* src1b;  // W_sc [K][C]
  u16* out2;         // shortcut output (NPQK)
  int64_t* stats2;    // its BN statistic slots
  int kt_c0, kt_c1;
  // DGRAD classes, shortcut fused (sc_kt > 0): the 1x1 stride-2 shortcut's input gradient is nonzero only
  // at the (even, even) pixels, where it is dsc[u][v] . W_sc -- a 1x1 GEMM on the class-(0, 0) grid with
  // the same reduction length as that class's single tap. Class (0, 0) runs sc_kt extra reduction steps
  // reading dsc (src0b) and W_sc^T (src1b), so dx there is one sum over [dc1 | dsc] x [W(1,1) ; W_sc].
  const u16* src0b;  // dsc (NPQK)
  int sc_kt;
};

template <int MODE, int BM, int BN, int WR, int WC, bool SLAB, int NSTAGE, bool SC = false>
__global__ void __launch_bounds__(256, 2) igemm_kernel(const IGemmParams p) {
  constexpr int FM = BM / (WR * 16);
  constexpr int FN = BN / (WC * 16);
  constexpr int A_BYTES = BM * 128;
  constexpr int SC_OFF = (BM + BN) * 128;             // SC: W_sc chunk after the A and B images
  constexpr int STAGE = SC_OFF + (SC ? BM * 128 : 0);
  constexpr int NIA = BM / 32;  // glds instructions per wave per stage, A side
  constexpr int NIB = BN / 32;  // B side
  constexpr bool A_TR = (MODE != MODE_FWD);
  constexpr bool B_TR = (MODE == MODE_WGRAD);
  static_assert(WR * WC == 4, "4 waves");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tile");
  static_assert(!SC || (MODE == MODE_FWD && !SLAB), "shortcut fusion: forward, no split-K");

  static_assert(NSTAGE == 2 || NSTAGE == 3, "stages");
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE];

  stamp_start(p.ts);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // XCD-aware remap (guide T1): blocks b and b+8 share an XCD's L2; give each XCD a contiguous
  // run of tile ids so the tiles that share a pixel tile (consecutive ids) share an L2.
  int bid = blockIdx.x;
  if (p.xcd_remap && gridDim.x >= 16) {
    const int nwg = gridDim.x, x8 = bid & 7, q = nwg >> 3, rr = nwg & 7;
    bid = (x8 < rr ? x8 * (q + 1) : rr * (q + 1) + (x8 - rr) * q) + (bid >> 3);
  }
  const int ta = bid % p.tiles_a;
  const int tb = bid / p.tiles_a;
  const int a0 = ta * BM, b0 = tb * BN;
  // DGRAD stride-2 parity class: only taps r = r0 + 2i (s = s0 + 2j) reach pixels with
  // h % 2 == ph, and they read dy row p = hh + dr - i for h = 2*hh + ph (a dense stride-1 GEMM)
  int cls_ph = 0, cls_pw = 0, r0 = 0, s0 = 0, tstep = 1, dr = 0, dsh = 0, Sdim = p.S;
  int num_kt = p.num_kt;
  if constexpr (MODE == MODE_DGRAD) {
    if (p.cls) {
      // heaviest class first: classes differ in tap count (pad 1: (0,0) 1 tap, (0,1)/(1,0) 2, (1,1) 4),
      // and the dispatcher starts workgroups in z order -- the 4-tap class launched last set the tail
      const int zc = (p.cls_order && (p.pad & 1)) ? 3 - (int)blockIdx.z : (int)blockIdx.z;
      cls_ph = zc >> 1;
      cls_pw = zc & 1;
      r0 = (cls_ph + p.pad) & 1;
      s0 = (cls_pw + p.pad) & 1;
      const int Rdim = (p.R - r0 + 1) >> 1;
      Sdim = (p.S - s0 + 1) >> 1;
      tstep = 2;
      dr = (cls_ph + p.pad - r0) >> 1;
      dsh = (cls_pw + p.pad - s0) >> 1;
      num_kt = Rdim * Sdim * (int)p.fd_cc.d;
      if (cls_ph == 0 && cls_pw == 0) num_kt += p.sc_kt;  // + the fused shortcut's steps (kt >= kt_sc0)
    }
  }
  const int kt_sc0 = num_kt - ((MODE == MODE_DGRAD && cls_ph == 0 && cls_pw == 0) ? p.sc_kt : 0);
  const int kt_begin = blockIdx.y * p.kt_per_split;
  const int kt_end = min(num_kt, kt_begin + p.kt_per_split);
  const int lrow = lane >> 3, pc = lane & 7;
  const u16* zp = (const u16*)g_zero_page + pc * 8;

  // ------------------------------------------------------------ loader state
  // A side
  int offA[NIA];
  // B side (FWD: pixel of y; DGRAD: pixel of dx)
  int64_t baseB[NIB];
  int hB[NIB], wB[NIB];
  // WGRAD: block-uniform tap, per-lane columns
  int colA[NIA], colB[NIB];
  int tap_r = 0, tap_s = 0;
  uint32_t wl_x[2] = {0, 0};
  int wl_ih[2] = {0, 0}, wl_row[2] = {0, 0};
  bool wl_iwok[2] = {false, false};

  int offAs[MODE == MODE_DGRAD ? NIA : 1];  // DGRAD: the W_sc^T tr image (row stride C)
  if constexpr (MODE == MODE_FWD) {
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
      const int row = (wave + 4 * j) * 8 + lrow;
      const int lc = pc ^ rowswz(row);
      offA[j] = (a0 + row) * p.RSC + lc * 8;
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
      const int row = (wave + 4 * j) * 8 + lrow;
      const int lc = pc ^ rowswz(row);
      const int pix = b0 + row;
      int ih0 = -(1 << 20), iw0 = -(1 << 20);
      int64_t base = 0;
      if (pix < p.M) {
        const int n = (int)fdiv((uint32_t)pix, p.fd_pq);
        const int rem = pix - n * p.P * p.Q;
        const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
        const int qq = rem - pp * p.Q;
        ih0 = pp * p.stride - p.pad;
        iw0 = qq * p.stride - p.pad;
        base = (((int64_t)n * p.H + ih0) * p.W + iw0) * p.C + lc * 8;
      }
      baseB[j] = base; hB[j] = ih0; wB[j] = iw0;
    }
  } else if constexpr (MODE == MODE_DGRAD) {
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
      const int ia = wave + 4 * j;
      const int img = ia >> 3, rowin = (ia & 7) * 8 + lrow;
      const int lc = pc ^ trswz(rowin);
      offA[j] = rowin * p.RSC + a0 + img * 64 + lc * 8;
      offAs[j] = rowin * p.C + a0 + img * 64 + lc * 8;
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
      const int row = (wave + 4 * j) * 8 + lrow;
      const int lc = pc ^ rowswz(row);
      const int pix = b0 + row;
      int h = -(1 << 20), w = -(1 << 20), nP = 0;
      if (pix < p.M) {  // (h, w) of dx, or (hh, ww) of the parity-class grid
        const int n = (int)fdiv((uint32_t)pix, p.fd_pq);
        const int rem = pix - n * (int)p.fd_pq.d;
        h = (int)fdiv((uint32_t)rem, p.fd_q);
        w = rem - h * (int)p.fd_q.d;
        nP = n * p.P;
      }
      baseB[j] = nP;
      colB[j] = lc * 8;
      hB[j] = h; wB[j] = w;
    }
  } else {  // WGRAD
    const int rs = a0 / p.C;
    const int c0 = a0 - rs * p.C;
    tap_r = rs / p.S;
    tap_s = rs - tap_r * p.S;
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
      const int ia = wave + 4 * j;
      const int img = ia >> 3, rowin = (ia & 7) * 8 + lrow;
      colA[j] = c0 + img * 64 + ((pc ^ trswz(rowin)) * 8);
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
      const int ib = wave + 4 * j;
      const int img = ib >> 3, rowin = (ib & 7) * 8 + lrow;
      colB[j] = b0 + img * 64 + ((pc ^ trswz(rowin)) * 8);
    }
    if (p.wg_fast) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // this lane's two pixel rows within a 64-pixel step
        const int rowin = (wave + 4 * h) * 8 + lrow;
        const int dn = (int)fdiv((uint32_t)rowin, p.fd_pq);
        const int rem = rowin - dn * (int)p.fd_pq.d;
        const int dp = (int)fdiv((uint32_t)rem, p.fd_q);
        const int dq = rem - dp * p.Q;
        const int iw = dq * p.stride - p.pad + tap_s;
        wl_iwok[h] = (unsigned)iw < (unsigned)p.W;
        wl_ih[h] = dp * p.stride - p.pad + tap_r;
        wl_x[h] = (uint32_t)((((dn * p.H + wl_ih[h]) * p.W) + iw) * p.C * 2);
        wl_row[h] = rowin;
      }
    }
  }

  // reduction-step decomposition (FWD/DGRAD): kt -> (r, s, chunk); kept incrementally
  int st_r = 0, st_s = 0, st_c = 0;
  const int nchunk = (int)p.fd_cc.d;
  if constexpr (MODE != MODE_WGRAD) {
    const int rs = (int)fdiv((uint32_t)kt_begin, p.fd_cc);
    st_c = kt_begin - rs * nchunk;
    st_r = rs / Sdim;
    st_s = rs - st_r * Sdim;
  }

  auto stage = [&](char* sb, int kt, int r, int s, int cc) {
    if constexpr (MODE == MODE_FWD) {
      const int wadd = (r * p.S + s) * p.C + cc * 64;
#pragma unroll
      for (int j = 0; j < NIA; ++j)
        glds16(p.src1 + offA[j] + wadd, sb + (wave + 4 * j) * 1024);
      if constexpr (SC) {
        if (kt >= p.kt_c0 && kt < p.kt_c1) {  // centre tap: W_sc rows a0.., chunk cc (same swizzle)
#pragma unroll
          for (int j = 0; j < NIA; ++j) {
            const int row = (wave + 4 * j) * 8 + lrow;
            glds16(p.src1b + (a0 + row) * p.C + (pc ^ rowswz(row)) * 8 + cc * 64, sb + SC_OFF + (wave + 4 * j) * 1024);
          }
        }
      }
      const int64_t xadd = ((int64_t)r * p.W + s) * p.C + cc * 64;
#pragma unroll
      for (int j = 0; j < NIB; ++j) {
        const int ih = hB[j] + r, iw = wB[j] + s;
        const bool ok = ((unsigned)ih < (unsigned)p.H) && ((unsigned)iw < (unsigned)p.W);
        const u16* src = ok ? (p.src0 + baseB[j] + xadd) : zp;
        glds16(src, sb + A_BYTES + (wave + 4 * j) * 1024);
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      if (kt >= kt_sc0) {  // fused shortcut step (class (0, 0)): W_sc^T chunk x dsc at the class pixel
        const int cs = kt - kt_sc0;
#pragma unroll
        for (int j = 0; j < NIA; ++j)
          glds16(p.src1b + offAs[j] + (int64_t)cs * 64 * p.C, sb + (wave + 4 * j) * 1024);
#pragma unroll
        for (int j = 0; j < NIB; ++j) {
          const bool ok = ((unsigned)hB[j] < (unsigned)p.P) && ((unsigned)wB[j] < (unsigned)p.Q);
          const u16* src = ok ? (p.src0b + ((baseB[j] + hB[j]) * p.Q + wB[j]) * p.K + cs * 64 + colB[j]) : zp;
          glds16(src, sb + A_BYTES + (wave + 4 * j) * 1024);
        }
        return;
      }
      const int wr_ = r0 + tstep * r, ws_ = s0 + tstep * s;  // filter tap
      const int64_t wadd = (int64_t)cc * 64 * p.RSC + (wr_ * p.S + ws_) * p.C;
#pragma unroll
      for (int j = 0; j < NIA; ++j)
        glds16(p.src1 + offA[j] + wadd, sb + (wave + 4 * j) * 1024);
#pragma unroll
      for (int j = 0; j < NIB; ++j) {
        int ph, pw;
        bool ok;
        if (p.cls) {
          ph = hB[j] + dr - r;
          pw = wB[j] + dsh - s;
          ok = true;
        } else {
          ph = hB[j] + p.pad - r;
          pw = wB[j] + p.pad - s;
          ok = (ph >= 0) && (pw >= 0);
          if (p.stride == 2) {
            ok = ok && !(ph & 1) && !(pw & 1);
            ph >>= 1; pw >>= 1;
          }
        }
        ok = ok && ((unsigned)ph < (unsigned)p.P) && ((unsigned)pw < (unsigned)p.Q);
        const u16* src = ok ? (p.src0 + ((baseB[j] + ph) * p.Q + pw) * p.K + cc * 64 + colB[j]) : zp;
        glds16(src, sb + A_BYTES + (wave + 4 * j) * 1024);
      }
    } else if (p.wg_fast) {  // WGRAD, 32-bit buffer offsets; out-of-range offsets zero-fill LDS
      const int m0 = kt * 64;
      const int n0 = (int)fdiv((uint32_t)m0, p.fd_pq);
      const int p0 = (int)fdiv((uint32_t)(m0 - n0 * (int)p.fd_pq.d), p.fd_q);
      const uint32_t ubase = (uint32_t)((n0 * p.H + p0 * p.stride) * p.W * p.C * 2);
      uint32_t xoff[2], doff[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pix = m0 + wl_row[h];
        const bool okd = pix < p.M;
        const int ih = p0 * p.stride + wl_ih[h];
        const bool okx = okd && wl_iwok[h] && ((unsigned)ih < (unsigned)p.H);
        xoff[h] = okx ? ubase + wl_x[h] : 0x80000000u;
        doff[h] = okd ? (uint32_t)pix * (uint32_t)(p.K * 2) : 0x80000000u;
      }
#pragma unroll
      for (int j = 0; j < NIA; ++j)
        buf_lds16(p.src0, p.src0_bytes, sb + (wave + 4 * j) * 1024, xoff[j & 1] + colA[j] * 2);
#pragma unroll
      for (int j = 0; j < NIB; ++j)
        buf_lds16(p.src1, p.src1_bytes, sb + A_BYTES + (wave + 4 * j) * 1024, doff[j & 1] + colB[j] * 2);
    } else {  // WGRAD generic: pixels kt*64 .. kt*64+63
      const int m0 = kt * 64;
      int64_t xo[2];
      int64_t dyo[2];
      bool okx[2], okd[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pix = m0 + (wave + 4 * h) * 8 + lrow;
        okd[h] = pix < p.M;
        dyo[h] = (int64_t)pix * p.K;
        const int n = (int)fdiv((uint32_t)pix, p.fd_pq);
        const int rem = pix - n * p.P * p.Q;
        const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
        const int qq = rem - pp * p.Q;
        const int ih = pp * p.stride - p.pad + tap_r;
        const int iw = qq * p.stride - p.pad + tap_s;
        okx[h] = okd[h] && ((unsigned)ih < (unsigned)p.H) && ((unsigned)iw < (unsigned)p.W);
        xo[h] = (((int64_t)n * p.H + ih) * p.W + iw) * p.C;
      }
#pragma unroll
      for (int j = 0; j < NIA; ++j) {
        const int h = j & 1;
        const u16* src = okx[h] ? (p.src0 + xo[h] + colA[j]) : zp;
        glds16(src, sb + (wave + 4 * j) * 1024);
      }
#pragma unroll
      for (int j = 0; j < NIB; ++j) {
        const int h = j & 1;
        const u16* src = okd[h] ? (p.src1 + dyo[h] + colB[j]) : zp;
        glds16(src, sb + A_BYTES + (wave + 4 * j) * 1024);
      }
    }
  };

  f32x4 acc[FM][FN];
  f32x4 acc2[SC ? FM : 1][SC ? FN : 1];  // SC: the shortcut's tile
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (SC) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int wr = wave / WC, wc = wave % WC;
  const int arow0 = wr * (BM / WR), bcol0 = wc * (BN / WC);

  auto advance = [&](int& r, int& s, int& cc) {
    if (++cc == nchunk) {
      cc = 0;
      if (++s == Sdim) { s = 0; ++r; }
    }
  };

  auto compute = [&](const char* cur, bool centre) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (A_TR) af[i] = frag_tr(cur, arow0 + i * 16, ks, lane);
        else af[i] = frag_row(cur, arow0 + i * 16, ks, lane);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (B_TR) bfr[j] = frag_tr(cur + A_BYTES, bcol0 + j * 16, ks, lane);
        else bfr[j] = frag_row(cur + A_BYTES, bcol0 + j * 16, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if constexpr (SC) {
        if (centre) {  // block-uniform
#pragma unroll
          for (int i = 0; i < FM; ++i) af[i] = frag_row(cur + SC_OFF, arow0 + i * 16, ks, lane);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc2[i][j], 0, 0, 0);
        }
      }
    }
  };

  // K loop over an NSTAGE-deep LDS ring filled by LDS-DMA. Iteration `it`: wait (counted
  // vmcnt: each wave issues NIA+NIB DMAs per stage) until stage `it` has landed for this wave,
  // barrier (then every wave's DMAs for `it` have landed and every wave finished reading the
  // buffer of stage it-1), refill that buffer with stage it+NSTAGE-1, compute stage `it`.
  // A raw s_barrier is used: __syncthreads() would also drain vmcnt to 0 (guide §5).
  if (kt_begin < kt_end) {
    const int nk = kt_end - kt_begin;
    int r = st_r, s = st_s, cc = st_c;
#pragma unroll
    for (int i = 0; i < NSTAGE - 1; ++i) {
      if (i < nk) {
        stage(smem + i * STAGE, kt_begin + i, r, s, cc);
        if constexpr (MODE != MODE_WGRAD) advance(r, s, cc);
      }
    }
    int cur = 0;
    for (int it = 0; it < nk; ++it) {
      if constexpr (NSTAGE == 3) {
        if (it + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIA + NIB) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int nxt = it + NSTAGE - 1;
      if (nxt < nk) {
        int slot = cur + NSTAGE - 1;
        if (slot >= NSTAGE) slot -= NSTAGE;
        stage(smem + slot * STAGE, kt_begin + nxt, r, s, cc);
        if constexpr (MODE != MODE_WGRAD) advance(r, s, cc);
      }
      compute(smem + cur * STAGE, SC && kt_begin + it >= p.kt_c0 && kt_begin + it < p.kt_c1);
      cur = (cur + 1 == NSTAGE) ? 0 : cur + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // all LDS reads done before the epilogue reuses smem
    asm volatile("" ::: "memory");
  }

  // ------------------------------------------------------------ epilogue
  // D[row][col]: row = A-side index (4 consecutive per lane), col = B-side index.
  const int rq = (lane >> 4) * 4;
  const int cl = lane & 15;
  if constexpr (MODE == MODE_WGRAD) {
    // slab[split][kout][rsc]
    float* slab = p.slab + (size_t)blockIdx.y * p.K * p.RSC;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rsc = a0 + arow0 + i * 16 + rq;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int kout = b0 + bcol0 + j * 16 + cl;
        *(f32x4*)(slab + (size_t)kout * p.RSC + rsc) = acc[i][j];
      }
    }
  } else if constexpr (SLAB) {
    const int ncols = (MODE == MODE_FWD) ? p.K : p.C;
    float* slab = p.slab + (size_t)blockIdx.y * p.M * ncols;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ch = a0 + arow0 + i * 16 + rq;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int pix = b0 + bcol0 + j * 16 + cl;
        if (pix < p.M) *(f32x4*)(slab + (size_t)pix * ncols + ch) = acc[i][j];
      }
    }
  } else if constexpr (MODE == MODE_FWD) {
    float* red = (float*)smem;  // [WC][BM][2]
    auto epi = [&](const f32x4 (&A)[FM][FN], u16* out, int64_t* stats) {
    const bool want_stats = (stats != nullptr);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int chl = arow0 + i * 16 + rq;
      const int ch = a0 + chl;
      float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int pix = b0 + bcol0 + j * 16 + cl;
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[t] = round_bf(A[i][j][t]);
          s4[t] += v[t];
          q4[t] += v[t] * v[t];
        }
        if (pix < p.M) {
          uint2 w;
          w.x = pack_bf2(v[0], v[1]);
          w.y = pack_bf2(v[2], v[3]);
          *(uint2*)(out + (size_t)pix * p.K + ch) = w;
        }
      }
      if (want_stats) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            s4[t] += __shfl_xor(s4[t], o, 64);
            q4[t] += __shfl_xor(q4[t], o, 64);
          }
        }
        if (cl == 0) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            red[(wc * BM + chl + t) * 2 + 0] = s4[t];
            red[(wc * BM + chl + t) * 2 + 1] = q4[t];
          }
        }
      }
    }
    if (want_stats) {
      __syncthreads();
      if ((int)threadIdx.x < BM) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WC; ++w) {
          s += red[(w * BM + threadIdx.x) * 2 + 0];
          q += red[(w * BM + threadIdx.x) * 2 + 1];
        }
        stat_add(stats, p.K, a0 + threadIdx.x, s, q);
      }
    }
    };
    epi(acc, p.out, p.stats);
    if constexpr (SC) {
      __syncthreads();  // the stats scratch is reused
      epi(acc2, p.out2, p.stats2);
    }
  } else {  // DGRAD bf16 (+ residual)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int pix = b0 + bcol0 + j * 16 + cl;
      size_t orow = (size_t)pix;
      if (p.cls && pix < p.M) {  // class pixel -> dx pixel (2*hh + ph, 2*ww + pw)
        const int n = (int)fdiv((uint32_t)pix, p.fd_pq);
        const int rem = pix - n * (int)p.fd_pq.d;
        const int hh = (int)fdiv((uint32_t)rem, p.fd_q);
        const int ww = rem - hh * (int)p.fd_q.d;
        orow = ((size_t)n * p.H + 2 * hh + cls_ph) * p.W + 2 * ww + cls_pw;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ch = a0 + arow0 + i * 16 + rq;
        if (pix < p.M) {
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          const size_t o = orow * p.C + ch;
          if (p.res && (!p.res_compact || (cls_ph == 0 && cls_pw == 0))) {
            const uint2 rr = *(const uint2*)(p.res + (p.res_compact ? (size_t)pix * p.C + ch : o));
            v[0] += bf_lo(rr.x); v[1] += bf_hi(rr.x); v[2] += bf_lo(rr.y); v[3] += bf_hi(rr.y);
          }
          uint2 w;
          w.x = pack_bf2(v[0], v[1]);
          w.y = pack_bf2(v[2], v[3]);
          *(uint2*)(p.out + o) = w;
        }
      }
    }
  }
  stamp_end(p.ts);
}

// ---------------------------------------------------------------- split-K reduction (FWD / DGRAD)
// out[m][n] = bf16( sum_s slab[s][m][n] (+ res[m][n]) ); optional per-channel stats of the
// bf16-rounded output (same semantics as the non-split epilogue).
// out may alias res: each element is read and then written by the same thread.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, int splits,
                                                            int M, int Nc, u16* out, const u16* res,
                                                            int64_t* __restrict__ stats, int rows_per_block,
                                                            u64* ts) {
  __shared__ float red[256 * 16];
  const int tpr = Nc >> 3;           // threads per row (8 channels each)
  const int rpp = 256 / tpr;         // rows per pass
  const int t = threadIdx.x;
  const int g = t % tpr, rr = t / tpr;
  const int m_begin = blockIdx.x * rows_per_block;
  const int m_end = min(M, m_begin + rows_per_block);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const size_t plane = (size_t)M * Nc;
  // one row's result: + residual (loaded earlier), then the statistics and the store
  auto finish = [&](float (&v)[8], size_t o, const uint4& rw) {
    if (res) {
      float rv[8];
      unpack8(rw, rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += rv[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = round_bf(v[k]);
      s[k] += v[k];
      q[k] += v[k] * v[k];
    }
    *(uint4*)(out + o) = pack8(v);
  };
  if (rr < rpp) {
    // four rows per round: their residuals and every split's partials are loaded before the first add (each
    // dependent global access costs ~1 us; one row at a time left these launches latency bound); per row the
    // same additions in the same order as one row at a time (splits in order, then the residual)
    constexpr int RU = 4;
    int m = m_begin + rr;
    for (; m + (RU - 1) * rpp < m_end; m += RU * rpp) {
      size_t o[RU];
      float v[RU][8];
      uint4 rw[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        o[u] = (size_t)(m + u * rpp) * Nc + g * 8;
        rw[u] = res ? *(const uint4*)(res + o[u]) : uint4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 8; ++k) v[u][k] = 0.f;
      }
#pragma unroll 2
      for (int sp = 0; sp < splits; ++sp) {
        f32x4 a[RU], b[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          a[u] = *(const f32x4*)(slab + sp * plane + o[u]);
          b[u] = *(const f32x4*)(slab + sp * plane + o[u] + 4);
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          v[u][0] += a[u][0]; v[u][1] += a[u][1]; v[u][2] += a[u][2]; v[u][3] += a[u][3];
          v[u][4] += b[u][0]; v[u][5] += b[u][1]; v[u][6] += b[u][2]; v[u][7] += b[u][3];
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) finish(v[u], o[u], rw[u]);
    }
    for (; m < m_end; m += rpp) {
      const size_t o = (size_t)m * Nc + g * 8;
      const uint4 rw = res ? *(const uint4*)(res + o) : uint4{0u, 0u, 0u, 0u};
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int sp = 0; sp < splits; ++sp) {
        const f32x4 a = *(const f32x4*)(slab + sp * plane + o);
        const f32x4 b = *(const f32x4*)(slab + sp * plane + o + 4);
        v[0] += a[0]; v[1] += a[1]; v[2] += a[2]; v[3] += a[3];
        v[4] += b[0]; v[5] += b[1]; v[6] += b[2]; v[7] += b[3];
      }
      finish(v, o, rw);
    }
  }
  if (stats) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[t * 16 + k] = s[k];
      red[t * 16 + 8 + k] = q[k];
    }
    __syncthreads();
    for (int c = t; c < Nc; c += 256) {
      const int gg = c >> 3, k = c & 7;
      float a = 0.f, b = 0.f;
      for (int r2 = 0; r2 < rpp; ++r2) {
        a += red[(r2 * tpr + gg) * 16 + k];
        b += red[(r2 * tpr + gg) * 16 + 8 + k];
      }
      stat_add(stats, Nc, c, a, b);
    }
  }
  stamp_end(ts);
}

// ---------------------------------------------------------------- wgrad split reduction
// grad[k][c] (row stride ld_out, first ncols columns) = scale * sum_s slab[s][k][c] (row stride ld_in).
// A workgroup owns 256/SG output float4s; SG lanes per output stride over the splits (independent
// loads in flight), then combine through LDS in a fixed order (deterministic).
struct WgOuts {
  float* dw[DTC_WG_BATCH];
  int ld[DTC_WG_BATCH];  // > 0: this problem's own row length (its slab plane is K x ld, its output dense K x ld)
};
template <int SG>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int K,
                                                           int ld_in, int ncols, int ld_out, float scale,
                                                           const WgOuts outs, size_t prob_stride, u64* ts) {
  // batched launches: blockIdx.y = problem (its own slab region and output)
  slab += blockIdx.y * prob_stride;
  float* __restrict__ grad = outs.dw[blockIdx.y];
  if (outs.ld[blockIdx.y] > 0) ncols = ld_out = ld_in = outs.ld[blockIdx.y];
  constexpr int OPB = 256 / SG;  // outputs (float4) per block
  __shared__ f32x4 red[256];
  const size_t plane = (size_t)K * ld_in;
  const int t = threadIdx.x;
  const int o = t / SG, sg = t % SG;
  const size_t v = (size_t)blockIdx.x * OPB + o;  // float4 index over [K][ld_in]
  const size_t nv = plane >> 2;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (v < nv) {
#pragma unroll 4
    for (int sp = sg; sp < splits; sp += SG) a += *(const f32x4*)(slab + sp * plane + v * 4);
  }
  red[t] = a;
  __syncthreads();
  if (sg == 0 && v < nv) {
#pragma unroll
    for (int k = 1; k < SG; ++k) a += red[t + k];
    a *= scale;
    if (ncols == ld_in && ld_out == ld_in) {
      *(f32x4*)(grad + v * 4) = a;
    } else {
      const size_t e = v * 4;
      const int k = (int)(e / ld_in), c = (int)(e % ld_in);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c + j < ncols) grad[(size_t)k * ld_out + c + j] = a[j];
    }
  }
  stamp_end(ts);
}

// per-call timing slots -> running totals (one launch per training step when profiling):
// slot i: start = min over its start cells, end = max over its end cells; if stamped,
// acc[i] += (end - start, 1). Cells reset to (~0, 0).
__global__ void prof_accumulate_kernel(u64* ts, int n, u64* acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u64* slot = ts + (size_t)i * DTC_PROF_SLOT_U64;
  u64 a = ~0ull, b = 0;
  for (int l = 0; l < DTC_PROF_LINES; ++l) {
    a = min(a, slot[l * DTC_PROF_LINE]);
    b = max(b, slot[(DTC_PROF_LINES + l) * DTC_PROF_LINE]);
    slot[l * DTC_PROF_LINE] = ~0ull;
    slot[(DTC_PROF_LINES + l) * DTC_PROF_LINE] = 0;
  }
  if (a != ~0ull && b > a) {
    acc[2 * i] += b - a;
    acc[2 * i + 1] += 1;
  }
}

// ---------------------------------------------------------------- host launchers
static int fill_common(IGemmParams& p, const ConvShape& s) {
  p.N = s.N; p.H = s.H; p.W = s.W; p.C = s.C; p.K = s.K; p.R = s.R; p.S = s.S;
  p.stride = s.stride; p.pad = s.pad;
  p.P = (s.H + 2 * s.pad - s.R) / s.stride + 1;
  p.Q = (s.W + 2 * s.pad - s.S) / s.stride + 1;
  p.RSC = s.R * s.S * s.C;
  DTC_CHECK_ARG(s.C % 64 == 0 && s.K % 64 == 0, "conv: C (%d) and K (%d) must be multiples of 64", s.C, s.K);
  DTC_CHECK_ARG(s.stride == 1 || s.stride == 2, "conv: stride must be 1 or 2");
  DTC_CHECK_ARG(s.N > 0 && s.H > 0 && s.W > 0 && p.P > 0 && p.Q > 0, "conv: bad geometry");
  return 0;
}

template <int MODE, int BM, int BN, int WR, int WC, bool SLAB, bool SC = false>
static int launch_igemm(IGemmParams& p, int tiles_b, int splits, hipStream_t st, int gz = 1) {
  dim3 grid(p.tiles_a * tiles_b, splits, gz);
  p.xcd_remap = option_get(OPT_XCD_REMAP);
  DTC_KLAUNCH((igemm_kernel<MODE, BM, BN, WR, WC, SLAB, 2, SC>), grid, dim3(256), 0, st, p);
  DTC_LAUNCH_CHECK();
  return 0;
}

static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// Choose split-K so that the grid holds about `target` workgroups while each split keeps
// at least `min_kt` reduction steps.
static int pick_splits(int tiles, int num_kt, int target, int min_kt) {
  int s = ceil_div(target, tiles);
  s = std::min(s, std::max(1, num_kt / min_kt));
  return std::max(1, s);
}

static bool dgrad_class_mode(const ConvShape& s) {
  return s.stride == 2 && (s.H % 2) == 0 && (s.W % 2) == 0 && option_get(OPT_DGRAD_CLASSES) != 0;
}

bool dgrad_class_ok(const ConvShape& s) { return dgrad_class_mode(s) && !conv_c64_ok(s) && conv_halo_plan(s, CONV_DGRAD).cfg < 0; }

ConvPlan plan_conv(const ConvShape& s, int mode) {
  ConvPlan pl{};
  const int P = (s.H + 2 * s.pad - s.R) / s.stride + 1;
  const int Q = (s.W + 2 * s.pad - s.S) / s.stride + 1;
  const bool cls = (mode == CONV_DGRAD) && dgrad_class_mode(s);
  if (mode == CONV_FWD || mode == CONV_DGRAD) {
    const int M = (mode == CONV_FWD) ? s.N * P * Q : (cls ? s.N * (s.H / 2) * (s.W / 2) : s.N * s.H * s.W);
    const int A = (mode == CONV_FWD) ? s.K : s.C;
    const int num_kt = s.R * s.S * ((mode == CONV_FWD) ? s.C : s.K) / 64;
    // big tiles while they fill the chip (>= ~2 waves of 256 CUs), else 64x64 tiles, else split-K
    if (A == 64) { pl.bm = 64; pl.bn = 256; }
    else { pl.bm = 128; pl.bn = 128; }
    if ((A / pl.bm) * ceil_div(M, pl.bn) < 400) { pl.bm = 64; pl.bn = 64; }
    const int ft = option_get(OPT_IGEMM_TILE);  // tuning override
    if (ft == 1) { pl.bm = 64; pl.bn = 64; }
    else if (ft == 2 && A % 128 == 0) { pl.bm = 128; pl.bn = 128; }
    else if (ft == 3) { pl.bm = 64; pl.bn = 256; }
    const int tiles = (A / pl.bm) * ceil_div(M, pl.bn);
    pl.splits = (tiles >= 256 || cls) ? 1 : pick_splits(tiles, num_kt, 480, 8);
    if (option_get(OPT_IGEMM_SPLIT) > 0 && !cls) pl.splits = std::min(option_get(OPT_IGEMM_SPLIT), num_kt);
    pl.slab_bytes = pl.splits > 1 ? (size_t)pl.splits * M * A * 4 : 0;
    pl.slab_bytes = std::max(pl.slab_bytes, conv_halo_slab_bytes(s, mode));
    pl.num_kt = num_kt;
  } else if (const int s2 = wgrad_s2_splits(s)) {  // stride-2 column-split halo kernel (wgrad_halo.hip)
    pl.bm = 576;
    pl.bn = 64;
    pl.splits = s2;
    pl.num_kt = s.N * P * Q / 64;
    pl.slab_bytes = conv_wgrad_s2_slab_bytes(s);
  } else if (const int hs = wgrad_halo_splits(s)) {  // halo-tiled kernel (wgrad_halo.hip)
    pl.bm = 576;
    pl.bn = 64;
    pl.splits = hs;
    pl.num_kt = s.N * P * Q / 64;
    pl.slab_bytes = (size_t)hs * s.K * s.R * s.S * s.C * 4;
  } else {
    const int M = s.N * P * Q;
    const int num_kt = ceil_div(M, 64);
    pl.bm = (s.C == 64 || s.K == 64) ? 64 : 128;
    pl.bn = pl.bm;
    if ((s.R * s.S * s.C / pl.bm) * (s.K / pl.bn) < 64) pl.bm = pl.bn = 64;  // few output tiles: more of them
    const int ft = option_get(OPT_IGEMM_TILE);  // tuning override
    if (ft == 1) pl.bm = pl.bn = 64;
    else if (ft == 2 && (s.R * s.S * s.C) % 128 == 0 && s.K % 128 == 0) pl.bm = pl.bn = 128;
    const int tiles = (s.R * s.S * s.C / pl.bm) * (s.K / pl.bn);
    pl.splits = pick_splits(tiles, num_kt, 512, tiles < 64 ? 8 : 16);
    if (option_get(OPT_IGEMM_SPLIT) > 0) pl.splits = std::min(option_get(OPT_IGEMM_SPLIT), num_kt);
    pl.slab_bytes = (size_t)pl.splits * s.K * s.R * s.S * s.C * 4;
    pl.num_kt = num_kt;
  }
  return pl;
}

int conv_fwd(const ConvShape& s, const u16* x, const u16* w, u16* y, int64_t* stats, float* slab,
             size_t slab_bytes, hipStream_t st, u64* ts, unsigned* tick) {
  if (conv_c64_ok(s)) return conv_c64(s, CONV_FWD, x, w, y, nullptr, stats, st, ts);
  {
    const HaloPlan hp = conv_halo_plan(s, CONV_FWD);
    if (hp.cfg >= 0)
      return conv_halo(s, CONV_FWD, hp, x, w, y, nullptr, stats, slab, slab_bytes, st, ts, nullptr, nullptr, nullptr,
                       tick);
  }
  IGemmParams p{};
  p.ts = ts;
  DTC_TRY(fill_common(p, s));
  ConvPlan pl = plan_conv(s, CONV_FWD);
  p.src0 = x; p.src1 = w; p.out = y; p.stats = stats;
  p.M = s.N * p.P * p.Q;
  p.fd_q = make_fastdiv(p.Q); p.fd_pq = make_fastdiv(p.P * p.Q); p.fd_cc = make_fastdiv(s.C / 64);
  p.num_kt = pl.num_kt;
  p.tiles_a = s.K / pl.bm;
  const int tiles_b = ceil_div(p.M, pl.bn);
  int splits = pl.splits;
  if (splits > 1 && (slab == nullptr || slab_bytes < pl.slab_bytes)) splits = 1;
  p.kt_per_split = ceil_div(p.num_kt, splits);
  splits = ceil_div(p.num_kt, p.kt_per_split);
  if (splits > 1) {
    p.slab = slab;
    if (pl.bn == 64) DTC_TRY((launch_igemm<MODE_FWD, 64, 64, 2, 2, true>(p, tiles_b, splits, st)));
    else if (pl.bm == 64) DTC_TRY((launch_igemm<MODE_FWD, 64, 256, 1, 4, true>(p, tiles_b, splits, st)));
    else DTC_TRY((launch_igemm<MODE_FWD, 128, 128, 2, 2, true>(p, tiles_b, splits, st)));
    return splitk_reduce(slab, splits, p.M, s.K, y, nullptr, stats, st, ts);
  }
  if (pl.bn == 64) return launch_igemm<MODE_FWD, 64, 64, 2, 2, false>(p, tiles_b, 1, st);
  if (pl.bm == 64) return launch_igemm<MODE_FWD, 64, 256, 1, 4, false>(p, tiles_b, 1, st);
  return launch_igemm<MODE_FWD, 128, 128, 2, 2, false>(p, tiles_b, 1, st);
}

// 3x3 stride-2 conv + its block's 1x1 stride-2 projection shortcut in one launch (option sc_fuse):
// the shortcut's reduction is the centre tap of the 3x3's, so it reuses those im2col tiles (one read
// of x, one launch). Same per-output MFMA order as the separate launch when that one has no split-K.
bool conv_fwd_sc_ok(const ConvShape& s, const ConvShape& sc) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && sc.R == 1 && sc.S == 1 && sc.stride == 2 &&
        sc.pad == 0 && sc.N == s.N && sc.H == s.H && sc.W == s.W && sc.C == s.C && sc.K == s.K && s.C % 64 == 0))
    return false;
  if (conv_c64_ok(s)) return false;
  if (conv_halo_plan(s, CONV_FWD).cfg >= 0) return s.stride == 2;  // column-split halo kernel with SC
  const ConvPlan pl = plan_conv(s, CONV_FWD);
  // sc_fuse=1: 64x64-tile plans of at most 512 workgroups (layer4 at B=256: 35.3 us fused vs 8.2 + 31.1
  // separate); 2: every 64x64 plan (layer3: 35.6 vs 9.7 + 23.0 -- the shortcut's own 1024-workgroup launch
  // is cheaper than the fused kernel's lower occupancy); 3: also 128x128 (layer2: its W_sc stage takes
  // LDS to 96 KB, one workgroup per CU: 44.1 vs 11.8 + 21.2)
  const int lvl = option_get(OPT_SC_FUSE);
  if (pl.splits > 1) return false;
  if (pl.bn == 64) return lvl >= 2 || (int64_t)(s.K / 64) * ceil_div(s.N * ((s.H + 1) / 2) * ((s.W + 1) / 2), 64) <= 512;
  return pl.bm != 64 && lvl >= 3;
}

int conv_fwd_sc(const ConvShape& s, const ConvShape& sc, const u16* x, const u16* w, u16* y, int64_t* stats,
                const u16* wsc, u16* ysc, int64_t* stats_sc, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(conv_fwd_sc_ok(s, sc) && x && w && y && wsc && ysc, "conv_fwd_sc: unsupported shapes");
  {
    const HaloPlan hp = conv_halo_plan(s, CONV_FWD);
    if (hp.cfg >= 0)
      return conv_halo(s, CONV_FWD, hp, x, w, y, nullptr, stats, nullptr, 0, st, ts, wsc, ysc, stats_sc);
  }
  IGemmParams p{};
  p.ts = ts;
  DTC_TRY(fill_common(p, s));
  const ConvPlan pl = plan_conv(s, CONV_FWD);
  p.src0 = x; p.src1 = w; p.out = y; p.stats = stats;
  p.src1b = wsc; p.out2 = ysc; p.stats2 = stats_sc;
  p.M = s.N * p.P * p.Q;
  p.fd_q = make_fastdiv(p.Q); p.fd_pq = make_fastdiv(p.P * p.Q); p.fd_cc = make_fastdiv(s.C / 64);
  p.num_kt = pl.num_kt;
  p.kt_per_split = p.num_kt;
  const int nchunk = s.C / 64;
  p.kt_c0 = (1 * s.S + 1) * nchunk;  // tap (r, s) = (1, 1): the pixel (2p, 2q) the 1x1 stride-2 conv reads
  p.kt_c1 = p.kt_c0 + nchunk;
  p.tiles_a = s.K / pl.bm;
  const int tiles_b = ceil_div(p.M, pl.bn);
  if (pl.bn == 64) return launch_igemm<MODE_FWD, 64, 64, 2, 2, false, true>(p, tiles_b, 1, st);
  return launch_igemm<MODE_FWD, 128, 128, 2, 2, false, true>(p, tiles_b, 1, st);
}

// The BN-backward pass after a dgrad whose kernel has no fused epilogue for it (in place on dx).
static int bnb_after(const BnbArgs* bnb, u16* dx, int64_t M, int C, hipStream_t st) {
  if (bnb == nullptr || !bnb_on(*bnb)) return 0;
  if (bnb->mb)  // mask bits: the sums only (dx stays the raw gradient; the BN apply masks it)
    return bn_bwd_reduce_mask(dx, bnb->mb, bnb->x1, bnb->mean1, bnb->invstd1, bnb->acc1, bnb->x2, bnb->mean2,
                              bnb->invstd2, bnb->acc2, M, C, st);
  return bn_bwd_reduce(dx, bnb->ym, bnb->x1, bnb->mean1, bnb->invstd1, bnb->acc1, bnb->x2, bnb->mean2, bnb->invstd2,
                       bnb->acc2, dx, M, C, st);
}

int conv_dgrad(const ConvShape& s, const u16* dy, const u16* w, u16* dx, const u16* res, float* slab,
               size_t slab_bytes, hipStream_t st, u64* ts, const BnbArgs* bnb, int res_compact, unsigned* tick) {
  if (bnb != nullptr && !bnb_on(*bnb)) bnb = nullptr;
  DTC_CHECK_ARG(!res_compact || (res && dgrad_class_mode(s) && !conv_c64_ok(s)),
                "conv_dgrad: a compact residual needs the stride-2 parity-class path");
  // the BN-backward sums of dx by a reduction pass after the conv (the round-3/4 epilogue fusions measured
  // slower than the separate pass and were removed in round 5)
  if (bnb != nullptr) {
    DTC_TRY(conv_dgrad(s, dy, w, dx, res, slab, slab_bytes, st, ts, nullptr, res_compact, tick));
    return bnb_after(bnb, dx, (int64_t)s.N * s.H * s.W, s.C, st);
  }
  const HaloPlan hp = conv_c64_ok(s) ? HaloPlan{-1, 0} : conv_halo_plan(s, CONV_DGRAD);
  const int kind = conv_c64_ok(s) ? 1 : (hp.cfg >= 0 ? 2 : 4);
  if (kind == 1) return conv_c64(s, CONV_DGRAD, dy, w, dx, res, nullptr, st, ts);
  if (kind == 2)
    return conv_halo(s, CONV_DGRAD, hp, dy, w, dx, res, nullptr, slab, slab_bytes, st, ts, nullptr, nullptr, nullptr,
                     tick);
  IGemmParams p{};
  p.ts = ts;
  DTC_TRY(fill_common(p, s));
  ConvPlan pl = plan_conv(s, CONV_DGRAD);
  p.src0 = dy; p.src1 = w; p.out = dx; p.res = res;
  p.fd_cc = make_fastdiv(s.K / 64);
  p.num_kt = pl.num_kt;
  p.tiles_a = s.C / pl.bm;
  if (dgrad_class_mode(s) && res == nullptr && dgrad_s2_halo_ok(s)) {  // the halo sub-pixel kernel (dgrad_s2.hip)
    DTC_TRY(conv_dgrad_s2_halo(s, dy, w, dx, nullptr, nullptr, st, ts));
    return bnb_after(bnb, dx, (int64_t)s.N * s.H * s.W, s.C, st);
  }
  if (dgrad_class_mode(s)) {  // four parity-class GEMMs in one launch (blockIdx.z), no split-K
    p.cls = 1;
    p.cls_order = option_get(OPT_DGRAD_CLASS_ORDER);
    p.res_compact = res_compact;
    p.M = s.N * (s.H / 2) * (s.W / 2);
    p.fd_q = make_fastdiv(s.W / 2);
    p.fd_pq = make_fastdiv((s.H / 2) * (s.W / 2));
    p.kt_per_split = p.num_kt;
    const int tb = ceil_div(p.M, pl.bn);
    if (pl.bn == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 64, 2, 2, false>(p, tb, 1, st, 4)));
    else if (pl.bm == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 256, 1, 4, false>(p, tb, 1, st, 4)));
    else DTC_TRY((launch_igemm<MODE_DGRAD, 128, 128, 2, 2, false>(p, tb, 1, st, 4)));
    return bnb_after(bnb, dx, (int64_t)s.N * s.H * s.W, s.C, st);
  }
  p.M = s.N * s.H * s.W;
  p.fd_q = make_fastdiv(s.W); p.fd_pq = make_fastdiv(s.H * s.W);
  const int tiles_b = ceil_div(p.M, pl.bn);
  int splits = pl.splits;
  if (splits > 1 && (slab == nullptr || slab_bytes < pl.slab_bytes)) splits = 1;
  p.kt_per_split = ceil_div(p.num_kt, splits);
  splits = ceil_div(p.num_kt, p.kt_per_split);
  if (splits > 1) {
    p.slab = slab;
    if (pl.bn == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 64, 2, 2, true>(p, tiles_b, splits, st)));
    else if (pl.bm == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 256, 1, 4, true>(p, tiles_b, splits, st)));
    else DTC_TRY((launch_igemm<MODE_DGRAD, 128, 128, 2, 2, true>(p, tiles_b, splits, st)));
    return splitk_reduce(slab, splits, p.M, s.C, dx, res, nullptr, st, ts);
  }
  if (pl.bn == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 64, 2, 2, false>(p, tiles_b, 1, st)));
  else if (pl.bm == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 256, 1, 4, false>(p, tiles_b, 1, st)));
  else DTC_TRY((launch_igemm<MODE_DGRAD, 128, 128, 2, 2, false>(p, tiles_b, 1, st)));
  return bnb_after(bnb, dx, p.M, s.C, st);
}

// conv1 (3x3 stride 2) of a projection block and its 1x1 stride-2 shortcut: dx = dgrad(dc1, W1) +
// dgrad(dsc, W_sc) in ONE parity-class launch (the shortcut's term lives at class (0, 0) only, as extra
// reduction steps there: no separate shortcut dgrad launch and no compact residual pass).
bool conv_dgrad_sc_ok(const ConvShape& s) { return dgrad_class_ok(s) && s.R == 3 && s.pad == 1 && option_get(OPT_DGRAD_SCF) != 0; }
int conv_dgrad_sc(const ConvShape& s, const u16* dy, const u16* w, u16* dx, const u16* dsc, const u16* wsc,
                  hipStream_t st, u64* ts, const BnbArgs* bnb) {
  DTC_CHECK_ARG(conv_dgrad_sc_ok(s) && dy && w && dx && dsc && wsc, "conv_dgrad_sc: unsupported geometry / args");
  if (bnb != nullptr && !bnb_on(*bnb)) bnb = nullptr;
  if (dgrad_s2_halo_ok(s)) {  // option dgrad_s2h: the halo sub-pixel kernel (dgrad_s2.hip), shortcut fused
    DTC_TRY(conv_dgrad_s2_halo(s, dy, w, dx, dsc, wsc, st, ts));
    return bnb_after(bnb, dx, (int64_t)s.N * s.H * s.W, s.C, st);
  }
  IGemmParams p{};
  p.ts = ts;
  DTC_TRY(fill_common(p, s));
  ConvPlan pl = plan_conv(s, CONV_DGRAD);
  p.src0 = dy; p.src1 = w; p.out = dx; p.res = nullptr;
  p.src0b = dsc; p.src1b = wsc; p.sc_kt = s.K / 64;
  p.fd_cc = make_fastdiv(s.K / 64);
  p.num_kt = pl.num_kt;
  p.tiles_a = s.C / pl.bm;
  p.cls = 1;
  p.cls_order = option_get(OPT_DGRAD_CLASS_ORDER);
  p.M = s.N * (s.H / 2) * (s.W / 2);
  p.fd_q = make_fastdiv(s.W / 2);
  p.fd_pq = make_fastdiv((s.H / 2) * (s.W / 2));
  p.kt_per_split = p.num_kt;
  const int tb = ceil_div(p.M, pl.bn);
  if (pl.bn == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 64, 2, 2, false>(p, tb, 1, st, 4)));
  else if (pl.bm == 64) DTC_TRY((launch_igemm<MODE_DGRAD, 64, 256, 1, 4, false>(p, tb, 1, st, 4)));
  else DTC_TRY((launch_igemm<MODE_DGRAD, 128, 128, 2, 2, false>(p, tb, 1, st, 4)));
  return bnb_after(bnb, dx, (int64_t)s.N * s.H * s.W, s.C, st);
}

static int launch_wgrad_reduce(const float* slab, int splits, int K, int RSC, int ncols, int ldo, float scale,
                               const WgOuts& outs, int nprob, size_t prob_stride, hipStream_t st, u64* ts) {
  const size_t nv = (size_t)K * RSC / 4;
  int sg = 1;
  while (sg < 16 && sg * 2 <= splits && (nv * sg * nprob) / 256 < 1024) sg *= 2;
  const dim3 grid((unsigned)((nv + (256 / sg) - 1) / (256 / sg)), nprob);
#define DTC_WR(SG_) \
  DTC_KLAUNCH(wgrad_reduce_kernel<SG_>, grid, dim3(256), 0, st, slab, splits, K, RSC, ncols, ldo, scale, outs, prob_stride, ts)
  switch (sg) {
    case 1: DTC_WR(1); break;
    case 2: DTC_WR(2); break;
    case 4: DTC_WR(4); break;
    case 8: DTC_WR(8); break;
    default: DTC_WR(16); break;
  }
#undef DTC_WR
  DTC_LAUNCH_CHECK();
  return 0;
}

int conv_wgrad(const ConvShape& s, const u16* x, const u16* dy, float* dw, int dw_cols, int dw_ld, float scale,
               float* slab, size_t slab_bytes, hipStream_t st, u64* ts) {
  if (wgrad_s2_splits(s) > 0 && (dw_cols <= 0 || dw_cols == 9 * s.C) && (dw_ld <= 0 || dw_ld == 9 * s.C) &&
      slab_bytes >= conv_wgrad_s2_slab_bytes(s))
    return conv_wgrad_s2(s, x, dy, nullptr, dw, nullptr, scale, slab, slab_bytes, st, ts);
  IGemmParams p{};
  p.ts = ts;
  DTC_TRY(fill_common(p, s));
  ConvPlan pl = plan_conv(s, CONV_WGRAD);
  DTC_CHECK_ARG(slab != nullptr && slab_bytes >= (size_t)s.K * p.RSC * 4, "wgrad: slab workspace too small");
  p.src0 = x; p.src1 = dy; p.slab = slab;
  p.M = s.N * p.P * p.Q;
  p.fd_q = make_fastdiv(p.Q); p.fd_pq = make_fastdiv(p.P * p.Q); p.fd_cc = make_fastdiv(1);
  {
    const int PQ = p.P * p.Q;
    const uint64_t xb = (uint64_t)s.N * s.H * s.W * s.C * 2, db = (uint64_t)p.M * s.K * 2;
    const bool rows = (PQ % 64 == 0) && (64 % p.Q == 0);
    const bool imgs = (64 % PQ == 0);
    p.wg_fast = (rows || imgs) && xb < (1ull << 31) && db < (1ull << 31) && option_get(OPT_WGRAD_FAST) != 0;
    p.src0_bytes = (uint32_t)xb;
    p.src1_bytes = (uint32_t)db;
  }
  int splits = pl.splits;
  if (pl.bm == 576 && slab_bytes >= pl.slab_bytes) {
    const bool whole = (dw_cols <= 0 || dw_cols == p.RSC) && (dw_ld <= 0 || dw_ld == p.RSC);
    DTC_TRY(conv_wgrad_halo(s, 1, &x, &dy, slab, pl.splits, &splits, st, ts, whole ? &dw : nullptr, scale));
    if (splits == 0) return 0;  // one split: the halo kernel wrote dw itself
  } else {
    if (pl.bm == 576) pl = ConvPlan{64, 64, 1, ceil_div(p.M, 64), 0};  // workspace too small for the halo plan
    p.num_kt = pl.num_kt;
    p.tiles_a = p.RSC / pl.bm;
    const int tiles_b = s.K / pl.bn;
    while (splits > 1 && (size_t)splits * s.K * p.RSC * 4 > slab_bytes) --splits;
    p.kt_per_split = ceil_div(p.num_kt, splits);
    splits = ceil_div(p.num_kt, p.kt_per_split);
    if (pl.bm == 64) DTC_TRY((launch_igemm<MODE_WGRAD, 64, 64, 2, 2, true>(p, tiles_b, splits, st)));
    else DTC_TRY((launch_igemm<MODE_WGRAD, 128, 128, 2, 2, true>(p, tiles_b, splits, st)));
  }
  const int ncols = dw_cols > 0 ? dw_cols : p.RSC;
  const int ldo = dw_ld > 0 ? dw_ld : p.RSC;
  WgOuts outs{};
  outs.dw[0] = dw;
  return launch_wgrad_reduce(slab, splits, s.K, p.RSC, ncols, ldo, scale, outs, 1, 0, st, ts);
}

int wgrad_reduce_to(const float* slab, int splits, int K, int RSC, int ncols, int ldo, float scale, float* dw,
                    hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(slab && dw && splits > 0 && K > 0 && RSC % 4 == 0 && ncols <= RSC, "wgrad_reduce_to: bad args");
  WgOuts outs{};
  outs.dw[0] = dw;
  return launch_wgrad_reduce(slab, splits, K, RSC, ncols, ldo, scale, outs, 1, 0, st, ts);
}

// two dense reductions in one launch: slab[splits][K][ld0] -> dw0 and (slab + stride)[splits][K][ld1] -> dw1
// (a stride-2 conv1's taps and its fused shortcut's; blockIdx.y = which, grid sized by the larger)
int wgrad_reduce_pair(const float* slab, int splits, int K, int ld0, float* dw0, size_t stride, int ld1, float* dw1,
                      float scale, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(slab && dw0 && dw1 && splits > 0 && K > 0 && ld0 % 4 == 0 && ld1 % 4 == 0 && ld1 <= ld0,
                "wgrad_reduce_pair: bad args");
  WgOuts outs{};
  outs.dw[0] = dw0;
  outs.ld[0] = ld0;
  outs.dw[1] = dw1;
  outs.ld[1] = ld1;
  return launch_wgrad_reduce(slab, splits, K, ld0, ld0, ld0, scale, outs, 2, stride, st, ts);
}

size_t conv_wgrad_batch_slab_bytes(const ConvShape& s, int nprob) {
  return (size_t)nprob * wgrad_halo_splits(s, nprob) * s.K * s.R * s.S * s.C * 4;
}

int conv_wgrad_batch(const ConvShape& s, int nprob, const u16* const* x, const u16* const* dy, float* const* dw,
                     float scale, float* slab, size_t slab_bytes, hipStream_t st, u64* ts) {
  const int hs = wgrad_halo_splits(s, nprob);
  if (hs <= 0 || slab == nullptr || slab_bytes < conv_wgrad_batch_slab_bytes(s, nprob))
    return set_error(DTC_EINVAL, "conv_wgrad_batch: no halo plan for %d problems or slab too small", nprob);
  int splits = hs;
  DTC_TRY(conv_wgrad_halo(s, nprob, x, dy, slab, hs, &splits, st, ts, dw, scale));
  if (splits == 0) return 0;  // one split: the halo kernel wrote dw itself
  const int RSC = s.R * s.S * s.C;
  WgOuts outs{};
  for (int i = 0; i < nprob; ++i) outs.dw[i] = dw[i];
  return launch_wgrad_reduce(slab, splits, s.K, RSC, RSC, RSC, scale, outs, nprob, (size_t)splits * s.K * RSC, st, ts);
}

int splitk_reduce(const float* slab, int splits, int M, int Nc, u16* out, const u16* res, int64_t* stats,
                  hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(Nc % 8 == 0 && Nc <= 2048, "splitk_reduce: channels %d", Nc);
  const int tpr = Nc / 8;
  const int rpp = 256 / tpr;
  // 256..1024 workgroups of >= 16K outputs where the tensor allows; whole 256-thread passes
  int rows_per_block = std::max({rpp, (M + 1023) / 1024, std::min((16384 + Nc - 1) / Nc, (M + 255) / 256)});
  rows_per_block = ((rows_per_block + rpp - 1) / rpp) * rpp;
  const int blocks = ceil_div(M, rows_per_block);
  DTC_KLAUNCH(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, slab, splits, M, Nc, out, res, stats,
                     rows_per_block, ts);
  DTC_LAUNCH_CHECK();
  return 0;
}

int prof_accumulate(u64* ts, int n, u64* acc, hipStream_t st) {
  DTC_KLAUNCH(prof_accumulate_kernel, dim3((n + 63) / 64), dim3(64), 0, st, ts, n, acc);
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
