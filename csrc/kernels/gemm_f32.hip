// Generic f32 GEMM / implicit-GEMM convolution on v_mfma_f32_16x16x4_f32 (see gemm_f32.h).
//
// Workgroup: 256 threads = 4 waves, a 64 x 64 output tile, reduction in slices of 16 staged through
// LDS.  Wave w owns the 32 x 32 quadrant (w & 1, w >> 1): 2 x 2 MFMA 16x16 blocks, 16 MFMAs per
// slice.  Operands are fetched into registers one slice ahead (the next slice's global loads are in
// flight while the MFMAs of this one issue), then written to LDS k-major:
//   As[k][m]: thread t loads 4 consecutive k of row m = t & 63 (one 16-B load when the 4 values are
//             contiguous in memory, e.g. 4 channels of one pixel); lanes of a wave write 64
//             consecutive m -> conflict-free scalar LDS writes.
//   Bs[k][n]: thread t loads 4 consecutive n of row k = t >> 4, one 16-B LDS write.
// Row pitch 80 floats: the MFMA operand reads (16 consecutive m or n, 4 consecutive k across the
// lane groups) hit 64 distinct banks.
//
// The convolution index decodes run on mixed-radix counters advanced by 16 per slice (a division
// only on wrap-around), not per-element integer divisions.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "gemm_f32.h"

namespace tdl {
namespace {

constexpr int kLd = 80;

// (hi, mid, lo) counter, lo fastest, radices (., nmid, nlo)
struct Ctr {
  int hi, mid, lo;
  __device__ void set(int v, int nmid, int nlo) {
    const int q = v / nlo;
    lo = v - q * nlo;
    mid = q % nmid;
    hi = q / nmid;
  }
  __device__ void step1(int nmid, int nlo) {  // += 1: compares only (no division)
    if (++lo == nlo) {
      lo = 0;
      if (++mid == nmid) {
        mid = 0;
        ++hi;
      }
    }
  }
  __device__ void step(int d, int nmid, int nlo) {
    lo += d;
    if (lo >= nlo) {
      const int q = lo / nlo;
      lo -= q * nlo;
      mid += q;
      if (mid >= nmid) {
        const int q2 = mid / nmid;
        mid -= q2 * nmid;
        hi += q2;
      }
    }
  }
};

__device__ __forceinline__ void out_store(const F32GemmArgs& a, int m, int n, float v) {
  if (m == a.ones_m || n == a.ones_n) {  // the bias-gradient row / column
    float* d = a.dbias + (m == a.ones_m ? n : m);
    if (a.accumulate) v += *d;
    *d = v;
    return;
  }
  if (a.bias != nullptr) v += a.bias[n];
  const int64_t i = a.trans_out ? (int64_t)n * a.ldo + m : (int64_t)m * a.ldo + n;
  if (a.accumulate) v += a.out[i];
  if (a.act == 1) v = fmaxf(v, 0.f);
  a.out[i] = v;
}

template <bool MA, bool MB>
struct Slice {
  float a[4], b[4];
  float ma[MA ? 4 : 1], mb[MB ? 4 : 1];
  unsigned va, vb;  // loaded value valid (else 0)
  unsigned oa, ob;  // the appended row / column of ones (value 1, unmasked)
  unsigned pa, pp;  // PIN: the 4 elements' argmax bytes and their own window positions (byte i each)
};

template <int MODE, bool MA, bool MB, bool VA, bool VB, bool PIN = false, bool BUF = false>
__global__ __launch_bounds__(256) void k_gemm_f32(F32GemmArgs a) {
  using I = std::conditional_t<BUF, int, int64_t>;  // operand element index (32-bit with buffer loads)
  __shared__ float As[16 * kLd];
  __shared__ float Bs[16 * kLd];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.x * kF32Tile, n0 = blockIdx.y * kF32Tile;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.Kred, kbeg + a.kchunk);
  const F32ConvGeom& g = a.g;

  // A: row ml, reduction quad kqa; B: reduction row kl, column quad nqb.  With 16-B quads (VA: the
  // reduction is contiguous in memory, e.g. the channels of an NHWC pixel) four adjacent lanes read the
  // 64 contiguous bytes of one row's slice, so a wave-instruction touches 16 rows instead of 64 (a 16-B
  // piece of 64 different 256-B pixel rows: 4x the cache lines per useful byte); the element-wise
  // loaders keep a row per lane (then consecutive lanes read consecutive rows, e.g. a transposed A).
  // (the quad-major As writes are 4-way bank-conflicted; the MFMA reads, 8x as many, stay conflict-free)
  const int ml = VA ? t >> 2 : lane, kqa = VA ? (t & 3) * 4 : wave * 4;
  const int kl = t >> 4, nqb = (t & 15) * 4;
  const int am = m0 + ml, bn = n0 + nqb;
  const bool arow = am < a.M;

  // per-thread fixed decodes
  int an = 0, ay = 0, ax = 0;  // conv fwd: image, top-left input row / col; dgrad: image, y + pt, x + pl
  if constexpr (MODE == kF32ConvFwd) {
    int oy, ox;
    if (a.pool) {  // rows (n, ph, pw, q): pixel (2 ph + q / 2, 2 pw + q % 2)
      const int wins = a.pool_h * a.pool_w;
      an = am / (4 * wins);
      const int rem = am - an * 4 * wins, win = rem >> 2, q = rem & 3;
      const int php = win / a.pool_w;
      oy = 2 * php + (q >> 1);
      ox = 2 * (win - php * a.pool_w) + (q & 1);
    } else {
      const int hw = g.oh * g.ow;
      an = am / hw;
      const int p = am - an * hw;
      oy = p / g.ow;
      ox = p - oy * g.ow;
    }
    ay = oy * g.sh - g.pt;
    ax = ox * g.sw - g.pl;
  } else if constexpr (MODE == kF32ConvDgrad) {
    const int hw = g.h * g.w;
    an = am / hw;
    const int p = am - an * hw, y = p / g.w;
    ay = y + g.pt;
    ax = p - y * g.w + g.pl;
  }
  int wr[4] = {0, 0, 0, 0}, ws_[4] = {0, 0, 0, 0}, wc[4] = {0, 0, 0, 0};  // wgrad: (r, s, c) of the B columns
  if constexpr (MODE == kF32ConvWgrad) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = bn + i, rs = n / g.c;
      wc[i] = n - rs * g.c;
      ws_[i] = rs % g.s;
      wr[i] = rs / g.s;
    }
  }
  // reduction counters: fwd (r, s, c) / dgrad (r, s, k) of this thread's A quad; wgrad (img, oy, ox) of its B row
  Ctr ka{0, 0, 0}, kb{0, 0, 0};
  if constexpr (MODE == kF32ConvFwd) ka.set(kbeg + kqa, g.s, g.c);
  if constexpr (MODE == kF32ConvDgrad) ka.set(kbeg + kqa, g.s, g.k);
  if constexpr (MODE == kF32ConvWgrad) kb.set(kbeg + kl, g.oh, g.ow);
  if constexpr (MODE == kF32ConvWgrad && PIN) ka.set(kbeg + kqa, g.oh, g.ow);  // (img, oy, ox) of the A quad

  const bool s1 = g.sh == 1 && g.sw == 1;
  using S = Slice<MA, MB>;

  // A element e (valid or not) into slot i; a 16-B quad at slot 0 when vec.  BUF: buffer loads at 32-bit
  // byte offsets, an invalid element reads offset 0x80000000 (out of range: 0); else a clamped address
  // (built unconditionally: scalar work only, dead without BUF)
  const auto ra = buf_rsrc(a.a, (unsigned)(a.na * 4)), rb = buf_rsrc(a.b, (unsigned)(a.nb * 4));
  const auto ram = buf_rsrc(MA ? a.amask : a.a, (unsigned)(a.na * 4));
  const auto rbm = buf_rsrc(MB ? a.bmask : a.b, (unsigned)(a.nb * 4));
  auto lda1 = [&](S& r, int i, bool ok, I e) {
    if constexpr (BUF) {
      const int vo = ok ? (int)e * 4 : (int)0x80000000;
      r.a[i] = ld1_buf(ra, vo, 0);
      if constexpr (MA) r.ma[i] = ld1_buf(ram, vo, 0);
    } else {
      const I q = ok ? e : 0;
      r.a[i] = a.a[q];
      if constexpr (MA) r.ma[i] = a.amask[q];
    }
    r.va |= ok ? 1u << i : 0u;
  };
  auto lda4 = [&](S& r, bool ok, I e) {
    f4 v, mv;
    if constexpr (BUF) {
      const int vo = ok ? (int)e * 4 : (int)0x80000000;
      v = ld4_buf(ra, vo, 0);
      if constexpr (MA) mv = ld4_buf(ram, vo, 0);
    } else {
      const I q = ok ? e : 0;
      v = ld4(a.a + q);
      if constexpr (MA) mv = ld4(a.amask + q);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r.a[i] = v[i];
    if constexpr (MA) {
#pragma unroll
      for (int i = 0; i < 4; ++i) r.ma[i] = mv[i];
    }
    r.va = ok ? 15u : 0u;
  };
  auto ldb1 = [&](S& r, int i, bool ok, I e) {
    if constexpr (BUF) {
      const int vo = ok ? (int)e * 4 : (int)0x80000000;
      r.b[i] = ld1_buf(rb, vo, 0);
      if constexpr (MB) r.mb[i] = ld1_buf(rbm, vo, 0);
    } else {
      const I q = ok ? e : 0;
      r.b[i] = a.b[q];
      if constexpr (MB) r.mb[i] = a.bmask[q];
    }
    r.vb |= ok ? 1u << i : 0u;
  };
  auto ldb4 = [&](S& r, bool ok, I e) {
    f4 v, mv;
    if constexpr (BUF) {
      const int vo = ok ? (int)e * 4 : (int)0x80000000;
      v = ld4_buf(rb, vo, 0);
      if constexpr (MB) mv = ld4_buf(rbm, vo, 0);
    } else {
      const I q = ok ? e : 0;
      v = ld4(a.b + q);
      if constexpr (MB) mv = ld4(a.bmask + q);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r.b[i] = v[i];
    if constexpr (MB) {
#pragma unroll
      for (int i = 0; i < 4; ++i) r.mb[i] = mv[i];
    }
    r.vb = ok ? 15u : 0u;
  };

  auto load = [&](int k0, S& r) {
    r.va = r.vb = r.oa = r.ob = 0u;
    r.pa = r.pp = 0u;
    const int kk = k0 + kqa;  // A: reduction index of slot 0
    if constexpr (MODE == kF32Gemm) {
      const bool ones = am == a.ones_m;  // the appended row of ones (bias gradient)
      if constexpr (VA) {
        lda4(r, !ones && arow && kk < kend, (I)am * (I)a.sam + kk);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          lda1(r, i, !ones && arow && kk + i < kend, (I)am * (I)a.sam + (I)(kk + i) * (I)a.sak);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) r.oa |= (ones && kk + i < kend) ? 1u << i : 0u;
    } else if constexpr (MODE == kF32ConvFwd || MODE == kF32ConvDgrad) {
      const int nlo = MODE == kF32ConvFwd ? g.c : g.k;
      Ctr c = ka;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!VA || i == 0) {  // a 16-B quad at slot 0, or one element per slot
          int iy, ix;
          bool ok;
          if constexpr (MODE == kF32ConvFwd) {
            iy = ay + c.hi * g.dh;
            ix = ax + c.mid * g.dw;
            ok = iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
          } else {
            const int ty = ay - c.hi * g.dh, tx = ax - c.mid * g.dw;
            iy = s1 ? ty : ty / g.sh;  // (stride 1: no integer division per element)
            ix = s1 ? tx : tx / g.sw;
            ok = ty >= 0 && tx >= 0 && (s1 || (iy * g.sh == ty && ix * g.sw == tx)) && iy < g.oh && ix < g.ow;
          }
          ok = ok && arow && kk + i < kend;
          I base = MODE == kF32ConvFwd ? (((I)an * g.h + iy) * g.w + ix) * g.c
                                             : (((I)an * g.oh + iy) * g.ow + ix) * g.k;
          if constexpr (PIN && MODE == kF32ConvDgrad) {  // the pool window of dy pixel (iy, ix)
            ok = ok && iy < 2 * a.pool_h && ix < 2 * a.pool_w;
            base = (((I)an * a.pool_h + (iy >> 1)) * a.pool_w + (ix >> 1)) * g.k;
            const unsigned pos = (unsigned)(((iy & 1) << 1) | (ix & 1));
            if constexpr (VA) {
              r.pa = *reinterpret_cast<const unsigned*>(a.pin_arg + (ok ? base + c.lo : 0));
              r.pp = pos * 0x01010101u;
            } else {
              r.pa |= (unsigned)a.pin_arg[ok ? base + c.lo : 0] << (8 * i);
              r.pp |= pos << (8 * i);
            }
          }
          if constexpr (VA)
            lda4(r, ok, base + c.lo);
          else
            lda1(r, i, ok, base + c.lo);
          if (!VA && i < 3) c.step1(g.s, nlo);
        }
      }
    } else if constexpr (PIN) {  // wgrad, pooled dy: pixel j = kk + i -> its window, argmax check
      Ctr c = ka;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i) c.step1(g.oh, g.ow);
        const bool ok = arow && kk + i < kend && c.mid < 2 * a.pool_h && c.lo < 2 * a.pool_w;
        const I e = (((I)c.hi * a.pool_h + (c.mid >> 1)) * a.pool_w + (c.lo >> 1)) * g.k + am;
        lda1(r, i, ok, e);
        r.pa |= (unsigned)a.pin_arg[ok ? e : 0] << (8 * i);
        r.pp |= (unsigned)(((c.mid & 1) << 1) | (c.lo & 1)) << (8 * i);
      }
    } else {  // wgrad: A(m = out channel, j) = dy[j][m]
#pragma unroll
      for (int i = 0; i < 4; ++i) lda1(r, i, arow && kk + i < kend, (I)(kk + i) * g.k + am);
    }

    const int kr = k0 + kl;  // B: reduction index of this thread's row
    const bool brow = kr < kend;
    if constexpr (MODE == kF32ConvWgrad) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = bn + i;
        const bool ones = n == a.ones_n;  // the appended column of ones (bias gradient)
        r.ob |= (ones && brow) ? 1u << i : 0u;
        if (!VB || i == 0) {  // a 16-B quad at slot 0 (the ones column starts a quad), or one element per slot
          const int iy = kb.mid * g.sh - g.pt + wr[i] * g.dh, ix = kb.lo * g.sw - g.pl + ws_[i] * g.dw;
          const bool ok = !ones && brow && n < a.N && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
          const I e = (((I)kb.hi * g.h + iy) * g.w + ix) * g.c + wc[i];
          if constexpr (VB)
            ldb4(r, ok, e);
          else
            ldb1(r, i, ok, e);
        }
      }
    } else if (MODE == kF32ConvDgrad && a.b_hwio) {  // w HWIO: B(kr = rs * K + kk, n = c) = w[rs][c][kk]
      const int rs = kr / g.k, kk2 = kr - rs * g.k;
      const I row = (I)rs * a.N * g.k + kk2;
#pragma unroll
      for (int i = 0; i < 4; ++i) ldb1(r, i, brow && bn + i < a.N, row + (I)(bn + i) * g.k);
    } else {
      const I sbk = MODE == kF32Gemm ? (I)a.sbk : (I)a.N;
      const I sbn = MODE == kF32Gemm ? (I)a.sbn : 1;
      if constexpr (VB) {
        ldb4(r, brow && bn < a.N, (I)kr * sbk + bn);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) ldb1(r, i, brow && bn + i < a.N, (I)kr * sbk + (I)(bn + i) * sbn);
      }
    }
  };

  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero4();

  const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
  const int lr = lane & 15, lk = lane >> 4;
  // Register ring of kDepth slices: slice k + kDepth is loaded while slice k is multiplied, so a
  // long reduction pays the global-load latency once per kDepth slices, not once per slice (the
  // small-M / long-K shapes of the generic engine are latency-bound: few workgroups, many slices).
  constexpr int kDepth = 4;
  S ring[kDepth];
  int kload = kbeg;  // reduction index of the next slice to load (the counters track the last one)
  // (no branches around the loads: slices past kend load clamped addresses and become zeros, so
  // the loop body is straight-line and the waits before each LDS write are exact vmcnt counts)
  auto issue = [&](S& r) {
    if (kload < kend) {  // (uniform; past the end the registers keep stale values, never stored)
      if (kload != kbeg) {
        if constexpr (MODE == kF32ConvFwd) ka.step(16, g.s, g.c);
        if constexpr (MODE == kF32ConvDgrad) ka.step(16, g.s, g.k);
        if constexpr (MODE == kF32ConvWgrad) kb.step(16, g.oh, g.ow);
        if constexpr (MODE == kF32ConvWgrad && PIN) ka.step(16, g.oh, g.ow);
      }
      load(kload, r);
    }
    kload += 16;
  };
#pragma unroll
  for (int d = 0; d < kDepth; ++d) issue(ring[d]);
  for (int k0 = kbeg; k0 < kend; k0 += 16 * kDepth) {
#pragma unroll
    for (int d = 0; d < kDepth; ++d) {
      // (the LDS / MFMA work of slices past kend is skipped by a uniform branch; the loads are not
      // (clamped, invalid), so no load sits in a branch and every wait stays an exact count)
      const bool live = k0 + 16 * d < kend;
      S& r = ring[d];
      if (live) {
        float av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[i] = (r.va >> i & 1u) ? r.a[i] : 0.f;
          bv[i] = (r.vb >> i & 1u) ? r.b[i] : 0.f;
          if constexpr (MA) av[i] = r.ma[i] > 0.f ? av[i] : 0.f;
          if constexpr (PIN) av[i] = ((r.pa >> (8 * i)) & 0xffu) == ((r.pp >> (8 * i)) & 0xffu) ? av[i] : 0.f;
          if constexpr (MB) bv[i] = r.mb[i] > 0.f ? bv[i] : 0.f;
          av[i] = (r.oa >> i & 1u) ? 1.f : av[i];
          bv[i] = (r.ob >> i & 1u) ? 1.f : bv[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) As[(kqa + i) * kLd + ml] = av[i];
        st4(&Bs[kl * kLd + nqb], f4{bv[0], bv[1], bv[2], bv[3]});
        __syncthreads();
      }
      issue(r);  // slice k0 + 16 (d + kDepth) into the registers just stored
      if (live) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int kr = (4 * ks + lk) * kLd;
          const float a0 = As[kr + wm + lr], a1 = As[kr + wm + 16 + lr];
          const float b0 = Bs[kr + wn + lr], b1 = Bs[kr + wn + 16 + lr];
          acc[0][0] = mfma16x16x4(a0, b0, acc[0][0]);
          acc[0][1] = mfma16x16x4(a0, b1, acc[0][1]);
          acc[1][0] = mfma16x16x4(a1, b0, acc[1][0]);
          acc[1][1] = mfma16x16x4(a1, b1, acc[1][1]);
        }
        __syncthreads();
      }
    }
  }

  // D[(lane >> 4) * 4 + r][lane & 15] of each 16x16 block
  if (a.splits > 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm + 16 * i + 4 * lk + r, n = n0 + wn + 16 * j + lr;
          if (m < a.M && n < a.N) a.ws[((int64_t)blockIdx.z * a.M + m) * a.N + n] = acc[i][j][r];
        }
    return;
  }
  // out_store's operands (bias, the accumulated output or bias gradient) for all 16 outputs of the
  // lane loaded first, then the stores: one memory round trip instead of one per output (each
  // load-add-store of out_store waited for its load with vmcnt(0)); same arithmetic order as out_store
  float bv[2][2][4], ov[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * lk + r, n = n0 + wn + 16 * j + lr;
        bv[i][j][r] = ov[i][j][r] = 0.f;
      }
  // (each batch behind ONE uniform branch, clamped addresses inside it: no per-element branch, so the
  // compiler waits once for the batch -- a vmcnt(0) per element would also wait for the stores)
  if (a.bias != nullptr) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn + 16 * j + lr;
        const float t = a.bias[n < a.N ? n : 0];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[i][j][r] = t;
      }
  }
  if (a.accumulate) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm + 16 * i + 4 * lk + r, n = n0 + wn + 16 * j + lr;
          const bool ok = m < a.M && n < a.N;
          const bool ones = m == a.ones_m || n == a.ones_n;
          const int64_t o = ones ? (int64_t)(m == a.ones_m ? n : m)
                                 : (a.trans_out ? (int64_t)n * a.ldo + m : (int64_t)m * a.ldo + n);
          ov[i][j][r] = (ones ? a.dbias : a.out)[ok ? o : 0];
        }
  }
  if (MODE == kF32ConvFwd && a.pool) {
    // a lane's 4 rows 4 lk + r of each 16-row block are one pool window (window-major rows, M % 4 == 0)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int mb = m0 + wm + 16 * i + 4 * lk, n = n0 + wn + 16 * j + lr;
        if (mb >= a.M || n >= a.N) continue;
        const int wins = a.pool_h * a.pool_w;
        const int img = mb / (4 * wins), win = (mb >> 2) - img * wins;
        const int php = win / a.pool_w, pwp = win - php * a.pool_w;
        float best = -INFINITY;
        uint32_t arg = 255u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // the same arithmetic as the unfused epilogue, then the pool's max
          float v = acc[i][j][r];
          if (a.bias != nullptr) v += bv[i][j][r];
          if (a.act == 1) v = fmaxf(v, 0.f);
          const int oy = 2 * php + (r >> 1), ox = 2 * pwp + (r & 1);
          a.out[(((int64_t)img * g.oh + oy) * g.ow + ox) * a.ldo + n] = v;
          if (v > best) {
            best = v;
            arg = (uint32_t)r;  // window position (dy * 2 + dx), first maximum wins
          }
        }
        const int64_t po = (((int64_t)img * a.pool_h + php) * a.pool_w + pwp) * a.N + n;
        a.pout[po] = best;
        a.parg[po] = (uint8_t)arg;
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * lk + r, n = n0 + wn + 16 * j + lr;
        if (m >= a.M || n >= a.N) continue;
        float v = acc[i][j][r];
        if (m == a.ones_m || n == a.ones_n) {  // the bias-gradient row / column
          if (a.accumulate) v += ov[i][j][r];
          a.dbias[m == a.ones_m ? n : m] = v;
          continue;
        }
        if (a.bias != nullptr) v += bv[i][j][r];
        if (a.accumulate) v += ov[i][j][r];
        if (a.act == 1) v = fmaxf(v, 0.f);
        a.out[a.trans_out ? (int64_t)n * a.ldo + m : (int64_t)m * a.ldo + n] = v;
      }
}

__device__ __forceinline__ void out_index(const F32GemmArgs& a, int64_t e, int& m, int& n) {
  // (selects, not branches writing through the references: the compiler spilled those to scratch)
  const int64_t inner = a.trans_out ? a.M : a.N;
  const int q = (int)(e / inner), r = (int)(e - (int64_t)q * inner);
  m = a.trans_out ? r : q;
  n = a.trans_out ? q : r;
}

// Split-reduction epilogue: the slices summed in a fixed order, then bias / accumulate / store.
// Outputs are walked in storage order (coalesced stores, strided partial reads when transposed).
// Few slices: one thread per output, 16 independent partial loads in flight.  R < 16: at most R slices
// (no full round), only R loads issued; the sum still adds all 16 terms (zeros past the end): same bits.
template <int R>
__global__ __launch_bounds__(256) void k_gemm_f32_reduce(F32GemmArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mn = (int64_t)a.M * a.N;
  if (e >= mn) return;
  int m, n;
  out_index(a, e, m, n);
  const float* src = a.ws + (int64_t)m * a.N + n;
  float v = 0.f;
  int z = 0;
  for (; z + 16 <= a.splits; z += 16) {  // 16 independent partial loads in flight per round
    float p[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) p[u] = src[(z + u) * mn];
#pragma unroll
    for (int u = 0; u < 16; ++u) v += p[u];
  }
  {
    float p[16];  // the remainder, also in one round (clamped loads, zero past the end)
#pragma unroll
    for (int u = 0; u < R; ++u) p[u] = src[(int64_t)min(z + u, a.splits - 1) * mn];
#pragma unroll
    for (int u = 0; u < 16; ++u) p[u] = u < R && z + u < a.splits ? p[u] : 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) v += p[u];
  }
  out_store(a, m, n, v);
}

// Split-reduction of the pooled conv (F32GemmArgs::pool, < 16 slices): one thread per (pool window,
// column) sums each of the window's 4 rows exactly as k_gemm_f32_reduce sums an output (slices in
// order, rounds of 16 with zero-filled remainders: the same bits as the unfused conv's reduction), then
// the pooled epilogue of k_gemm_f32 (bias, ReLU, y, maximum, argmax).
template <bool HOIST, int R = 16>
__global__ __launch_bounds__(256) void k_gemm_f32_reduce_pool(F32GemmArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t wins = (int64_t)(a.M >> 2) * a.N;
  if (e >= wins) return;
  const int win = (int)(e / a.N), n = (int)(e - (int64_t)win * a.N);
  const int64_t mn = (int64_t)a.M * a.N;
  const int wpi = a.pool_h * a.pool_w;
  const int img = win / wpi, wi = win - img * wpi;
  const int php = wi / a.pool_w, pwp = wi - php * a.pool_w;
  const float bias = a.bias != nullptr ? a.bias[n] : 0.f;
  float best = -INFINITY;
  uint32_t arg = 255u;
  if (HOIST && a.splits < 16) {
    // the 4 rows' partials all loaded before any store (the stores to out may alias the slab for the
    // compiler, which then kept each row's loads behind the previous row's store: 4 serial round trips)
    float p[4][16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* src = a.ws + (int64_t)(4 * win + r) * a.N + n;
#pragma unroll
      for (int u = 0; u < R; ++u) p[r][u] = src[(int64_t)min(u, a.splits - 1) * mn];  // (R >= splits)
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = 0.f;  // = k_gemm_f32_reduce's remainder round: slices in order, zeros past the end
#pragma unroll
      for (int u = 0; u < 16; ++u) v += u < R && u < a.splits ? p[r][u] : 0.f;
      if (a.bias != nullptr) v += bias;
      if (a.act == 1) v = fmaxf(v, 0.f);
      const int oy = 2 * php + (r >> 1), ox = 2 * pwp + (r & 1);
      a.out[(((int64_t)img * a.g.oh + oy) * a.g.ow + ox) * a.ldo + n] = v;
      if (v > best) {
        best = v;
        arg = (uint32_t)r;
      }
    }
    const int64_t po = (((int64_t)img * a.pool_h + php) * a.pool_w + pwp) * a.N + n;
    a.pout[po] = best;
    a.parg[po] = (uint8_t)arg;
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* src = a.ws + (int64_t)(4 * win + r) * a.N + n;
    float v = 0.f;
    int z = 0;
    for (; z + 16 <= a.splits; z += 16) {
      float p[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) p[u] = src[(z + u) * mn];
#pragma unroll
      for (int u = 0; u < 16; ++u) v += p[u];
    }
    {
      float p[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) p[u] = src[(int64_t)min(z + u, a.splits - 1) * mn];
#pragma unroll
      for (int u = 0; u < 16; ++u) p[u] = z + u < a.splits ? p[u] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) v += p[u];
    }
    if (a.bias != nullptr) v += bias;
    if (a.act == 1) v = fmaxf(v, 0.f);
    const int oy = 2 * php + (r >> 1), ox = 2 * pwp + (r & 1);
    a.out[(((int64_t)img * a.g.oh + oy) * a.g.ow + ox) * a.ldo + n] = v;
    if (v > best) {
      best = v;
      arg = (uint32_t)r;
    }
  }
  const int64_t po = (((int64_t)img * a.pool_h + php) * a.pool_w + pwp) * a.N + n;
  a.pout[po] = best;
  a.parg[po] = (uint8_t)arg;
}

// Many slices over few outputs (a small weight gradient over a long reduction): one wave per output,
// lane l sums slices l, l + 64, .. in order, then a fixed xor butterfly over the wave (deterministic).
__global__ __launch_bounds__(256) void k_gemm_f32_reduce_wave(F32GemmArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t mn = (int64_t)a.M * a.N;
  if (e >= mn) return;
  int m, n;
  out_index(a, e, m, n);
  const float* src = a.ws + (int64_t)m * a.N + n;
  float v = 0.f;
  for (int z = lane; z < a.splits; z += 64) v += src[z * mn];
  v = wave_sum(v);
  if (lane == 0) out_store(a, m, n, v);
}

// Many slices over many outputs: a wave sums OUT (16, or 4 for a few hundred outputs) consecutive
// partial-slab entries (OUT * 4 contiguous bytes of each slice as 16-B loads per lane, instead of a 4-B
// load per output and slice spread over 64 cache lines).  Per output the arithmetic of k_gemm_f32_reduce_wave: lane l sums slices l, l + 64, .. in
// order, then the same xor butterfly (whose result is the same on every lane) -- bit-identical.
template <int OUT, bool V4>
__global__ __launch_bounds__(256) void k_gemm_f32_reduce_wave16(F32GemmArgs a) {
  const int64_t mn = (int64_t)a.M * a.N;
  const int64_t f0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * OUT;
  const int lane = threadIdx.x & 63;
  if (f0 >= mn) return;
  const int nv = (int)(mn - f0 < OUT ? mn - f0 : OUT);
  const float* src = a.ws + f0;
  float acc[OUT];
#pragma unroll
  for (int i = 0; i < OUT; ++i) acc[i] = 0.f;
#pragma unroll 2
  for (int z = lane; z < a.splits; z += 64) {
    const float* q = src + (int64_t)z * mn;
    float p[OUT];
    if (V4 && nv == OUT) {
#pragma unroll
      for (int i = 0; i < OUT / 4; ++i) {
        const f4 u = reinterpret_cast<const f4*>(q)[i];
        p[4 * i] = u.x;
        p[4 * i + 1] = u.y;
        p[4 * i + 2] = u.z;
        p[4 * i + 3] = u.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < OUT; ++i) p[i] = i < nv ? q[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < OUT; ++i) acc[i] += p[i];
  }
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < OUT; ++i) {
    const float s = wave_sum(acc[i]);
    v = lane == i ? s : v;
  }
  if (lane < nv) {
    const int64_t f = f0 + lane;
    const int m = (int)(f / a.N), n = (int)(f - (int64_t)m * a.N);
    out_store(a, m, n, v);
  }
}

// TDL_F32_REDUCE16=0: every many-slice reduction one wave per output (A/B hook)
bool g_reduce16 = [] {
  const char* e = std::getenv("TDL_F32_REDUCE16");
  return e == nullptr || std::atoi(e) != 0;
}();

bool reduce16_on() { return g_reduce16; }

// TDL_F32_REDUCE_NARROW=0: the few-slice reduces issue 16 loads whatever the slice count (A/B hook)
bool reduce_narrow() {
  static const bool on = [] {
    const char* e = std::getenv("TDL_F32_REDUCE_NARROW");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

// the operand-vectorisation instantiation of a (mode, mask) kernel
template <int MODE, bool MA, bool MB, bool PIN, bool BUF>
void launch_vb(const F32GemmArgs& a, dim3 grid, hipStream_t s) {
  if (a.vec_a && a.vec_b) hipLaunchKernelGGL((k_gemm_f32<MODE, MA, MB, true, true, PIN, BUF>), grid, dim3(256), 0, s, a);
  else if (a.vec_a) hipLaunchKernelGGL((k_gemm_f32<MODE, MA, MB, true, false, PIN, BUF>), grid, dim3(256), 0, s, a);
  else if (a.vec_b) hipLaunchKernelGGL((k_gemm_f32<MODE, MA, MB, false, true, PIN, BUF>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_gemm_f32<MODE, MA, MB, false, false, PIN, BUF>), grid, dim3(256), 0, s, a);
}

// buffer-resource operand loads when both operands (and their masks) fit 32-bit byte offsets
// (TDL_F32_BUF=0 keeps the 64-bit address form everywhere: A/B hook)
bool f32_buf_ok(const F32GemmArgs& a) {
  static const bool on = [] {
    const char* e = std::getenv("TDL_F32_BUF");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on && a.na > 0 && a.nb > 0 && a.na < (int64_t(1) << 29) && a.nb < (int64_t(1) << 29);
}

template <int MODE, bool MA, bool MB, bool PIN = false>
void launch_v(const F32GemmArgs& a, dim3 grid, hipStream_t s) {
  if (f32_buf_ok(a) && !PIN) launch_vb<MODE, MA, MB, PIN, true>(a, grid, s);
  else launch_vb<MODE, MA, MB, PIN, false>(a, grid, s);
}

}  // namespace

void f32_reduce16(bool on) { g_reduce16 = on; }

void f32_gemm_launch(int mode, const F32GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  const dim3 grid((a.M + kF32Tile - 1) / kF32Tile, (a.N + kF32Tile - 1) / kF32Tile, a.splits);
  const bool ma = a.amask != nullptr, mb = a.bmask != nullptr;
  switch (mode) {
    case kF32Gemm:
      if (ma && mb) launch_v<kF32Gemm, true, true>(a, grid, s);
      else if (ma) launch_v<kF32Gemm, true, false>(a, grid, s);
      else if (mb) launch_v<kF32Gemm, false, true>(a, grid, s);
      else launch_v<kF32Gemm, false, false>(a, grid, s);
      break;
    case kF32ConvFwd: launch_v<kF32ConvFwd, false, false>(a, grid, s); break;
    case kF32ConvDgrad:
      if (a.pin_arg != nullptr) launch_v<kF32ConvDgrad, true, false, true>(a, grid, s);  // (amask = the maximum)
      else if (ma) launch_v<kF32ConvDgrad, true, false>(a, grid, s);
      else launch_v<kF32ConvDgrad, false, false>(a, grid, s);
      break;
    default:
      if (a.pin_arg != nullptr) launch_v<kF32ConvWgrad, true, false, true>(a, grid, s);
      else if (ma) launch_v<kF32ConvWgrad, true, false>(a, grid, s);
      else launch_v<kF32ConvWgrad, false, false>(a, grid, s);
      break;
  }
  if (a.splits > 1 && a.pool) {
    const int64_t wins = (int64_t)(a.M >> 2) * a.N;
    static const bool hoist = [] {  // TDL_F32_POOLRED_HOIST=0: row by row (A/B hook)
      const char* e = std::getenv("TDL_F32_POOLRED_HOIST");
      return e == nullptr || std::atoi(e) != 0;
    }();
    const bool narrow = reduce_narrow();
    if (hoist && narrow && a.splits <= 4)  // (only the loads the slices need: the 16-term sums unchanged)
      hipLaunchKernelGGL((k_gemm_f32_reduce_pool<true, 4>), dim3((unsigned)((wins + 255) / 256)), dim3(256), 0, s, a);
    else if (hoist && narrow && a.splits <= 8)
      hipLaunchKernelGGL((k_gemm_f32_reduce_pool<true, 8>), dim3((unsigned)((wins + 255) / 256)), dim3(256), 0, s, a);
    else if (hoist)
      hipLaunchKernelGGL(k_gemm_f32_reduce_pool<true>, dim3((unsigned)((wins + 255) / 256)), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(k_gemm_f32_reduce_pool<false>, dim3((unsigned)((wins + 255) / 256)), dim3(256), 0, s, a);
  } else if (a.splits > 1) {
    const int64_t mn = (int64_t)a.M * a.N;
    if (a.splits >= 16 && mn >= 512 * 16 && reduce16_on()) {  // >= 512 waves of 16 outputs
      const dim3 gr((unsigned)((mn + 63) / 64));
      if (mn % 4 == 0)
        hipLaunchKernelGGL((k_gemm_f32_reduce_wave16<16, true>), gr, dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((k_gemm_f32_reduce_wave16<16, false>), gr, dim3(256), 0, s, a);
    } else if (a.splits >= 16 && mn >= 64 * 4 && reduce16_on()) {  // >= 64 waves of 4 outputs
      const dim3 gr((unsigned)((mn + 15) / 16));
      if (mn % 4 == 0)
        hipLaunchKernelGGL((k_gemm_f32_reduce_wave16<4, true>), gr, dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((k_gemm_f32_reduce_wave16<4, false>), gr, dim3(256), 0, s, a);
    } else if (a.splits >= 16)  // one wave per output: every partial of an output in one load round
      hipLaunchKernelGGL(k_gemm_f32_reduce_wave, dim3((unsigned)((mn + 3) / 4)), dim3(256), 0, s, a);
    else {
      const bool narrow = reduce_narrow();
      const dim3 gr((unsigned)((mn + 255) / 256));
      if (narrow && a.splits <= 4)
        hipLaunchKernelGGL(k_gemm_f32_reduce<4>, gr, dim3(256), 0, s, a);
      else if (narrow && a.splits <= 8)
        hipLaunchKernelGGL(k_gemm_f32_reduce<8>, gr, dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL(k_gemm_f32_reduce<16>, gr, dim3(256), 0, s, a);
    }
  }
}

}  // namespace tdl
