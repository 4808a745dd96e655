// Fused MNIST-CNN training step for gfx950 (MI355X), f32 end to end.
//
// Replaces, for the reference model of tf_dist_example.py:40-52, the ~35 TF/cuDNN/Eigen kernels
// of one replica step by eight launches:
//
//   K1 conv1_pool   : gather(idx) + conv1 3x3 (1->32) + bias + ReLU + maxpool2  (VALU; K=9)
//   K2 conv2_pool   : conv2 3x3 (32->64) implicit GEMM on v_mfma_f32_16x16x4_f32, epilogue
//                     bias + ReLU + maxpool2 done in registers (a 16-row MFMA tile = 4 windows)
//   K3 dense1       : [b,1600]x[1600,128] MFMA, 8-wave in-workgroup split-K, bias + ReLU
//   K4 head         : dense2 + softmax-xent + dlogits*(1/(b*R)) + loss/accuracy accumulators
//                     + dW4/db4 + dH (ReLU mask), one workgroup
//   K5 dense1_bwd   : dW3 = P2^T dH, db3, dP2 = dH W3^T -> pool2/ReLU backward scatter to dC2
//   K6 conv2_wgrad  : dW2 (+db2 as an extra "ones" row) split-K MFMA partial slabs
//   K7 conv2_dgrad  : dP1 = dC2 (*) W2^T on MFMA, epilogue = pool1/ReLU backward AND conv1
//                     wgrad (dC1 is never materialised), per-block partial slabs
//   K9 finalize     : deterministic reduction of the partial slabs into the flat gradient slab,
//                     optionally fused with the SGD update (single replica)
//
// All reductions are slab-based (no float atomics) so every replica computes bit-identical
// updates from identical inputs.
#include "common.h"
#include "mnist_cnn.h"

namespace tdl {

// --------------------------------------------------------------------------------------------
// K1: conv1 + bias + relu + maxpool.  One thread = one pooled pixel x 4 output channels.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_conv1_pool(MnistArgs a) {
  __shared__ float sw[320];
  for (int i = threadIdx.x; i < 320; i += 256)
    sw[i] = (i < 288) ? a.W[a.ow1 + i] : a.W[a.ob1 + i - 288];
  __syncthreads();
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= a.b * 169 * 8) return;
  const int cg = t & 7, pix = t >> 3;
  const int bi = pix / 169, p = pix - bi * 169, ph = p / 13, pw = p - ph * 13;
  const float* img = a.X + (size_t)a.idx[bi] * 784 + (2 * ph) * 28 + 2 * pw;
  float in[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) in[r][c] = img[r * 28 + c];
  const int co = cg * 4;
  float best[4];
  unsigned arg[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int dy = q >> 1, dx = q & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) acc = fmaf(in[dy + kh][dx + kw], sw[(kh * 3 + kw) * 32 + co + j], acc);
      if (q == 0 || acc > best[j]) { best[j] = acc; arg[j] = q; }
    }
  }
  f4 o;
  o.x = fmaxf(best[0] + sw[288 + co + 0], 0.f);
  o.y = fmaxf(best[1] + sw[288 + co + 1], 0.f);
  o.z = fmaxf(best[2] + sw[288 + co + 2], 0.f);
  o.w = fmaxf(best[3] + sw[288 + co + 3], 0.f);
  st4(a.P1 + (size_t)pix * 32 + co, o);
  *reinterpret_cast<unsigned*>(a.A1 + (size_t)pix * 32 + co) =
      arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
}

// --------------------------------------------------------------------------------------------
// K2: conv2 + bias + relu + maxpool on MFMA.  Workgroup = 4 waves = one 16-row tile (4 pool
// windows x 4 positions) x 4 column tiles of 16 output channels.  K = 9 taps x 32 ci.
// Lane group g owns k-slot g; each lane loads 4 consecutive ci (float4) and feeds them to 4
// successive MFMAs, so the same permuted k order is used for A and B.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_conv2_pool(MnistArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int n0 = wave * 16;
  const int npp = a.b * 25;
  const int pp = blockIdx.x * 4 + (i >> 2), q = i & 3;
  const bool valid = pp < npp;
  const int ppc = valid ? pp : 0;
  const int bi = ppc / 25, r = ppc - bi * 25, ph = r / 5, pw = r - ph * 5;
  const int oh = 2 * ph + (q >> 1), ow = 2 * pw + (q & 1);
  const float* abase = a.P1 + ((size_t)(bi * 13 + oh) * 13 + ow) * 32 + 4 * g;
  const float* bbase = a.W + a.ow2 + (4 * g) * 64 + n0 + i;
  // Issue every load of the wave up front (18 k-steps x (float4 A + 4 B) = 144 VGPRs) so the
  // whole K loop costs one memory round trip; the MFMAs then drain them in order.
  f4 av[18];
  float bv[18][4];
#pragma unroll
  for (int s = 0; s < 18; ++s) {
    const int kk = s >> 1, cb = (s & 1) * 16, kh = kk / 3, kw = kk % 3;
    av[s] = ld4(abase + (kh * 13 + kw) * 32 + cb);
    const float* bp = bbase + (kk * 32 + cb) * 64;
#pragma unroll
    for (int t = 0; t < 4; ++t) bv[s][t] = bp[t * 64];
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every load above the MFMAs (one round trip)
  f4 acc0 = zero4(), acc1 = zero4();
  const float vm = valid ? 1.f : 0.f;
#pragma unroll
  for (int s = 0; s < 18; ++s) {
    const f4 x = av[s] * vm;
    acc0 = mfma16x16x4(x.x, bv[s][0], acc0);
    acc1 = mfma16x16x4(x.y, bv[s][1], acc1);
    acc0 = mfma16x16x4(x.z, bv[s][2], acc0);
    acc1 = mfma16x16x4(x.w, bv[s][3], acc1);
  }
  const f4 acc = acc0 + acc1;
  // lane holds rows 4g..4g+3 == the 4 positions of pool window g, column n0+i.
  const int ppo = blockIdx.x * 4 + g;
  if (ppo < npp) {
    float m = acc.x;
    unsigned am = 0;
    if (acc.y > m) { m = acc.y; am = 1; }
    if (acc.z > m) { m = acc.z; am = 2; }
    if (acc.w > m) { m = acc.w; am = 3; }
    const int co = n0 + i;
    a.P2[(size_t)ppo * 64 + co] = fmaxf(m + a.W[a.ob2 + co], 0.f);
    a.A2[(size_t)ppo * 64 + co] = (uint8_t)am;
  }
}

// --------------------------------------------------------------------------------------------
// K3: H = relu(P2 W3 + b3).  grid (ceil(b/16), 8); 8 waves split K=1600 (100 chunks of 16).
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void k_dense1(MnistArgs a) {
  __shared__ float red[8][256];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int mt = blockIdx.x, nt = blockIdx.y;
  const int row = mt * 16 + i;
  const bool valid = row < a.b;
  const float* ap = a.P2 + (size_t)(valid ? row : 0) * 1600 + 4 * g;
  const float* bp = a.W + a.ow3 + (4 * g) * 128 + nt * 16 + i;
  // 13 k-chunks per wave (chunk c = wave + 8j < 100), all loads issued before the MFMAs.
  f4 av[13];
  float bv[13][4];
#pragma unroll
  for (int j = 0; j < 13; ++j) {
    const int c = min(wave + 8 * j, 99), k0 = c * 16;
    av[j] = ld4(ap + k0);
    const float* b = bp + k0 * 128;
#pragma unroll
    for (int t = 0; t < 4; ++t) bv[j][t] = b[t * 128];
  }
  __builtin_amdgcn_sched_barrier(0);
  f4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
  for (int j = 0; j < 13; ++j) {
    const float m = (valid && wave + 8 * j < 100) ? 1.f : 0.f;
    const f4 x = av[j] * m;
    acc0 = mfma16x16x4(x.x, bv[j][0], acc0);
    acc1 = mfma16x16x4(x.y, bv[j][1], acc1);
    acc0 = mfma16x16x4(x.z, bv[j][2], acc0);
    acc1 = mfma16x16x4(x.w, bv[j][3], acc1);
  }
  const f4 acc = acc0 + acc1;
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][(4 * g + r) * 16 + i] = acc[r];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int o = threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[w][o];
    const int rr = mt * 16 + (o >> 4), cc = nt * 16 + (o & 15);
    if (rr < a.b) a.H[rr * 128 + cc] = fmaxf(s + a.W[a.ob3 + cc], 0.f);
  }
}

// --------------------------------------------------------------------------------------------
// K4: dense2 + sparse softmax cross-entropy + metrics + dense2 grads + dH.  One workgroup.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_head(MnistArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = a.b, tid = threadIdx.x;
  float* sH = sm;                 // b*128
  float* sW = sH + b * 128;       // 1280
  float* sB = sW + 1280;          // 16
  float* sD = sB + 16;            // b*16 logits -> dlogits
  float* sRed = sD + b * 16;      // 64
  // every LDS-latency chain below is split over 4 independent accumulators and unrolled, so
  // the single workgroup is issue-bound rather than LDS-latency-bound.
  for (int o = tid; o < b * 32; o += 1024) st4(sH + o * 4, ld4(a.H + o * 4));
  for (int o = tid; o < 1280; o += 1024) sW[o] = a.W[a.ow4 + o];
  if (tid < 10) sB[tid] = a.W[a.ob4 + tid];
  const int yl = (tid < b) ? a.Y[a.idx[tid]] : 0;  // prefetch labels (b <= 1024 rows per pass)
  __syncthreads();
  for (int o = tid; o < b * 10; o += 1024) {
    const int r = o / 10, c = o - r * 10;
    const f4* h4 = reinterpret_cast<const f4*>(sH + r * 128);
    float s0 = sB[c], s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 8
    for (int k4 = 0; k4 < 32; ++k4) {
      const f4 h = h4[k4];
      const float* w = sW + k4 * 40 + c;
      s0 = fmaf(h.x, w[0], s0);
      s1 = fmaf(h.y, w[10], s1);
      s2 = fmaf(h.z, w[20], s2);
      s3 = fmaf(h.w, w[30], s3);
    }
    sD[r * 16 + c] = (s0 + s1) + (s2 + s3);
  }
  __syncthreads();
  float lsum = 0.f, lcor = 0.f;
  for (int r = tid; r < b; r += 1024) {
    float* l = sD + r * 16;
    const int y = (r < 1024 && r == tid) ? yl : a.Y[a.idx[r]];
    float v[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) v[c] = l[c];
    float m = v[0];
    int am = 0;
#pragma unroll
    for (int c = 1; c < 10; ++c)
      if (v[c] > m) { m = v[c]; am = c; }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) se += expf(v[c] - m);
    const float lse = m + logf(se);
    float ly = v[0];
#pragma unroll
    for (int c = 1; c < 10; ++c) ly = (c == y) ? v[c] : ly;
    lsum += lse - ly;
    lcor += (am == y) ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) l[c] = (expf(v[c] - lse) - (c == y ? 1.f : 0.f)) * a.scale;
  }
  lsum = wave_sum(lsum);
  lcor = wave_sum(lcor);
  if ((tid & 63) == 0) { sRed[tid >> 6] = lsum; sRed[32 + (tid >> 6)] = lcor; }
  __syncthreads();
  if (tid == 0) {
    float s = 0.f, c = 0.f;
    for (int w = 0; w < 16; ++w) { s += sRed[w]; c += sRed[32 + w]; }
    a.metrics[0] += s;
    a.metrics[1] += c;
    a.metrics[2] += (float)b;
  }
  // dW4 (1280) and db4 (10): sum over rows, 4 accumulators
  for (int o = tid; o < 1290; o += 1024) {
    const bool bias = o >= 1280;
    const int k = bias ? 0 : o / 10, c = bias ? o - 1280 : o - (o / 10) * 10;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int r = 0;
    for (; r + 3 < b; r += 4) {
      const float h0 = bias ? 1.f : sH[r * 128 + k], h1 = bias ? 1.f : sH[(r + 1) * 128 + k];
      const float h2 = bias ? 1.f : sH[(r + 2) * 128 + k], h3 = bias ? 1.f : sH[(r + 3) * 128 + k];
      s0 = fmaf(h0, sD[r * 16 + c], s0);
      s1 = fmaf(h1, sD[(r + 1) * 16 + c], s1);
      s2 = fmaf(h2, sD[(r + 2) * 16 + c], s2);
      s3 = fmaf(h3, sD[(r + 3) * 16 + c], s3);
    }
    for (; r < b; ++r) s0 = fmaf(bias ? 1.f : sH[r * 128 + k], sD[r * 16 + c], s0);
    a.G[(bias ? a.ob4 : a.ow4) + (bias ? c : o)] = (s0 + s1) + (s2 + s3);
  }
  for (int o = tid; o < b * 128; o += 1024) {
    const int r = o >> 7, k = o & 127;
    const float h = sH[o];
    const f4 d0 = ld4(sD + r * 16), d1 = ld4(sD + r * 16 + 4);
    const float* w = sW + k * 10;
    float s = d0.x * w[0];
    s = fmaf(d0.y, w[1], s); s = fmaf(d0.z, w[2], s); s = fmaf(d0.w, w[3], s);
    s = fmaf(d1.x, w[4], s); s = fmaf(d1.y, w[5], s); s = fmaf(d1.z, w[6], s); s = fmaf(d1.w, w[7], s);
    s = fmaf(sD[r * 16 + 8], w[8], s); s = fmaf(sD[r * 16 + 9], w[9], s);
    a.dH[o] = h > 0.f ? s : 0.f;
  }
}

// --------------------------------------------------------------------------------------------
// K5: dense1 backward.  blocks [0,200): dW3 tiles; [200, 200+nP): dP2 tiles with the pool2 /
// relu backward scatter into dC2; last block: db3.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dense1_bwd(MnistArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int b = a.b;
  const int MT = (b + 15) >> 4;
  const int nP = (MT * 100 + 3) >> 2;
  const int blk = blockIdx.x;
  if (blk < 200) {
    // dW3[k][n] = sum_r P2[r][k] dH[r][n]   (M = 1600 features, N = 128, K = b)
    const int T = blk * 4 + wave, mt = T >> 3, nt = T & 7;
    const int kf = mt * 16 + i, n = nt * 16 + i;
    // rows in batches of 64 (16 MFMA k-steps); all 32 loads of a batch in flight together.
    f4 acc0 = zero4(), acc1 = zero4();
    for (int r0 = 0; r0 < b; r0 += 64) {
      float av[16], bv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int rr = min(r0 + 4 * s + g, b - 1);
        av[s] = a.P2[(size_t)rr * 1600 + kf];
        bv[s] = a.dH[rr * 128 + n];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float x = (r0 + 4 * s + g < b) ? av[s] : 0.f;
        if (s & 1) acc1 = mfma16x16x4(x, bv[s], acc1);
        else acc0 = mfma16x16x4(x, bv[s], acc0);
      }
    }
    const f4 acc = acc0 + acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r) a.G[a.ow3 + (mt * 16 + 4 * g + r) * 128 + nt * 16 + i] = acc[r];
  } else if (blk < 200 + nP) {
    // dP2[r][k] = sum_n dH[r][n] W3[k][n]  (M = b, N = 1600, K = 128)
    const int T = (blk - 200) * 4 + wave;
    if (T >= MT * 100) return;
    const int mt = T % MT, nt = T / MT;
    const int row = mt * 16 + i;
    const bool valid = row < b;
    const float* ap = a.dH + (valid ? row : 0) * 128 + 4 * g;
    const float* bp = a.W + a.ow3 + (size_t)(nt * 16 + i) * 128 + 4 * g;
    f4 av[8], bv[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      av[s] = ld4(ap + s * 16);
      bv[s] = ld4(bp + s * 16);
    }
    __builtin_amdgcn_sched_barrier(0);
    const float vm = valid ? 1.f : 0.f;
    f4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const f4 x = av[s] * vm;
      acc0 = mfma16x16x4(x.x, bv[s].x, acc0);
      acc1 = mfma16x16x4(x.y, bv[s].y, acc1);
      acc0 = mfma16x16x4(x.z, bv[s].z, acc0);
      acc1 = mfma16x16x4(x.w, bv[s].w, acc1);
    }
    const f4 acc = acc0 + acc1;
    const int k = nt * 16 + i, pp = k >> 6, co = k & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = mt * 16 + 4 * g + r;
      if (rr < b) {
        const size_t e = (size_t)rr * 1600 + k;
        const float v = a.P2[e] > 0.f ? acc[r] : 0.f;
        const unsigned qa = a.A2[e];
        float* d = a.dC2 + ((size_t)(rr * 25 + pp) * 4) * 64 + co;
        d[0] = qa == 0 ? v : 0.f;
        d[64] = qa == 1 ? v : 0.f;
        d[128] = qa == 2 ? v : 0.f;
        d[192] = qa == 3 ? v : 0.f;
      }
    }
  } else {
    if (threadIdx.x < 128) {
      float s = 0.f;
      for (int r = 0; r < b; ++r) s += a.dH[r * 128 + threadIdx.x];
      a.G[a.ob3 + threadIdx.x] = s;
    }
  }
}

// --------------------------------------------------------------------------------------------
// K6: conv2 weight gradient.  M = 288 (+16 bias rows) = 19 tiles, N = 64 = 4 tiles,
// K = b*25 pool windows x 4 positions; one MFMA k-step == one pool window (k-slot g == dy*2+dx).
// grid = 76 tiles x 4 splits; each of the 4 waves takes 1/16 of the windows; the 4 waves of a
// block reduce through LDS and the 4 splits are summed (deterministically) by K9.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_conv2_wgrad(MnistArgs a) {
  __shared__ float red[4][256];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x >> 2, split = blockIdx.x & 3;
  const int mt = tile >> 2, nt = tile & 3;
  const int slice = split * 4 + wave;
  const int NW = a.b * 25;
  const int chunk = (NW + 15) / 16;
  const int w0 = slice * chunk, w1 = min(NW, w0 + chunk);
  const bool bias_tile = mt == 18;
  const int k = mt * 16 + i;
  const int kk9 = bias_tile ? 0 : (k >> 5), ci = k & 31;
  const int kh = kk9 / 3, kw = kk9 - kh * 3;
  const int dy = g >> 1, dx = g & 1;
  const float* pa = a.P1 + ((dy + kh) * 13 + (dx + kw)) * 32 + ci;
  const float* pb = a.dC2 + g * 64 + nt * 16 + i;
  const float one = (i == 0) ? 1.f : 0.f;
  // windows in batches of 16, double-buffered: batch j+1's 32 loads are in flight while the
  // MFMAs of batch j run.
  f4 acc0 = zero4(), acc1 = zero4();
  float ca[16], cb[16], na[16], nb[16];
  auto load = [&](int base, float (&ra)[16], float (&rb)[16]) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int w = min(base + s, w1 - 1);
      const int bi0 = w / 25, pp0 = w - bi0 * 25, ph0 = pp0 / 5, pw0 = pp0 - ph0 * 5;
      ra[s] = pa[((bi0 * 13 + 2 * ph0) * 13 + 2 * pw0) * 32];
      rb[s] = pb[(size_t)w * 256];
    }
  };
  auto comp = [&](int base, const float (&ra)[16], const float (&rb)[16]) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float x = (base + s < w1) ? (bias_tile ? one : ra[s]) : 0.f;
      if (s & 1) acc1 = mfma16x16x4(x, rb[s], acc1);
      else acc0 = mfma16x16x4(x, rb[s], acc0);
    }
  };
  if (w0 < w1) {
    load(w0, ca, cb);
    int base = w0;
    while (true) {
      const int nxt = base + 16;
      if (nxt < w1) load(nxt, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      comp(base, ca, cb);
      __builtin_amdgcn_sched_barrier(0);
      if (nxt >= w1) break;
      const int nn = nxt + 16;
      if (nn < w1) load(nn, ca, cb);
      __builtin_amdgcn_sched_barrier(0);
      comp(nxt, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      if (nn >= w1) break;
      base = nn;
    }
  }
  const f4 acc = acc0 + acc1;
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][(4 * g + r) * 16 + i] = acc[r];
  __syncthreads();
  const int o = threadIdx.x;
  const float s = red[0][o] + red[1][o] + red[2][o] + red[3][o];
  const int row = mt * 16 + (o >> 4), col = nt * 16 + (o & 15);
  a.part2[((size_t)split * kMnistPart2Rows + row) * 64 + col] = s;
}

// --------------------------------------------------------------------------------------------
// K7: conv2 data gradient on MFMA (M = b*169 pooled-conv1 pixels, N = 32, K = 9 x 64) with the
// pool1 + relu backward and the conv1 weight/bias gradient fused into the epilogue.
// Workgroup = 8 waves = 4 row tiles x 2 column tiles = 64 pixels x 32 channels.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void k_conv2_dgrad(MnistArgs a) {
  __shared__ float red[8][10][16];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int rt = wave & 3, ct = wave >> 2;
  const int npix = a.b * 169;
  const int P = blockIdx.x * 64 + rt * 16 + i;
  const bool valid = P < npix;
  const int Pc = valid ? P : 0;
  const int bi = Pc / 169, rem = Pc - bi * 169, ih = rem / 13, iw = rem - ih * 13;
  const float* w2 = a.W + a.ow2 + (size_t)(ct * 16 + i) * 64 + 4 * g;
  f4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
  for (int kk = 0; kk < 9; ++kk) {
    const int kh = kk / 3, kw = kk % 3;
    const int oh = ih - kh, ow = iw - kw;
    const bool rv = valid && oh >= 0 && oh < 10 && ow >= 0 && ow < 10;
    const int ohc = rv ? oh : 0, owc = rv ? ow : 0;
    const float* ap = a.dC2 + ((size_t)((bi * 25 + (ohc >> 1) * 5 + (owc >> 1)) * 4 + (ohc & 1) * 2 + (owc & 1))) * 64 + 4 * g;
    const float* bp = w2 + kk * 32 * 64;
    const float m = rv ? 1.f : 0.f;
#pragma unroll
    for (int c0 = 0; c0 < 64; c0 += 16) {
      const f4 av = ld4(ap + c0) * m;
      const f4 bv = ld4(bp + c0);
      acc0 = mfma16x16x4(av.x, bv.x, acc0);
      acc1 = mfma16x16x4(av.y, bv.y, acc1);
      acc0 = mfma16x16x4(av.z, bv.z, acc0);
      acc1 = mfma16x16x4(av.w, bv.w, acc1);
    }
  }
  const f4 acc = acc0 + acc1;
  // epilogue: lane holds dP1 for pixels P_r = base + 4g + r, channel c.
  const int c = ct * 16 + i;
  float dw[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) dw[j] = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int Pr = blockIdx.x * 64 + rt * 16 + 4 * g + r;
    if (Pr < npix) {
      const size_t e = (size_t)Pr * 32 + c;
      const float v = a.P1[e] > 0.f ? acc[r] : 0.f;
      const unsigned q1 = a.A1[e];
      const int br = Pr / 169, rr = Pr - br * 169, ph = rr / 13, pw = rr - ph * 13;
      const int y = 2 * ph + (q1 >> 1), x = 2 * pw + (q1 & 1);
      const float* img = a.X + (size_t)a.idx[br] * 784 + y * 28 + x;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) dw[kh * 3 + kw] = fmaf(img[kh * 28 + kw], v, dw[kh * 3 + kw]);
      dw[9] += v;
    }
  }
#pragma unroll
  for (int j = 0; j < 10; ++j) dw[j] = sum_lane_groups(dw[j]);
  if (g == 0) {
#pragma unroll
    for (int j = 0; j < 10; ++j) red[wave][j][i] = dw[j];
  }
  __syncthreads();
  if (threadIdx.x < 320) {
    const int j = threadIdx.x >> 5, cc = threadIdx.x & 31;
    const int ctt = cc >> 4, ii = cc & 15;
    const float s = red[ctt * 4 + 0][j][ii] + red[ctt * 4 + 1][j][ii] + red[ctt * 4 + 2][j][ii] +
                    red[ctt * 4 + 3][j][ii];
    a.part1[(size_t)blockIdx.x * kMnistPart1Cols + j * 32 + cc] = s;
  }
}

// --------------------------------------------------------------------------------------------
// K9: reduce partial slabs into G (+ optional fused SGD).  Blocks [0, nbs) sweep the slab,
// blocks [nbs, nbs+20) reduce the conv1 partials (16 outputs per block).
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finalize(MnistArgs a, int apply_sgd, int nbs) {
  const float lr = *a.lr;
  if ((int)blockIdx.x < nbs) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= a.nslab) return;
    if ((e >= a.ow1 && e < a.ow1 + 288) || (e >= a.ob1 && e < a.ob1 + 32)) return;
    float gv;
    if (e >= a.ow2 && e < a.ow2 + 18432) {
      const int k = e - a.ow2;
      gv = 0.f;
#pragma unroll
      for (int s = 0; s < kMnistConv2Splits; ++s) gv += a.part2[(size_t)s * kMnistPart2Rows * 64 + k];
      a.G[e] = gv;
    } else if (e >= a.ob2 && e < a.ob2 + 64) {
      const int co = e - a.ob2;
      gv = 0.f;
#pragma unroll
      for (int s = 0; s < kMnistConv2Splits; ++s) gv += a.part2[((size_t)s * kMnistPart2Rows + 288) * 64 + co];
      a.G[e] = gv;
    } else {
      gv = a.G[e];
    }
    if (apply_sgd) a.W[e] -= lr * gv;
    return;
  }
  __shared__ float red[256];
  const int ob = (blockIdx.x - nbs) * 16;
  const int o = ob + (threadIdx.x & 15), u = threadIdx.x >> 4;
  const int nb7 = mnist_nb7(a.b);
  float s = 0.f;
  for (int p = u; p < nb7; p += 16) s += a.part1[(size_t)p * kMnistPart1Cols + o];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) t += red[v * 16 + threadIdx.x];
    const int e = (o < 288) ? a.ow1 + o : a.ob1 + (o - 288);
    a.G[e] = t;
    if (apply_sgd) a.W[e] -= lr * t;
  }
}

// --------------------------------------------------------------------------------------------
// Optimizer kernels over flat slabs.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sgd(float* __restrict__ w, const float* __restrict__ g,
                                             const float* __restrict__ lrp, int64_t n) {
  const float lr = *lrp;
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    f4 wv = ld4(w + i4);
    const f4 gv = ld4(g + i4);
    wv -= lr * gv;
    st4(w + i4, wv);
  } else {
    for (int64_t j = i4; j < n; ++j) w[j] -= lr * g[j];
  }
}

__global__ __launch_bounds__(256) void k_sgd_momentum(float* __restrict__ w, const float* __restrict__ g,
                                                      float* __restrict__ v, const float* __restrict__ lrp,
                                                      float m, int nesterov, int64_t n) {
  const float lr = *lrp;
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    f4 wv = ld4(w + i4), vv = ld4(v + i4);
    const f4 gv = ld4(g + i4);
    vv = m * vv - lr * gv;
    wv += nesterov ? (m * vv - lr * gv) : vv;
    st4(w + i4, wv);
    st4(v + i4, vv);
  } else {
    for (int64_t j = i4; j < n; ++j) {
      const float vj = m * v[j] - lr * g[j];
      v[j] = vj;
      w[j] += nesterov ? (m * vj - lr * g[j]) : vj;
    }
  }
}

// --------------------------------------------------------------------------------------------
// launchers
// --------------------------------------------------------------------------------------------
void mnist_conv1_pool(const MnistArgs& a, hipStream_t s) {
  const int n = a.b * 169 * 8;
  hipLaunchKernelGGL(k_conv1_pool, dim3((n + 255) / 256), dim3(256), 0, s, a);
}
void mnist_conv2_pool(const MnistArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_conv2_pool, dim3((a.b * 25 + 3) / 4), dim3(256), 0, s, a);
}
void mnist_dense1(const MnistArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_dense1, dim3((a.b + 15) / 16, 8), dim3(512), 0, s, a);
}
void mnist_head(const MnistArgs& a, hipStream_t s) {
  const size_t lds = (size_t)(a.b * 128 + 1280 + 16 + a.b * 16 + 64) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_head, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(k_head, dim3(1), dim3(1024), lds, s, a);
}
void mnist_dense1_bwd(const MnistArgs& a, hipStream_t s) {
  const int MT = (a.b + 15) / 16;
  const int nP = (MT * 100 + 3) / 4;
  hipLaunchKernelGGL(k_dense1_bwd, dim3(200 + nP + 1), dim3(256), 0, s, a);
}
void mnist_conv2_wgrad(const MnistArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_conv2_wgrad, dim3(19 * 4 * kMnistConv2Splits), dim3(256), 0, s, a);
}
void mnist_conv2_dgrad(const MnistArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_conv2_dgrad, dim3(mnist_nb7(a.b)), dim3(512), 0, s, a);
}
void mnist_finalize(const MnistArgs& a, bool apply_sgd, hipStream_t s) {
  const int nbs = (a.nslab + 255) / 256;
  hipLaunchKernelGGL(k_finalize, dim3(nbs + 20), dim3(256), 0, s, a, apply_sgd ? 1 : 0, nbs);
}
void sgd_apply(float* w, const float* g, const float* lr, int64_t n, hipStream_t s) {
  const int64_t nt = (n + 3) / 4;
  hipLaunchKernelGGL(k_sgd, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, w, g, lr, n);
}
void sgd_momentum_apply(float* w, const float* g, float* v, const float* lr, float momentum, bool nesterov,
                        int64_t n, hipStream_t s) {
  const int64_t nt = (n + 3) / 4;
  hipLaunchKernelGGL(k_sgd_momentum, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, w, g, v, lr, momentum,
                     nesterov ? 1 : 0, n);
}

}  // namespace tdl
