// Generic data-movement kernels: device-resident dataset batch gather (SURVEY.md §3.2 target:
// zero H2D traffic in the hot loop).  One workgroup per gathered row, 16-byte vector accesses.
#include "common.h"
#include "ops.h"

#include <algorithm>

namespace tdl {

__global__ __launch_bounds__(256) void k_gather_rows_f32(const float* __restrict__ src, const int* __restrict__ idx,
                                                         float* __restrict__ out, int64_t row_elems, float scale) {
  const int64_t r = blockIdx.x;
  const float* s = src + (int64_t)idx[r] * row_elems;
  float* o = out + r * row_elems;
  if ((row_elems & 3) == 0) {
    for (int64_t e = threadIdx.x * 4; e < row_elems; e += 1024) st4(o + e, ld4(s + e) * scale);
  } else {
    for (int64_t e = threadIdx.x; e < row_elems; e += 256) o[e] = s[e] * scale;
  }
}

__global__ __launch_bounds__(256) void k_gather_rows_u8(const uint8_t* __restrict__ src, const int* __restrict__ idx,
                                                        float* __restrict__ out, int64_t row_elems, float scale) {
  const int64_t r = blockIdx.x;
  const uint8_t* s = src + (int64_t)idx[r] * row_elems;
  float* o = out + r * row_elems;
  if ((row_elems & 3) == 0 && ((uintptr_t)s & 3) == 0) {
    for (int64_t e = threadIdx.x * 4; e < row_elems; e += 1024) {
      const unsigned v = *reinterpret_cast<const unsigned*>(s + e);
      st4(o + e, f4{(float)(v & 255), (float)((v >> 8) & 255), (float)((v >> 16) & 255), (float)(v >> 24)} * scale);
    }
  } else {
    for (int64_t e = threadIdx.x; e < row_elems; e += 256) o[e] = (float)s[e] * scale;
  }
}

__global__ __launch_bounds__(256) void k_gather_i32(const int* __restrict__ src, const int* __restrict__ idx,
                                                    int* __restrict__ out, int64_t rows) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < rows) out[r] = src[idx[r]];
}

// a batch of (f32 feature row, label) pairs of a device-resident dataset in ONE launch (the generic
// engine's device input path): workgroup r copies row idx[r] and its thread 0 the label (4 or 8 bytes)
__global__ __launch_bounds__(256) void k_gather_xy(const float* __restrict__ src, const void* __restrict__ lab,
                                                   const int* __restrict__ idx, float* __restrict__ out,
                                                   void* __restrict__ out_lab, int64_t row_elems, int lab_bytes) {
  const int64_t r = blockIdx.x;
  const int64_t i = idx[r];
  const float* s = src + i * row_elems;
  float* o = out + r * row_elems;
  if ((row_elems & 3) == 0) {
    for (int64_t e = threadIdx.x * 4; e < row_elems; e += 1024) st4(o + e, ld4(s + e));
  } else {
    for (int64_t e = threadIdx.x; e < row_elems; e += 256) o[e] = s[e];
  }
  if (threadIdx.x == 0) {
    if (lab_bytes == 8)
      static_cast<long long*>(out_lab)[r] = static_cast<const long long*>(lab)[i];
    else
      static_cast<int*>(out_lab)[r] = static_cast<const int*>(lab)[i];
  }
}

void gather_xy(const float* src, const void* lab, const int* idx, float* out, void* out_lab, int64_t rows,
               int64_t row_elems, int lab_bytes, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL(k_gather_xy, dim3((unsigned)rows), dim3(256), 0, s, src, lab, idx, out, out_lab, row_elems,
                     lab_bytes);
}

void gather_rows_f32(const float* src, const int* idx, float* out, int64_t rows, int64_t row_elems, float scale,
                     hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL(k_gather_rows_f32, dim3((unsigned)rows), dim3(256), 0, s, src, idx, out, row_elems, scale);
}
void gather_rows_u8(const uint8_t* src, const int* idx, float* out, int64_t rows, int64_t row_elems, float scale,
                    hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL(k_gather_rows_u8, dim3((unsigned)rows), dim3(256), 0, s, src, idx, out, row_elems, scale);
}
void gather_i32(const int* src, const int* idx, int* out, int64_t rows, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL(k_gather_i32, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, src, idx, out, rows);
}

namespace {

__global__ __launch_bounds__(256) void k_slab_transpose_bf16(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                            const int4* __restrict__ entries,
                                                            const int4* __restrict__ tiles) {
  __shared__ float t[64][65];
  const int4 tl = tiles[blockIdx.x];
  const int4 e = entries[tl.x];
  const int R = e.z, K = e.w, r0 = tl.y * 64, k0 = tl.z * 64;
  const int tid = threadIdx.x;
  // read 64 rows (r) x 64 columns (k): thread -> column k0 + (tid & 63), rows (tid >> 6) + 4 i
  const int kc = tid & 63;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = (tid >> 6) + 4 * i;
    t[r][kc] = (r0 + r < R && k0 + kc < K) ? src[(long long)e.x + (long long)(r0 + r) * K + k0 + kc] : 0.f;
  }
  __syncthreads();
  // write 64 rows (k) x 64 columns (r): thread -> r column r0 + (tid & 63), k rows (tid >> 6) + 4 i
  const int rc = tid & 63;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = (tid >> 6) + 4 * i;
    if (k0 + k < K && r0 + rc < R) {
      uint32_t u = __float_as_uint(t[rc][k]);
      u += 0x7fffu + ((u >> 16) & 1u);
      dst[(long long)e.y + (long long)(k0 + k) * R + r0 + rc] = (uint16_t)(u >> 16);
    }
  }
}

}  // namespace

void slab_transpose_bf16(const float* src, uint16_t* dst, const int* entries, const int* tiles, int ntiles,
                         hipStream_t s) {
  if (ntiles <= 0) return;
  hipLaunchKernelGGL(k_slab_transpose_bf16, dim3(ntiles), dim3(256), 0, s, src, dst,
                     reinterpret_cast<const int4*>(entries), reinterpret_cast<const int4*>(tiles));
}

namespace {

// dst[i] = bf16(src[i]), 8 elements (two 16-B loads, one 16-B store) per thread per iteration
__global__ __launch_bounds__(256) void k_cast_bf16(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                  long long n8) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long v = (long long)blockIdx.x * 256 + threadIdx.x; v < n8; v += stride) {
    const f4 a = reinterpret_cast<const f4*>(src)[2 * v], b = reinterpret_cast<const f4*>(src)[2 * v + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t lo = __float_as_uint(f[2 * j]), hi = __float_as_uint(f[2 * j + 1]);
      lo += 0x7fffu + ((lo >> 16) & 1u);
      hi += 0x7fffu + ((hi >> 16) & 1u);
      o[j] = (lo >> 16) | (hi & 0xffff0000u);
    }
    reinterpret_cast<uint4*>(dst)[v] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

void cast_bf16(const float* src, uint16_t* dst, long long n, hipStream_t s) {
  const long long n8 = n / 8;
  if (n8 > 0) {
    const long long blocks = std::min<long long>((n8 + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(k_cast_bf16, dim3((unsigned)blocks), dim3(256), 0, s, src, dst, n8);
  }
}

}  // namespace tdl
