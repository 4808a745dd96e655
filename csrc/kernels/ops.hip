// Generic data-movement kernels: device-resident dataset batch gather (SURVEY.md §3.2 target:
// zero H2D traffic in the hot loop).  One workgroup per gathered row, 16-byte vector accesses.
#include "common.h"
#include "ops.h"

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

}  // namespace tdl
