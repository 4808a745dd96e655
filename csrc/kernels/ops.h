// Host-visible interface of the generic (shape-agnostic) HIP ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

// out[r, :] = src[idx[r], :] * scale   (row gather of a device-resident dataset; f32 rows)
void gather_xy(const float* src, const void* lab, const int* idx, float* out, void* out_lab, int64_t rows,
               int64_t row_elems, int lab_bytes, hipStream_t s);
void gather_rows_f32(const float* src, const int* idx, float* out, int64_t rows, int64_t row_elems, float scale,
                     hipStream_t s);
// out[r, :] = float(src[idx[r], :]) * scale   (uint8 images -> f32, the reference's map(scale))
void gather_rows_u8(const uint8_t* src, const int* idx, float* out, int64_t rows, int64_t row_elems, float scale,
                    hipStream_t s);
// out[r] = src[idx[r]]   (labels)
void gather_i32(const int* src, const int* idx, int* out, int64_t rows, hipStream_t s);

// Weight-slab cast with transposes: for every 64 x 64 tile listed in `tiles` (int4: entry, row
// tile, column tile, unused) of every entry e (int4 in `entries`: src offset, dst offset, R, K),
// dst[e.dst + k * R + r] = bf16(src[e.src + r * K + k]) -- HWIO [R = KH*KW*C][K] f32 conv kernels
// into the OHWI bf16 rows the implicit-GEMM forward reads, for all convs of a model in one launch.
void slab_transpose_bf16(const float* src, uint16_t* dst, const int* entries, const int* tiles, int ntiles,
                         hipStream_t s);

// dst = bf16(src) (round to nearest even), n % 8 == 0 (the trainer's whole-slab compute copy)
void cast_bf16(const float* src, uint16_t* dst, long long n, hipStream_t s);

}  // namespace tdl
