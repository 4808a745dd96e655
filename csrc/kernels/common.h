// Shared device helpers for the gfx950 (CDNA4) kernels of this framework.
//
// Everything here is written for 64-lane wavefronts and the f32-input MFMA
// instructions of gfx950 (v_mfma_f32_16x16x4_f32: exact f32, one f32 A and one
// f32 B value per lane, four f32 accumulators per lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// D(16x16) += A(16x4) * B(4x16), f32 in / f32 accumulate.
// Lane l supplies A[l & 15][l >> 4] and B[l >> 4][l & 15];
// lane l receives D[(l >> 4) * 4 + r][l & 15] in acc[r].
__device__ __forceinline__ f4 mfma16x16x4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// two f32 -> packed bf16 (lo in bits 0-15), round to nearest even: one v_cvt_pk_bf16_f32 (the same bits
// as the integer RNE `u + 0x7fff + lsb` sequence for finite values, at a fraction of its VALU cost)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_t{lo, hi}, b2_t));
}

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// Raw buffer resource over [base, base + bytes) (gfx9-family dword3 0x00020000).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// 16-B load through a raw buffer resource: byte offset = voffset (per lane) + soffset (SGPR, e.g. a
// compile-time stride) -- no 64-bit address arithmetic on the VALU per load
__device__ __forceinline__ f4 ld4_buf(__amdgpu_buffer_rsrc_t r, int voffset, int soffset) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voffset, soffset, 0));
}

// 4-B load through a raw buffer resource (offsets past the resource's size read 0)
__device__ __forceinline__ float ld1_buf(__amdgpu_buffer_rsrc_t r, int voffset, int soffset) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voffset, soffset, 0));
}

// LDS-DMA: one 16-B chunk per lane from a raw buffer straight into LDS (buffer_load_dwordx4 ... lds).
// The 64 lanes of the wave write 1 KiB linearly from `wave_dst` (wave-uniform): lane L lands at
// wave_dst + 16 L bytes.  Out-of-range voffsets (e.g. 0x80000000) land zeros.
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, uint16_t* wave_dst, int voffset, int soffset) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)wave_dst, 16, voffset,
                                           soffset, 0, 0);
}

// 16-byte WRITE-THROUGH (sc1, aux 16) store: the bytes reach memory past this XCD's L2, so a
// consumer workgroup on any XCD reads them with sc1 loads after the producer's vmcnt(0) drain and
// an agent-scope counter/flag (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void st4_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, f4 v) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, byte_off, 0, 16);
}

// Workgroup barrier for LDS data only: waits for this wave's LDS operations, not for its global
// loads still in flight (__syncthreads() also drains vmcnt, i.e. waits for every outstanding
// global load of the wave -- e.g. operand prefetches meant to overlap the next phase).  The
// memory clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---- cross-lane exchanges on the VALU (gfx950 v_permlane{16,32}_swap, DPP) instead of
// ds_bpermute (__shfl_xor), which goes through the LDS pipe with its latency ----
// Reduce-scatter step across the 16-lane row pairs (lane l <-> l ^ 16): a lane in an even row
// returns lo(l) + lo(l ^ 16), a lane in an odd row hi(l) + hi(l ^ 16).  v_permlane16_swap swaps the
// odd rows of its first operand with the even rows of its second, which leaves exactly those two
// addends in the two results.
__device__ __forceinline__ float rs_swap16(float lo, float hi) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// the same across the wave halves (lane l <-> l ^ 32)
__device__ __forceinline__ float rs_swap32(float lo, float hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// DPP partner values within a 16-lane row: xor 8 (row_ror:8), the 8-lane half mirror (l <-> 7 - l:
// pairs each lane of a 4-lane half with one of the other half, as xor 4 does), xor 2 / xor 1 (quad_perm)
__device__ __forceinline__ float dpp_xor8(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_mirror8(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_xor2(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_xor1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

// Sum across the four 16-lane groups of a wave (lanes l, l^16, l^32, l^48), in every lane.
__device__ __forceinline__ float sum_lane_groups(float v) {
  v = rs_swap16(v, v);
  return rs_swap32(v, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Phase timestamp (100 MHz s_memrealtime) of wave (threadIdx.x / 64) of workgroup blockIdx.x,
// slot k < 8, into buf[grid][8 waves][8 slots]; no-op when buf == null.
__device__ __forceinline__ void stamp(unsigned long long* buf, int k) {
  if (buf != nullptr && (threadIdx.x & 63) == 0)
    buf[((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace tdl
