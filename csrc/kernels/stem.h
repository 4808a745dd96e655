// Small-channel stride-2 convolution on the gfx950 bf16 matrix cores: the ResNet-50 stem (7x7 / 2,
// 3 input channels), which the 64-channel-chunk implicit GEMM of conv.h cannot take (see stem.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

// C <= 4 input channels, KH <= 8, KW <= 8, column stride 2, K % 64 == 0
bool stem_supported(int C, int KH, int KW, int SW, int K);
// x [N][H][W][C] (bf16 or f32) -> xp [N][HP][WP][4] bf16: zero border (PT top, PL left, the rest
// bottom / right) and zero channels C..3
void stem_pack(const void* x, bool x_bf16, void* xp, int N, int H, int W, int C, int HP, int WP, int PT, int PL,
               hipStream_t s);
// w_hwio [KH][KW][C][K] bf16 -> wp [K][KH][32] bf16 (tap t = kw * 4 + c, zero-filled)
void stem_wpack(const void* w_hwio, void* wp, int KH, int KW, int C, int K, hipStream_t s);
// y [N][OH][OW][K] = valid conv of xp with wp, row stride SH, column stride 2; stats (optional):
// [ceil(N*OH*OW / stem_fwd_row_tile())][2][K] per-tile channel sums of y and y^2 (bf16 values)
void stem_fwd(const void* xp, const void* wp, void* y, float* stats, int N, int HP, int WP, int OH, int OW, int K,
              int KH, int SH, hipStream_t s);
int stem_fwd_row_tile();
// dW (HWIO [KH][KW][C][K]) from xp and dy [N][OH][OW][K]: into dw_bf16, or (dw_bf16 == nullptr) the
// f32 dw_f32 (added to when accumulate); ws: stem_wgrad_ws_elems f32 (deterministic slice partials)
long long stem_wgrad_ws_elems(int M, int K, int KH);
void stem_wgrad(const void* xp, const void* dy, float* ws, int N, int HP, int WP, int OH, int OW, int K, int KH, int KW,
                int C, int SH, float* dw_f32, void* dw_bf16, bool accumulate, hipStream_t s);

}  // namespace tdl
