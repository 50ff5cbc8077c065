// ResNet50 bottleneck tail: conv2 (3x3, w -> w, + BN + ReLU) and conv3 (1x1, w -> 4w, + BN)
// + identity residual + ReLU in ONE kernel, for the stride-1 blocks of layer1 (w = 64, 56x56)
// — torchvision Bottleneck.forward (v1.5), restated by oracle/image.py:backbone.
//
// Unfused, conv2 writes its w-channel output to HBM and conv3 reads it back, and conv2's
// implicit GEMM re-gathers every input pixel for all 9 taps through L2. Here a workgroup owns
// a TOxTO tile of output pixels of one image:
//   1. the conv1 output tile with its 3x3 halo ((TO+2)^2 pixels x w channels, f16) is staged
//      in LDS once, zero outside the image (the conv's padding);
//   2. conv2 on MFMA (v_mfma_f32_16x16x32_f16): out^T[co][q] = W2[co][(tap, ci)] . T1[p(q,tap)][ci],
//      the 32-deep k steps never straddle a tap, so each B fragment is ONE 16-B LDS read of a
//      shifted pixel row; + BN shift, ReLU, f16 -> LDS;
//   3. conv3 on MFMA over that tile, in passes of 256 output channels; + BN shift + the
//      residual (prefetched into registers before step 1), ReLU, f16, staged through LDS and
//      written with 16-B row-contiguous stores.
// HBM traffic per block: the conv1 output once (+ halo, mostly L2), the block input once (as
// the residual), the block output once. Accumulation is fp32 over the same (tap, ci) k order
// as the A_CONV GEMM, with the same f16 rounding of the conv2 output: the outputs are bit-
// identical to the unfused GEMMs. MEASURED SLOWER (see g_resnet_fused_tail in resnet.hip), so
// it is off by default; a persistent form that keeps the weights resident and prefetches the
// next tile under the current one's MFMAs is the version that could pay.
#include "models.h"

namespace mec {

// Layer1 form (w = 64, 256 output channels, 56x56): a workgroup owns an 8x14 tile (112
// output pixels = 7 MFMA q-tiles) and stages ALL of conv2's weights (64 x 576 f16, 72 KB) in
// LDS next to the halo tile, so the 18 conv2 k steps read only LDS; after conv2 the weight
// region becomes the output staging buffer. One workgroup per CU (~110 KB LDS).
template <int TOY, int TOX>
__global__ __launch_bounds__(256, 1) void bneck_tail64_kernel(const f16* __restrict__ t1, const f16* __restrict__ x,
                                                              const f16* __restrict__ w2, const float* __restrict__ b2,
                                                              const f16* __restrict__ w3, const float* __restrict__ b3,
                                                              f16* __restrict__ y, int H) {
  constexpr int W = 64, C4 = 256;
  constexpr int IRY = TOY + 2, IRX = TOX + 2, NP = IRY * IRX, MP = (NP + 15) / 16 * 16;
  constexpr int NQ = TOY * TOX, NQT = NQ / 16;  // q-tiles of 16 output pixels
  static_assert(NQ % 16 == 0, "tile must be a whole number of q-tiles");
  constexpr int K2 = 9 * W, LDW = K2 + 8;    // conv2 weights in LDS, padded row (conflict-free b128)
  constexpr int LD1 = W + 8, LDO = C4 + 8;
  constexpr int KS2 = K2 / 32;
  constexpr int WT3 = C4 / 16 / 4;           // conv3 channel tiles per wave
  constexpr int OFF_T1 = W * LDW, OFF_T2 = OFF_T1 + MP * LD1, SMEM = OFF_T2 + NQ * LD1;
  static_assert(NQ * LDO <= W * LDW, "output staging fits the weight region");
  __shared__ __attribute__((aligned(16))) f16 smem[SMEM];
  f16* sW2 = smem;
  f16* sT1 = smem + OFF_T1;
  f16* sT2 = smem + OFF_T2;
  f16* sO = smem;  // after conv2

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int tpy = H / TOY, tpx = H / TOX, tpi = tpy * tpx;
  int bid = blockIdx.x;
  {  // XCD-aware: the tiles of one image (which share halo rows) run on one XCD's L2
    const int nwg = gridDim.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int n = bid / tpi, tt = bid - n * tpi;
  const int oy0 = (tt / tpx) * TOY, ox0 = (tt - (tt / tpx) * tpx) * TOX;
  const size_t img = (size_t)n * H * H;

  // ---- one burst of loads: conv2 weights, conv1-output halo tile, conv3 weights, residual
  constexpr int NW2 = W * K2 / 8 / 256;  // 16-B pieces per thread
  static_assert(W * K2 / 8 % 256 == 0, "w2 pieces");
  half8 wv[NW2];
#pragma unroll
  for (int j = 0; j < NW2; ++j) wv[j] = reinterpret_cast<const half8*>(w2)[tid + 256 * j];
  constexpr int NT1 = (MP * (W / 8) + 255) / 256;
  half8 tv[NT1];
#pragma unroll
  for (int j = 0; j < NT1; ++j) {
    const int i = tid + 256 * j;
    const int p = i >> 3, c8 = i & 7;
    const int iy = oy0 - 1 + p / IRX, ix = ox0 - 1 + p % IRX;
    tv[j] = half8{0, 0, 0, 0, 0, 0, 0, 0};
    if (i < MP * 8 && p < NP && iy >= 0 && iy < H && ix >= 0 && ix < H)
      tv[j] = *reinterpret_cast<const half8*>(t1 + (img + (size_t)iy * H + ix) * W + c8 * 8);
  }
  half8 a3[WT3][W / 32];  // conv3 A fragments: rows c = 16 (wave + 4 t) + l16
#pragma unroll
  for (int t = 0; t < WT3; ++t)
#pragma unroll
    for (int ks = 0; ks < W / 32; ++ks)
      a3[t][ks] = *reinterpret_cast<const half8*>(w3 + (size_t)(16 * (wave + 4 * t) + l16) * W + 32 * ks + 8 * lq);
  half4 res[WT3][NQT];  // x[q = 16 nt + l16][c = 16 (wave + 4 t) + 4 lq ..]
#pragma unroll
  for (int nt = 0; nt < NQT; ++nt) {
    const int q = 16 * nt + l16;
    const size_t pix = img + (size_t)(oy0 + q / TOX) * H + ox0 + q % TOX;
#pragma unroll
    for (int t = 0; t < WT3; ++t)
      res[t][nt] = *reinterpret_cast<const half4*>(x + pix * C4 + 16 * (wave + 4 * t) + 4 * lq);
  }
#pragma unroll
  for (int j = 0; j < NW2; ++j) {
    const int i = tid + 256 * j;  // piece i = row i / 72, chunk i % 72
    *reinterpret_cast<half8*>(sW2 + (i / (K2 / 8)) * LDW + (i % (K2 / 8)) * 8) = wv[j];
  }
#pragma unroll
  for (int j = 0; j < NT1; ++j) {
    const int i = tid + 256 * j;
    if (i < MP * 8) *reinterpret_cast<half8*>(sT1 + (i >> 3) * LD1 + (i & 7) * 8) = tv[j];
  }
  __syncthreads();

  // ---- conv2: wave w -> output channels 16w .. 16w+15, all q-tiles (out^T: lane holds 4 channels)
  {
    floatx4 acc2[NQT];
#pragma unroll
    for (int nt = 0; nt < NQT; ++nt) acc2[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    int pq[NQT];
#pragma unroll
    for (int nt = 0; nt < NQT; ++nt) {
      const int q = 16 * nt + l16;
      pq[nt] = (q / TOX) * IRX + q % TOX;
    }
    const f16* wrow = sW2 + (16 * wave + l16) * LDW + 8 * lq;
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      const int tap = (32 * ks) / W, ci = 32 * ks - tap * W;
      const int dp = (tap / 3) * IRX + tap % 3;
      const half8 af = *reinterpret_cast<const half8*>(wrow + 32 * ks);
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) {
        const half8 bf = *reinterpret_cast<const half8*>(sT1 + (pq[nt] + dp) * LD1 + ci + 8 * lq);
        acc2[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, acc2[nt], 0, 0, 0);
      }
    }
    const int co = 16 * wave + 4 * lq;
    const float4 bv = *reinterpret_cast<const float4*>(b2 + co);
#pragma unroll
    for (int nt = 0; nt < NQT; ++nt) {
      half4 hv;
      hv[0] = (f16)fmaxf(acc2[nt][0] + bv.x, 0.f);
      hv[1] = (f16)fmaxf(acc2[nt][1] + bv.y, 0.f);
      hv[2] = (f16)fmaxf(acc2[nt][2] + bv.z, 0.f);
      hv[3] = (f16)fmaxf(acc2[nt][3] + bv.w, 0.f);
      *reinterpret_cast<half4*>(sT2 + (16 * nt + l16) * LD1 + co) = hv;
    }
  }
  __syncthreads();  // conv2 output complete; the weight region is free

  // ---- conv3 + BN shift + residual + ReLU -> staging -> 16-B row stores
  {
    floatx4 acc3[WT3][NQT];
#pragma unroll
    for (int t = 0; t < WT3; ++t)
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) acc3[t][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < W / 32; ++ks)
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) {
        const half8 bf = *reinterpret_cast<const half8*>(sT2 + (16 * nt + l16) * LD1 + 32 * ks + 8 * lq);
#pragma unroll
        for (int t = 0; t < WT3; ++t)
          acc3[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a3[t][ks], bf, acc3[t][nt], 0, 0, 0);
      }
#pragma unroll
    for (int t = 0; t < WT3; ++t) {
      const int c = 16 * (wave + 4 * t) + 4 * lq;
      const float4 bv = *reinterpret_cast<const float4*>(b3 + c);
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) {
        half4 hv;
        hv[0] = (f16)fmaxf(acc3[t][nt][0] + bv.x + (float)res[t][nt][0], 0.f);
        hv[1] = (f16)fmaxf(acc3[t][nt][1] + bv.y + (float)res[t][nt][1], 0.f);
        hv[2] = (f16)fmaxf(acc3[t][nt][2] + bv.z + (float)res[t][nt][2], 0.f);
        hv[3] = (f16)fmaxf(acc3[t][nt][3] + bv.w + (float)res[t][nt][3], 0.f);
        *reinterpret_cast<half4*>(sO + (16 * nt + l16) * LDO + c) = hv;
      }
    }
  }
  __syncthreads();
  constexpr int C8 = C4 / 8;
#pragma unroll
  for (int j = 0; j < NQ * C8 / 256; ++j) {
    const int i = tid + 256 * j;
    const int q = i / C8, c8 = i - (i / C8) * C8;
    const size_t pix = img + (size_t)(oy0 + q / TOX) * H + ox0 + q % TOX;
    *reinterpret_cast<half8*>(y + pix * C4 + c8 * 8) = *reinterpret_cast<const half8*>(sO + q * LDO + c8 * 8);
  }
}

int launch_bneck_tail(const f16* t1, const f16* x, const f16* w2, const float* b2, const f16* w3, const float* b3,
                      f16* y, int B, int H, int w, hipStream_t s) {
  if (w == 64 && H % 8 == 0 && H % 14 == 0) {
    hipLaunchKernelGGL((bneck_tail64_kernel<8, 14>), dim3(B * (H / 8) * (H / 14)), dim3(256), 0, s, t1, x, w2, b2, w3,
                       b3, y, H);
  } else {
    set_error("bneck_tail: unsupported block shape");
    return -1;
  }
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
