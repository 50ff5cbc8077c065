// ResNet50 bottleneck tail: conv2 (3x3, w -> w, + BN + ReLU) and conv3 (1x1, w -> 4w, + BN)
// + identity residual + ReLU in ONE kernel, for the stride-1 blocks of layer1 (w = 64, 56x56)
// — torchvision Bottleneck.forward (v1.5), restated by oracle/image.py:backbone.
//
// Unfused, conv2 writes its w-channel output to HBM and conv3 reads it back, and conv2's
// implicit GEMM re-gathers every input pixel for all 9 taps through L2. Here, per output
// tile of one image:
//   1. the conv1 output tile with its 3x3 halo ((TOY+2)x(TOX+2) pixels x w channels, f16) is
//      staged in LDS, zero outside the image (the conv's padding);
//   2. conv2 on MFMA (v_mfma_f32_16x16x32_f16): out^T[co][q] = W2[co][(tap, ci)] . T1[p(q,tap)][ci],
//      the 32-deep k steps never straddle a tap, so each B fragment is ONE 16-B LDS read of a
//      shifted pixel row; + BN shift, ReLU, f16 -> LDS;
//   3. conv3 on MFMA over that tile; + BN shift + the residual, ReLU, f16 -> HBM.
// HBM traffic per block: the conv1 output once (+ halo, mostly L2), the block input once (as
// the residual), the block output once. Accumulation is fp32 over the same (tap, ci) k order
// as the A_CONV GEMM, with the same f16 rounding of the conv2 output: the outputs are bit-
// identical to the unfused GEMMs. MEASURED SLOWER (315 us per block vs 275 us for the two
// GEMMs, see opt().resnet_fused_tail in resnet.hip), so it is opt-in: at one 4-wave workgroup
// per CU the per-k-step LDS reads and the barriers are not hidden; two waves per SIMD (the
// q-tiles split over 8 waves) is the next form to try.
#include <algorithm>

#include "models.h"

namespace mec {

// Layer1 form (w = 64, 256 output channels, 56x56), persistent: one 4-wave workgroup per CU
// loads conv2's weights (64 x 576 f16, 72 KB) into LDS and conv3's A fragments into registers
// ONCE, then walks 8x14 output tiles (112 pixels = 7 MFMA q-tiles). While a tile computes,
// the next tile's conv1-output halo and residual are already in flight into registers, so
// the kernel streams at the rate of its bytes (halo + residual in, output out) instead of
// paying each tile's load latency. Outputs go straight from registers (8 B per lane: 4
// channels of one pixel; a pixel's 512-B row is completed by 16 stores of the workgroup).
template <int TOY, int TOX>
__global__ __launch_bounds__(256, 1) void bneck_tail64_kernel(const f16* __restrict__ t1, const f16* __restrict__ x,
                                                              const f16* __restrict__ w2, const float* __restrict__ b2,
                                                              const f16* __restrict__ w3, const float* __restrict__ b3,
                                                              f16* __restrict__ y, int H, int ntiles) {
  constexpr int W = 64, C4 = 256;
  constexpr int IRY = TOY + 2, IRX = TOX + 2, NP = IRY * IRX, MP = (NP + 15) / 16 * 16;
  constexpr int NQ = TOY * TOX, NQT = NQ / 16;  // q-tiles of 16 output pixels
  static_assert(NQ % 16 == 0, "tile must be a whole number of q-tiles");
  constexpr int K2 = 9 * W, LDW = K2 + 8;    // conv2 weights in LDS, padded row (conflict-free b128)
  constexpr int LD1 = W + 8;
  constexpr int KS2 = K2 / 32;
  constexpr int WT3 = C4 / 16 / 4;           // conv3 channel tiles per wave
  constexpr int OFF_T1 = W * LDW, OFF_T2 = OFF_T1 + MP * LD1, SMEM = OFF_T2 + NQ * LD1;
  __shared__ __attribute__((aligned(16))) f16 smem[SMEM];
  f16* sW2 = smem;
  f16* sT1 = smem + OFF_T1;
  f16* sT2 = smem + OFF_T2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int tpy = H / TOY, tpx = H / TOX, tpi = tpy * tpx;

  // ---- per-workgroup constants: conv2 weights -> LDS, conv3 fragments + biases -> registers
  {
    constexpr int NW2 = W * K2 / 8 / 256;
    static_assert(W * K2 / 8 % 256 == 0, "w2 pieces");
    half8 wv[NW2];
#pragma unroll
    for (int j = 0; j < NW2; ++j) wv[j] = reinterpret_cast<const half8*>(w2)[tid + 256 * j];
#pragma unroll
    for (int j = 0; j < NW2; ++j) {
      const int i = tid + 256 * j;
      *reinterpret_cast<half8*>(sW2 + (i / (K2 / 8)) * LDW + (i % (K2 / 8)) * 8) = wv[j];
    }
  }
  half8 a3[WT3][W / 32];  // conv3 A fragments: rows c = 16 (wave + 4 t) + l16
#pragma unroll
  for (int t = 0; t < WT3; ++t)
#pragma unroll
    for (int ks = 0; ks < W / 32; ++ks)
      a3[t][ks] = *reinterpret_cast<const half8*>(w3 + (size_t)(16 * (wave + 4 * t) + l16) * W + 32 * ks + 8 * lq);
  const float4 bias2 = *reinterpret_cast<const float4*>(b2 + 16 * wave + 4 * lq);
  float4 bias3[WT3];
#pragma unroll
  for (int t = 0; t < WT3; ++t) bias3[t] = *reinterpret_cast<const float4*>(b3 + 16 * (wave + 4 * t) + 4 * lq);
  int pq[NQT];  // top-left tap pixel of each q-tile's lane pixel
#pragma unroll
  for (int nt = 0; nt < NQT; ++nt) {
    const int q = 16 * nt + l16;
    pq[nt] = (q / TOX) * IRX + q % TOX;
  }

  constexpr int NT1 = (MP * (W / 8) + 255) / 256;
  auto tile_origin = [&](int t, size_t& img, int& oy0, int& ox0) {
    const int n = t / tpi, tt = t - n * tpi;
    img = (size_t)n * H * H;
    oy0 = (tt / tpx) * TOY;
    ox0 = (tt - (tt / tpx) * tpx) * TOX;
  };
  // the tile's conv1-output halo (tv) and residual (res[t3][nt] = x[q = 16 nt + l16][c = 16
  // (wave + 4 t3) + 4 lq ..]) -> registers
  // Loads are unconditional from clamped in-image addresses ("pad, don't mask": a load
  // under a lane condition makes hipcc branch around it and drain vmcnt); the halo pixels
  // outside the image are zeroed when the tile is written to LDS, from the `tok` bits.
  auto prefetch = [&](int t, half8 (&tv)[NT1], uint32_t& tok, half4 (&res)[WT3][NQT]) {
    size_t img;
    int oy0, ox0;
    tile_origin(t, img, oy0, ox0);
    tok = 0;
#pragma unroll
    for (int j = 0; j < NT1; ++j) {
      const int i = tid + 256 * j;
      const int p = min(i >> 3, NP - 1), c8 = i & 7;
      const int iy = oy0 - 1 + p / IRX, ix = ox0 - 1 + p % IRX;
      const bool ok = i < NP * 8 && iy >= 0 && iy < H && ix >= 0 && ix < H;
      tok |= (uint32_t)ok << j;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), H - 1);
      tv[j] = *reinterpret_cast<const half8*>(t1 + (img + (size_t)cy * H + cx) * W + c8 * 8);
    }
#pragma unroll
    for (int nt = 0; nt < NQT; ++nt) {
      const int q = 16 * nt + l16;
      const size_t pix = img + (size_t)(oy0 + q / TOX) * H + ox0 + q % TOX;
#pragma unroll
      for (int t3 = 0; t3 < WT3; ++t3)
        res[t3][nt] = *reinterpret_cast<const half4*>(x + pix * C4 + 16 * (wave + 4 * t3) + 4 * lq);
    }
  };
  // One tile from registers (tv, res) while the next tile (t + gridDim.x) lands in (tvn, resn).
  // Two register sets alternate (the loop below is unrolled by two), so no copy orders a
  // wait on the previous tile's output stores.
  auto step = [&](int t, const half8 (&tv)[NT1], uint32_t tok, const half4 (&res)[WT3][NQT], half8 (&tvn)[NT1],
                  uint32_t& tokn, half4 (&resn)[WT3][NQT]) {
#pragma unroll
    for (int j = 0; j < NT1; ++j) {
      const int i = tid + 256 * j;
      const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      if (i < MP * 8) *reinterpret_cast<half8*>(sT1 + (i >> 3) * LD1 + (i & 7) * 8) = ((tok >> j) & 1) ? tv[j] : z;
    }
    size_t img;
    int oy0, ox0;
    tile_origin(t, img, oy0, ox0);
    // raw barriers: __syncthreads()' fence would also drain the previous tile's output stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + (int)gridDim.x < ntiles) prefetch(t + gridDim.x, tvn, tokn, resn);  // in flight under the MFMAs

    // ---- conv2: wave w -> output channels 16w .. 16w+15, all q-tiles
    {
      floatx4 acc2[NQT];
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) acc2[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
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
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) {
        half4 hv;
        hv[0] = (f16)fmaxf(acc2[nt][0] + bias2.x, 0.f);
        hv[1] = (f16)fmaxf(acc2[nt][1] + bias2.y, 0.f);
        hv[2] = (f16)fmaxf(acc2[nt][2] + bias2.z, 0.f);
        hv[3] = (f16)fmaxf(acc2[nt][3] + bias2.w, 0.f);
        *reinterpret_cast<half4*>(sT2 + (16 * nt + l16) * LD1 + co) = hv;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // conv2 output complete (and every wave is done reading sT1)

    // ---- conv3 + BN shift + residual + ReLU -> straight to HBM
    {
      floatx4 acc3[WT3][NQT];
#pragma unroll
      for (int t3 = 0; t3 < WT3; ++t3)
#pragma unroll
        for (int nt = 0; nt < NQT; ++nt) acc3[t3][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < W / 32; ++ks)
#pragma unroll
        for (int nt = 0; nt < NQT; ++nt) {
          const half8 bf = *reinterpret_cast<const half8*>(sT2 + (16 * nt + l16) * LD1 + 32 * ks + 8 * lq);
#pragma unroll
          for (int t3 = 0; t3 < WT3; ++t3)
            acc3[t3][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a3[t3][ks], bf, acc3[t3][nt], 0, 0, 0);
        }
#pragma unroll
      for (int nt = 0; nt < NQT; ++nt) {
        const int q = 16 * nt + l16;
        f16* dst = y + (img + (size_t)(oy0 + q / TOX) * H + ox0 + q % TOX) * C4 + 4 * lq;
#pragma unroll
        for (int t3 = 0; t3 < WT3; ++t3) {
          half4 hv;
          hv[0] = (f16)fmaxf(acc3[t3][nt][0] + bias3[t3].x + (float)res[t3][nt][0], 0.f);
          hv[1] = (f16)fmaxf(acc3[t3][nt][1] + bias3[t3].y + (float)res[t3][nt][1], 0.f);
          hv[2] = (f16)fmaxf(acc3[t3][nt][2] + bias3[t3].z + (float)res[t3][nt][2], 0.f);
          hv[3] = (f16)fmaxf(acc3[t3][nt][3] + bias3[t3].w + (float)res[t3][nt][3], 0.f);
          *reinterpret_cast<half4*>(dst + 16 * (wave + 4 * t3)) = hv;
        }
      }
    }
  };

  half8 tvA[NT1], tvB[NT1];
  uint32_t tokA = 0, tokB = 0;
  half4 resA[WT3][NQT], resB[WT3][NQT];
  int t = blockIdx.x;
  if (t < ntiles) prefetch(t, tvA, tokA, resA);
#pragma unroll 1
  while (t < ntiles) {
    step(t, tvA, tokA, resA, tvB, tokB, resB);
    t += gridDim.x;
    if (t >= ntiles) break;
    step(t, tvB, tokB, resB, tvA, tokA, resA);
    t += gridDim.x;
  }
}

int launch_bneck_tail(const f16* t1, const f16* x, const f16* w2, const float* b2, const f16* w3, const float* b3,
                      f16* y, int B, int H, int w, hipStream_t s) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    MEC_HIP(hipGetDevice(&dev));
    MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (w == 64 && H % 8 == 0 && H % 14 == 0) {
    const int ntiles = B * (H / 8) * (H / 14);
    hipLaunchKernelGGL((bneck_tail64_kernel<8, 14>), dim3(std::min(ntiles, ncu)), dim3(256), 0, s, t1, x, w2, b2, w3,
                       b3, y, H, ntiles);
  } else {
    set_error("bneck_tail: unsupported block shape");
    return -1;
  }
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
