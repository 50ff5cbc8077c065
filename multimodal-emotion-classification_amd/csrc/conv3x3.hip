// 3x3 / stride-1 / pad-1 convolution, 64 -> 64 channels on 56x56 NHWC f16, + BN shift + ReLU:
// ResNet50 layer1's conv2 (torchvision Bottleneck.conv2/bn2/relu, oracle/image.py:backbone).
//
// As an implicit GEMM (gemm_glds_kernel, A_CONV) every input pixel is gathered through L2
// once per tap, 9 x 128 B per output pixel, and that L2 -> LDS stream, not the MFMAs, bounds
// it (≈130 us at B = 256). Here a persistent workgroup (4 waves, one per SIMD, one per CU)
// walks tiles of 8 output rows x 56 columns of one image (B x 7 tiles):
//   * the tile's input halo (10 rows x 58 columns x 64 channels, 74 KB) is DMA'd once
//     (global_load_lds_dwordx4) into one of two LDS buffers while the previous tile computes:
//     1.3 x 128 B per output pixel instead of 9 x 128 B;
//   * the weights (64 x 576 f16) live in registers for the whole launch: wave (h, g) holds
//     output channels 32h .. 32h+31 as 2 x 18 A fragments and computes tile rows 4g .. 4g+3
//     (224 pixels = 14 B fragments), so each 16-B LDS read feeds two MFMAs;
//   * out^T[co][px] = W[co][(tap, ci)] . X[px + tap][ci] on v_mfma_f32_16x16x32_f16: the
//     32-deep k steps run in the A_CONV GEMM's (kh, kw, ci) order, so every output is the
//     same fp32 chain as the GEMM path, then the same bias / ReLU / f16 epilogue: the result
//     is bit-identical to it (tests/test_gpu_kernels.py::test_conv3x3_c64_bit_identical);
//   * the output tile is staged through the consumed halo buffer and written as contiguous
//     1-KB runs (the tile is one contiguous block of the NHWC image).
// LDS pixel rows are 128 B; a pixel's 16-B channel chunk c is stored at c ^ (halo column & 7)
// (applied on the DMA source side). Every fragment's 16 pixels are consecutive columns (the
// 56-pixel row break is a multiple of 8), so the ds_read_b128 lane groups are conflict-free
// and each read address is one of 12 per-lane bases plus a compile-time immediate.
// Measured (tools/bench_conv3x3.py, B = 256): 71 us against 126-133 us for the GEMM path.
#include <algorithm>

#include "models.h"

namespace mec {

__device__ __attribute__((aligned(64))) uint4 g_c3_zero[4];

constexpr int C3_H = 56, C3_C = 64, C3_K = 9 * C3_C;   // image side, channels, GEMM depth
constexpr int C3_TR = 8;                               // output rows per tile
constexpr int C3_HR = C3_TR + 2, C3_PITCH = C3_H + 2;  // halo rows, halo row pitch (pixels)
constexpr int C3_CHUNKS = C3_HR * C3_PITCH * 8;        // 16-B chunks per halo (4640)
constexpr int C3_FULL = C3_CHUNKS / 256;               // whole 256-lane DMA passes (18)
constexpr int C3_TAIL = C3_CHUNKS - C3_FULL * 256;     // the rest, loaded by wave 0 (32)
constexpr int C3_BUF = (C3_FULL * 256 + 64) * 8;       // halfs per halo buffer (74,752 B)
constexpr int C3_KS = C3_K / 32;                       // 32-deep k steps (18)
static_assert(C3_TAIL > 0 && C3_TAIL <= 64, "halo tail must fit one wave");

// LDS DMA (global_load_lds_dwordx4: 16 B per lane to M0 + 16 x lane) issued from inline asm.
// Issued as the builtin, hipcc's waitcnt pass treats every in-flight DMA as an unordered
// LGKM event and drains lgkmcnt(0) before each use of a fragment read (33 drains per tile);
// hidden from it, the fragment reads get counted waits. The DMA is ordered only by this
// kernel's explicit vmcnt waits and barriers (MI355X_MICROARCH.md: nothing else orders a
// ds_read behind a pending LDS DMA).
#pragma clang diagnostic ignored "-Winline-asm"  // m0: see pw_chain.hip
__device__ __forceinline__ void c3_dma(const void* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

template <int DBG>
__global__ __launch_bounds__(256, 1) void conv3x3_c64_kernel(const f16* __restrict__ x, const f16* __restrict__ w,
                                                             const float* __restrict__ bias, f16* __restrict__ y,
                                                             int ntiles) {
  __shared__ __attribute__((aligned(16))) f16 smem[2 * C3_BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = wave & 1, rg = wave >> 1;  // output-channel half, row group (4 rows) of the tile
  const int l16 = lane & 15, lq = lane >> 4;

  // One tile's halo -> LDS buffer `b`. Lane-linear destination chunk q = (pixel slot, chunk
  // kc'); it fetches channel chunk kc' ^ (slot & 7) of that pixel (the read-side swizzle).
  // Out-of-image pixels read the zero page: the DMA writes the padding itself.
  auto issue = [&](int t, int b) {
    const int n = t / 7, r0 = (t - n * 7) * C3_TR;
    const f16* img = x + (size_t)n * C3_H * C3_H * C3_C;
    const uint32_t lds_dst =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) f16*)smem) + (uint32_t)(b * C3_BUF * 2);
    const f16* zero = reinterpret_cast<const f16*>(g_c3_zero);
    int tq = tid;
    asm volatile("" : "+v"(tq));  // recomputed per tile rather than hoisted (VGPR budget)
#pragma unroll
    for (int it = 0; it <= C3_FULL; ++it) {
      if (it == C3_FULL && wave != 0) break;
      const int q = it * 256 + (it == C3_FULL ? (tq & 63) : tq);
      const int ps = q >> 3;
      const int hr = ps / C3_PITCH, hc = ps - hr * C3_PITCH;
      const int kc = (q & 7) ^ (hc & 7);
      const int iy = r0 - 1 + hr, ix = hc - 1;
      const bool ok = q < C3_CHUNKS && iy >= 0 && iy < C3_H && ix >= 0 && ix < C3_H;
      const f16* src = ok ? img + ((size_t)iy * C3_H + ix) * C3_C + kc * 8 : zero;
      c3_dma(src, lds_dst + (uint32_t)(it * 256 + (it == C3_FULL ? 0 : wave * 64)) * 16u);
    }
  };

  // weights: A fragment (co = 32h + 16cf + l16, k = 32s + 8lq .. +7), resident for the launch
  half8 wf[2][C3_KS];
#pragma unroll
  for (int cf = 0; cf < 2; ++cf)
#pragma unroll
    for (int s = 0; s < C3_KS; ++s)
      wf[cf][s] = *reinterpret_cast<const half8*>(w + (size_t)(32 * h + 16 * cf + l16) * C3_K + 32 * s + 8 * lq);
  // opaque: the weights stay in registers (never re-loaded inside the tile loop)
#pragma unroll
  for (int cf = 0; cf < 2; ++cf)
#pragma unroll
    for (int s = 0; s < C3_KS; ++s) asm volatile("" : "+v"(wf[cf][s]));
  float4 bs[2];
#pragma unroll
  for (int cf = 0; cf < 2; ++cf) bs[cf] = *reinterpret_cast<const float4*>(bias + 32 * h + 16 * cf + 4 * lq);
  // B fragment f of the wave: pixel p = 16f + l16 of its 224 (rows 4rg .. 4rg+3 of the tile,
  // 56 each); its tap-(0,0) halo slot is (p / 56) * 58 + p % 56 = sl + 16f + 2 (p / 56), where
  // p / 56 is lane-dependent only in fragments 3 and 10 (they straddle a row break)
  int sl = 4 * rg * C3_PITCH + l16;
  int brk = l16 >= 8 ? 2 : 0;

  int t = blockIdx.x, b = 0;
  bool first = true;
  if (t < ntiles) issue(t, 0);
#pragma unroll 1
  while (t < ntiles) {
    const int tn = t + gridDim.x;
    // this tile's halo has landed: only the previous tile's 14 output stores (issued after
    // it) may still be in flight
    if (first)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    first = false;
    __builtin_amdgcn_s_barrier();  // every wave's DMA for tile t landed; buffer b^1 is free
    if (tn < ntiles && !(DBG & 1)) issue(tn, b ^ 1);

    // Fragment addresses: pixel p = 16f + l16 at tap (kh, kw) sits in halo slot
    // sl + 16f + roff(f) [+ brk] + 58 kh + kw, and its chunk (4j + lq) is stored at
    // (4j + lq) ^ (halo column & 7) = (4j + lq) ^ ((l16 + kw) & 7) (16f and the 56-pixel row
    // break are multiples of 8). So the address is one of 12 per-lane bases (kw, j, brk)
    // plus a compile-time immediate: no address arithmetic per read.
    uint32_t abase[2][3][2];
    {
      const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) f16*)smem);  // LDS offset
      const uint32_t buf = lds0 + (uint32_t)(b * C3_BUF * 2);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint32_t ch = (uint32_t)((4 * j + lq) ^ ((l16 + kw) & 7));
          abase[0][kw][j] = buf + (uint32_t)sl * 128u + ch * 16u;
          abase[1][kw][j] = abase[0][kw][j] + (uint32_t)brk * 128u;
        }
    }
    auto rd = [&](int s, int f) {
      const int tap = s >> 1, j = s & 1, kh = tap / 3, kw = tap % 3;
      const int roff = f < 4 ? 0 : (f < 7 ? 2 : (f < 11 ? 4 : 6));  // 2 x (row of the fragment's first pixel)
      const uint32_t imm = (uint32_t)(16 * f + roff + kh * C3_PITCH + kw) * 128u;
      const uint32_t addr = abase[(f == 3 || f == 10) ? 1 : 0][kw][j] + imm;
      return *(const __attribute__((address_space(3))) half8*)(uintptr_t)addr;
    };
    floatx4 acc[14][2];
#pragma unroll
    for (int f = 0; f < 14; ++f)
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) acc[f][cf] = floatx4{0.f, 0.f, 0.f, 0.f};
    // rotating fragment schedule over the flat sequence i = 14 s + f of (step, fragment)
    // MFMA pairs: the fragment of pair i + 7 is read right after pair i, into the slot pair
    // i - 7 freed, so each LDS read has 14 MFMAs to land (counted lgkmcnt(6) waits; a
    // 12-pair lookahead measured the same)
    constexpr int NP = 14 * C3_KS, LA = 7;
    half8 a[14];
#pragma unroll
    for (int i = 0; i < LA; ++i) a[i] = rd(0, i);
#pragma unroll
    for (int st = 0; st < C3_KS; ++st)
#pragma unroll
      for (int f = 0; f < 14; ++f) {
#pragma unroll
        for (int cf = 0; cf < 2; ++cf)
          acc[f][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[cf][st], a[f], acc[f][cf], 0, 0, 0);
        const int i = 14 * st + f + LA;
        if (i < NP && !(DBG & 4)) a[i % 14] = rd(i / 14, i % 14);
        __builtin_amdgcn_sched_barrier(0);
      }
    // epilogue as the GEMM's: (acc + bias) + 0 (no residual), ReLU, f16. Staged through the
    // halo buffer just consumed (the tile's 448 x 128 B output is ONE contiguous block of the
    // NHWC image), then written as whole 1-KB runs: 16 B per lane, 8 lanes per pixel row.
    // Direct 8-B stores from the MFMA layout (16 pixel rows touched per instruction) took
    // 55 of the kernel's 80 us.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading buffer b
    char* stg = reinterpret_cast<char*>(smem + b * C3_BUF);
#pragma unroll
    for (int f = 0; f < 14; ++f) {
      const int pt = 224 * rg + 16 * f + l16;  // tile-local pixel
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) {
        const float bb[4] = {bs[cf].x, bs[cf].y, bs[cf].z, bs[cf].w};
        half4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[f][cf][e] + bb[e];
          v += 0.f;
          hv[e] = (f16)fmaxf(v, 0.f);
        }
        const int ch = 4 * h + 2 * cf + (lq >> 1);  // 16-B chunk of channels 32h + 16cf + 4lq ..
        *reinterpret_cast<half4*>(stg + pt * 128 + ((ch ^ (pt & 7)) << 4) + (lq & 1) * 8) = hv;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      const int n = t / 7, r0 = (t - n * 7) * C3_TR;
      f16* out = y + ((size_t)n * C3_H + r0) * C3_H * C3_C;
#pragma unroll
      for (int i = 0; i < 448 * 8 / 256; ++i) {
        const int q = i * 256 + tid, pt = q >> 3, c = q & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(stg + pt * 128 + ((c ^ (pt & 7)) << 4));
        if (!(DBG & 2) || v.x == 0x12345678u) *reinterpret_cast<uint4*>(out + (size_t)q * 8) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(DBG & 1)) b ^= 1;
    t = tn;
  }
}


int launch_conv3x3_c64(const f16* x, const f16* w, const float* bias, f16* y, int B, int H, int C, int Cout,
                       hipStream_t s) {
  MEC_REQUIRE(H == C3_H && C == C3_C && Cout == C3_C, "conv3x3_c64: needs 56x56, 64 -> 64 channels");
  MEC_REQUIRE(x && w && bias && y && B > 0, "conv3x3_c64: bad arguments");
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    MEC_HIP(hipGetDevice(&dev));
    MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int ntiles = B * (C3_H / C3_TR);
  const dim3 grd(std::min(ntiles, ncu)), blk(256);
  switch (opt().conv3x3_debug) {  // probe builds (wrong results): 1 no next-tile DMA, 2 no stores, 4 no LDS reads
    case 0: hipLaunchKernelGGL(conv3x3_c64_kernel<0>, grd, blk, 0, s, x, w, bias, y, ntiles); break;
#ifdef MEC_PROBES
    case 1: hipLaunchKernelGGL(conv3x3_c64_kernel<1>, grd, blk, 0, s, x, w, bias, y, ntiles); break;
    case 2: hipLaunchKernelGGL(conv3x3_c64_kernel<2>, grd, blk, 0, s, x, w, bias, y, ntiles); break;
    case 4: hipLaunchKernelGGL(conv3x3_c64_kernel<4>, grd, blk, 0, s, x, w, bias, y, ntiles); break;
    case 7: hipLaunchKernelGGL(conv3x3_c64_kernel<7>, grd, blk, 0, s, x, w, bias, y, ntiles); break;
#endif
    default: set_error("conv3x3_debug: bad value"); return -1;
  }
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
