// 3x3 / stride-1 / pad-1 convolutions of ResNet50 layers 2-3 (torchvision Bottleneck.conv2 +
// bn2 + relu, oracle/image.py:backbone) on NHWC f16: 28x28x128 and 14x14x256, C -> C.
//
// As an implicit GEMM (gemm_glds_kernel, A_CONV) every input pixel row is fetched from L2 into
// LDS once per tap: 9 x 2C bytes per output pixel, with 128-256 output pixels per tile. That
// L2 -> LDS stream bounds those convs at 75-100 us each (15-30 % MFMA busy). Here a tile is 224
// output pixels (7 rows x 32 of a 28x28 image, or a whole 14x14 image as 14 x 16) x 128 output
// channels:
//   * per 32-channel chunk, the tile's input halo ((rows + 2) x pitch pixels x 64 B) is DMA'd
//     (global_load_lds_dwordx4) into one of two LDS buffers a chunk ahead, ONCE for all nine
//     taps: the 9x re-read of the implicit GEMM becomes ~1.3x;
//   * the weight slice of one (tap, chunk) k-step (128 channels x 64 B) streams through a
//     3-slot LDS ring, issued two k-steps ahead;
//   * out^T[co][px] = W[co][(tap, ci)] . X[px + tap][ci] on v_mfma_f32_16x16x32_f16; 4 waves =
//     2 (64 output channels) x 2 (112 pixels): 4 x 7 accumulator tiles per wave, 11 LDS reads
//     for 28 MFMAs per k-step, single-buffered (the other workgroup on the CU computes while a
//     wave reads; double-buffered fragments did not fit 256 VGPRs next to the accumulators);
//   * output columns are padded to a multiple of 16 (WP: 32 / 16) so every 16-pixel MFMA
//     fragment is 16 consecutive halo slots; padded pixels are computed, not stored (12.5 % of
//     the MFMAs);
//   * halo pitch P and image stride are multiples of 8 slots and a pixel's 16-B channel chunk k
//     sits at k ^ ((slot >> 1) & 3): every ds_read_b128 lane group of the fragment reads is
//     conflict-free for all nine tap offsets (checked exhaustively for both geometries, and for
//     the 7x7 four-image layout below), and each read address is the sum of two per-lane
//     registers plus an immediate;
//   * k order per output: chunk-major, tap-minor (c, kh, kw, ci in c) — fp32 accumulation like
//     the GEMM path but a different summation order, so results agree with it to rounding, not
//     bit for bit (tests/test_gpu_kernels.py::test_conv3x3_halo); any batch split gives the same
//     bits (a tile never mixes the work of two launches);
//   * epilogue: + BN shift, ReLU, f16, staged through LDS (chunk XOR swizzle) and written as
//     256-B pixel runs; blocks map to tiles XCD-aware (one output-channel tile per XCD).
// Two workgroups per CU (72 KB of LDS, 216 VGPRs each). Routed from launch_gemm while
// opt().conv3x3_halo is set.
#include <algorithm>
#include <type_traits>

#include "models.h"

namespace mec {

__device__ __attribute__((aligned(64))) uint4 g_ch_zero[4];

#pragma clang diagnostic ignored "-Winline-asm"  // m0: see pw_chain.hip
__device__ __forceinline__ void ch_dma(const void* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void ch_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int V>
using ic = std::integral_constant<int, V>;

// HW: image side; WP: padded output width; P: halo pitch (slots); R: output rows per tile;
// G: images per tile; C: channels in = out.
template <int HW, int WP, int P, int R, int G, int C>
struct HaloCfg {
  static constexpr int K = 9 * C, NC = C / 32, NCT = C / 128, RB = HW / R;
  static constexpr int HR = R + 2, IS = HR * P, SLOTS = G * IS;
  static constexpr int HI = ((SLOTS + 15) / 16 + 3) / 4;  // 1-KB halo DMA instructions per wave per chunk
  static constexpr int HBUF = HI * 4 * 1024;        // bytes per halo buffer
  static constexpr int WSLOT = 128 * 64;            // bytes per weight slice
  static constexpr int LDS = 2 * HBUF + 3 * WSLOT;
  static constexpr int T = 9 * NC;                  // k-steps
  static_assert(R * WP * G == 224, "224-pixel tiles");
  static_assert(T % 3 == 0 && NC % 2 == 0 && HW % R == 0 && P % 8 == 0 && IS % 8 == 0 && P >= WP + 2, "geometry");
  static_assert(LDS >= 224 * 256, "epilogue staging fits");
  static_assert(8 % NCT == 0, "output-channel tiles per XCD");
};

// DBG (probe builds only, conv3x3_debug): 1 = no DMA inside the k loop, 2 = no output stores,
// 4 = no fragment reads inside the k loop (all return wrong results)
template <int HW, int WP, int P, int R, int G, int C, int DBG = 0>
__global__ __launch_bounds__(256, G == 1 ? 2 : 1) void conv3x3_halo_kernel(const f16* __restrict__ x, const f16* __restrict__ w,
                                                              const float* __restrict__ bias, f16* __restrict__ y,
                                                              int B) {
  using Cf = HaloCfg<HW, WP, P, R, G, C>;
  constexpr int K = Cf::K, NC = Cf::NC, NCT = Cf::NCT, RB = Cf::RB, IS = Cf::IS, HI = Cf::HI;
  constexpr int HBUF = Cf::HBUF, WSLOT = Cf::WSLOT, T = Cf::T;
  __shared__ __attribute__((aligned(1024))) char smem[Cf::LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wco = wave & 1, wpx = wave >> 1;
  const int j = lane & 15, kc = lane >> 4;

  // ---- tile: output-channel tile ct is fixed per XCD (blocks b, b + 8 share one)
  const int nsp = ((B + G - 1) / G) * RB;
  const int b = blockIdx.x, xcd = b & 7;
  const int ct = xcd % NCT;
  const int sp = (b >> 3) * (8 / NCT) + xcd / NCT;
  if (sp >= nsp) return;
  const int ig = sp / RB, rb = sp - (sp / RB) * RB;

  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const f16* zero = reinterpret_cast<const f16*>(g_ch_zero);

  // ---- per-lane DMA sources. Halo: slot s = 16 gi + lane/4 holds input pixel (n, ih, iw) of
  // its (image, halo row, halo column); the lane fetches logical chunk (lane&3) ^ ((s>>1)&3).
  auto halo_off = [&](int i) {  // element offset of the lane's source for halo instruction i, or -1
    int s = (i * 4 + wave) * 16 + (lane >> 2);
    asm volatile("" : "+v"(s));  // recomputed at each halo issue (every 9 k-steps): VGPR budget
    int off = -1;
    if (s < Cf::SLOTS) {
      const int g = s / IS, rem = s - (s / IS) * IS;
      const int hr = rem / P, hc = rem - (rem / P) * P;
      const int n = ig * G + g, ih = rb * R - 1 + hr, iw = hc - 1;
      if (n < B && ih >= 0 && ih < HW && iw >= 0 && iw < HW)
        off = ((n * HW + ih) * HW + iw) * C + (((lane & 3) ^ ((s >> 1) & 3)) * 8);
    }
    return off;
  };
  // weights: slice row rr = 16 gi + lane/4 (output channel 128 ct + rr), same chunk swizzle
  int woff[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rr = (wave * 2 + q) * 16 + (lane >> 2);
    woff[q] = (ct * 128 + rr) * K + (((lane & 3) ^ ((rr >> 1) & 3)) * 8);
  }
  auto issue_halo = [&](int c, int bsel) {
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int o = halo_off(i);
      const f16* src = o >= 0 ? x + o + c * 32 : zero;
      ch_dma(src, lds0 + (uint32_t)(bsel * HBUF + (i * 4 + wave) * 1024));
    }
  };
  auto issue_w = [&](int c, int tap, int slot) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int o = woff[q];
      asm volatile("" : "+v"(o));
      ch_dma(w + o + tap * C + c * 32, lds0 + (uint32_t)(2 * HBUF + slot * WSLOT + (wave * 2 + q) * 1024));
    }
  };

  // ---- per-lane fragment addresses. Weights: row 64 wco + 16 cf + j, chunk kc.
  const uint32_t aw = lds0 + 2 * HBUF + (uint32_t)((wco * 64 + j) * 64 + ((kc ^ ((j >> 1) & 3)) * 16));
  // Pixels: fragment pf of the wave covers output pixels q = 16 pfg + j; at tap (kh, kw) it reads
  // halo slot S(q) + kh P + kw, whose chunk kc sits at kc ^ ((((j & 7) + kw) & 7) >> 1) (S(q) = j
  // mod 8, P = 0 mod 8). ap[pf][kw] = 64 S(q) + that chunk offset; the rest is an immediate.
  auto pfg_of = [&](int pf) { return WP == 32 ? 2 * pf + wpx : 7 * wpx + pf; };
  uint32_t apb[7], ask[3];
#pragma unroll
  for (int pf = 0; pf < 7; ++pf) {
    const int q = pfg_of(pf) * 16 + j;
    const int g = q / (R * WP), rem = q - g * (R * WP);
    const int r = rem / WP, c = rem - r * WP;
    apb[pf] = lds0 + (uint32_t)((g * IS + r * P + c) * 64);
  }
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) ask[kw] = (uint32_t)((kc ^ ((((j & 7) + kw) & 7) >> 1)) * 16);

  typedef __attribute__((address_space(3))) const half8 lds_h8;
  // fragments of one k-step, single-buffered: each wave reads them after the step's barrier and
  // then issues its 28 MFMAs; the co-resident workgroup's MFMAs cover the read latency
  half8 wf[4], xf[7];

  floatx4 acc[7][4];
#pragma unroll
  for (int pf = 0; pf < 7; ++pf)
#pragma unroll
    for (int cf = 0; cf < 4; ++cf) acc[pf][cf] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: halo chunks 0 / 1, weight slices of k-steps 0 / 1
  issue_halo(0, 0);
  issue_w(0, 0, 0);
  issue_halo(1, 1);
  issue_w(0, 1, 1);
  ch_vmwait<2>();  // halo 0, slice 0 and halo 1 landed (slice 1 may fly)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // k-step t = 9 c + tap (U = t % 3 compile-time: weight ring slot and kw). Slice t sits in ring
  // slot t % 3, halo chunk c in buffer c % 2. At step t (after its barrier, which published
  // slice t): slice t + 2 goes into slot (t + 2) % 3, read at step t - 1; at tap 0, halo chunk
  // c + 1 goes into buffer (c + 1) % 2, read during chunk c - 1.
  auto step = [&](auto Uc, int t) {
    constexpr int U = decltype(Uc)::value, kw = U;
    const int c = t / 9, tap = t - c * 9, kh = tap / 3;
    const bool more_w = t + 2 < T;
    if (more_w && !(DBG & 1)) {
      const int c2 = (t + 2) / 9;
      issue_w(c2, t + 2 - c2 * 9, (U + 2) % 3);
    }
    const bool halo_now = tap == 0 && c >= 1 && c + 1 < NC;
    if (halo_now && !(DBG & 1)) issue_halo(c + 1, (c + 1) & 1);
    if (!(DBG & 4) || t == 0) {
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) wf[cf] = *(lds_h8*)(uintptr_t)(aw + (uint32_t)(U * WSLOT + cf * 1024));
      const uint32_t xl = ask[kw] + (uint32_t)((c & 1) * HBUF + (kh * P + kw) * 64);
#pragma unroll
      for (int pf = 0; pf < 7; ++pf) xf[pf] = *(lds_h8*)(uintptr_t)(apb[pf] + xl);
    }
#pragma unroll
    for (int pf = 0; pf < 7; ++pf)
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
        acc[pf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[cf], xf[pf], acc[pf][cf], 0, 0, 0);
    // slice t + 1 must have landed before the barrier that publishes it: younger than it are
    // slice t + 2 (2 per wave) and a halo chunk issued at this step or the previous one
    const bool halo_recent = (tap == 0 || tap == 1) && c >= 1 && c + 1 < NC;
    if (!more_w)
      ch_vmwait<0>();
    else if (halo_recent)
      ch_vmwait<2 + HI>();
    else
      ch_vmwait<2>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll 1
  for (int t = 0; t < T; t += 3) {
    step(ic<0>{}, t);
    step(ic<1>{}, t + 1);
    step(ic<2>{}, t + 2);
  }

  // ---- epilogue: + BN shift, ReLU, f16 -> LDS [224 px][128 co] (16-B chunk x stored at
  // x ^ (px & 15)) -> 16-B stores, 16 lanes per 256-B pixel run
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  char* stg = smem;
#pragma unroll
  for (int cf = 0; cf < 4; ++cf) {
    const int col = wco * 64 + cf * 16 + 4 * kc;  // 4 consecutive output channels of the lane
    const float4 bb = *reinterpret_cast<const float4*>(bias + ct * 128 + col);
#pragma unroll
    for (int pf = 0; pf < 7; ++pf) {
      const int q = pfg_of(pf) * 16 + j;
      half4 hv;
      hv[0] = (f16)fmaxf(acc[pf][cf][0] + bb.x, 0.f);
      hv[1] = (f16)fmaxf(acc[pf][cf][1] + bb.y, 0.f);
      hv[2] = (f16)fmaxf(acc[pf][cf][2] + bb.z, 0.f);
      hv[3] = (f16)fmaxf(acc[pf][cf][3] + bb.w, 0.f);
      *reinterpret_cast<half4*>(stg + q * 256 + (((col >> 3) ^ (q & 15)) << 4) + (col & 4) * 2) = hv;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int it = 0; it < 224 * 16 / 256; ++it) {
    const int idx = it * 256 + tid, q = idx >> 4, xq = idx & 15;
    const int g = q / (R * WP), rem = q - g * (R * WP);
    const int r = rem / WP, c = rem - r * WP;
    const int n = ig * G + g;
    const uint4 v = *reinterpret_cast<const uint4*>(stg + q * 256 + ((xq ^ (q & 15)) << 4));
    if (c < HW && n < B && (!(DBG & 2) || v.x == 0x12345678u))
      *reinterpret_cast<uint4*>(y + ((size_t)(n * HW + rb * R + r) * HW + c) * C + ct * 128 + xq * 8) = v;
  }
}

template <int HW, int WP, int P, int R, int G, int C>
static int launch_halo(const f16* x, const f16* w, const float* bias, f16* y, int B, hipStream_t s) {
  using Cf = HaloCfg<HW, WP, P, R, G, C>;
  const int nsp = ((B + G - 1) / G) * Cf::RB;
  const int per8 = 8 / Cf::NCT;  // spatial tiles per group of 8 blocks
  const dim3 grd(8 * ((nsp + per8 - 1) / per8)), blk(256);
#ifdef MEC_PROBES
  switch (opt().conv3x3_debug) {
    case 1: hipLaunchKernelGGL((conv3x3_halo_kernel<HW, WP, P, R, G, C, 1>), grd, blk, 0, s, x, w, bias, y, B); break;
    case 2: hipLaunchKernelGGL((conv3x3_halo_kernel<HW, WP, P, R, G, C, 2>), grd, blk, 0, s, x, w, bias, y, B); break;
    case 4: hipLaunchKernelGGL((conv3x3_halo_kernel<HW, WP, P, R, G, C, 4>), grd, blk, 0, s, x, w, bias, y, B); break;
    case 7: hipLaunchKernelGGL((conv3x3_halo_kernel<HW, WP, P, R, G, C, 7>), grd, blk, 0, s, x, w, bias, y, B); break;
    default: hipLaunchKernelGGL((conv3x3_halo_kernel<HW, WP, P, R, G, C>), grd, blk, 0, s, x, w, bias, y, B);
  }
#else
  hipLaunchKernelGGL((conv3x3_halo_kernel<HW, WP, P, R, G, C>), grd, blk, 0, s, x, w, bias, y, B);
#endif
  MEC_LAUNCH_CHECK();
  return 0;
}

// Routed geometries: 28x28x128 (73 vs 97 us for the GEMM path at B = 256) and 14x14x256 (66 vs
// 74 us). The 7x7x512 instance (four images per tile, 96 KB of LDS: one workgroup per CU) took
// 101 us against the GEMM path's 82 us, so layer4 stays on the GEMM path (not instantiated;
// launch_halo<7, 8, 16, 7, 4, 512> builds it). Probe split at B = 256 (28x28 / 14x14): without the in-loop DMA
// 62 / 55 us, without the fragment reads 63 / 58, MFMAs + barriers alone 49 / 43 (1.2-1.37 PF,
// the chip's clock-limited f16 rate on random data).
bool conv3x3_halo_supported(int H, int C, int N) {
  return N == C && ((H == 28 && C == 128) || (H == 14 && C == 256));
}

int launch_conv3x3_halo(const f16* x, const f16* w, const float* bias, f16* y, int B, int H, int C, hipStream_t s) {
  MEC_REQUIRE(x && w && bias && y && B > 0, "conv3x3_halo: bad arguments");
  if (H == 28 && C == 128) return launch_halo<28, 32, 40, 7, 1, 128>(x, w, bias, y, B, s);
  if (H == 14 && C == 256) return launch_halo<14, 16, 24, 14, 1, 256>(x, w, bias, y, B, s);
  set_error("conv3x3_halo: unsupported geometry (28x28x128, 14x14x256 only)");
  return -1;
}

}  // namespace mec
