// The layer-2 bottleneck seams of the fp32x3 ResNet50 in one kernel each: block i's conv3 (1x1,
// 128 -> 512) + BN shift + identity residual + ReLU, then block i+1's conv1 (1x1, 512 -> N1) + BN
// shift + ReLU on the rows just produced (torchvision Bottleneck.forward, restated by
// oracle/image.py:backbone; the reference builds the network at inference/image_inference.py:57).
// Unfused, the block output's hi / lo planes (411 MB at B = 256) are written by one split GEMM and
// read back in full by the next.
//
// Why a new form and not pw_chain_x3.hip's: that kernel keeps both weight matrices in registers for
// the launch (layer1: 2 x 64 KB of planes) and a tile's whole 256-channel block output in LDS. Here the
// weights are 2 x 256 KB of planes and a 64-row block output 128 KB: neither fits. So a 64-row tile
// walks the block output in 32-channel chunks. Chunk c is
//   X[:, c] = ReLU(T2 . W3[c]^T 2^-e + b3[c] + R[:, c])      (conv3, K = 128, one 32-channel slice)
// stored to HBM (it is the next block's residual) and at once consumed as one 32-deep k step of
//   acc1 += X[:, c] . W1[:, c]^T                              (conv1, accumulated in registers)
// so conv1 sums its k steps in ascending order into one accumulator, each as the split engine's
// three K-interleaved terms (act lo . w hi, act hi . w lo, act hi . w hi), exactly as the split GEMM
// does (gemm_glds.hip SP = 2): both outputs are bit-identical to the two GEMMs
// (tests/test_gpu_fp32x3.py::test_resnet_fp32x3_layer2_seams_bit_identical).
//
// Data movement (one 8-wave workgroup per CU, two waves per SIMD, persistent over 64-row tiles; each
// wave owns one 16-pixel block of the tile: conv3 for 16 of the chunk's channels, conv1 for half of N1,
// so one wave's DMA issue and epilogue run under its partner's MFMAs):
//   * T2 panel of the tile [64][128] hi + lo (32 KB), DMA'd one tile ahead (two buffers) or, for
//     N1 = 256, at the end of the previous tile (one buffer);
//   * per chunk, a weight stage: W3 rows [32][128] + W1 columns [N1][32], both planes (32 / 48 KB),
//     DMA'd one chunk ahead from L2 (the 512-KB weight set is shared by every tile);
//   * per chunk, the residual slice R[:, c] [64][32] both planes (8 KB), DMA'd two chunks ahead; the
//     conv3 epilogue overwrites it in place with X[:, c] (each lane rewrites only the elements it read),
//     which conv1 then reads as its B operand and the whole workgroup stores in 16-B runs.
// Every LDS DMA is global_load_lds_dwordx4 (lane-linear destination, the XOR swizzle applied on the
// source side), waited for with counted vmcnt waits and published with a barrier.
// LDS rows of 16 or more 16-B chunks store chunk c at c ^ (row & 15); rows of 4 chunks (64 B) at
// c ^ ((row >> 2) & 3): the 16 lanes of every ds_read_b128 lane group hit 16 distinct bank slots.
#include <algorithm>

#include "models.h"

namespace mec {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#pragma clang diagnostic ignored "-Winline-asm"
// m0 is listed as clobbered although the compiler reserves it (as pw_chain_x3.hip)
__device__ __forceinline__ void sm_dma(const void* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ uint32_t sm_lds(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
template <typename T>
__device__ __forceinline__ T sm_ld(uint32_t a) {
  return *(const __attribute__((address_space(3))) T*)(uintptr_t)a;
}
template <typename T>
__device__ __forceinline__ void sm_st(uint32_t a, const T& v) {
  *(__attribute__((address_space(3))) T*)(uintptr_t)a = v;
}
template <int N>
__device__ __forceinline__ void sm_wait() {
  static_assert(N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most n of this wave's vector-memory operations are outstanding (n wave-uniform; a smaller
// count than allowed is always safe)
__device__ __forceinline__ void sm_wait_le(int n) {
  if (n >= 17) sm_wait<17>();
  else if (n >= 16) sm_wait<16>();
  else if (n >= 10) sm_wait<10>();
  else if (n >= 8) sm_wait<8>();
  else if (n >= 6) sm_wait<6>();
  else if (n >= 2) sm_wait<2>();
  else if (n >= 1) sm_wait<1>();
  else sm_wait<0>();
}
__device__ __forceinline__ void sm_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int sw16(int row, int c) { return c ^ (row & 15); }
__device__ __forceinline__ int sw4(int row, int c) { return c ^ ((row >> 2) & 3); }

struct SeamX3Args {
  const f16* a;    // conv3's input T2, hi plane [M][K3]
  const f16* r;    // the block input, hi plane [M][N3] (identity residual)
  long long L;     // every activation's lo plane sits L elements after its hi plane
  const f16* w3;   // conv3 weights [N3][K3] hi, lo at + w3_lo
  long long w3_lo;
  float os3;       // 2^-e: undoes the weights' pre-scale
  const float* b3;
  const f16* w1;   // next conv1 weights [N1][N3] hi, lo at + w1_lo
  long long w1_lo;
  float os1;
  const float* b1;
  f16* x;          // block output, hi plane [M][N3]
  f16* t1;         // next conv1 output, hi plane [M][N1]
  unsigned* flag;  // the handle's fp32x3 range flag
  int M, ntiles;   // rows, ceil(M / 64)
};

template <int K3, int N1, int T2B>
__global__ __launch_bounds__(512, 1) void pw_seam_x3_kernel(const SeamX3Args p) {
  constexpr int BM = 64, CC = 32, N3 = 4 * K3, NC = N3 / CC, KS3 = K3 / 32;
  constexpr int CHR = K3 / 8;                       // 16-B chunks per T2 / W3 row
  static_assert(CHR >= 16, "sw16 rows");
  constexpr int T2PL = BM * K3 * 2, T2BUF = 2 * T2PL;
  constexpr int W3PL = CC * K3 * 2, W1PL = N1 * CC * 2, WST = 2 * W3PL + 2 * W1PL;
  constexpr int RPL = BM * CC * 2, RST = 2 * RPL;
  constexpr int NWS = 2, NRS = 3;                   // weight stages (1 chunk ahead), residual slots (2 ahead)
  constexpr int LDS = T2B * T2BUF + NWS * WST + NRS * RST;
  static_assert(LDS + (N3 + N1) * 4 <= 163840, "LDS");
  // per-wave vector-memory operations: DMA instructions of 1 KB (a region's bytes / 1 KB / 8 waves), stores
  constexpr int NB1 = N1 / 32;                      // conv1 16-channel blocks per wave
  constexpr int NT = T2BUF / 8192, NR = RST / 8192, NX = 1, NS1 = NB1 * 2;
  constexpr int I3 = 2 * W3PL / 8192, I1 = 2 * W1PL / 8192;
  static_assert(RST == 512 * 16, "one 16-B X store per thread and chunk");
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  __shared__ __attribute__((aligned(16))) float sb3[N3];
  __shared__ __attribute__((aligned(16))) float sb1[N1];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const uint32_t lds0 = sm_lds(smem);
  const uint32_t t2_0 = lds0, w_0 = lds0 + T2B * T2BUF, r_0 = w_0 + NWS * WST;
  const int G = gridDim.x;
  const int ntk = (p.ntiles - (int)blockIdx.x + G - 1) / G;  // tiles of this workgroup
  const int total = ntk * NC;                                  // chunks of this workgroup
  // wave roles: conv3 channels 16 chb .. +15 of the chunk, conv1 channel blocks nb0 .. nb0 + NB1 - 1,
  // both over pixel block pxb of the tile
  const int chb = wave & 1, pxb = wave >> 1, nb0 = NB1 * (wave & 1);

  for (int i = tid; i < N3; i += 512) sb3[i] = p.b3[i];
  for (int i = tid; i < N1; i += 512) sb1[i] = p.b1[i];
  __syncthreads();

  auto tile_row0 = [&](int k) { return ((int)blockIdx.x + k * G) * BM; };
  auto issue_t2 = [&](int k) {
    const uint32_t base = t2_0 + (k % T2B) * T2BUF;
    const int row0 = tile_row0(k);
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int i = NT * wave + q, pl = i / (T2PL / 1024), s = (i % (T2PL / 1024)) * 64 + lane;
      const int row = s / CHR, sc = sw16(row, s % CHR);
      sm_dma(p.a + pl * p.L + (size_t)min(row0 + row, p.M - 1) * K3 + sc * 8, base + i * 1024);
    }
  };
  auto issue_w = [&](int g) {
    const int c0 = (g % NC) * CC;
    const uint32_t base = w_0 + (g % NWS) * WST;
#pragma unroll
    for (int q = 0; q < I3; ++q) {  // W3 rows c0 .. c0 + 31, all of K3
      const int i = I3 * wave + q, pl = i / (W3PL / 1024), s = (i % (W3PL / 1024)) * 64 + lane;
      const int row = s / CHR, sc = sw16(row, s % CHR);
      sm_dma(p.w3 + pl * p.w3_lo + (size_t)(c0 + row) * K3 + sc * 8, base + i * 1024);
    }
#pragma unroll
    for (int q = 0; q < I1; ++q) {  // W1 columns c0 .. c0 + 31 of every output row
      const int i = I1 * wave + q, pl = i / (W1PL / 1024), s = (i % (W1PL / 1024)) * 64 + lane;
      const int row = s >> 2, sc = sw4(row, s & 3);
      sm_dma(p.w1 + pl * p.w1_lo + (size_t)row * N3 + c0 + sc * 8, base + 2 * W3PL + i * 1024);
    }
  };
  auto issue_r = [&](int g) {
    const int k = g / NC, c0 = (g % NC) * CC, row0 = tile_row0(k);
    const uint32_t base = r_0 + (g % NRS) * RST;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int i = NR * wave + q, pl = i / (RPL / 1024), s = (i % (RPL / 1024)) * 64 + lane;
      const int row = s >> 2, sc = sw4(row, s & 3);
      sm_dma(p.r + pl * p.L + (size_t)min(row0 + row, p.M - 1) * N3 + c0 + sc * 8, base + i * 1024);
    }
  };

  if (total > 0) {
    issue_t2(0);
    issue_w(0);
    issue_r(0);
    if (1 < total) issue_r(1);
  }
  floatx4 acc1[NB1];
#pragma unroll
  for (int q = 0; q < NB1; ++q) acc1[q] = floatx4{0.f, 0.f, 0.f, 0.f};
  bool bad = false;
  int allow = 0;  // vector-memory operations issued after W(g) that may stay in flight at chunk g's wait
  const int px = 16 * pxb + l16;  // this lane's pixel (B-operand column) in the tile
#pragma unroll 1
  for (int g = 0; g < total; ++g) {
    const int k = g / NC, c = g - k * NC, c0 = c * CC, row0 = tile_row0(k);
    sm_wait_le(allow);
    sm_barrier();  // W(g), R(g) (and T2(k)) landed for every wave; chunk g - 1's slots are free
    allow = NX;
    if (g + 1 < total) issue_w(g + 1);
    if (g + 2 < total) {
      issue_r(g + 2);
      allow += NR;
    }
    if (T2B == 2 && c == 0 && k + 1 < ntk) {
      issue_t2(k + 1);
      allow += NT;
    }
    const uint32_t t2b = t2_0 + (k % T2B) * T2BUF;
    const uint32_t wb = w_0 + (g % NWS) * WST;
    const uint32_t rb = r_0 + (g % NRS) * RST;

    // ---- conv3 chunk: X^T[ch][px] = W3[c0 + ch] . T2[px]^T over channels 16 chb .. +15, pixel block pxb
    floatx4 acc3 = {0.f, 0.f, 0.f, 0.f};
    {
      half8 wh[KS3], wl[KS3], xh[KS3], xl[KS3];
      const int wr = 16 * chb + l16;
#pragma unroll
      for (int s = 0; s < KS3; ++s) {
        const int kc = 4 * s + lq;
        const uint32_t wo = wb + wr * (K3 * 2) + (sw16(wr, kc) << 4);
        const uint32_t xo = t2b + px * (K3 * 2) + (sw16(px, kc) << 4);
        wh[s] = sm_ld<half8>(wo);
        wl[s] = sm_ld<half8>(wo + W3PL);
        xh[s] = sm_ld<half8>(xo);
        xl[s] = sm_ld<half8>(xo + T2PL);
      }
#pragma unroll
      for (int s = 0; s < KS3; ++s) {
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[s], xl[s], acc3, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[s], xh[s], acc3, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[s], xh[s], acc3, 0, 0, 0);
      }
    }
    // epilogue: fma(acc, os3, shift) + residual (hi + lo), ReLU, split -> X in place of R in the slot
    {
      const int ch = 16 * chb + 4 * lq;
      const uint32_t ad = rb + px * 64 + (sw4(px, ch >> 3) << 4) + (lq & 1) * 8;
      const half4 rh = sm_ld<half4>(ad), rl = sm_ld<half4>(ad + RPL);
      const float4 bv = *reinterpret_cast<const float4*>(sb3 + c0 + ch);
      const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
      half4 hv, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float rv = (float)rh[e];
        rv += (float)rl[e];
        float v = __builtin_fmaf(acc3[e], p.os3, bb[e]);
        v += rv;
        v = fmaxf(v, 0.f);
        hv[e] = (f16)v;
        lv[e] = (f16)(v - (float)hv[e]);
        bad |= x3_out_of_range(v);
      }
      sm_st(ad, hv);
      sm_st(ad + RPL, lv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sm_barrier();  // X[:, c] complete in the slot
    if (T2B == 1 && c == NC - 1 && k + 1 < ntk) {  // every wave is past its last read of T2(k)
      issue_t2(k + 1);
      allow = NX;  // chunk g + 1 waits for T2(k + 1), issued after everything but this chunk's stores
    }
    // ---- X[:, c] -> HBM: 2 planes x 64 rows x 64 B, one 16-B run per thread
    {
      const int pl = tid >> 8, q = tid & 255, row = q >> 2, cc = q & 3;
      const u32x4 v = sm_ld<u32x4>(rb + pl * RPL + row * 64 + (sw4(row, cc) << 4));
      if (row0 + row < p.M) *reinterpret_cast<u32x4*>(p.x + pl * p.L + (size_t)(row0 + row) * N3 + c0 + cc * 8) = v;
    }
    // ---- conv1 k step c: acc1^T[n][px] += W1[n][c0 ..] . X[px][c0 ..]^T
    {
      const uint32_t xo = rb + px * 64 + (sw4(px, lq) << 4);
      const half8 xh = sm_ld<half8>(xo), xl = sm_ld<half8>(xo + RPL);
      half8 wh[NB1], wl[NB1];
#pragma unroll
      for (int q = 0; q < NB1; ++q) {
        const int n = 16 * (nb0 + q) + l16;
        const uint32_t wo = wb + 2 * W3PL + n * 64 + (sw4(n, lq) << 4);
        wh[q] = sm_ld<half8>(wo);
        wl[q] = sm_ld<half8>(wo + W1PL);
      }
#pragma unroll
      for (int q = 0; q < NB1; ++q) acc1[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[q], xl, acc1[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < NB1; ++q) acc1[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[q], xh, acc1[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < NB1; ++q) acc1[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[q], xh, acc1[q], 0, 0, 0);
    }
    if (c == NC - 1) {
      // conv1 epilogue: fma(acc, os1, shift) + 0, ReLU, split -> T1 rows (4 channels = 8 B per plane and lane)
#pragma unroll
      for (int q = 0; q < NB1; ++q) {
        const int n = 16 * (nb0 + q) + 4 * lq;
        const float4 bv = *reinterpret_cast<const float4*>(sb1 + n);
        const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
        half4 hv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = __builtin_fmaf(acc1[q][e], p.os1, bb[e]);
          v += 0.f;
          v = fmaxf(v, 0.f);
          hv[e] = (f16)v;
          lv[e] = (f16)(v - (float)hv[e]);
          bad |= x3_out_of_range(v);
        }
        if (row0 + px < p.M) {
          f16* o = p.t1 + (size_t)(row0 + px) * N1 + n;
          *reinterpret_cast<half4*>(o) = hv;
          *reinterpret_cast<half4*>(o + p.L) = lv;
        }
        acc1[q] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      allow += NS1;
    }
  }
  sm_wait<0>();  // no DMA into LDS may outlive the workgroup
  x3_raise(p.flag, bad);
}

template <int K3, int N1, int T2B>
void launch_seam(const SeamX3Args& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((pw_seam_x3_kernel<K3, N1, T2B>), dim3(grid), dim3(512), 0, s, a);
}

}  // namespace

int launch_pw_seam_x3(const f16* t2, const f16* xin, long long L, const f16* w3, long long w3_lo, float os3,
                      const float* b3, const f16* w1, long long w1_lo, float os1, const float* b1, f16* xout, f16* t1,
                      int M, int K3, int N1, hipStream_t s) {
  MEC_REQUIRE(M > 0, "pw_seam_x3: no rows");
  MEC_REQUIRE(t2 && xin && w3 && b3 && w1 && b1 && xout && t1 && L > 0, "pw_seam_x3: null pointer");
  MEC_REQUIRE(K3 == 128 && (N1 == 128 || N1 == 256), "pw_seam_x3: shapes K3 = 128, N1 = 128 | 256 only");
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    MEC_HIP(hipGetDevice(&dev));
    MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  SeamX3Args a;
  a.a = t2; a.r = xin; a.L = L;
  a.w3 = w3; a.w3_lo = w3_lo; a.os3 = os3; a.b3 = b3;
  a.w1 = w1; a.w1_lo = w1_lo; a.os1 = os1; a.b1 = b1;
  a.x = xout; a.t1 = t1; a.flag = range_flag();
  a.M = M; a.ntiles = (M + 63) / 64;
  const int grid = std::min(a.ntiles, ncu);
  if (N1 == 128) launch_seam<128, 128, 2>(a, grid, s);
  else launch_seam<128, 256, 1>(a, grid, s);
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
