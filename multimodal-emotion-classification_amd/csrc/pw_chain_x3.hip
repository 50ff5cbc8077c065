// The layer1 bottleneck seams of the fp32x3 ResNet50 in one kernel each (the split-operand form of
// pw_chain.hip): block i's conv3 (1x1, 64 -> 256) + BN shift + residual + ReLU, then block i+1's
// conv1 (1x1, 256 -> N2) + BN shift + ReLU on the rows just produced (torchvision
// Bottleneck.forward, restated by oracle/image.py:backbone). Unfused, the block output's hi / lo
// planes (822 MB at B = 256) are written by one split GEMM and read back by the next; here conv1
// reads them from LDS.
//
//   * DUAL = false: identity residual (layer1 blocks 2 and 3). DUAL = true: layer1 block 1, whose
//     conv3 and downsample run as ONE product over K = [T2 (64) | X0 (64)] with the summed shift
//     (the A_DUAL GEMM's concatenation), no residual.
//   * Persistent: one 4-wave workgroup per CU walks 32-row tiles (rows = NHWC pixels). A tile's
//     operand rows (hi and lo planes of T2 [and X0] and of the residual) arrive by LDS DMA
//     (global_load_lds_dwordx4) two tiles ahead, in three 40-KB (16-KB dual) buffers.
//   * Weights live in registers for the launch, split over the waves: wave w holds conv3 output
//     channels 64w .. 64w+63 and conv1 output channels (N2/4)w .. , both planes, and computes all 32
//     rows of its channels (out^T = W . X^T on v_mfma_f32_16x16x32_f16).
//   * Both products run the split GEMM's K-interleaved terms (per 32-deep k chunk, in this order:
//     act lo . w hi, act hi . w lo, act hi . w hi, into one fp32 accumulator) and its epilogue
//     (fma(acc, oscale, shift) + residual (hi + lo) or + 0, ReLU, hi = f16(v), lo = f16(v - hi)),
//     so both outputs are bit-identical to the two split GEMMs
//     (tests/test_gpu_fp32x3.py::test_resnet_fp32x3_seams_bit_identical).
//   * The block output is written back in place of the residual rows (DUAL: into a staging
//     slot), stored as whole 512-B runs per plane, then read as conv1's operand; conv1's output is
//     staged through the same rows and stored.
// LDS rows of 2^j 16-B chunks store chunk c at c ^ (row & (2^j - 1)) (applied on the DMA source
// side): the 16 lanes of each ds_read_b128 lane group hit 16 distinct bank slots.
#include <algorithm>

#include "models.h"

namespace mec {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// m0 is listed as clobbered although the compiler reserves it: it sets m0 itself before any
// instruction of its own that reads it (see pw_chain.hip)
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void px_dma(const void* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

__device__ __forceinline__ uint32_t px_lds(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

template <typename T>
__device__ __forceinline__ T px_ld(uint32_t a) {
  return *(const __attribute__((address_space(3))) T*)(uintptr_t)a;
}
template <typename T>
__device__ __forceinline__ void px_st(uint32_t a, const T& v) {
  *(__attribute__((address_space(3))) T*)(uintptr_t)a = v;
}

template <int N>
__device__ __forceinline__ void px_wait() {
  static_assert(N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void px_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct PwX3Args {
  const f16* a;   // conv3's input T2, hi plane [M][64]
  const f16* a2;  // DUAL: the block input X0, hi plane [M][64] (the downsample's operand)
  const f16* r;   // !DUAL: the block input, hi plane [M][256] (identity residual)
  long long L;    // every activation's lo plane sits L elements after its hi plane
  const f16* w3;  // conv3 weights [256][K3] hi (DUAL: [W3' | Wds'], K3 = 128), lo at + w3_lo
  long long w3_lo;
  float os3;         // 2^-e: undoes the weights' pre-scale
  const float* b3;   // conv3 shift (DUAL: b3 + bds)
  const f16* w1;     // next conv1 weights [N2][256] hi, lo at + w1_lo
  long long w1_lo;
  float os1;
  const float* b1;
  f16* x;            // block output, hi plane [M][256]
  f16* t1;           // next conv1 output, hi plane [M][N2]
  unsigned* flag;    // the handle's fp32x3 range flag
  int ntiles;        // M / 32
};

template <int N2, bool DUAL>
__global__ __launch_bounds__(256, 1) void pw_chain_x3_kernel(const PwX3Args p) {
  static_assert(N2 == 64 || N2 == 128, "N2");
  constexpr int BM = 32, N3 = 256, K3 = DUAL ? 128 : 64, KS3 = K3 / 32;
  constexpr int ACH = K3 / 8;                    // 16-B chunks per operand row (8 / 16)
  constexpr int APL = BM * K3 * 2;               // bytes per operand plane of a tile (4 / 8 KB)
  constexpr int RPL = BM * N3 * 2;               // bytes per block-output plane of a tile (16 KB)
  constexpr int BUF = DUAL ? 2 * APL : 2 * APL + 2 * RPL;
  constexpr int NB = 3;                          // tile buffers: NB - 1 tiles in flight (dual: 5 measured the same)
  constexpr int STG = DUAL ? 2 * RPL : 0;        // DUAL: separate block-output staging
  constexpr int DMA_PER_TILE = BUF / 16 / 256;   // 10 (4 dual) per lane
  constexpr int T1C = N2 / 8;                    // 16-B chunks per conv1 output row
  constexpr int T1PL = BM * N2 * 2;              // bytes per conv1-output plane of a tile
  constexpr int ST_X = 2 * RPL / 16 / 256;       // 8 stores per lane per tile
  constexpr int ST_T1 = 2 * T1PL / 16 / 256;     // 2 / 4
  constexpr int CF3 = 4, CF1 = N2 / 64;          // 16-channel fragments per wave
  __shared__ __attribute__((aligned(16))) char smem[NB * BUF + STG];
  __shared__ float sb3[N3], sb1[N2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const uint32_t lds0 = px_lds(smem);

  for (int i = tid; i < N3; i += 256) sb3[i] = p.b3[i];
  if (tid < N2) sb1[tid] = p.b1[tid];
  // A fragments [plane][cf][k step]: co = 64 wave + 16 cf + l16 (conv3), (N2/4) wave + 16 cf + l16
  // (conv1); k = 32 s + 8 lq .. +7
  half8 wf3[2][CF3][KS3], wf1[2][CF1][8];
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)
#pragma unroll
    for (int cf = 0; cf < CF3; ++cf)
#pragma unroll
      for (int s = 0; s < KS3; ++s)
        wf3[pl][cf][s] = *reinterpret_cast<const half8*>(p.w3 + pl * p.w3_lo +
                                                         (size_t)(64 * wave + 16 * cf + l16) * K3 + 32 * s + 8 * lq);
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)
#pragma unroll
    for (int cf = 0; cf < CF1; ++cf)
#pragma unroll
      for (int s = 0; s < 8; ++s)
        wf1[pl][cf][s] = *reinterpret_cast<const half8*>(p.w1 + pl * p.w1_lo +
                                                         (size_t)((N2 / 4) * wave + 16 * cf + l16) * N3 + 32 * s + 8 * lq);

  // one tile's operand rows (both planes) into buffer b
  auto issue = [&](int t, int b) {
    const uint32_t base = lds0 + b * BUF;
    const size_t row0 = (size_t)t * BM;
    if constexpr (!DUAL) {
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {  // T2: 32 rows x 8 chunks per plane
        const int row = tid >> 3, c = (tid & 7) ^ (row & 7);
        px_dma(p.a + pl * p.L + (row0 + row) * 64 + c * 8, base + pl * APL + (uint32_t)(wave * 64) * 16u);
      }
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // residual: 32 rows x 32 chunks per plane
          const int q = i * 256 + tid, row = q >> 5, c = (q & 31) ^ (row & 15);
          px_dma(p.r + pl * p.L + (row0 + row) * N3 + c * 8,
                 base + 2 * APL + pl * RPL + (uint32_t)(i * 256 + wave * 64) * 16u);
        }
    } else {
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // [T2 | X0]: 32 rows x 16 chunks per plane
          const int q = i * 256 + tid, row = q >> 4, c = (q & 15) ^ (row & 15);
          const f16* src = c < 8 ? p.a + pl * p.L + (row0 + row) * 64 + c * 8
                                 : p.a2 + pl * p.L + (row0 + row) * 64 + (c - 8) * 8;
          px_dma(src, base + pl * APL + (uint32_t)(i * 256 + wave * 64) * 16u);
        }
    }
  };

  int t = blockIdx.x;
  const int G = gridDim.x;
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (t + k * G < p.ntiles) issue(t + k * G, k);
  __syncthreads();  // shifts in LDS
  int b = 0, prev_stores = 0;
  bool bad = false;
#pragma unroll 1
  for (; t < p.ntiles; t += G) {
    // in flight, in issue order: this tile's DMAs, those of the `ahead` later tiles issued so far,
    // the previous tile's stores: wait until only the last two groups remain
    const int ahead = min(NB - 2, (p.ntiles - 1 - t) / G);
    if (prev_stores) {
      if (NB > 4 && ahead == 3) px_wait<3 * DMA_PER_TILE + ST_X + ST_T1>();
      else if (NB > 3 && ahead == 2) px_wait<2 * DMA_PER_TILE + ST_X + ST_T1>();
      else if (ahead == 1) px_wait<DMA_PER_TILE + ST_X + ST_T1>();
      else px_wait<ST_X + ST_T1>();
    } else {
      if (NB > 4 && ahead == 3) px_wait<3 * DMA_PER_TILE>();
      else if (NB > 3 && ahead == 2) px_wait<2 * DMA_PER_TILE>();
      else if (ahead == 1) px_wait<DMA_PER_TILE>();
      else px_wait<0>();
    }
    px_barrier();  // every wave's DMA for tile t landed; buffer (b - 1) and the staging rows are free
    if (t + (NB - 1) * G < p.ntiles) issue(t + (NB - 1) * G, (b + NB - 1) % NB);
    const uint32_t ab = lds0 + b * BUF;
    const uint32_t rb = DUAL ? lds0 + NB * BUF : ab + 2 * APL;

    // ---- conv3: out^T[co][px] over this wave's 64 channels x 32 rows
    floatx4 acc[2][CF3];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int cf = 0; cf < CF3; ++cf) acc[j][cf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS3; ++s) {
      half8 xh[2], xl[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 16 * j + l16, kc = 4 * s + lq;
        const uint32_t off = row * (2 * K3) + ((kc ^ (row & (ACH - 1))) << 4);
        xh[j] = px_ld<half8>(ab + off);
        xl[j] = px_ld<half8>(ab + APL + off);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < CF3; ++cf)
          acc[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf3[0][cf][s], xl[j], acc[j][cf], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < CF3; ++cf)
          acc[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf3[1][cf][s], xh[j], acc[j][cf], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < CF3; ++cf)
          acc[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf3[0][cf][s], xh[j], acc[j][cf], 0, 0, 0);
    }
    // epilogue: fma(acc, os3, shift) + residual (hi + lo) or + 0, ReLU, split -> block-output rows
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 16 * j + l16;
#pragma unroll
      for (int cf = 0; cf < CF3; ++cf) {
        const int co = 64 * wave + 16 * cf + 4 * lq;
        const uint32_t ad = rb + row * 512 + (((co >> 3) ^ (row & 15)) << 4) + (lq & 1) * 8;
        float rv[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (!DUAL) {
          const half4 rh = px_ld<half4>(ad), rl = px_ld<half4>(ad + RPL);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rv[e] = (float)rh[e];
            rv[e] += (float)rl[e];
          }
        }
        half4 hv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = __builtin_fmaf(acc[j][cf][e], p.os3, sb3[co + e]);
          v += rv[e];
          v = fmaxf(v, 0.f);
          hv[e] = (f16)v;
          lv[e] = (f16)(v - (float)hv[e]);
          bad |= x3_out_of_range(v);
        }
        px_st(ad, hv);
        px_st(ad + RPL, lv);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    px_barrier();  // the tile's block output is complete in LDS

    // ---- block output -> HBM: per plane, whole 512-B rows
    {
      f16* xo = p.x + (size_t)t * BM * N3;
#pragma unroll
      for (int i = 0; i < ST_X; ++i) {
        const int pl = i / (ST_X / 2);
        const int q = (i % (ST_X / 2)) * 256 + tid, rr = q >> 5, c = q & 31;
        const u32x4 v = px_ld<u32x4>(rb + pl * RPL + rr * 512 + ((c ^ (rr & 15)) << 4));
        *reinterpret_cast<u32x4*>(xo + pl * p.L + (size_t)q * 8) = v;
      }
    }
    // ---- conv1 of the next block over this wave's N2/4 channels x 32 rows (k = 0..255)
    floatx4 acc1[2][CF1];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int cf = 0; cf < CF1; ++cf) acc1[j][cf] = floatx4{0.f, 0.f, 0.f, 0.f};
    half8 xf[2][2][2];  // [register set][plane][row block]: step s+1 is read before step s's MFMAs
    auto rd1 = [&](int s, int k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 16 * j + l16, kc = 4 * s + lq;
        const uint32_t off = row * 512 + ((kc ^ (row & 15)) << 4);
        xf[k][0][j] = px_ld<half8>(rb + off);
        xf[k][1][j] = px_ld<half8>(rb + RPL + off);
      }
    };
    rd1(0, 0);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s + 1 < 8) rd1(s + 1, (s + 1) & 1);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < CF1; ++cf)
          acc1[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[0][cf][s], xf[s & 1][1][j], acc1[j][cf], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < CF1; ++cf)
          acc1[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[1][cf][s], xf[s & 1][0][j], acc1[j][cf], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < CF1; ++cf)
          acc1[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[0][cf][s], xf[s & 1][0][j], acc1[j][cf], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    px_barrier();  // every wave is done reading the block-output rows
    // conv1 epilogue: fma(acc, os1, shift) + 0, ReLU, split -> staged [32][N2] rows per plane
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 16 * j + l16;
#pragma unroll
      for (int cf = 0; cf < CF1; ++cf) {
        const int co = (N2 / 4) * wave + 16 * cf + 4 * lq;
        const uint32_t ad = rb + row * (N2 * 2) + (((co >> 3) ^ (row & (T1C - 1))) << 4) + (lq & 1) * 8;
        half4 hv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = __builtin_fmaf(acc1[j][cf][e], p.os1, sb1[co + e]);
          v += 0.f;
          v = fmaxf(v, 0.f);
          hv[e] = (f16)v;
          lv[e] = (f16)(v - (float)hv[e]);
          bad |= x3_out_of_range(v);
        }
        px_st(ad, hv);
        px_st(ad + T1PL, lv);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    px_barrier();
    {
      f16* to = p.t1 + (size_t)t * BM * N2;
#pragma unroll
      for (int i = 0; i < ST_T1; ++i) {
        const int pl = i / (ST_T1 / 2);
        const int q = (i % (ST_T1 / 2)) * 256 + tid, rr = q / T1C, c = q % T1C;
        const u32x4 v = px_ld<u32x4>(rb + pl * T1PL + rr * (N2 * 2) + ((c ^ (rr & (T1C - 1))) << 4));
        *reinterpret_cast<u32x4*>(to + pl * p.L + (size_t)q * 8) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    prev_stores = 1;
    b = (b + 1) % NB;
  }
  x3_raise(p.flag, bad);
}

}  // namespace

int launch_pw_chain_x3(const f16* t2, const f16* xin, long long L, const f16* w3, long long w3_lo, float os3,
                       const float* b3, const f16* w1, long long w1_lo, float os1, const float* b1, f16* xout, f16* t1,
                       int M, int N2, bool dual, hipStream_t s) {
  MEC_REQUIRE(M > 0 && M % 32 == 0, "pw_chain_x3: rows must be a multiple of 32");
  MEC_REQUIRE(t2 && xin && w3 && b3 && w1 && b1 && xout && t1 && L > 0, "pw_chain_x3: null pointer");
  MEC_REQUIRE(N2 == 64 || (N2 == 128 && !dual), "pw_chain_x3: N2 must be 64 (or 128 without the downsample)");
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    MEC_HIP(hipGetDevice(&dev));
    MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  PwX3Args a;
  a.a = t2; a.a2 = dual ? xin : nullptr; a.r = dual ? nullptr : xin; a.L = L;
  a.w3 = w3; a.w3_lo = w3_lo; a.os3 = os3; a.b3 = b3;
  a.w1 = w1; a.w1_lo = w1_lo; a.os1 = os1; a.b1 = b1;
  a.x = xout; a.t1 = t1; a.flag = range_flag(); a.ntiles = M / 32;
  const dim3 grd(std::min(a.ntiles, ncu)), blk(256);
  if (dual) hipLaunchKernelGGL((pw_chain_x3_kernel<64, true>), grd, blk, 0, s, a);
  else if (N2 == 64) hipLaunchKernelGGL((pw_chain_x3_kernel<64, false>), grd, blk, 0, s, a);
  else hipLaunchKernelGGL((pw_chain_x3_kernel<128, false>), grd, blk, 0, s, a);
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
