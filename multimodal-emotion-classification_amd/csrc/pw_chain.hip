// The seam between two ResNet50 layer1 bottlenecks in one kernel: block i's conv3 (1x1,
// 64 -> 256) + BN shift + identity residual + ReLU, then block i+1's conv1 (1x1, 256 -> N2)
// + BN shift + ReLU on the rows just produced (torchvision Bottleneck.forward, restated by
// oracle/image.py:backbone). Unfused, the 256-channel block output (411 MB at B = 256) is
// written by one GEMM and read back by the next; here it is read back from LDS.
//
// Persistent: one 4-wave workgroup per CU walks 64-row tiles (rows = NHWC pixels).
//   * conv3's weights (256 x 64 f16) live in registers for the launch: every wave holds all
//     256 output channels (16 x 2 A fragments) for its 16 pixel rows;
//   * each tile's T2 rows (64 x 128 B) and residual rows (64 x 512 B) arrive by LDS DMA
//     (global_load_lds_dwordx4) NB - 1 tiles ahead;
//   * conv3's epilogue rewrites the residual rows in place with the block output (f16), which
//     is then (a) stored as whole 1-KB runs and (b) the B operand of conv1, whose weights
//     (N2 x 256 f16) sit in LDS; conv1's output is staged through the same rows and stored;
//   * both products run the A_PLAIN GEMM's k order (32-deep steps on
//     v_mfma_f32_16x16x32_f16, out^T = W . X^T) and epilogue ((acc + bias) + residual, ReLU,
//     f16), so both outputs are bit-identical to the two GEMMs
//     (tests/test_gpu_kernels.py::test_pw_chain_bit_identical).
// LDS rows of 2^j 16-B chunks store chunk c at c ^ (row & (2^j - 1)) (applied on the DMA
// source side): 16 consecutive rows at one chunk hit 16 distinct bank slots.
#include <algorithm>

#include "models.h"

namespace mec {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int PC_BM = 64, PC_K3 = 64, PC_N3 = 256;
constexpr int PC_AB = PC_BM * PC_K3 * 2;   // T2 rows per tile (bytes)
constexpr int PC_RB = PC_BM * PC_N3 * 2;   // residual / output rows per tile (bytes)
constexpr int PC_BUF = PC_AB + PC_RB;      // one tile buffer (40 KB)

// m0 is listed as clobbered although the compiler reserves it: it sets m0 itself before any
// instruction of its own that reads it
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void pc_dma(const void* src, uint32_t lds) {
  // LDS DMA from inline asm: hidden from hipcc's waitcnt pass, which would otherwise drain
  // lgkmcnt(0) before every LDS read while a DMA is in flight (see conv3x3.hip)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

__device__ __forceinline__ uint32_t pc_lds(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

template <typename T>
__device__ __forceinline__ T pc_ld(uint32_t a) {
  return *(const __attribute__((address_space(3))) T*)(uintptr_t)a;
}
template <typename T>
__device__ __forceinline__ void pc_st(uint32_t a, const T& v) {
  *(__attribute__((address_space(3))) T*)(uintptr_t)a = v;
}

template <int N2>
__global__ __launch_bounds__(256, 1) void pw_chain_kernel(const f16* __restrict__ a, const f16* __restrict__ r,
                                                          const f16* __restrict__ w3, const float* __restrict__ b3,
                                                          const f16* __restrict__ w1, const float* __restrict__ b1,
                                                          f16* __restrict__ x, f16* __restrict__ t1, int ntiles) {
  static_assert(N2 == 64 || N2 == 128, "N2");
  constexpr int NB = N2 == 64 ? 3 : 2;        // tile buffers (LDS: NB x 40 KB + N2 x 512 B)
  constexpr int W1B = N2 * PC_N3 * 2;
  constexpr int DMA_PER_TILE = (PC_AB + PC_RB) / 16 / 256;  // 10 per lane
  constexpr int T1C = N2 / 8;                 // 16-B chunks per conv1 output row
  constexpr int ST_X = PC_RB / 16 / 256, ST_T1 = PC_BM * T1C / 256;  // stores per lane per tile
  __shared__ __attribute__((aligned(16))) char smem[NB * PC_BUF + W1B];
  __shared__ float sb3[PC_N3], sb1[N2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const uint32_t lds0 = pc_lds(smem), ldsw1 = lds0 + NB * PC_BUF;

  // ---- per-launch constants: conv1 weights + biases -> LDS, conv3 weights -> registers
#pragma unroll
  for (int i = 0; i < W1B / 16 / 256; ++i) {
    const int q = i * 256 + tid, row = q / 32, c = q % 32;  // 32 chunks per 512-B row
    const u32x4 v = reinterpret_cast<const u32x4*>(w1)[q];
    pc_st(ldsw1 + row * 512 + ((c ^ (row & 15)) << 4), v);
  }
  for (int i = tid; i < PC_N3; i += 256) sb3[i] = b3[i];
  if (tid < N2) sb1[tid] = b1[tid];
  half8 wf[16][2];  // A fragments: co = 16 cf + l16, k = 32 s + 8 lq .. +7
#pragma unroll
  for (int cf = 0; cf < 16; ++cf)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      wf[cf][s] = *reinterpret_cast<const half8*>(w3 + (size_t)(16 * cf + l16) * PC_K3 + 32 * s + 8 * lq);
#pragma unroll
  for (int cf = 0; cf < 16; ++cf)
#pragma unroll
    for (int s = 0; s < 2; ++s) asm volatile("" : "+v"(wf[cf][s]));  // resident: never re-loaded in the loop

  // one tile's T2 rows (8 chunks per 128-B row) and residual rows (32 chunks per 512-B row)
  auto issue = [&](int t, int b) {
    const uint32_t base = lds0 + b * PC_BUF;
    const f16* at = a + (size_t)t * PC_BM * PC_K3;
    const f16* rt = r + (size_t)t * PC_BM * PC_N3;
#pragma unroll
    for (int i = 0; i < PC_AB / 16 / 256; ++i) {
      const int q = i * 256 + tid, row = q >> 3, c = (q & 7) ^ (row & 7);
      pc_dma(at + row * PC_K3 + c * 8, base + (uint32_t)(i * 256 + wave * 64) * 16u);
    }
#pragma unroll
    for (int i = 0; i < PC_RB / 16 / 256; ++i) {
      const int q = i * 256 + tid, row = q >> 5, c = (q & 31) ^ (row & 15);
      pc_dma(rt + row * PC_N3 + c * 8, base + PC_AB + (uint32_t)(i * 256 + wave * 64) * 16u);
    }
  };

  int t = blockIdx.x;
  const int G = gridDim.x;
  // prologue: NB - 1 tiles in flight
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (t + k * G < ntiles) issue(t + k * G, k);
  __syncthreads();  // weights / biases in LDS (the DMAs stay in flight: no vmcnt drain here)
  int b = 0, prev_stores = 0;
  const int row = 16 * wave + l16;  // this lane's pixel row within a tile (B operand)
#pragma unroll 1
  for (; t < ntiles; t += G) {
    // tile t landed: allow the later tiles' DMAs and the previous tile's stores in flight
    const bool ahead = NB == 3 && t + G < ntiles;
    if (ahead) {
      if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE + ST_X + ST_T1) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE) : "memory");
    } else {
      if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST_X + ST_T1) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMA for tile t landed; buffer (b-1) is free
    if (t + (NB - 1) * G < ntiles) issue(t + (NB - 1) * G, (b + NB - 1) % NB);
    const uint32_t ab = lds0 + b * PC_BUF, rb = ab + PC_AB;

    // ---- conv3: out^T[co][px] over k = 0..63 (two 32-deep steps)
    floatx4 acc[16];
#pragma unroll
    for (int cf = 0; cf < 16; ++cf) acc[cf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const half8 xf = pc_ld<half8>(ab + row * 128 + (((4 * s + lq) ^ (row & 7)) << 4));
#pragma unroll
      for (int cf = 0; cf < 16; ++cf) acc[cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[cf][s], xf, acc[cf], 0, 0, 0);
    }
    // epilogue: (acc + bias) + residual, ReLU, f16 -> back into the residual's LDS slot
#pragma unroll
    for (int cf = 0; cf < 16; ++cf) {
      const int co = 16 * cf + 4 * lq;
      const uint32_t ad = rb + row * 512 + (((2 * cf + (lq >> 1)) ^ (row & 15)) << 4) + (lq & 1) * 8;
      const half4 rv = pc_ld<half4>(ad);
      half4 hv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[cf][e] + sb3[co + e];
        v += (float)rv[e];
        hv[e] = (f16)fmaxf(v, 0.f);
      }
      pc_st(ad, hv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the tile's block output is complete in LDS

    // ---- block output rows -> HBM (whole 1-KB runs)
    {
      f16* xo = x + (size_t)t * PC_BM * PC_N3;
#pragma unroll
      for (int i = 0; i < ST_X; ++i) {
        const int q = i * 256 + tid, rr = q >> 5, c = q & 31;
        const u32x4 v = pc_ld<u32x4>(rb + rr * 512 + ((c ^ (rr & 15)) << 4));
        *reinterpret_cast<u32x4*>(xo + (size_t)q * 8) = v;
      }
    }
    // ---- conv1 of the next block: out^T[co][px] over k = 0..255 (eight 32-deep steps)
    floatx4 acc1[N2 / 16];
#pragma unroll
    for (int cf = 0; cf < N2 / 16; ++cf) acc1[cf] = floatx4{0.f, 0.f, 0.f, 0.f};
    // fragments of step s+1 are read before step s's MFMAs (two register sets)
    half8 xf[2], wv[2][N2 / 16];
    auto rd1 = [&](int s, int k) {
      const int kc = 4 * s + lq;
      xf[k] = pc_ld<half8>(rb + row * 512 + ((kc ^ (row & 15)) << 4));
#pragma unroll
      for (int cf = 0; cf < N2 / 16; ++cf) {
        const int co = 16 * cf + l16;
        wv[k][cf] = pc_ld<half8>(ldsw1 + co * 512 + ((kc ^ (co & 15)) << 4));
      }
    };
    rd1(0, 0);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s + 1 < 8) rd1(s + 1, (s + 1) & 1);
#pragma unroll
      for (int cf = 0; cf < N2 / 16; ++cf)
        acc1[cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wv[s & 1][cf], xf[s & 1], acc1[cf], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading the block-output rows
    // conv1 epilogue: (acc + bias) + 0, ReLU, f16 -> staged [64][N2] rows in the same slot
#pragma unroll
    for (int cf = 0; cf < N2 / 16; ++cf) {
      const int co = 16 * cf + 4 * lq;
      half4 hv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc1[cf][e] + sb1[co + e];
        v += 0.f;
        hv[e] = (f16)fmaxf(v, 0.f);
      }
      pc_st(rb + row * (N2 * 2) + (((2 * cf + (lq >> 1)) ^ (row & (T1C - 1))) << 4) + (lq & 1) * 8, hv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      f16* to = t1 + (size_t)t * PC_BM * N2;
#pragma unroll
      for (int i = 0; i < ST_T1; ++i) {
        const int q = i * 256 + tid, rr = q / T1C, c = q % T1C;
        const u32x4 v = pc_ld<u32x4>(rb + rr * (N2 * 2) + ((c ^ (rr & (T1C - 1))) << 4));
        *reinterpret_cast<u32x4*>(to + (size_t)q * 8) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    prev_stores = 1;
    b = (b + 1) % NB;
  }
}

// Register-weight form of the residual seam: both products' weights live in registers, split
// over the waves: wave (h, g) holds conv3 channels 128h .. 128h+127 (8 x 2 A fragments) and
// conv1 channels (N2/2)h .. (N2/2)(h+1) - 1 ((N2/32) x 8 A fragments) and computes tile rows
// 32g .. 32g+31 of both. No weights in LDS, so three 40-KB tile buffers fit at any N2.
template <int N2>
__global__ __launch_bounds__(256, 1) void pw_chain2_kernel(const f16* __restrict__ a, const f16* __restrict__ r,
                                                           const f16* __restrict__ w3, const float* __restrict__ b3,
                                                           const f16* __restrict__ w1, const float* __restrict__ b1,
                                                           f16* __restrict__ x, f16* __restrict__ t1, int ntiles) {
  static_assert(N2 == 64 || N2 == 128, "N2");
  constexpr int NB = 3;
  constexpr int DMA_PER_TILE = (PC_AB + PC_RB) / 16 / 256;  // 10 per lane
  constexpr int T1C = N2 / 8;
  constexpr int ST_X = PC_RB / 16 / 256, ST_T1 = PC_BM * T1C / 256;
  constexpr int CF1 = N2 / 32;  // conv1 16-channel fragments per wave
  __shared__ __attribute__((aligned(16))) char smem[NB * PC_BUF];
  __shared__ float sb3[PC_N3], sb1[N2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int h = wave & 1, g = wave >> 1;
  const uint32_t lds0 = pc_lds(smem);

  for (int i = tid; i < PC_N3; i += 256) sb3[i] = b3[i];
  if (tid < N2) sb1[tid] = b1[tid];
  half8 wf3[8][2], wf1[CF1][8];
#pragma unroll
  for (int cf = 0; cf < 8; ++cf)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      wf3[cf][s] = *reinterpret_cast<const half8*>(w3 + (size_t)(128 * h + 16 * cf + l16) * PC_K3 + 32 * s + 8 * lq);
#pragma unroll
  for (int cf = 0; cf < CF1; ++cf)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      wf1[cf][s] = *reinterpret_cast<const half8*>(w1 + (size_t)((N2 / 2) * h + 16 * cf + l16) * PC_N3 + 32 * s + 8 * lq);
#pragma unroll
  for (int cf = 0; cf < 8; ++cf)
#pragma unroll
    for (int s = 0; s < 2; ++s) asm volatile("" : "+v"(wf3[cf][s]));
#pragma unroll
  for (int cf = 0; cf < CF1; ++cf)
#pragma unroll
    for (int s = 0; s < 8; ++s) asm volatile("" : "+v"(wf1[cf][s]));

  auto issue = [&](int t, int b) {
    const uint32_t base = lds0 + b * PC_BUF;
    const f16* at = a + (size_t)t * PC_BM * PC_K3;
    const f16* rt = r + (size_t)t * PC_BM * PC_N3;
#pragma unroll
    for (int i = 0; i < PC_AB / 16 / 256; ++i) {
      const int q = i * 256 + tid, row = q >> 3, c = (q & 7) ^ (row & 7);
      pc_dma(at + row * PC_K3 + c * 8, base + (uint32_t)(i * 256 + wave * 64) * 16u);
    }
#pragma unroll
    for (int i = 0; i < PC_RB / 16 / 256; ++i) {
      const int q = i * 256 + tid, row = q >> 5, c = (q & 31) ^ (row & 15);
      pc_dma(rt + row * PC_N3 + c * 8, base + PC_AB + (uint32_t)(i * 256 + wave * 64) * 16u);
    }
  };

  int t = blockIdx.x;
  const int G = gridDim.x;
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (t + k * G < ntiles) issue(t + k * G, k);
  __syncthreads();
  int b = 0, prev_stores = 0;
#pragma unroll 1
  for (; t < ntiles; t += G) {
    const bool ahead = t + G < ntiles;
    if (ahead) {
      if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE + ST_X + ST_T1) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE) : "memory");
    } else {
      if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST_X + ST_T1) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (t + (NB - 1) * G < ntiles) issue(t + (NB - 1) * G, (b + NB - 1) % NB);
    const uint32_t ab = lds0 + b * PC_BUF, rb = ab + PC_AB;

    // ---- conv3 over this wave's 128 channels x 32 rows
    floatx4 acc[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int cf = 0; cf < 8; ++cf) acc[j][cf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 xf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rw = 32 * g + 16 * j + l16;
        xf[j] = pc_ld<half8>(ab + rw * 128 + (((4 * s + lq) ^ (rw & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < 8; ++cf)
          acc[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf3[cf][s], xf[j], acc[j][cf], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rw = 32 * g + 16 * j + l16;
#pragma unroll
      for (int cf = 0; cf < 8; ++cf) {
        const int co = 128 * h + 16 * cf + 4 * lq;
        const uint32_t ad = rb + rw * 512 + (((co >> 3) ^ (rw & 15)) << 4) + (lq & 1) * 8;
        const half4 rv = pc_ld<half4>(ad);
        half4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[j][cf][e] + sb3[co + e];
          v += (float)rv[e];
          hv[e] = (f16)fmaxf(v, 0.f);
        }
        pc_st(ad, hv);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      f16* xo = x + (size_t)t * PC_BM * PC_N3;
#pragma unroll
      for (int i = 0; i < ST_X; ++i) {
        const int q = i * 256 + tid, rr = q >> 5, c = q & 31;
        const u32x4 v = pc_ld<u32x4>(rb + rr * 512 + ((c ^ (rr & 15)) << 4));
        *reinterpret_cast<u32x4*>(xo + (size_t)q * 8) = v;
      }
    }
    // ---- conv1 over this wave's N2/2 channels x 32 rows (k = 0..255)
    floatx4 acc1[2][CF1];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int cf = 0; cf < CF1; ++cf) acc1[j][cf] = floatx4{0.f, 0.f, 0.f, 0.f};
    half8 xf[2][2];
    auto rd1 = [&](int s, int k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rw = 32 * g + 16 * j + l16;
        xf[k][j] = pc_ld<half8>(rb + rw * 512 + (((4 * s + lq) ^ (rw & 15)) << 4));
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
          acc1[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[cf][s], xf[s & 1][j], acc1[j][cf], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rw = 32 * g + 16 * j + l16;
#pragma unroll
      for (int cf = 0; cf < CF1; ++cf) {
        const int co = (N2 / 2) * h + 16 * cf + 4 * lq;
        half4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc1[j][cf][e] + sb1[co + e];
          v += 0.f;
          hv[e] = (f16)fmaxf(v, 0.f);
        }
        pc_st(rb + rw * (N2 * 2) + (((co >> 3) ^ (rw & (T1C - 1))) << 4) + (lq & 1) * 8, hv);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      f16* to = t1 + (size_t)t * PC_BM * N2;
#pragma unroll
      for (int i = 0; i < ST_T1; ++i) {
        const int q = i * 256 + tid, rr = q / T1C, c = q % T1C;
        const u32x4 v = pc_ld<u32x4>(rb + rr * (N2 * 2) + ((c ^ (rr & (T1C - 1))) << 4));
        *reinterpret_cast<u32x4*>(to + (size_t)q * 8) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    prev_stores = 1;
    b = (b + 1) % NB;
  }
}

// 0: per-N2 default (N2 = 64: LDS-weight form; N2 = 128: register-weight form), 1: LDS-weight
// form, 2: register-weight form. At N2 = 64 the two forms time the same (3.826 / 3.828 ms for
// the image encoder); at N2 = 128 the LDS-weight form holds only two tile buffers.

int launch_pw_chain(const f16* t2, const f16* xin, const f16* w3, const float* b3, const f16* w1, const float* b1,
                    f16* xout, f16* t1, int M, int N2, hipStream_t s) {
  MEC_REQUIRE(M > 0 && M % PC_BM == 0, "pw_chain: rows must be a multiple of 64");
  MEC_REQUIRE(t2 && xin && w3 && b3 && w1 && b1 && xout && t1, "pw_chain: null pointer");
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    MEC_HIP(hipGetDevice(&dev));
    MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int ntiles = M / PC_BM;
  const dim3 grd(std::min(ntiles, ncu)), blk(256);
  const int form = opt().pw_chain_form ? opt().pw_chain_form : (N2 == 64 ? 1 : 2);
  if (N2 == 64 && form == 1)
    hipLaunchKernelGGL(pw_chain_kernel<64>, grd, blk, 0, s, t2, xin, w3, b3, w1, b1, xout, t1, ntiles);
  else if (N2 == 64)
    hipLaunchKernelGGL(pw_chain2_kernel<64>, grd, blk, 0, s, t2, xin, w3, b3, w1, b1, xout, t1, ntiles);
  else if (N2 == 128 && form == 1)
    hipLaunchKernelGGL(pw_chain_kernel<128>, grd, blk, 0, s, t2, xin, w3, b3, w1, b1, xout, t1, ntiles);
  else if (N2 == 128)
    hipLaunchKernelGGL(pw_chain2_kernel<128>, grd, blk, 0, s, t2, xin, w3, b3, w1, b1, xout, t1, ntiles);
  else {
    set_error("pw_chain: N2 must be 64 or 128");
    return -1;
  }
  MEC_LAUNCH_CHECK();
  return 0;
}

// Block 1 -> block 2 seam of layer1: block 1's conv3 and its downsample projection as ONE
// product over K = [T2 (64) | X0 (64)] (the A_DUAL GEMM's concatenation: bn3(conv3(t)) +
// bn_ds(conv_ds(x)) = [t | x] . [W3' | Wds']^T + (b3 + bds)) + ReLU, then block 2's conv1
// (256 -> 64) + ReLU on the rows just produced. No residual rows to stream: the tile's input
// is 64 x 256 B (T2 | X0), its outputs 64 x 512 B (block output) and 64 x 128 B (conv1).
// conv3 weights (256 x 128) are split over the waves: wave (h, g) holds output channels
// 128h .. 128h+127 (8 x 4 A fragments in registers) for tile rows 32g .. 32g+31.
__global__ __launch_bounds__(256, 1) void pw_chain_dual_kernel(const f16* __restrict__ a, const f16* __restrict__ a2,
                                                               const f16* __restrict__ w3, const float* __restrict__ b3,
                                                               const f16* __restrict__ w1, const float* __restrict__ b1,
                                                               f16* __restrict__ x, f16* __restrict__ t1, int ntiles) {
  constexpr int N2 = 64, NB = 3, K3 = 128;
  constexpr int AB = PC_BM * K3 * 2;          // 16 KB of [T2 | X0] rows per tile
  constexpr int W1B = N2 * PC_N3 * 2;
  constexpr int DMA_PER_TILE = AB / 16 / 256;  // 4 per lane
  constexpr int T1C = N2 / 8;
  constexpr int ST_X = PC_RB / 16 / 256, ST_T1 = PC_BM * T1C / 256;
  __shared__ __attribute__((aligned(16))) char smem[NB * AB + PC_RB + W1B];
  __shared__ float sb3[PC_N3], sb1[N2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int h = wave & 1, g = wave >> 1;
  const uint32_t lds0 = pc_lds(smem), rb = lds0 + NB * AB, ldsw1 = rb + PC_RB;

#pragma unroll
  for (int i = 0; i < W1B / 16 / 256; ++i) {
    const int q = i * 256 + tid, row = q / 32, c = q % 32;
    const u32x4 v = reinterpret_cast<const u32x4*>(w1)[q];
    pc_st(ldsw1 + row * 512 + ((c ^ (row & 15)) << 4), v);
  }
  for (int i = tid; i < PC_N3; i += 256) sb3[i] = b3[i];
  if (tid < N2) sb1[tid] = b1[tid];
  half8 wf[8][4];  // A fragments: co = 128h + 16cf + l16, k = 32s + 8lq .. +7
#pragma unroll
  for (int cf = 0; cf < 8; ++cf)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      wf[cf][s] = *reinterpret_cast<const half8*>(w3 + (size_t)(128 * h + 16 * cf + l16) * K3 + 32 * s + 8 * lq);
#pragma unroll
  for (int cf = 0; cf < 8; ++cf)
#pragma unroll
    for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(wf[cf][s]));

  // one tile's [T2 | X0] rows: 16 chunks per 256-B row, chunk c at c ^ (row & 15)
  auto issue = [&](int t, int b) {
    const uint32_t base = lds0 + b * AB;
    const f16* at = a + (size_t)t * PC_BM * 64;
    const f16* a2t = a2 + (size_t)t * PC_BM * 64;
#pragma unroll
    for (int i = 0; i < DMA_PER_TILE; ++i) {
      const int q = i * 256 + tid, row = q >> 4, c = (q & 15) ^ (row & 15);
      const f16* src = c < 8 ? at + row * 64 + c * 8 : a2t + row * 64 + (c - 8) * 8;
      pc_dma(src, base + (uint32_t)(i * 256 + wave * 64) * 16u);
    }
  };

  int t = blockIdx.x;
  const int G = gridDim.x;
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (t + k * G < ntiles) issue(t + k * G, k);
  __syncthreads();
  int b = 0, prev_stores = 0;
#pragma unroll 1
  for (; t < ntiles; t += G) {
    const bool ahead = t + G < ntiles;
    if (ahead) {
      if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE + ST_X + ST_T1) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE) : "memory");
    } else {
      if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST_X + ST_T1) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // tile t landed; buffer (b-1) and the staging rows are free
    if (t + (NB - 1) * G < ntiles) issue(t + (NB - 1) * G, (b + NB - 1) % NB);
    const uint32_t ab = lds0 + b * AB;

    // ---- conv3 + downsample: out^T[co][px], k = 0..127 (four 32-deep steps)
    floatx4 acc[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int cf = 0; cf < 8; ++cf) acc[j][cf] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8 xf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rw = 32 * g + 16 * j + l16;
        xf[j] = pc_ld<half8>(ab + rw * 256 + (((4 * s + lq) ^ (rw & 15)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cf = 0; cf < 8; ++cf)
          acc[j][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[cf][s], xf[j], acc[j][cf], 0, 0, 0);
    }
    // epilogue: (acc + bias) + 0, ReLU, f16 -> staged block-output rows
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rw = 32 * g + 16 * j + l16;
#pragma unroll
      for (int cf = 0; cf < 8; ++cf) {
        const int co = 128 * h + 16 * cf + 4 * lq;
        half4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[j][cf][e] + sb3[co + e];
          v += 0.f;
          hv[e] = (f16)fmaxf(v, 0.f);
        }
        pc_st(rb + rw * 512 + (((co >> 3) ^ (rw & 15)) << 4) + (lq & 1) * 8, hv);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    {
      f16* xo = x + (size_t)t * PC_BM * PC_N3;
#pragma unroll
      for (int i = 0; i < ST_X; ++i) {
        const int q = i * 256 + tid, rr = q >> 5, c = q & 31;
        const u32x4 v = pc_ld<u32x4>(rb + rr * 512 + ((c ^ (rr & 15)) << 4));
        *reinterpret_cast<u32x4*>(xo + (size_t)q * 8) = v;
      }
    }
    // ---- block 2's conv1: wave w -> tile rows 16w .. 16w+15, all 64 output channels
    const int row = 16 * wave + l16;
    floatx4 acc1[N2 / 16];
#pragma unroll
    for (int cf = 0; cf < N2 / 16; ++cf) acc1[cf] = floatx4{0.f, 0.f, 0.f, 0.f};
    half8 xf[2], wv[2][N2 / 16];
    auto rd1 = [&](int s, int k) {
      const int kc = 4 * s + lq;
      xf[k] = pc_ld<half8>(rb + row * 512 + ((kc ^ (row & 15)) << 4));
#pragma unroll
      for (int cf = 0; cf < N2 / 16; ++cf) {
        const int co = 16 * cf + l16;
        wv[k][cf] = pc_ld<half8>(ldsw1 + co * 512 + ((kc ^ (co & 15)) << 4));
      }
    };
    rd1(0, 0);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s + 1 < 8) rd1(s + 1, (s + 1) & 1);
#pragma unroll
      for (int cf = 0; cf < N2 / 16; ++cf)
        acc1[cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wv[s & 1][cf], xf[s & 1], acc1[cf], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading the block-output rows
#pragma unroll
    for (int cf = 0; cf < N2 / 16; ++cf) {
      const int co = 16 * cf + 4 * lq;
      half4 hv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc1[cf][e] + sb1[co + e];
        v += 0.f;
        hv[e] = (f16)fmaxf(v, 0.f);
      }
      pc_st(rb + row * (N2 * 2) + (((2 * cf + (lq >> 1)) ^ (row & (T1C - 1))) << 4) + (lq & 1) * 8, hv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      f16* to = t1 + (size_t)t * PC_BM * N2;
#pragma unroll
      for (int i = 0; i < ST_T1; ++i) {
        const int q = i * 256 + tid, rr = q / T1C, c = q % T1C;
        const u32x4 v = pc_ld<u32x4>(rb + rr * (N2 * 2) + ((c ^ (rr & (T1C - 1))) << 4));
        *reinterpret_cast<u32x4*>(to + (size_t)q * 8) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    prev_stores = 1;
    b = (b + 1) % NB;
  }
}

int launch_pw_chain_dual(const f16* t2, const f16* x0, const f16* w3ds, const float* b3ds, const f16* w1,
                         const float* b1, f16* xout, f16* t1, int M, hipStream_t s) {
  MEC_REQUIRE(M > 0 && M % PC_BM == 0, "pw_chain_dual: rows must be a multiple of 64");
  MEC_REQUIRE(t2 && x0 && w3ds && b3ds && w1 && b1 && xout && t1, "pw_chain_dual: null pointer");
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    MEC_HIP(hipGetDevice(&dev));
    MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int ntiles = M / PC_BM;
  hipLaunchKernelGGL(pw_chain_dual_kernel, dim3(std::min(ntiles, ncu)), dim3(256), 0, s, t2, x0, w3ds, b3ds, w1, b1,
                     xout, t1, ntiles);
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
