// fp32 GEMM / implicit-GEMM conv engine for gfx950: the precision the reference computes in
// (torch / Keras fp32, inference/*.py), on v_mfma_f32_32x32x2_f32. That instruction is an
// exact f32 fmaf chain per output (cdna_hip_programming.md, "FP32-input MFMA"; no xf32 on
// gfx950), at 64 FLOP/clk/SIMD = 157 TFLOP/s dense, 1/16 of the f16 rate.
//
//   C[M,N] = epilogue( A'[M,K] . B32[N,K]^T ),  A' = A (A_PLAIN) or im2col(NHWC A) (A_CONV)
//
// * K tiles of 32 floats, so an LDS row is 128 B like the f16 engine's 64-half rows: the same
//   global_load_lds_dwordx4 ring (no VGPR staging), the same chunk swizzle kc ^ ((row>>1)&7)
//   on the per-lane source address, the same zero-page redirect for conv padding and M tails.
// * A 16-B chunk c of a row holds k = 4c .. 4c+3. Lane (r = l&31, h = l>>5) reads chunk
//   2s + h of its A row and of its B row (one ds_read_b128 each) and feeds element j to MFMA
//   step (s, j): the two lane halves supply k = 8s + j and 8s + 4 + j. The read pattern is the
//   f16 engine's 32x32x16 one (conflict-free).
// * Per wave 64 x 64 (or 64 x 32) of 32 x 32 accumulators; one ds_read_b128 pair feeds 4 x
//   TI x TJ MFMAs of 64 cycles, so LDS and the DMA ring are far from the bound: the kernel is
//   MFMA-bound by construction.
// * Epilogue: gemm_common.h (bias, f32 residual, ReLU / exact-erf GELU, f32 out).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

#include "gemm_common.h"

namespace mec {

__device__ __attribute__((aligned(64))) uint4 g_zero_page_f32[16];

// LDS DMA issued from inline asm (16 B per lane to M0 + 16 x lane). Issued as the builtin,
// hipcc's waitcnt pass drains vmcnt(0) before the first fragment read of every K tile, i.e.
// waits for the DMA of the NEXT tile too, which serialises the ring (the f16 engine's float-
// free reads escape it; see conv3x3.hip). Hidden from it, the ring is ordered only by this
// kernel's counted vmcnt waits and barriers.
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void f32_dma(const void* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

// MF 32: v_mfma_f32_32x32x2_f32 (64 cycles, 16 accumulators); MF 16: v_mfma_f32_16x16x4_f32
// (32 cycles, 4 accumulators; lane (r = l&15, q = l>>4) reads chunk 4s + q and supplies
// k = 16s + 4q + j to step (s, j): the f16 engine's 16x16x32 read pattern). Same products,
// same k set per output; the two shapes differ only in summation order.
template <int BM, int BN, int WM, int WN, int NS, int AM, int MF = 32>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 4) ? 2 : 1) void gemm_f32_kernel(const GemmParams p) {
  constexpr int BK = 32;                    // floats per K tile (128-B LDS rows)
  constexpr int RPI = 8;                    // rows per glds wave-instruction (1 KB)
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int TI = TM / MF, TJ = TN / MF;
  typedef float accv __attribute__((ext_vector_type(MF == 32 ? 16 : 4)));
  constexpr int NACC = MF == 32 ? 16 : 4;
  constexpr int AI = BM / RPI / NW, BI = BN / RPI / NW;
  static_assert(AI >= 1 && BI >= 1 && TI >= 1 && TJ >= 1, "tile");
  constexpr int LPT = AI + BI;
  constexpr int STAGE = (BM + BN) * BK;     // floats per stage
  constexpr int EPI = NW * 32 * (TN + 4);   // floats for the epilogue staging
  constexpr int SMEM_F = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) float smem[SMEM_F];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / BN;
  const int nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  int bid = blockIdx.x;
  {  // XCD-aware bijective remap: consecutive tiles (sharing an A panel) on one XCD's L2
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  int bm, bn;
  tile_coords(bid, nbm, nbn, p.group_m, bm, bn);
  const int m0 = bm * BM, n0 = bn * BN;

  const int lrow = lane >> 3, pchunk = lane & 7;
  const float* a_src[AI];
  int a_ih0[AI], a_iw0[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (wave * AI + i) * RPI + lrow;
    const int m = m0 + r;
    a_ok[i] = m < M;
    const int mc = a_ok[i] ? m : 0;
    const int kc = sw<64>(r, pchunk);
    if constexpr (AM == A_PLAIN) {
      a_src[i] = reinterpret_cast<const float*>(p.A) + (size_t)mc * K + kc * 4;
      a_ih0[i] = a_iw0[i] = 0;
    } else {
      const int ohw = p.OH * p.OW;
      const int n = mc / ohw;
      const int rem = mc - n * ohw;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      a_ih0[i] = oh * p.stride - p.pad;
      a_iw0[i] = ow * p.stride - p.pad;
      a_src[i] = reinterpret_cast<const float*>(p.A) + (size_t)n * p.H * p.W * p.C + kc * 4;
    }
  }
  const float* b_src[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int r = (wave * BI + j) * RPI + lrow;
    b_src[j] = p.B32 + (size_t)(n0 + r) * K + sw<64>(r, pchunk) * 4;
  }
  const float* zero = reinterpret_cast<const float*>(g_zero_page_f32);

  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)smem);
  auto issue = [&](int stage, int kt) {
    const int k0 = kt * BK;
    const uint32_t sA = lds0 + (uint32_t)(stage * STAGE) * 4u;
    const uint32_t sB = sA + (uint32_t)(BM * BK) * 4u;
    if constexpr (AM == A_PLAIN) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const float* src = a_ok[i] ? a_src[i] + k0 : zero;
        f32_dma(src, sA + (uint32_t)((wave * AI + i) * RPI * BK) * 4u);
      }
    } else {
      const int tap = k0 / p.C;
      const int c0 = k0 - tap * p.C;
      const int kh = tap / p.ks;
      const int kw = tap - kh * p.ks;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        const bool ok = a_ok[i] && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        const float* src = ok ? a_src[i] + ((size_t)ih * p.W + iw) * p.C + c0 : zero;
        f32_dma(src, sA + (uint32_t)((wave * AI + i) * RPI * BK) * 4u);
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j)
      f32_dma(b_src[j] + k0, sB + (uint32_t)((wave * BI + j) * RPI * BK) * 4u);
  };

  accv acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < NACC; ++e) acc[i][j][e] = 0.f;

  const int nk = K / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);

  const int lr = lane & 31, lh = lane >> 5;
  for (int t = 0; t < nk; ++t) {
    const int ahead = min(nk - 1 - t, NS - 2);
    if constexpr (NS >= 4) {
      if (ahead >= 2) wait_vm<LPT * 2>();
      else if (ahead == 1) wait_vm<LPT>();
      else wait_vm<0>();
    } else if constexpr (NS == 3) {
      if (ahead >= 1) wait_vm<LPT>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    (void)ahead;
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < nk) issue((t + NS - 1) % NS, t + NS - 1);
    const float* sA = smem + (t % NS) * STAGE;
    const float* sB = sA + BM * BK;
    if constexpr (MF == 32) {
#pragma unroll
      for (int s = 0; s < BK / 8; ++s) {
        const int kcs = 2 * s + lh;
        float4 af[TI], bf[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int r = wm * TM + i * 32 + lr;
          af[i] = *reinterpret_cast<const float4*>(sA + r * BK + sw<64>(r, kcs) * 4);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wn * TN + j * 32 + lr;
          bf[j] = *reinterpret_cast<const float4*>(sB + r * BK + sw<64>(r, kcs) * 4);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][q], bf[j][q], acc[i][j], 0, 0, 0);
      }
    } else {
      const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        const int kcs = 4 * s + lq;
        float4 af[TI], bf[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int r = wm * TM + i * 16 + l16;
          af[i] = *reinterpret_cast<const float4*>(sA + r * BK + sw<64>(r, kcs) * 4);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wn * TN + j * 16 + l16;
          bf[j] = *reinterpret_cast<const float4*>(sB + r * BK + sw<64>(r, kcs) * 4);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][q], bf[j][q], acc[i][j], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  gemm_epilogue<BM, BN, WM, WN, MF>(p, acc, reinterpret_cast<f16*>(smem), m0, n0, wm, wn, wave, lane);
}

// Tiles (id): 1 = 256 x 128 on 8 waves (2 stages, 96 KB), 2 = 128 x 128 on 4 waves (2 stages,
// 64 KB: two blocks per CU), 3 = 128 x 64 on 4 waves (3 stages), 4 = 256 x 256 on 8 waves
// (wave tile 128 x 64, 2 stages, 128 KB), all on the 32x32x2 MFMA; 5..8 = the same tiles on
// the 16x16x4 MFMA. Tiles of one MFMA shape accumulate each output along the same k order
// (bit-identical); the two shapes sum in different orders (rounding-level difference).
static int tile_n(int id) { const int b = (id - 1) % 4 + 1; return b == 3 ? 64 : (b == 4 ? 256 : 128); }

template <int BM, int BN, int WM, int WN, int NS, int MF = 32>
static int launch_f32(const GemmParams& p0, hipStream_t s) {
  GemmParams p = p0;
  p.group_m = opt().gemm_group_m;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  const dim3 blk(64 * WM * WN);
  if (p.amode == A_PLAIN)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, NS, A_PLAIN, MF>), dim3(nwg), blk, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, NS, A_CONV, MF>), dim3(nwg), blk, 0, s, p);
  MEC_LAUNCH_CHECK();
  return 0;
}

static int launch_tile(const GemmParams& p, hipStream_t s, int id) {
  switch (id) {
    case 1: return launch_f32<256, 128, 4, 2, 2>(p, s);
    case 2: return launch_f32<128, 128, 2, 2, 2>(p, s);
    case 3: return launch_f32<128, 64, 2, 2, 3>(p, s);
    case 4: return launch_f32<256, 256, 2, 4, 2>(p, s);
    case 5: return launch_f32<256, 128, 4, 2, 2, 16>(p, s);
    case 6: return launch_f32<128, 128, 2, 2, 2, 16>(p, s);
    case 7: return launch_f32<128, 64, 2, 2, 3, 16>(p, s);
    case 8: return launch_f32<256, 256, 2, 4, 2, 16>(p, s);
    default: set_error("gemm_f32: unsupported tile id"); return -1;
  }
}

// Cache key: engine 1 (this engine) + the shape, in the calling handle's tune_cache().
// engine slot: 1 + the MFMA family allowed when the shape was tuned, so changing
// gemm_f32_family on a handle never reuses a tile of the other family (other k order)
static int f32_engine() { return 1 + opt().gemm_f32_family; }

static std::array<int, 11> f32_key(const GemmParams& p) {
  return {f32_engine(), p.amode, p.M, p.N, p.K, p.H, p.W, p.C, p.ks, p.stride, p.pad};
}

// MFMA family allowed by opt().gemm_f32_family (0: both; 16: ids 5..8 on 16x16x4; 32: ids 1..4
// on 32x32x2). The two families sum in different k orders, so one family for every shape makes
// a row's result independent of the batch size (the tuned tile may change with M, its bits not).
static bool family_ok(int id) {
  const int fam = opt().gemm_f32_family;
  return fam == 0 || (fam == 16 ? id >= 5 : id <= 4);
}

static int heuristic_tile(const GemmParams& p) {
  const int id = (p.N % 128) ? 3 : ((long)((p.M + 255) / 256) * (p.N / 128) >= 512 ? 1 : 2);
  return opt().gemm_f32_family == 16 ? id + 4 : id;
}

// First launch of a shape: time every legal tile (median of 3 launches, hipEvents on the
// caller's stream; skipped while the stream is being captured) and keep the fastest.
static int tune_tile(const GemmParams& p, hipStream_t s, int* out) {
  constexpr int REPS = 3;
  hipEvent_t ev[REPS + 1];
  for (auto& e : ev) MEC_HIP(hipEventCreate(&e));
  float best = 1e30f;
  int best_id = heuristic_tile(p);
  for (int id = 1; id <= 8; ++id) {
    if (p.N % tile_n(id) || !family_ok(id)) continue;
    MEC_TRY(launch_tile(p, s, id));
    MEC_HIP(hipEventRecord(ev[0], s));
    for (int r = 0; r < REPS; ++r) {
      MEC_TRY(launch_tile(p, s, id));
      MEC_HIP(hipEventRecord(ev[r + 1], s));
    }
    MEC_HIP(hipEventSynchronize(ev[REPS]));
    float t[REPS];
    for (int r = 0; r < REPS; ++r) MEC_HIP(hipEventElapsedTime(&t[r], ev[r], ev[r + 1]));
    std::sort(t, t + REPS);
    if (t[REPS / 2] < best) { best = t[REPS / 2]; best_id = id; }
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  *out = best_id;
  return 0;
}

int gemm_f32_tuned(int amode, int M, int N, int K) { return tune_cache().find_shape(f32_engine(), amode, M, N, K); }

int launch_gemm_f32(const GemmParams& p, hipStream_t s, Prof* prof, int tag) {
  MEC_REQUIRE(p.M > 0 && p.N > 0 && p.K > 0, "gemm_f32: empty shape");
  MEC_REQUIRE(p.N % 64 == 0, "gemm_f32: N % 64 != 0");
  MEC_REQUIRE(p.K % 32 == 0, "gemm_f32: K % 32 != 0");
  MEC_REQUIRE(p.A && p.B32, "gemm_f32: null operand");
  MEC_REQUIRE(p.C32 && !p.C16, "gemm_f32: f32 output only");
  MEC_REQUIRE(!p.R || p.r_f32, "gemm_f32: residual must be f32");
  MEC_REQUIRE(!p.r_stats, "gemm_f32: no deferred LayerNorm on the fp32 path");
  if (p.amode == A_CONV) {
    MEC_REQUIRE(p.C % 32 == 0 && p.K == p.ks * p.ks * p.C, "conv_f32: C % 32 != 0 or K != ks*ks*C");
  } else {
    MEC_REQUIRE(p.amode == A_PLAIN, "gemm_f32: plain or conv A only");
  }
  const auto key = f32_key(p);
  int id = opt().gemm_f32_tile;
  if (!id && tag > 0 && tag < TAG_COUNT && opt().gemm_f32_tag[tag] && p.N % tile_n(opt().gemm_f32_tag[tag]) == 0 &&
      family_ok(opt().gemm_f32_tag[tag])) {
    id = opt().gemm_f32_tag[tag];
    tune_cache().put(key, id);  // so mec_model_gemm_query reports the tile that runs
  }
  if (id) {
    MEC_REQUIRE(id >= 1 && id <= 8 && p.N % tile_n(id) == 0, "gemm_f32: forced tile does not fit N");
  } else {
    id = tune_cache().find(key);
  }
  if (!id) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing = !(hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone);
    if (opt().gemm_autotune && !capturing) {
      MEC_TRY(tune_tile(p, s, &id));
    } else {
      id = heuristic_tile(p);
    }
    // inside capture the heuristic tile is untimed: not cached while the autotune family is held to one
    // MFMA shape (gemm_f32_family 16 / 32: every tile sums in one k order, same bits), so the first
    // eager launch still tunes; cached with both families allowed, so replay and eager bits agree
    if (!capturing || !opt().gemm_f32_family) tune_cache().put(key, id);
    if (getenv("MEC_GEMM_TRACE"))
      fprintf(stderr, "MEC_GEMM_F32 amode=%d M=%d N=%d K=%d H=%d C=%d ks=%d stride=%d act=%d R=%d tile=%d\n", p.amode,
              p.M, p.N, p.K, p.H, p.C, p.ks, p.stride, p.act, p.R != nullptr, id);
  }
  if (prof) MEC_TRY(prof->begin(tag, s));
  MEC_TRY(launch_tile(p, s, id));
  if (prof) MEC_TRY(prof->end(tag, s));
  return 0;
}

}  // namespace mec
