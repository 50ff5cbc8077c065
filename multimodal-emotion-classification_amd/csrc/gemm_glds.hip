// Pipelined fp16 MFMA GEMM / implicit-GEMM conv for gfx950 (the main GEMM engine).
//
//   C[M,N] = epilogue( A'[M,K] . B[N,K]^T ),  A' = A (A_PLAIN) or im2col(NHWC) (A_CONV)
//   or [A | 1x1/stride-s view of A2] concatenated along K (A_DUAL: a ResNet bottleneck's
//   conv3 and its downsample projection as one GEMM)
//
// * Tile BM=256 x BN (64/128/256) x BK=64, 512 threads = 8 waves (WM x WN), each wave a
//   (BM/WM) x (BN/WN) block of v_mfma_f32_32x32x16_f16 accumulators.
// * Operands move HBM/L2 -> LDS by global_load_lds_dwordx4 (no VGPR staging) into an
//   NS-stage ring; a tile is waited for with a counted `s_waitcnt vmcnt` (later tiles
//   stay in flight) and published with a raw s_barrier. LDS rows are 128 B with the
//   chunk XOR swizzle kc ^ ((row>>1)&7) applied on the per-lane SOURCE address (the DMA
//   destination is lane-linear), so the ds_read_b128 fragment reads are conflict-free.
// * Conv padding / M-tail rows: the lane's source is redirected to a zero page, so the
//   DMA itself writes the zeros (no predicated stores into the image).
// * Epilogue: each wave stages 32-row slabs of its accumulators through LDS and writes
//   them back row-contiguous: bias, residual (f16/f32), ReLU/GELU, f16 and/or f32 out
//   with 16-byte loads/stores.
// * XCD-aware bijective block remap: blocks that share an A panel share an L2.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

#include "gemm_common.h"

namespace mec {

__device__ __attribute__((aligned(64))) uint4 g_zero_page[16];

template <int BM, int BN, int WM, int WN, int NS, int AM, int DBG = 0, int MF = 32, int BK = 64, int PRE = 0,
          int ACT = -1, int SP = 0, int ER = 0>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 4) ? 2 : 1) void gemm_glds_kernel(const GemmParams p) {
  // MF: 32 = v_mfma_f32_32x32x16_f16 tiles, 16 = v_mfma_f32_16x16x32_f16 tiles
  // DBG (probe builds only): 1 = no operand loads inside the K loop, 2 = no epilogue
  // PRE: the residual tile (1 = f16, 2 = f32, 3 = f16 hi / lo planes of a split residual) is
  // loaded into registers before the main loop,
  // so its HBM read hides under the operand loads and MFMAs instead of following them
  // (ResNet's short-K conv3 GEMMs, BERT's O-projection)
  // SP: split-f16 operands (GemmParams::split). SP = 1 (pass-major): the K loop runs over 3 K
  // passes, pass 0 reading the A lo plane, pass 1 the B lo plane, pass 2 both hi planes. SP = 2
  // (interleaved, opt().gemm_x3_order 1): one K loop; a stage holds the hi AND lo tiles of A and B
  // (two halves), and each 32-deep k chunk runs its three MFMA terms (lo.hi, hi.lo, hi.hi) back to
  // back: every operand byte is fetched and staged once instead of 1.5 times on average, and four
  // fragment reads feed three MFMAs instead of six. 16x16x32 tiles only (one k-chunk order).
  static_assert(BK == 64 || BK == 32, "BK");
  static_assert(SP == 0 || PRE == 0 || PRE == 3, "split operands: split residual prefetch only");
  static_assert(SP != 2 || MF == 16, "interleaved split: 16x16x32 tiles only");
  // ER (early restage, opt().gemm_x3_restage; interleaved split tiles with a 2-stage ring and 32-deep stages):
  // each k step reads its whole stage into fragment registers first, so once every wave holds them the
  // stage is refilled with k step t + 2 while step t's MFMAs run -- two steps in flight on two buffers
  // instead of one (bert_qkv_attn_x3_kernel's schedule). Same fragments, same MFMA order: same bits.
  // NS = 1 (tile 72128): one stage, read whole into fragments and restaged for step t + 1 under step t's MFMAs;
  // 48 KB of LDS lets two workgroups share a CU, so one's barriers, loads and epilogue run under the other's
  // MFMAs
  constexpr bool ERS = ER != 0 && SP == 2 && (NS == 2 || NS == 1) && BK == 32 && DBG == 0;
  constexpr int CH = BK / 8;                   // 16-B chunks per LDS row
  constexpr int RPI = 64 / CH;                 // rows per glds wave-instruction (1 KB)
  constexpr int NW = WM * WN;
  static_assert(NW == 8 || NW == 4, "4 or 8 waves");
  constexpr int TM = BM / WM, TN = BN / WN;    // wave tile
  constexpr int TI = TM / MF, TJ = TN / MF;    // MFxMF MFMA tiles per wave
  typedef float accv __attribute__((ext_vector_type(MF == 32 ? 16 : 4)));
  constexpr int NACC = MF == 32 ? 16 : 4;
  constexpr int AI = BM / RPI / NW;            // glds wave-instructions per stage (A)
  constexpr int BI = BN / RPI / NW;            // (B)
  static_assert(BI >= 1 && AI >= 1, "tile too small for 8 waves");
  constexpr int NPL = SP == 2 ? 2 : 1;         // operand planes per stage
  constexpr int LPT = (AI + BI) * NPL;
  constexpr int HALF = (BM + BN) * BK;         // halfs per plane of a stage
  constexpr int STAGE = HALF * NPL;            // halfs per stage
  constexpr int EPI_LD = TN + 4;               // f32 staging row (padded)
  constexpr int EPI = NW * 32 * EPI_LD;        // floats for the epilogue staging
  constexpr int SMEM_H = (NS * STAGE > EPI * 2) ? NS * STAGE : EPI * 2;
  __shared__ __attribute__((aligned(16))) f16 smem[SMEM_H];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / BN;
  const int nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  int bm, bn;
  tile_coords(bid, nbm, nbn, p.group_m, bm, bn);
  const int m0 = bm * BM, n0 = bn * BN;
  if (p.stagger && (int)blockIdx.x >= p.stagger_lo && (int)blockIdx.x < p.stagger_hi) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)p.stagger) __builtin_amdgcn_s_sleep(16);
  }

  // ---- per-lane DMA sources: lane -> (row in its 8-row group, physical chunk)
  const int lrow = lane / CH, pchunk = lane % CH;
  const f16* a_src[AI];
  const f16* a2_src[AI];  // A_DUAL: second source (1x1 / stride-s view of an NHWC tensor)
  int a_ih0[AI], a_iw0[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (wave * AI + i) * RPI + lrow;  // row within tile
    const int m = m0 + r;
    a_ok[i] = m < M;
    const int mc = a_ok[i] ? m : 0;
    const int kc = sw<BK>(r, pchunk);
    if constexpr (AM == A_PLAIN) {
      a_src[i] = reinterpret_cast<const f16*>(p.A) + (size_t)mc * K + kc * 8;
    } else if constexpr (AM == A_DUAL) {
      a_src[i] = reinterpret_cast<const f16*>(p.A) + (size_t)mc * p.K1 + kc * 8;
      const int ohw = p.OH * p.OW;
      const int n = mc / ohw;
      const int rem = mc - n * ohw;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      a2_src[i] = reinterpret_cast<const f16*>(p.A2) +
                  (((size_t)n * p.H + oh * p.stride) * p.W + ow * p.stride) * p.C + kc * 8;
    } else {
      const int ohw = p.OH * p.OW;
      const int n = mc / ohw;
      const int rem = mc - n * ohw;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      a_ih0[i] = oh * p.stride - p.pad;
      a_iw0[i] = ow * p.stride - p.pad;
      a_src[i] = reinterpret_cast<const f16*>(p.A) + (size_t)n * p.H * p.W * p.C + kc * 8;
    }
  }
  const f16* b_src[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int r = (wave * BI + j) * RPI + lrow;
    const int kc = sw<BK>(r, pchunk);
    b_src[j] = p.B + (size_t)(n0 + r) * K + kc * 8;
  }
  const f16* zero = reinterpret_cast<const f16*>(g_zero_page);

  const int nk0 = K / BK;  // K tiles per pass
  // one plane of K tile kt into stage `stage` (its half h): A at aoff, B at boff from the hi planes (glds16:
  // the fragment reads below keep counted lgkmcnt waits)
  auto issue_plane = [&](int stage, int kt, int h, long long aoff, long long boff) {
    const int k0 = kt * BK;
    f16* sA = smem + stage * STAGE + h * HALF;
    f16* sB = sA + BM * BK;
    if constexpr (AM == A_PLAIN) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const f16* src = a_ok[i] ? a_src[i] + aoff + k0 : zero;
        glds16(src, (lds_vptr)(sA + (wave * AI + i) * RPI * BK));
      }
    } else if constexpr (AM == A_DUAL) {
      const bool first = k0 < p.K1;
#pragma unroll
      for (int i = 0; i < AI; ++i) {  // split: both sources' lo planes at the same offset a_lo
        const f16* src = !a_ok[i] ? zero : (first ? a_src[i] + aoff + k0 : a2_src[i] + aoff + (k0 - p.K1));
        glds16(src, (lds_vptr)(sA + (wave * AI + i) * RPI * BK));
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
        const f16* src = ok ? a_src[i] + aoff + ((size_t)ih * p.W + iw) * p.C + c0 : zero;
        glds16(src, (lds_vptr)(sA + (wave * AI + i) * RPI * BK));
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j)
      glds16(b_src[j] + boff + k0, (lds_vptr)(sB + (wave * BI + j) * RPI * BK));
  };
  auto issue = [&](int stage, int kt) {
    if constexpr (SP == 1) {  // pass 0: A_lo . B_hi, pass 1: A_hi . B_lo, pass 2: A_hi . B_hi
      const int pl = (kt >= nk0) + (kt >= 2 * nk0);
      issue_plane(stage, kt - pl * nk0, 0, pl == 0 ? p.a_lo : 0, pl == 1 ? p.b_lo : 0);
    } else if constexpr (SP == 2) {  // hi planes into half 0, lo planes into half 1
      issue_plane(stage, kt, 0, 0, 0);
      issue_plane(stage, kt, 1, p.a_lo, p.b_lo);
    } else {
      issue_plane(stage, kt, 0, 0, 0);
    }
  };

  using EG = EpiGeom<BM, BN, WM, WN>;
  half8 rpre[(PRE == 1 || PRE == 3) ? EG::SLABS : 1][EG::NPS];
  half8 rplo[PRE == 3 ? EG::SLABS : 1][EG::NPS];
  float4 rpre32[PRE == 2 ? EG::SLABS : 1][EG::NPS][2];
  if constexpr (PRE != 0) {
    const int ech = lane % EG::CPR, erow = lane / EG::CPR;
    const int col0 = n0 + wn * TN + ech * 8;
#pragma unroll
    for (int i = 0; i < EG::SLABS; ++i)
#pragma unroll
      for (int ps = 0; ps < EG::NPS; ++ps) {
        const size_t off = (size_t)min(m0 + wm * TM + i * 32 + ps * EG::RPP + erow, M - 1) * N + col0;
        if constexpr (PRE == 1 || PRE == 3) {
          rpre[i][ps] = *reinterpret_cast<const half8*>(reinterpret_cast<const f16*>(p.R) + off);
          if constexpr (PRE == 3) rplo[i][ps] = *reinterpret_cast<const half8*>(reinterpret_cast<const f16*>(p.R) + off + p.r_lo);
        } else {
          const float* R = reinterpret_cast<const float*>(p.R) + off;
          rpre32[i][ps][0] = *reinterpret_cast<const float4*>(R);
          rpre32[i][ps][1] = *reinterpret_cast<const float4*>(R + 4);
        }
      }
  }

  accv acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < NACC; ++e) acc[i][j][e] = 0.f;

  const int nk = SP == 1 ? 3 * nk0 : nk0;
#pragma unroll
  for (int s = 0; s < (ERS ? NS : NS - 1); ++s)
    if (s < nk) issue(s, s);

  const int lr = lane & 31, lh = lane >> 5;
  if constexpr (ERS) {
    const int l16 = lane & 15, lq = lane >> 4;
    for (int t = 0; t < nk; ++t) {
      if (NS == 2 && t + 1 < nk) wait_vm<LPT>();  // step t landed; step t + 1 may stay in flight
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const f16* sA = smem + (NS == 1 ? 0 : (t & 1)) * STAGE;
      const f16* sB = sA + BM * BK;
      half8 af[2][TI], bf[2][TJ];  // [plane: 0 hi, 1 lo]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int r = wm * TM + i * 16 + l16;
          af[h][i] = *reinterpret_cast<const half8*>(sA + h * HALF + r * BK + sw<BK>(r, lq) * 8);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wn * TN + j * 16 + l16;
          bf[h][j] = *reinterpret_cast<const half8*>(sB + h * HALF + r * BK + sw<BK>(r, lq) * 8);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave holds its fragments: the stage is free
      if (t + NS < nk) issue(NS == 1 ? 0 : (t & 1), t + NS);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1][i], bf[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0][i], bf[1][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0][i], bf[0][j], acc[i][j], 0, 0, 0);
    }
  } else
  for (int t = 0; t < nk; ++t) {
    // tile t must have landed; tiles t+1..t+ahead (issued) may stay in flight
    const int ahead = min(nk - 1 - t, NS - 2);
    if constexpr (NS >= 5) {
      if (ahead >= 3) wait_vm<LPT * 3>();
      else if (ahead == 2) wait_vm<LPT * 2>();
      else if (ahead == 1) wait_vm<LPT>();
      else wait_vm<0>();
    } else if constexpr (NS == 4) {
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
    // late_dma (split tiles, opt().gemm_x3_late_dma): the upper half of the waves -- the second wave of each
    // SIMD -- issues its share of the next stage's DMA after its first term group of MFMAs instead of right
    // after the barrier, so the two waves of a SIMD never both sit in the DMA issue (≈ 60-185 cycles per
    // instruction, MI355X_MICROARCH.md) while the matrix core idles. The stage is free either way (every
    // wave passed this barrier, so step t - 1's reads of it are done); same fragments and MFMAs: same bits
    // (late_dma 1: after the lo.hi terms; 2: after the hi.lo terms; 3: the hi planes after lo.hi, the lo planes
    // after hi.lo)
    // (measured and dropped, DESIGN.md §0: the first half of the waves issuing after its first fragment reads;
    // the second half issuing after the first I1 rows of lo.hi, or halfway through hi.lo)
    const bool late = SP == 2 && p.late_dma && wave >= NW / 2;
    const bool nxt = DBG != 1 && t + NS - 1 < nk;
    if (nxt && !late) issue((t + NS - 1) % NS, t + NS - 1);
    // x3_prio (opt().gemm_x3_prio): a wave's MFMA sections at wave priority 1, its DMA issue and the barrier at 0,
    // so the SIMD's other wave, issuing DMA, takes the issue slots the MFMAs leave
    const bool prio = SP == 2 && p.x3_prio;
    if (prio) __builtin_amdgcn_s_setprio(1);
    auto issue_late = [&](int part) {  // part: 0 = both planes, 1 = hi planes, 2 = lo planes
      if constexpr (SP == 2) {
        const int st = (t + NS - 1) % NS, kt = t + NS - 1;
        __builtin_amdgcn_sched_barrier(0);
        if (prio) __builtin_amdgcn_s_setprio(0);
        if (part != 2) issue_plane(st, kt, 0, 0, 0);
        if (part != 1) issue_plane(st, kt, 1, p.a_lo, p.b_lo);
        if (prio) __builtin_amdgcn_s_setprio(1);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    const f16* sA = smem + ((DBG == 1 ? 0 : t) % NS) * STAGE;
    const f16* sB = sA + BM * BK;
    if constexpr (MF == 32) {
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        const int kcs = 2 * s + lh;
        half8 af[TI], bf[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int r = wm * TM + i * 32 + lr;
          af[i] = *reinterpret_cast<const half8*>(sA + r * BK + sw<BK>(r, kcs) * 8);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wn * TN + j * 32 + lr;
          bf[j] = *reinterpret_cast<const half8*>(sB + r * BK + sw<BK>(r, kcs) * 8);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    } else if constexpr (SP == 2) {
      // interleaved split: per 32-deep k chunk the hi and lo fragments of A and B, then the three
      // terms term-major (each accumulator: lo.hi, hi.lo, hi.hi of the chunk, in that order).
      // The fragment reads go in two groups, each ahead of the terms that consume it: (B hi, A lo) for
      // lo.hi, then (B lo, A hi) once the first I1 rows of lo.hi have their operands, so that no more than
      // 15 LDS reads are ever outstanding. lgkmcnt is a 4-bit field: with all 2 (TI + TJ) reads issued at
      // once (24 on the 256 x 256 tile) the compiler drains every one before the first MFMA, and the waves,
      // in step after the barrier, leave the MFMAs idle while the LDS serves the whole stage. In groups,
      // the second lands under the first's MFMAs. Same MFMAs in the same order per accumulator: same bits.
      const int l16 = lane & 15, lq = lane >> 4;
      constexpr int KS = BK / 32;
      constexpr int GR = TI + TJ;  // reads per group
      constexpr int I1 = 2 * GR <= 15 ? 0 : (TI + GR - 15 > 1 ? TI + GR - 15 : 1);
      static_assert(GR <= 15 && I1 <= TI, "fragment read groups");
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kcs = 4 * s + lq;
        half8 af[2][TI], bf[2][TJ];  // [plane: 0 hi, 1 lo]
        auto read_a = [&](int h) {
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            const int r = wm * TM + i * 16 + l16;
            af[h][i] = *reinterpret_cast<const half8*>(sA + h * HALF + r * BK + sw<BK>(r, kcs) * 8);
          }
        };
        auto read_b = [&](int h) {
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            const int r = wn * TN + j * 16 + l16;
            bf[h][j] = *reinterpret_cast<const half8*>(sB + h * HALF + r * BK + sw<BK>(r, kcs) * 8);
          }
        };
        read_b(0);
        read_a(1);
        if constexpr (I1 == 0) {
          read_b(1);
          read_a(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (I1 > 0) {
#pragma unroll
          for (int i = 0; i < I1; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1][i], bf[0][j], acc[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          read_b(1);
          read_a(0);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = I1; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1][i], bf[0][j], acc[i][j], 0, 0, 0);
        if (late && s == 0 && nxt && (p.late_dma == 1 || p.late_dma == 3)) issue_late(p.late_dma == 1 ? 0 : 1);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0][i], bf[1][j], acc[i][j], 0, 0, 0);
        if (late && s == 0 && nxt && (p.late_dma == 2 || p.late_dma == 3)) issue_late(p.late_dma == 2 ? 0 : 2);
        if (prio && s == KS - 1) {
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_setprio(0);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0][i], bf[0][j], acc[i][j], 0, 0, 0);
      }
    } else {
      // 16x16x32: lane l holds A[row l&15][k 8(l>>4)..+7] of each 32-deep k step. Both
      // k steps' fragments are requested up front, so the second step's LDS reads are in
      // flight under the first step's MFMAs (counted lgkmcnt instead of a drain per group).
      const int l16 = lane & 15, lq = lane >> 4;
      constexpr int KS = BK / 32;
      half8 af[KS][TI], bf[KS][TJ];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kcs = 4 * s + lq;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int r = wm * TM + i * 16 + l16;
          af[s][i] = *reinterpret_cast<const half8*>(sA + r * BK + sw<BK>(r, kcs) * 8);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wn * TN + j * 16 + l16;
          bf[s][j] = *reinterpret_cast<const half8*>(sB + r * BK + sw<BK>(r, kcs) * 8);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep all fragment reads ahead of the MFMAs
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][i], bf[s][j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  if constexpr (DBG == 2) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < NACC; ++e) s += acc[i][j][e];
    if (s == 12345.678f) p.C32[0] = s;  // keeps the accumulators live
    return;
  }
  // DBG 3 (probe builds only): the whole epilogue but (almost) no stores, pricing the plane stores
  gemm_epilogue<BM, BN, WM, WN, MF, accv, TI, TJ, PRE, DBG == 3, ACT>(p, acc, smem, m0, n0, wm, wn, wave, lane, rpre,
                                                                      rpre32, rplo);
}



// Epilogue of the ping-pong tile. Its MFMAs compute out^T = W . X^T, so a lane holds 4
// consecutive output features of one token per 16x16 block (acc[ia][jb]: token block ia of the
// wave's BM/2 rows, feature block jb of its 64 columns): the LDS staging writes are whole 8-B
// (f16) / 16-B (f32) vectors instead of single floats, and every wave stages and stores its own
// region (no workgroup barrier). Same expressions and order as gemm_epilogue, so the same bits:
// ((acc + bias) + residual') -> act -> f16 / f32, residual' = R, or the deferred LayerNorm
// fma((R - mean) rstd, g, b), or +0.
//   * no residual, f16 out only (BERT FFN1, ResNet 1x1): bias, act and the f16 rounding happen
//     in registers; the wave's f16 region (BM/2 rows x 128 B, 16-B chunk x of row r at
//     x ^ ((r >> 1) & 7)) is then stored as whole 128-B row segments;
//   * otherwise (BERT FFN2): (acc + bias) in f32 slabs of 32 rows x 256 B per wave (chunk x of row
//     r at x ^ (r & 15)); each slab's residual loads are all issued before any is consumed.
// NOSTORE (probe builds only): everything computed, (almost) nothing stored.
template <int BM, bool NOSTORE = false, int ACT = -1>
__device__ __forceinline__ void pp_epilogue(const GemmParams& p, floatx4 (&acc)[BM / 32][4], char* smem, int m0,
                                            int n0, int wm, int wn, int tid, int lane) {
  constexpr int HB = BM / 2;    // rows per wave
  constexpr int NIA = BM / 32;  // 16-row token blocks per wave
  const int M = p.M, N = p.N;
  const int l16 = lane & 15, q = lane >> 4;
  const int wave = tid >> 6;
  const int rw0 = m0 + wm * HB, cw0 = n0 + wn * 64;  // the wave's first row / column
  char* reg = smem + wave * (HB * 128 > 8192 ? HB * 128 : 8192);
  float4 bb[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
    bb[jb] = p.bias ? *reinterpret_cast<const float4*>(p.bias + cw0 + jb * 16 + 4 * q)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
  const int act = ACT >= 0 ? ACT : p.act;  // compile-time where the launch knows it
  auto act4 = [&](float (&v)[4]) {
    if (act == ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    } else if (act == ACT_RELU6) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fminf(fmaxf(v[e], 0.f), 6.f);
    } else if (act == ACT_GELU) {
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const f32x2 r = gelu_erf_x2(f32x2{v[e], v[e + 1]});
        v[e] = r.x;
        v[e + 1] = r.y;
      }
    } else if (act == ACT_GELU_EXACT) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (v[e] * 0.5f) * (1.0f + erff(v[e] * 0.70710678118654752f));
    } else if (act == ACT_GELU_F32) {
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const f32x2 r = gelu_f32_x2(f32x2{v[e], v[e + 1]});
        v[e] = r.x;
        v[e + 1] = r.y;
      }
    }
  };
  const float os = p.oscale;  // 1 except on split operands: fma(acc, 1, b) == acc + b
  if (!p.R && p.C16 && !p.C32 && !p.c_lo) {
#pragma unroll
    for (int ia = 0; ia < NIA; ++ia)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        float v[4] = {__builtin_fmaf(acc[ia][jb][0], os, bb[jb].x), __builtin_fmaf(acc[ia][jb][1], os, bb[jb].y),
                      __builtin_fmaf(acc[ia][jb][2], os, bb[jb].z), __builtin_fmaf(acc[ia][jb][3], os, bb[jb].w)};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += 0.f;  // gemm_epilogue's "+ residual" with none: -0 -> +0
        act4(v);
        half4 h;
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = (f16)v[e];
        const int r = ia * 16 + l16, x = jb * 2 + (q >> 1);
        *reinterpret_cast<half4*>(reg + r * 128 + ((x ^ ((r >> 1) & 7)) << 4) + (q & 1) * 8) = h;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < HB / 8; ++it) {
      const int r = it * 8 + (lane >> 3), x = lane & 7;
      const uint4 v = *reinterpret_cast<const uint4*>(reg + r * 128 + ((x ^ ((r >> 1) & 7)) << 4));
      if (rw0 + r < M && (!NOSTORE || v.x == 0x12345678u))
        *reinterpret_cast<uint4*>(p.C16 + (size_t)(rw0 + r) * N + cw0 + x * 8) = v;
    }
    return;
  }
  // f32 slabs: lane -> row (lane >> 4) of each 4-row group, 16-B chunk (lane & 15) = 4 features
  const int sc = lane & 15, col = cw0 + sc * 4;
  bool x3bad = false;  // split output left the f16 range (raised once, after the slabs)
  float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f), b4 = g4;
  if (p.r_stats) {
    g4 = *reinterpret_cast<const float4*>(p.r_g + col);
    b4 = *reinterpret_cast<const float4*>(p.r_b + col);
  }
#pragma unroll
  for (int sl = 0; sl < HB / 32; ++sl) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int ia = sl * 2 + a;
        const float4 v = make_float4(__builtin_fmaf(acc[ia][jb][0], os, bb[jb].x),
                                     __builtin_fmaf(acc[ia][jb][1], os, bb[jb].y),
                                     __builtin_fmaf(acc[ia][jb][2], os, bb[jb].z),
                                     __builtin_fmaf(acc[ia][jb][3], os, bb[jb].w));
        const int r = a * 16 + l16, x = jb * 4 + q;
        *reinterpret_cast<float4*>(reg + r * 256 + ((x ^ (r & 15)) << 4)) = v;
      }
    float rv[8][4];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rowc = min(rw0 + sl * 32 + it * 4 + (lane >> 4), M - 1);
      const size_t base = (size_t)rowc * N + col;
#pragma unroll
      for (int e = 0; e < 4; ++e) rv[it][e] = 0.f;
      if (p.R) {
        if (p.r_f32) {
          const float4 r4 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.R) + base);
          rv[it][0] = r4.x; rv[it][1] = r4.y; rv[it][2] = r4.z; rv[it][3] = r4.w;
          if (p.r_stats) {
            const float2 st = p.r_stats[rowc];
            rv[it][0] = __builtin_fmaf((rv[it][0] - st.x) * st.y, g4.x, b4.x);
            rv[it][1] = __builtin_fmaf((rv[it][1] - st.x) * st.y, g4.y, b4.y);
            rv[it][2] = __builtin_fmaf((rv[it][2] - st.x) * st.y, g4.z, b4.z);
            rv[it][3] = __builtin_fmaf((rv[it][3] - st.x) * st.y, g4.w, b4.w);
          }
        } else {
          const f16* R16 = reinterpret_cast<const f16*>(p.R) + base;
          const half4 r4 = *reinterpret_cast<const half4*>(R16);
#pragma unroll
          for (int e = 0; e < 4; ++e) rv[it][e] = (float)r4[e];
          if (p.r_lo) {  // split residual: hi + lo (exact in f32)
            const half4 l4 = *reinterpret_cast<const half4*>(R16 + p.r_lo);
#pragma unroll
            for (int e = 0; e < 4; ++e) rv[it][e] += (float)l4[e];
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int r = it * 4 + (lane >> 4), row = rw0 + sl * 32 + r;
      const float4 sv = *reinterpret_cast<const float4*>(reg + r * 256 + ((sc ^ (r & 15)) << 4));
      float v[4] = {sv.x + rv[it][0], sv.y + rv[it][1], sv.z + rv[it][2], sv.w + rv[it][3]};
      act4(v);
      if (row < M && (!NOSTORE || v[0] == 1234.5f)) {
        const size_t base = (size_t)row * N + col;
        if (p.C16 && p.c_lo) {  // split output: planes of v * cscale, the lo plane carries the rest
          float u[4] = {v[0], v[1], v[2], v[3]};
          if (p.cscale != 1.f) {  // (a uniform branch: most split outputs carry their scale in the bias)
#pragma unroll
            for (int e = 0; e < 4; ++e) u[e] *= p.cscale;
          }
          half4 h, l;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            h[e] = (f16)u[e];
            l[e] = (f16)(u[e] - (float)h[e]);
            x3bad |= x3_out_of_range(u[e]);
          }
          *reinterpret_cast<half4*>(p.C16 + base) = h;
          *reinterpret_cast<half4*>(p.C16 + p.c_lo + base) = l;
        } else if (p.C16) {
          half4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = (f16)v[e];
          *reinterpret_cast<half4*>(p.C16 + base) = h;
        }
        if (p.C32) *reinterpret_cast<float4*>(p.C32 + base) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (p.c_lo) x3_raise(p.ovf, x3bad);
}

// ---- 256x256x64 ping-pong GEMM (A_PLAIN), v_mfma_f32_16x16x32_f16, 8 waves (2 x 4).
// Each K tile lives in one of two LDS buffers as four 16-KB pieces: A0/A1 = the 64-row
// halves of both wave rows' 128-row strips, B0/B1 = the 32-column halves of the four wave
// columns. A K tile is consumed in four phases, one output quadrant each:
//   ph0 (A0,B0)  ph1 (A0,B1)  ph2 (A1,B1)  ph3 (A1,B0)
// so the pieces fall free in the order A0, B1, A1, B0 and each is restaged for tile t+2
// (same buffer) one phase after its last read: ph1 A0, ph2 B1, ph3 A1, next ph0 B0.
// Every phase: ds_read its fragments + issue one piece (2 glds per lane), retire the
// reads (lgkmcnt(0)) BEFORE the first barrier, then 16 MFMAs between two barriers. The
// second wave row runs one barrier behind the first, so on each SIMD one wave is in its
// MFMA section while its partner loads. ph3 waits vmcnt(6): everything but the three
// pieces issued for tile t+2 has landed, i.e. all of tile t+1, read one phase later.
// Same k order per output as every other tile, so results are bit-identical to them.
// DBG = 4 (probe build, tools/pp_trace.py): s_memtime at four points of every phase of the
// first 12 K tiles, per wave, kept in spare LDS and dumped by one block into C32. DBG = 5
// (probe): the epilogue computes everything but stores nothing.
template <int AM, int DBG = 0, int BM = 256, int ACT = -1, int SP = 0>
__global__ __launch_bounds__(512) void gemm_pp_kernel(const GemmParams p) {
  static_assert(AM == A_PLAIN, "ping-pong tile: plain A only");
  static_assert(BM == 256 || BM == 128, "BM");
  constexpr int BN = 256, BK = 64, WM = 2, WN = 4;
  constexpr int PA = BM / 2;            // rows per A piece (two wave rows x BM/4)
  constexpr int PB = 128;               // rows per B piece (four wave columns x 32)
  constexpr int GA = PA / 64, GB = 2;   // glds per lane per piece
  constexpr int QI = BM / 64;           // 16-row MFMA tiles per quadrant
  constexpr int OFF_A1 = PA * BK, OFF_B0 = 2 * PA * BK, OFF_B1 = OFF_B0 + PB * BK;
  constexpr int BUF = 2 * (PA + PB) * BK;  // halfs per buffer
  constexpr int VM = (2 * GA + GB) * 1;    // glds of the three pieces issued for tile t+2
  typedef float accv __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) f16 smem[2 * BUF];
  constexpr int TRN = DBG == 4 ? 12 * 4 * 4 : 1;  // DBG 4 (probe): s_memtime phase trace
  __shared__ unsigned long long trace[DBG == 4 ? 8 : 1][TRN];
  int trk = 0;
  auto tmark = [&]() {
    if constexpr (DBG == 4) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if ((threadIdx.x & 63) == 0 && trk < TRN) trace[threadIdx.x >> 6][trk] = t;
      ++trk;
    }
  };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / BN;
  const int nbm = (M + BM - 1) / BM;
  const int nwg = nbm * nbn;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  int bm, bn;
  tile_coords(bid, nbm, nbn, p.group_m, bm, bn);
  const int m0 = bm * BM, n0 = bn * BN;

  const int lrow = lane >> 3, pchunk = lane & 7;
  const f16* a_src[2][GA];
  const f16* b_src[2][GB];
  bool a_ok[2][GA];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int pr = (wave * GA + i) * 8 + lrow;  // A-piece row
      const int m = m0 + (pr / (PA / 2)) * (BM / 2) + h * (BM / 4) + pr % (PA / 2);
      a_ok[h][i] = m < M;
      a_src[h][i] = reinterpret_cast<const f16*>(p.A) + (size_t)(a_ok[h][i] ? m : 0) * K + sw<64>(pr, pchunk) * 8;
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int pr = (wave * GB + i) * 8 + lrow;  // B-piece row
      const int n = n0 + (pr >> 5) * 64 + h * 32 + (pr & 31);
      b_src[h][i] = p.B + (size_t)n * K + sw<64>(pr, pchunk) * 8;
    }
  }
  const f16* zero = reinterpret_cast<const f16*>(g_zero_page);
  const int nk0 = K / BK;  // K tiles per pass (SP: three passes, as gemm_glds_kernel)
  // piece: 0 = A0, 1 = A1, 2 = B0, 3 = B1
  auto issue = [&](const int piece, const int kt) {
    f16* base = smem + (kt & 1) * BUF;
    int kk = kt;
    long long aoff = 0, boff = 0;
    if constexpr (SP) {
      const int pl = (kt >= nk0) + (kt >= 2 * nk0);
      kk = kt - pl * nk0;
      aoff = pl == 0 ? p.a_lo : 0;
      boff = pl == 1 ? p.b_lo : 0;
    }
    const int k0 = kk * BK;
    if (piece < 2) {
      f16* dst = base + piece * OFF_A1;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const f16* src = a_ok[piece][i] ? a_src[piece][i] + aoff + k0 : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_vptr)(dst + (wave * GA + i) * 8 * BK), 16, 0, 0);
      }
    } else {
      f16* dst = base + (piece == 2 ? OFF_B0 : OFF_B1);
#pragma unroll
      for (int i = 0; i < GB; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(b_src[piece - 2][i] + boff + k0),
                                         (lds_vptr)(dst + (wave * GB + i) * 8 * BK), 16, 0, 0);
    }
  };

  accv acc[2 * QI][4];
#pragma unroll
  for (int i = 0; i < 2 * QI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = accv{0.f, 0.f, 0.f, 0.f};

  const int l16 = lane & 15, lq = lane >> 4;
  half8 af[2][QI], bf[2][2];
  auto read_a = [&](const int buf, const int h) {
    const f16* s = smem + buf * BUF + h * OFF_A1;
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < QI; ++i) {
        const int r = wm * (PA / 2) + i * 16 + l16;
        af[k][i] = *reinterpret_cast<const half8*>(s + r * BK + sw<64>(r, 4 * k + lq) * 8);
      }
  };
  auto read_b = [&](const int buf, const int h) {
    const f16* s = smem + buf * BUF + (h ? OFF_B1 : OFF_B0);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 32 + j * 16 + l16;
        bf[k][j] = *reinterpret_cast<const half8*>(s + r * BK + sw<64>(r, 4 * k + lq) * 8);
      }
  };
  auto mma = [&](const int qa, const int qb) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tmark();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    tmark();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < QI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qa * QI + i][qb * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[k][j], af[k][i], acc[qa * QI + i][qb * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    tmark();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const int nk = SP ? 3 * nk0 : nk0;
  issue(0, 0);
  issue(3, 0);
  issue(1, 0);
  issue(2, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(3, 1);
    issue(1, 1);
    wait_vm<VM>();
  } else {
    wait_vm<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger the second wave row by one barrier
  __builtin_amdgcn_sched_barrier(0);

  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // ph0 (A0, B0)
    tmark();
    read_a(buf, 0);
    read_b(buf, 0);
    if (n1) issue(2, t + 1);
    mma(0, 0);
    // ph1 (A0, B1)
    tmark();
    read_b(buf, 1);
    if (n2) issue(0, t + 2);
    mma(0, 1);
    // ph2 (A1, B1)
    tmark();
    read_a(buf, 1);
    if (n2) issue(3, t + 2);
    mma(1, 1);
    // ph3 (A1, B0)
    tmark();
    read_b(buf, 0);
    if (n2) {
      issue(1, t + 2);
      wait_vm<VM>();
    } else {
      wait_vm<0>();
    }
    mma(1, 0);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // re-align the two wave rows
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (DBG == 4) {  // probe build: block gridDim.x / 2 dumps its trace into C32
    __syncthreads();
    if (blockIdx.x == gridDim.x / 2)
      for (int i = tid; i < 8 * TRN; i += blockDim.x)
        reinterpret_cast<unsigned long long*>(p.C32)[i] = trace[i / TRN][i % TRN];
    return;
  }
  if constexpr (DBG == 2) {  // probe build: no epilogue
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * QI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 12345.678f) p.C32[0] = s;
    return;
  }
  pp_epilogue<BM, DBG == 5, ACT>(p, acc, reinterpret_cast<char*>(smem), m0, n0, wm, wn, tid, lane);
}

// BM=256 tiles: (BN, WM, WN, NS)

// K-interleaved split operands (16x16x32, 32-deep stages) in each A mode; ER = the early-restage schedule
template <int BM, int BN, int WM, int WN, int NS, int BK, int ER>
static int launch_x3i(const GemmParams& p, hipStream_t s, int nwg, dim3 blk) {
  if (BM * BN <= 128 * 128 && opt().gemm_prefetch_r && p.amode == A_PLAIN && p.R && p.r_lo && p.K <= 512) {
    if constexpr (BM * BN <= 128 * 128)
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, 16, BK, 3, -1, 2, ER>), dim3(nwg), blk, 0, s, p);
  } else if (p.amode == A_PLAIN)
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, 16, BK, 0, -1, 2, ER>), dim3(nwg), blk, 0, s, p);
  else if (p.amode == A_CONV)
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_CONV, 0, 16, BK, 0, -1, 2, ER>), dim3(nwg), blk, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_DUAL, 0, 16, BK, 0, -1, 2, ER>), dim3(nwg), blk, 0, s, p);
  MEC_LAUNCH_CHECK();
  return 0;
}

template <int BM, int BN, int WM, int WN, int NS, int MF, int BK, int ACT>
static int launch_cfg_act(const GemmParams& p, hipStream_t s, int nwg, dim3 blk) {
  if (p.split == 2) {  // split-f16 operands, K-interleaved terms (16x16x32 tiles only)
    if constexpr (MF == 16 && BK == 32 && 4 * (BM + BN) * BK * NS <= 160 * 1024) {
      // ER: the early-restage schedule of the 2-stage tiles (opt().gemm_x3_restage; same bits)
      if (NS == 1 ||
          (NS == 2 && (opt().gemm_x3_restage == 1 || (opt().gemm_x3_restage == 2 && p.amode != A_PLAIN))))
        return launch_x3i<BM, BN, WM, WN, NS, BK, 1>(p, s, nwg, blk);
      return launch_x3i<BM, BN, WM, WN, NS, BK, 0>(p, s, nwg, blk);
    } else {
      set_error("gemm_glds: interleaved split operands need a 16x16x32 tile with 32-deep stages (tiles 7xxxx)");
      return -1;
    }
  } else if (p.split) {  // split-f16 operands (fp32x3 path): three K passes, runtime activation
    if (BM * BN <= 128 * 128 && opt().gemm_prefetch_r && p.amode == A_PLAIN && p.R && p.r_lo && p.K <= 512) {
      // split identity residual of ResNet's conv3 GEMMs, both planes prefetched (PRE = 3)
      if constexpr (BM * BN <= 128 * 128)
        hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, MF, BK, 3, -1, 1>), dim3(nwg), blk, 0, s, p);
    } else if (p.amode == A_PLAIN)
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, MF, BK, 0, -1, 1>), dim3(nwg), blk, 0, s, p);
    else if (p.amode == A_CONV)
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_CONV, 0, MF, BK, 0, -1, 1>), dim3(nwg), blk, 0, s, p);
    else
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_DUAL, 0, MF, BK, 0, -1, 1>), dim3(nwg), blk, 0, s, p);
  } else if (BM * BN <= 128 * 128 && opt().gemm_prefetch_r && p.amode == A_PLAIN && p.R && !p.r_f32 && p.K <= 512) {
    // f16 residual prefetch for ResNet's short-K conv3 GEMMs (small tiles only: no spills);
    // 225 -> 170 us on layer1's conv3. The f32 form (PRE = 2, BERT's O-projection, K = 768)
    // measured 10-15% slower than no prefetch, so it is not dispatched.
    if constexpr (BM * BN <= 128 * 128)
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, MF, BK, 1, ACT>), dim3(nwg), blk, 0, s, p);
  } else if (p.amode == A_PLAIN)
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, MF, BK, 0, ACT>), dim3(nwg), blk, 0, s, p);
  else if (p.amode == A_DUAL)
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_DUAL, 0, MF, BK, 0, ACT>), dim3(nwg), blk, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_CONV, 0, MF, BK, 0, ACT>), dim3(nwg), blk, 0, s, p);
  MEC_LAUNCH_CHECK();
  return 0;
}

template <int BM, int BN, int WM, int WN, int NS, int MF = 32, int BK = 64>
static int launch_cfg(const GemmParams& p0, hipStream_t s) {
  GemmParams p = p0;
  p.group_m = opt().gemm_glds_group_m;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  const dim3 blk(64 * WM * WN);
  // split tiles whose stages leave room for a second workgroup per CU (72128: one 48-KB stage; 71128 /
  // 71064: 2 x 32 / 2 x 24 KB): the first pass's second workgroups (blocks 256..511) start late
  p.late_dma = p.split ? opt().gemm_x3_late_dma : 0;
  p.x3_prio = p.split ? opt().gemm_x3_prio : 0;
  if (p.split && opt().gemm_x3_stagger && NS * (BM + BN) * BK * 4 <= 80 * 1024 && nwg > 256) {
    p.stagger = opt().gemm_x3_stagger * 100;
    p.stagger_lo = 256;
    p.stagger_hi = 512;
  }
#ifdef MEC_PROBES
  // the K-interleaved split tile (the fp32x3 FFN1 roofline kernel) with no operand loads inside its K loop
  // (gemm_debug 1: MFMA + LDS fragment reads + epilogue only, so its time against the real kernel's prices
  // the loads) or with no epilogue (gemm_debug 2: prices the epilogue)
  // (gemm_debug 3: the epilogue without its stores; 6: with a plain (no GELU) epilogue -- prices the GELU)
  if ((opt().gemm_debug == 1 || opt().gemm_debug == 2 || opt().gemm_debug == 3 || opt().gemm_debug == 6) &&
      p.split == 2 && BN == 256 && BM == 256 && p.amode == A_PLAIN) {
    if constexpr (MF == 16 && BK == 32 && 4 * (BM + BN) * BK * NS <= 160 * 1024) {
      if (opt().gemm_debug == 1)
        hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 1, MF, BK, 0, -1, 2>), dim3(nwg), blk, 0, s, p);
      else if (opt().gemm_debug == 2)
        hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 2, MF, BK, 0, -1, 2>), dim3(nwg), blk, 0, s, p);
      else if (opt().gemm_debug == 3)
        hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 3, MF, BK, 0, -1, 2>), dim3(nwg), blk, 0, s, p);
      else {
        GemmParams q = p;
        q.act = ACT_NONE;
        hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 0, MF, BK, 0, -1, 2>), dim3(nwg), blk, 0, s, q);
      }
    }
    MEC_LAUNCH_CHECK();
    return 0;
  }
  if (opt().gemm_debug && BN == 256 && BM == 256 && p.amode == A_PLAIN) {
    if (opt().gemm_debug == 1)
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 1, MF, BK>), dim3(nwg), blk, 0, s, p);
    else
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM, WN, NS, A_PLAIN, 2, MF, BK>), dim3(nwg), blk, 0, s, p);
    MEC_LAUNCH_CHECK();
    return 0;
  }
#endif
  // the activation is a template argument for ReLU (ResNet) and none (BERT O-proj); others runtime
  if (p.split) return launch_cfg_act<BM, BN, WM, WN, NS, MF, BK, -1>(p, s, nwg, blk);
  if (p.act == ACT_RELU) return launch_cfg_act<BM, BN, WM, WN, NS, MF, BK, ACT_RELU>(p, s, nwg, blk);
  if (p.act == ACT_NONE) return launch_cfg_act<BM, BN, WM, WN, NS, MF, BK, ACT_NONE>(p, s, nwg, blk);
  return launch_cfg_act<BM, BN, WM, WN, NS, MF, BK, -1>(p, s, nwg, blk);
}

// Tile-width choice. Every BN computes each output with the same k-ordered MFMA chain, so
// the choice changes speed only, never results. The first launch of each distinct shape
// times every legal width on the caller's stream (hipEvents; skipped while the stream is
// being captured into a graph) and caches the fastest; `gemm_bn` forces a width.
// Cache key: engine 0 (this engine) + the shape; the cache is the calling handle's
// (tune_cache(), mec_common.h).
static std::array<int, 11> gemm_key(const GemmParams& p) {  // engine slot: 0, 2 split pass-major, 3 interleaved
  return {p.split == 2 ? 3 : p.split ? 2 : 0, p.amode, p.M, p.N, p.K, p.H, p.W, p.C, p.ks, p.stride, p.pad};
}

// Tile configs (id): 256 / 128 / 64 = 256 x BN with 8 waves; 1128 / 1064 = 128 x BN with
// 4 waves (64 / 48 KB of LDS, so two blocks share a CU and one block's epilogue overlaps
// the other's MFMA loop).
// +10000: the same tile on v_mfma_f32_16x16x32_f16.
// +20000 / +30000: 16x16x32 MFMA with 32-deep K stages and a deeper ring (256 x 256: 4 / 5
// stages = 3 / 4 tiles in flight; 256 x 128: 6 stages), same K order, so same results.
// 40256 / 41256: the 256 x 256 / 128 x 256 ping-pong schedule (gemm_pp_kernel), plain A only.
// 50128 / 60128: 256 x 128 on 4 waves (wave tile 128 x 64), 32-deep K stages, 3 / 2 stages
// (74 / 49 KB LDS): two blocks per CU, so one block's epilogue runs under the other's MFMAs.
// 50256: the same for 128 x 256.
static int tile_bn(int id) {
  if (id >= 40000 && id < 50000) return 256;  // ping-pong tiles are 256 wide
  if (id >= 70000 && id < 80000) return id % 1000;  // interleaved split tiles: 7 | shape | width
  id %= 10000;
  return id > 1000 ? id - 1000 : id;
}

static int launch_bn(const GemmParams& p, hipStream_t s, int id) {
  const GemmParams& p0 = p;
  switch (id) {
    case 256: return launch_cfg<256, 256, 2, 4, 2>(p, s);
    case 128: return launch_cfg<256, 128, 4, 2, 3>(p, s);
    case 64: return launch_cfg<256, 64, 4, 2, 3>(p, s);
    case 1128: return launch_cfg<128, 128, 2, 2, 2>(p, s);
    case 1064: return launch_cfg<128, 64, 2, 2, 2>(p, s);
    case 10256: return launch_cfg<256, 256, 2, 4, 2, 16>(p, s);
    case 10128: return launch_cfg<256, 128, 4, 2, 3, 16>(p, s);
    case 10064: return launch_cfg<256, 64, 4, 2, 3, 16>(p, s);
    case 11128: return launch_cfg<128, 128, 2, 2, 2, 16>(p, s);
    case 11064: return launch_cfg<128, 64, 2, 2, 2, 16>(p, s);
    case 20256: return launch_cfg<256, 256, 2, 4, 4, 16, 32>(p, s);
    case 30256: return launch_cfg<256, 256, 2, 4, 5, 16, 32>(p, s);
    case 20128: return launch_cfg<256, 128, 4, 2, 6, 16, 32>(p, s);
    case 50128: return launch_cfg<256, 128, 2, 2, 3, 16, 32>(p, s);
    case 60128: return launch_cfg<256, 128, 2, 2, 2, 16, 32>(p, s);
    case 50256: return launch_cfg<128, 256, 2, 2, 3, 16, 32>(p, s);
    // interleaved split operands only (split == 2, gemm_x3_order 1; id = 7 | shape | width): 32-deep
    // K stages holding the hi and lo tiles of A and B (LDS: 256 x 256 2 x 64 KB; 256 x 128 3 x 48 KB;
    // 128 x 128 2 x 32 KB, two blocks per CU; 128 x 64 2 x 24 KB; 256 x 64 on 4 waves 2 x 40 KB)
    case 70256: return launch_cfg<256, 256, 2, 4, 2, 16, 32>(p, s);
    case 70128: return launch_cfg<256, 128, 4, 2, 3, 16, 32>(p, s);
    case 71128: return launch_cfg<128, 128, 2, 2, 2, 16, 32>(p, s);
    case 71064: return launch_cfg<128, 64, 2, 2, 2, 16, 32>(p, s);
    case 70064: return launch_cfg<256, 64, 2, 2, 2, 16, 32>(p, s);
    // 256 x 128 on 4 waves (wave tile 128 x 64) with ONE 48-KB stage (the restage schedule, ERS): two
    // workgroups per CU (BERT FFN2's pin outside the fused step; not an autotune candidate)
    case 72128: return launch_cfg<256, 128, 2, 2, 1, 16, 32>(p, s);
    // (measured and dropped: 4-wave 128 x 256, 256 x 128 and 256 x 256 forms, one wave per SIMD with
    // 64 x 128 / 128 x 64 / 128 x 128 wave tiles: 10-45 % slower on every BERT shape,
    // profiles/r03_split_tiles_x3i.log)
    case 40256:
    case 41256: {
      if (p0.amode != A_PLAIN) { set_error("gemm_glds: ping-pong tiles take a plain A only"); return -1; }
      GemmParams p = p0;
      p.group_m = opt().gemm_group_m;
      const dim3 blk(512);
      const int nbn = p.N / 256;
      const dim3 grd(((p.M + (id == 40256 ? 255 : 127)) / (id == 40256 ? 256 : 128)) * nbn);
#ifdef MEC_PROBES
      const int dbg = opt().gemm_debug;
      if (id == 40256 && dbg == 4)
        hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 4, 256>), grd, blk, 0, s, p);
      else if (id == 40256 && dbg == 5 && p.act == ACT_GELU)
        hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 5, 256, ACT_GELU>), grd, blk, 0, s, p);
      else if (id == 40256 && dbg == 5)
        hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 5, 256>), grd, blk, 0, s, p);
      else if (id == 40256 && dbg == 2)
        hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 2, 256>), grd, blk, 0, s, p);
      else if (dbg == 2)
        hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 2, 128>), grd, blk, 0, s, p);
      else
#endif
      // the activation is a template argument for the common cases: one epilogue path per kernel
      if (p.split) {
        if (id == 40256)
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 256, -1, 1>), grd, blk, 0, s, p);
        else
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 128, -1, 1>), grd, blk, 0, s, p);
      } else if (id == 40256) {
        if (p.act == ACT_GELU)
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 256, ACT_GELU>), grd, blk, 0, s, p);
        else if (p.act == ACT_RELU)
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 256, ACT_RELU>), grd, blk, 0, s, p);
        else if (p.act == ACT_NONE)
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 256, ACT_NONE>), grd, blk, 0, s, p);
        else
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 256>), grd, blk, 0, s, p);
      } else {
        if (p.act == ACT_RELU)
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 128, ACT_RELU>), grd, blk, 0, s, p);
        else if (p.act == ACT_NONE)
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 128, ACT_NONE>), grd, blk, 0, s, p);
        else
          hipLaunchKernelGGL((gemm_pp_kernel<A_PLAIN, 0, 128>), grd, blk, 0, s, p);
      }
      MEC_LAUNCH_CHECK();
      return 0;
    }
    default: set_error("gemm_glds: unsupported tile id"); return -1;
  }
}

// Untuned tile (gemm_autotune 0, or a first launch inside graph capture). K-interleaved split
// operands take only the 7xxxx tiles: every one of them sums in the same k order, so this choice,
// like the autotuner's, changes speed only.
static int heuristic_bn(const GemmParams& p) {
  const long nbm = (p.M + 255) / 256;
  if (p.split == 2) {
    if (p.N % 256 == 0 && nbm * (p.N / 256) >= 256) return 70256;
    if (p.N % 128 == 0) return 71128;
    return 71064;
  }
  if (p.N % 256 == 0 && nbm * (p.N / 256) >= 4 * 256 && p.K >= 768) return 256;
  if (p.N % 128 == 0 && p.K >= 1024) return 128;
  if (p.N % 128 == 0 && p.K <= 64) return 128;
  return 64;
}

static bool x3i_tile(int id) { return id >= 70000 && id < 80000; }

static int tune_bn(const GemmParams& p, hipStream_t s, int* out_bn) {
  constexpr int REPS = 5;
  const int cands[] = {64,    128,   256,   1128,  1064,  10064, 10128, 10256, 11128,
                       11064, 20256, 30256, 20128, 40256, 41256, 50128, 60128, 50256};
  const int cands_x3i[] = {70256, 70128, 71128, 71064, 70064};  // 72128: pinned only (mec_common.h gemm_x3_tag)
  hipEvent_t ev[REPS + 1];
  for (auto& e : ev) MEC_HIP(hipEventCreate(&e));
  float best = 1e30f;
  int best_bn = heuristic_bn(p);
  const int* cb = p.split == 2 ? cands_x3i : cands;
  const int nc = p.split == 2 ? (int)(sizeof(cands_x3i) / sizeof(int)) : (int)(sizeof(cands) / sizeof(int));
  for (int ci = 0; ci < nc; ++ci) {
    const int bn = cb[ci];
    if (p.N % tile_bn(bn)) continue;
    if (bn >= 40000 && bn < 50000 && p.amode != A_PLAIN) continue;
    MEC_TRY(launch_bn(p, s, bn));  // warm
    MEC_HIP(hipEventRecord(ev[0], s));
    for (int r = 0; r < REPS; ++r) {
      MEC_TRY(launch_bn(p, s, bn));
      MEC_HIP(hipEventRecord(ev[r + 1], s));
    }
    MEC_HIP(hipEventSynchronize(ev[REPS]));
    float t[REPS];
    for (int r = 0; r < REPS; ++r) MEC_HIP(hipEventElapsedTime(&t[r], ev[r], ev[r + 1]));
    std::sort(t, t + REPS);
    if (t[REPS / 2] < best) { best = t[REPS / 2]; best_bn = bn; }  // median launch
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  *out_bn = best_bn;
  return 0;
}

int gemm_tuned_bn(int amode, int M, int N, int K) {
  int t = tune_cache().find_shape(0, amode, M, N, K);
  if (!t) t = tune_cache().find_shape(2, amode, M, N, K);  // else the split-operand engines'
  return t ? t : tune_cache().find_shape(3, amode, M, N, K);
}

int launch_gemm_glds(const GemmParams& p0, hipStream_t s, int force_bn) {
  GemmParams p = p0;
  if (p.split && opt().gemm_x3_order == 1) p.split = 2;  // K-interleaved split terms
  if (force_bn) {
    MEC_REQUIRE(p.N % tile_bn(force_bn) == 0, "gemm_glds: forced tile width does not divide N");
    MEC_REQUIRE((p.split == 2) == x3i_tile(force_bn), "gemm_glds: tiles 7xxxx serve (only) interleaved split operands");
    return launch_bn(p, s, force_bn);
  }
  const auto key = gemm_key(p);
  int bn = tune_cache().find(key);
  if (!bn) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing = !(hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone);
    if (opt().gemm_autotune && !capturing) {
      MEC_TRY(tune_bn(p, s, &bn));
      tune_cache().put(key, bn);
    } else {
      bn = heuristic_bn(p);
      // a launch inside graph capture cannot time tiles: it runs the heuristic tile. For K-interleaved
      // split operands it does not cache it, so the first launch outside capture still tunes the shape
      // (every 7xxxx tile sums in one k order: same bits either way); other operands cache it, since
      // their tiles differ in MFMA shape and k order, and a graph replay and an eager launch of one
      // shape must compute the same bits
      if (!capturing || p.split != 2) tune_cache().put(key, bn);
    }
    if (getenv("MEC_GEMM_TRACE"))  // one line per distinct shape, at its first launch
      fprintf(stderr, "MEC_GEMM amode=%d M=%d N=%d K=%d H=%d C=%d ks=%d stride=%d act=%d R=%d r_f32=%d split=%d tile=%d\n",
              p.amode, p.M, p.N, p.K, p.H, p.C, p.ks, p.stride, p.act, p.R != nullptr, p.r_f32, p.split, bn);
  }
  return launch_bn(p, s, bn);
}

}  // namespace mec
