// Device helpers shared by the GEMM engines (gemm_glds.hip: f16 operands; gemm_f32.hip:
// f32 operands): the LDS chunk swizzle, counted vmcnt waits, the erf-GELU and the
// LDS-staged epilogue. The MFMA C/D layout is the same for the f16 and the f32-input
// instructions (cdna_hip_programming.md), so one epilogue serves both engines.
#pragma once
#include "mec_common.h"

namespace mec {

typedef __attribute__((address_space(3))) void* lds_vptr;


// LDS chunk swizzle (16-B chunks): BK=64 rows are 128 B, BK=32 rows are 64 B. Both make
// every ds_read_b128 lane group of the 32x32x16 and 16x16x32 fragment reads cover the 16
// slots of a 256-B bank row (MI355X_MICROARCH.md, LDS lane groups).
template <int BK>
__device__ __forceinline__ int sw(int row, int kc) {
  if constexpr (BK == 64) return kc ^ ((row >> 1) & 7);
  else return kc ^ ((4 - ((row >> 2) & 3)) & 3);
}

// GELU(x) = x Phi(x) = x/2 (1 + erf(x/sqrt2)) (HF "gelu") with Phi(x) - 1/2 = c P(c^2) / Q(c^2),
// c = clamp(x, -5.5, 5.5), a (4, 3) rational minimax fit (|GELU error| <= 3.0e-6 max(|x|, 1) in
// f32, about 0.6 % of the f16 ulp of FFN1's output; Phi(-5.5) = 1.9e-8): 12 VALU + one v_rcp per
// element, where the Abramowitz-Stegun 7.1.26 erf it replaces took two transcendentals (v_rcp,
// v_exp) and ~13 VALU (|err| <= 4.6e-7): the BERT FFN1 epilogue's GELU 37 -> ~28 us at B = 256.
// Fit: least squares in s = c^2 weighted by c, refined by Levenberg-Marquardt, then rounded to
// f32 (tools/gelu_fit.py).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float gelu_rat(float x) {
  const float c = __builtin_amdgcn_fmed3f(x, -5.5f, 5.5f);
  const float s = c * c;
  float pn = __builtin_fmaf(s, -1.0374993308914782e-07f, 4.8630190576659516e-05f);
  pn = __builtin_fmaf(pn, s, 0.004202467855066061f);
  pn = __builtin_fmaf(pn, s, 0.028525715693831444f);
  pn = __builtin_fmaf(pn, s, 0.39895108342170715f);
  float qd = __builtin_fmaf(s, 0.001403174945153296f, 0.02511732093989849f);
  qd = __builtin_fmaf(qd, s, 0.2382698804140091f);
  qd = __builtin_fmaf(qd, s, 1.0f);
  const float phi = __builtin_fmaf(c * pn, __builtin_amdgcn_rcpf(qd), 0.5f);
  return x * phi;
}
__device__ __forceinline__ f32x2 gelu_erf_x2(f32x2 x) { return f32x2{gelu_rat(x.x), gelu_rat(x.y)}; }

// fp32 GELU for the fp32x3 path (ACT_GELU_F32): x/2 (1 + erf(x/sqrt2)) with the device library's
// erff polynomials (|z| < 1: z + z p(z^2); |z| >= 1: 1 - exp(-(|z| + |z| q(|z|)))) evaluated
// branch-free, the exp as one v_exp_f32 of the exponent times -log2(e) instead of the library's
// extended-precision range reduction: ~20 VALU instead of ~38 for the two branches a wave64 takes
// anyway; |erf error| grows by at most ~0.3 f32 ulp (tests/test_gpu_fp32x3.py: the GEMM against
// float64 GELU within the fp32 engine's bar)
__device__ __forceinline__ float gelu_f32(float x) {
  const float z = x * 0.70710678118654752f, a = fabsf(z);
  const float s = z * z;
  float ps = __builtin_fmaf(s, __builtin_bit_cast(float, 0xba1345e1u), __builtin_bit_cast(float, 0x3ba10414u));
  ps = __builtin_fmaf(s, ps, __builtin_bit_cast(float, 0xbcdac9b8u));
  ps = __builtin_fmaf(s, ps, __builtin_bit_cast(float, 0x3de703beu));
  ps = __builtin_fmaf(s, ps, __builtin_bit_cast(float, 0xbec09330u));
  ps = __builtin_fmaf(s, ps, __builtin_bit_cast(float, 0x3e0375d0u));
  const float es = __builtin_fmaf(a, ps, a);
  float q = __builtin_fmaf(a, __builtin_bit_cast(float, 0x378e98abu), __builtin_bit_cast(float, 0xb9c68948u));
  q = __builtin_fmaf(a, q, __builtin_bit_cast(float, 0x3b7cd369u));
  q = __builtin_fmaf(a, q, __builtin_bit_cast(float, 0xbcc618b2u));
  q = __builtin_fmaf(a, q, __builtin_bit_cast(float, 0x3dda74e4u));
  q = __builtin_fmaf(a, q, __builtin_bit_cast(float, 0x3f228afdu));
  q = __builtin_fmaf(a, q, __builtin_bit_cast(float, 0x3e03c728u));
  q = __builtin_fmaf(a, q, a);
  const float el = 1.0f - __builtin_amdgcn_exp2f(q * -1.44269504088896341f);
  const float e = copysignf(a < 1.0f ? es : el, z);
  return (x * 0.5f) * (1.0f + e);
}
// gelu_f32 on two values: the same operations in the same order, each fma / mul / add as one v_pk_*_f32 for
// both (every lane rounds as the scalar instruction does: the same bits at about half the VALU issue)
__device__ __forceinline__ f32x2 gelu_f32_x2(f32x2 x) {
  auto fma2 = [](f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); };
  auto k = [](unsigned u) { const float f = __builtin_bit_cast(float, u); return f32x2{f, f}; };
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 a = f32x2{fabsf(z.x), fabsf(z.y)};
  const f32x2 s = z * z;
  f32x2 ps = fma2(s, k(0xba1345e1u), k(0x3ba10414u));
  ps = fma2(s, ps, k(0xbcdac9b8u));
  ps = fma2(s, ps, k(0x3de703beu));
  ps = fma2(s, ps, k(0xbec09330u));
  ps = fma2(s, ps, k(0x3e0375d0u));
  const f32x2 es = fma2(a, ps, a);
  f32x2 q = fma2(a, k(0x378e98abu), k(0xb9c68948u));
  q = fma2(a, q, k(0x3b7cd369u));
  q = fma2(a, q, k(0xbcc618b2u));
  q = fma2(a, q, k(0x3dda74e4u));
  q = fma2(a, q, k(0x3f228afdu));
  q = fma2(a, q, k(0x3e03c728u));
  q = fma2(a, q, a);
  const f32x2 t = q * -1.44269504088896341f;
  const f32x2 el = 1.0f - f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  const f32x2 e = f32x2{copysignf(a.x < 1.0f ? es.x : el.x, z.x), copysignf(a.y < 1.0f ? es.y : el.y, z.y)};
  return (x * 0.5f) * (1.0f + e);
}

// Tile coordinates of logical tile `bid` (after the XCD remap, which gives each XCD a
// contiguous range): row-major over (bm, bn), or with group_m = G > 0 groups of G M panels
// walked M-fastest (the last group may be short), so the tiles an XCD runs at once share G
// A panels and fewer weight panels (opt().gemm_group_m). Result-neutral: every output keeps
// its k chain.
__device__ __forceinline__ void tile_coords(int bid, int nbm, int nbn, int group_m, int& bm, int& bn) {
  if (group_m > 0) {
    const int gsz = group_m * nbn, grp = bid / gsz, in = bid - grp * gsz;
    const int gm = min(group_m, nbm - grp * group_m);
    bm = grp * group_m + in % gm;
    bn = in / gm;
  } else {
    bm = bid / nbn;
    bn = bid - bm * nbn;
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// global_load_lds_dwordx4 (16 B per lane into LDS at m0 + 16 lane; counted on vmcnt) issued from asm.
// The compiler models the builtin's LDS write as an LDS access through FLAT and counts it on lgkmcnt too:
// while one is outstanding its LDS-read counting is out of order, so it drains every outstanding
// ds_read (lgkmcnt(0)) before the first use of any fragment. Issued from asm, the load is invisible to
// its counters and the fragment reads keep counted waits; the kernel waits for the load itself (wait_vm,
// as before: vmcnt completes in order, so the compiler's own vmcnt waits only get stricter). m0 takes the
// (uniform) LDS destination; a kernel that issues its loads through glds16 has no other m0 user.
__device__ __forceinline__ void glds16(const void* src, lds_vptr dst) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src),
               "s"((unsigned)(size_t)dst)
               : "memory", "m0");
#pragma clang diagnostic pop
}

// Shared epilogue: accumulators (16x16x32 or 32x32x16 layout, wave tile (BM/WM)x(BN/WN))
// -> bias, residual, activation -> C16 / C32. `smem` must be free (all waves past the
// main loop's last LDS read).
// Epilogue geometry shared with the residual prefetch (gemm_glds_kernel, PRE): a lane covers 8
// columns (16 B) of RPP-row passes through each 32-row slab of its wave tile.
template <int BM, int BN, int WM, int WN>
struct EpiGeom {
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int CPR = TN / 8;      // lanes per row
  static constexpr int RPP = 64 / CPR;    // rows per pass
  static constexpr int SLABS = TM / 32;
  static constexpr int NPS = 32 / RPP;    // passes per slab
};

// NOSTORE (probe builds only): every value is computed but (almost) never stored
// ACT >= 0: the activation as a compile-time constant (one epilogue path per kernel)
template <int BM, int BN, int WM, int WN, int MF, typename accv, int TI, int TJ, int PRE = 0, bool NOSTORE = false,
          int ACT = -1>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, accv (&acc)[TI][TJ], f16* smem, int m0, int n0,
                                              int wm, int wn, int wave, int lane,
                                              const half8 (*rpre)[EpiGeom<BM, BN, WM, WN>::NPS] = nullptr,
                                              const float4 (*rpre32)[EpiGeom<BM, BN, WM, WN>::NPS][2] = nullptr,
                                              const half8 (*rplo)[EpiGeom<BM, BN, WM, WN>::NPS] = nullptr) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int EPI_LD = TN + 4;
  const int M = p.M, N = p.N;
  const int lr = lane & 31, lh = lane >> 5;
  // ---- epilogue: per wave, 32-row slabs staged through LDS (f32), then written with
  // 8-element chunks where consecutive lanes cover consecutive 16-B pieces of a row
  // (CPR lanes per row), so every store / residual load instruction covers whole lines.
  float* stg = reinterpret_cast<float*>(smem) + wave * 32 * EPI_LD;
  constexpr int CPR = TN / 8;          // lanes per row (8 columns each)
  constexpr int RPP = 64 / CPR;        // rows per pass
  const int ech = lane % CPR, erow = lane / CPR;
  const int col0 = n0 + wn * TN + ech * 8;
  float bias[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bias[q] = 0.f;
  if (p.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(p.bias + col0);
    const float4 b1 = *reinterpret_cast<const float4*>(p.bias + col0 + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
    bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  float lng[8], lnb[8];
  if (p.r_stats) {
#pragma unroll
    for (int q = 0; q < 8; ++q) { lng[q] = p.r_g[col0 + q]; lnb[q] = p.r_b[col0 + q]; }
  }
  constexpr int SLABS = TM / 32;
  bool x3bad = false;  // split output left the f16 range (raised once, after the slabs)
#pragma unroll
  for (int i = 0; i < SLABS; ++i) {
    if constexpr (MF == 32) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rr = (e & 3) + 8 * (e >> 2) + 4 * lh;
          stg[rr * EPI_LD + j * 32 + lr] = acc[i][j][e];
        }
    } else {  // 16x16 D layout: col = lane&15, row = 4(lane>>4) + e
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            stg[(16 * a + 4 * (lane >> 4) + e) * EPI_LD + j * 16 + (lane & 15)] = acc[2 * i + a][j][e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int NPS = 32 / RPP;
    float rv[NPS][8];
    if (PRE == 1) {  // f16 residual already in registers (loaded before the main loop)
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps)
#pragma unroll
        for (int q = 0; q < 8; ++q) rv[ps][q] = (float)rpre[i][ps][q];
    } else if (PRE == 3) {  // split residual in registers: hi + lo (exact in f32), as the load path below
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps)
#pragma unroll
        for (int q = 0; q < 8; ++q) rv[ps][q] = (float)rpre[i][ps][q] + (float)rplo[i][ps][q];
    } else if (PRE == 2) {  // f32 residual already in registers; deferred LayerNorm applied here
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps) {
        const float4 r0 = rpre32[i][ps][0], r1 = rpre32[i][ps][1];
        rv[ps][0] = r0.x; rv[ps][1] = r0.y; rv[ps][2] = r0.z; rv[ps][3] = r0.w;
        rv[ps][4] = r1.x; rv[ps][5] = r1.y; rv[ps][6] = r1.z; rv[ps][7] = r1.w;
        if (p.r_stats) {
          const int row = min(m0 + wm * TM + i * 32 + ps * RPP + erow, M - 1);
          const float2 st = p.r_stats[row];
#pragma unroll
          for (int q = 0; q < 8; ++q) rv[ps][q] = __builtin_fmaf((rv[ps][q] - st.x) * st.y, lng[q], lnb[q]);
        }
      }
    } else if (p.R) {  // issue every residual load of the slab before any is consumed
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps) {
        const int row = min(m0 + wm * TM + i * 32 + ps * RPP + erow, M - 1);
        const size_t base = (size_t)row * N + col0;
        if (p.r_f32) {
          const float* R = reinterpret_cast<const float*>(p.R) + base;
          const float4 r0 = *reinterpret_cast<const float4*>(R);
          const float4 r1 = *reinterpret_cast<const float4*>(R + 4);
          rv[ps][0] = r0.x; rv[ps][1] = r0.y; rv[ps][2] = r0.z; rv[ps][3] = r0.w;
          rv[ps][4] = r1.x; rv[ps][5] = r1.y; rv[ps][6] = r1.z; rv[ps][7] = r1.w;
          if (p.r_stats) {
            const float2 st = p.r_stats[row];
#pragma unroll
            for (int q = 0; q < 8; ++q) rv[ps][q] = __builtin_fmaf((rv[ps][q] - st.x) * st.y, lng[q], lnb[q]);
          }
        } else {
          const f16* R16 = reinterpret_cast<const f16*>(p.R) + base;
          const half8 r8 = *reinterpret_cast<const half8*>(R16);
#pragma unroll
          for (int q = 0; q < 8; ++q) rv[ps][q] = (float)r8[q];
          if (p.r_lo) {  // split residual: hi + lo (exact in f32)
            const half8 l8 = *reinterpret_cast<const half8*>(R16 + p.r_lo);
#pragma unroll
            for (int q = 0; q < 8; ++q) rv[ps][q] += (float)l8[q];
          }
        }
      }
    } else {
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps)
#pragma unroll
        for (int q = 0; q < 8; ++q) rv[ps][q] = 0.f;
    }
#pragma unroll
    for (int ps = 0; ps < NPS; ++ps) {
      const int sr = ps * RPP + erow;
      const int row = m0 + wm * TM + i * 32 + sr;
      float v[8];
      const float4 x0 = *reinterpret_cast<const float4*>(stg + sr * EPI_LD + ech * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(stg + sr * EPI_LD + ech * 8 + 4);
      // acc * oscale + bias (oscale = 1 except on split operands: then fma(acc, 1, b) == acc + b)
      const float os = p.oscale;
      v[0] = __builtin_fmaf(x0.x, os, bias[0]); v[1] = __builtin_fmaf(x0.y, os, bias[1]);
      v[2] = __builtin_fmaf(x0.z, os, bias[2]); v[3] = __builtin_fmaf(x0.w, os, bias[3]);
      v[4] = __builtin_fmaf(x1.x, os, bias[4]); v[5] = __builtin_fmaf(x1.y, os, bias[5]);
      v[6] = __builtin_fmaf(x1.z, os, bias[6]); v[7] = __builtin_fmaf(x1.w, os, bias[7]);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += rv[ps][q];
      const int act = ACT >= 0 ? ACT : p.act;
      if (act == ACT_RELU) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
      } else if (act == ACT_RELU6) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fminf(fmaxf(v[q], 0.f), 6.f);
      } else if (act == ACT_GELU) {
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          const f32x2 r = gelu_erf_x2(f32x2{v[q], v[q + 1]});
          v[q] = r.x;
          v[q + 1] = r.y;
        }
      } else if (act == ACT_GELU_EXACT) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (v[q] * 0.5f) * (1.0f + erff(v[q] * 0.70710678118654752f));
      } else if (act == ACT_GELU_F32) {
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          const f32x2 r = gelu_f32_x2(f32x2{v[q], v[q + 1]});
          v[q] = r.x;
          v[q + 1] = r.y;
        }
      }
      if (row < M && (!NOSTORE || v[0] == 1234.5f)) {
        const size_t base = (size_t)row * N + col0;
        if (p.C16 && p.c_lo) {  // split output: planes of v * cscale, the lo plane carries the rest
          float u[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) u[q] = v[q];
          if (p.cscale != 1.f) {  // (a uniform branch: most split outputs carry their scale in the bias)
#pragma unroll
            for (int q = 0; q < 8; ++q) u[q] *= p.cscale;
          }
          half8 h, l;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            h[q] = (f16)u[q];
            l[q] = (f16)(u[q] - (float)h[q]);
            x3bad |= x3_out_of_range(u[q]);
          }
          *reinterpret_cast<half8*>(p.C16 + base) = h;
          *reinterpret_cast<half8*>(p.C16 + p.c_lo + base) = l;
        } else if (p.C16) {
          half8 h;
#pragma unroll
          for (int q = 0; q < 8; ++q) h[q] = (f16)v[q];
          *reinterpret_cast<half8*>(p.C16 + base) = h;
        }
        if (p.C32) {
          *reinterpret_cast<float4*>(p.C32 + base) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(p.C32 + base + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (p.c_lo) x3_raise(p.ovf, x3bad);
}

}  // namespace mec
