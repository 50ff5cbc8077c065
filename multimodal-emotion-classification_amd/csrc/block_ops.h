// Block-level fp32 building blocks for the latency-bound parts of the path (speech DNN,
// fusion model, classification heads). R samples per workgroup live in LDS; weights are
// streamed from L2/HBM with coalesced loads (Wt is [K][N], N contiguous); reductions use
// 64-lane wavefront shuffles. All arithmetic is fp32 like the reference.
#pragma once
#include "mec_common.h"

namespace mec {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

enum BlockAct : int { BACT_NONE = 0, BACT_RELU = 1, BACT_TANH = 2 };

__device__ __forceinline__ float block_act(float v, int act) {
  return act == BACT_RELU ? fmaxf(v, 0.f) : (act == BACT_TANH ? tanhf(v) : v);
}

// Y[r][n] = act(sum_k X[r][k] * Wt[k*ldw + n] + b[n]) for r < R (R samples), n < N.
// X: LDS (row stride ldx); Y: LDS or global (row stride ldy).
// Quad path (N % 4 == 0, N >= 64): each thread owns 4 consecutive output columns and a
// contiguous K chunk, weights are fetched as 16-B vectors 8 k-rows deep (the loop is bound
// by bytes in flight from L2/MALL), partial sums are combined through LDS scratch `red`
// (>= 4 * R * blockDim floats). Otherwise threads own single columns (K split into
// G = T/N groups when N < T, `red` >= R * blockDim floats).
typedef __attribute__((address_space(3))) const float lds_cf;

template <int R>
__device__ __noinline__ void block_linear(const float* Xg, int ldx, int K, const float* __restrict__ Wt, int ldw,
                                          const float* __restrict__ b, int N, float* Y, int ldy, float* red,
                                          int act) {
  // X always lives in LDS: address it as such (ds_read, broadcast across the wave) rather
  // than through a generic pointer (flat loads wait on both vmcnt and lgkmcnt).
  lds_cf* X = (lds_cf*)Xg;
  const int T = blockDim.x, tid = threadIdx.x;
  const int G = (N >= T || red == nullptr) ? 1 : (T / N);
  const int cols = (G == 1) ? T : N;
  const int g = tid / cols, c = tid - g * cols;
  const int kchunk = ((K + G - 1) / G + 3) & ~3;  // multiple of 4: float4 reads of X stay aligned
  const int kb = g * kchunk, ke = min(K, kb + kchunk);
  const bool x4 = (ldx & 3) == 0;
  // quad path: N % 4 == 0, 16-B aligned rows, enough columns, room in `red` (R*4*T floats)
  const int QCOLS = N / 4;
  const bool quad = red != nullptr && x4 && (N & 3) == 0 && (ldw & 3) == 0 && QCOLS >= 16 && QCOLS <= T;
  const int QG = quad ? T / QCOLS : 1;
  const int qg = quad ? tid / QCOLS : 0, qc = quad ? tid - qg * QCOLS : 0;
  const int qchunk = ((K + QG - 1) / QG + 7) & ~7;
  const int qkb = qg * qchunk, qke = min(K, qkb + qchunk);
  if (quad) {
    // 4 consecutive output columns per thread (16-B weight loads: 4x the bytes in flight),
    // K split over QG thread groups, partial sums combined through `red`.
    if (qg < QG) {
      const int n = 4 * qc;
      float acc[R][4];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r][j] = 0.f;
      int k = qkb;
      for (; k + 8 <= qke; k += 8) {
        floatx4 w[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w[q] = *reinterpret_cast<const floatx4*>(Wt + (size_t)(k + q) * ldw + n);
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const floatx4 xv = *(const __attribute__((address_space(3))) floatx4*)(X + r * ldx + k + 4 * h);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[r][j] = fmaf(xv[q], w[4 * h + q][j], acc[r][j]);
          }
        }
      }
      for (; k < qke; ++k) {
        const floatx4 wv = *reinterpret_cast<const floatx4*>(Wt + (size_t)k * ldw + n);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[r][j] = fmaf(X[r * ldx + k], wv[j], acc[r][j]);
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(qg * R + r) * N + n + j] = acc[r][j];
    }
    __syncthreads();
    for (int idx = tid; idx < R * N; idx += T) {
      const int r = idx / N, nn = idx - r * N;
      float sum = 0.f;
      for (int gg = 0; gg < QG; ++gg) sum += red[(gg * R + r) * N + nn];
      Y[r * ldy + nn] = block_act(sum + (b ? b[nn] : 0.f), act);
    }
    __syncthreads();
    return;
  }
  if (g < G) {
    for (int n = c; n < N; n += cols) {
      float acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.f;
      int k = kb;
      for (; k + 16 <= ke; k += 16) {
        float w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) w[q] = Wt[(size_t)(k + q) * ldw + n];
        if (x4) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              const __attribute__((address_space(3))) floatx4* p4 =
                  (const __attribute__((address_space(3))) floatx4*)(X + r * ldx + k + 4 * q4);
              const floatx4 xv = *p4;
              acc[r] = fmaf(xv.x, w[4 * q4 + 0], acc[r]);
              acc[r] = fmaf(xv.y, w[4 * q4 + 1], acc[r]);
              acc[r] = fmaf(xv.z, w[4 * q4 + 2], acc[r]);
              acc[r] = fmaf(xv.w, w[4 * q4 + 3], acc[r]);
            }
          }
        } else {
#pragma unroll
          for (int q = 0; q < 16; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = fmaf(X[r * ldx + k + q], w[q], acc[r]);
        }
      }
      for (; k < ke; ++k) {
        const float w = Wt[(size_t)k * ldw + n];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fmaf(X[r * ldx + k], w, acc[r]);
      }
      if (G == 1) {
        const float bv = b ? b[n] : 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) Y[r * ldy + n] = block_act(acc[r] + bv, act);
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) red[(g * R + r) * N + n] = acc[r];
      }
    }
  }
  if (G > 1) {
    __syncthreads();
    for (int idx = tid; idx < R * N; idx += T) {
      const int r = idx / N, nn = idx - r * N;
      float s = 0.f;
      for (int gg = 0; gg < G; ++gg) s += red[(gg * R + r) * N + nn];
      Y[r * ldy + nn] = block_act(s + (b ? b[nn] : 0.f), act);
    }
  }
  __syncthreads();
}

// In-place LayerNorm of R rows of length N (N % 64 == 0, N <= 1024) in LDS; one wave
// per row. Biased variance, eps inside the sqrt (torch.nn.functional.layer_norm).
// Optional ReLU after the affine.
template <int R>
__device__ __noinline__ void block_layernorm(float* X, int ldx, int N, const float* __restrict__ g,
                                const float* __restrict__ bta, float eps, bool relu) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = wave; r < R; r += nw) {
    float* x = X + r * ldx;
    float s = 0.f;
    for (int i = lane; i < N; i += 64) s += x[i];
    const float mean = wave_sum(s) / (float)N;
    float v = 0.f;
    for (int i = lane; i < N; i += 64) {
      const float d = x[i] - mean;
      v += d * d;
    }
    const float var = wave_sum(v) / (float)N;
    const float rstd = 1.0f / sqrtf(var + eps);
    for (int i = lane; i < N; i += 64) {
      float y = (x[i] - mean) * rstd * g[i] + bta[i];
      x[i] = relu ? fmaxf(y, 0.f) : y;
    }
  }
  __syncthreads();
}

// Softmax of R rows of length N (N <= 64) in LDS, one wave per row; optional copy out.
template <int R>
__device__ void block_softmax_small(float* X, int ldx, int N, float* out, int ldo) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = wave; r < R; r += nw) {
    float* x = X + r * ldx;
    const float v = lane < N ? x[lane] : -INFINITY;
    const float m = wave_max(v);
    const float e = lane < N ? expf(v - m) : 0.f;
    const float s = wave_sum(e);
    if (lane < N) {
      const float p = e / s;
      x[lane] = p;
      if (out) out[r * ldo + lane] = p;
    }
  }
  __syncthreads();
}

// Batched fp32 linear for the encoder heads (ResNet fc[1] 2048->512, MobileNetV2
// classifier[1] 1280->512, BERT pooler 768->768) on v_mfma_f32_16x16x4f32 (exact f32 products,
// f32 accumulate, MI355X_MICROARCH.md):
//   Y[b, n] = act(X[b, :] . Wt[:, n] + bias[n]),   Wt [K][N] (N contiguous), X rows ldx apart.
// Grid (ceil(B/32), N/16), 512 threads: a workgroup owns 32 rows x 16 columns and its eight
// waves split K in eighths of NG 16-deep k groups (K = 128 NG). A lane issues every load of
// its K range before the first MFMA (one memory round trip per wave): per k group one float4
// of each of its two rows (k = 16t + 4q .. +3, q = lane >> 4) and the four matching weights,
// then 2 x 4 MFMAs per group (the k order inside a group is permuted the same way for A and
// B, so the sum covers the same terms). The eighths are added in a fixed order through LDS,
// so a row's result never depends on B or on its position in the batch. At B = 256 the grid
// is 256-384 workgroups, two waves per SIMD: the f32 MFMA time is ~3.4 us for ResNet fc[1]
// (537 MFLOP at 157 TF), where linear_rows_kernel (32 x N/64 workgroups, each re-reading a
// 64-column weight slice) took 47 us alone and 179 us beside BERT
// (profiles/r01_kernel_stats_bench_final4.txt). A first form with four waves and 4-group trips
// (a memory round trip every 4 groups) measured 60 us.
template <int ACT, int NG>
__global__ __launch_bounds__(512) void linear_mfma_kernel(const float* __restrict__ X, size_t ldx, int B,
                                                          const float* __restrict__ Wt,
                                                          const float* __restrict__ bias, int N,
                                                          float* __restrict__ Y, int ldy,
                                                          float* __restrict__ Xcopy, int ldxc) {
  constexpr int K = 128 * NG, KW = 16 * NG;  // K per wave
  __shared__ __attribute__((aligned(16))) float red[8][32 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * 32, n0 = blockIdx.y * 16;
  const int kb = wave * KW;
  const int ra = min(r0 + c16, B - 1), rb = min(r0 + 16 + c16, B - 1);
  const float* xa = X + (size_t)ra * ldx + kb + 4 * q;
  const float* xb = X + (size_t)rb * ldx + kb + 4 * q;
  const float* w = Wt + (size_t)(kb + 4 * q) * N + n0 + c16;
  floatx4 a0[NG], a1[NG];
  float bw[NG][4];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    a0[g] = *reinterpret_cast<const floatx4*>(xa + 16 * g);
    a1[g] = *reinterpret_cast<const floatx4*>(xb + 16 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j) bw[g][j] = w[(size_t)(16 * g + j) * N];
  }
  // one drain for all of them (left to itself, hipcc interleaves the loads with the MFMAs at
  // 43 VGPRs and waits on each: a memory round trip per k group)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    asm volatile("" : "+v"(a0[g]), "+v"(a1[g]));
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(bw[g][j]));
  }
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[g][j], bw[g][j], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[g][j], bw[g][j], acc1, 0, 0, 0);
    }
  // D layout (16x16 f32): lane holds rows 4q + e of column c16
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[wave][(4 * q + e) * 16 + c16] = acc0[e];
    red[wave][(16 + 4 * q + e) * 16 + c16] = acc1[e];
  }
  __syncthreads();
  {
    const int row = tid >> 4, col = tid & 15;
    float s = red[0][tid];
#pragma unroll
    for (int v = 1; v < 8; ++v) s += red[v][tid];
    const float y = block_act(s + bias[n0 + col], ACT);
    if (r0 + row < B) Y[(size_t)(r0 + row) * ldy + n0 + col] = y;
  }
  if (Xcopy && blockIdx.y == 0) {
    const int nr = min(32, B - r0);
    for (int idx = tid; idx < nr * K; idx += 512) {
      const int r = idx / K, k = idx - r * K;
      Xcopy[(size_t)(r0 + r) * ldxc + k] = X[(size_t)(r0 + r) * ldx + k];
    }
  }
}

template <int ACT>
static inline int launch_linear_mfma(const float* X, size_t ldx, int B, int K, const float* Wt, const float* bias,
                                     int N, float* Y, int ldy, float* Xcopy, int ldxc, hipStream_t s) {
  MEC_REQUIRE((K == 768 || K == 1280 || K == 2048) && N % 16 == 0 && ldx % 4 == 0,
              "linear_mfma: K must be 768, 1280 or 2048, N % 16 and ldx % 4 must be 0");
  if (B <= 0) return 0;
  const dim3 grid((B + 31) / 32, N / 16), blk(512);
  if (K == 768)
    hipLaunchKernelGGL((linear_mfma_kernel<ACT, 6>), grid, blk, 0, s, X, ldx, B, Wt, bias, N, Y, ldy, Xcopy, ldxc);
  else if (K == 1280)
    hipLaunchKernelGGL((linear_mfma_kernel<ACT, 10>), grid, blk, 0, s, X, ldx, B, Wt, bias, N, Y, ldy, Xcopy, ldxc);
  else
    hipLaunchKernelGGL((linear_mfma_kernel<ACT, 16>), grid, blk, 0, s, X, ldx, B, Wt, bias, N, Y, ldy, Xcopy, ldxc);
  MEC_LAUNCH_CHECK();
  return 0;
}

// Classification head, one wave per row: logits = X[b] . Wt + b (N = 7, Wt [K][7]),
// probs = softmax(logits). Grid ceil(B/4), 256 threads; K % 64 == 0, K <= 1024.
__global__ __launch_bounds__(256) static __attribute__((unused)) void head7_kernel(
    const float* __restrict__ X, int B, int K, const float* __restrict__ Wt, const float* __restrict__ b,
    float* __restrict__ logits, float* __restrict__ probs) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* x = X + (size_t)row * K;
  float z[7];
#pragma unroll
  for (int o = 0; o < 7; ++o) z[o] = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float xv = x[k];
#pragma unroll
    for (int o = 0; o < 7; ++o) z[o] = fmaf(xv, Wt[(size_t)k * 7 + o], z[o]);
  }
  float m = -INFINITY;
#pragma unroll
  for (int o = 0; o < 7; ++o) {
    z[o] = wave_sum(z[o]) + b[o];  // every lane holds every logit
    m = fmaxf(m, z[o]);
  }
  float e[7], s = 0.f;
#pragma unroll
  for (int o = 0; o < 7; ++o) {
    e[o] = expf(z[o] - m);
    s += e[o];
  }
  if (lane < 7) {
    float zl = z[0], el = e[0];
#pragma unroll
    for (int o = 1; o < 7; ++o)
      if (lane == o) { zl = z[o]; el = e[o]; }
    logits[(size_t)row * 7 + lane] = zl;
    probs[(size_t)row * 7 + lane] = el / s;
  }
}

static inline int launch_head7(const float* X, int B, int K, const float* Wt, const float* b, float* logits,
                               float* probs, hipStream_t s) {
  MEC_REQUIRE(K % 64 == 0, "head7: K % 64 must be 0");
  if (B <= 0) return 0;
  hipLaunchKernelGGL(head7_kernel, dim3((B + 3) / 4), dim3(256), 0, s, X, B, K, Wt, b, logits, probs);
  MEC_LAUNCH_CHECK();
  return 0;
}

// Global average pool, NHWC f16 [B, HW, C] -> f32 [B, C], 16-B loads: a thread sums 8 channels over every 4th pixel (four
// thread groups per image), the four partial sums are added in a fixed order through LDS;
// grid B, (C / 8) x 4 threads (C % 8 == 0, C <= 2048).
__global__ __launch_bounds__(1024) static __attribute__((unused)) void avgpool8_kernel(const f16* __restrict__ x,
                                                                                       int HW, int C,
                                                                                       float* __restrict__ y) {
  __shared__ float part[3][2048];
  const int b = blockIdx.x, ng = C / 8, g = threadIdx.x / ng, c = (threadIdx.x - g * ng) * 8;
  const f16* p = x + (size_t)b * HW * C + c;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  for (int q = g; q < HW; q += 4) {
    const half8 v = *reinterpret_cast<const half8*>(p + (size_t)q * C);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
  }
  if (g > 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) part[g - 1][c + j] = s[j];
  }
  __syncthreads();
  if (g == 0) {
    float* o = y + (size_t)b * C + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (((s[j] + part[0][c + j]) + part[1][c + j]) + part[2][c + j]) / (float)HW;
  }
}

// Global average pool, NHWC f32 [B, HW, C] -> f32 [B, C]; grid (B, ceil(C/256)).
__global__ __launch_bounds__(256) static __attribute__((unused)) void avgpool_f32_kernel(const float* __restrict__ x,
                                                                                         int HW, int C,
                                                                                         float* __restrict__ y) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const float* p = x + (size_t)b * HW * C + c;
  float s = 0.f;
  for (int q = 0; q < HW; ++q) s += p[(size_t)q * C];
  y[(size_t)b * C + c] = s / (float)HW;
}

// Row gather of up to four arrays in one launch: row b of array i is copied from
// src[i] + b * sstride[i] to dst[i] + b * bytes[i] (bytes % 4 == 0). BERT's last layer runs on the
// [CLS] rows only (bert_cls_last): this packs those rows of the residual stream / GEMM operand
// planes / LayerNorm stats into dense [B, .] buffers. Grid B, 256 threads.
struct RowGather {
  const char* src[4];
  char* dst[4];
  long long sstride[4];
  int bytes[4];
  int n;
};
__global__ __launch_bounds__(256) static __attribute__((unused)) void gather_rows_kernel(const RowGather g) {
  const int b = blockIdx.x;
  for (int i = 0; i < g.n; ++i) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(g.src[i] + (size_t)b * g.sstride[i]);
    uint32_t* d = reinterpret_cast<uint32_t*>(g.dst[i] + (size_t)b * g.bytes[i]);
    for (int w = threadIdx.x; w < g.bytes[i] / 4; w += 256) d[w] = s[w];
  }
}
static inline int launch_gather_rows(const RowGather& g, int B, hipStream_t s) {
  MEC_REQUIRE(g.n >= 1 && g.n <= 4, "gather_rows: 1..4 arrays");
  for (int i = 0; i < g.n; ++i) MEC_REQUIRE(g.bytes[i] % 4 == 0 && g.sstride[i] % 4 == 0, "gather_rows: 4-B rows");
  if (B <= 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(B), dim3(256), 0, s, g);
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
