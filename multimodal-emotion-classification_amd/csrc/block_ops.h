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

// Multi-block fp32 linear over a batch: grid (ceil(B/R), ceil(N/cols)), 256 threads.
// Y[b, n] = act(X[b,:] . Wt[:, n] + bias[n]); optional copy of the X rows to Xcopy
// (done by the blockIdx.y == 0 blocks).
template <int R, int KMAX>
__global__ __launch_bounds__(256) void linear_rows_kernel(const float* __restrict__ X, size_t ldx, int B, int K,
                                                          const float* __restrict__ Wt, const float* __restrict__ bias,
                                                          int N, int cols, float* __restrict__ Y, int ldy, int act,
                                                          float* __restrict__ Xcopy, int ldxc) {
  __shared__ __attribute__((aligned(16))) float sX[R * KMAX];
  __shared__ __attribute__((aligned(16))) float sY[R * 256];
  __shared__ __attribute__((aligned(16))) float red[R * 4 * 256];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * R, nr = min(R, B - r0);
  const int col0 = blockIdx.y * cols, nc = min(cols, N - col0);
  for (int idx = tid; idx < R * K; idx += blockDim.x) {
    const int r = idx / K, k = idx - r * K;
    const float v = r < nr ? X[(size_t)(r0 + r) * ldx + k] : 0.f;
    sX[idx] = v;
    if (Xcopy && blockIdx.y == 0 && r < nr) Xcopy[(size_t)(r0 + r) * ldxc + k] = v;
  }
  __syncthreads();
  block_linear<R>(sX, K, K, Wt + col0, N, bias + col0, nc, sY, cols, red, act);
  for (int idx = tid; idx < nr * nc; idx += blockDim.x) {
    const int r = idx / nc, c = idx - r * nc;
    Y[(size_t)(r0 + r) * ldy + col0 + c] = sY[r * cols + c];
  }
}

// Classification head: logits = X . Wt + b (N = 7), probs = softmax(logits); R rows/block.
template <int R, int KMAX>
__global__ __launch_bounds__(256) void head_softmax_kernel(const float* __restrict__ X, int B, int K,
                                                           const float* __restrict__ Wt, const float* __restrict__ b,
                                                           float* __restrict__ logits, float* __restrict__ probs) {
  __shared__ __attribute__((aligned(16))) float sX[R * KMAX];
  __shared__ __attribute__((aligned(16))) float sY[R * 8];
  __shared__ __attribute__((aligned(16))) float red[R * 256];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * R, nr = min(R, B - r0);
  for (int idx = tid; idx < R * K; idx += blockDim.x) {
    const int r = idx / K, k = idx - r * K;
    sX[idx] = r < nr ? X[(size_t)(r0 + r) * K + k] : 0.f;
  }
  __syncthreads();
  block_linear<R>(sX, K, K, Wt, 7, b, 7, sY, 8, red, BACT_NONE);
  for (int idx = tid; idx < nr * 7; idx += blockDim.x) {
    const int r = idx / 7, c = idx - r * 7;
    logits[(size_t)(r0 + r) * 7 + c] = sY[r * 8 + c];
  }
  __syncthreads();
  block_softmax_small<R>(sY, 8, 7, nullptr, 0);
  for (int idx = tid; idx < nr * 7; idx += blockDim.x) {
    const int r = idx / 7, c = idx - r * 7;
    probs[(size_t)(r0 + r) * 7 + c] = sY[r * 8 + c];
  }
}

// Global average pool, NHWC f16 [B, HW, C] -> f32 [B, C]; grid (B, ceil(C/256)).
__global__ __launch_bounds__(256) static __attribute__((unused)) void avgpool_kernel(const f16* __restrict__ x, int HW, int C,
                                                             float* __restrict__ y) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const f16* p = x + (size_t)b * HW * C + c;
  float s = 0.f;
  for (int q = 0; q < HW; ++q) s += (float)p[(size_t)q * C];
  y[(size_t)b * C + c] = s / (float)HW;
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

}  // namespace mec
