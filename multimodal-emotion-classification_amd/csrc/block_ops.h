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

// Y[r][n] = sum_k X[r][k] * Wt[k][n] + b[n] for r < R (R samples), n < N.
// X: LDS (row stride ldx); Y: LDS or global (row stride ldy).
// Threads own output columns; when N < blockDim the K loop is split over thread groups
// and combined through LDS scratch `red` (needs R * blockDim floats).
template <int R>
__device__ __noinline__ void block_linear(const float* X, int ldx, int K, const float* __restrict__ Wt,
                             const float* __restrict__ b, int N, float* Y, int ldy, float* red) {
  const int T = blockDim.x, tid = threadIdx.x;
  if (N >= T / 2 || red == nullptr) {
    for (int n = tid; n < N; n += T) {
      float acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.f;
      int k = 0;
      for (; k + 4 <= K; k += 4) {
        const float w0 = Wt[(size_t)(k + 0) * N + n], w1 = Wt[(size_t)(k + 1) * N + n];
        const float w2 = Wt[(size_t)(k + 2) * N + n], w3 = Wt[(size_t)(k + 3) * N + n];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float* x = X + r * ldx + k;
          acc[r] = fmaf(x[0], w0, acc[r]);
          acc[r] = fmaf(x[1], w1, acc[r]);
          acc[r] = fmaf(x[2], w2, acc[r]);
          acc[r] = fmaf(x[3], w3, acc[r]);
        }
      }
      for (; k < K; ++k) {
        const float w = Wt[(size_t)k * N + n];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fmaf(X[r * ldx + k], w, acc[r]);
      }
      const float bv = b ? b[n] : 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) Y[r * ldy + n] = acc[r] + bv;
    }
  } else {
    // split-K: G groups of N threads; group g handles k = g, g+G, ...
    const int G = T / N;
    const int g = tid / N, n = tid - g * N;
    if (g < G) {
      float acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.f;
      for (int k = g; k < K; k += G) {
        const float w = Wt[(size_t)k * N + n];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fmaf(X[r * ldx + k], w, acc[r]);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) red[(r * G + g) * N + n] = acc[r];
    }
    __syncthreads();
    for (int idx = tid; idx < R * N; idx += T) {
      const int r = idx / N, nn = idx - r * N;
      float s = 0.f;
      for (int gg = 0; gg < G; ++gg) s += red[(r * G + gg) * N + nn];
      Y[r * ldy + nn] = s + (b ? b[nn] : 0.f);
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

}  // namespace mec
