// ResNet50 image path in fp32 end to end (mec_create_ex(..., MEC_PREC_FP32)), the reference's
// own precision (inference/image_inference.py:28-32 transform, :55-65 network + head):
//   resize      PIL-exact u8 bilinear 48 -> 224 (resnet.hip, shared with the f16 path)
//   stem, gray  (the FER path: convert('RGB') replicates the channel) conv 7x7/2 + BN + ReLU +
//               maxpool 3x3/2 in one kernel, stem_pool_gray_f32_kernel (below)
//   stem, RGB   explicit im2col of ToTensor + Normalize (x / 255 - mean) / std, exactly as
//               torchvision computes it, k = c*49 + kh*7 + kw (the torch weight order), K
//               padded 147 -> 160; then one fp32 GEMM [B*112*112, 160] x [64, 160]^T + BN + ReLU;
//               maxpool 3x3/2 pad 1, NHWC f32
//   bottlenecks conv1 / conv2 (3x3, stride on the 3x3: v1.5) / conv3 + residual (identity or
//               the 1x1/s downsample GEMM) + ReLU, all on gemm_f32 (A_PLAIN / A_CONV), BN
//               folded into f32 weights and bias
//   avgpool     NHWC f32 -> [B, 2048]; head as on the f16 path (fc1 + ReLU = 512-d feature,
//               fc2, softmax; block_ops.h)
#include <algorithm>
#include <cmath>

#include "block_ops.h"
#include "models.h"

namespace mec {

namespace {
constexpr int STEM_K = 160;  // 3 * 49 = 147 taps, zero-padded to a multiple of 32
const int kLayers32[4][3] = {{64, 3, 1}, {128, 4, 2}, {256, 6, 2}, {512, 3, 2}};
}  // namespace

// One thread per 4 consecutive k of one output pixel's im2col row. img: u8 [B,224,224,C]
// (C = 1: the gray image replicated to RGB by convert('RGB'); C = 3: RGB).
__global__ __launch_bounds__(256) void stem_im2col_f32_kernel(const uint8_t* __restrict__ img, int B, int C,
                                                              float* __restrict__ A) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)B * 112 * 112 * (STEM_K / 4);
  if (idx >= total) return;
  const int q = (int)(idx % (STEM_K / 4));
  const size_t m = idx / (STEM_K / 4);
  const int ow = (int)(m % 112), oh = (int)((m / 112) % 112);
  const size_t b = m / (112 * 112);
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * q + j;
    float x = 0.f;
    if (k < 147) {
      const int c = k / 49, tap = k - c * 49, kh = tap / 7, kw = tap - kh * 7;
      const int ih = 2 * oh - 3 + kh, iw = 2 * ow - 3 + kw;
      if (ih >= 0 && ih < 224 && iw >= 0 && iw < 224) {
        const uint8_t px = img[((b * 224 + ih) * 224 + iw) * C + (C == 3 ? c : 0)];
        x = ((float)px / 255.0f - mean[c]) / stdv[c];  // ToTensor, then Normalize (sub_, div_)
      }
    }
    v[j] = x;
  }
  *reinterpret_cast<float4*>(A + m * STEM_K + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
}

// MaxPool2d(3, 2, 1) on NHWC f32 [B,H,H,C] -> [B,OH,OH,C]; one thread per 4 channels.
__global__ __launch_bounds__(256) void maxpool_f32_kernel(const float* __restrict__ x, int B, int Hin, int C, int OH,
                                                          float* __restrict__ y) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int C4 = C / 4;
  const size_t total = (size_t)B * OH * OH * C4;
  if (idx >= total) return;
  const int c4 = (int)(idx % C4);
  const size_t pix = idx / C4;
  const int ow = (int)(pix % OH), oh = (int)((pix / OH) % OH);
  const size_t b = pix / ((size_t)OH * OH);
  float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  for (int dy = 0; dy < 3; ++dy) {
    const int ih = 2 * oh - 1 + dy;
    if (ih < 0 || ih >= Hin) continue;
    for (int dx = 0; dx < 3; ++dx) {
      const int iw = 2 * ow - 1 + dx;
      if (iw < 0 || iw >= Hin) continue;
      const float4 v = *reinterpret_cast<const float4*>(x + ((b * Hin + ih) * Hin + iw) * C + 4 * c4);
      m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
    }
  }
  *reinterpret_cast<float4*>(y + idx * 4) = m;
}

// Stem of a gray image (the FER path), fp32. With the channel replicated to RGB and
// Normalize affine, conv(Normalize(x)) over the 3 channels of one 7x7 window is
//   sum over in-image taps t of ( px_t Wg[t] + 1 . Wm[t] ),
//   Wg[t] = sum_c W[c][t] / (255 std_c),   Wm[t] = -sum_c W[c][t] mean_c / std_c
// (BN scale folded in; host-folded in float64), i.e. a 2-channel conv over (pixel, in-image
// indicator): K = 49 taps x 2 = 98, exactly 49 steps of v_mfma_f32_32x32x2_f32 with the two
// lane halves on the two channels, against 147 -> 160 taps of the im2col GEMM. The sums are
// reassociated against torch's 3-channel conv (fp32 rounding, well inside the 1e-5 probs bar).
// A persistent workgroup (8 waves, one per CU) walks tiles of 8 x 8 pooled outputs of one image:
//   * the tile's 39 x 39 u8 input patch sits in LDS as (px, inside) float pairs; the next tile's
//     patch is loaded into registers under this tile's MFMAs and written after its last read;
//   * the 17 x 17 stem pixels it pools from (289 rows, 10 M-tiles of 32) x 64 channels (2 N-tiles)
//     are 20 (M, N) tile pairs: wave w takes pairs w, w + 8, w + 16, so each SIMD's two waves
//     carry 5; the folded weights [49][2][64] stay in LDS for the launch;
//   * bias + ReLU -> the stem tile in LDS -> MaxPool2d(3, 2, 1) (stem pixels outside the
//     112 x 112 map skipped, as padding -inf) -> float4 stores of [B, 56, 56, 64].
// The im2col path it replaces wrote and re-read 2 GB at B = 256 (im2col 844 + GEMM 698 + pool
// 207 us, profiles/r02_enc_fp32_image.txt).
constexpr int SGF_P = 39, SGF_S = 17, SGF_NPIX = SGF_S * SGF_S;  // patch side, stem tile side, stem pixels
constexpr int SGF_PL = (SGF_P * SGF_P + 511) / 512;              // patch entries per thread (3)

__global__ __launch_bounds__(512, 1) void stem_pool_gray_f32_kernel(const uint8_t* __restrict__ img, int ntiles,
                                                                   const float* __restrict__ wg,
                                                                   const float* __restrict__ bias,
                                                                   float* __restrict__ y) {
  __shared__ float sw[49 * 2 * 64];                           // folded weights [tap][channel][co]
  __shared__ __attribute__((aligned(16))) float2 patch[SGF_P * SGF_P];
  __shared__ __attribute__((aligned(16))) float stg[SGF_NPIX * 64];  // ReLU'd stem tile [pixel][co]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, kk = lane >> 5;
  for (int i = tid; i < 49 * 2 * 64; i += 512) sw[i] = wg[i];
  int base[3], nt[3];
  float bv[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {  // pair w + 8q: M-tile (p >> 1), N-tile (p & 1)
    const int pr = wave + 8 * q;
    const int i = min((pr >> 1) * 32 + li, SGF_NPIX - 1);
    const int sr = i / SGF_S, sc = i - (i / SGF_S) * SGF_S;
    base[q] = 2 * sr * SGF_P + 2 * sc;  // patch slot of tap (0, 0) of the lane's stem pixel
    nt[q] = pr & 1;
    bv[q] = bias[nt[q] * 32 + li];
  }
  const int npair = wave < 4 ? 3 : 2;
  const float* pf = reinterpret_cast<const float*>(patch);
  // patch entries of tile t: (row, col) slots tid + 512 j; -1 = outside the image
  auto patch_load = [&](int t, int (&v)[SGF_PL]) {
    const int b = t / 49, tt = t - (t / 49) * 49;
    const int r0 = 4 * (tt / 7) * 8 - 5, c0 = 4 * (tt - (tt / 7) * 7) * 8 - 5;
#pragma unroll
    for (int j = 0; j < SGF_PL; ++j) {
      const int i = tid + 512 * j;
      const int pr = i / SGF_P, pc = i - (i / SGF_P) * SGF_P;
      const int ih = r0 + pr, iw = c0 + pc;
      v[j] = (i < SGF_P * SGF_P && ih >= 0 && ih < 224 && iw >= 0 && iw < 224) ? (int)img[((size_t)b * 224 + ih) * 224 + iw]
                                                                                : -1;
    }
  };
  auto patch_store = [&](const int (&v)[SGF_PL]) {
#pragma unroll
    for (int j = 0; j < SGF_PL; ++j) {
      const int i = tid + 512 * j;
      if (i < SGF_P * SGF_P) patch[i] = v[j] >= 0 ? make_float2((float)v[j], 1.f) : make_float2(0.f, 0.f);
    }
  };
  int pv[SGF_PL];
  if (blockIdx.x < ntiles) {
    patch_load(blockIdx.x, pv);
    patch_store(pv);
  }
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int b = t / 49, tt = t - (t / 49) * 49;
    const int py0 = (tt / 7) * 8, px0 = (tt - (tt / 7) * 7) * 8;
    __syncthreads();  // this tile's patch and the weights are in LDS; the last pool read stg
    const int tn = t + gridDim.x;
    if (tn < ntiles) patch_load(tn, pv);  // lands under the MFMAs
    floatx16 acc[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;
#pragma unroll 7
    for (int st = 0; st < 49; ++st) {
      const int kh = st / 7, kw = st - (st / 7) * 7;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q < npair) {
          const float av = pf[(base[q] + kh * SGF_P + kw) * 2 + kk];
          const float w = sw[(st * 2 + kk) * 64 + nt[q] * 32 + li];
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, w, acc[q], 0, 0, 0);
        }
      }
    }
    // D[row (e & 3) + 8 (e >> 2) + 4 kk][col li] of each 32 x 32 block: stem pixel x channel
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < npair)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int pix = ((wave + 8 * q) >> 1) * 32 + (e & 3) + 8 * (e >> 2) + 4 * kk;
          if (pix < SGF_NPIX) stg[pix * 64 + nt[q] * 32 + li] = fmaxf(acc[q][e] + bv[q], 0.f);
        }
    __syncthreads();  // stg complete; every patch read of this tile done
    if (tn < ntiles) patch_store(pv);
    const float4* stg4 = reinterpret_cast<const float4*>(stg);
#pragma unroll
    for (int it = 0; it < 2; ++it) {  // 64 pooled pixels x 16 channel quads
      const int idx = it * 512 + tid, pp = idx >> 4, cq = idx & 15;
      const int py = pp >> 3, px = pp & 7;
      float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int sr = 2 * py + dy, R = 2 * py0 - 1 + sr;
        if (R < 0 || R >= 112) continue;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int sc = 2 * px + dx, Cc = 2 * px0 - 1 + sc;
          if (Cc < 0 || Cc >= 112) continue;
          const float4 v = stg4[(sr * SGF_S + sc) * 16 + cq];
          m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
        }
      }
      *reinterpret_cast<float4*>(y + (((size_t)b * 56 + py0 + py) * 56 + px0 + px) * 64 + cq * 4) = m;
    }
  }
}

// fp32x3 form of the gray stem: the same (pixel, inside) 2-channel conv + BN + ReLU + max-pool,
// on v_mfma_f32_32x32x8_f16. The A operand (pixel value 0..255, inside 0 / 1) is exact in f16,
// so only the folded weights are split (w 2^e = hi + lo, wscale = 2^-e): two f16 products per
// fp32 product (A.lo, then A.hi), 49 taps padded to 52 = 13 k-steps of 8 (4 taps x 2 channels;
// lane half kk supplies taps 4s + 2kk, 4s + 2kk + 1). Writes the pooled map as hi / lo planes
// (y, y + lo): the first bottleneck's split operand, no f32 intermediate.
typedef _Float16 hpair __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(512, 1) void stem_pool_gray_x3_kernel(const uint8_t* __restrict__ img, int ntiles,
                                                                  const float* __restrict__ wg, float wsc_up,
                                                                  float wscale, const float* __restrict__ bias,
                                                                  f16* __restrict__ y, long long lo,
                                                                  unsigned* flag) {
  __shared__ __attribute__((aligned(16))) f16 swh[52 * 2 * 64];  // [tap][channel][co], taps 49..51 zero
  __shared__ __attribute__((aligned(16))) f16 swl[52 * 2 * 64];
  __shared__ __attribute__((aligned(16))) hpair patch[SGF_P * SGF_P];  // (pixel, inside)
  __shared__ __attribute__((aligned(16))) float stg[SGF_NPIX * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, kk = lane >> 5;
  for (int i = tid; i < 52 * 2 * 64; i += 512) {
    const float x = i < 49 * 2 * 64 ? wg[i] * wsc_up : 0.f;  // w 2^e (exact)
    const f16 h = (f16)x;
    swh[i] = h;
    swl[i] = (f16)(x - (float)h);
  }
  int base[3], nt[3];
  float bv[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int pr = wave + 8 * q;
    const int i = min((pr >> 1) * 32 + li, SGF_NPIX - 1);
    const int sr = i / SGF_S, sc = i - (i / SGF_S) * SGF_S;
    base[q] = 2 * sr * SGF_P + 2 * sc;
    nt[q] = pr & 1;
    bv[q] = bias[nt[q] * 32 + li];
  }
  const int npair = wave < 4 ? 3 : 2;
  auto patch_load = [&](int t, int (&v)[SGF_PL]) {
    const int b = t / 49, tt = t - (t / 49) * 49;
    const int r0 = 4 * (tt / 7) * 8 - 5, c0 = 4 * (tt - (tt / 7) * 7) * 8 - 5;
#pragma unroll
    for (int j = 0; j < SGF_PL; ++j) {
      const int i = tid + 512 * j;
      const int pr = i / SGF_P, pc = i - (i / SGF_P) * SGF_P;
      const int ih = r0 + pr, iw = c0 + pc;
      v[j] = (i < SGF_P * SGF_P && ih >= 0 && ih < 224 && iw >= 0 && iw < 224) ? (int)img[((size_t)b * 224 + ih) * 224 + iw]
                                                                                : -1;
    }
  };
  auto patch_store = [&](const int (&v)[SGF_PL]) {
#pragma unroll
    for (int j = 0; j < SGF_PL; ++j) {
      const int i = tid + 512 * j;
      if (i < SGF_P * SGF_P) {
        hpair h;
        h.x = v[j] >= 0 ? (f16)(float)v[j] : (f16)0.f;
        h.y = v[j] >= 0 ? (f16)1.f : (f16)0.f;
        patch[i] = h;
      }
    }
  };
  // per k-step s, this lane half's two taps t0 = 4s + 2kk, t1 = t0 + 1: patch offsets (kh * P + kw)
  int toff[13][2];
  bool tin[13][2];
#pragma unroll
  for (int st = 0; st < 13; ++st)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = 4 * st + 2 * kk + u;
      tin[st][u] = t < 49;
      toff[st][u] = t < 49 ? (t / 7) * SGF_P + (t - (t / 7) * 7) : 0;
    }
  int pv[SGF_PL];
  if (blockIdx.x < ntiles) {
    patch_load(blockIdx.x, pv);
    patch_store(pv);
  }
  // the B operands for the launch, in registers: nt[q] = (wave + 8 q) & 1 is the same for every q,
  // so a lane needs one (lo, hi) pair of half4 per k-step (52 VGPRs) instead of 8 two-byte LDS
  // reads per MFMA pair inside the tile loop
  __syncthreads();  // swh / swl complete
  half4 wl[13], wh[13];
#pragma unroll
  for (int st = 0; st < 13; ++st) {
    const int w0 = ((4 * st + 2 * kk) * 2) * 64 + nt[0] * 32 + li;  // [tap t0][ch 0][co]
    wl[st] = half4{swl[w0], swl[w0 + 64], swl[w0 + 128], swl[w0 + 192]};
    wh[st] = half4{swh[w0], swh[w0 + 64], swh[w0 + 128], swh[w0 + 192]};
  }
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int b = t / 49, tt = t - (t / 49) * 49;
    const int py0 = (tt / 7) * 8, px0 = (tt - (tt / 7) * 7) * 8;
    __syncthreads();
    const int tn = t + gridDim.x;
    if (tn < ntiles) patch_load(tn, pv);
    floatx16 acc[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;
#pragma unroll
    for (int st = 0; st < 13; ++st) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q < npair) {
          const hpair p0 = tin[st][0] ? patch[base[q] + toff[st][0]] : hpair{(f16)0.f, (f16)0.f};
          const hpair p1 = tin[st][1] ? patch[base[q] + toff[st][1]] : hpair{(f16)0.f, (f16)0.f};
          const half4 av = {p0.x, p0.y, p1.x, p1.y};
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x8f16(av, wl[st], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x8f16(av, wh[st], acc[q], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < npair)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int pix = ((wave + 8 * q) >> 1) * 32 + (e & 3) + 8 * (e >> 2) + 4 * kk;
          if (pix < SGF_NPIX) stg[pix * 64 + nt[q] * 32 + li] = fmaxf(__builtin_fmaf(acc[q][e], wscale, bv[q]), 0.f);
        }
    __syncthreads();
    if (tn < ntiles) patch_store(pv);
    const float4* stg4 = reinterpret_cast<const float4*>(stg);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = it * 512 + tid, pp = idx >> 4, cq = idx & 15;
      const int py = pp >> 3, px = pp & 7;
      float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int sr = 2 * py + dy, R = 2 * py0 - 1 + sr;
        if (R < 0 || R >= 112) continue;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int sc = 2 * px + dx, Cc = 2 * px0 - 1 + sc;
          if (Cc < 0 || Cc >= 112) continue;
          const float4 v = stg4[(sr * SGF_S + sc) * 16 + cq];
          m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
        }
      }
      const size_t o = (((size_t)b * 56 + py0 + py) * 56 + px0 + px) * 64 + cq * 4;
      const half4 h = {(f16)m.x, (f16)m.y, (f16)m.z, (f16)m.w};
      const half4 l = {(f16)(m.x - (float)h[0]), (f16)(m.y - (float)h[1]), (f16)(m.z - (float)h[2]),
                       (f16)(m.w - (float)h[3])};
      *reinterpret_cast<half4*>(y + o) = h;
      *reinterpret_cast<half4*>(y + lo + o) = l;
      x3_raise(flag, x3_out_of_range4(m));
    }
  }
}

int ImageModel::create_f32(const float* blob, size_t n) {
  BlobReader rd(blob, n);
  std::vector<float> w;
  std::vector<float> pr;
  // BN output estimate (fp32x3 activation planes, activation_exp): max_c |beta_c| + 6 |gamma_c|
  double est = 0.0;
  auto bn_fold = [&](int c, std::vector<float>& scale) {
    const float* g = rd.take(c);
    const float* b = rd.take(c);
    const float* rm = rd.take(c);
    const float* rv = rd.take(c);
    scale.resize(c);
    const size_t off = pr.size();
    est = 0.0;
    for (int i = 0; i < c; ++i) {
      const double sc = (double)g[i] / std::sqrt((double)rv[i] + 1e-5);
      scale[i] = (float)sc;
      pr.push_back((float)((double)b[i] - (double)rm[i] * sc));
      est = std::max(est, std::fabs((double)b[i]) + 6.0 * std::fabs((double)g[i]));
    }
    return off;
  };
  auto conv = [&](int cout, int cin, int ks, int stride, int pad) {
    ConvLayer L;
    L.cin = cin; L.cout = cout; L.ks = ks; L.stride = stride; L.pad = pad;
    const float* src = rd.take((size_t)cout * cin * ks * ks);
    std::vector<float> scale;
    L.b_off = bn_fold(cout, scale);
    L.x3_est = est;
    L.w_off = w.size();
    w.resize(w.size() + (size_t)cout * cin * ks * ks);
    if (!rd.ok) return L;
    for (int o = 0; o < cout; ++o)
      for (int kh = 0; kh < ks; ++kh)
        for (int kw = 0; kw < ks; ++kw)
          for (int c = 0; c < cin; ++c)
            w[L.w_off + (((size_t)o * ks + kh) * ks + kw) * cin + c] =
                (float)((double)src[(((size_t)o * cin + c) * ks + kh) * ks + kw] * scale[o]);
    return L;
  };
  {  // stem: [64][160], k = c*49 + kh*7 + kw (torch [64][3][7][7] order), BN scale folded
    const float* src = rd.take((size_t)64 * 3 * 49);
    std::vector<float> scale;
    stem.b_off = bn_fold(64, scale);
    stem.x3_est = est;
    stem.cin = 3; stem.cout = 64; stem.ks = 7; stem.stride = 2; stem.pad = 3;
    stem.w_off = w.size();
    w.resize(w.size() + (size_t)64 * STEM_K, 0.f);
    if (rd.ok)
      for (int o = 0; o < 64; ++o)
        for (int k = 0; k < 147; ++k) w[stem.w_off + (size_t)o * STEM_K + k] = (float)((double)src[o * 147 + k] * scale[o]);
    // gray-input fold (stem_pool_gray_f32_kernel): [49 taps][pixel, inside][64]
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
    stem_gray32_off = w.size();
    w.resize(w.size() + 49 * 2 * 64, 0.f);
    if (rd.ok)
      for (int o = 0; o < 64; ++o)
        for (int t = 0; t < 49; ++t) {
          double g = 0.0, m = 0.0;
          for (int c = 0; c < 3; ++c) {
            const double wc = (double)src[o * 147 + c * 49 + t] * scale[o];
            g += wc / (255.0 * stdv[c]);
            m -= wc * mean[c] / stdv[c];
          }
          w[stem_gray32_off + ((size_t)t * 2 + 0) * 64 + o] = (float)g;
          w[stem_gray32_off + ((size_t)t * 2 + 1) * 64 + o] = (float)m;
        }
  }
  blocks.clear();
  int cin = 64;
  for (int li = 0; li < 4; ++li) {
    const int wd = kLayers32[li][0], nb = kLayers32[li][1], st = kLayers32[li][2];
    for (int b = 0; b < nb; ++b) {
      Bottleneck bk;
      const int s = b == 0 ? st : 1;
      bk.c1 = conv(wd, cin, 1, 1, 0);
      bk.c2 = conv(wd, wd, 3, s, 1);
      bk.c3 = conv(4 * wd, wd, 1, 1, 0);
      if (b == 0) {
        bk.has_ds = true;
        bk.ds = conv(4 * wd, cin, 1, s, 0);
      }
      blocks.push_back(bk);
      cin = 4 * wd;
    }
  }
  const float* f1w = rd.take((size_t)512 * 2048);
  const float* f1b = rd.take(512);
  const float* f2w = rd.take((size_t)7 * 512);
  const float* f2b = rd.take(7);
  MEC_REQUIRE(rd.ok && rd.off == n, "image blob size mismatch");
  fc1_off = pr.size();
  pr.resize(pr.size() + (size_t)2048 * 512);
  for (int i = 0; i < 2048; ++i)
    for (int j = 0; j < 512; ++j) pr[fc1_off + (size_t)i * 512 + j] = f1w[(size_t)j * 2048 + i];
  fc1b_off = pr.size();
  pr.insert(pr.end(), f1b, f1b + 512);
  fc2_off = pr.size();
  pr.resize(pr.size() + 512 * 7);
  for (int i = 0; i < 512; ++i)
    for (int j = 0; j < 7; ++j) pr[fc2_off + (size_t)i * 7 + j] = f2w[(size_t)j * 512 + i];
  fc2b_off = pr.size();
  pr.insert(pr.end(), f2b, f2b + 7);
  MEC_TRY(upload(wts32, w.data(), w.size() * sizeof(float)));
  MEC_TRY(upload(prm, pr.data(), pr.size() * sizeof(float)));
  if (prec == PREC_FP32X3) {
    // every bottleneck conv's weights scaled by 2^e and split into f16 hi / lo planes, at the
    // same offsets as in wts32 (the stem keeps its f32 weights: it runs the fp32 kernels)
    std::vector<f16> hl(2 * w.size(), (f16)0.f);
    x3_lo = w.size();
    {  // the gray stem's folded weights: split on the device (stem_pool_gray_x3_kernel) at scale 2^e
      float mx = 0.f;
      for (int i = 0; i < 49 * 2 * 64; ++i) mx = std::max(mx, std::fabs(w[stem_gray32_off + i]));
      int e = 0;
      if (mx > 0.f) {
        e = (int)std::floor(std::log2(16384.0 / (double)mx));
        while (std::ldexp((double)mx, e) > 16384.0) --e;
      }
      stem_x3_up = std::ldexp(1.0f, e);
      stem.x3_scale = std::ldexp(1.0f, -e);
    }
    // Activation-plane scales (activation_exp, BN estimates): the stem output, each block's conv1 /
    // conv2 outputs, and one scale per stage for the residual stream (a block's output and its
    // identity input share it). A conv's planes then carry y 2^s_out for input planes x 2^s_in: its
    // epilogue scale becomes 2^-e 2^(s_out - s_in) and its BN shift b 2^s_out (ReLU and the residual
    // add commute with the power of two: the f32 values are the unscaled ones times 2^s_out exactly).
    // The downsample of a stage's first block reads the block input (s_in) beside conv3's T2 (s_t2)
    // in one dual GEMM: its weights are pre-scaled by 2^(s_t2 - s_in) so both halves of K carry 2^s_t2.
    // opts.x3_plane_scale 0: every exponent 0 (the unscaled planes, A/B only)
    // opts.x3_headroom: 2^-x3_headroom of the target (a handle re-created after a range trip)
    auto aexp = [&](double b, double t) {
      return opts.x3_plane_scale ? activation_exp(b, std::ldexp(t, -opts.x3_headroom)) : 0;
    };
    stem.x3_s = aexp(stem.x3_est, kX3EstimateTarget);
    x3_note("stem", stem.x3_s, stem.x3_est);
    {
      int s_prev = stem.x3_s;
      int stage = 0;
      double e_stream = stem.x3_est;
      for (size_t b0 = 0; b0 < blocks.size();) {
        size_t b1 = b0 + 1;
        while (b1 < blocks.size() && !blocks[b1].has_ds) ++b1;  // [b0, b1): one stage
        double e_max = 0.0;
        for (size_t bi = b0; bi < b1; ++bi) {
          Bottleneck& bk = blocks[bi];
          e_stream = bk.c3.x3_est + (bk.has_ds ? bk.ds.x3_est : e_stream);
          e_max = std::max(e_max, e_stream);
        }
        const int s_stage = aexp(e_max, kX3EstimateTarget);
        const std::string st = "layer" + std::to_string(stage + 1);
        x3_note(st + ".out", s_stage, e_max);
        for (size_t bi = b0; bi < b1; ++bi) {
          Bottleneck& bk = blocks[bi];
          bk.c1.x3_s = aexp(bk.c1.x3_est, kX3EstimateTarget);
          bk.c2.x3_s = aexp(bk.c2.x3_est, kX3EstimateTarget);
          bk.c3.x3_s = s_stage;
          bk.x3_s_in = bi == b0 ? s_prev : s_stage;
          const std::string bn = st + "." + std::to_string(bi - b0);
          x3_note(bn + ".conv1", bk.c1.x3_s, bk.c1.x3_est);
          x3_note(bn + ".conv2", bk.c2.x3_s, bk.c2.x3_est);
        }
        ++stage;
        s_prev = s_stage;
        b0 = b1;
      }
      x3_s_out = s_prev;
    }
    auto scaled_bias = [&](size_t b_off, int cout, int s) {
      const size_t off = pr.size();
      for (int o = 0; o < cout; ++o) pr.push_back(std::ldexp(pr[b_off + o], s));
      return off;
    };
    stem.x3b_off = scaled_bias(stem.b_off, 64, stem.x3_s);
    auto split = [&](ConvLayer& L, int s_in) {
      const size_t cnt = (size_t)L.cout * L.cin * L.ks * L.ks;
      L.x3_scale = std::ldexp(split_planes(w.data() + L.w_off, cnt, hl.data() + L.w_off, hl.data() + x3_lo + L.w_off),
                              L.x3_s - s_in);
      L.x3b_off = scaled_bias(L.b_off, L.cout, L.x3_s);
    };
    for (Bottleneck& bk : blocks) {
      split(bk.c1, bk.x3_s_in);
      split(bk.c2, bk.c1.x3_s);
      split(bk.c3, bk.c2.x3_s);
    }
    // block 0 of each stage: conv3 and the downsample as ONE dual-source GEMM over K = [w | cin]
    // (the f16 path's A_DUAL), weights [W3 | Wds 2^(s_t2 - s_in)] split with one scale, bias b3 + bds
    std::vector<float> cat;
    std::vector<f16> hl2;
    for (Bottleneck& bk : blocks) {
      if (!bk.has_ds) continue;
      const int wd = bk.c3.cin, cin = bk.ds.cin, Kt = wd + cin, No = bk.c3.cout;
      const int dsh = bk.c2.x3_s - bk.x3_s_in;
      cat.assign((size_t)No * Kt, 0.f);
      for (int o = 0; o < No; ++o) {
        for (int k = 0; k < wd; ++k) cat[(size_t)o * Kt + k] = w[bk.c3.w_off + (size_t)o * wd + k];
        for (int k = 0; k < cin; ++k) cat[(size_t)o * Kt + wd + k] = std::ldexp(w[bk.ds.w_off + (size_t)o * cin + k], dsh);
      }
      bk.c3ds_w_off = hl2.size();
      hl2.resize(hl2.size() + 2 * cat.size());
      bk.c3ds_x3_scale = std::ldexp(split_planes(cat.data(), cat.size(), hl2.data() + bk.c3ds_w_off,
                                                 hl2.data() + bk.c3ds_w_off + cat.size()),
                                    bk.c3.x3_s - bk.c2.x3_s);
      bk.c3ds_x3_lo = cat.size();
      bk.c3ds_b_off = pr.size();
      for (int o = 0; o < No; ++o) pr.push_back(std::ldexp(pr[bk.c3.b_off + o] + pr[bk.ds.b_off + o], bk.c3.x3_s));
    }
    MEC_TRY(upload(wts, hl.data(), hl.size() * sizeof(f16)));
    MEC_TRY(upload(wts_dual, hl2.data(), hl2.size() * sizeof(f16)));
    MEC_TRY(upload(prm, pr.data(), pr.size() * sizeof(float)));  // + the dual biases
  }
  return 0;
}

// fp32 tensor -> f16 hi / lo planes (the fp32x3 path's stem output): hi = f16(x up), lo = f16(x up - hi)
__global__ __launch_bounds__(256) void split_f32_kernel(const float* __restrict__ x, size_t n4, float up,
                                                        f16* __restrict__ hi, long long lo, unsigned* flag) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 v = reinterpret_cast<const float4*>(x)[i];
  v.x *= up; v.y *= up; v.z *= up; v.w *= up;  // the planes' scale (a power of two: exact)
  const half4 h = {(f16)v.x, (f16)v.y, (f16)v.z, (f16)v.w};
  const half4 l = {(f16)(v.x - (float)h[0]), (f16)(v.y - (float)h[1]), (f16)(v.z - (float)h[2]),
                   (f16)(v.w - (float)h[3])};
  reinterpret_cast<half4*>(hi)[i] = h;
  reinterpret_cast<half4*>(hi + lo)[i] = l;
  x3_raise(flag, x3_out_of_range4(v));
}

// global average pool of an NHWC tensor held as f16 hi / lo planes (x 2^s = hi + lo exactly), the
// same summation order as avgpool_f32_kernel, then times down = 2^-s (exact)
__global__ __launch_bounds__(256) void avgpool_split_kernel(const f16* __restrict__ x, long long lo, int HW, int C,
                                                            float down, float* __restrict__ y) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const f16* p = x + (size_t)b * HW * C + c;
  float s = 0.f;
  for (int q = 0; q < HW; ++q) s += (float)p[(size_t)q * C] + (float)p[(size_t)q * C + lo];
  y[(size_t)b * C + c] = (s / (float)HW) * down;
}

int ImageModel::forward_f32(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                            hipStream_t s) {
  MEC_REQUIRE(wts32.p, "image: fp32 weights missing (handle created at f16 precision)");
  const bool fer = (H == 48 && W == 48 && C == 1);
  // per image (floats): im2col 12544 x 160; X, Y, DS 56*56*256 (also the 112*112*64 stem
  // output); T1 56*56*128; T2 56*56*64; pooled 2048
  const size_t big = (size_t)56 * 56 * 256;
  const size_t per_img = 224 * 224 + ((size_t)12544 * STEM_K + 3 * big + 56 * 56 * 128 + 56 * 56 * 64 + 2048) * 4;
  const size_t need = per_img * (size_t)B + 8192;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  float* A0 = reinterpret_cast<float*>(p); p += (size_t)B * 12544 * STEM_K * 4;
  float* X = reinterpret_cast<float*>(p); p += (size_t)B * big * 4;
  float* Y = reinterpret_cast<float*>(p); p += (size_t)B * big * 4;
  float* DS = reinterpret_cast<float*>(p); p += (size_t)B * big * 4;
  float* T1 = reinterpret_cast<float*>(p); p += (size_t)B * 56 * 56 * 128 * 4;
  float* T2 = reinterpret_cast<float*>(p); p += (size_t)B * 56 * 56 * 64 * 4;
  float* pooled = reinterpret_cast<float*>(p);

  const float* Wt = wts32.as<float>();
  const float* P = prm.as<float>();
  const uint8_t* stem_in = img;
  int Cin = C;
  if (fer) {
    MEC_TRY(resize_u8(img, B, 48, 48, resized, 224, 224, s));
    stem_in = resized;
    Cin = 1;
  }
  MEC_TRY(prof.begin(TAG_RESNET_STEM, s));
  if (Cin == 1 && opt().stem_gray_f32) {  // conv + BN + ReLU + maxpool in one kernel -> X
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      MEC_HIP(hipGetDevice(&dev));
      MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int ntiles = B * 49;
    hipLaunchKernelGGL(stem_pool_gray_f32_kernel, dim3(std::min(ntiles, ncu)), dim3(512), 0, s, stem_in, ntiles,
                       Wt + stem_gray32_off, P + stem.b_off, X);
    MEC_LAUNCH_CHECK();
    MEC_TRY(prof.end(TAG_RESNET_STEM, s));
  } else {
    {
      const size_t total = (size_t)B * 112 * 112 * (STEM_K / 4);
      hipLaunchKernelGGL(stem_im2col_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, stem_in, B,
                         Cin, A0);
      MEC_LAUNCH_CHECK();
    }
    MEC_TRY(prof.end(TAG_RESNET_STEM, s));
    GemmParams g;
    g.A = A0; g.B32 = Wt + stem.w_off; g.bias = P + stem.b_off; g.act = ACT_RELU; g.C32 = Y;
    g.M = B * 112 * 112; g.N = 64; g.K = STEM_K;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_RESNET_STEM));
    const size_t total = (size_t)B * 56 * 56 * 16;
    hipLaunchKernelGGL(maxpool_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, Y, B, 112, 64, 56, X);
    MEC_LAUNCH_CHECK();
  }
  GemmParams g;
  float* cur = X;
  float* other = Y;
  int Hc = 56;
  for (const Bottleneck& bk : blocks) {
    const int wd = bk.c1.cout, cin = bk.c1.cin, st = bk.c2.stride;
    const int OH = (Hc + 2 - 3) / st + 1;
    g = GemmParams();
    g.A = cur; g.B32 = Wt + bk.c1.w_off; g.bias = P + bk.c1.b_off; g.act = ACT_RELU; g.C32 = T1;
    g.M = B * Hc * Hc; g.N = wd; g.K = cin;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_RESNET_CONV1X1));
    g = GemmParams();
    g.amode = A_CONV; g.A = T1; g.B32 = Wt + bk.c2.w_off; g.bias = P + bk.c2.b_off; g.act = ACT_RELU; g.C32 = T2;
    g.M = B * OH * OH; g.N = wd; g.K = 9 * wd;
    g.H = Hc; g.W = Hc; g.C = wd; g.OH = OH; g.OW = OH; g.ks = 3; g.stride = st; g.pad = 1;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_RESNET_CONV3X3));
    const float* idn = cur;
    if (bk.has_ds) {  // downsample = BN(conv1x1/s(x)), no activation
      g = GemmParams();
      g.amode = A_CONV; g.A = cur; g.B32 = Wt + bk.ds.w_off; g.bias = P + bk.ds.b_off; g.C32 = DS;
      g.M = B * OH * OH; g.N = 4 * wd; g.K = cin;
      g.H = Hc; g.W = Hc; g.C = cin; g.OH = OH; g.OW = OH; g.ks = 1; g.stride = st; g.pad = 0;
      MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_RESNET_CONV1X1));
      idn = DS;
    }
    g = GemmParams();  // relu(bn3(conv3(t2)) + identity)
    g.A = T2; g.B32 = Wt + bk.c3.w_off; g.bias = P + bk.c3.b_off; g.R = idn; g.r_f32 = 1; g.act = ACT_RELU;
    g.C32 = other; g.M = B * OH * OH; g.N = 4 * wd; g.K = wd;
    MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_RESNET_CONV1X1));
    std::swap(cur, other);
    Hc = OH;
  }
  hipLaunchKernelGGL(avgpool_f32_kernel, dim3(B, 2048 / 256), dim3(256), 0, s, cur, Hc * Hc, 2048, pooled);
  MEC_LAUNCH_CHECK();
  MEC_TRY(launch_linear_mfma<BACT_RELU>(pooled, 2048, B, 2048, P + fc1_off, P + fc1b_off, 512, feat, 512, nullptr, 0, s));
  MEC_TRY(launch_head7(feat, B, 512, P + fc2_off, P + fc2b_off, logits, probs, s));
  return 0;
}

// fp32x3 path: the fp32 path with every bottleneck conv on split-f16 operands (gemm_glds.hip
// split mode: A_PLAIN 1x1 convs, A_CONV 3x3 convs, and each stage's first block's conv3 +
// downsample as one A_DUAL GEMM over K = [w | cin]; three f16 MFMA passes into one fp32
// accumulator, weights pre-scaled by 2^e and undone in the epilogue). Activations between convs
// are f16 hi / lo planes (the same bytes as f32) in one arena whose lo half sits a fixed L
// elements after the hi half, so every operand -- both sources of a dual GEMM included -- finds
// its lo plane at the same offset; an identity residual is added as hi + lo (exact). The stem
// (conv + BN + ReLU + max-pool), the average pool and the head are the fp32 path's kernels.
int ImageModel::forward_x3(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                           hipStream_t s) {
  MEC_REQUIRE(wts.p && wts32.p && wts_dual.p && x3_lo, "image: fp32x3 weights missing");
  const bool fer = (H == 48 && W == 48 && C == 1);
  // per image: im2col 12544 x 160 f32 (RGB stem); S32 f32 56*56*64 (stem out; the RGB stem's
  // 112*112*64 pre-pool map goes to the arena's bytes); arena hi half: X, Y (56*56*256), T1
  // (56*56*128), T2 (56*56*64) halfs, then the lo half (same layout)
  const size_t big = (size_t)56 * 56 * 256, t1n = (size_t)56 * 56 * 128, t2n = (size_t)56 * 56 * 64;
  const size_t arena_img = 2 * big + t1n + t2n;  // halfs per image per half-arena
  const size_t per_img = 224 * 224 + ((size_t)12544 * STEM_K + (size_t)56 * 56 * 64 + 2048) * 4 + arena_img * 2 * 2;
  const size_t need = per_img * (size_t)B + 8192;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  float* A0 = reinterpret_cast<float*>(p); p += (size_t)B * 12544 * STEM_K * 4;
  float* S32 = reinterpret_cast<float*>(p); p += (size_t)B * 56 * 56 * 64 * 4;
  float* pooled = reinterpret_cast<float*>(p); p += (size_t)B * 2048 * 4;
  f16* arena = reinterpret_cast<f16*>(p);
  const long long L = (long long)B * arena_img;  // lo plane = hi plane + L, for every activation
  f16* X = arena;
  f16* Y = X + (size_t)B * big;
  // the stem output [B,56,56,64] sits in the last quarter of X: a chunk's layer-1 outputs (4x the
  // per-image stride) then never reach the stem output of a later chunk's images (resnet_chunk)
  f16* Xs = X + (size_t)3 * B * 56 * 56 * 64;
  f16* T1 = Y + (size_t)B * big;
  f16* T2 = T1 + (size_t)B * t1n;

  const float* Wt32 = wts32.as<float>();
  const f16* Wt = wts.as<f16>();
  const f16* Wd = wts_dual.as<f16>();
  const long long wlo = (long long)x3_lo;
  const float* P = prm.as<float>();
  const uint8_t* stem_in = img;
  int Cin = C;
  if (fer) {
    MEC_TRY(resize_u8(img, B, 48, 48, resized, 224, 224, s));
    stem_in = resized;
    Cin = 1;
  }
  // stem -> S32 f32 [B,56,56,64] (the fp32 path's kernels), then split into X's planes
  MEC_TRY(prof.begin(TAG_RESNET_STEM, s));
  if (Cin == 1 && opt().stem_gray_f32) {  // conv + BN + ReLU + pool on split weights -> X's planes
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      MEC_HIP(hipGetDevice(&dev));
      MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int ntiles = B * 49;
    hipLaunchKernelGGL(stem_pool_gray_x3_kernel, dim3(std::min(ntiles, ncu)), dim3(512), 0, s, stem_in, ntiles,
                       Wt32 + stem_gray32_off, stem_x3_up, std::ldexp(stem.x3_scale, stem.x3_s), P + stem.x3b_off, Xs, L,
                       range_flag());
    MEC_LAUNCH_CHECK();
  } else {
    const size_t total = (size_t)B * 112 * 112 * (STEM_K / 4);
    hipLaunchKernelGGL(stem_im2col_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, stem_in, B,
                       Cin, A0);
    MEC_LAUNCH_CHECK();
    GemmParams g;  // the 112 x 112 pre-pool map (B * 802816 floats) fits in the arena's bytes
    float* Y32 = reinterpret_cast<float*>(arena);
    g.A = A0; g.B32 = Wt32 + stem.w_off; g.bias = P + stem.b_off; g.act = ACT_RELU; g.C32 = Y32;
    g.M = B * 112 * 112; g.N = 64; g.K = STEM_K;
    MEC_TRY(launch_gemm_f32(g, s, nullptr, 0));
    const size_t tp = (size_t)B * 56 * 56 * 16;
    hipLaunchKernelGGL(maxpool_f32_kernel, dim3((unsigned)((tp + 255) / 256)), dim3(256), 0, s, Y32, B, 112, 64, 56, S32);
    MEC_LAUNCH_CHECK();
    const size_t n4 = (size_t)B * 56 * 56 * 64 / 4;
    hipLaunchKernelGGL(split_f32_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, S32, n4,
                       std::ldexp(1.0f, stem.x3_s), Xs, L, range_flag());
    MEC_LAUNCH_CHECK();
  }
  MEC_TRY(prof.end(TAG_RESNET_STEM, s));
  // Bottleneck blocks [b0, b1) over images [i0, i0 + nb) (NHWC planes are image-major: an image range
  // is a pointer offset; the lo planes stay L elements after their hi planes). cur/other swap per block.
  // a layer-2 seam into layer3's first block (pw_seam_x3 2) runs that block's conv1 in the previous call
  bool carry_conv1 = false;
  auto run_blocks = [&](size_t b0, size_t b1, int i0, int nb, int Hin, f16*& cur, f16*& other, bool cross) -> int {
    int Hc = Hin;
    bool conv1_done = carry_conv1;  // this block's conv1 already ran in the previous block's seam kernel
    carry_conv1 = false;
    for (size_t bi = b0; bi < b1; ++bi) {
      const Bottleneck& bk = blocks[bi];
      const int wd = bk.c1.cout, cin = bk.c1.cin, st = bk.c2.stride;
      const int OH = (Hc + 2 - 3) / st + 1;
      f16* in = (bi == 0 ? Xs : cur) + (size_t)i0 * Hc * Hc * cin;
      f16* out = other + (size_t)i0 * OH * OH * 4 * wd;
      f16* t1 = T1 + (size_t)i0 * Hc * Hc * wd;
      f16* t2 = T2 + (size_t)i0 * OH * OH * wd;
      GemmParams g;
      if (!conv1_done) {
        g.split = 1; g.A = in; g.a_lo = L; g.B = Wt + bk.c1.w_off; g.b_lo = wlo; g.oscale = bk.c1.x3_scale;
        g.bias = P + bk.c1.x3b_off; g.act = ACT_RELU; g.C16 = t1; g.c_lo = L;
        g.M = nb * Hc * Hc; g.N = wd; g.K = cin;
        MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
      }
      conv1_done = false;
      g = GemmParams();
      g.split = 1; g.amode = A_CONV; g.A = t1; g.a_lo = L; g.B = Wt + bk.c2.w_off; g.b_lo = wlo;
      g.oscale = bk.c2.x3_scale; g.bias = P + bk.c2.x3b_off; g.act = ACT_RELU; g.C16 = t2; g.c_lo = L;
      g.M = nb * OH * OH; g.N = wd; g.K = 9 * wd;
      g.H = Hc; g.W = Hc; g.C = wd; g.OH = OH; g.OW = OH; g.ks = 3; g.stride = st; g.pad = 1;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV3X3));
      // layer1 seams (pw_chain_x3.hip): conv3 (+ downsample or + residual) + ReLU, then the next
      // block's conv1 on the rows just produced; the block output's planes are not read back
      const int sx = opt().pw_chain_x3;
      const Bottleneck* nx = bi + 1 < b1 ? &blocks[bi + 1] : nullptr;
      const bool seam = sx && nx && wd == 64 && OH == 56 && nx->c1.cin == 256 &&
                        (nx->c1.cout == 64 || (sx == 2 && nx->c1.cout == 128)) &&
                        (!bk.has_ds || (st == 1 && cin == 64 && nx->c1.cout == 64));
      if (seam) {
        MEC_TRY(prof.begin(TAG_RESNET_CONV1X1, s));
        if (bk.has_ds)
          MEC_TRY(launch_pw_chain_x3(t2, in, L, Wd + bk.c3ds_w_off, (long long)bk.c3ds_x3_lo, bk.c3ds_x3_scale,
                                     P + bk.c3ds_b_off, Wt + nx->c1.w_off, wlo, nx->c1.x3_scale, P + nx->c1.x3b_off, out,
                                     T1 + (size_t)i0 * OH * OH * nx->c1.cout, nb * OH * OH, nx->c1.cout, true, s));
        else
          MEC_TRY(launch_pw_chain_x3(t2, in, L, Wt + bk.c3.w_off, wlo, bk.c3.x3_scale, P + bk.c3.x3b_off,
                                     Wt + nx->c1.w_off, wlo, nx->c1.x3_scale, P + nx->c1.x3b_off, out,
                                     T1 + (size_t)i0 * OH * OH * nx->c1.cout, nb * OH * OH, nx->c1.cout, false, s));
        MEC_TRY(prof.end(TAG_RESNET_CONV1X1, s));
        conv1_done = true;
        std::swap(cur, other);
        Hc = OH;
        continue;
      }
      // layer-2 seams (pw_seam_x3.hip): conv3 + identity residual + ReLU, then the next block's conv1 (in
      // layer2, or layer3's first block when `cross`), the block output walked in 32-channel chunks
      const int sq = opt().pw_seam_x3;
      const Bottleneck* nq = bi + 1 < b1 ? &blocks[bi + 1] : (cross && bi + 1 < blocks.size() ? &blocks[bi + 1] : nullptr);
      const bool seam2 = sq && nq && !bk.has_ds && wd == 128 && nq->c1.cin == 512 &&
                         (nq->c1.cout == 128 || (sq == 2 && nq->c1.cout == 256));
      if (seam2) {
        MEC_TRY(prof.begin(TAG_RESNET_CONV1X1, s));
        MEC_TRY(launch_pw_seam_x3(t2, in, L, Wt + bk.c3.w_off, wlo, bk.c3.x3_scale, P + bk.c3.x3b_off,
                                  Wt + nq->c1.w_off, wlo, nq->c1.x3_scale, P + nq->c1.x3b_off, out,
                                  T1 + (size_t)i0 * OH * OH * nq->c1.cout, nb * OH * OH, wd, nq->c1.cout, s));
        MEC_TRY(prof.end(TAG_RESNET_CONV1X1, s));
        if (bi + 1 < b1) conv1_done = true;
        else carry_conv1 = true;
        std::swap(cur, other);
        Hc = OH;
        continue;
      }
      g = GemmParams();
      g.split = 1; g.a_lo = L; g.act = ACT_RELU; g.C16 = out; g.c_lo = L; g.M = nb * OH * OH; g.N = 4 * wd;
      if (bk.has_ds) {  // relu(bn3(conv3(t2)) + bn_ds(conv_ds/s(x))) as one GEMM over K = [w | cin]
        g.amode = A_DUAL; g.A = t2; g.K1 = wd; g.A2 = in; g.B = Wd + bk.c3ds_w_off; g.b_lo = (long long)bk.c3ds_x3_lo;
        g.oscale = bk.c3ds_x3_scale; g.bias = P + bk.c3ds_b_off; g.K = wd + cin;
        g.H = Hc; g.W = Hc; g.C = cin; g.OH = OH; g.OW = OH; g.ks = 1; g.stride = st; g.pad = 0;
      } else {  // relu(bn3(conv3(t2)) + x)
        g.A = t2; g.B = Wt + bk.c3.w_off; g.b_lo = wlo; g.oscale = bk.c3.x3_scale; g.bias = P + bk.c3.x3b_off;
        g.R = in; g.r_lo = L; g.K = wd;
      }
      MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
      std::swap(cur, other);
      Hc = OH;
    }
    return 0;
  };
  // Layers 1-2 over chunks of opt().resnet_chunk images (0 = the whole batch), so that a chunk's hi /
  // lo activations can stay in the 256-MB Infinity Cache between a block's producer and consumer
  // kernels. Every GEMM row and conv pixel is computed the same way at any batch split (every
  // interleaved split tile sums in one k order), so the outputs do not depend on the chunk size.
  constexpr size_t kL12 = 7;  // layer1 (3 blocks) + layer2 (4 blocks)
  f16* cur = X;
  f16* other = Y;
  const int chunk = opt().resnet_chunk > 0 ? std::min(opt().resnet_chunk, B) : B;
  for (int i0 = 0; i0 < B; i0 += chunk) {
    f16* c = X;
    f16* o = Y;
    MEC_TRY(run_blocks(0, kL12, i0, std::min(chunk, B - i0), 56, c, o, chunk == B));
    cur = c;
    other = o;
  }
  MEC_TRY(run_blocks(kL12, blocks.size(), 0, B, 28, cur, other, false));
  const int Hc = 7;
  hipLaunchKernelGGL(avgpool_split_kernel, dim3(B, 2048 / 256), dim3(256), 0, s, cur, L, Hc * Hc, 2048,
                     std::ldexp(1.0f, -x3_s_out), pooled);
  MEC_LAUNCH_CHECK();
  MEC_TRY(launch_linear_mfma<BACT_RELU>(pooled, 2048, B, 2048, P + fc1_off, P + fc1b_off, 512, feat, 512, nullptr, 0, s));
  MEC_TRY(launch_head7(feat, B, 512, P + fc2_off, P + fc2b_off, logits, probs, s));
  return 0;
}

}  // namespace mec
