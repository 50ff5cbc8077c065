// MobileNetV2 image path in fp32 (mec_create_ex(MEC_IMAGE_MBV2, ..., MEC_PREC_FP32)): the
// same head and transform as the ResNet50 path (inference/image_inference.py:28-32, :59-65) on
// torchvision's mobilenet_v2 backbone (README.md:13; oracle/image_mbv2.py restates it), every
// operand and product in fp32:
//   stem        explicit im2col of ToTensor + Normalize (torchvision's order), k = c*9 + kh*3
//               + kw (the torch weight order) padded 27 -> 32, then one fp32 GEMM to 32 channels
//               (stored 64 wide: the GEMM engine's N granularity) + BN + ReLU6
//   blocks      expand 1x1 (gemm_f32) + BN + ReLU6 -> depthwise 3x3/s + BN + ReLU6
//               (mbv2_dw_f32_kernel, fp32 FMA in torch's tap order) -> project 1x1 (gemm_f32)
//               + BN (+ the block input when stride 1 and cin == cout)
//   features[18] 1x1 320 -> 1280 + BN + ReLU6 (gemm_f32), average pool, fc head (block_ops.h)
// Activations are NHWC f32 with channels zero-padded to multiples of 64 (the engine's N
// granularity and a multiple of its 32-float K tiles): the padded channels stay exactly zero
// through every layer (zero weights and zero biases), so they never touch a real output.
#include <algorithm>
#include <cmath>

#include "block_ops.h"
#include "models.h"

namespace mec {

namespace {
constexpr int MB_STEM_K = 32;  // 27 taps padded to a 32-float K tile
int pad64(int v) { return (v + 63) / 64 * 64; }
}  // namespace

// stem im2col: one thread per 4 consecutive k of one 112 x 112 output pixel's row
__global__ __launch_bounds__(256) void mbv2_stem_im2col_f32_kernel(const uint8_t* __restrict__ img, int B, int C,
                                                                   float* __restrict__ A) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)B * 112 * 112 * (MB_STEM_K / 4);
  if (idx >= total) return;
  const int q = (int)(idx % (MB_STEM_K / 4));
  const size_t m = idx / (MB_STEM_K / 4);
  const int ow = (int)(m % 112), oh = (int)((m / 112) % 112);
  const size_t b = m / (112 * 112);
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * q + j;
    float x = 0.f;
    if (k < 27) {
      const int c = k / 9, tap = k - c * 9, kh = tap / 3, kw = tap - kh * 3;
      const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;
      if (ih >= 0 && ih < 224 && iw >= 0 && iw < 224) {
        const uint8_t px = img[((b * 224 + ih) * 224 + iw) * C + (C == 3 ? c : 0)];
        x = ((float)px / 255.0f - mean[c]) / stdv[c];
      }
    }
    v[j] = x;
  }
  *reinterpret_cast<float4*>(A + m * MB_STEM_K + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
}

// Depthwise 3x3 / stride S, padding 1, + BN shift + ReLU6 on NHWC f32 [B,H,H,Cp]: one thread
// per (output pixel, 4 channels); the taps accumulate in torch's (kh, kw) order from 0.
// Weights [9][Cp] (BN scale folded), bias [Cp].
__global__ __launch_bounds__(256) void mbv2_dw_f32_kernel(const float* __restrict__ x, int B, int H, int Cp, int S,
                                                          int OH, const float* __restrict__ w,
                                                          const float* __restrict__ bias, float* __restrict__ y) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int C4 = Cp / 4;
  const size_t total = (size_t)B * OH * OH * C4;
  if (idx >= total) return;
  const int c4 = (int)(idx % C4);
  const size_t pix = idx / C4;
  const int ow = (int)(pix % OH), oh = (int)((pix / OH) % OH);
  const size_t b = pix / ((size_t)OH * OH);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int ih = S * oh - 1 + kh;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int iw = S * ow - 1 + kw;
      if (ih < 0 || ih >= H || iw < 0 || iw >= H) continue;
      const float4 v = *reinterpret_cast<const float4*>(x + ((b * H + ih) * H + iw) * Cp + 4 * c4);
      const float4 k = *reinterpret_cast<const float4*>(w + (kh * 3 + kw) * Cp + 4 * c4);
      acc.x = fmaf(v.x, k.x, acc.x); acc.y = fmaf(v.y, k.y, acc.y);
      acc.z = fmaf(v.z, k.z, acc.z); acc.w = fmaf(v.w, k.w, acc.w);
    }
  }
  const float4 bb = *reinterpret_cast<const float4*>(bias + 4 * c4);
  float4 o;
  o.x = fminf(fmaxf(acc.x + bb.x, 0.f), 6.f); o.y = fminf(fmaxf(acc.y + bb.y, 0.f), 6.f);
  o.z = fminf(fmaxf(acc.z + bb.z, 0.f), 6.f); o.w = fminf(fmaxf(acc.w + bb.w, 0.f), 6.f);
  *reinterpret_cast<float4*>(y + idx * 4) = o;
}

int MobileNetModel::create_f32(const float* blob, size_t n) {
  BlobReader rd(blob, n);
  std::vector<float> w, pr;
  auto bn = [&](int c, std::vector<double>& scale, std::vector<double>& shift) {
    const float* g = rd.take(c);
    const float* b = rd.take(c);
    const float* rm = rd.take(c);
    const float* rv = rd.take(c);
    scale.assign(c, 0.0);
    shift.assign(c, 0.0);
    if (!rd.ok) return;
    for (int i = 0; i < c; ++i) {
      scale[i] = (double)g[i] / std::sqrt((double)rv[i] + 1e-5);
      shift[i] = (double)b[i] - (double)rm[i] * scale[i];
    }
  };
  auto align4 = [&](std::vector<float>& v) { while (v.size() % 4) v.push_back(0.f); };
  std::vector<double> sc, sh;
  {  // stem [64][32] (32 real output channels, k = c*9 + kh*3 + kw), bias [64]
    const float* src = rd.take((size_t)32 * 27);
    bn(32, sc, sh);
    stem_w_off = w.size();
    w.resize(w.size() + (size_t)64 * MB_STEM_K, 0.f);
    align4(pr);
    stem_corr_off = pr.size();  // fp32 path: the stem bias
    pr.resize(pr.size() + 64, 0.f);
    if (rd.ok)
      for (int o = 0; o < 32; ++o) {
        for (int k = 0; k < 27; ++k) w[stem_w_off + (size_t)o * MB_STEM_K + k] = (float)((double)src[o * 27 + k] * sc[o]);
        pr[stem_corr_off + o] = (float)sh[o];
      }
  }
  static const int kSet[7][4] = {{1, 16, 1, 1}, {6, 24, 2, 2}, {6, 32, 3, 2}, {6, 64, 4, 2},
                                 {6, 96, 3, 1}, {6, 160, 3, 2}, {6, 320, 1, 1}};
  blocks.clear();
  int cin = 32;
  for (int si = 0; si < 7; ++si)
    for (int r = 0; r < kSet[si][2]; ++r) {
      MbBlock b;
      b.t = kSet[si][0]; b.cin = cin; b.hid = cin * b.t; b.cout = kSet[si][1]; b.stride = r == 0 ? kSet[si][3] : 1;
      b.cinp = pad64(cin); b.hidp = pad64(b.hid); b.coutp = pad64(b.cout);
      if (b.t != 1) {  // expand [hidp][cinp], bias [hidp]
        const float* we = rd.take((size_t)b.hid * cin);
        bn(b.hid, sc, sh);
        b.we_off = w.size();
        w.resize(w.size() + (size_t)b.hidp * b.cinp, 0.f);
        align4(pr);
        b.be_off = pr.size();
        pr.resize(pr.size() + b.hidp, 0.f);
        if (rd.ok)
          for (int h = 0; h < b.hid; ++h) {
            for (int c = 0; c < cin; ++c) w[b.we_off + (size_t)h * b.cinp + c] = (float)((double)we[(size_t)h * cin + c] * sc[h]);
            pr[b.be_off + h] = (float)sh[h];
          }
      }
      {  // depthwise [9][hidp], bias [hidp]
        const float* wd = rd.take((size_t)b.hid * 9);
        bn(b.hid, sc, sh);
        align4(pr);
        b.wd_off = pr.size();
        pr.resize(pr.size() + (size_t)9 * b.hidp, 0.f);
        b.bd_off = pr.size();
        pr.resize(pr.size() + b.hidp, 0.f);
        if (rd.ok)
          for (int h = 0; h < b.hid; ++h) {
            for (int t = 0; t < 9; ++t) pr[b.wd_off + (size_t)t * b.hidp + h] = (float)((double)wd[(size_t)h * 9 + t] * sc[h]);
            pr[b.bd_off + h] = (float)sh[h];
          }
      }
      {  // project [coutp][hidp], bias [coutp]
        const float* wp = rd.take((size_t)b.cout * b.hid);
        bn(b.cout, sc, sh);
        b.wp_off = w.size();
        w.resize(w.size() + (size_t)b.coutp * b.hidp, 0.f);
        align4(pr);
        b.bp_off = pr.size();
        pr.resize(pr.size() + b.coutp, 0.f);
        if (rd.ok)
          for (int o = 0; o < b.cout; ++o) {
            for (int h = 0; h < b.hid; ++h) w[b.wp_off + (size_t)o * b.hidp + h] = (float)((double)wp[(size_t)o * b.hid + h] * sc[o]);
            pr[b.bp_off + o] = (float)sh[o];
          }
      }
      blocks.push_back(b);
      cin = b.cout;
    }
  {  // features[18]: [1280][320]
    const float* wl = rd.take((size_t)1280 * 320);
    bn(1280, sc, sh);
    last_w_off = w.size();
    w.resize(w.size() + (size_t)1280 * 320, 0.f);
    align4(pr);
    last_b_off = pr.size();
    pr.resize(pr.size() + 1280, 0.f);
    if (rd.ok)
      for (int o = 0; o < 1280; ++o) {
        for (int c = 0; c < 320; ++c) w[last_w_off + (size_t)o * 320 + c] = (float)((double)wl[(size_t)o * 320 + c] * sc[o]);
        pr[last_b_off + o] = (float)sh[o];
      }
  }
  const float* f1w = rd.take((size_t)512 * 1280);
  const float* f1b = rd.take(512);
  const float* f2w = rd.take((size_t)7 * 512);
  const float* f2b = rd.take(7);
  MEC_REQUIRE(rd.ok && rd.off == n, "image_mbv2 blob size mismatch");
  align4(pr);
  fc1_off = pr.size();
  pr.resize(pr.size() + (size_t)1280 * 512);
  for (int i = 0; i < 1280; ++i)
    for (int j = 0; j < 512; ++j) pr[fc1_off + (size_t)i * 512 + j] = f1w[(size_t)j * 1280 + i];
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
  return 0;
}

int MobileNetModel::forward_f32(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits,
                                float* probs, hipStream_t s) {
  MEC_REQUIRE(wts32.p, "image_mbv2: fp32 weights missing (handle created at f16 precision)");
  const bool fer = (H == 48 && W == 48 && C == 1);
  // per image (floats): the largest block input/output, expanded and depthwise tensors
  size_t big_io = (size_t)112 * 112 * 64, big_e = 0, big_d = 0;
  {
    int h = 112;
    for (const MbBlock& b : blocks) {
      const int oh = b.stride == 2 ? h / 2 : h;
      big_e = std::max(big_e, (size_t)h * h * b.hidp);
      big_d = std::max(big_d, (size_t)oh * oh * b.hidp);
      big_io = std::max(big_io, (size_t)oh * oh * b.coutp);
      h = oh;
    }
  }
  const size_t per_img = 224 * 224 + ((size_t)12544 * MB_STEM_K + 2 * big_io + big_e + big_d + 49 * 1280 + 1280) * 4;
  const size_t need = per_img * (size_t)B + 8192;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  float* A0 = reinterpret_cast<float*>(p); p += (size_t)B * 12544 * MB_STEM_K * 4;
  float* X = reinterpret_cast<float*>(p); p += (size_t)B * big_io * 4;
  float* Y = reinterpret_cast<float*>(p); p += (size_t)B * big_io * 4;
  float* E = reinterpret_cast<float*>(p); p += (size_t)B * big_e * 4;
  float* D = reinterpret_cast<float*>(p); p += (size_t)B * big_d * 4;
  float* Lst = reinterpret_cast<float*>(p); p += (size_t)B * 49 * 1280 * 4;
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
  MEC_TRY(prof.begin(TAG_MBV2_BLOCK, s));
  {
    const size_t total = (size_t)B * 112 * 112 * (MB_STEM_K / 4);
    hipLaunchKernelGGL(mbv2_stem_im2col_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, stem_in,
                       B, Cin, A0);
    MEC_LAUNCH_CHECK();
  }
  GemmParams g;
  g.A = A0; g.B32 = Wt + stem_w_off; g.bias = P + stem_corr_off; g.act = ACT_RELU6; g.C32 = X;
  g.M = B * 112 * 112; g.N = 64; g.K = MB_STEM_K;
  MEC_TRY(launch_gemm_f32(g, s, nullptr, TAG_NONE));
  float* cur = X;
  float* other = Y;
  int h = 112;
  for (const MbBlock& b : blocks) {
    const int oh = b.stride == 2 ? h / 2 : h;
    const float* dw_in = cur;
    if (b.t != 1) {  // expand 1x1 + BN + ReLU6
      g = GemmParams();
      g.A = cur; g.B32 = Wt + b.we_off; g.bias = P + b.be_off; g.act = ACT_RELU6; g.C32 = E;
      g.M = B * h * h; g.N = b.hidp; g.K = b.cinp;
      MEC_TRY(launch_gemm_f32(g, s, nullptr, TAG_NONE));
      dw_in = E;
    }
    {
      const size_t total = (size_t)B * oh * oh * (b.hidp / 4);
      hipLaunchKernelGGL(mbv2_dw_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, dw_in, B, h,
                         b.hidp, b.stride, oh, P + b.wd_off, P + b.bd_off, D);
      MEC_LAUNCH_CHECK();
    }
    g = GemmParams();  // project 1x1 + BN (+ residual)
    g.A = D; g.B32 = Wt + b.wp_off; g.bias = P + b.bp_off; g.C32 = other;
    if (b.stride == 1 && b.cin == b.cout) { g.R = cur; g.r_f32 = 1; }
    g.M = B * oh * oh; g.N = b.coutp; g.K = b.hidp;
    MEC_TRY(launch_gemm_f32(g, s, nullptr, TAG_NONE));
    std::swap(cur, other);
    h = oh;
  }
  MEC_TRY(prof.end(TAG_MBV2_BLOCK, s));
  g = GemmParams();  // features[18] 1x1 320 -> 1280 + BN + ReLU6
  g.A = cur; g.B32 = Wt + last_w_off; g.bias = P + last_b_off; g.act = ACT_RELU6; g.C32 = Lst;
  g.M = B * h * h; g.N = 1280; g.K = 320;
  MEC_TRY(launch_gemm_f32(g, s, &prof, TAG_MBV2_LAST));
  hipLaunchKernelGGL(avgpool_f32_kernel, dim3(B, 1280 / 256), dim3(256), 0, s, Lst, h * h, 1280, pooled);
  MEC_LAUNCH_CHECK();
  MEC_TRY(launch_linear_mfma<BACT_RELU>(pooled, 1280, B, 1280, P + fc1_off, P + fc1b_off, 512, feat, 512, nullptr, 0, s));
  MEC_TRY(launch_head7(feat, B, 512, P + fc2_off, P + fc2b_off, logits, probs, s));
  return 0;
}

}  // namespace mec
