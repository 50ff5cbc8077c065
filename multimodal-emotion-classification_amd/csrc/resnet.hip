// Image path: PIL-exact bilinear resize (u8) -> ResNet50 (NHWC f16, BN folded, MFMA
// implicit-GEMM convs) -> avgpool + 2048->512->7 head (fp32), restating
// inference/image_inference.py:28-32 (transform), :55-65 (network + head), :70-90 (512-d
// fc[2] feature), :117-119 (softmax).
#include <cmath>

#include "block_ops.h"
#include "models.h"

namespace mec {

// ----------------------------------------------------------------------------- resize
// Pillow ImagingResample (bilinear, 8bpc): 22-bit fixed-point taps, horizontal pass into
// a u8 intermediate, then the vertical pass; clip8((acc + 2^21) >> 22).
constexpr int RS_MAXK = 3;  // upscale: support 1 -> ksize = 3
constexpr int RS_PREC = 22;

struct ResizeTaps {
  int xmin[224], xn[224], xk[224][RS_MAXK];
  int ymin[224], yn[224], yk[224][RS_MAXK];
};

static bool make_taps(int in_size, int out_size, int* mins, int* ns, int (*kk)[RS_MAXK]) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  if (ksize > RS_MAXK) return false;  // downscale not needed on this path
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double w[RS_MAXK] = {0, 0, 0}, ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0) t = -t;
      w[x] = t < 1.0 ? 1.0 - t : 0.0;
      ww += w[x];
    }
    for (int x = 0; x < RS_MAXK; ++x) {
      double v = (x < xmax && ww != 0.0) ? w[x] / ww : (x < xmax ? w[x] : 0.0);
      kk[xx][x] = v < 0 ? (int)(-0.5 + v * (1 << RS_PREC)) : (int)(0.5 + v * (1 << RS_PREC));
    }
    mins[xx] = xmin;
    ns[xx] = xmax;
  }
  return true;
}

template <int IH, int IW, int OH, int OW>
__global__ __launch_bounds__(256) void resize_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                        const ResizeTaps* __restrict__ taps) {
  __shared__ uint8_t src[IH * IW];
  __shared__ uint8_t tmp[IH * OW];
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint8_t* im = in + (size_t)b * IH * IW;
  for (int i = tid; i < IH * IW; i += 256) src[i] = im[i];
  __syncthreads();
  for (int i = tid; i < IH * OW; i += 256) {  // horizontal
    const int y = i / OW, xx = i - y * OW;
    int acc = 1 << (RS_PREC - 1);
    const int x0 = taps->xmin[xx];
    for (int x = 0; x < taps->xn[xx]; ++x) acc += (int)src[y * IW + x0 + x] * taps->xk[xx][x];
    acc >>= RS_PREC;
    tmp[i] = (uint8_t)(acc < 0 ? 0 : (acc > 255 ? 255 : acc));
  }
  __syncthreads();
  uint8_t* o = out + (size_t)b * OH * OW;
  for (int i = tid; i < OH * OW; i += 256) {  // vertical
    const int yy = i / OW, x = i - yy * OW;
    int acc = 1 << (RS_PREC - 1);
    const int y0 = taps->ymin[yy];
    for (int y = 0; y < taps->yn[yy]; ++y) acc += (int)tmp[(y0 + y) * OW + x] * taps->yk[yy][y];
    acc >>= RS_PREC;
    o[i] = (uint8_t)(acc < 0 ? 0 : (acc > 255 ? 255 : acc));
  }
}

static ResizeTaps* g_taps = nullptr;  // device copy, built once per process

static int ensure_taps() {
  if (g_taps) return 0;
  ResizeTaps h;
  if (!make_taps(48, 224, h.xmin, h.xn, h.xk) || !make_taps(48, 224, h.ymin, h.yn, h.yk)) {
    set_error("resize taps");
    return -1;
  }
  MEC_HIP(hipMalloc(&g_taps, sizeof(ResizeTaps)));
  MEC_HIP(hipMemcpy(g_taps, &h, sizeof(ResizeTaps), hipMemcpyHostToDevice));
  return 0;
}

int resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, hipStream_t s) {
  MEC_REQUIRE(H == 48 && W == 48 && OH == 224 && OW == 224, "resize: only 48x48 -> 224x224 (FER2013 -> IMAGE_SIZE)");
  if (B == 0) return 0;
  MEC_TRY(ensure_taps());
  hipLaunchKernelGGL((resize_u8_kernel<48, 48, 224, 224>), dim3(B), dim3(256), 0, s, in, out, g_taps);
  MEC_LAUNCH_CHECK();
  return 0;
}

// ----------------------------------------------------------------------------- maxpool
// 3x3 / stride 2 / pad 1 on NHWC f16 (torch max_pool2d pads with -inf).
__global__ __launch_bounds__(256) void maxpool3s2_kernel(const f16* __restrict__ x, f16* __restrict__ y, int B,
                                                         int H, int W, int C, int OH, int OW) {
  const int c8 = C / 8;
  const size_t total = (size_t)B * OH * OW * c8;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % c8);
  size_t r = i / c8;
  const int ow = (int)(r % OW); r /= OW;
  const int oh = (int)(r % OH);
  const int n = (int)(r / OH);
  float m[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
  for (int kh = 0; kh < 3; ++kh) {
    const int ih = oh * 2 - 1 + kh;
    if (ih < 0 || ih >= H) continue;
    for (int kw = 0; kw < 3; ++kw) {
      const int iw = ow * 2 - 1 + kw;
      if (iw < 0 || iw >= W) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(x + (((size_t)n * H + ih) * W + iw) * C + cc * 8);
      const f16* hv = reinterpret_cast<const f16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)hv[e]);
    }
  }
  half8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (f16)m[e];
  *reinterpret_cast<half8*>(y + (((size_t)n * OH + oh) * OW + ow) * C + cc * 8) = o;
}

// ----------------------------------------------------------------------------- avgpool
// AdaptiveAvgPool2d(1) on NHWC f16 -> f32 [B, C]: one thread per (sample, channel).
__global__ __launch_bounds__(256) void avgpool_kernel(const f16* __restrict__ x, int HW, int C, float* __restrict__ y) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const f16* p = x + (size_t)b * HW * C + c;
  float s = 0.f;
  for (int q = 0; q < HW; ++q) s += (float)p[(size_t)q * C];
  y[(size_t)b * C + c] = s / (float)HW;
}

// ----------------------------------------------------------------------------- model
static const int kLayers[4][3] = {{64, 3, 1}, {128, 4, 2}, {256, 6, 2}, {512, 3, 2}};

int ImageModel::create(const float* blob, size_t n) {
  BlobReader rd(blob, n);
  std::vector<f16> w;
  std::vector<float> pr;
  auto bn_fold = [&](int c, std::vector<float>& scale) {  // -> bias offset in pr
    const float* g = rd.take(c);
    const float* b = rd.take(c);
    const float* rm = rd.take(c);
    const float* rv = rd.take(c);
    scale.resize(c);
    size_t off = pr.size();
    for (int i = 0; i < c; ++i) {
      const double s = (double)g[i] / std::sqrt((double)rv[i] + 1e-5);
      scale[i] = (float)s;
      pr.push_back((float)((double)b[i] - (double)rm[i] * s));
    }
    return off;
  };
  auto conv = [&](int cout, int cin, int ks, int stride, int pad) {
    ConvLayer L;
    L.cin = cin; L.cout = cout; L.ks = ks; L.stride = stride; L.pad = pad;
    const float* src = rd.take((size_t)cout * cin * ks * ks);
    std::vector<float> scale;
    L.b_off = bn_fold(cout, scale);
    L.w_off = w.size();
    w.resize(w.size() + (size_t)cout * cin * ks * ks);
    if (!rd.ok) return L;
    for (int o = 0; o < cout; ++o)
      for (int kh = 0; kh < ks; ++kh)
        for (int kw = 0; kw < ks; ++kw)
          for (int c = 0; c < cin; ++c)
            w[L.w_off + (((size_t)o * ks + kh) * ks + kw) * cin + c] =
                (f16)((double)src[(((size_t)o * cin + c) * ks + kh) * ks + kw] * scale[o]);
    return L;
  };
  // stem: fold ToTensor(/255) + Normalize + BN scale into the K rows (see gemm.hip A_STEM):
  // gray input folds the three replicated channels into one (K=128); RGB keeps them (K=256).
  {
    const float* src = rd.take((size_t)64 * 3 * 49);
    std::vector<float> scale;
    stem.b_off = bn_fold(64, scale);
    stem.cin = 1; stem.cout = 64; stem.ks = 7; stem.stride = 2; stem.pad = 3;
    stem_rgb = stem;
    stem_rgb.cin = 3;
    stem.w_off = w.size();
    w.resize(w.size() + 64 * 128, (f16)0.f);
    stem_rgb.w_off = w.size();
    w.resize(w.size() + 64 * 256, (f16)0.f);
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
    if (rd.ok) {
      for (int o = 0; o < 64; ++o)
        for (int t = 0; t < 49; ++t) {
          double a = 0.0, c0 = 0.0;
          for (int c = 0; c < 3; ++c) {
            const double wv = src[((size_t)o * 3 + c) * 49 + t];
            const double mf = (double)(float)mean[c], sf = (double)(float)stdv[c];
            a += wv / (255.0 * sf);
            c0 -= wv * mf / sf;
            w[stem_rgb.w_off + (size_t)o * 256 + 64 * c + t] = (f16)(wv / (255.0 * sf) * scale[o]);
          }
          w[stem.w_off + (size_t)o * 128 + t] = (f16)(a * scale[o]);
          w[stem.w_off + (size_t)o * 128 + 64 + t] = (f16)(c0 * scale[o]);
          w[stem_rgb.w_off + (size_t)o * 256 + 192 + t] = (f16)(c0 * scale[o]);
        }
    }
  }
  blocks.clear();
  int cin = 64;
  for (int li = 0; li < 4; ++li) {
    const int wd = kLayers[li][0], nb = kLayers[li][1], st = kLayers[li][2];
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
  MEC_TRY(upload(wts, w.data(), w.size() * sizeof(f16)));
  MEC_TRY(upload(prm, pr.data(), pr.size() * sizeof(float)));
  return ensure_taps();
}

int ImageModel::forward(const uint8_t* gray, int B, float* feat, float* logits, float* probs, hipStream_t s) {
  return forward_u8(gray, B, 48, 48, 1, feat, logits, probs, s);
}

int ImageModel::forward_u8(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                           hipStream_t s) {
  MEC_REQUIRE(B >= 0, "image: B < 0");
  if (B == 0) return 0;
  MEC_REQUIRE(img && feat && logits && probs, "image: null pointer");
  const bool fer = (H == 48 && W == 48 && C == 1);
  MEC_REQUIRE(fer || (H == 224 && W == 224 && (C == 1 || C == 3)),
              "image: input must be u8 [B,48,48,1] (GPU resize) or [B,224,224,{1,3}] (already resized)");
  const size_t per_img_big = (size_t)56 * 56 * 256;  // largest NHWC activation (elements)
  const size_t per_t1 = (size_t)56 * 56 * 128, per_t2 = (size_t)56 * 56 * 64;
  const size_t per_img = 224 * 224 + (3 * per_img_big + per_t1 + per_t2) * sizeof(f16) + 256 + 2048 * sizeof(float);
  if (B > ws_batch) {
    MEC_TRY(ws.ensure(per_img * (size_t)B + 4096));
    ws_batch = B;
  }
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  f16* X = reinterpret_cast<f16*>(p); p += (size_t)B * per_img_big * sizeof(f16);
  f16* Y = reinterpret_cast<f16*>(p); p += (size_t)B * per_img_big * sizeof(f16);
  f16* DS = reinterpret_cast<f16*>(p); p += (size_t)B * per_img_big * sizeof(f16);
  f16* T1 = reinterpret_cast<f16*>(p); p += (size_t)B * per_t1 * sizeof(f16);
  f16* T2 = reinterpret_cast<f16*>(p);
  p += (size_t)B * per_t2 * sizeof(f16);
  float* pooled = reinterpret_cast<float*>(p);  // [B,2048]

  const f16* Wt = wts.as<f16>();
  const float* P = prm.as<float>();
  const uint8_t* stem_in = img;
  if (fer) {
    MEC_TRY(resize_u8(img, B, 48, 48, resized, 224, 224, s));
    stem_in = resized;
  }
  {  // stem conv 7x7/2 + BN + ReLU -> Y [B,112,112,64]
    const ConvLayer& st = C == 3 ? stem_rgb : stem;
    GemmParams g;
    g.amode = A_STEM; g.A = stem_in; g.B = Wt + st.w_off; g.bias = P + st.b_off; g.act = ACT_RELU;
    g.C16 = Y; g.M = B * 112 * 112; g.N = 64; g.K = 64 * (C + 1);
    g.H = 224; g.W = 224; g.C = C; g.OH = 112; g.OW = 112; g.ks = 7; g.stride = 2; g.pad = 3;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_STEM));
  }
  {  // maxpool -> X [B,56,56,64]
    const size_t total = (size_t)B * 56 * 56 * 8;
    hipLaunchKernelGGL(maxpool3s2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, Y, X, B, 112, 112,
                       64, 56, 56);
    MEC_LAUNCH_CHECK();
  }
  f16* cur = X;
  f16* other = Y;
  H = 56;
  for (const Bottleneck& bk : blocks) {
    const int wd = bk.c1.cout, cin = bk.c1.cin, st = bk.c2.stride;
    const int OH = (H + 2 - 3) / st + 1;
    GemmParams g;
    g.A = cur; g.B = Wt + bk.c1.w_off; g.bias = P + bk.c1.b_off; g.act = ACT_RELU; g.C16 = T1;
    g.M = B * H * H; g.N = wd; g.K = cin;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
    g = GemmParams();
    g.amode = A_CONV; g.A = T1; g.B = Wt + bk.c2.w_off; g.bias = P + bk.c2.b_off; g.act = ACT_RELU; g.C16 = T2;
    g.M = B * OH * OH; g.N = wd; g.K = 9 * wd;
    g.H = H; g.W = H; g.C = wd; g.OH = OH; g.OW = OH; g.ks = 3; g.stride = st; g.pad = 1;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV3X3));
    const f16* res = cur;
    if (bk.has_ds) {
      g = GemmParams();
      g.B = Wt + bk.ds.w_off; g.bias = P + bk.ds.b_off; g.C16 = DS; g.A = cur;
      g.M = B * OH * OH; g.N = 4 * wd; g.K = cin;
      if (st != 1) {
        g.amode = A_CONV; g.H = H; g.W = H; g.C = cin; g.OH = OH; g.OW = OH; g.ks = 1; g.stride = st; g.pad = 0;
      }
      MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
      res = DS;
    }
    g = GemmParams();
    g.A = T2; g.B = Wt + bk.c3.w_off; g.bias = P + bk.c3.b_off; g.R = res; g.act = ACT_RELU; g.C16 = other;
    g.M = B * OH * OH; g.N = 4 * wd; g.K = wd;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
    std::swap(cur, other);
    H = OH;
  }
  hipLaunchKernelGGL(avgpool_kernel, dim3(B, 2048 / 256), dim3(256), 0, s, cur, H * H, 2048, pooled);
  MEC_LAUNCH_CHECK();
  // fc[1] Linear(2048,512) + fc[2] ReLU -> the 512-d feature (extract_features)
  hipLaunchKernelGGL((linear_rows_kernel<8, 2048>), dim3((B + 7) / 8, 512 / 64), dim3(256), 0, s, pooled, (size_t)2048,
                     B, 2048, P + fc1_off, P + fc1b_off, 512, 64, feat, 512, (int)BACT_RELU, (float*)nullptr, 0);
  MEC_LAUNCH_CHECK();
  hipLaunchKernelGGL((head_softmax_kernel<8, 768>), dim3((B + 7) / 8), dim3(256), 0, s, feat, B, 512, P + fc2_off,
                     P + fc2b_off, logits, probs);
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
