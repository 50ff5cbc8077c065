// Image path: PIL-exact bilinear resize (u8) -> ResNet50 (NHWC f16, BN folded, MFMA
// implicit-GEMM convs) -> avgpool + 2048->512->7 head (fp32), restating
// inference/image_inference.py:28-32 (transform), :55-65 (network + head), :70-90 (512-d
// fc[2] feature), :117-119 (softmax).
#include <algorithm>
#include <cmath>

#include "block_ops.h"
#include "models.h"

namespace mec {

// Images per layer1-2 pass (0 = whole batch). Measured at B = 256 (tools/encoder_profile.py
// --opt resnet_chunk=N): 0 -> 4.23-4.25 ms, 128 -> 4.38, 64 -> 4.44-4.49, 32 -> 5.08: the
// smaller GEMMs lose more than the cache residency gains, so chunking is off.
// layer1 seam kernels (pw_chain.hip): 0 off, 1 the 256 -> 64 seams (block 1 -> 2, 2 -> 3),
// 2 also the 256 -> 128 seam into layer2 (block 3 -> layer2 block 1). Image encoder at
// B = 256 (tools/ab_option.py, one process): 4.03 / 3.83 / 3.75 ms for 0 / 1 / 2.

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

// Packed taps: per output coordinate (first source index, k0, k1, k2); taps past the
// filter support are 0, so every output sums exactly three terms (same value as Pillow).
struct ResizeTaps4 {
  int4 x[224], y[224];
};

// grid (B, 224 / RS_BAND): one band of RS_BAND output rows per workgroup. The band's few
// source rows are resampled horizontally into LDS (u8, like Pillow's intermediate), then
// each thread produces 4 adjacent output pixels of the vertical pass (one u32 store).
constexpr int RS_BAND = 28;
__global__ __launch_bounds__(256) void resize_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                        const ResizeTaps4* __restrict__ taps) {
  constexpr int IH = 48, IW = 48, OW = 224, MAXR = 12;
  __shared__ __attribute__((aligned(16))) uint8_t src[IH * IW];
  __shared__ __attribute__((aligned(16))) uint8_t tmp[MAXR * OW];
  const int b = blockIdx.x, r0 = blockIdx.y * RS_BAND, tid = threadIdx.x;
  const uint8_t* im = in + (size_t)b * IH * IW;
  if (tid < IH * IW / 16) reinterpret_cast<uint4*>(src)[tid] = reinterpret_cast<const uint4*>(im)[tid];
  const int ys = taps->y[r0].x;                                  // first source row of the band
  const int ye = min(taps->y[r0 + RS_BAND - 1].x + 3, IH);        // one past the last
  __syncthreads();
  for (int i = tid; i < (ye - ys) * OW; i += 256) {  // horizontal
    const int yr = i / OW, xx = i - yr * OW;
    const int4 t = taps->x[xx];
    const uint8_t* row = src + (ys + yr) * IW;
    int acc = (1 << (RS_PREC - 1)) + (int)row[t.x] * t.y + (int)row[min(t.x + 1, IW - 1)] * t.z +
              (int)row[min(t.x + 2, IW - 1)] * t.w;
    acc >>= RS_PREC;
    tmp[i] = (uint8_t)(acc < 0 ? 0 : (acc > 255 ? 255 : acc));
  }
  __syncthreads();
  uint8_t* o = out + (size_t)b * OW * OW;
  for (int i = tid; i < RS_BAND * OW / 4; i += 256) {  // vertical, 4 pixels per thread
    const int yl = i / (OW / 4), x4 = (i - yl * (OW / 4)) * 4;
    const int yy = r0 + yl;
    const int4 t = taps->y[yy];
    const int y0 = t.x - ys;
    const int y1 = min(t.x + 1, IH - 1) - ys, y2 = min(t.x + 2, IH - 1) - ys;
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = x4 + j;
      int acc = (1 << (RS_PREC - 1)) + (int)tmp[y0 * OW + x] * t.y + (int)tmp[min(y1, MAXR - 1) * OW + x] * t.z +
                (int)tmp[min(y2, MAXR - 1) * OW + x] * t.w;
      // all taps and pixels are >= 0 (upscale), so only the 255 clamp can apply. Writing
      // the [0,255] clamp here lets the compiler (ROCm 7.2) pair two bytes into
      // v_ashr_pk_u8_i32, whose upper 16 result bits leak into the packed word.
      packed |= (uint32_t)min(acc >> RS_PREC, 255) << (8 * j);
    }
    *reinterpret_cast<uint32_t*>(o + (size_t)yy * OW + x4) = packed;
  }
}

static ResizeTaps4* g_taps = nullptr;  // device copy, built once per process

static int ensure_taps() {
  if (g_taps) return 0;
  ResizeTaps h;
  if (!make_taps(48, 224, h.xmin, h.xn, h.xk) || !make_taps(48, 224, h.ymin, h.yn, h.yk)) {
    set_error("resize taps");
    return -1;
  }
  ResizeTaps4 p;
  for (int i = 0; i < 224; ++i) {
    int kx[3] = {0, 0, 0}, ky[3] = {0, 0, 0};
    for (int j = 0; j < h.xn[i]; ++j) kx[j] = h.xk[i][j];
    for (int j = 0; j < h.yn[i]; ++j) ky[j] = h.yk[i][j];
    p.x[i] = make_int4(h.xmin[i], kx[0], kx[1], kx[2]);
    p.y[i] = make_int4(h.ymin[i], ky[0], ky[1], ky[2]);
  }
  // the band's source rows fit the kernel's LDS buffer
  for (int r0 = 0; r0 < 224; r0 += RS_BAND)
    if (std::min(p.y[r0 + RS_BAND - 1].x + 3, 48) - p.y[r0].x > 12) { set_error("resize: band too tall"); return -1; }
  MEC_HIP(hipMalloc(&g_taps, sizeof(ResizeTaps4)));
  MEC_HIP(hipMemcpy(g_taps, &p, sizeof(ResizeTaps4), hipMemcpyHostToDevice));
  return 0;
}

int resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, hipStream_t s) {
  MEC_REQUIRE(H == 48 && W == 48 && OH == 224 && OW == 224, "resize: only 48x48 -> 224x224 (FER2013 -> IMAGE_SIZE)");
  if (B == 0) return 0;
  MEC_TRY(ensure_taps());
  hipLaunchKernelGGL(resize_u8_kernel, dim3(B, 224 / RS_BAND), dim3(256), 0, s, in, out, g_taps);
  MEC_LAUNCH_CHECK();
  return 0;
}

// ----------------------------------------------------------------------------- stem + maxpool
// Fused conv7x7/2 + BN + ReLU (MFMA) + maxpool3x3/2 on the u8 224x224 image.
// One workgroup = an 8x8 tile of pooled outputs = a 17x17 region of stem outputs (with the
// pool's halo), from a 40x46 input patch. K is ordered (channel, kh, kw) with kw padded to
// 8 (and kh to 8): one 16-deep MFMA k step covers two kernel rows, one per lane half, so a
// lane's A fragment for stem pixel (y, x) and kernel row kh is the 8 consecutive patch
// pixels [2y+kh][2x .. 2x+7] (the 8th meets a zero weight). The patch is kept as four f16
// copies shifted by 0/2/4/6 pixels, so that slice always starts 16-B aligned in copy x&3:
// every A fragment is ONE ds_read_b128 straight from the patch (no im2col tile).
// ToTensor/Normalize is folded into the weights; the -mean/std term summed over the
// in-image taps depends only on the border class of the stem pixel (rows/cols 0, 1, 111
// have out-of-image taps), so it is a [16 classes][64] table added in the epilogue.
// Stem pixels outside the 112x112 image become 0: outputs are post-ReLU (>= 0) and every
// pool window holds a valid pixel, so this equals torch's -inf padding. Pooling f16 values
// is exact (max commutes with monotone rounding).
constexpr int SP_T = 8;              // pooled tile
constexpr int SP_S = 2 * SP_T + 1;   // 17 stem rows/cols
constexpr int SP_M = 320;            // 289 padded to 10 x 32
constexpr int SP_R = 40;             // patch rows: 2*16 + 8 (kh padded to 8)
constexpr int SP_W = 46;             // patch cols loaded: 2*16 + 8 + 6 (largest copy shift)
constexpr int SP_CW = 40;            // cols per shifted copy
constexpr int SP_COPY = SP_R * SP_CW + 32;  // halfs per copy, padded: copies land 12 bank slots apart
constexpr int SO_LD = 72;            // stem-output row (f16), padded: 144 B

__device__ __forceinline__ int sp_swz(int row, int kc) { return kc ^ ((row >> 1) & 7); }

// border class of a stem coordinate: 0 -> 0, 1 -> 1, 111 -> 3, else 2 (interior)
__device__ __forceinline__ int sp_cls(int o) { return o == 0 ? 0 : (o == 1 ? 1 : (o == 111 ? 3 : 2)); }

template <int C, int DBG = 0>
__global__ __launch_bounds__(256, 2) void stem_pool_kernel(const uint8_t* __restrict__ img, int ntiles,
                                                        const f16* __restrict__ Wst, const float* __restrict__ bias,
                                                        const float* __restrict__ corr, f16* __restrict__ out) {
  // Persistent: each workgroup walks tiles blockIdx.x, +gridDim.x, ...; the weights, bias
  // and border table are loaded once, and the next tile's patch bytes are fetched into
  // registers while the current tile computes.
  constexpr int PATCH = C * 4 * SP_COPY;
  constexpr int SOH = SP_S * SP_S * SO_LD;  // live stem-output rows only
  constexpr int SMEM = PATCH + C * 64 * 64 + SOH;
  // patch copies | weights (written once) | stem outputs: separate regions, so the weights
  // stay resident and the epilogue needs no barrier behind the MFMA reads of the patch
  __shared__ __attribute__((aligned(16))) f16 smem[SMEM];
  __shared__ float sCorr[16 * 64];  // border-class correction minus the interior one
  __shared__ float sBias[64];       // bias + interior correction
  f16* sP = smem;
  f16* sB = smem + PATCH;
  f16* const sOut = smem + PATCH + C * 64 * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint4 wreg[C][2];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + 256 * j, n = i >> 3, kc = i & 7;
      wreg[c][j] = *reinterpret_cast<const uint4*>(Wst + (size_t)n * 64 * C + c * 64 + kc * 8);
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = tid + 256 * j;
    sCorr[i] = corr[i] - corr[(2 * 4 + 2) * 64 + (i & 63)];
  }
  if (tid < 64) sBias[tid] = bias[tid] + corr[(2 * 4 + 2) * 64 + tid];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + 256 * j, n = i >> 3, kc = i & 7;
      *reinterpret_cast<uint4*>(sB + c * 4096 + n * 64 + sp_swz(n, kc) * 8) = wreg[c][j];
    }

  // patch loader: thread -> a fixed pixel pair (cols 2k, 2k+1) walking rows r0, r0+11, ...;
  // each shifted copy then gets one whole dword per pair (shifts are even)
  constexpr int PAIRS = SP_W / 2;                   // 23 pairs per patch row
  constexpr int RSTEP = 256 / PAIRS;                // 11 rows per sweep
  constexpr int ITER = (SP_R + RSTEP - 1) / RSTEP;  // 4
  const int k = tid % PAIRS, r0 = tid / PAIRS;      // tid < 253 active
  const bool act = tid < PAIRS * RSTEP;
  uint32_t px[C][ITER][2];
  auto load_patch = [&](int tile) {
    const int b = tile / 49, t = tile - (tile / 49) * 49;
    const int ph0 = (t / 7) * SP_T, pw0 = (t - (t / 7) * 7) * SP_T;
    const int ir0 = 2 * (2 * ph0 - 1) - 3, ic0 = 2 * (2 * pw0 - 1) - 3;
    const uint8_t* im = img + (size_t)b * 224 * 224 * C;
    const int x0 = ic0 + 2 * k;
    const bool okx0 = x0 >= 0 && x0 < 224, okx1 = x0 + 1 >= 0 && x0 + 1 < 224;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int j = 0; j < ITER; ++j) {
        const int pr = r0 + RSTEP * j, y = ir0 + pr;
        const bool oky = act && pr < SP_R && y >= 0 && y < 224;
        const uint8_t* row = im + ((size_t)(oky ? y : 0) * 224) * C + c;
        px[c][j][0] = (oky && okx0) ? row[(size_t)x0 * C] : 0u;
        px[c][j][1] = (oky && okx1) ? row[(size_t)(x0 + 1) * C] : 0u;
      }
  };
  const int lr = lane & 31, lh = lane >> 5;
  const int jt = wave & 1;          // N tile (32 of the 64 channels)
  const int it0 = wave >> 1;        // row tiles it0, it0+2, ..., it0+8
  int aoff[5];                      // per row tile: this lane's stem pixel -> patch offset
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int m = min(32 * (it0 + 2 * q) + lr, SP_S * SP_S - 1);  // pad rows read a valid pixel
    const int y = m / SP_S, x = m - (m / SP_S) * SP_S;
    aoff[q] = (x & 3) * SP_COPY + (2 * y + lh) * SP_CW + 8 * (x >> 2);
  }
  int tile = blockIdx.x;
  if (tile < ntiles) load_patch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int b = tile / 49, t = tile - (tile / 49) * 49;
    const int ph0 = (t / 7) * SP_T, pw0 = (t - (t / 7) * 7) * SP_T;
    const int sr0 = 2 * ph0 - 1, sc0 = 2 * pw0 - 1;  // first stem row/col of the region
    __syncthreads();  // previous tile's pool reads done (first tile: tables written)
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int j = 0; j < ITER; ++j) {
        const int pr = r0 + RSTEP * j;
        const bool rok = act && pr < SP_R;
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 v = {(f16)(float)px[c][j][0], (f16)(float)px[c][j][1]};
#pragma unroll
        for (int sh = 0; sh < 4; ++sh) {  // copy sh holds patch[pr][jj + 2 sh]
          // branch-free: writes that fall outside the copy go to its 32-half pad tail
          const int jj = 2 * k - 2 * sh;
          const bool ok = rok && jj >= 0 && jj < SP_CW;
          const int off = ok ? pr * SP_CW + jj : SP_R * SP_CW + 2 * (k & 15);
          *reinterpret_cast<h2*>(sP + (c * 4 + sh) * SP_COPY + off) = v;
        }
      }
    if (!(DBG & 4) && tile + (int)gridDim.x < ntiles) load_patch(tile + gridDim.x);  // in flight under this tile
    __syncthreads();  // patch copies + weights ready
    floatx16 acc[5];
#pragma unroll
    for (int q = 0; q < 5; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;
#pragma unroll
    for (int ch = 0; ch < (DBG & 1 ? 0 : C); ++ch) {
      const f16* pc = sP + ch * 4 * SP_COPY;
#pragma unroll
      for (int s = 0; s < 4; ++s) {  // k step s: kernel rows 2s (lanes 0-31) and 2s+1 (32-63)
        const int kcs = 2 * s + lh;
        const int rb = 32 * jt + lr;
        const half8 bf = *reinterpret_cast<const half8*>(sB + ch * 4096 + rb * 64 + sp_swz(rb, kcs) * 8);
#pragma unroll
        for (int q = 0; q < 5; ++q) {
          const half8 af = *reinterpret_cast<const half8*>(pc + aoff[q] + 2 * s * SP_CW);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bf, af, acc[q], 0, 0, 0);  // D[channel][pixel]
        }
      }
    }
    {  // conv + bias (+ the border class's correction) -> sO [m][SO_LD] f16, pre-ReLU; stem
       // pixels outside the 112x112 image -> 0 (every pool window holds an in-image pixel and
       // the pooled values are post-ReLU >= 0, so this equals torch's -inf pool padding). The
       // accumulators are transposed (lane = stem pixel, 4 consecutive channels per register
       // quad): 8-B writes.
      f16* sO = sOut;
      const bool border = ph0 == 0 || pw0 == 0 || ph0 + SP_T == 56 || pw0 + SP_T == 56;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int m = 32 * (it0 + 2 * q) + lr;
        if (m < SP_S * SP_S) {
          const int y = m / SP_S, x = m - (m / SP_S) * SP_S;
          const int oh = sr0 + y, ow = sc0 + x;
          const bool ok = oh >= 0 && oh < 112 && ow >= 0 && ow < 112;
          const int cls = sp_cls(oh) * 4 + sp_cls(ow);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int ch = 32 * jt + 8 * g + 4 * lh;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[q][4 * g + e] + sBias[ch + e];
            if (border) {  // sCorr holds each class's correction minus the interior one
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = ok ? v[e] + sCorr[cls * 64 + ch + e] : 0.f;
            }
            const half4 h = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
            *reinterpret_cast<half4*>(sO + m * SO_LD + ch) = h;
          }
        }
      }
    }
    __syncthreads();
  {  // ReLU + 3x3/2 max on packed f16 (max commutes with the monotone f16 rounding).
     // Thread -> 16-B channel chunk c of pooled pixel (px, py), py = wave + 4 pass; the lane
     // bits are dealt to (c, px) so that every ds_read_b128 lane group hits 16 distinct bank
     // slots on the 144-B stem-output rows (3x fewer LDS cycles than 16 channels per thread).
    const f16* sO = sOut;
    const int c = ((lane >> 2) & 1) | (((lane >> 3) & 1) << 1) | ((lane & 1) << 2);
    const int pxx = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 1) & 1) << 2);
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int py = wave + 4 * pass;
      half8 m0 = {0, 0, 0, 0, 0, 0, 0, 0};  // post-ReLU values are >= 0
#pragma unroll
      for (int dy = 0; dy < (DBG & 2 ? 0 : 3); ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int mm = (2 * py + dy) * SP_S + 2 * pxx + dx;
          m0 = __builtin_elementwise_max(m0, *reinterpret_cast<const half8*>(sO + mm * SO_LD + 8 * c));
        }
      *reinterpret_cast<half8*>(out + (((size_t)b * 56 + ph0 + py) * 56 + pw0 + pxx) * 64 + 8 * c) = m0;
    }
  }
  }
}

// ----------------------------------------------------------------------------- avgpool
// AdaptiveAvgPool2d(1) on NHWC f16 -> f32 [B, C]: one thread per (sample, channel).

// ----------------------------------------------------------------------------- model
static const int kLayers[4][3] = {{64, 3, 1}, {128, 4, 2}, {256, 6, 2}, {512, 3, 2}};

int ImageModel::create(const float* blob, size_t n) {
  if (prec == PREC_FP32 || prec == PREC_FP32X3) {  // resnet_f32.hip
    MEC_TRY(create_f32(blob, n));
    return ensure_taps();
  }
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
  // stem (stem_pool_kernel): ToTensor(/255) + Normalize + BN scale folded into per-channel
  // pixel weights (gray: the three replicated channels summed into one); the -mean/std
  // term summed over in-image taps goes to a [16 border classes][64] table.
  {
    const float* src = rd.take((size_t)64 * 3 * 49);
    std::vector<float> scale;
    stem.b_off = bn_fold(64, scale);
    stem.cin = 1; stem.cout = 64; stem.ks = 7; stem.stride = 2; stem.pad = 3;
    stem_rgb = stem;
    stem_rgb.cin = 3;
    stem.w_off = w.size();
    w.resize(w.size() + 64 * 64, (f16)0.f);
    stem_rgb.w_off = w.size();
    w.resize(w.size() + 64 * 192, (f16)0.f);
    stem_corr_off = pr.size();
    pr.resize(pr.size() + 16 * 64, 0.f);
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
    if (rd.ok) {
      std::vector<double> c0(64 * 49);
      for (int o = 0; o < 64; ++o)
        for (int t = 0; t < 49; ++t) {
          double a = 0.0, cc = 0.0;
          for (int c = 0; c < 3; ++c) {
            const double wv = src[((size_t)o * 3 + c) * 49 + t];
            const double mf = (double)(float)mean[c], sf = (double)(float)stdv[c];
            a += wv / (255.0 * sf);
            cc -= wv * mf / sf;
            w[stem_rgb.w_off + (size_t)o * 192 + 64 * c + (t / 7) * 8 + t % 7] = (f16)(wv / (255.0 * sf) * scale[o]);
          }
          w[stem.w_off + (size_t)o * 64 + (t / 7) * 8 + t % 7] = (f16)(a * scale[o]);  // k = kh*8 + kw
          c0[o * 49 + t] = cc * scale[o];
        }
      // border classes of a stem coordinate: 0, 1, interior, 111 (see sp_cls)
      const int rep[4] = {0, 1, 50, 111};
      for (int rc = 0; rc < 4; ++rc)
        for (int cc = 0; cc < 4; ++cc)
          for (int o = 0; o < 64; ++o) {
            double sum = 0.0;
            for (int kh = 0; kh < 7; ++kh)
              for (int kw = 0; kw < 7; ++kw) {
                const int ih = 2 * rep[rc] - 3 + kh, iw = 2 * rep[cc] - 3 + kw;
                if (ih >= 0 && ih < 224 && iw >= 0 && iw < 224) sum += c0[o * 49 + kh * 7 + kw];
              }
            pr[stem_corr_off + (rc * 4 + cc) * 64 + o] = (float)sum;
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
        // conv3 and the downsample projection as one GEMM over K = [w | cin] (A_DUAL):
        // bn3(conv3(t)) + bn_ds(conv_ds(x)) = [t | x] . [W3' | Wds']^T + (b3 + bds)
        bk.c3ds_w_off = w.size();
        const int K3 = wd, K2 = cin, Kt = wd + cin;
        w.resize(w.size() + (size_t)4 * wd * Kt);
        for (int o = 0; o < 4 * wd; ++o) {
          for (int k = 0; k < K3; ++k) w[bk.c3ds_w_off + (size_t)o * Kt + k] = w[bk.c3.w_off + (size_t)o * K3 + k];
          for (int k = 0; k < K2; ++k) w[bk.c3ds_w_off + (size_t)o * Kt + K3 + k] = w[bk.ds.w_off + (size_t)o * K2 + k];
        }
        bk.c3ds_b_off = pr.size();
        for (int o = 0; o < 4 * wd; ++o) pr.push_back(pr[bk.c3.b_off + o] + pr[bk.ds.b_off + o]);
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

int ImageModel::forward_u8(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits, float* probs,
                           hipStream_t s) {
  MEC_REQUIRE(B >= 0, "image: B < 0");
  if (B == 0) return 0;
  MEC_REQUIRE(img && feat && logits && probs, "image: null pointer");
  const bool fer = (H == 48 && W == 48 && C == 1);
  MEC_REQUIRE(fer || (H == 224 && W == 224 && (C == 1 || C == 3)),
              "image: input must be u8 [B,48,48,1] (GPU resize) or [B,224,224,{1,3}] (already resized)");
  if (prec == PREC_FP32) return forward_f32(img, B, H, W, C, feat, logits, probs, s);
  if (prec == PREC_FP32X3) return forward_x3(img, B, H, W, C, feat, logits, probs, s);
  const size_t per_img_big = (size_t)56 * 56 * 256;  // largest NHWC activation (elements)
  const size_t per_t1 = (size_t)56 * 56 * 128, per_t2 = (size_t)56 * 56 * 64;
  const size_t per_img = 224 * 224 + (2 * per_img_big + per_t1 + per_t2) * sizeof(f16) + 256 + 2048 * sizeof(float);
  if (B > ws_batch) {
    MEC_TRY(ws.ensure(per_img * (size_t)B + 4096));
    ws_batch = B;
  }
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  f16* X = reinterpret_cast<f16*>(p); p += (size_t)B * per_img_big * sizeof(f16);
  f16* Y = reinterpret_cast<f16*>(p); p += (size_t)B * per_img_big * sizeof(f16);
  // the stem output [B,56,56,64] sits in the last quarter of X: a chunk's layer-1 outputs (4x the
  // per-image stride) then never reach the stem output of a later chunk's images (resnet_chunk)
  f16* Xs = X + (size_t)3 * B * 56 * 56 * 64;
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
  {  // fused stem conv 7x7/2 + BN + ReLU + maxpool 3x3/2 -> X [B,56,56,64]
    const ConvLayer& st = C == 3 ? stem_rgb : stem;
    MEC_TRY(prof.begin(TAG_RESNET_STEM, s));
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      MEC_HIP(hipGetDevice(&dev));
      MEC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int ntiles = B * 49;  // two resident workgroups per CU (VGPR-bound)
    const dim3 sg(std::min(ntiles, 2 * ncu)), sb(256);
    const f16* sw = Wt + st.w_off;
    const float *sbias = P + st.b_off, *scorr = P + stem_corr_off;
    if (C == 3)
      hipLaunchKernelGGL(stem_pool_kernel<3>, sg, sb, 0, s, stem_in, ntiles, sw, sbias, scorr, Xs);
#ifdef MEC_PROBES
    else if (opt().stem_debug == 1)  // probe builds (wrong results): no MFMA / no pool / no prefetch
      hipLaunchKernelGGL((stem_pool_kernel<1, 1>), sg, sb, 0, s, stem_in, ntiles, sw, sbias, scorr, Xs);
    else if (opt().stem_debug == 2)
      hipLaunchKernelGGL((stem_pool_kernel<1, 2>), sg, sb, 0, s, stem_in, ntiles, sw, sbias, scorr, Xs);
    else if (opt().stem_debug == 4)
      hipLaunchKernelGGL((stem_pool_kernel<1, 4>), sg, sb, 0, s, stem_in, ntiles, sw, sbias, scorr, Xs);
    else if (opt().stem_debug == 7)
      hipLaunchKernelGGL((stem_pool_kernel<1, 7>), sg, sb, 0, s, stem_in, ntiles, sw, sbias, scorr, Xs);
#endif
    else
      hipLaunchKernelGGL(stem_pool_kernel<1>, sg, sb, 0, s, stem_in, ntiles, sw, sbias, scorr, Xs);
    MEC_LAUNCH_CHECK();
    MEC_TRY(prof.end(TAG_RESNET_STEM, s));
  }
  // Bottleneck blocks [b0, b1) over images [i0, i0 + nb) of the batch (NHWC buffers are
  // image-major, so an image range is a pointer offset). cur/other swap once per block.
  auto run_blocks = [&](size_t b0, size_t b1, int i0, int nb, int Hin, f16*& cur, f16*& other) -> int {
    int H = Hin;
    bool conv1_done = false;  // this block's conv1 already ran in the previous block's seam kernel
    for (size_t bi = b0; bi < b1; ++bi) {
      const Bottleneck& bk = blocks[bi];
      const int wd = bk.c1.cout, cin = bk.c1.cin, st = bk.c2.stride;
      const int OH = (H + 2 - 3) / st + 1;
      f16* in = (bi == 0 ? Xs : cur) + (size_t)i0 * H * H * cin;
      f16* out = other + (size_t)i0 * OH * OH * 4 * wd;
      f16* t1 = T1 + (size_t)i0 * H * H * wd;
      f16* t2 = T2 + (size_t)i0 * OH * OH * wd;
      GemmParams g;
      if (!conv1_done) {
        g.A = in; g.B = Wt + bk.c1.w_off; g.bias = P + bk.c1.b_off; g.act = ACT_RELU; g.C16 = t1;
        g.M = nb * H * H; g.N = wd; g.K = cin;
        MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
      }
      conv1_done = false;
      g = GemmParams();
      g.amode = A_CONV; g.A = t1; g.B = Wt + bk.c2.w_off; g.bias = P + bk.c2.b_off; g.act = ACT_RELU; g.C16 = t2;
      g.M = nb * OH * OH; g.N = wd; g.K = 9 * wd;
      g.H = H; g.W = H; g.C = wd; g.OH = OH; g.OW = OH; g.ks = 3; g.stride = st; g.pad = 1;
      MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV3X3));
      if (bk.has_ds && opt().pw_chain && wd == 64 && st == 1 && cin == 64 && OH == 56 && bi + 1 < b1 &&
          blocks[bi + 1].c1.cin == 256 && blocks[bi + 1].c1.cout == 64) {
        // layer1 block 1: conv3 + downsample + ReLU, then block 2's conv1 (pw_chain.hip)
        const Bottleneck& nx = blocks[bi + 1];
        MEC_TRY(prof.begin(TAG_RESNET_CONV1X1, s));
        MEC_TRY(launch_pw_chain_dual(t2, in, Wt + bk.c3ds_w_off, P + bk.c3ds_b_off, Wt + nx.c1.w_off,
                                     P + nx.c1.b_off, out, T1 + (size_t)i0 * OH * OH * 64, nb * OH * OH, s));
        MEC_TRY(prof.end(TAG_RESNET_CONV1X1, s));
        conv1_done = true;
      } else if (bk.has_ds) {  // conv3 + downsample + add + ReLU in one dual-source GEMM
        g = GemmParams();
        g.amode = A_DUAL; g.A = t2; g.K1 = wd; g.A2 = in; g.B = Wt + bk.c3ds_w_off; g.bias = P + bk.c3ds_b_off;
        g.act = ACT_RELU; g.C16 = out; g.M = nb * OH * OH; g.N = 4 * wd; g.K = wd + cin;
        g.H = H; g.W = H; g.C = cin; g.OH = OH; g.OW = OH; g.ks = 1; g.stride = st; g.pad = 0;
        MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
      } else if (opt().pw_chain && wd == 64 && OH == 56 && bi + 1 < b1 && blocks[bi + 1].c1.cin == 256 &&
                 (blocks[bi + 1].c1.cout == 64 || (opt().pw_chain == 2 && blocks[bi + 1].c1.cout == 128))) {
        // conv3 + residual + ReLU, then the next block's conv1 on the rows just produced
        // (pw_chain.hip): the block output is not read back from HBM. Block 2 -> 3: 186 us
        // against 164 + 111 us for the two GEMMs; block 3 -> layer2 (N2 = 128) in the
        // register-weight form (the LDS-weight form, two tile buffers, took 297 us against
        // 162 + 132).
        const Bottleneck& nx = blocks[bi + 1];
        MEC_TRY(prof.begin(TAG_RESNET_CONV1X1, s));
        MEC_TRY(launch_pw_chain(t2, in, Wt + bk.c3.w_off, P + bk.c3.b_off, Wt + nx.c1.w_off, P + nx.c1.b_off, out,
                                T1 + (size_t)i0 * OH * OH * nx.c1.cout, nb * OH * OH, nx.c1.cout, s));
        MEC_TRY(prof.end(TAG_RESNET_CONV1X1, s));
        conv1_done = true;
      } else {
        g = GemmParams();
        g.A = t2; g.B = Wt + bk.c3.w_off; g.bias = P + bk.c3.b_off; g.R = in; g.act = ACT_RELU; g.C16 = out;
        g.M = nb * OH * OH; g.N = 4 * wd; g.K = wd;
        MEC_TRY(launch_gemm(g, s, &prof, TAG_RESNET_CONV1X1));
      }
      std::swap(cur, other);
      H = OH;
    }
    return 0;
  };
  // Layers 1-2 can run over chunks of opt().resnet_chunk images, so that a chunk's activations
  // stay in the 256-MB Infinity Cache between a block's producer and consumer kernels (off by
  // default: measured slower, see opt().resnet_chunk). Every GEMM row and conv pixel is computed
  // the same way at any batch split, so the outputs do not depend on the chunk size.
  constexpr size_t kL12 = 7;  // layer1 (3 blocks) + layer2 (4 blocks)
  f16* cur = X;
  f16* other = Y;
  const int chunk = opt().resnet_chunk > 0 ? std::min(opt().resnet_chunk, B) : B;
  for (int i0 = 0; i0 < B; i0 += chunk) {
    f16* c = X;
    f16* o = Y;
    MEC_TRY(run_blocks(0, kL12, i0, std::min(chunk, B - i0), 56, c, o));
    cur = c;
    other = o;
  }
  MEC_TRY(run_blocks(kL12, blocks.size(), 0, B, 28, cur, other));
  H = 7;
  hipLaunchKernelGGL(avgpool8_kernel, dim3(B), dim3(2048 / 8 * 4), 0, s, cur, H * H, 2048, pooled);
  MEC_LAUNCH_CHECK();
  // fc[1] Linear(2048,512) + fc[2] ReLU -> the 512-d feature (extract_features), then fc[4] + softmax
  MEC_TRY(launch_linear_mfma<BACT_RELU>(pooled, 2048, B, 2048, P + fc1_off, P + fc1b_off, 512, feat, 512, nullptr, 0, s));
  MEC_TRY(launch_head7(feat, B, 512, P + fc2_off, P + fc2b_off, logits, probs, s));
  return 0;
}

}  // namespace mec
