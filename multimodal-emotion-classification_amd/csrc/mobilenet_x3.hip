// MobileNetV2 image path on the fp32x3 engine (mec_create_ex(MEC_IMAGE_MBV2, ..., MEC_PREC_FP32X3)):
// the fp32 arithmetic of mobilenet_f32.hip (torchvision mobilenet_v2 features, README.md:13, restated
// by oracle/image_mbv2.py, with the reference's transform and head: inference/image_inference.py:28-32,
// :59-65) in the fused one-kernel-per-block form of mobilenet.hip, with every 1x1 product on the f16
// MFMA as hi.hi + hi.lo + lo.hi of exact f16 hi / lo pairs (the split GEMM engine's arithmetic,
// gemm_glds.hip) into one fp32 accumulator:
//   expand   E = ReLU6(We X 2^-e + be): X (the block input, f32 in HBM) split into hi / lo planes as the
//            tile is staged in LDS, We pre-split on the host (per-matrix power-of-two scale); E in fp32
//   dw       D = ReLU6(bd + sum_taps E w) in fp32 (torch's (kh, kw) tap order), split into planes
//   project  Y = Wp D 2^-e + bp (+ the block input, read back from HBM in f32: an exact residual)
// Block outputs are f32 NHWC in HBM (the same bytes as two f16 planes); the expanded (6x wider)
// tensors never leave the CU. Block 1 (t = 1) also computes the stem (3x3/2 on the u8 image,
// ToTensor / Normalize / BN folded into fp32 weights with a border-class bias) for its tile, kept in
// fp32 for its depthwise conv. features[18] (1x1 320 -> 1280 + BN + ReLU6) runs on the split GEMM.
#include <algorithm>
#include <cmath>

#include "block_ops.h"
#include "models.h"

namespace mec {

namespace {

constexpr int MX_HC = 32;  // hidden channels per chunk

struct MbX3Args {
  const void* x;        // block input f32 NHWC [B,H,H,cin] (STEM == 0) or the u8 image [B,224,224,STEM]
  float* y;             // block output f32 NHWC [B,OH,OH,cout]
  int H, OH, cin, cout;
  const f16* We;        // expand hi plane [HIDP][CINP]; lo plane at We + we_lo
  long long we_lo;
  float x_up;           // 2^s: the block input's plane scale (the planes carry x 2^s)
  float we_scale;       // 2^-e 2^-s: undoes the expand planes' pre-scale and the input's plane scale
  const float* be;      // [HIDP]
  const float* Wd;      // [HIDP/8][9][8]
  const float* bd;      // [HIDP]
  const f16* Wp;        // project hi plane [COUTP][HIDP]; lo plane at Wp + wp_lo
  long long wp_lo;
  float wp_scale;       // 2^-e 2^-13: the project planes' pre-scale and the depthwise output's (kDwUp)
  const float* bp;      // [COUTP]
  const float* stem_w;     // [C*9][32] folded stem weights (STEM > 0)
  const float* stem_corr;  // [4][32] bias per border class (STEM > 0)
  unsigned* flag;          // range flag (x3_raise): a block input outside the f16 range
  int ntiles;              // B * (OH / TO)^2 output tiles, walked with a stride of gridDim.x
};

__device__ __forceinline__ float relu6x(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

// The depthwise output (ReLU6: in [0, 6]) is split at a fixed scale 2^13 (6 2^13 = 49152 < 65504): its
// planes keep 22 significant bits down to 2^-16 and can never overflow
constexpr float kDwUp = 8192.f;

// 16-B chunk c of f16 plane row p of CH chunks sits at chunk mx_sw<CH>(p, c): the rows are unpadded, and
// the XOR puts the 16 lanes of every ds_read_b128 lane group of a 16x16x32 fragment read (rows p, chunks
// 4 k + (lane >> 4)) on 16 distinct 4-bank slots (MI355X_MICROARCH.md, LDS lane groups): CH = 4 (mod 8)
// rows (64 / 192 / 320 B) take gemm_common.h's sw<32> swizzle, CH = 8 (128 B) its sw<64>. Same values,
// same arithmetic: only the LDS addresses move.
template <int CH>
__device__ __forceinline__ int mx_sw(int p, int c) {
  static_assert(CH % 4 == 0, "rows of whole 32-deep k chunks");
  if constexpr (CH % 8 == 0) return c ^ ((p >> 1) & 7);
  else return c ^ ((4 - ((p >> 2) & 3)) & 3);
}

template <int SEL>
__device__ __forceinline__ int se_sw(int p) {
  if constexpr (SEL < 0) return 0;  // unswizzled 36-float rows (opt().mbv2_x3_sesw 0)
  else if constexpr (SEL == 0) return (p ^ (p >> 4)) & 7;
  else if constexpr (SEL == 1) return (p ^ (p >> 1)) & 7;
  else if constexpr (SEL == 2) return (p ^ (p >> 3)) & 7;
  else return ((p >> 1) ^ (p >> 2)) & 7;
}

template <int S, int TO, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM, bool SW = true>
struct MxGeom {
  static constexpr int IR = (TO - 1) * S + 3, NP = IR * IR, MP = (NP + 15) / 16 * 16;
  static constexpr int XLD = CINP;       // f16 plane row (halfs; chunks swizzled, mx_sw)
  // f32 row of the non-expand (stem) input tile: unpadded with its 16-B chunks XOR-swizzled by bit 1 of the
  // row (SW: a depthwise / stem ds_*_b128 lane group covers 4 consecutive rows x 4 even or 4 odd chunks,
  // which then fall on 16 distinct 4-bank slots), else padded to 36 floats
  static constexpr int XF = SW ? CINP : CINP + 4;
  // f32 row of the expanded chunk (floats) and the 16-B chunk swizzle se_sw of its rows, per tile shape:
  // the rows the depthwise's ds_read_b128 lane groups read (4 - 8 input pixels, one per output pixel of
  // the group, at one tap) spread over distinct 4-bank slots; the expand epilogue's ds_write_b128 stays
  // conflict-free (a python search over every tap, lane group and row stride 32..64 floats: LDS cycles of
  // the depthwise reads -40 / -50 / -15 / -60 % for the 4x4/2, 8x8/1, 7x7/1 and 7x7/2 tiles against the
  // unswizzled 36-float rows)
  static constexpr int SEL = !SW ? -1 : (S == 2 && TO == 4) ? 0 : (S == 1 && TO == 8) ? 1 : (S == 1) ? 2 : 3;
  static constexpr int EF = SEL < 0 ? MX_HC + 4 : (SEL == 1 || SEL == 2) ? MX_HC : MX_HC + 16;
  static constexpr int ELD = MX_HC;      // f16 plane row of the depthwise output (chunks swizzled)
  static constexpr int NQ = TO * TO;
  // depthwise-output rows: the output pixels rounded up to whole 16-pixel project fragments (16 for
  // a 4 x 4 tile, where 64 rows put the stride-2 blocks at three workgroups per CU instead of four)
  static constexpr int NDR = (NQ + 15) / 16 * 16;
  static constexpr int OT = COUTP / 16, KX = CINP / 32;
  static constexpr size_t LDS_FIXED = (size_t)(EXPAND ? 2 * MP * XLD * 2 + MP * EF * 4 : MP * XF * 4) +
                                      2 * NDR * ELD * 2 + (HIDP * (EXPAND ? 2 : 1) + COUTP) * 4;
  // depthwise weights staged in LDS when they fit beside the tile (else read through L1 / L2)
  static constexpr bool DWL = LDS_FIXED + HIDP * 9 * 4 <= 128 * 1024;
};

// OCC: workgroups per CU the register allocation targets (launch bounds). 4 for most shapes (16 waves per
// CU; the wider ones exceed it and run at the occupancy their registers allow); the stride-2 4x4-tile
// shapes take opt().mbv2_x3_occ (3: 168 VGPRs, no spill; 4: 128 VGPRs and an 84-B spill per lane).
template <int S, int TO, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM, int OCC = 4, bool SW = true>
__global__ __launch_bounds__(256, OCC) void mbv2_x3_kernel(const MbX3Args a) {
  using G = MxGeom<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, SW>;
  constexpr int IR = G::IR, NP = G::NP, MP = G::MP, XLD = G::XLD, XF = G::XF, EF = G::EF, ELD = G::ELD;
  constexpr int NQ = G::NQ, NDR = G::NDR, OT = G::OT, KX = G::KX;
  static_assert(NQ <= 64, "tile");
  static_assert(!STEM || (CINP == 32 && HIDP == 32 && !EXPAND && S == 1), "stem fuses into block 1 only");
  static_assert(STEM || EXPAND, "t = 1 blocks only as block 1 (with the stem)");
  __shared__ __attribute__((aligned(16))) f16 sXh[EXPAND ? MP * XLD : 8];
  __shared__ __attribute__((aligned(16))) f16 sXl[EXPAND ? MP * XLD : 8];
  __shared__ __attribute__((aligned(16))) float sXf[EXPAND ? 4 : MP * XF];
  __shared__ __attribute__((aligned(16))) float sE[EXPAND ? MP * EF : 4];
  __shared__ __attribute__((aligned(16))) f16 sDh[NDR * ELD];
  __shared__ __attribute__((aligned(16))) f16 sDl[NDR * ELD];
  __shared__ __attribute__((aligned(16))) float sWd[G::DWL ? HIDP * 9 : 4];
  __shared__ __attribute__((aligned(16))) float sBd[HIDP];
  __shared__ __attribute__((aligned(16))) float sBe[EXPAND ? HIDP : 4];
  __shared__ __attribute__((aligned(16))) float sBp[COUTP];
  constexpr int PR = 2 * (TO + 2) + 1;  // stem: u8 patch side
  __shared__ __attribute__((aligned(16))) float sSW[STEM ? STEM * 9 * 32 : 4];
  __shared__ uint8_t sPatch[STEM ? PR * PR * STEM : 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpr = a.OH / TO;
  // float offset of 16-B chunk c of row p of the stem tile sXf
  auto xf = [](int p, int c) { return p * XF + (SW ? (c ^ ((p >> 1) & 1)) : c) * 4; };
  const int H = a.H;
  const int l16 = lane & 15, lq = lane >> 4;

  // ---- per-block constants -> LDS
  if constexpr (G::DWL)
    for (int i = tid; i < HIDP * 9 / 4; i += 256) reinterpret_cast<float4*>(sWd)[i] = reinterpret_cast<const float4*>(a.Wd)[i];
  for (int i = tid; i < HIDP / 4; i += 256) {
    reinterpret_cast<float4*>(sBd)[i] = reinterpret_cast<const float4*>(a.bd)[i];
    if constexpr (EXPAND) reinterpret_cast<float4*>(sBe)[i] = reinterpret_cast<const float4*>(a.be)[i];
  }
  if (tid < COUTP / 4) reinterpret_cast<float4*>(sBp)[tid] = reinterpret_cast<const float4*>(a.bp)[tid];

  // expand weights of a chunk (A fragments, rows = hidden channels), hi and lo planes: each wave computes
  // one 16-channel half of the chunk (ht = wave & 1) for every other 16-pixel tile, so it loads that half
  const int eht = wave & 1;
  half8 afh[KX], afl[KX];
  auto load_af = [&](int h0) {
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const size_t o = (size_t)(h0 + 16 * eht + l16) * CINP + 32 * k + 8 * lq;
      afh[k] = *reinterpret_cast<const half8*>(a.We + o);
      afl[k] = *reinterpret_cast<const half8*>(a.We + a.we_lo + o);
    }
  };
  // block input tile t (+ halo) -> registers: zeros outside the image and past cin
  constexpr int C4 = CINP / 4;
  constexpr int NIT = STEM == 0 ? (MP * C4 + 255) / 256 : 1;
  auto load_in = [&](int t, float4 (&v)[NIT]) {
    const int n = t / (tpr * tpr), tt = t - n * tpr * tpr;
    const int iy0 = (tt / tpr) * TO * S - 1, ix0 = (tt - (tt / tpr) * tpr) * TO * S - 1;
    const float* xin = reinterpret_cast<const float*>(a.x) + (size_t)n * H * H * a.cin;
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
      const int i = tid + 256 * j;
      const int p = i / C4, c4 = i - (i / C4) * C4;
      const int py = p / IR, px = p - (p / IR) * IR;
      const int iy = iy0 + py, ix = ix0 + px;
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < MP * C4 && p < NP && iy >= 0 && iy < H && ix >= 0 && ix < H && c4 * 4 < a.cin)
        v[j] = *reinterpret_cast<const float4*>(xin + ((size_t)iy * H + ix) * a.cin + c4 * 4);
    }
  };
  float4 xv[NIT];
  if constexpr (STEM == 0)
    if (blockIdx.x < a.ntiles) load_in(blockIdx.x, xv);

  // depthwise item of this thread: output pixel dq, channels 8 dcg .. 8 dcg + 7 of the chunk
  const int dq = tid >> 2, dcg = tid & 3;
  const int dqy = dq / TO, dqx = dq - (dq / TO) * TO;
  const int dp0 = (dqy * S) * IR + dqx * S;  // top-left tap of the 3x3 window
  const float* wdsrc = G::DWL ? sWd : a.Wd;

  // Tiles blockIdx.x, + gridDim.x, ...: tile t + gridDim.x's input is loaded into registers while tile
  // t computes. No barrier is needed before the next tile's LDS stores: every wave has passed the
  // barrier after the last chunk's depthwise (sX, sE and sXf are read before it), and the next
  // tile's depthwise writes sD only after the barrier behind its staging, which no wave passes while
  // another still projects.
#pragma unroll 1
  for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
  const int n = t / (tpr * tpr);
  const int tt = t - n * tpr * tpr;
  const int oy0 = (tt / tpr) * TO, ox0 = (tt - (tt / tpr) * tpr) * TO;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;  // input tile origin (pad 1)
  if constexpr (EXPAND) load_af(0);

  // ---- stage the block input tile
  if constexpr (STEM == 0) {
    // f32 x 2^s -> hi / lo planes (x_up = 2^s: exact): x 2^s - hi is exact in f32, lo = f16(x 2^s - hi)
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NIT; ++j) {  // ... then the split and the LDS stores
      const int i = tid + 256 * j;
      const int p = i / C4, c4 = i - (i / C4) * C4;
      if (i < MP * C4) {
        const float4 u = make_float4(xv[j].x * a.x_up, xv[j].y * a.x_up, xv[j].z * a.x_up, xv[j].w * a.x_up);
        const half4 h = {(f16)u.x, (f16)u.y, (f16)u.z, (f16)u.w};
        const half4 l = {(f16)(u.x - (float)h[0]), (f16)(u.y - (float)h[1]), (f16)(u.z - (float)h[2]),
                         (f16)(u.w - (float)h[3])};
        const int xo = p * XLD + mx_sw<CINP / 8>(p, c4 >> 1) * 8 + (c4 & 1) * 4;
        *reinterpret_cast<half4*>(sXh + xo) = h;
        *reinterpret_cast<half4*>(sXl + xo) = l;
        bad |= x3_out_of_range4(u);
      }
    }
    x3_raise(a.flag, bad);
    if (t + (int)gridDim.x < a.ntiles) load_in(t + gridDim.x, xv);  // lands under this tile's MFMAs
  } else {
    // stem conv 3x3/2 pad 1 on the u8 image for stem pixel (iy, ix) of the 112x112 grid, in fp32
    const uint8_t* img = reinterpret_cast<const uint8_t*>(a.x) + (size_t)n * 224 * 224 * STEM;
    const int ry0 = 2 * iy0 - 1, rx0 = 2 * ix0 - 1;
    for (int i = tid; i < PR * PR * STEM; i += 256) {
      const int c = i % STEM, pix = i / STEM;
      const int yy = ry0 + pix / PR, xx = rx0 + pix % PR;
      sPatch[i] = (yy >= 0 && yy < 224 && xx >= 0 && xx < 224) ? img[((size_t)yy * 224 + xx) * STEM + c] : 0;
    }
    for (int i = tid; i < STEM * 9 * 8; i += 256)
      reinterpret_cast<float4*>(sSW)[i] = reinterpret_cast<const float4*>(a.stem_w)[i];
    __syncthreads();
    for (int i = tid; i < MP * 4; i += 256) {
      const int p = i >> 2, cg = i & 3;
      const int py = p / IR, px = p - (p / IR) * IR;
      const int iy = iy0 + py, ix = ix0 + px;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (p < NP && iy >= 0 && iy < 112 && ix >= 0 && ix < 112) {
        const int cls = (iy == 0 ? 2 : 0) + (ix == 0 ? 1 : 0);
        const float4 c0 = *reinterpret_cast<const float4*>(a.stem_corr + cls * 32 + cg * 8);
        const float4 c1 = *reinterpret_cast<const float4*>(a.stem_corr + cls * 32 + cg * 8 + 4);
        acc[0] = c0.x; acc[1] = c0.y; acc[2] = c0.z; acc[3] = c0.w;
        acc[4] = c1.x; acc[5] = c1.y; acc[6] = c1.z; acc[7] = c1.w;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int c = 0; c < STEM; ++c) {
              const float u = (float)sPatch[((2 * py + ky) * PR + 2 * px + kx) * STEM + c];
              const float* w = sSW + ((c * 3 + ky) * 3 + kx) * 32 + cg * 8;
              const float4 w0 = *reinterpret_cast<const float4*>(w);
              const float4 w1 = *reinterpret_cast<const float4*>(w + 4);
              acc[0] = __builtin_fmaf(u, w0.x, acc[0]); acc[1] = __builtin_fmaf(u, w0.y, acc[1]);
              acc[2] = __builtin_fmaf(u, w0.z, acc[2]); acc[3] = __builtin_fmaf(u, w0.w, acc[3]);
              acc[4] = __builtin_fmaf(u, w1.x, acc[4]); acc[5] = __builtin_fmaf(u, w1.y, acc[5]);
              acc[6] = __builtin_fmaf(u, w1.z, acc[6]); acc[7] = __builtin_fmaf(u, w1.w, acc[7]);
            }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = relu6x(acc[j]);
      }
      *reinterpret_cast<float4*>(sXf + xf(p, 2 * cg)) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(sXf + xf(p, 2 * cg + 1)) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
  }
  __syncthreads();

  floatx4 acc[OT];
#pragma unroll
  for (int o = 0; o < OT; ++o) acc[o] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int h0 = 0; h0 < HIDP; h0 += MX_HC) {
    // project weights of this chunk (hi and lo): in flight during expand + depthwise; only the waves that
    // project load them (a 4x4 tile's 16 pixels: wave 0 alone)
    half8 pfh[OT], pfl[OT];
    if (16 * wave < NDR) {
#pragma unroll
      for (int o = 0; o < OT; ++o) {
        const size_t off = (size_t)(16 * o + l16) * HIDP + h0 + 8 * lq;
        pfh[o] = *reinterpret_cast<const half8*>(a.Wp + off);
        pfl[o] = *reinterpret_cast<const half8*>(a.Wp + a.wp_lo + off);
      }
    }
    const float* src;  // fp32 depthwise input for this chunk: row p at src + p * sld
    int sld;
    if constexpr (EXPAND) {
      // E^T[h][p] = sum_c We[h0+h][c] X[p][c] (A = weights, B = X^T: a lane ends with 4 consecutive
      // hidden channels of one pixel); per 32-deep k chunk the split engine's terms lo.hi, hi.lo, hi.hi.
      // The (16-pixel tile, 16-channel half) units go round the waves: wave w takes half w & 1 of tiles
      // (w >> 1), (w >> 1) + 2, ... (a 9x9 input tile's six pixel tiles: three units per wave, not 4-4-2-2)
      float eb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) eb[e] = sBe[h0 + 16 * eht + 4 * lq + e];
      for (int pt = wave >> 1; pt < MP / 16; pt += 2) {
        const int p = pt * 16 + l16;
        const int py = p / IR, px = p - (p / IR) * IR;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool valid = p < NP && iy >= 0 && iy < H && ix >= 0 && ix < H;
        floatx4 e2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KX; ++k) {
          const int xo = p * XLD + mx_sw<CINP / 8>(p, 4 * k + lq) * 8;
          const half8 bh = *reinterpret_cast<const half8*>(sXh + xo);
          const half8 bl = *reinterpret_cast<const half8*>(sXl + xo);
          e2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(afl[k], bh, e2, 0, 0, 0);
          e2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(afh[k], bl, e2, 0, 0, 0);
          e2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(afh[k], bh, e2, 0, 0, 0);
        }
        float4 ev;
        ev.x = valid ? relu6x(__builtin_fmaf(e2[0], a.we_scale, eb[0])) : 0.f;  // dw zero pad
        ev.y = valid ? relu6x(__builtin_fmaf(e2[1], a.we_scale, eb[1])) : 0.f;
        ev.z = valid ? relu6x(__builtin_fmaf(e2[2], a.we_scale, eb[2])) : 0.f;
        ev.w = valid ? relu6x(__builtin_fmaf(e2[3], a.we_scale, eb[3])) : 0.f;
        *reinterpret_cast<float4*>(sE + p * EF + ((4 * eht + lq) ^ se_sw<G::SEL>(p)) * 4) = ev;
      }
      if (h0 + MX_HC < HIDP) load_af(h0 + MX_HC);  // next chunk's expand weights: in flight during dw + project
      __syncthreads();
      src = sE;
      sld = EF;
    } else {
      src = sXf + h0;
      sld = XF;
    }

    // ---- depthwise 3x3/S + BN + ReLU6 (fp32) -> sDh / sDl planes [q][h]
    if constexpr (EXPAND && NQ == 16 && NDR == 16) {
      // a 4x4 tile: its 16 pixels x 32 channels over all 256 threads (pixel tid >> 4, channels 2 (tid & 15)
      // and + 1), so no wave waits at the next barrier for one wave's depthwise; each channel's FMAs in the
      // same (ky, kx) order from the shift as below (the same bits)
      const int q = tid >> 4, cp = tid & 15;
      const int p0 = ((q >> 2) * S) * IR + (q & 3) * S;
      const int hc = h0 + 2 * cp;
      float d0 = sBd[hc], d1 = sBd[hc + 1];
      const float* wd = wdsrc + (size_t)(hc / 8) * 72 + (hc & 7);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int pp = p0 + ky * IR + kx;
          const float2 e = *reinterpret_cast<const float2*>(sE + pp * EF + ((cp >> 1) ^ se_sw<G::SEL>(pp)) * 4 +
                                                            (cp & 1) * 2);
          const float2 w = *reinterpret_cast<const float2*>(wd + (ky * 3 + kx) * 8);
          d0 = __builtin_fmaf(e.x, w.x, d0);
          d1 = __builtin_fmaf(e.y, w.y, d1);
        }
      const float v0 = relu6x(d0) * kDwUp, v1 = relu6x(d1) * kDwUp;  // in [0, 6 2^13]
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
      const h2 hh = {(f16)v0, (f16)v1};
      const h2 hl = {(f16)(v0 - (float)hh[0]), (f16)(v1 - (float)hh[1])};
      const int dof = q * ELD + mx_sw<MX_HC / 8>(q, cp >> 2) * 8 + (cp & 3) * 2;
      *reinterpret_cast<h2*>(sDh + dof) = hh;
      *reinterpret_cast<h2*>(sDl + dof) = hl;
    } else {
      half8 oh = {0, 0, 0, 0, 0, 0, 0, 0}, ol = {0, 0, 0, 0, 0, 0, 0, 0};
      if (dq < NQ) {
        const int hc = h0 + 8 * dcg;
        float d[8];
        {
          const float4 b0 = *reinterpret_cast<const float4*>(sBd + hc);
          const float4 b1 = *reinterpret_cast<const float4*>(sBd + hc + 4);
          d[0] = b0.x; d[1] = b0.y; d[2] = b0.z; d[3] = b0.w; d[4] = b1.x; d[5] = b1.y; d[6] = b1.z; d[7] = b1.w;
        }
        const float* wd = wdsrc + (size_t)(hc / 8) * 72;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int pp = dp0 + ky * IR + kx;
            float4 e0, e1;
            if constexpr (EXPAND) {  // sE: chunks swizzled (se_sw)
              const int f = se_sw<G::SEL>(pp);
              e0 = *reinterpret_cast<const float4*>(src + pp * sld + ((2 * dcg) ^ f) * 4);
              e1 = *reinterpret_cast<const float4*>(src + pp * sld + ((2 * dcg + 1) ^ f) * 4);
            } else {  // sXf: chunks swizzled (xf)
              e0 = *reinterpret_cast<const float4*>(sXf + xf(pp, h0 / 4 + 2 * dcg));
              e1 = *reinterpret_cast<const float4*>(sXf + xf(pp, h0 / 4 + 2 * dcg + 1));
            }
            const float4 w0 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8);
            const float4 w1 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8 + 4);
            d[0] = __builtin_fmaf(e0.x, w0.x, d[0]); d[1] = __builtin_fmaf(e0.y, w0.y, d[1]);
            d[2] = __builtin_fmaf(e0.z, w0.z, d[2]); d[3] = __builtin_fmaf(e0.w, w0.w, d[3]);
            d[4] = __builtin_fmaf(e1.x, w1.x, d[4]); d[5] = __builtin_fmaf(e1.y, w1.y, d[5]);
            d[6] = __builtin_fmaf(e1.z, w1.z, d[6]); d[7] = __builtin_fmaf(e1.w, w1.w, d[7]);
          }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = relu6x(d[j]) * kDwUp;  // in [0, 6 2^13]: always inside the f16 range
          oh[j] = (f16)v;
          ol[j] = (f16)(v - (float)oh[j]);
        }
      }
      if (dq < NDR) {  // rows NQ .. NDR - 1: zeros for the last fragment's padding pixels
        const int dof = dq * ELD + mx_sw<MX_HC / 8>(dq, dcg) * 8;
        *reinterpret_cast<half8*>(sDh + dof) = oh;
        *reinterpret_cast<half8*>(sDl + dof) = ol;
      }
    }
    __syncthreads();

    // ---- project: out^T[o][q] += Wp[o][h0..h0+31] . D[q][:]; wave w owns pixels 16w..16w+15 (the
    // waves past the tile's pixels have nothing to project)
    if (16 * wave < NDR) {
      const int r = 16 * wave + l16, dof = r * ELD + mx_sw<MX_HC / 8>(r, lq) * 8;
      const half8 bh = *reinterpret_cast<const half8*>(sDh + dof);
      const half8 bl = *reinterpret_cast<const half8*>(sDl + dof);
#pragma unroll
      for (int o = 0; o < OT; ++o) {
        acc[o] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pfl[o], bh, acc[o], 0, 0, 0);
        acc[o] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pfh[o], bl, acc[o], 0, 0, 0);
        acc[o] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pfh[o], bh, acc[o], 0, 0, 0);
      }
    }
    if constexpr (!EXPAND) __syncthreads();  // next chunk's dw rewrites sD
  }

  // ---- epilogue: acc 2^-e + BN shift (+ the exact f32 block input) -> f32 NHWC
  {
    const int q = 16 * wave + l16;
    if (q < NQ) {
      const int qy = q / TO, qx = q - (q / TO) * TO;
      const size_t pix = (size_t)n * a.OH * a.OH + (size_t)(oy0 + qy) * a.OH + ox0 + qx;
      float4 r[OT];
      if constexpr (RES) {  // stride 1 and cin == cout: the same pixel of the block input
#pragma unroll
        for (int o = 0; o < OT; ++o) {
          const int c = 16 * o + 4 * lq;
          r[o] = c < a.cout ? *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.x) + pix * a.cin + c)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int o = 0; o < OT; ++o) {
        const int c = 16 * o + 4 * lq;
        if (c >= a.cout) continue;
        const float4 bv = *reinterpret_cast<const float4*>(sBp + c);
        float4 v = make_float4(__builtin_fmaf(acc[o][0], a.wp_scale, bv.x), __builtin_fmaf(acc[o][1], a.wp_scale, bv.y),
                               __builtin_fmaf(acc[o][2], a.wp_scale, bv.z), __builtin_fmaf(acc[o][3], a.wp_scale, bv.w));
        if constexpr (RES) {
          v.x += r[o].x; v.y += r[o].y; v.z += r[o].z; v.w += r[o].w;
        }
        *reinterpret_cast<float4*>(a.y + pix * a.cout + c) = v;
      }
    }
  }
  }  // tiles
}

// f32 [rows][cin] -> f16 hi / lo planes [rows][ld] of x up (up = 2^s; lo at + lo), channels cin .. ld-1
// zero: the first layered block's input
__global__ __launch_bounds__(256) void mbv2_split_pad_kernel(const float* __restrict__ x, size_t rows, int cin, int ld,
                                                             float up, f16* __restrict__ hi, long long lo,
                                                             unsigned* flag) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // one 4-channel group of one row
  const int G = ld / 4;
  if (i >= rows * G) return;
  const size_t r = i / G;
  const int c = (int)(i - r * G) * 4;
  float4 v = c < cin ? *reinterpret_cast<const float4*>(x + r * cin + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  v.x *= up; v.y *= up; v.z *= up; v.w *= up;
  const half4 h = {(f16)v.x, (f16)v.y, (f16)v.z, (f16)v.w};
  const half4 l = {(f16)(v.x - (float)h[0]), (f16)(v.y - (float)h[1]), (f16)(v.z - (float)h[2]),
                   (f16)(v.w - (float)h[3])};
  *reinterpret_cast<half4*>(hi + r * ld + c) = h;
  *reinterpret_cast<half4*>(hi + lo + r * ld + c) = l;
  x3_raise(flag, x3_out_of_range4(v));
}

// Depthwise 3x3/S (pad 1) + BN shift + ReLU6 of a layered block: E f32 NHWC [B,H,H,C] (the expand GEMM's
// ReLU6 output) -> hi / lo planes of D 2^13 (kDwUp) NHWC [B,OH,OH,C] (lo at D + dlo), the project GEMM's A operand. A
// thread owns one output row of one 8-channel group: its 72 tap weights and a 3-row x 3-column window
// of input pixels stay in registers while it walks the row, so each input pixel is loaded about 3 / S
// times instead of 9 (consecutive threads take consecutive channel groups: every load is part of a
// contiguous run). Per output: fp32 FMAs in torch's (kh, kw) tap order from the shift, as the fused
// kernel's depthwise (whose zero-padded taps add exact zeros).
template <int S>
__global__ __launch_bounds__(256) void mbv2_dw_x3_kernel(const float* __restrict__ E, int H, int OH, int C,
                                                         const float* __restrict__ Wd, const float* __restrict__ bd,
                                                         f16* __restrict__ D, long long dlo, size_t items) {
  const size_t it = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (it >= items) return;
  const int G = C / 8;
  const size_t row = it / G;  // (image, output row)
  const int g = (int)(it - row * G);
  const size_t n = row / OH;
  const int oy = (int)(row - n * OH);
  float w[9][8], bias[8];
  {
    const float* wd = Wd + (size_t)g * 72;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w0 = *reinterpret_cast<const float4*>(wd + t * 8);
      const float4 w1 = *reinterpret_cast<const float4*>(wd + t * 8 + 4);
      w[t][0] = w0.x; w[t][1] = w0.y; w[t][2] = w0.z; w[t][3] = w0.w;
      w[t][4] = w1.x; w[t][5] = w1.y; w[t][6] = w1.z; w[t][7] = w1.w;
    }
    const float4 b0 = *reinterpret_cast<const float4*>(bd + 8 * g);
    const float4 b1 = *reinterpret_cast<const float4*>(bd + 8 * g + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
    bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  bool rok[3];
  const float* rp[3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * S - 1 + ky;
    rok[ky] = iy >= 0 && iy < H;
    rp[ky] = E + ((n * H + (rok[ky] ? iy : 0)) * H) * C + 8 * g;
  }
  // input column ix of the three rows -> e[ky][0..7] (zeros outside the image: those taps are skipped)
  auto load_col = [&](int ix, float (&e)[3][8], bool& ok) {
    ok = ix >= 0 && ix < H;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
      if (ok && rok[ky]) {
        a = *reinterpret_cast<const float4*>(rp[ky] + (size_t)ix * C);
        c = *reinterpret_cast<const float4*>(rp[ky] + (size_t)ix * C + 4);
      }
      e[ky][0] = a.x; e[ky][1] = a.y; e[ky][2] = a.z; e[ky][3] = a.w;
      e[ky][4] = c.x; e[ky][5] = c.y; e[ky][6] = c.z; e[ky][7] = c.w;
    }
  };
  float win[3][3][8];  // [kx][ky][channel]: input columns ox S - 1 + kx
  bool cok[3];
  load_col(-1, win[0], cok[0]);
  load_col(0, win[1], cok[1]);
  f16* dst = D + (row * OH) * C + 8 * g;
  for (int ox = 0; ox < OH; ++ox) {
    if (S == 1) {
      load_col(ox + 1, win[2], cok[2]);
    } else {
      load_col(2 * ox, win[1], cok[1]);
      load_col(2 * ox + 1, win[2], cok[2]);
    }
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = bias[j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      if (!rok[ky]) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        if (!cok[kx]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = __builtin_fmaf(win[kx][ky][j], w[ky * 3 + kx][j], d[j]);
      }
    }
    half8 oh, ol;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = relu6x(d[j]) * kDwUp;  // in [0, 6 2^13]: inside the f16 range
      oh[j] = (f16)v;
      ol[j] = (f16)(v - (float)oh[j]);
    }
    *reinterpret_cast<half8*>(dst + (size_t)ox * C) = oh;
    *reinterpret_cast<half8*>(dst + dlo + (size_t)ox * C) = ol;
    // slide: the next output's first column(s)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        win[0][ky][j] = S == 1 ? win[1][ky][j] : win[2][ky][j];
        if (S == 1) win[1][ky][j] = win[2][ky][j];
      }
    cok[0] = S == 1 ? cok[1] : cok[2];
    if (S == 1) cok[1] = cok[2];
  }
}

template <int S, int TO, int CINP, int HIDP, int COUTP, bool EXPAND, bool RES, int STEM>
int launch_x3_block(const MbX3Args& a0, int B, hipStream_t s) {
  const int tpr = a0.OH / TO;
  MbX3Args a = a0;
  a.ntiles = B * tpr * tpr;
  // opt().mbv2_x3_tpw tiles per workgroup (1: one tile each, no prefetch)
  const int tpw = std::max(1, opt().mbv2_x3_tpw);
  const dim3 grid((a.ntiles + tpw - 1) / tpw);
  // opt().mbv2_x3_sesw: the expanded chunk's rows swizzled (1) or unswizzled (0); same bits
  const bool sw = opt().mbv2_x3_sesw != 0;
  if constexpr (TO == 4) {
    if (opt().mbv2_x3_occ == 3 && sw)
      hipLaunchKernelGGL((mbv2_x3_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 3, true>), grid, dim3(256), 0, s, a);
    else if (opt().mbv2_x3_occ == 3)
      hipLaunchKernelGGL((mbv2_x3_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 3, false>), grid, dim3(256), 0, s, a);
    else if (sw)
      hipLaunchKernelGGL((mbv2_x3_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 4, true>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((mbv2_x3_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 4, false>), grid, dim3(256), 0, s, a);
  } else if (sw) {
    hipLaunchKernelGGL((mbv2_x3_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 4, true>), grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((mbv2_x3_kernel<S, TO, CINP, HIDP, COUTP, EXPAND, RES, STEM, 4, false>), grid, dim3(256), 0, s, a);
  }
  MEC_LAUNCH_CHECK();
  return 0;
}

// The 17 block shapes of mobilenet_v2 at 224x224 (as mobilenet.hip dispatch_block)
int dispatch_x3_block(const MbBlock& b, const MbX3Args& a, int B, int stem_c, hipStream_t s) {
  const bool res = b.stride == 1 && b.cin == b.cout;
  // stride-2 blocks at 56 / 28 outputs: 4x4 output tiles (9x9 inputs, 36-39 KB of LDS, four workgroups
  // per CU) when opt().mbv2_x3_tile == 4, else 8x8 / 7x7 tiles (17x17 / 15x15 inputs, one per CU)
  const int TO = (opt().mbv2_x3_tile == 4 && b.stride == 2 && a.OH % 4 == 0) ? 4 : (a.OH % 8 == 0) ? 8 : 7;
#define MX_CASE(S_, TO_, CI_, HI_, CO_, RS_)                                                                      \
  if (b.stride == S_ && TO == TO_ && b.cinp == CI_ && b.hidp == HI_ && b.coutp == CO_ && b.t != 1 && res == RS_) \
    return launch_x3_block<S_, TO_, CI_, HI_, CO_, true, RS_, 0>(a, B, s);
  if (b.t == 1) {
    MEC_REQUIRE(b.stride == 1 && b.cinp == 32 && b.hidp == 32 && b.coutp == 16 && !res && TO == 8 && stem_c,
                "mbv2 x3: block 1 shape");
    if (stem_c == 3) return launch_x3_block<1, 8, 32, 32, 16, false, false, 3>(a, B, s);
    return launch_x3_block<1, 8, 32, 32, 16, false, false, 1>(a, B, s);
  }
  MX_CASE(2, 4, 32, 96, 32, false)     // 16 -> 24, 112 -> 56 (4x4 tiles)
  MX_CASE(2, 4, 32, 160, 32, false)    // 24 -> 32, 56 -> 28 (4x4 tiles)
  MX_CASE(2, 8, 32, 96, 32, false)     // 16 -> 24, 112 -> 56
  MX_CASE(1, 8, 32, 160, 32, true)     // 24 -> 24 @ 56
  MX_CASE(2, 7, 32, 160, 32, false)    // 24 -> 32, 56 -> 28
  MX_CASE(1, 7, 32, 192, 32, true)     // 32 -> 32 @ 28
  MX_CASE(2, 7, 32, 192, 64, false)    // 32 -> 64, 28 -> 14
  MX_CASE(1, 7, 64, 384, 64, true)     // 64 -> 64 @ 14
  MX_CASE(1, 7, 64, 384, 96, false)    // 64 -> 96 @ 14
  MX_CASE(1, 7, 96, 576, 96, true)     // 96 -> 96 @ 14
  MX_CASE(2, 7, 96, 576, 160, false)   // 96 -> 160, 14 -> 7
  MX_CASE(1, 7, 160, 960, 160, true)   // 160 -> 160 @ 7
  // (160 -> 320 @ 7, features[17], always runs layered: fused, its 20 project fragments of 16 channels
  // (acc and hi / lo weights: 200 registers) spill at any occupancy)
#undef MX_CASE
  set_error("mbv2 x3: no kernel instance for this block shape");
  return -1;
}

}  // namespace

// fp32x3 weights: the f16 path's layouts (channels padded to 32 / 32 / 16, depthwise [hidp/8][9][8],
// stem folded per pixel with a border-class bias) built in fp32, then every 1x1 matrix split into
// hi / lo planes after a per-matrix power-of-two pre-scale (split_planes)
int MobileNetModel::create_x3(const float* blob, size_t n) {
  BlobReader rd(blob, n);
  std::vector<float> w, pr;
  auto align4 = [&]() { while (pr.size() % 4) pr.push_back(0.f); };
  auto pad_to = [](int v, int m) { return (v + m - 1) / m * m; };
  double est = 0.0;  // the last BN's output estimate, max_c |beta_c| + 6 |gamma_c| (activation_exp)
  auto bn_scale_shift = [&](int c, std::vector<double>& scale, std::vector<double>& shift) {
    const float* g = rd.take(c);
    const float* b = rd.take(c);
    const float* rm = rd.take(c);
    const float* rv = rd.take(c);
    scale.assign(c, 0.0);
    shift.assign(c, 0.0);
    est = 0.0;
    if (!rd.ok) return;
    for (int i = 0; i < c; ++i) {
      scale[i] = (double)g[i] / std::sqrt((double)rv[i] + 1e-5);
      shift[i] = (double)b[i] - (double)rm[i] * scale[i];
      est = std::max(est, std::fabs((double)b[i]) + 6.0 * std::fabs((double)g[i]));
    }
  };
  std::vector<double> sc, sh;
  {  // stem, as MobileNetModel::create (mobilenet.hip)
    const float* src = rd.take((size_t)32 * 3 * 9);
    bn_scale_shift(32, sc, sh);
    align4();
    stem_w_off = pr.size();
    pr.resize(pr.size() + 9 * 32, 0.f);
    stem_rgb_off = pr.size();
    pr.resize(pr.size() + 27 * 32, 0.f);
    stem_corr_off = pr.size();
    pr.resize(pr.size() + 4 * 32, 0.f);
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
    if (rd.ok)
      for (int o = 0; o < 32; ++o) {
        double cterm[9] = {};
        for (int t = 0; t < 9; ++t) {
          double gsum = 0.0;
          for (int c = 0; c < 3; ++c) {
            const double wv = src[((size_t)o * 3 + c) * 9 + t];
            const double mf = (double)(float)mean[c], sf = (double)(float)stdv[c];
            gsum += wv / (255.0 * sf);
            cterm[t] -= wv * mf / sf;
            pr[stem_rgb_off + (size_t)(c * 9 + t) * 32 + o] = (float)(wv / (255.0 * sf) * sc[o]);
          }
          pr[stem_w_off + (size_t)t * 32 + o] = (float)(gsum * sc[o]);
        }
        for (int cls = 0; cls < 4; ++cls) {
          double sum = sh[o];
          for (int t = 0; t < 9; ++t) {
            const int ky = t / 3, kx = t % 3;
            if (((cls & 2) && ky == 0) || ((cls & 1) && kx == 0)) continue;
            sum += cterm[t] * sc[o];
          }
          pr[stem_corr_off + (size_t)cls * 32 + o] = (float)sum;
        }
      }
  }
  static const int kSet[7][4] = {{1, 16, 1, 1}, {6, 24, 2, 2}, {6, 32, 3, 2}, {6, 64, 4, 2},
                                 {6, 96, 3, 1}, {6, 160, 3, 2}, {6, 320, 1, 1}};
  blocks.clear();
  x3_scale.clear();
  lx3_scale.clear();
  int cin = 32, prev_lcoutp = 32;
  for (int si = 0; si < 7; ++si)
    for (int r = 0; r < kSet[si][2]; ++r) {
      MbBlock b;
      b.t = kSet[si][0]; b.cin = cin; b.hid = cin * b.t; b.cout = kSet[si][1]; b.stride = r == 0 ? kSet[si][3] : 1;
      b.cinp = pad_to(cin, 32); b.hidp = pad_to(b.hid, 32); b.coutp = pad_to(b.cout, 16);
      if (b.t != 1) {
        const float* we = rd.take((size_t)b.hid * cin);
        bn_scale_shift(b.hid, sc, sh);
        b.we_off = w.size();
        w.resize(w.size() + (size_t)b.hidp * b.cinp, 0.f);
        align4();
        b.be_off = pr.size();
        pr.resize(pr.size() + b.hidp, 0.f);
        if (rd.ok)
          for (int h = 0; h < b.hid; ++h) {
            for (int c = 0; c < cin; ++c) w[b.we_off + (size_t)h * b.cinp + c] = (float)((double)we[(size_t)h * cin + c] * sc[h]);
            pr[b.be_off + h] = (float)sh[h];
          }
      }
      {
        const float* wd = rd.take((size_t)b.hid * 9);
        bn_scale_shift(b.hid, sc, sh);
        align4();
        b.wd_off = pr.size();
        pr.resize(pr.size() + (size_t)b.hidp * 9, 0.f);
        b.bd_off = pr.size();
        pr.resize(pr.size() + b.hidp, 0.f);
        if (rd.ok)
          for (int h = 0; h < b.hid; ++h) {
            for (int t = 0; t < 9; ++t)
              pr[b.wd_off + (size_t)(h / 8) * 72 + t * 8 + (h % 8)] = (float)((double)wd[(size_t)h * 9 + t] * sc[h]);
            pr[b.bd_off + h] = (float)sh[h];
          }
      }
      {
        const float* wp = rd.take((size_t)b.cout * b.hid);
        bn_scale_shift(b.cout, sc, sh);
        b.x3_est = est;
        b.wp_off = w.size();
        w.resize(w.size() + (size_t)b.coutp * b.hidp, 0.f);
        align4();
        b.bp_off = pr.size();
        pr.resize(pr.size() + b.coutp, 0.f);
        if (rd.ok)
          for (int o = 0; o < b.cout; ++o) {
            for (int h = 0; h < b.hid; ++h) w[b.wp_off + (size_t)o * b.hidp + h] = (float)((double)wp[(size_t)o * b.hid + h] * sc[o]);
            pr[b.bp_off + o] = (float)sh[o];
          }
      }
      b.lcinp = prev_lcoutp;
      b.lcoutp = pad_to(b.cout, 64);
      prev_lcoutp = b.lcoutp;
      if (b.t != 1 && b.hidp % 64 == 0) {  // layered form: the same matrices, K / N padded with zeros
        b.lwe_off = w.size();
        w.resize(w.size() + (size_t)b.hidp * b.lcinp, 0.f);
        for (int h = 0; h < b.hidp; ++h)
          for (int c = 0; c < b.cinp && c < b.lcinp; ++c)
            w[b.lwe_off + (size_t)h * b.lcinp + c] = w[b.we_off + (size_t)h * b.cinp + c];
        b.lwp_off = w.size();
        w.resize(w.size() + (size_t)b.lcoutp * b.hidp, 0.f);
        std::copy(w.begin() + b.wp_off, w.begin() + b.wp_off + (size_t)b.coutp * b.hidp, w.begin() + b.lwp_off);
        b.lbp_off = pr.size();
        pr.resize(pr.size() + b.lcoutp, 0.f);
        std::copy(pr.begin() + b.bp_off, pr.begin() + b.bp_off + b.coutp, pr.begin() + b.lbp_off);
      }
      blocks.push_back(b);
      cin = b.cout;
    }
  {  // features[18]: [1280][320]
    const float* wl = rd.take((size_t)1280 * 320);
    bn_scale_shift(1280, sc, sh);
    last_w_off = w.size();
    w.resize(w.size() + (size_t)1280 * 320, 0.f);
    align4();
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
  align4();
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
  // Activation-plane exponents (activation_exp, BN estimates): one per stage (a (t, c, n, s) setting:
  // its first block is the only one without a residual, so a stage's outputs -- a residual block's output
  // and its input -- share it), the stage estimate being the running sum of the projection BN estimates
  // along the residual chain. Block inputs are the previous stage's planes; the depthwise outputs are at
  // kDwUp. Every epilogue scale below folds in 2^(s_out - s_in) (the fused blocks' and the expand GEMMs'
  // outputs are f32: s_out = 0 there).
  // opts.x3_plane_scale 0: every exponent 0 (the unscaled planes, A/B only)
  // opts.x3_headroom: 2^-x3_headroom of the target (a handle re-created after a range trip)
  auto aexp = [&](double b, double t) {
    return opts.x3_plane_scale ? activation_exp(b, std::ldexp(t, -opts.x3_headroom)) : 0;
  };
  {
    int s_prev = 0;
    for (size_t b0 = 0; b0 < blocks.size();) {
      size_t b1 = b0 + 1;
      while (b1 < blocks.size() && blocks[b1].stride == 1 && blocks[b1].cin == blocks[b1].cout) ++b1;
      double e = 0.0, e_max = 0.0;
      for (size_t i = b0; i < b1; ++i) {
        e = blocks[i].x3_est + (i > b0 ? e : 0.0);
        e_max = std::max(e_max, e);
      }
      const int st = aexp(e_max, kX3EstimateTarget);
      x3_note("features" + std::to_string(b0 + 1) + "-" + std::to_string(b1) + ".out", st, e_max);
      for (size_t i = b0; i < b1; ++i) {
        blocks[i].x3_s_in = i == b0 ? s_prev : st;
        blocks[i].x3_s_out = st;
      }
      s_prev = st;
      b0 = b1;
    }
  }
  for (MbBlock& b : blocks)
    if (b.lwe_off) {
      align4();
      b.lbp_x3_off = pr.size();
      for (int o = 0; o < b.lcoutp; ++o) pr.push_back(std::ldexp(pr[b.lbp_off + o], b.x3_s_out));
    }
  // split every 1x1 matrix: hi planes at the f32 offsets, lo planes x3_lo halfs later
  x3_lo = w.size();
  std::vector<f16> hl(2 * w.size(), (f16)0.f);
  auto split = [&](size_t off, size_t cnt) { return split_planes(w.data() + off, cnt, hl.data() + off, hl.data() + x3_lo + off); };
  const int dw_s = (int)std::log2(kDwUp);
  for (MbBlock& b : blocks) {
    x3_scale.push_back(b.t != 1 ? std::ldexp(split(b.we_off, (size_t)b.hidp * b.cinp), -b.x3_s_in) : 1.f);
    x3_scale.push_back(std::ldexp(split(b.wp_off, (size_t)b.coutp * b.hidp), -dw_s));
    lx3_scale.push_back(b.lwe_off ? std::ldexp(split(b.lwe_off, (size_t)b.hidp * b.lcinp), -b.x3_s_in) : 1.f);
    lx3_scale.push_back(b.lwe_off ? std::ldexp(split(b.lwp_off, (size_t)b.lcoutp * b.hidp), b.x3_s_out - dw_s) : 1.f);
  }
  x3_scale.push_back(std::ldexp(split(last_w_off, (size_t)1280 * 320), -blocks.back().x3_s_out));
  MEC_TRY(upload(wts, hl.data(), hl.size() * sizeof(f16)));
  MEC_TRY(upload(prm, pr.data(), pr.size() * sizeof(float)));
  return 0;
}

int MobileNetModel::forward_x3(const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits,
                               float* probs, hipStream_t s) {
  MEC_REQUIRE(wts.p && x3_lo && x3_scale.size() == 2 * blocks.size() + 1 && lx3_scale.size() == 2 * blocks.size(),
              "image_mbv2: fp32x3 weights missing");
  const bool fer = (H == 48 && W == 48 && C == 1);
  // layered tail: blocks[l0 ..] (features[l0 + 1 ..]) as expand GEMM -> depthwise -> project GEMM
  // (features[17], 160 -> 320, is layered at every setting: dispatch_x3_block has no fused form of it)
  size_t l0 = blocks.size() - 1;
  if (opt().mbv2_layered) l0 = std::min(l0, (size_t)opt().mbv2_layered - 1);
  for (size_t i = l0; i < blocks.size(); ++i)
    MEC_REQUIRE(blocks[i].lwe_off, "mbv2 x3: mbv2_layered names a block without a layered form");
  // per-image element counts of the layered buffers: E (f32), D / block-I/O planes (halfs per plane)
  size_t pe = 0, pd = 0, pp = 0;
  {
    int hh = 112;
    for (size_t i = 0; i < blocks.size(); ++i) {
      const MbBlock& b = blocks[i];
      const int oh = b.stride == 2 ? hh / 2 : hh;
      if (i >= l0) {
        pe = std::max(pe, (size_t)hh * hh * b.hidp);
        pd = std::max(pd, (size_t)oh * oh * b.hidp);
        pp = std::max(pp, std::max((size_t)hh * hh * b.lcinp, (size_t)oh * oh * b.lcoutp));
      }
      hh = oh;
    }
  }
  const size_t per_big = (size_t)112 * 112 * 16;  // largest block output (features[1]), floats
  const size_t per_last = (size_t)49 * 1280;
  const size_t per_img = 224 * 224 + (2 * per_big + per_last + 1280) * sizeof(float) +
                         pe * sizeof(float) + (pd + 2 * pp) * 2 * sizeof(f16);
  const size_t need = per_img * (size_t)B + 8192;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  uint8_t* resized = reinterpret_cast<uint8_t*>(p);
  p += ((size_t)B * 224 * 224 + 255) / 256 * 256;
  float* X = reinterpret_cast<float*>(p); p += (size_t)B * per_big * sizeof(float);
  float* Y = reinterpret_cast<float*>(p); p += (size_t)B * per_big * sizeof(float);
  float* Lst = reinterpret_cast<float*>(p); p += (size_t)B * per_last * sizeof(float);
  float* pooled = reinterpret_cast<float*>(p); p += (size_t)B * 1280 * sizeof(float);
  float* Eb = reinterpret_cast<float*>(p); p += (size_t)B * pe * sizeof(float);
  const long long dlo = (long long)B * pd, plo = (long long)B * pp;  // plane offsets (halfs)
  f16* Db = reinterpret_cast<f16*>(p); p += (size_t)B * pd * 2 * sizeof(f16);
  f16* P0 = reinterpret_cast<f16*>(p); p += (size_t)B * pp * 2 * sizeof(f16);
  f16* P1 = reinterpret_cast<f16*>(p);

  const f16* Wt = wts.as<f16>();
  const long long wlo = (long long)x3_lo;
  const float* P = prm.as<float>();
  const uint8_t* stem_in = img;
  if (fer) {
    MEC_TRY(resize_u8(img, B, 48, 48, resized, 224, 224, s));
    stem_in = resized;
  }
  MEC_TRY(prof.begin(TAG_MBV2_BLOCK, s));
  const void* cur = stem_in;
  float* out = X;
  int h = 112;
  f16* pin = P0;  // layered blocks: input / output planes
  for (size_t i = 0; i < blocks.size(); ++i) {
    const MbBlock& b = blocks[i];
    if (i >= l0) {
      const int oh = b.stride == 2 ? h / 2 : h;
      if (i == l0) {  // the fused blocks' f32 output -> planes with the layered row stride
        const size_t rows = (size_t)B * h * h, items = rows * (b.lcinp / 4);
        hipLaunchKernelGGL(mbv2_split_pad_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s,
                           reinterpret_cast<const float*>(cur), rows, b.cin, b.lcinp, std::ldexp(1.0f, b.x3_s_in), pin,
                           plo, range_flag());
        MEC_LAUNCH_CHECK();
      }
      f16* pout = pin == P0 ? P1 : P0;
      GemmParams g;  // expand: E = ReLU6(We X 2^-e + be), f32
      g.split = 1; g.A = pin; g.a_lo = plo; g.B = Wt + b.lwe_off; g.b_lo = wlo; g.oscale = lx3_scale[2 * i];
      g.bias = P + b.be_off; g.act = ACT_RELU6; g.C32 = Eb;
      g.M = B * h * h; g.N = b.hidp; g.K = b.lcinp;
      MEC_TRY(launch_gemm(g, s, nullptr, 0));  // inside the TAG_MBV2_BLOCK window
      const size_t items = (size_t)B * oh * (b.hidp / 8);  // one output row of one 8-channel group each
      if (b.stride == 2)
        hipLaunchKernelGGL(mbv2_dw_x3_kernel<2>, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, Eb, h, oh,
                           b.hidp, P + b.wd_off, P + b.bd_off, Db, dlo, items);
      else
        hipLaunchKernelGGL(mbv2_dw_x3_kernel<1>, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, Eb, h, oh,
                           b.hidp, P + b.wd_off, P + b.bd_off, Db, dlo, items);
      MEC_LAUNCH_CHECK();
      g = GemmParams();  // project: Y 2^s = Wp D 2^-e 2^(s - 13) + bp 2^s (+ the block input's planes), hi / lo planes
      g.split = 1; g.A = Db; g.a_lo = dlo; g.B = Wt + b.lwp_off; g.b_lo = wlo; g.oscale = lx3_scale[2 * i + 1];
      g.bias = P + b.lbp_x3_off; g.act = ACT_NONE; g.C16 = pout; g.c_lo = plo;
      if (b.stride == 1 && b.cin == b.cout) {
        g.R = pin;
        g.r_lo = plo;
      }
      g.M = B * oh * oh; g.N = b.lcoutp; g.K = b.hidp;
      MEC_TRY(launch_gemm(g, s, nullptr, 0));  // inside the TAG_MBV2_BLOCK window
      pin = pout;
      h = oh;
      continue;
    }
    MbX3Args a;
    a.x = cur; a.y = out; a.H = h; a.OH = b.stride == 2 ? h / 2 : h;
    a.cin = b.cin; a.cout = b.cout;
    a.We = Wt + b.we_off; a.we_lo = wlo; a.we_scale = x3_scale[2 * i]; a.x_up = std::ldexp(1.0f, b.x3_s_in);
    a.be = P + b.be_off; a.Wd = P + b.wd_off; a.bd = P + b.bd_off;
    a.Wp = Wt + b.wp_off; a.wp_lo = wlo; a.wp_scale = x3_scale[2 * i + 1];
    a.bp = P + b.bp_off;
    a.stem_w = P + (C == 3 ? stem_rgb_off : stem_w_off);
    a.stem_corr = P + stem_corr_off;
    a.flag = range_flag();
    MEC_TRY(dispatch_x3_block(b, a, B, i == 0 ? (C == 3 ? 3 : 1) : 0, s));
    cur = out;
    out = (out == X) ? Y : X;
    h = a.OH;
  }
  MEC_TRY(prof.end(TAG_MBV2_BLOCK, s));
  {  // features[18] 1x1 320 -> 1280 + BN + ReLU6 on the split GEMM engine
    const f16* A = pin;  // the layered tail's planes (320 channels: no padding)
    const long long llo = plo;
    GemmParams g;
    g.split = 1; g.A = A; g.a_lo = llo; g.B = Wt + last_w_off; g.b_lo = wlo; g.oscale = x3_scale.back();
    g.bias = P + last_b_off; g.act = ACT_RELU6; g.C32 = Lst;
    g.M = B * h * h; g.N = 1280; g.K = 320;
    MEC_TRY(launch_gemm(g, s, &prof, TAG_MBV2_LAST));
  }
  hipLaunchKernelGGL(avgpool_f32_kernel, dim3(B, 1280 / 256), dim3(256), 0, s, Lst, h * h, 1280, pooled);
  MEC_LAUNCH_CHECK();
  MEC_TRY(launch_linear_mfma<BACT_RELU>(pooled, 1280, B, 1280, P + fc1_off, P + fc1b_off, 512, feat, 512, nullptr, 0, s));
  MEC_TRY(launch_head7(feat, B, 512, P + fc2_off, P + fc2b_off, logits, probs, s));
  return 0;
}

}  // namespace mec
