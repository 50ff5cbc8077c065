// MobileNetV2's 14x14 and 7x7 stages (features[8..17]: ten inverted-residual blocks) as ONE kernel
// per image (the f16 path, mbv2_tail 1): a workgroup holds the image's whole activation map in LDS
// (14x14x96 f16 at most, 40 KB), walks the ten blocks in order and writes only the last block's
// output (7x7x320) to HBM. The per-block kernels (mobilenet.hip) instead re-stage each block's input
// from HBM with a 3x3 halo per 7x7 tile (a 9x9 expand for 49 outputs at 14x14: 1.65x the expand
// work) and pay a launch, a fill and a drain per block: ten launches of 36-101 us at B = 256 that
// run the matrix cores at 5-8 % (profiles/r04_pmc_report_*). Here:
//   * expand    E[p][h0..h0+31] for every input pixel of the image (no halo recompute) on
//               v_mfma_f32_16x16x32_f16, k over cin in the same order as mbv2_block_kernel
//   * depthwise 3x3/s + BN + ReLU6 in fp32, taps in (kh, kw) order, image-border taps as +0 inputs
//               (exactly the per-block kernels' zero-padded halo)
//   * project   accumulated over the hidden chunks in registers; + BN shift (+ the block input)
// The roundings sit where the per-block kernels put them (E, D and the block output in f16), so the
// outputs are bit-identical to them (tests/test_gpu_mbv2.py::test_mbv2_tail_bit_identical).
#include <algorithm>

#include "models.h"

namespace mec {

constexpr int MT_NB = 10;        // blocks features[8..17] (indices 7..16 of MobileNetModel::blocks)
constexpr int MT_HC = 32;        // hidden channels per chunk
constexpr int MT_ALD_MAX = 20480;  // halfs per activation buffer: max over blocks of pixels x (C + 8)
constexpr int MT_PMAX = 208;     // 14 x 14 = 196 pixels, padded to 13 16-pixel MFMA tiles
constexpr int MT_ELD = MT_HC + 8;
constexpr int MT_ACC = 10;       // project tiles per wave: max over blocks of ceil(OT x PT / 8)

struct MtBlock {
  int H, S, cin, cinp, hidp, cout, coutp, res;
  const f16* We;
  const float* be;
  const float* Wd;
  const float* bd;
  const f16* Wp;
  const float* bp;
};
struct MtArgs {
  const MtBlock* blk;  // [MT_NB] block descriptors in device memory (the handle's mbv2_tail table)
  const f16* x;        // features[7]'s output, NHWC [B,14,14,64]
  f16* y;              // features[17]'s output, NHWC [B,7,7,320]
};

__device__ __forceinline__ float mt_relu6(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

__global__ __launch_bounds__(512, 1) void mbv2_tail_kernel(const MtArgs a) {
  __shared__ __attribute__((aligned(16))) f16 sAct[2][MT_ALD_MAX];
  __shared__ __attribute__((aligned(16))) f16 sE[MT_PMAX * MT_ELD];
  __shared__ __attribute__((aligned(16))) f16 sD[MT_PMAX * MT_ELD];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int n = blockIdx.x;

  // ---- the image's input map (14 x 14 x 64) -> sAct[0], rows of cinp + 8 halfs
  {
    const MtBlock& b0 = a.blk[0];
    const int ld = b0.cinp + 8, c8n = b0.cinp / 8;
    const f16* xin = a.x + (size_t)n * b0.H * b0.H * b0.cin;
    for (int i = tid; i < b0.H * b0.H * c8n; i += 512) {
      const int p = i / c8n, c8 = i - p * c8n;
      half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (c8 * 8 < b0.cin) v = *reinterpret_cast<const half8*>(xin + (size_t)p * b0.cin + c8 * 8);
      *reinterpret_cast<half8*>(&sAct[0][p * ld + c8 * 8]) = v;
    }
  }
  __syncthreads();

  int cur = 0;
#pragma unroll 1
  for (int bi = 0; bi < MT_NB; ++bi) {
    const MtBlock& b = a.blk[bi];
    const int H = b.H, S = b.S, OH = H / S;
    const int NPI = H * H, NPO = OH * OH;
    const int PTI = (NPI + 15) / 16, PTO = (NPO + 15) / 16;
    const int KX = b.cinp / 32, OT = b.coutp / 16;
    const int ildp = b.cinp + 8, oldp = b.coutp + 8;
    const f16* X = sAct[cur];
    f16* Y = sAct[cur ^ 1];
    const int ntile = OT * PTO;

    floatx4 acc[MT_ACC];
#pragma unroll
    for (int j = 0; j < MT_ACC; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int ht = wave & 1, pg = wave >> 1;  // expand: hidden tile, pixel-tile group
#pragma unroll 1
    for (int h0 = 0; h0 < b.hidp; h0 += MT_HC) {
      // ---- expand: E^T[h][p] = sum_c We[h0+h][c] X[p][c] (A = weights, B = X^T), all input pixels
      half8 af[5];
#pragma unroll
      for (int k = 0; k < 5; ++k)
        if (k < KX) af[k] = *reinterpret_cast<const half8*>(b.We + (size_t)(h0 + 16 * ht + l16) * b.cinp + 32 * k + 8 * lq);
      float eb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) eb[e] = b.be[h0 + 16 * ht + 4 * lq + e];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pt = pg + 4 * j;
        if (pt < PTI) {
          const int p = 16 * pt + l16;
          floatx4 e2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 5; ++k)
            if (k < KX) {
              const half8 bf = p < NPI ? *reinterpret_cast<const half8*>(X + p * ildp + 32 * k + 8 * lq)
                                       : half8{0, 0, 0, 0, 0, 0, 0, 0};
              e2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[k], bf, e2, 0, 0, 0);
            }
          half4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = (f16)mt_relu6(e2[e] + eb[e]);
          *reinterpret_cast<half4*>(sE + p * MT_ELD + 16 * ht + 4 * lq) = hv;
        }
      }
      __syncthreads();
      // ---- depthwise 3x3/S + BN + ReLU6 (fp32): item = (output pixel, 8 channels)
      for (int it = tid; it < PTO * 16 * 4; it += 512) {
        const int q = it >> 2, cg = it & 3;
        half8 out = {0, 0, 0, 0, 0, 0, 0, 0};
        if (q < NPO) {
          const int oy = q / OH, ox = q - (q / OH) * OH;
          const int hc = h0 + 8 * cg;
          float d[8];
          {
            const float4 b0 = *reinterpret_cast<const float4*>(b.bd + hc);
            const float4 b1 = *reinterpret_cast<const float4*>(b.bd + hc + 4);
            d[0] = b0.x; d[1] = b0.y; d[2] = b0.z; d[3] = b0.w; d[4] = b1.x; d[5] = b1.y; d[6] = b1.z; d[7] = b1.w;
          }
          const float* wd = b.Wd + (size_t)(hc / 8) * 72;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const int iy = oy * S - 1 + ky, ix = ox * S - 1 + kx;
              const bool in = iy >= 0 && iy < H && ix >= 0 && ix < H;
              // a tap outside the image reads +0 (the per-block kernels' zero-padded halo)
              const half8 ev = in ? *reinterpret_cast<const half8*>(sE + (iy * H + ix) * MT_ELD + 8 * cg)
                                  : half8{0, 0, 0, 0, 0, 0, 0, 0};
              const float4 w0 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8);
              const float4 w1 = *reinterpret_cast<const float4*>(wd + (ky * 3 + kx) * 8 + 4);
              d[0] = __builtin_fmaf((float)ev[0], w0.x, d[0]); d[1] = __builtin_fmaf((float)ev[1], w0.y, d[1]);
              d[2] = __builtin_fmaf((float)ev[2], w0.z, d[2]); d[3] = __builtin_fmaf((float)ev[3], w0.w, d[3]);
              d[4] = __builtin_fmaf((float)ev[4], w1.x, d[4]); d[5] = __builtin_fmaf((float)ev[5], w1.y, d[5]);
              d[6] = __builtin_fmaf((float)ev[6], w1.z, d[6]); d[7] = __builtin_fmaf((float)ev[7], w1.w, d[7]);
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
          for (int j = 0; j < 8; ++j) out[j] = (f16)mt_relu6(d[j]);
        }
        *reinterpret_cast<half8*>(sD + q * MT_ELD + 8 * cg) = out;
      }
      __syncthreads();
      // ---- project: out^T[o][q] += Wp[o][h0..h0+31] . D[q][:]; tile t = (ot, pt), wave-strided
#pragma unroll
      for (int j = 0; j < MT_ACC; ++j) {
        const int t = wave + 8 * j;
        if (t < ntile) {
          const int ot = t / PTO, pt = t - (t / PTO) * PTO;
          const half8 pf = *reinterpret_cast<const half8*>(b.Wp + (size_t)(16 * ot + l16) * b.hidp + h0 + 8 * lq);
          const half8 bf = *reinterpret_cast<const half8*>(sD + (16 * pt + l16) * MT_ELD + 8 * lq);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, bf, acc[j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // one tile's operands live at a time (register budget)
      }
    }
    // ---- epilogue: + BN shift (+ the block input) -> f16 -> the next block's input (the last block: HBM)
    const bool last = bi == MT_NB - 1;
#pragma unroll
    for (int j = 0; j < MT_ACC; ++j) {
      const int t = wave + 8 * j;
      if (t < ntile) {
        const int ot = t / PTO, pt = t - (t / PTO) * PTO;
        const int q = 16 * pt + l16, c = 16 * ot + 4 * lq;
        if (q < NPO && c < b.cout) {
          const float4 bv = *reinterpret_cast<const float4*>(b.bp + c);
          float v[4] = {acc[j][0] + bv.x, acc[j][1] + bv.y, acc[j][2] + bv.z, acc[j][3] + bv.w};
          if (b.res) {
            const half4 r = *reinterpret_cast<const half4*>(X + q * ildp + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
          }
          half4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = (f16)v[e];
          if (last)
            *reinterpret_cast<half4*>(a.y + ((size_t)n * NPO + q) * b.cout + c) = hv;
          else
            *reinterpret_cast<half4*>(Y + q * oldp + c) = hv;
        } else if (!last && q < NPO && c < b.coutp) {
          *reinterpret_cast<half4*>(Y + q * oldp + c) = half4{0, 0, 0, 0};  // padded channels stay zero
        }
      }
    }
    __syncthreads();  // Y complete; every wave is done reading X and sD
    cur ^= 1;
  }
}

// The block table of features[8..17] (device pointers into the handle's weights), built once at
// handle creation into m.tail_tab (MobileNetModel::create)
int build_mbv2_tail_table(MobileNetModel& m) {
  MEC_REQUIRE(m.blocks.size() == 17, "mbv2 tail: 17 blocks expected");
  MtBlock tab[MT_NB];
  const f16* W = m.wts.as<f16>();
  const float* P = m.prm.as<float>();
  int H = 14;
  for (int i = 0; i < MT_NB; ++i) {
    const MbBlock& b = m.blocks[7 + i];
    MtBlock& t = tab[i];
    t.H = H; t.S = b.stride; t.cin = b.cin; t.cinp = b.cinp; t.hidp = b.hidp; t.cout = b.cout; t.coutp = b.coutp;
    t.res = b.stride == 1 && b.cin == b.cout;
    t.We = W + b.we_off; t.be = P + b.be_off; t.Wd = P + b.wd_off; t.bd = P + b.bd_off;
    t.Wp = W + b.wp_off; t.bp = P + b.bp_off;
    MEC_REQUIRE(b.t != 1 && b.cinp <= 160 && b.cinp % 32 == 0 && b.hidp % 32 == 0 && b.coutp % 16 == 0,
                "mbv2 tail: block shape");
    const int OH = H / b.stride;
    MEC_REQUIRE(H * H * (b.cinp + 8) <= MT_ALD_MAX && OH * OH * (b.coutp + 8) <= MT_ALD_MAX &&
                    (b.coutp / 16) * ((OH * OH + 15) / 16) <= 8 * MT_ACC,
                "mbv2 tail: activation / accumulator budget");
    H = OH;
  }
  MEC_REQUIRE(H == 7 && tab[MT_NB - 1].cout == 320, "mbv2 tail: output 7x7x320");
  return upload(m.tail_tab, tab, sizeof(tab));
}

int launch_mbv2_tail(const MobileNetModel& m, const f16* x, f16* y, int B, hipStream_t s) {
  MEC_REQUIRE(m.tail_tab.p, "mbv2 tail: block table missing");
  MtArgs a;
  a.blk = m.tail_tab.as<MtBlock>();
  a.x = x;
  a.y = y;
  hipLaunchKernelGGL(mbv2_tail_kernel, dim3(B), dim3(512), 0, s, a);
  MEC_LAUNCH_CHECK();
  return 0;
}

}  // namespace mec
