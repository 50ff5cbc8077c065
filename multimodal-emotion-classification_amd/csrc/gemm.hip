// f16-operand / fp32-accumulate GEMM dispatch for gfx950: routes each GEMM / implicit-GEMM
// conv to the halo-tile 3x3 conv kernels (conv3x3.hip, conv3x3_halo.hip) where they apply, else
// to the glds pipelined engine (gemm_glds.hip). A-operand views:
//   A_PLAIN  A[M,K] row-major (BERT projections/FFN, ResNet 1x1 stride-1 convs)
//   A_CONV   implicit im2col of an NHWC f16 tensor (ResNet 3x3 convs, strided 1x1
//            downsample convs); K ordered (kh, kw, c), C % 64 == 0 so a 64-deep K tile
//            never straddles two filter taps
//   A_DUAL   [A | A2] concatenated along K (a bottleneck's conv3 + its downsample)
// B is the weight matrix [N,K] (K contiguous = torch Linear layout).
#include "mec_common.h"

namespace mec {

constexpr int GBK = 64;

// Per launch class (profiling tag): forced tile id, 0 = autotune. The BERT O-projection
// (32768 x 768 x 768, f32 deferred-LN residual) is pinned to 128 x 128: its candidates time
// within 2% of each other alone, so the isolated autotune flips between them run to run, but
// inside the encoder 128 x 128 is the fastest (text 8.22 ms vs 8.43 with 256 x 128 / 4 waves;
// fused step 11.40 vs 11.48 ms).

int launch_gemm(const GemmParams& p0, hipStream_t s, Prof* prof, int tag) {
  GemmParams p = p0;
  if (p.c_lo && !p.ovf) p.ovf = range_flag();  // split output: the calling handle's range flag
  MEC_REQUIRE(p.M > 0 && p.N > 0 && p.K > 0, "gemm: empty shape");
  MEC_REQUIRE(p.N % 64 == 0, "gemm: N % 64 != 0");
  MEC_REQUIRE(p.K % GBK == 0, "gemm: K % 64 != 0");
  MEC_REQUIRE(p.A && p.B, "gemm: null operand");
  MEC_REQUIRE(p.C16 || p.C32, "gemm: no output");
  MEC_REQUIRE(!p.r_stats || (p.R && p.r_f32 && p.r_g && p.r_b), "gemm: deferred-LN residual needs f32 R, gamma, beta");
  if (p.amode == A_CONV) {
    MEC_REQUIRE(p.C % 64 == 0 && p.K == p.ks * p.ks * p.C, "conv: C % 64 != 0 or K != ks*ks*C");
  } else if (p.amode == A_DUAL) {
    MEC_REQUIRE(p.A2 && p.K1 > 0 && p.K1 % 64 == 0 && p.C % 64 == 0 && p.K == p.K1 + p.C && p.ks == 1 && p.pad == 0,
                "dual gemm: need K = K1 + C, K1 % 64 == 0, C % 64 == 0, 1x1 unpadded second source");
  } else {
    MEC_REQUIRE(p.amode == A_PLAIN, "gemm: unknown A mode");
  }
  if (prof) MEC_TRY(prof->begin(tag, s));
  int rc;
  if (p.split) {  // split-f16 operands: the glds engine only (the halo conv kernels read one plane); autotuned,
    // except the launch classes gemm_x3_tag pins (BERT FFN1 -> 70256 by default, mec_common.h) where the
    // pinned tile's grid fills half the chip; the pass-major order pins FFN1 to 10256 (it and the ping-pong
    // tile time within 3-7 %, tools/bench_split.py)
    int pin = (tag > 0 && tag < TAG_COUNT) ? opt().gemm_x3_tag[tag] : 0;
    if (pin) {
      const int bm = (pin / 1000) % 10 == 1 ? 128 : 256, bn = pin % 1000;
      // the one-stage 72128 tile pays off only with two workgroups on every CU (BERT B = 256: 768 tiles); at
      // B = 128 (384 tiles, BASELINE configs[2]) it ran the text encoder at 8.81 ms against 8.45 autotuned
      // (profiles/r06s_ab_ffn2pin_text_b128.txt)
      const long min_tiles = pin == 72128 ? 2 * 256 : kX3PinMinTiles;
      if ((long)((p.M + bm - 1) / bm) * (p.N / bn) < min_tiles) pin = 0;  // small batch: autotune (same bits)
    }
    rc = launch_gemm_glds(p, s, opt().gemm_bn ? opt().gemm_bn
                                : !opt().gemm_x3_order ? (tag == TAG_BERT_FFN1 ? 10256 : 0)
                                : pin);
  } else if (opt().conv3x3_direct && !opt().gemm_bn && p.amode == A_CONV && p.ks == 3 && p.stride == 1 && p.pad == 1 && p.H == 56 &&
      p.W == 56 && p.C == 64 && p.N == 64 && p.act == ACT_RELU && !p.R && p.C16 && !p.C32 && p.M % (56 * 56) == 0)
    rc = launch_conv3x3_c64(reinterpret_cast<const f16*>(p.A), p.B, p.bias, p.C16, p.M / (56 * 56), 56, 64, 64, s);
  else if (opt().conv3x3_halo && !opt().gemm_bn && p.amode == A_CONV && p.ks == 3 && p.stride == 1 && p.pad == 1 &&
           p.H == p.W && p.OH == p.H && p.OW == p.W && conv3x3_halo_supported(p.H, p.C, p.N) && p.act == ACT_RELU &&
           !p.R && p.bias && p.C16 && !p.C32 && p.M % (p.H * p.W) == 0)
    rc = launch_conv3x3_halo(reinterpret_cast<const f16*>(p.A), p.B, p.bias, p.C16, p.M / (p.H * p.W), p.H, p.C, s);
  else
    rc = launch_gemm_glds(p, s, opt().gemm_bn ? opt().gemm_bn : (tag > 0 && tag < TAG_COUNT ? opt().gemm_bn_tag[tag] : 0));
  if (rc) return rc;
  if (prof) MEC_TRY(prof->end(tag, s));
  return 0;
}

}  // namespace mec
