/*
 * mec.h — C ABI of libmec_hip.so, the MI355X (gfx950) batched tri-modal emotion
 * inference path. Drop-in boundary for the reference's inference/ classes
 * (RachaCodez/multimodal-emotion-classification); see INTEGRATION.md for the Python
 * (ctypes) binding the reference-side classes use.
 *
 * Conventions
 *   - Every data pointer is a DEVICE pointer owned by the caller; row-major, contiguous.
 *   - Calls are asynchronous on `stream` (a hipStream_t; NULL = default stream).
 *   - Return 0 on success, -1 on failure; mec_last_error() (thread-local) says why.
 *   - A model handle owns its packed device weights and a grow-only workspace; it may be
 *     used by one host thread at a time.
 *   - Host weight blobs are fp32, in the canonical order of mec/synthetic.py:spec(kind),
 *     i.e. the reference's own state_dict / Keras layer order.
 */
#ifndef MEC_H_
#define MEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mec_model mec_model;

enum { MEC_SPEECH = 0, MEC_TEXT = 1, MEC_IMAGE = 2, MEC_FUSION = 3, MEC_IMAGE_MBV2 = 4, MEC_AUDIO = 5 };
/* MEC_IMAGE is the reference's ResNet50 image model (inference/image_inference.py:55-65);
 * MEC_IMAGE_MBV2 the same head on a torchvision mobilenet_v2 backbone (README.md:13 names
 * MobileNetV2; blob = state_dict order of mec/synthetic.py:image_mbv2_spec). Both kinds are
 * accepted by mec_image_fwd / mec_image_fwd_u8. */

/* Version / diagnostics. */
const char* mec_version(void);
const char* mec_last_error(void);

/* Number of fp32 values the host blob for `kind` must hold (-1 if kind is unknown). */
long long mec_blob_size(int kind);

/* Create a model of `kind` on `device` from a host fp32 blob of `n` floats.
 * Replaces the per-request model loads of the reference:
 *   speech  tf.keras.models.load_model + joblib scaler   inference/speech_inference.py:21-28
 *   text    BertForSequenceClassification.from_pretrained inference/text_inference.py:40-43
 *   image   _build_model + load_state_dict               inference/image_inference.py:35-40
 *           (MEC_IMAGE_MBV2: the same with base = mobilenet_v2, base.classifier = the head)
 *   fusion  _build_fusion_model + load_state_dict        inference/multimodal_fusion.py:43-56 */
int mec_create(int kind, const float* host_blob, size_t n, int device, mec_model** out);

/* Arithmetic of a handle. MEC_PREC_F16 (mec_create's default, the fast path): BERT and the
 * image backbones on f16 MFMA operands with fp32 accumulation, LayerNorm, softmax, GELU,
 * residual stream and heads; outside the north_star's 1e-3 / argmax-exact contract margin (text
 * probs within 8.2e-4 of the oracle on the bench batch, rows with a smaller top-2 margin can flip:
 * INTEGRATION.md). MEC_PREC_FP32: every operand and product in fp32
 * (v_mfma_f32_32x32x2_f32, an exact fmaf chain), the precision the reference computes in
 * (inference/text_inference.py:91-93, inference/image_inference.py:116-118).
 * MEC_PREC_FP32X3 (BERT, ResNet50, MobileNetV2): the fp32 path's arithmetic with every GEMM / conv
 * operand carried as a pair of f16 planes (x = hi + lo) and each product as hi.hi + hi.lo + lo.hi
 * on the f16 MFMA into one fp32 accumulator; LayerNorm, softmax, attention, GELU, depthwise convs,
 * residual stream and heads fp32. Envelope: weights are split after a per-matrix power-of-two
 * pre-scale (22 significant bits each); each activation tensor is split at a power-of-two plane
 * scale 2^s fixed at creation (hi = f16(x 2^s), lo = f16(x 2^s - hi); the consumer's epilogue folds
 * in 2^-s, exactly): from rigorous bounds for BERT (LayerNorm outputs and their projections: no
 * plane can overflow) and from the BatchNorm parameters for ResNet50 / MobileNetV2 (64x headroom
 * over a 6-sigma estimate), so the planes hold 22 significant bits for the tensor's whole working
 * range (INTEGRATION.md "fp32x3 envelope"). A plane value at |x 2^s| >= 65520 (activations far above
 * what the BN parameters predict) or a NaN / inf raises the handle's range flag and mec_model_check
 * fails. Speech, fusion and audio handles are fp32 at every setting. */
enum { MEC_PREC_F16 = 0, MEC_PREC_FP32 = 1, MEC_PREC_FP32X3 = 2 };
int mec_create_ex(int kind, const float* host_blob, size_t n, int device, int precision, mec_model** out);
/* mec_create_ex with this handle's own knobs, "key=value[,key=value...]" (the keys of mec_set_option),
 * applied over the process defaults BEFORE the weights are packed; NULL or "" = the defaults. The
 * creation-time knobs live here: "x3_headroom" 0..24 [0] (fp32x3: every activation-plane exponent chosen
 * for 2^-x3_headroom of the default target, i.e. that many binades more room above the bound / BN
 * estimate before the range flag trips; the Python engine re-creates a handle with +8 after a trip, once
 * the batch has been re-run on an MEC_PREC_FP32 handle) and "x3_plane_scale". Same semantics as the
 * reference's model loads (see mec_create). */
int mec_create_opt(int kind, const float* host_blob, size_t n, int device, int precision, const char* opts,
                   mec_model** out);
/* fp32x3 handles: the activation-plane exponents chosen at creation, one line per tensor (group),
 * "name s=<exponent> bound=<rigorous bound or BN estimate>", after a first line with the creation knobs;
 * "" for other precisions, NULL on a null handle. Owned by the handle (valid until mec_destroy). For
 * diagnosing a range-flag failure (mec_model_check returning MEC_ERR_X3_RANGE). */
const char* mec_model_x3_report(mec_model* m);
/* The handle's precision (MEC_PREC_*), -1 on a null handle. */
int mec_precision(const mec_model* m);
int mec_destroy(mec_model* m);

/* Speech DNN. x: raw (pre-scaler) features f32[B,56]. Outputs feat f32[B,64] (block-5
 * ReLU = layers[-3]), logits f32[B,7], probs f32[B,7].
 * Replaces SpeechInference.predict / extract_features model arithmetic
 *   inference/speech_inference.py:66-69, :86-103. */
int mec_speech_fwd(mec_model* m, const float* x, int B, float* feat, float* logits, float* probs,
                   void* stream);

/* BERT-base text encoder + classifier. ids/mask int32[B,L] with L == 128
 * (padding='max_length'). Outputs cls f32[B,768] (last_hidden_state[:,0]), logits,
 * probs f32[B,7]. Replaces TextInference.predict / extract_features model arithmetic
 *   inference/text_inference.py:87-94, :119-128. */
int mec_text_fwd(mec_model* m, const int32_t* ids, const int32_t* mask, int B, int L, float* cls,
                 float* logits, float* probs, void* stream);

/* ResNet50 image encoder + head. gray: u8[B,48,48]; the PIL RGB/resize/ToTensor/Normalize
 * transform runs on the GPU. Outputs feat f32[B,512] (fc[2]), logits, probs f32[B,7].
 * Replaces ImageInference.predict / extract_features (after Image.open)
 *   inference/image_inference.py:112-119, :137-144. */
int mec_image_fwd(mec_model* m, const uint8_t* gray, int B, float* feat, float* logits, float* probs,
                  void* stream);

/* Generic image entry: img u8[B,H,W,C] in one of
 *   (48,48,1)    FER2013 gray, resized on the GPU (same as mec_image_fwd),
 *   (224,224,1)  gray already resized by PIL on the host (any input size),
 *   (224,224,3)  RGB already resized by PIL on the host (colour inputs).
 * Replaces ImageInference.predict for arbitrary image files (image_inference.py:112-113). */
int mec_image_fwd_u8(mec_model* m, const uint8_t* img, int B, int H, int W, int C, float* feat, float* logits,
                     float* probs, void* stream);

/* Attention-MLP fusion. Outputs logits/probs f32[B,7], attn_w/dec_w f32[B,3].
 * Replaces MultimodalFusion.fuse_with_attention  inference/multimodal_fusion.py:201-239. */
int mec_fusion_fwd(mec_model* m, const float* s_feat, const float* t_feat, const float* i_feat,
                   const float* s_pred, const float* t_pred, const float* i_pred, int B, float* logits,
                   float* probs, float* attn_w, float* dec_w, void* stream);

/* Speech features on the GPU (MEC_AUDIO handle; blob = {sample_rate, 2048, 512, 128, n_mfcc},
 * i.e. config.py's SAMPLE_RATE / N_MFCC and librosa's n_fft / hop / n_mels). wave: f32[B, n]
 * fixed-length waveforms (load_audio's pad/trim applied). feat: f32[B, n_mfcc + 16] =
 * [mean MFCC | mean chroma (12) | mean zcr, centroid, rolloff, rms]; tuning: f32[B] (the
 * estimate_tuning value chroma used) or NULL. Replaces preprocess_audio's feature arithmetic
 *   preprocessing/audio_preprocessing.py:22-46 (librosa 0.10.0 mfcc / chroma_stft /
 *   zero_crossing_rate / spectral_centroid / spectral_rolloff / rms). */
int mec_audio_fwd(mec_model* m, const float* wave, int B, int n_samples, float* feat, float* tuning, void* stream);

/* Weighted-average fallback (float64, like numpy); any of s/t/i may be NULL (= zeros).
 * Replaces MultimodalFusion.fuse_predictions  inference/multimodal_fusion.py:184-199. */
int mec_fuse_weighted(const float* s_probs, const float* t_probs, const float* i_probs, int B,
                      double* out, void* stream);

/* Same with float64 inputs (per-request dicts carry Python floats, e.g. heuristic 0.1/6). */
int mec_fuse_weighted_f64(const double* s_probs, const double* t_probs, const double* i_probs, int B,
                          double* out, void* stream);

/* Kernel-level entry points (parity tests / microbenchmarks). */
int mec_resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, void* stream);
/* C[M,N] = act(A[M,K] . B[N,K]^T + bias (+ R)); f16 operands, fp32 accumulate.
 * act: 0 none, 1 relu, 2 gelu(erf). Any of bias/R/C16/C32 may be NULL (not both outputs). */
/* Split-f16 GEMM (the MEC_PREC_FP32X3 engine): A and B each an f16 hi plane with its lo plane
 * a_lo / b_lo elements further on (x = hi + lo); C = act((A_lo.B_hi + A_hi.B_lo + A_hi.B_hi) *
 * oscale + bias (+ R f32)); C16 (hi plane, lo plane at C16 + c_lo when c_lo != 0) and/or C32.
 * act: 0 none, 1 relu, 4 exact-erf GELU. */
int mec_gemm_f16x3(const void* A, long long a_lo, const void* B, long long b_lo, float oscale, const float* bias,
                   const float* R, void* C16, long long c_lo, float* C32, int M, int N, int K, int act,
                   void* stream);
int mec_gemm_f16(const void* A, const void* B, const float* bias, const void* R, int r_is_f32, void* C16,
                 float* C32, int M, int N, int K, int act, void* stream);
/* Implicit-GEMM conv on NHWC f16: x[n,H,W,C], w[Cout][ks][ks][C], y[n,OH,OW,Cout]. */
int mec_conv_f16(const void* x, const void* w, const float* bias, const void* R, void* y, int n, int H, int W,
                 int C, int Cout, int ks, int stride, int pad, int act, void* stream);
/* fp32 engine (the MEC_PREC_FP32 path): C[M,N] = act(A[M,K] . B[N,K]^T + bias (+ R)), all f32;
 * K % 32 == 0, N % 64 == 0; act 0 none, 1 relu, 4 gelu (libm erf). */
int mec_gemm_f32(const float* A, const float* B, const float* bias, const float* R, float* C, int M, int N, int K,
                 int act, void* stream);
/* Implicit-GEMM conv on NHWC f32 (C % 32 == 0), same geometry as mec_conv_f16. */
int mec_conv_f32(const float* x, const float* w, const float* bias, const float* R, float* y, int n, int H, int W,
                 int C, int Cout, int ks, int stride, int pad, int act, void* stream);

/* Tuning knobs (A/B benchmarking; defaults in brackets). Every handle owns its own copy of
 * the knobs and its own GEMM autotune cache, so two handles in one process never perturb
 * each other: mec_model_set_option sets one handle's knob; mec_set_option sets the process
 * default that handles created AFTERWARDS copy (and that the handle-less kernel entry points
 * use). Every pair of settings of one knob gives bit-identical outputs, except "fusion_r" 4 vs
 * 1|2, "conv3x3_halo" 0 vs 1, "gemm_x3_order" 0 vs 1 and "gelu_x3" 0 vs 1 (fp32 reassociation or
 * erf evaluation, all within the oracle tolerance).
 *   "gemm_bn" [0]|id       force one f16 GEMM tile (0 = autotune), "gemm_autotune" 0|[1]
 *   "gemm_bn_tag" tag*100000+id   force a tile for one launch class (e.g. 3 = BERT O-proj)
 *   "gemm_f32_tile" [0]|1..8  force one fp32 GEMM tile (0 = autotune; 5..8 = 1..4 on 16x16x4)
 *   "gemm_f32_tag" tag*100000+id  pin an fp32 tile for one launch class (default: BERT FFN1 -> 8)
 *   "gemm_f32_family" 0|[16]|32  fp32 tiles of one MFMA shape only (16x16x4 / 32x32x2): one k order
 *                          for every shape, so rows do not depend on the batch size
 *   "gemm_prefetch_r" 0|[1]  f16 (and split hi / lo) residual prefetch in short-K GEMMs
 *   "gemm_group_m" 0|2|4|[8]|16  ping-pong GEMM tile order inside each XCD's tile range (0: row-major,
 *                          G: G-panel groups of M walked M-fastest, fewer weight re-fetches)
 *   "gemm_glds_group_m" 0|2|4|[8]|16  the same tile order for the multi-stage GEMM engine
 *   "gemm_x3_order" 0|[1]  split-f16 (fp32x3) GEMM term order: 0 = pass-major (K for lo.hi, then
 *                          hi.lo, then hi.hi), 1 = K-interleaved (each 32-deep k chunk's three terms
 *                          back to back, 16x16x32 tiles 70256 / 70128 / 71128 / 71064 / 70064 / 72128 only);
 *                          both fp32-accurate, not the same bits
 *   "gemm_x3_tag" tag*100000+id  pin an interleaved split tile (7xxxx; 0 = autotune) for one launch
 *                          class (FusedPipeline pins BERT FFN2 to 70256 at fp32x3); a pin applies where
 *                          its grid has >= 128 tiles (half the CUs), smaller batches autotune (same bits)
 *   GEMM shapes first launched inside hipGraph capture cannot be timed: split (fp32x3) shapes run
 *   the heuristic tile uncached and are autotuned at their first eager launch (every split tile
 *   gives the same bits); f16 / f32 shapes cache the heuristic tile for the handle's lifetime, so
 *   an eager launch after the capture computes the same bits as the graph replay (tiles of those
 *   engines differ in MFMA shape and k order)
 *   "gelu_x3" 0|[1]        fp32x3 BERT FFN1 GELU: 1 = branch-free erf with a one-instruction exp
 *                          (error 1.21e-7 x max(|x|, 1) vs float64), 0 = libm erff (not the same bits)
 *   "conv3x3_direct" 0|[1] layer1 3x3 conv on the halo-tile kernel (mec_conv_f16 too)
 *   "conv3x3_halo" 0|[1]   layers 2-3 stride-1 3x3 convs on the halo kernel (mec_conv_f16 too;
 *                          fp32 accumulation in another order: not bit-identical to 0)
 *   "pw_chain" 0|1|[2]     layer1 seam kernels (1: the 256->64 seams, 2: also 256->128)
 *   "pw_chain_form" [0]|1|2  seam weight placement (LDS / registers)
 *   "pw_chain_x3" 0|1|[2]  fp32x3 layer1 seam kernels (1: the 256->64 seams incl. the downsample one, 2: also 256->128)
 *   "pw_seam_x3" 0|[1]|2  fp32x3 layer2 seam kernels (1: the 512->128 seams, 2: also 512->256 into layer3; same bits)
 *   "bert_qkv_attn_x3_heads" [1]|2  fp32x3 fused QKV + attention: heads per workgroup (same bits)
 *   "bert_qkv_attn_heads" [1]|2  the same for the f16 fused QKV + attention
 *   "bert_qkv_attn" 0|[1]  fused BERT QKV projection + attention
 *   "bert_ln_rows" 1|[2]|4  BERT LayerNorm rows per wave (all loads of a wave's rows in flight first)
 *   "bert_cls_last" 0|[1]  BERT's last layer on the [CLS] rows only (K / V still for every token):
 *                          the pooler, logits and CLS feature read nothing else of it; same bits as 0
 *   "resnet_chunk" [0]|n   ResNet layers 1-2 over n-image chunks (f16 and fp32x3; measured slower)
 *   "mbv2_x3_tile" 0|[4]   fp32x3 MobileNetV2: 4x4 output tiles for the stride-2 blocks at 56 / 28 outputs
 *   "mbv2_x3_tpw" 1|[2]..16 fp32x3 MobileNetV2 fused blocks: output tiles per workgroup, the next tile's
 *                          input loaded into registers while one computes (same bits for every value)
 *   "mbv2_x3_occ" [3]|4    fp32x3 MobileNetV2 4x4-tile blocks: workgroups per CU the registers are
 *                          allocated for (4: 128 VGPRs with an 84-B spill, 3: 168 VGPRs); same bits
 *   "mbv2_x3_sesw" 0|[1]   fp32x3 MobileNetV2 fused blocks: the expanded chunk's rows chunk-swizzled per tile
 *                          shape (fewer LDS bank conflicts on the depthwise reads) or unswizzled; same bits
 *   "gemm_x3_restage" [0]|1|2 K-interleaved split tiles with 2 stages: refill a stage for k step t + 2 once
 *                          every wave holds step t's fragments (two steps in flight) in every A mode (1), in the
 *                          convs only (2), or never (0: after step t's barrier); same bits
 *   "gemm_x3_late_dma" 0|[1]|2|3  interleaved split tiles: the second wave of each SIMD issues its share of the
 *                          next stage's LDS DMA after its first MFMA term group (1), its second (2), hi planes
 *                          after the first and lo after the second (3), or right after the barrier with the
 *                          first wave (0); same bits (1: fused fp32x3 step -1.2 to -1.6 %)
 *   "gemm_x3_prio" [0]|1   the same tiles: MFMA sections at wave priority 1 (measured neutral); same bits
 *   "qkv_x3_late_dma" [0]|1|2  fp32x3 fused QKV + attention: every other 256-block of workgroups issues its
 *                          stage refill after its first / second MFMA term group (measured neutral); same bits
 *   "gemm_x3_stagger" [0]..200  split tiles with two workgroups per CU: the first pass's second workgroups start
 *                          this many microseconds late (co-resident epilogues and MFMAs desynchronized;
 *                          measured neutral-to-slower on BERT FFN1); same bits
 *   "x3_plane_scale" 0|[1] fp32x3 activation-plane scales, creation-time (mec_create_opt, or the process
 *                          default before mec_create_ex; mec_model_set_option rejects it): 1 = per-tensor
 *                          power-of-two exponents (the envelope above), 0 = unscaled planes (A/B only:
 *                          narrower envelope, different bits)
 *   "x3_headroom" [0]..24  fp32x3 extra binades of plane headroom, creation-time like x3_plane_scale
 *                          (mec_create_opt above)
 *   "mbv2_layered" 0|7..17 [8]  fp32x3 MobileNetV2: features[k..17] as expand GEMM -> depthwise -> project GEMM
 *                          (0: every block fused but features[17], layered at every setting)
 *   "mbv2_layered16" 0|7..17 [8]  the same on the f16 path
 *   "mbv2_impl" [0]|1|2    MobileNetV2 block form: 0 = time both per block shape, 1 = workgroup, 2 = wave
 *   "fusion_r" 1|2|[4]     samples per fusion workgroup
 *   "fusion_split" 0|[1]   fusion as 3 launches (per-modality projection, cross-attention, head)
 * Probe values, which skip work to time a kernel's parts and return WRONG results, exist only
 * in the -DMEC_PROBES build (libmec_hip_probes.so, `make probes`; tools/ only): "gemm_debug"
 * 1..5, "conv3x3_debug" / "stem_debug" 1|2|4|7, "bert_qkv_attn" 2|3,
 * "audio_debug" 1|2|4|8|15, "speech_debug" 1, "speech_spin_limit" >= 0 (the speech DNN's
 * hand-off wait limit: forces expired waits). The product library rejects them (-1). */
int mec_set_option(const char* key, int value);
int mec_model_set_option(mec_model* m, const char* key, int value);

/* Build flags of the loaded library: MEC_BUILD_PROBES set = probe values accepted. */
enum { MEC_BUILD_PROBES = 1 };
int mec_build_flags(void);

/* Tile width the autotuner chose for a plain (amode 0) or conv (amode 1) GEMM shape; 0 = not yet seen. */
int mec_gemm_query(int amode, int M, int N, int K);
/* The same for the fp32 engine: tile id 1 = 256x128 (8 waves), 2 = 128x128, 3 = 128x64, 4 = 256x256
 * on v_mfma_f32_32x32x2_f32; 5..8 the same tiles on v_mfma_f32_16x16x4_f32.
 * Both query the process-default cache of the handle-less entry points (mec_gemm_f16/f32). */
int mec_gemm_f32_query(int amode, int M, int N, int K);
/* The tile a handle's own autotuner chose for a shape it ran (its precision's engine); 0 = not seen. */
int mec_model_gemm_query(mec_model* m, int amode, int M, int N, int K);

/* Errors a kernel can only report after the fact, since the handle's last check: 0 = none,
 * -1 = mec_last_error() says what (and the flag is cleared); MEC_ERR_X3_RANGE (-2) = the fp32x3
 * range flag below (the batch can be re-run on an MEC_PREC_FP32 handle of the same weights). Call once the stream that ran
 * the handle's forwards has been synchronized. Speech: a stage hand-off wait of
 * speech_flow_kernel expired (that forward's probs are NaN). MEC_PREC_FP32X3 text / image
 * handles: an activation left the f16 hi / lo range (|x| >= 65520, NaN or inf; that forward's
 * outputs are invalid). Always 0 for the other kinds and precisions. No reference counterpart:
 * the reference's predict calls have no asynchronous failure (inference/speech_inference.py:69). */
enum { MEC_ERR_X3_RANGE = -2 };
int mec_model_check(mec_model* m);

/* hipEvent timing hook: time every launch of kernel class `tag`. */
int mec_prof_enable(mec_model* m, int tag);
int mec_prof_read(mec_model* m, double* total_ms, int* count);

#ifdef __cplusplus
}
#endif

#endif /* MEC_H_ */
