// 56-d speech features on the GPU: preprocessing/audio_preprocessing.py:12-46 (the
// reference's librosa==0.10.0 calls, requirements.txt:10) for a batch of fixed-length
// waveforms (load_audio's pad/trim already applied; decoding is host I/O):
//   [ mean_t MFCC_40 | mean_t chroma_12 | mean zcr, centroid, rolloff, rms ]
//
// audio_frame_kernel — one workgroup per (frame, clip), 130 frames x B:
//   * the frame's 2048 samples (center=True: zero padding for the STFT and rms, edge padding
//     for zero_crossing_rate);
//   * rms (float32) and the zero-crossing count (sign bits, |y| <= 1e-10 -> 0);
//   * the STFT column in float64 like librosa (float64 periodic Hann x frame, then a float64
//     FFT: the 2048 real samples packed as 1024 complex, radix-2 in LDS, then split), rounded
//     to complex64 as librosa stores it; |X| as glibc's hypotf, power = |X|^2 in float32;
//   * from the column: the 128 Slaney mel bands (sparse triangles) -> 10 log10(max(1e-10, .)),
//     the spectral centroid (float64 sums over the float32 L1-normalised magnitudes), the
//     85% rolloff (numpy's sequential float32 cumsum, one lane), and piptrack's peak list
//     (freq-masked local maxima of S * (S > 0.1 max S), parabolic shift, float32 like numpy);
//   * writes the power column (for chroma), the mel-dB column, 4 per-frame scalars and the
//     peak list.
// audio_clip_kernel — one workgroup per clip:
//   * MFCC: top_db clamp against the clip's max, mean over frames, DCT-II ortho (float64);
//   * estimate_tuning: median peak magnitude (radix select on order-preserving keys), the
//     residual histogram of the surviving peaks on numpy's 101 float64 edges, argmax;
//   * chroma: the filterbank of that tuning (host-built table of the 100 possible ones),
//     per-frame max normalisation, mean;
//   * the spectral means; one 56-float row.
// HBM-/latency-bound small kernels (no MFMA): the filterbanks are sparse (mel) or small
// (12 x 1025 chroma); DESIGN.md §4 gives the bytes per clip.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "block_ops.h"
#include "models.h"

namespace mec {

namespace {
constexpr double kPi = 3.14159265358979323846;
constexpr int A_NFFT = 2048, A_HOP = 512, A_NBIN = 1025, A_NMEL = 128, A_NCHROMA = 12, A_NTUNE = 100;
constexpr int A_CMAX = 184;  // peaks per frame: local maxima of 358 band bins are <= 179
constexpr int A_BAND_LO = 1, A_BAND_HI = 1024;  // bins that may hold a peak (mask applied too)
constexpr int A_TMAX = 4096;   // frames per clip (95 s at 22050 Hz)
constexpr int A_NLDS = 24576;  // peak magnitudes kept in LDS for the median (more: read from HBM)
static_assert(A_NCHROMA * A_NBIN <= A_NLDS, "the chroma filterbank reuses the peak buffer");
constexpr int A_MSEG = 1024;   // mel segments (band x thread-chunk runs)
}  // namespace

struct AudioTables {
  const double* hann;     // [2048] float64 periodic Hann
  const double2* tw;      // [512] exp(-2 pi i j / 1024)
  const double2* post;    // [1025] exp(-2 pi i k / 2048)
  const double* freq;     // [1025] fft_frequencies
  const int* mel_bin;     // nonzero bins of the mel triangles, band-major
  const float* mel_w;     // their float32 weights (librosa's float32 filterbank)
  const int* mel_seg;     // per nonzero: segment = run of one band inside one thread's chunk
  const int* mel_segoff;  // [129] first segment of each band
  int mel_nnz, mel_ch;    // nonzeros, nonzeros per thread (mel_ch * 256 >= mel_nnz)
  const double* dct;      // [n_mfcc][128] DCT-II ortho
  const float* chroma;    // [100][12][1025] float32 filterbanks, one per tuning bin
  int lo_bin, hi_bin;     // piptrack freq mask [lo, hi): 150 <= f < 4000
  int n_mfcc;
  double sr;              // sample rate (piptrack's pitch = (bin + shift) * sr / n_fft)
};

__device__ __forceinline__ int bitrev10(int x) { return (int)(__builtin_bitreverse32((unsigned)x) >> 22); }

template <typename T>
__device__ __forceinline__ T block_reduce_sum(T v, T* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  T s = 0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// Exact-rounding helpers: librosa's float32 expressions evaluated without FMA contraction.
#pragma clang fp contract(off)

// DBG (probe builds only, option "audio_debug"; wrong results): bit 1 skips the FFT stages,
// 2 the rolloff cumsum, 4 the mel sums and the peak search, 8 the spectrum split
template <int DBG = 0>
__global__ __launch_bounds__(256) void audio_frame_kernel(const float* __restrict__ wave, int L, int T,
                                                          AudioTables tb, float* __restrict__ pow_out,
                                                          float* __restrict__ meldb_out, double* __restrict__ scal,
                                                          float2* __restrict__ cand, int* __restrict__ ccount) {
  __shared__ double2 z[1024];
  __shared__ double2 stw[512];  // FFT twiddles, loaded once per workgroup
  __shared__ __attribute__((aligned(16))) float smag[A_NBIN + 3];
  __shared__ __attribute__((aligned(16))) float spow[A_NBIN + 3];
  __shared__ double redd[4];
  __shared__ float redf[4];
  __shared__ int redi[4];
  __shared__ int sb_last[256];
  __shared__ int ncand;
  __shared__ float mpart[A_MSEG];
  const int tid = threadIdx.x;
  const int t = blockIdx.x, b = blockIdx.y;
  const float* y = wave + (size_t)b * L;
  const size_t fr = (size_t)b * T + t;

  stw[tid] = tb.tw[tid];
  stw[tid + 256] = tb.tw[tid + 256];
  // ---- samples n = 8 tid .. 8 tid + 7 of frame t (padded offset t * hop)
  float vz[8], ve[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int j = t * A_HOP + 8 * tid + i - A_NFFT / 2;
    const int jc = min(max(j, 0), L - 1);
    ve[i] = y[jc];
    vz[i] = (j >= 0 && j < L) ? ve[i] : 0.f;
  }
  // rms: mean of squares over the zero-padded frame, float32
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) sq += vz[i] * vz[i];
  const float sumsq = block_reduce_sum<float>(sq, redf);
  // zero crossings of the edge-padded frame: sign bits after |y| <= 1e-10 -> 0, pad=False
  int sbit[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float v = fabsf(ve[i]) <= 1e-10f ? 0.f : ve[i];
    sbit[i] = (int)(__float_as_uint(v) >> 31);
  }
  sb_last[tid] = sbit[7];
  int cross = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i) cross += sbit[i] != sbit[i - 1];
  __syncthreads();
  if (tid > 0) cross += sbit[0] != sb_last[tid - 1];
  const int ncross = block_reduce_sum<int>(cross, redi);

  // ---- float64 windowed frame packed as 1024 complex, bit-reversed into LDS
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = 4 * tid + i;
    double2 v;
    v.x = tb.hann[2 * m] * (double)vz[2 * i];
    v.y = tb.hann[2 * m + 1] * (double)vz[2 * i + 1];
    z[bitrev10(m)] = v;
  }
  __syncthreads();
  // radix-2 DIT, 10 stages, 512 butterflies per stage (2 per thread)
  for (int s = 0; s < ((DBG & 1) ? 0 : 10); ++s) {
    const int half = 1 << s;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + 256 * r;
      const int j = i & (half - 1);
      const int i0 = ((i >> s) << (s + 1)) + j, i1 = i0 + half;
      const double2 w = stw[j << (9 - s)];
      const double2 a = z[i0], c = z[i1];
      const double2 tt = make_double2(w.x * c.x - w.y * c.y, w.x * c.y + w.y * c.x);
      z[i0] = make_double2(a.x + tt.x, a.y + tt.y);
      z[i1] = make_double2(a.x - tt.x, a.y - tt.y);
    }
    __syncthreads();
  }
  // ---- split into the 2048-point real spectrum, complex64 -> |X| (hypotf) and |X|^2 (float32)
  for (int k = tid; k < ((DBG & 8) ? 0 : A_NBIN); k += 256) {
    const double2 zk = z[k & 1023], zn = z[(1024 - k) & 1023];
    const double er = 0.5 * (zk.x + zn.x), ei = 0.5 * (zk.y - zn.y);   // E = (Z[k] + conj Z[N-k]) / 2
    const double orr = 0.5 * (zk.y + zn.y), oi = -0.5 * (zk.x - zn.x);  // O = (Z[k] - conj Z[N-k]) / 2i
    const double2 w = tb.post[k];
    const float xr = (float)(er + (w.x * orr - w.y * oi));
    const float xi = (float)(ei + (w.x * oi + w.y * orr));
    const float mg = (float)sqrt((double)xr * (double)xr + (double)xi * (double)xi);
    smag[k] = mg;
    const float pw = mg * mg;
    spow[k] = pw;
    pow_out[fr * A_NBIN + k] = pw;
  }
  if (tid == 0) ncand = 0;
  __syncthreads();

  // ---- frame max of the power column (piptrack's ref = 0.1 * max)
  float mx = 0.f;
  for (int k = tid; k < A_NBIN; k += 256) mx = fmaxf(mx, spow[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) redf[tid >> 6] = mx;
  // ---- L1 length of the magnitude column (float64)
  double l1 = 0.0;
  for (int k = tid; k < A_NBIN; k += 256) l1 += (double)smag[k];
  __syncthreads();
  const float fmax_pow = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
  double length = block_reduce_sum<double>(l1, redd);
  if (length < (double)FLT_MIN) length = 1.0;
  double cen = 0.0;
  for (int k = tid; k < A_NBIN; k += 256) cen += tb.freq[k] * (double)(float)((double)smag[k] / length);
  const double centroid = block_reduce_sum<double>(cen, redd);

  // ---- mel bands (sparse Slaney triangles): each thread sums its chunk of the band-major
  // nonzeros into per-segment partials, then each band adds its segments in order (fixed
  // summation order: deterministic); power_to_db before the clip-level top_db clamp
  {
    const int e0 = tid * tb.mel_ch, e1 = (DBG & 4) ? e0 : min(e0 + tb.mel_ch, tb.mel_nnz);
    if (e0 < e1) {
      float acc = 0.f;
      int seg = tb.mel_seg[e0];
      for (int e = e0; e < e1; ++e) {
        const int sg = tb.mel_seg[e];
        if (sg != seg) {
          mpart[seg] = acc;
          acc = 0.f;
          seg = sg;
        }
        acc += tb.mel_w[e] * spow[tb.mel_bin[e]];
      }
      mpart[seg] = acc;
    }
  }
  __syncthreads();
  if (tid < A_NMEL) {
    float acc = 0.f;
    for (int g = tb.mel_segoff[tid]; g < tb.mel_segoff[tid + 1]; ++g) acc += mpart[g];
    meldb_out[fr * A_NMEL + tid] = 10.0f * log10f(fmaxf(1e-10f, acc));
  }
  // ---- piptrack peaks in the band: S * (S > ref) local maxima, parabolic shift (float32)
  const float ref = 0.1f * fmax_pow;
  for (int k = tb.lo_bin + tid; k < ((DBG & 4) ? 0 : tb.hi_bin); k += 256) {
    const float s0 = spow[k - 1], s1 = spow[k], s2 = spow[k + 1];
    const float x0 = s0 > ref ? s0 : 0.f, x1 = s1 > ref ? s1 : 0.f, x2 = s2 > ref ? s2 : 0.f;
    if (x1 > x0 && x1 >= x2) {
      const float a = (s2 + s0) - 2.f * s1;
      const float bb = (s2 - s0) / 2.f;
      const float shift = fabsf(bb) >= fabsf(a) ? 0.f : -bb / a;
      const float dskew = (0.5f * bb) * shift;  // 0.5 * np.gradient * shift
      const float pitch = (float)((((double)k + (double)shift) * tb.sr) / (double)A_NFFT);
      const int slot = atomicAdd(&ncand, 1);
      if (slot < A_CMAX) cand[fr * A_CMAX + slot] = make_float2(pitch, s1 + dskew);
    }
  }
  // ---- spectral rolloff: numpy's sequential float32 cumsum, one lane; first bin >= 0.85 total
  __syncthreads();
  if (tid == 0 && !(DBG & 2)) {  // the power column is no longer needed: spow receives the cumsum
    float c = 0.f;
    for (int k4 = 0; k4 < A_NBIN / 4; ++k4) {
      const float4 m = *reinterpret_cast<const float4*>(smag + 4 * k4);
      float4 o;
      c += m.x; o.x = c;
      c += m.y; o.y = c;
      c += m.z; o.z = c;
      c += m.w; o.w = c;
      *reinterpret_cast<float4*>(spow + 4 * k4) = o;
    }
    c += smag[A_NBIN - 1];
    spow[A_NBIN - 1] = c;
  }
  __syncthreads();
  const float thr = 0.85f * spow[A_NBIN - 1];
  int first = A_NBIN;
  for (int k = tid; k < A_NBIN; k += 256)
    if (spow[k] >= thr) first = min(first, k);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
  if ((tid & 63) == 0) redi[tid >> 6] = first;
  __syncthreads();
  if (tid == 0) {
    const int kf = min(min(redi[0], redi[1]), min(redi[2], redi[3]));
    double* sc = scal + fr * 4;
    sc[0] = (double)ncross / (double)A_NFFT;
    sc[1] = centroid;
    sc[2] = tb.freq[min(kf, A_NBIN - 1)];
    sc[3] = (double)sqrtf(sumsq / (float)A_NFFT);
    ccount[fr] = min(ncand, A_CMAX);
  }
}

// order-preserving uint key of a float (ascending)
__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// rank-r smallest of the clip's n peak magnitudes (radix select on order-preserving keys, 4
// passes of 8 bits; hist holds 256 x (1 + waves) ints: per-wave histograms, then their sum). The magnitudes come from LDS (smag) when the clip's peaks fit there,
// else straight from the per-frame peak lists (soff = per-frame prefix offsets).
__device__ unsigned radix_select(const float* smag, int n, const float2* cd, const int* soff, int T, unsigned r,
                                 int* hist, unsigned* sh) {
  unsigned prefix = 0, pmask = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int* wh = hist + 256 * (1 + wave);  // this wave's own histogram: 8x less same-address contention
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = threadIdx.x; i < 256 * (1 + nw); i += blockDim.x) hist[i] = 0;
    __syncthreads();
    if (smag) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned k = fkey(smag[i]);
        if ((k & pmask) == prefix) atomicAdd(&wh[(k >> shift) & 255], 1);
      }
    } else {
      for (int t = wave; t < T; t += nw) {
        const int cnt = soff[t + 1] - soff[t];
        for (int i = lane; i < cnt; i += 64) {
          const unsigned k = fkey(cd[(size_t)t * A_CMAX + i].y);
          if ((k & pmask) == prefix) atomicAdd(&wh[(k >> shift) & 255], 1);
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
      int s = 0;
      for (int w = 0; w < nw; ++w) s += hist[256 * (1 + w) + i];
      hist[i] = s;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // first bin d < 255 whose inclusive count exceeds r (else 255): one wave,
      // 4 bins per lane, a lane prefix sum, the lowest qualifying lane by ballot
      const int l = threadIdx.x;
      const unsigned h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
      const unsigned tot = h0 + h1 + h2 + h3;
      unsigned inc = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(inc, o, 64);
        if (l >= o) inc += v;
      }
      const unsigned c0 = inc - tot, c1 = c0 + h0, c2 = c1 + h1, c3 = c2 + h2;  // counts before bins 4l+j
      const int dj = c1 > r ? 0 : c2 > r ? 1 : c3 > r ? 2 : (c3 + h3 > r && l < 63) ? 3 : -1;
      const unsigned long long bal = __ballot(dj >= 0);
      const int src = bal ? __ffsll((long long)bal) - 1 : 63;
      if (l == src) {
        const int d = bal ? 4 * l + dj : 255;
        const unsigned acc = bal ? (dj == 0 ? c0 : dj == 1 ? c1 : dj == 2 ? c2 : c3) : c3;
        sh[0] = prefix | ((unsigned)d << shift);
        sh[1] = r - acc;
      }
    }
    __syncthreads();
    prefix = sh[0];
    r = sh[1];
    pmask |= 255u << shift;
    __syncthreads();
  }
  return prefix;
}

// estimate_tuning's histogram bin of a peak frequency (pitch_tuning: residual of 12 log2(f /
// 27.5) folded to [-0.5, 0.5), numpy's 101 float64 edges, last bin closed); 255 = no bin (f <= 0)
__device__ __noinline__ int tuning_bin(float fx) {  // out of line: the float64 log2 inlined 12x cost registers
  if (!(fx > 0.f)) return 255;
  const float o = (float)log2((double)(fx / 27.5f));
  const float x = 12.0f * o;
  float r = x - floorf(x);  // np.mod(x, 1.0), x > 0
  if (r >= 0.5f) r -= 1.0f;
  const double rd = (double)r;
  int bi = (int)floor((rd + 0.5) * 100.0);
  bi = min(max(bi, 0), A_NTUNE - 1);
  // exact edges: edges[i] = i * 0.01 + (-0.5) (numpy linspace), last bin closed
  while (bi > 0 && rd < (double)bi * 0.01 + (-0.5)) --bi;
  while (bi < A_NTUNE - 1 && rd >= (double)(bi + 1) * 0.01 + (-0.5)) ++bi;
  return bi;
}

// The order statistic after rank r whose key is k (rank r + 1): k itself when more than r + 1
// keys are <= k, else the smallest key above k. One counting pass instead of a second radix
// select (scratch: 2 words).
__device__ unsigned next_order_key(const float* smag, int n, const float2* cd, const int* soff, int T, unsigned k,
                                   unsigned r, unsigned* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x == 0) {
    scratch[0] = 0u;
    scratch[1] = 0xffffffffu;
  }
  __syncthreads();
  unsigned le = 0, gt = 0xffffffffu;
  auto visit = [&](unsigned q) {
    if (q <= k) ++le;
    else gt = min(gt, q);
  };
  if (smag) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) visit(fkey(smag[i]));
  } else {
    for (int t = wave; t < T; t += nw) {
      const int cnt = soff[t + 1] - soff[t];
      for (int i = lane; i < cnt; i += 64) visit(fkey(cd[(size_t)t * A_CMAX + i].y));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    le += __shfl_xor(le, o, 64);
    gt = min(gt, (unsigned)__shfl_xor(gt, o, 64));
  }
  if (lane == 0) {
    atomicAdd(&scratch[0], le);
    atomicMin(&scratch[1], gt);
  }
  __syncthreads();
  const unsigned res = scratch[0] > r + 1 ? k : scratch[1];
  __syncthreads();
  return res;
}

// STOP (probe builds only, audio_debug 32 * STOP; wrong results): return after phase STOP
// (1 MFCC + peak compaction, 2 median, 3 tuning histogram, 4 chroma)
template <int STOP = 0>
__global__ __launch_bounds__(512) void audio_clip_kernel(const float* __restrict__ pow_in,
                                                         const float* __restrict__ meldb, const double* __restrict__ scal,
                                                         const float2* __restrict__ cand, const int* __restrict__ ccount,
                                                         int T, AudioTables tb, float* __restrict__ feat, int F,
                                                         float* __restrict__ tuning_out) {
  __shared__ float smag[A_NLDS];
  __shared__ unsigned char sbin[A_NLDS];  // each peak's tuning bin (255: none), beside smag
  __shared__ int soff[A_TMAX + 1];
  __shared__ double band4[4][A_NMEL];
  __shared__ double redd[8][4];
  __shared__ float redf[8];
  __shared__ int hist[256 * 9];  // the radix select's histogram + one per wave
  __shared__ unsigned sh[2];
  __shared__ int counts[A_NTUNE];
  __shared__ int s_tidx;
  __shared__ double chroma_acc[8][A_NCHROMA];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const float* md = meldb + (size_t)b * T * A_NMEL;
  const int* cnt = ccount + (size_t)b * T;
  const float2* cd = cand + (size_t)b * T * A_CMAX;

  // ---- MFCC: top_db = 80 clamp against the clip max, frame mean, DCT-II ortho
  // loads batched 8 deep (a load-use chain per element was one memory round trip each)
  float mx = -INFINITY;
  for (int i0 = tid; i0 < T * A_NMEL; i0 += 512 * 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = i0 + 512 * j < T * A_NMEL ? md[i0 + 512 * j] : -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) redf[wave] = mx;
  {  // per-frame peak offsets: exclusive prefix of the counts (T <= A_TMAX = 8 per thread)
    const int per = (T + 511) / 512, t0 = min(tid * per, T), t1 = min(t0 + per, T);
    int c[8], own = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c[i] = t0 + i < t1 ? cnt[t0 + i] : 0;
      own += c[i];
    }
    int inc = own;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) hist[wave] = inc;  // per-wave totals (hist is free until the median)
    __syncthreads();
    int acc = inc - own;
    for (int w = 0; w < wave; ++w) acc += hist[w];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (t0 + i < t1) {
        soff[t0 + i] = acc;
        acc += c[i];
      }
    if (tid == 511) soff[T] = acc;
  }
  __syncthreads();
  float floor_db = redf[0];
  for (int i = 1; i < 8; ++i) floor_db = fmaxf(floor_db, redf[i]);
  floor_db -= 80.0f;
  {
    const int m = tid & (A_NMEL - 1), q = tid >> 7;
    double sacc = 0.0;
    for (int t0 = q; t0 < T; t0 += 4 * 8) {  // 8 loads in flight, summed in frame order
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = t0 + 4 * j < T ? md[(size_t)(t0 + 4 * j) * A_NMEL + m] : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (t0 + 4 * j < T) sacc += (double)fmaxf(v[j], floor_db);
    }
    band4[q][m] = sacc;
  }
  const int n = soff[T];
  const bool in_lds = n <= A_NLDS;
  if (in_lds) {  // the peaks compacted into LDS: magnitude (for the median) and tuning bin
    static_assert(A_CMAX <= 3 * 64, "three loads per lane cover a frame's peaks");
    for (int t0 = wave; t0 < T; t0 += 8 * 4) {  // four frames' loads in flight per wave
      float2 v[4][3];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int tf = t0 + 8 * f;
        const int c = tf < T ? soff[tf + 1] - soff[tf] : 0;
#pragma unroll
        for (int j = 0; j < 3; ++j)
          v[f][j] = lane + 64 * j < c ? cd[(size_t)tf * A_CMAX + lane + 64 * j] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int tf = t0 + 8 * f;
        const int o = tf < T ? soff[tf] : 0, c = tf < T ? soff[tf + 1] - o : 0;
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (lane + 64 * j < c) {
            smag[o + lane + 64 * j] = v[f][j].y;
            sbin[o + lane + 64 * j] = (unsigned char)tuning_bin(v[f][j].x);
          }
      }
    }
  }
  __syncthreads();
  if (tid < tb.n_mfcc) {
    double c = 0.0;
    for (int m0 = 0; m0 < A_NMEL; m0 += 16) {  // 16 DCT loads in flight, summed in m order
      double d[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) d[j] = tb.dct[tid * A_NMEL + m0 + j];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int m = m0 + j;
        c += d[j] * ((band4[0][m] + band4[1][m] + band4[2][m] + band4[3][m]) / (double)T);
      }
    }
    feat[(size_t)b * F + tid] = (float)c;
  }

  if constexpr (STOP == 1) return;
  // ---- estimate_tuning: median peak magnitude, residual histogram, argmax
  float med = 0.f;
  if (n > 0) {
    const float* sm = in_lds ? smag : nullptr;
    const unsigned k1 = radix_select(sm, n, cd, soff, T, (unsigned)((n - 1) / 2), hist, sh);
    const float v1 = fkey_inv(k1);
    if (n & 1) {
      med = v1;
    } else {
      const unsigned k2 = next_order_key(sm, n, cd, soff, T, k1, (unsigned)((n - 1) / 2), reinterpret_cast<unsigned*>(hist));
      med = (v1 + fkey_inv(k2)) / 2.0f;
    }
  }
  if constexpr (STOP == 2) {
    if (tid == 0) feat[b] = med;
    return;
  }
  for (int i = tid; i < A_NTUNE; i += 512) counts[i] = 0;
  __syncthreads();
  if (in_lds) {
    for (int i = tid; i < n; i += 512)
      if (smag[i] >= med && sbin[i] != 255) atomicAdd(&counts[sbin[i]], 1);
  } else {
    for (int t = wave; t < T; t += 8) {
      const int c = soff[t + 1] - soff[t];
      for (int i = lane; i < c; i += 64) {
        const float2 pm = cd[(size_t)t * A_CMAX + i];
        if (!(pm.y >= med)) continue;
        const int bi = tuning_bin(pm.x);
        if (bi != 255) atomicAdd(&counts[bi], 1);
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int best = 50;  // pitch_tuning of an empty set: 0.0 = edges[50]
    if (n > 0) {
      int bc = -1;
      for (int i = 0; i < A_NTUNE; ++i)
        if (counts[i] > bc) { bc = counts[i]; best = i; }
      if (bc <= 0) best = 50;
    }
    s_tidx = best;
    if (tuning_out) tuning_out[b] = (float)((double)best * 0.01 + (-0.5));
  }
  __syncthreads();

  // ---- chroma at that tuning: per frame raw = fb . P, / max |raw|, frame mean
  if constexpr (STOP == 3) return;
  // the tuning's filterbank (48 KB) staged into the peak-magnitude buffer, free after the median
  float* fb = smag;
  {
    const float* fbg = tb.chroma + (size_t)s_tidx * A_NCHROMA * A_NBIN;
    constexpr int NI = (A_NCHROMA * A_NBIN + 511) / 512;  // 25 loads per thread, all in flight
    float v[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) v[j] = tid + 512 * j < A_NCHROMA * A_NBIN ? fbg[tid + 512 * j] : 0.f;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (tid + 512 * j < A_NCHROMA * A_NBIN) fb[tid + 512 * j] = v[j];
  }
  __syncthreads();
  // lane c (< 12) keeps chroma c's running sum: one float64 divide per lane and frame, and no
  // 12-double array per lane (the kernel was at 256 VGPRs with scratch spills)
  double cacc = 0.0;
  constexpr int KI = (A_NBIN + 63) / 64;
  for (int t = wave; t < T; t += 8) {
    const float* P = pow_in + ((size_t)b * T + t) * A_NBIN;
    float pv[KI];  // the frame's power column, all loads in flight at once
#pragma unroll
    for (int i = 0; i < KI; ++i) pv[i] = lane + 64 * i < A_NBIN ? P[lane + 64 * i] : 0.f;
    float part[A_NCHROMA];
#pragma unroll
    for (int c = 0; c < A_NCHROMA; ++c) part[c] = 0.f;
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = lane + 64 * i;
      if (k < A_NBIN) {
#pragma unroll
        for (int c = 0; c < A_NCHROMA; ++c) part[c] += fb[c * A_NBIN + k] * pv[i];
      }
    }
#pragma unroll
    for (int c = 0; c < A_NCHROMA; ++c)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) part[c] += __shfl_xor(part[c], o, 64);
    double m = 0.0;
    float mine = 0.f;
#pragma unroll
    for (int c = 0; c < A_NCHROMA; ++c) {
      m = fmax(m, fabs((double)part[c]));
      if (lane == c) mine = part[c];
    }
    if (m < (double)FLT_MIN) m = 1.0;
    cacc += (double)(float)((double)mine / m);
  }
  if (lane < A_NCHROMA) chroma_acc[wave][lane] = cacc;
  if constexpr (STOP == 4) {
    if (lane == 0) feat[b * F + wave] = (float)cacc;
    return;
  }
  // ---- spectral means: zcr, centroid, rolloff, rms (frames over the block)
  double sp[4] = {0.0, 0.0, 0.0, 0.0};
  for (int t = tid; t < T; t += 512)
#pragma unroll
    for (int j = 0; j < 4; ++j) sp[j] += scal[((size_t)b * T + t) * 4 + j];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sp[j] += __shfl_xor(sp[j], o, 64);
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < 4; ++j) redd[wave][j] = sp[j];
  __syncthreads();
  if (tid < A_NCHROMA) {
    double s = 0.0;
    for (int w = 0; w < 8; ++w) s += chroma_acc[w][tid];
    feat[(size_t)b * F + tb.n_mfcc + tid] = (float)(s / (double)T);
  } else if (tid >= 64 && tid < 68) {
    const int j = tid - 64;
    double s = 0.0;
    for (int w = 0; w < 8; ++w) s += redd[w][j];
    feat[(size_t)b * F + tb.n_mfcc + A_NCHROMA + j] = (float)(s / (double)T);
  }
}

// ----------------------------------------------------------------------------- host tables
// Built in float64 on the host exactly as librosa 0.10.0 builds them (oracle/audio.py
// restates the same functions in numpy): fft_frequencies = rfftfreq(n_fft, 1/sr), Slaney mel
// triangles rounded to float32 then scaled by the float64 area factor, the chroma filterbank
// for each of the 100 tuning bins pitch_tuning can return, the periodic Hann window of
// scipy.signal.get_window (linspace(-pi, pi, n + 1) cosine form), the DCT-II ortho matrix.
static double hz_to_mel(double f) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp, logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
static double mel_to_hz(double m) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp, logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

int AudioModel::create(const float* blob, size_t n) {
  MEC_REQUIRE(n == 5, "audio blob: [sample_rate, n_fft, hop, n_mels, n_mfcc]");
  sr = (int)blob[0];
  MEC_REQUIRE(sr >= 8000 && sr <= 96000, "audio: sample_rate out of range");
  MEC_REQUIRE((int)blob[1] == A_NFFT && (int)blob[2] == A_HOP && (int)blob[3] == A_NMEL,
              "audio: the kernels implement n_fft 2048, hop 512, 128 mel bands (librosa defaults)");
  n_mfcc = (int)blob[4];
  MEC_REQUIRE(n_mfcc >= 1 && n_mfcc <= A_NMEL, "audio: n_mfcc must be in [1, 128]");
  const double d = 1.0 / sr, val = 1.0 / (A_NFFT * d);
  std::vector<double> freq(A_NBIN);
  for (int k = 0; k < A_NBIN; ++k) freq[k] = k * val;
  // Hann (scipy general_cosine, sym=False): fac = linspace(-pi, pi, 2049)
  std::vector<double> hann(A_NFFT);
  const double step = (kPi - (-kPi)) / 2048.0;
  for (int i = 0; i < A_NFFT; ++i) hann[i] = 0.5 + 0.5 * std::cos(i * step + (-kPi));
  std::vector<double2> tw(512), post(A_NBIN);
  for (int j = 0; j < 512; ++j) tw[j] = make_double2(std::cos(-2.0 * kPi * j / 1024.0), std::sin(-2.0 * kPi * j / 1024.0));
  for (int k = 0; k < A_NBIN; ++k)
    post[k] = make_double2(std::cos(-2.0 * kPi * k / 2048.0), std::sin(-2.0 * kPi * k / 2048.0));
  // mel filterbank
  std::vector<double> mel_f(A_NMEL + 2);
  const double mmin = hz_to_mel(0.0), mmax = hz_to_mel((double)sr / 2);
  for (int i = 0; i < A_NMEL + 2; ++i) {
    const double m = i == A_NMEL + 1 ? mmax : i * ((mmax - mmin) / (A_NMEL + 1)) + mmin;  // np.linspace
    mel_f[i] = mel_to_hz(m);
  }
  std::vector<int> off(A_NMEL + 1, 0), bins;
  std::vector<float> wts;
  for (int i = 0; i < A_NMEL; ++i) {
    const double fd0 = mel_f[i + 1] - mel_f[i], fd1 = mel_f[i + 2] - mel_f[i + 1];
    const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
    for (int k = 0; k < A_NBIN; ++k) {
      const double lower = -(mel_f[i] - freq[k]) / fd0, upper = (mel_f[i + 2] - freq[k]) / fd1;
      const float w32 = (float)std::max(0.0, std::min(lower, upper));
      if (w32 != 0.f) {
        bins.push_back(k);
        wts.push_back((float)((double)w32 * enorm));
      }
    }
    off[i + 1] = (int)bins.size();
  }
  // mel segments: nonzeros split into 256 contiguous chunks (one per thread); a segment is a
  // run of one band inside one chunk
  const int nnz = (int)bins.size();
  mel_nnz = nnz;
  mel_ch = (nnz + 255) / 256;
  std::vector<int> seg(nnz), segoff(A_NMEL + 1, 0);
  {
    int sgi = -1, prev_band = -1, prev_chunk = -1, band = 0;
    for (int e = 0; e < nnz; ++e) {
      while (e >= off[band + 1]) ++band;
      const int chunk = e / mel_ch;
      if (band != prev_band || chunk != prev_chunk) {
        ++sgi;
        for (int m = prev_band + 1; m <= band; ++m) segoff[m] = sgi;
        prev_band = band;
        prev_chunk = chunk;
      }
      seg[e] = sgi;
    }
    for (int m = prev_band + 1; m <= A_NMEL; ++m) segoff[m] = sgi + 1;
    MEC_REQUIRE(sgi + 1 <= A_MSEG, "audio: too many mel segments");
  }
  // DCT-II ortho [n_mfcc][128]
  std::vector<double> dct((size_t)n_mfcc * A_NMEL);
  for (int k = 0; k < n_mfcc; ++k)
    for (int m = 0; m < A_NMEL; ++m)
      dct[(size_t)k * A_NMEL + m] = (k == 0 ? std::sqrt(1.0 / A_NMEL) : std::sqrt(2.0 / A_NMEL)) *
                                    std::cos(kPi * k * (2 * m + 1) / (2.0 * A_NMEL));
  // chroma filterbanks for tuning = i * 0.01 - 0.5, i = 0..99
  std::vector<float> chroma((size_t)A_NTUNE * A_NCHROMA * A_NBIN);
  {
    const double fstep = (double)sr / A_NFFT;  // np.linspace(0, sr, n_fft, endpoint=False)
    std::vector<double> frq(A_NFFT), bw(A_NFFT), w((size_t)A_NCHROMA * A_NFFT);
    for (int ti = 0; ti < A_NTUNE; ++ti) {
      const double tuning = (double)ti * 0.01 + (-0.5);
      const double a440 = 440.0 * std::pow(2.0, tuning / A_NCHROMA);
      for (int k = 1; k < A_NFFT; ++k) frq[k] = A_NCHROMA * std::log2((k * fstep) / (a440 / 16));
      frq[0] = frq[1] - 1.5 * A_NCHROMA;
      for (int k = 0; k < A_NFFT - 1; ++k) bw[k] = std::max(frq[k + 1] - frq[k], 1.0);
      bw[A_NFFT - 1] = 1.0;
      const double nc2 = std::round(A_NCHROMA / 2.0);
      for (int c = 0; c < A_NCHROMA; ++c)
        for (int k = 0; k < A_NFFT; ++k) {
          double dd = frq[k] - c + nc2 + 10 * A_NCHROMA;
          dd = dd - std::floor(dd / A_NCHROMA) * A_NCHROMA;  // np.remainder
          dd -= nc2;
          const double q = 2 * dd / bw[k];
          w[(size_t)c * A_NFFT + k] = std::exp(-0.5 * q * q);
        }
      for (int k = 0; k < A_NFFT; ++k) {  // L2 column norm, then the octave weighting
        double s = 0.0;
        for (int c = 0; c < A_NCHROMA; ++c) s += w[(size_t)c * A_NFFT + k] * w[(size_t)c * A_NFFT + k];
        double len = std::pow(s, 0.5);
        if (len < DBL_MIN) len = 1.0;
        const double q = (frq[k] / A_NCHROMA - 5.0) / 2;
        const double oct = std::exp(-0.5 * q * q);
        for (int c = 0; c < A_NCHROMA; ++c) w[(size_t)c * A_NFFT + k] = w[(size_t)c * A_NFFT + k] / len * oct;
      }
      for (int c = 0; c < A_NCHROMA; ++c)  // base_c: roll by -3
        for (int k = 0; k < A_NBIN; ++k)
          chroma[((size_t)ti * A_NCHROMA + c) * A_NBIN + k] = (float)w[(size_t)((c + 3) % A_NCHROMA) * A_NFFT + k];
    }
  }
  int lo = A_NBIN, hi = 0;
  for (int k = 0; k < A_NBIN; ++k)
    if (150.0 <= freq[k] && freq[k] < std::min(4000.0, (double)sr / 2)) { lo = std::min(lo, k); hi = std::max(hi, k + 1); }
  lo_bin = std::max(lo, A_BAND_LO);
  hi_bin = std::min(hi, A_BAND_HI);
  // a frame's peaks are local maxima of the band (no two adjacent bins), so at most
  // ceil(band / 2) of them; the per-frame peak list holds A_CMAX (sr >= ~21.6 kHz)
  MEC_REQUIRE((hi_bin - lo_bin + 1) / 2 <= A_CMAX,
              "audio: sample_rate too low for the per-frame peak list (piptrack band 150-4000 Hz holds more than "
              "184 local maxima below ~21.6 kHz); resample to Config.SAMPLE_RATE (22050) first");
  // one device block: doubles first (8-B alignment), then ints / floats
  off_hann = 0;
  off_tw = off_hann + A_NFFT * 8;
  off_post = off_tw + 512 * 16;
  off_freq = off_post + A_NBIN * 16;
  off_dct = off_freq + A_NBIN * 8;
  off_chroma = off_dct + dct.size() * 8;
  off_meloff = off_chroma + chroma.size() * 4;  // mel segment offsets [129]
  off_melbin = off_meloff + segoff.size() * 4;
  off_melw = off_melbin + bins.size() * 4;
  off_melseg = off_melw + wts.size() * 4;
  const size_t total = off_melseg + seg.size() * 4;
  std::vector<char> h(total);
  std::memcpy(h.data() + off_hann, hann.data(), hann.size() * 8);
  std::memcpy(h.data() + off_tw, tw.data(), tw.size() * 16);
  std::memcpy(h.data() + off_post, post.data(), post.size() * 16);
  std::memcpy(h.data() + off_freq, freq.data(), freq.size() * 8);
  std::memcpy(h.data() + off_dct, dct.data(), dct.size() * 8);
  std::memcpy(h.data() + off_chroma, chroma.data(), chroma.size() * 4);
  std::memcpy(h.data() + off_meloff, segoff.data(), segoff.size() * 4);
  std::memcpy(h.data() + off_melseg, seg.data(), seg.size() * 4);
  std::memcpy(h.data() + off_melbin, bins.data(), bins.size() * 4);
  std::memcpy(h.data() + off_melw, wts.data(), wts.size() * 4);
  return upload(tables, h.data(), total);
}

int AudioModel::forward(const float* wave, int B, int L, float* feat, float* tuning, hipStream_t s) {
  MEC_REQUIRE(B >= 0, "audio: B < 0");
  if (B == 0) return 0;
  MEC_REQUIRE(wave && feat, "audio: null pointer");
  MEC_REQUIRE(L >= A_NFFT / 2 + 1 && L / A_HOP + 1 <= A_TMAX, "audio: n_samples out of range (1025 .. 2^21)");
  const int T = 1 + L / A_HOP;  // center=True frames
  const size_t fr = (size_t)B * T;
  const size_t need = fr * (A_NBIN * 4 + A_NMEL * 4 + 4 * 8 + A_CMAX * 8 + 4) + 1024;
  if (ws.bytes < need) MEC_TRY(ws.ensure(need));
  char* p = ws.as<char>();
  double* scal = reinterpret_cast<double*>(p); p += fr * 4 * 8;
  float2* cand = reinterpret_cast<float2*>(p); p += fr * A_CMAX * 8;
  float* pw = reinterpret_cast<float*>(p); p += fr * A_NBIN * 4;
  float* mdb = reinterpret_cast<float*>(p); p += fr * A_NMEL * 4;
  int* cc = reinterpret_cast<int*>(p);
  const char* tb0 = tables.as<char>();
  AudioTables tb;
  tb.hann = reinterpret_cast<const double*>(tb0 + off_hann);
  tb.tw = reinterpret_cast<const double2*>(tb0 + off_tw);
  tb.post = reinterpret_cast<const double2*>(tb0 + off_post);
  tb.freq = reinterpret_cast<const double*>(tb0 + off_freq);
  tb.dct = reinterpret_cast<const double*>(tb0 + off_dct);
  tb.chroma = reinterpret_cast<const float*>(tb0 + off_chroma);
  tb.mel_segoff = reinterpret_cast<const int*>(tb0 + off_meloff);
  tb.mel_seg = reinterpret_cast<const int*>(tb0 + off_melseg);
  tb.mel_nnz = mel_nnz;
  tb.mel_ch = mel_ch;
  tb.mel_bin = reinterpret_cast<const int*>(tb0 + off_melbin);
  tb.mel_w = reinterpret_cast<const float*>(tb0 + off_melw);
  tb.lo_bin = lo_bin;
  tb.hi_bin = hi_bin;
  tb.n_mfcc = n_mfcc;
  tb.sr = (double)sr;
  MEC_TRY(prof.begin(TAG_AUDIO, s));
#ifdef MEC_PROBES
  switch (opt().audio_debug) {
    case 1: hipLaunchKernelGGL(audio_frame_kernel<1>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc); break;
    case 2: hipLaunchKernelGGL(audio_frame_kernel<2>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc); break;
    case 4: hipLaunchKernelGGL(audio_frame_kernel<4>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc); break;
    case 8: hipLaunchKernelGGL(audio_frame_kernel<8>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc); break;
    case 15: hipLaunchKernelGGL(audio_frame_kernel<15>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc); break;
    default: hipLaunchKernelGGL(audio_frame_kernel<0>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc);  // 0, and 32..128 (clip-kernel probes)
  }
#else
  hipLaunchKernelGGL(audio_frame_kernel<0>, dim3(T, B), dim3(256), 0, s, wave, L, T, tb, pw, mdb, scal, cand, cc);
#endif
  MEC_LAUNCH_CHECK();
#ifdef MEC_PROBES
  if (opt().audio_debug >= 32) {
    const int F = n_mfcc + A_NCHROMA + 4;
    switch (opt().audio_debug >> 5) {
      case 1: hipLaunchKernelGGL(audio_clip_kernel<1>, dim3(B), dim3(512), 0, s, pw, mdb, scal, cand, cc, T, tb, feat, F, tuning); break;
      case 2: hipLaunchKernelGGL(audio_clip_kernel<2>, dim3(B), dim3(512), 0, s, pw, mdb, scal, cand, cc, T, tb, feat, F, tuning); break;
      case 3: hipLaunchKernelGGL(audio_clip_kernel<3>, dim3(B), dim3(512), 0, s, pw, mdb, scal, cand, cc, T, tb, feat, F, tuning); break;
      default: hipLaunchKernelGGL(audio_clip_kernel<4>, dim3(B), dim3(512), 0, s, pw, mdb, scal, cand, cc, T, tb, feat, F, tuning);
    }
  } else
#endif
  hipLaunchKernelGGL(audio_clip_kernel<0>, dim3(B), dim3(512), 0, s, pw, mdb, scal, cand, cc, T, tb, feat,
                     n_mfcc + A_NCHROMA + 4, tuning);
  MEC_LAUNCH_CHECK();
  MEC_TRY(prof.end(TAG_AUDIO, s));
  return 0;
}

}  // namespace mec
