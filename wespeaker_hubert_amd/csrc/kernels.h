// Launcher interfaces of the hand-written gfx950 kernels.
#pragma once

#include <vector>

#include "common.h"

namespace wsp {

// ---------------------------------------------------------------------------
// Implicit-GEMM 1-D convolution over channels-last frames (fp32 MFMA).
//
//   out[m][n] = epi( sum_{j<taps} sum_{c<cin} A(m + j*dil - pad, c) * W[n][j*cin + c] )
//
// Rows m = b*T + t index (utterance, frame); a tap that leaves [0, T) of its
// utterance reads zero (the reference's zero padding).  A(row, c) is one of
//   kACat : channel c taken from segment s (cseg[s] <= c < cseg[s+1]) of
//           up to 3 row-major buffers -> torch.cat(dim=1) without a copy
//   kAAdd : a[0][row][c] + a[1][row][c]   (Res2Net's `sp + spx[i]`)
// epi(y) = ((y + bias[n] + row_bias[b][n] + res[m][n]) -> act) * scale[n] + shift[n]
// ---------------------------------------------------------------------------
enum AMode { kACat = 0, kAAdd = 1 };
enum Act { kActNone = 0, kActRelu = 1, kActTanh = 2, kActGelu = 3 };  // GELU: exact erf form

struct ConvGemmArgs {
  const float* a[3];
  int lda[3];
  int cseg[4];
  int cin, taps, dil, pad;
  int M, T, N;
  const float* w;  // [N][Kp] packed, Kp = round_up(taps*cin, 32), zero padded
  int K, Kp;
  const float* bias;      // [N] or null
  const float* row_bias;  // [M/T][N] or null
  const float* res;       // [M][ldres] or null
  int ldres;
  const float* scale;  // [N] or null (then shift ignored)
  const float* shift;
  float* out;
  int ldo;
  int act;
  int amode;
  int role;  // 1 = SE-Res2Block 1x1 CxC conv (own kernel symbol for profiling); 2 = residual
             // conv whose residual is loaded ahead of the last two k-tiles (narrow bf16x3 tiles)
  // 2-D (NHWC, ResNet) mode: input [B][Fi][Ti][cin], output rows m = (b*Fo + fo)*To + to,
  // taps = kh*kw with tap j = kf*kw + kt, input (fo*stride + kf - pad, to*stride + kt - pad).
  int conv2d;
  int Fi, Ti, Fo, To, stride, kw;
  // ResNet bottleneck conv3 + projection shortcut in one 1x1 GEMM (x3 tile family 7 only): A
  // segment 0 (channels [0, cseg[1])) is dense, row m; segment 1 ([cseg[1], cseg[2])) is read at
  // the shortcut's 2-D strided position of output row m = (b*Fo + fo)*To + to, input row
  // (b*Fi + fo*stride)*Ti + to*stride of a[1] (conv2d stays 0; Fi / Ti / Fo / To / stride carry
  // the shortcut geometry).
  int sc2d;
  // 1-D strided conv (HuBERT feature extractor): rows m = b*T + t read input
  // frame t*stride + j*dil - pad of [b][Ti]; stride 0 -> 1, Ti 0 -> T.
  // Grouped conv (HuBERT pos_conv): output columns are grouped gcols wide
  // (a block never straddles a group) and group g reads input channels
  // [g*gcin, g*gcin + cin).  gcols 0 = ungrouped.
  int gcols, gcin;
  // Segmented (ragged) batch, 1-D convs: utterance b owns output rows
  // [seg[b], seg[b+1]) and input rows [iseg[b], iseg[b+1]) (device int32
  // [nseg+1]; iseg null = seg, stride 1); taps outside it read zero.
  // seg null = uniform T.
  const int* seg;
  const int* iseg;
  int nseg;
  // bf16x3 kernels, uniform batches with T >= block rows: per-utterance column
  // sums of the epilogue output y, f64 partials [M / BM][2][N] (slot 0 = the
  // utterance of the block's first row, 1 = the next); conv_gemm_colsum_mean()
  // turns them into per-utterance means (the SE squeeze, ecapa_tdnn.py:118).
  double* colsum;
  // HuBERT LayerNorm fold (x3 tile family 7, dense 1x1 GEMMs only; conv_gemm_x3_t6.hip).
  // lnmode bits: 1 = emit the row statistics of the output y as (mean, M2) partials of its
  // 128-column pieces, ln_out [M][N / 128][2]; 2 = fold: y = (acc - mu ln_cs[n]) rstd + bias
  // (A = the un-normalised rows, W pre-scaled by gamma, bias = b + W beta); 4 = the residual
  // is normalised on the fly: res = (res - mu) rstd ln_g + ln_b.  Modes 2 / 4 read mu, rstd
  // from ln_in [M][ln_parts][2] (partials of 128 columns, ln_parts x 128 = the normalised width).
  int lnmode;
  float* ln_out;
  const float* ln_in;
  int ln_parts;
  const float* ln_cs;
  const float* ln_g;
  const float* ln_b;
  float ln_eps;
};

// Fills the 1-D defaults (stride 1, Ti = T) of a zero-initialised ConvGemmArgs.
inline ConvGemmArgs normalized(ConvGemmArgs p) {
  if (!p.conv2d && !p.sc2d) {
    if (p.stride <= 0) p.stride = 1;
    if (p.Ti <= 0) p.Ti = p.T;
  }
  return p;
}

// bf16x3 split-precision variant (conv_gemm_x3.hip); whi/wlo = packed [N][Kp]
// bf16 hi/lo images of W.  variant (N % 128 == 0): 3 = 128x128 / 4 waves,
// 4 = 256x128 / 8 waves, 5 = 256x256 / 8 waves where N % 256 == 0 (else 4);
// all with XOR-swizzled LDS rows.
// Rows per block of the bf16x3 tile launch_conv_gemm_x3 picks for p / variant
// (the colsum partials' granularity).
int conv_gemm_x3_block_rows(const ConvGemmArgs& p, int variant);
// mean[b][n] = sum over the row blocks of utterance b of colsum partials / T
// (fixed block order: the same sums whatever the batch), f32 out[b * ldo + n].
void launch_colsum_mean(const double* part, int block_rows, int T, int B, int N, float* out, int ldo,
                        hipStream_t s);
void launch_conv_gemm_x3(const ConvGemmArgs& p, const void* whi, const void* wlo, int variant,
                         hipStream_t s);


// tile: 0 = 128x128 block (N % 128 == 0), 1 = 128x64 block (N % 64 == 0)
void launch_conv_gemm(const ConvGemmArgs& p, hipStream_t s);
int conv_gemm_tile_for(int N);

// ---------------------------------------------------------------------------
// Small row-batched linear: out[r][n] = act(bias[n] + sum_k in[r][k] * Wt[k][n])
// followed by an optional affine (scale/shift).  Wt is [K][N] (k-major).
// act: 0 none, 1 relu, 2 tanh, 3 sigmoid
// ---------------------------------------------------------------------------
struct SmallLinearArgs {
  const float* in;
  int ldin;
  const float* wt;
  const float* bias;
  float* out;
  int ldo;
  int R, K, N;
  int act;
  // optional scratch for long K (>= 4096): the k range splits over blocks (split-K partials
  // [KS][R][N], summed in slice order by a second pass); null = one pass, 4 rows per block
  float* scratch = nullptr;
  size_t scratch_floats = 0;
};
void launch_small_linear(const SmallLinearArgs& p, hipStream_t s);
// scratch floats the split-K path needs (0 below K = 4096); offering less is an error
size_t small_linear_scratch_floats(int R, int N, int K);

// Segmented (ragged) batches: `seg` = device int32 [B+1] row offsets, utterance
// b owning rows [seg[b], seg[b+1]); null = uniform rows b*T .. b*T + T-1.

// Per-utterance statistics over frames of a channels-last buffer x [rows][ldx]:
// mean[b][c] -> out[b*ldo + c]; if with_std: sqrt(var_unbiased + 1e-7)
// -> out[b*ldo + std_off + c]  (pooling_layers.py TSTP / GLOB context).
void launch_frame_stats(const float* x, int ldx, int B, int T, int C, float* out, int ldo,
                        int with_std, int std_off, hipStream_t s, const int* seg = nullptr);

// out[m][c] = x[m][c] + h[m][c] * g[b][c]  (SE_Res2Block residual, ecapa_tdnn.py:156);
// M = total rows when segmented.
void launch_residual_scale(const float* x, const float* h, const float* g, float* out, int B,
                           int T, int C, hipStream_t s, const int* seg = nullptr, int M = 0);

// ASTP attentive statistics (pooling_layers.py:135-144): softmax over frames
// of logits e [rows][C], weighted mean/std of x [rows][C] -> out [B][2C];
// std = sqrt(clamp(E[x^2] - mu^2, var_floor)) (1e-7 ASTP, 1e-5 ASP pooling_layers.py:170).
void launch_astp_pool(const float* e, const float* x, int B, int T, int C, float* out,
                      hipStream_t s, const int* seg = nullptr, float var_floor = 1e-7f);

// SimAM attention + shortcut + ReLU of a SimAMBasicBlock (samresnet.py:56-69):
// out = relu(z * sigmoid((z - mean)^2 / (4 (var_{n-1} + 1e-4)) + 0.5) + res), statistics
// per (utterance, channel) over the `rows` = F*T positions of z [B][rows][C] (NHWC).
// part: f64 scratch [B][simam_chunks(B, rows)][2][C]; coef: f32 scratch [B][2][C].
int simam_chunks(int B, int rows);
void launch_simam(const float* z, const float* res, float* out, int B, int rows, int C, double* part, float* coef,
                  hipStream_t s);
// [B][F][T][C] -> [B][T][F][C]: ASP's x.reshape(B, C*F, T) as frame rows (channel order f*C + c).
void launch_nhwc_to_tfc(const float* in, float* out, int B, int F, int T, int C, hipStream_t s);

// ResNet stem: 1 -> C0 3x3 conv + folded BN + ReLU, (B,T,F) feats -> NHWC [B][F][T][C0].
void launch_resnet_stem(const float* feats, int B, int T, int F, int C0, const float* w, const float* bias,
                        float* out, hipStream_t s);

// Kaldi fbank (float64 arithmetic) + optional fused CMN (fbank.hip).
// torchaudio.compliance.kaldi.fbank options the extraction path passes
// (processor.py:472-502, cli/speaker.py:89-104): bins, rate, frame length /
// shift in ms, window; low / high mel edges (torchaudio defaults 20 / 0).
struct FbankConfig {
  int num_bins = 80, sample_rate = 16000, window = 0;  // window: WSP_WINDOW_*
  double frame_length_ms = 25.0, frame_shift_ms = 10.0, low_freq = 20.0, high_freq = 0.0;
  // derived (fbank_config_resolve): samples per frame / shift, padded FFT size
  int frame_len = 0, frame_shift = 0, padded = 0;
};
// Validates `c` and fills frame_len / frame_shift / padded (torchaudio's
// int(sr * ms * 0.001) and round_to_power_of_two); padded must be 256 or 512.
void fbank_config_resolve(FbankConfig& c);
// torchaudio get_mel_banks(num_bins, padded, sr, low, high) in its float32
// arithmetic (correctly rounded log): w = [num_bins][padded / 2 + 1], the
// Nyquist column 0 (kaldi.py pads it).  Computed here, at plan time.
void fbank_mel_banks(const FbankConfig& c, std::vector<float>& w);
// Device-side description of one configuration: table (window, twiddles,
// lane-interleaved mel filters) + geometry.
struct FbankPlan {
  FbankConfig cfg;
  bool fixed = false;  // the 80-bin 16 kHz 25 / 10 ms hamming instance (compile-time geometry)
  int len0 = 0, len1 = 0;  // padded filter lengths of bins 0..63 / 64..
  std::vector<double> host_tab;
  const double* tab = nullptr;  // device copy (owned by the caller's cache)
};
void fbank_plan(const FbankConfig& c, FbankPlan& p);  // host part (table)
// Segmented: wseg / fseg = device int32 [B+1] sample / frame offsets, T = frames
// of the longest utterance (grid size); N, ld unused.
void launch_fbank(const void* wav, int dtype, int B, int N, int ld, float scale, float* feats,
                  int T, int cmn, const FbankPlan& plan, hipStream_t s, const int* wseg = nullptr,
                  const int* fseg = nullptr);

// HuBERT-base front end (hubert.hip).
// conv0 (1 -> 512, k10 s5, no bias) + GroupNorm(512, 512) + GELU:
// wav [B][ldw] (N samples) -> out [B][T0][512]; stats = [2][B][512] doubles scratch (65 per utterance used).
// Segmented: wseg / oseg = device int32 [B+1] sample / output-row offsets, T0 = frames of
// the longest utterance.
void launch_hubert_conv0(const float* wav, int B, int N, int ldw, int T0, const float* w, const float* gamma,
                         const float* beta, double* stats, float* out, hipStream_t s, const int* wseg = nullptr,
                         const int* oseg = nullptr);
// doubles of launch_hubert_conv0's `stats` scratch for B utterances of at most T0 conv0 frames
size_t hubert_conv0_stats_doubles(int B, int T0);
// Positional conv (pos_conv.hip): out[row][g*gout + n] = GELU(bias[g*gout + n] + sum_{tap, c}
// x[row + tap - 64][48 g + c] * W[g*gout + n][tap*48 + c]) for the 16 groups x 48 outputs, per
// utterance of seg (int32 [B+1] device offsets, at most maxT frames, M rows in all); W = the
// bf16 hi / lo grouped pack (ldw elements per row), bf16x3 products.
void launch_hubert_pos_conv(const float* x, int ldx, const int* seg, int B, int maxT, int M, const void* whi,
                            const void* wlo, int ldw, int gout, const float* bias, float* out, int ldo,
                            hipStream_t s);
// out[row] = LayerNorm(x[row] (+ add[row][remap(c)])) with remap(c) = (c/gin)*gout + c%gin;
// if feat: feat[b][t'] (=|+=) feat_w * out[row] for t' = t, and t' in [T, Tout) when t = T-1.
struct LayerNormArgs {
  const float* x;
  int ldx;
  const float* add;
  int ldadd, gin, gout;
  const float* gamma;
  const float* beta;
  float eps;
  float* out;
  int ldo;
  int M, D;
  float* feat;
  float feat_w;
  int feat_init, T, Tout;
  // segmented featurizer: hidden-state rows [seg[b], seg[b+1]) -> feature rows [fseg[b], fseg[b+1])
  const int* seg;
  const int* fseg;
  int nseg;
};
void launch_layernorm(const LayerNormArgs& p, hipStream_t s);
// x [B][T][D] -= mean over T  (apply_cmvn(norm_mean=True, norm_var=False))
void launch_cmn_rows(float* x, int B, int T, int D, hipStream_t s, const int* seg = nullptr);
// apply_cmvn(norm_mean, norm_var) (dataset_utils.py:19-26): x -= mean_T; then
// x /= sqrt(var_T(unbiased) + 1e-7) — the variance about the (new) mean, so
// norm_var alone on already mean-normalised rows equals the pair.
void launch_cmvn_rows(float* x, int B, int T, int D, int norm_mean, int norm_var, hipStream_t s,
                      const int* seg = nullptr);

// Scoring helpers.
void launch_l2_normalize(const float* x, const float* sub, float* y, int R, int D, hipStream_t s);
void launch_cosine_pairs(const float* E, int D, const int32_t* ia, const int32_t* ib, int P,
                         double* score, hipStream_t s);
void asnorm_layout(int Ne, int Nc, int D, int* Ncp, int* Dp, size_t* bytes);
void launch_asnorm_stats(const float* E, int Ne, const float* C, int Nc, int D, int top_n,
                         double* mu, double* sd, float* ws, hipStream_t s);
void launch_row_mean_accum(const float* x, const int32_t* group, int R, int D, double* acc,
                           double* cnt, hipStream_t s);

// ------------------------------------------------------------ resampling --
// torchaudio.transforms.Resample (sinc_interp_hann) — resample.hip.
struct ResamplePlan {
  int orig = 1, nw = 1, width = 0, L = 1;  // reduced rates, half-width, taps per phase
  bool identity = true;
  std::vector<float> kern;  // [nw][L]
  std::vector<int> band;    // [nw][2] nonzero tap range per phase
};
void resample_plan(int orig_freq, int new_freq, int lowpass_filter_width, double rolloff, ResamplePlan& p);
long long resample_out_len(const ResamplePlan& p, long long n);
void launch_resample(const ResamplePlan& p, const float* d_kern, const int* d_band, const float* x, int B, int N,
                     long ldx, float* y, long ldy, hipStream_t s);

}  // namespace wsp
