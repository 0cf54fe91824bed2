/*
 * wespeaker_amd.h — C-ABI of the MI355X-native speaker-embedding extraction
 * path (libwsp_hip.so).  Plain pointers and sizes only; no torch types.
 *
 * Device pointers are HIP device pointers (e.g. torch.Tensor.data_ptr() of a
 * cuda tensor); `stream` is a hipStream_t passed as void* (NULL = default
 * stream).  Every entry point returns 0 on success or a negative WSP_E* code;
 * the message of the last failure on the calling thread is wsp_last_error().
 * The library never frees caller memory and never synchronises the stream
 * except where a function says so.  A model handle is bound to the device
 * that was current when it was created; it is thread-compatible, not
 * thread-safe.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository JunyiPeng00/wespeaker_hubert):
 *   wsp_fbank            torchaudio.compliance.kaldi.fbank as called at
 *                        wespeaker/cli/speaker.py:89-104 and
 *                        wespeaker/dataset/processor.py:472-502 (+ CMN of
 *                        speaker.py:102-103 / dataset_utils.py:19-26);
 *                        native restatement runtime/core/frontend/fbank.h:138-198
 *   wsp_model_*          get_speaker_model(name)(**model_args) + load_checkpoint
 *                        (wespeaker/models/speaker_model.py:30-57,
 *                        wespeaker/utils/checkpoint.py:20-27) and the
 *                        `model(feats)[-1]` forward (cli/speaker.py:164-167,
 *                        bin/extract.py:114-116); C++ plugin analogue
 *                        SpeakerModel::ExtractEmbedding
 *                        (runtime/core/speaker/speaker_model.h:25-32)
 *   wsp_cmn              cli/speaker.py:106-110 (subsegment CMN), dataset_utils.py:19-26
 *   wsp_resample*        cli/speaker.py:155-157, dataset/processor.py:242-260
 *                        (torchaudio.transforms.Resample)
 *   wsp_l2_normalize,
 *   wsp_cosine_pairs     bin/score.py:38-72 trials_cosine_score;
 *                        Speaker.cosine_similarity cli/speaker.py:189-192
 *   wsp_asnorm_stats     bin/score_norm.py:26-36 get_mean_std
 *   wsp_row_mean_accum   bin/score.py:25-35 calculate_mean_from_kaldi_vec,
 *                        tools/vector_mean.py:24-53 compute_vector_mean
 */
#ifndef WESPEAKER_AMD_H_
#define WESPEAKER_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WSP_OK 0
#define WSP_E_INVALID (-1)   /* bad argument / shape */
#define WSP_E_HIP (-2)       /* HIP runtime error */
#define WSP_E_STATE (-3)     /* call order (e.g. forward before finalize) */
#define WSP_E_UNSUPPORTED (-4)

#define WSP_DTYPE_F32 0
#define WSP_DTYPE_S16 1

/* kaldi.fbank window_type (torchaudio compliance/kaldi.py _feature_window_function;
 * Speaker.set_window_type, cli/speaker.py:62) */
#define WSP_WINDOW_HAMMING 0
#define WSP_WINDOW_POVEY 1
#define WSP_WINDOW_HANNING 2
#define WSP_WINDOW_RECTANGULAR 3
#define WSP_WINDOW_BLACKMAN 4

typedef struct wsp_model wsp_model;

int wsp_abi_version(void);
const char* wsp_last_error(void);

/* ------------------------------------------------------------- fbank --- */
/* Number of snip-edges frames: 1 + (num_samples - frame_len) / frame_shift,
 * 0 when num_samples < frame_len. */
int wsp_fbank_num_frames(int num_samples, int frame_len, int frame_shift);

/* torchaudio.compliance.kaldi.fbank options on the extraction path
 * (dataset_args.fbank_args -> processor.compute_fbank, processor.py:472-502;
 * Speaker.compute_fbank, cli/speaker.py:89-104).  Fixed as the reference
 * calls it: dither 0 (bin/extract.py:66-67), DC removal, pre-emphasis 0.97,
 * snip edges, power spectrum, log, no energy, no VTLN.  Implemented: 4..128
 * bins and any frame that pads to 256 or 512 samples (25 ms at 8 or 16 kHz,
 * examples/sre/v2,v3/conf/resnet.yaml and the voxceleb recipes). */
typedef struct wsp_fbank_opts {
  int num_mel_bins;       /* 80 */
  int sample_rate;        /* sample_frequency, Hz (16000) */
  double frame_length_ms; /* 25 */
  double frame_shift_ms;  /* 10 */
  int window_type;        /* WSP_WINDOW_* (hamming) */
  double low_freq;        /* 20 */
  double high_freq;       /* 0 = Nyquist; < 0 = offset below Nyquist */
} wsp_fbank_opts;

/* Fills torchaudio's defaults with the reference's window (hamming). */
int wsp_fbank_opts_default(wsp_fbank_opts* o);
/* Frame geometry of `o`: samples per frame / shift (int(sr * ms * 0.001)) and
 * the padded FFT size; WSP_E_INVALID for options outside the set above. */
int wsp_fbank_geometry(const wsp_fbank_opts* o, int* frame_len, int* frame_shift, int* padded);
/* Host-only: torchaudio get_mel_banks(num_mel_bins, padded, ...) as the kernel
 * uses it, banks = [num_mel_bins][padded / 2 + 1] f32 (Nyquist column 0). */
int wsp_fbank_mel_banks(const wsp_fbank_opts* o, float* banks);

/* Batched Kaldi log-mel fbank.
 *   wav    [B][ld] samples (f32 or s16), first num_samples of each row used
 *   scale  multiplies samples first (32768 for [-1,1] input on the
 *          dataset path, processor.py:492; 1 for int16-valued input)
 *   feats  [B][T][num_mel_bins] f32, T = wsp_fbank_num_frames(num_samples,
 *          frame_len, frame_shift) of wsp_fbank_geometry
 *   cmn    1: subtract the per-utterance mean over frames (speaker.py:102-103) */
int wsp_fbank_ex(const void* wav, int wav_dtype, int B, int num_samples, int ld, float scale,
                 float* feats, const wsp_fbank_opts* opts, int cmn, void* stream);
/* Same with 25 ms / 10 ms frames and 20 Hz .. Nyquist filters. */
int wsp_fbank(const void* wav, int wav_dtype, int B, int num_samples, int ld, float scale,
              float* feats, int num_bins, int sample_rate, int window_type, int cmn,
              void* stream);

/* Segmented (ragged) batch of B whole utterances of different lengths in one
 * launch — the batch_size=1 whole-utterance extraction of bin/extract.py:78-80
 * (Dataset(whole_utt=True)) and Speaker.extract_embedding_list (speaker.py:170-179)
 * without per-utterance launches.  Device int32 offsets: utterance b = samples
 * [sample_offsets[b], sample_offsets[b+1]) of `wav` and frames
 * [frame_offsets[b], frame_offsets[b+1]) of `feats` (frames_b =
 * wsp_fbank_num_frames(samples_b, frame_len, frame_shift) >= 1); max_frames =
 * largest frames_b. */
int wsp_fbank_segments_ex(const void* wav, int wav_dtype, int B, const int32_t* sample_offsets,
                          const int32_t* frame_offsets, int max_frames, float scale, float* feats,
                          const wsp_fbank_opts* opts, int cmn, void* stream);
int wsp_fbank_segments(const void* wav, int wav_dtype, int B, const int32_t* sample_offsets,
                       const int32_t* frame_offsets, int max_frames, float scale, float* feats,
                       int num_bins, int sample_rate, int window_type, int cmn, void* stream);

/* ------------------------------------------------------------- model --- */
/* arch: "ECAPA_TDNN_c512", "ECAPA_TDNN_GLOB_c512", "ECAPA_TDNN_c1024",
 * "ECAPA_TDNN_GLOB_c1024", "ResNet18/34/50/101/152/221/293"
 * (wespeaker/models/speaker_model.py:30-57), or the SSL front end
 * "HuBERT_base" (embed_dim 768; wespeaker/frontend/s3prl.py:23-75). */
int wsp_model_create(const char* arch, int feat_dim, int embed_dim, int emb_bn,
                     int two_emb_layer, wsp_model** out);
int wsp_model_destroy(wsp_model* m);
/* Parameters follow the reference state_dict order (wsp_model_param_info). */
int wsp_model_num_params(const wsp_model* m);
int wsp_model_param_info(const wsp_model* m, int index, const char** name, int* ndim,
                         int64_t shape[4]);
/* Copy one parameter from HOST memory (float32, numel elements). */
int wsp_model_set_param(wsp_model* m, int index, const float* host_data, int64_t numel);
/* Fold BatchNorms, pack weights for the kernels, upload.  Synchronous. */
int wsp_model_finalize(wsp_model* m);
int wsp_model_embed_dim(const wsp_model* m);
int wsp_model_feat_dim(const wsp_model* m);
/* Bytes of device workspace a forward over B utterances of T frames needs. */
int wsp_model_workspace_bytes(const wsp_model* m, int B, int T, size_t* bytes);
/* feats [B][T][feat_dim] f32 (channels-last, exactly the reference's (B,T,F)
 * input) -> embed [B][embed_dim] f32.  Asynchronous on `stream`. */
int wsp_model_forward(wsp_model* m, const float* feats, int B, int T, float* embed,
                      void* workspace, size_t workspace_bytes, void* stream);

/* Segmented (ragged) batch, ECAPA-TDNN handles: utterance b = rows
 * [frame_offsets[b], frame_offsets[b+1]) of feats [total_frames][feat_dim]
 * (device int32 offsets, frame_offsets[B] = total_frames) -> embed [B][embed_dim];
 * each embedding equals a batch-of-one forward of that utterance
 * (ecapa_tdnn.py:208-234 convs pad at utterance edges; pooling per utterance). */
int wsp_model_workspace_bytes_segments(const wsp_model* m, int B, int total_frames, size_t* bytes);
int wsp_model_forward_segments(wsp_model* m, const float* feats, int B, const int32_t* frame_offsets,
                               int total_frames, float* embed, void* workspace, size_t workspace_bytes,
                               void* stream);

/* Runtime options (any time after create unless noted):
 *   "precision"    1 = bf16x3 split MFMA (default; fp32-class accuracy),
 *                  0 = exact f32 MFMA (ECAPA-TDNN and HuBERT)
 *   "streams"      1..8: the batch's utterances are split into this many contiguous
 *                  ranges forwarded on concurrent HIP streams (forked from and joined
 *                  back to the caller's stream; each range has its own workspace
 *                  slice, so query the workspace size after setting it); results are
 *                  bit-identical to 1.  Default 2 for ResNet / SimAM-ResNet / HuBERT,
 *                  1 for ECAPA-TDNN; segmented ECAPA batches always run as one range
 *   "x3_variant"   bf16x3 conv-GEMM tile family (all with swizzled LDS rows): 3 = 128x128,
 *                  4 = 256x128 (ResNet default), 5 = 256x256 where N % 256 == 0, else 256x128
 *                  (SimAM-ResNet default), 6 = 5 with the 256x256 tile on 16x16x32 MFMAs,
 *                  7 = 6 with the 1-D GEMMs (N % 256 == 0, one or three concatenated A
 *                  segments) on one LDS-DMA tile kernel (conv_gemm_x3_t6.hip: A fp32 and
 *                  W hi / lo staged by buffer_load ... lds, A split at fragment time, outputs
 *                  through LDS as whole rows; bit-identical to 6; ECAPA-TDNN and HuBERT default)
 *   "res2_fused"   1 = one res2_chain launch per SE_Res2Block (default), 0 = 7 GEMMs
 *   "res2_variant" res2_chain kernel: 128-row windows with halo recompute: 0 = 2 x 2 waves,
 *                  2 = 4 waves on N with 4 W k-steps in flight (C = 128; else as 0), 3 = 8 waves
 *                  (2 on M x 4 on N for C = 128, 4 x 2 for C = 64; the C = 64 default);
 *                  4 = halo-free strips of ~M / (2 x CUs) rows walked in skewed 96-row chunks
 *                  (C = 128, default; C = 64 runs 3).  All bit-identical
 *   "astp_fused"   ECAPA-TDNN ASTP linear2 + softmax statistics in one kernel (astp_fused.hip,
 *                  default 1); 0 = linear2 GEMM + separate pooling kernel
 *   "conv3x3_img"  ResNet / SimAM-ResNet stride-1 3x3 convs from an LDS image of the input
 *                  patch (bit-identical to the implicit GEMM): 1 = 32 / 64 channels, 2 = also
 *                  128 channels, 4 x 32 positions x 4 column tiles per wave (default), 3 = also
 *                  128 channels, 8 waves x 2 column tiles; 0 = implicit GEMM throughout
 *   "res_prefetch" ResNet: 1 = the 1x1 residual convs (bottleneck conv3) load their residual
 *                  ahead of the last two k-tiles (default), 0 = in the epilogue (bit-identical)
 *   "res_tail"     ResNet: 2 = the bottleneck conv2 (3x3) + conv3 (1x1) + residual + ReLU of
 *                  stride-1 blocks with 32 / 64 / 128 planes in one launch, conv2's output kept in
 *                  registers; 1 = that, plus the next block's conv1 on the output while it is on chip,
 *                  every wave on two position runs (tail2_kernel, default); 0 = conv2, conv3 and
 *                  conv1 as separate launches through HBM
 *   "cat_gate"     ECAPA-TDNN: 1 = conv_cat on [out2, out3, out4 - out3] with weights
 *                  [W_a, W_b + W_c, W_c], so the last SE block stores only its gated branch
 *                  (default; equal to 0 up to rounding, ~1e-6), 0 = conv_cat on [out2, out3, out4]
 *   "in_planes"    SimAM-ResNet, before the weights: 32 or 64
 *   "attn_pipe"    HuBERT front end: 1 = the persistent pipelined attention kernel (keys in
 *                  LDS halves of 128 frames, the next half in flight; default), 0 = one block
 *                  per (utterance, head, 128-query block); both bf16x3 MFMA
 *   "pos_conv"     HuBERT front end, precision 1: 1 = the positional conv as a direct grouped
 *                  conv (pos_conv.hip: one block per 256 frames x group, input patch split into
 *                  bf16 hi / lo once in LDS; default), 0 = the grouped implicit GEMM (48 of 64
 *                  padded columns per group); equal up to fp32 rounding
 *   "ln_fold"      HuBERT front end, x3_variant 7: 1 = the post-attention LayerNorm folded into
 *                  the GEMMs (out_proj emits per-row mean / M2 partials, fc1 runs on the
 *                  un-normalised rows with gamma in W, fc2 normalises its residual on the fly;
 *                  12 fewer launches per forward, measured neutral), 0 = LayerNorm kernels (default).
 *                  fc1's fold computes (W'u - mu colsum(W')) rstd: rows whose |mean| is far above
 *                  their std cancel there (fp32), which is one reason it stays off by default
 *   "tail_batch"   HuBERT front end: 1 = when the feature extractor runs in utterance chunks
 *                  (conv0 output > 2 GiB), CNN layers 4-6 run once over the whole batch
 *                  (default), 0 = per chunk; same per-row arithmetic, bit-identical rows
 *   "layer"        HuBERT front end only, before finalize: -1 = weighted sum of all
 *                  hidden states (default), k = hidden state k alone (s3prl.py:84-87)
 * Deprecated (accepted, mapped to the shipped kernels since r3 pruned the others):
 *   "attn_lds" and "conv1x1_rows" (any value: no effect), "astp_fused" 2 / 3 (= 1),
 *   "x3_variant" 0 / 1 / 2 / 9 (= 5), 8 (= 7). */
int wsp_model_set_option(wsp_model* m, const char* key, int value);
/* The current value of a runtime option above (the per-architecture default until set). */
int wsp_model_get_option(const wsp_model* m, const char* key, int* value);

/* Per-kernel-class timing with HIP events recorded on the launch stream
 * around every launch (used by bench.py for the roofline figure). */
int wsp_model_profile(wsp_model* m, int enable);
/* Synchronises the events; returns launches, summed ms and algorithmic
 * FLOPs per launch (mean over the launches) of the named kernel class, then clears it. */
int wsp_model_profile_query(wsp_model* m, const char* kernel_class, int* launches,
                            double* total_ms, double* flops_per_launch);

/* ----------------------------------------------- SSL front end (HuBERT) --- */
/* Replaces S3prlFrontend.forward (wespeaker/frontend/s3prl.py:80-93): s3prl
 * HuBERT-base upstream -> Featurizer (softmax-weighted sum of the 13 hidden
 * states, or the single state chosen with wsp_model_set_option(m, "layer", k)
 * before finalize) -> s3prl length match, optionally followed by
 * bin/extract.py:104-106's apply_cmvn (cmn = 1).  Handles come from
 * wsp_model_create("HuBERT_base", 1, 768, 0, 0, &m); parameters are the
 * reference checkpoint's "frontend.*" entries. */
/* Frames per utterance: len(range(0, num_samples, 320)). num_samples >= 1; inputs
 * shorter than 800 samples run zero-padded to 800 (s3prl MIN_SECOND = 0.05 s). */
int wsp_frontend_out_frames(const wsp_model* m, int num_samples, int* frames);
int wsp_frontend_workspace_bytes(const wsp_model* m, int B, int num_samples, size_t* bytes);
/* wav [B][num_samples] f32 in [-1, 1] (bin/extract.py:100-102: not x32768)
 * -> feats [B][frames][768] f32.  Asynchronous on `stream`. */
int wsp_frontend_forward(wsp_model* m, const float* wav, int B, int num_samples, float* feats, int cmn,
                         void* workspace, size_t workspace_bytes, void* stream);

/* Ragged batch: B whole utterances concatenated in `wav` (device), utterance b =
 * num_samples[b] samples (HOST int32 array, each >= 1) -> feats rows
 * [frame_offsets[b], frame_offsets[b+1]) of [sum_b ceil(num_samples[b]/320)][768]
 * (frame_offsets: HOST int32 [B+1] output, may be NULL).  Each utterance's rows
 * equal its batch-of-one result (conv padding, attention, length match, CMN per
 * utterance). */
int wsp_frontend_workspace_bytes_segments(const wsp_model* m, int B, const int32_t* num_samples, size_t* bytes);
int wsp_frontend_forward_segments(wsp_model* m, const float* wav, int B, const int32_t* num_samples, float* feats,
                                  int32_t* frame_offsets, int cmn, void* workspace, size_t workspace_bytes,
                                  void* stream);

/* Per-row mean subtraction over frames, in place: x [B][T][D] f32, x[b][t][:] -=
 * mean_t x[b][t][:].  Replaces the subsegment CMN of Speaker.extract_embedding_feats
 * (wespeaker/cli/speaker.py:106-110, np.mean over axis 1) and apply_cmvn(norm_mean)
 * (wespeaker/dataset/dataset_utils.py:19-26) on feature tensors already on the device. */
int wsp_cmn(float* x, int B, int T, int D, void* stream);
/* apply_cmvn(feats, norm_mean, norm_var) of wespeaker/dataset/dataset_utils.py:19-26
 * as bin/extract.py:104-106 applies it with dataset_args.cmvn_args: per utterance,
 * x -= mean over frames (norm_mean), then x /= sqrt(var over frames (unbiased) +
 * 1e-7) (norm_var; T = 1 gives NaN, as torch.var).  x [B][T][D] in place, or a
 * ragged batch: frame_offsets = device int32 [B+1] row offsets (T ignored). */
int wsp_cmvn(float* x, int B, int T, int D, const int32_t* frame_offsets, int norm_mean, int norm_var,
             void* stream);

/* --------------------------------------------------------- resampling --- */
/* Replaces torchaudio.transforms.Resample(orig_freq, new_freq) as the reference
 * applies it before fbank (wespeaker/cli/speaker.py:155-157) and in the data
 * pipeline (wespeaker/dataset/processor.py:242-260): band-limited sinc with a
 * Hann window (torchaudio's default "sinc_interp_hann"; lowpass_filter_width 6,
 * rolloff 0.99 reproduce Resample's defaults).  create() builds the kernel on
 * the host; resample() maps
 * x [B][num_samples] (row stride ld) to y [B][out_len] (row stride ldy),
 * out_len = ceil(new * num_samples / orig) after reducing the rates by their gcd;
 * orig == new copies x. */
typedef struct wsp_resampler wsp_resampler;
int wsp_resampler_create(int orig_freq, int new_freq, int lowpass_filter_width, float rolloff,
                         wsp_resampler** out);
int wsp_resampler_destroy(wsp_resampler* r);
int wsp_resampler_out_len(const wsp_resampler* r, int num_samples, int* out_len);
int wsp_resample(const wsp_resampler* r, const float* x, int B, int num_samples, int ld, float* y, int ldy,
                 void* stream);
/* Host copy of the plan: reduced rates, half-width, taps per phase and (kernel
 * != NULL) the [reduced_new][taps] f32 kernel.  Creation is host-only; the
 * device copy is made by the first wsp_resample on the then-current device. */
int wsp_resampler_kernel(const wsp_resampler* r, int* reduced_orig, int* reduced_new, int* width, int* taps,
                         float* kernel);

/* ------------------------------------------------------------ scoring --- */
/* y[r] = x[r] - sub (sub may be NULL), then L2-normalised; [R][D] f32. */
int wsp_l2_normalize(const float* x, const float* sub, float* y, int R, int D, void* stream);
/* score[p] = cos(E[idx_a[p]], E[idx_b[p]]) for P pairs (E rows need not be
 * normalised; accumulation in f64 like sklearn). */
int wsp_cosine_pairs(const float* E, int D, const int32_t* idx_a, const int32_t* idx_b,
                     int P, double* score, void* stream);
/* AS-Norm statistics (get_mean_std): E [Ne][D], C [Nc][D] (both already
 * L2-normalised), top_n <= Nc.  mu/sd [Ne] f64 (sd: population std). */
int wsp_asnorm_stats(const float* E, int Ne, const float* C, int Nc, int D, int top_n,
                     double* mu, double* sd, void* workspace, size_t workspace_bytes,
                     void* stream);
int wsp_asnorm_workspace_bytes(int Ne, int Nc, int D, size_t* bytes);
/* acc[group[r]][:] += x[r][:] (f64), cnt[group[r]] += 1 — per-speaker /
 * global embedding sums for mean vectors and cohorts. */
int wsp_row_mean_accum(const float* x, const int32_t* group, int R, int D, double* acc,
                       double* cnt, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WESPEAKER_AMD_H_ */
