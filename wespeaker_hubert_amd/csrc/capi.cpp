// extern "C" boundary (include/wespeaker_amd.h): argument checks, exception
// -> status translation, thread-local last error.
#include "../../include/wespeaker_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"
#include "model.h"

namespace wsp {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
const std::string& get_error() { return g_err; }

// fbank plans (tables computed on the host at first use, one device copy per
// device and configuration; never freed: a handful of KB per configuration)
static const FbankPlan& fbank_plan_dev(const FbankConfig& c) {
  static std::mutex mu;
  static std::vector<std::unique_ptr<FbankPlan>> plans;
  static std::vector<int> devs;
  int dev = 0;
  WSP_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  for (size_t i = 0; i < plans.size(); ++i) {
    const FbankConfig& q = plans[i]->cfg;
    if (devs[i] == dev && q.num_bins == c.num_bins && q.sample_rate == c.sample_rate && q.window == c.window &&
        q.frame_length_ms == c.frame_length_ms && q.frame_shift_ms == c.frame_shift_ms &&
        q.low_freq == c.low_freq && q.high_freq == c.high_freq)
      return *plans[i];
  }
  auto p = std::make_unique<FbankPlan>();
  fbank_plan(c, *p);
  double* d = nullptr;
  WSP_HIP(hipMalloc(&d, p->host_tab.size() * sizeof(double)));
  WSP_HIP(hipMemcpy(d, p->host_tab.data(), p->host_tab.size() * sizeof(double), hipMemcpyHostToDevice));
  p->tab = d;
  plans.push_back(std::move(p));
  devs.push_back(dev);
  return *plans.back();
}

static FbankConfig fbank_config(const wsp_fbank_opts* o) {
  WSP_CHECK(o != nullptr, "fbank: null options");
  FbankConfig c;
  c.num_bins = o->num_mel_bins;
  c.sample_rate = o->sample_rate;
  c.frame_length_ms = o->frame_length_ms;
  c.frame_shift_ms = o->frame_shift_ms;
  c.window = o->window_type;
  c.low_freq = o->low_freq;
  c.high_freq = o->high_freq;
  fbank_config_resolve(c);
  return c;
}
}  // namespace wsp

struct wsp_model {
  wsp::Model m;
};

#define WSP_GUARD(...)                                                           \
  try {                                                                          \
    __VA_ARGS__;                                                                      \
    return WSP_OK;                                                               \
  } catch (const wsp::InvalidArg& e) {                                           \
    wsp::set_error(e.msg);                                                       \
    return WSP_E_INVALID;                                                        \
  } catch (const wsp::HipError& e) {                                             \
    wsp::set_error(std::string("HIP error ") + hipGetErrorString(e.err) + " at " + e.where); \
    return WSP_E_HIP;                                                            \
  } catch (const std::exception& e) {                                            \
    wsp::set_error(e.what());                                                    \
    return WSP_E_STATE;                                                          \
  }

static hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

extern "C" {

int wsp_abi_version(void) { return 1; }
const char* wsp_last_error(void) { return wsp::get_error().c_str(); }

int wsp_fbank_num_frames(int num_samples, int frame_len, int frame_shift) {
  if (frame_len <= 0 || frame_shift <= 0 || num_samples < frame_len) return 0;
  return 1 + (num_samples - frame_len) / frame_shift;
}

int wsp_fbank_opts_default(wsp_fbank_opts* o) {
  if (!o) return WSP_E_INVALID;
  o->num_mel_bins = 80;
  o->sample_rate = 16000;
  o->frame_length_ms = 25.0;
  o->frame_shift_ms = 10.0;
  o->window_type = WSP_WINDOW_HAMMING;
  o->low_freq = 20.0;
  o->high_freq = 0.0;
  return WSP_OK;
}

int wsp_fbank_geometry(const wsp_fbank_opts* o, int* frame_len, int* frame_shift, int* padded) {
  WSP_GUARD({
    const wsp::FbankConfig c = wsp::fbank_config(o);
    wsp::FbankPlan p;  // host tables only: rejects filters the kernel's LDS table cannot hold
    wsp::fbank_plan(c, p);
    if (frame_len) *frame_len = c.frame_len;
    if (frame_shift) *frame_shift = c.frame_shift;
    if (padded) *padded = c.padded;
  });
}

int wsp_fbank_mel_banks(const wsp_fbank_opts* o, float* banks) {
  WSP_GUARD({
    WSP_CHECK(banks != nullptr, "fbank: null output");
    std::vector<float> w;
    wsp::fbank_mel_banks(wsp::fbank_config(o), w);
    std::copy(w.begin(), w.end(), banks);
  });
}

int wsp_fbank_ex(const void* wav, int wav_dtype, int B, int num_samples, int ld, float scale, float* feats,
                 const wsp_fbank_opts* opts, int cmn, void* stream) {
  WSP_GUARD({
    const wsp::FbankConfig c = wsp::fbank_config(opts);
    WSP_CHECK(wav_dtype == WSP_DTYPE_F32 || wav_dtype == WSP_DTYPE_S16, "fbank: bad dtype");
    WSP_CHECK(B >= 0 && num_samples >= 0 && ld >= num_samples, "fbank: bad shape");
    const int T = wsp_fbank_num_frames(num_samples, c.frame_len, c.frame_shift);
    if (B > 0 && T > 0) {
      WSP_CHECK(wav && feats, "fbank: null pointer");
      wsp::launch_fbank(wav, wav_dtype, B, num_samples, ld, scale, feats, T, cmn, wsp::fbank_plan_dev(c), S(stream));
    }
  });
}

int wsp_fbank(const void* wav, int wav_dtype, int B, int num_samples, int ld, float scale,
              float* feats, int num_bins, int sample_rate, int window_type, int cmn,
              void* stream) {
  wsp_fbank_opts o;
  wsp_fbank_opts_default(&o);
  o.num_mel_bins = num_bins;
  o.sample_rate = sample_rate;
  o.window_type = window_type;
  return wsp_fbank_ex(wav, wav_dtype, B, num_samples, ld, scale, feats, &o, cmn, stream);
}

int wsp_fbank_segments_ex(const void* wav, int wav_dtype, int B, const int32_t* sample_offsets,
                          const int32_t* frame_offsets, int max_frames, float scale, float* feats,
                          const wsp_fbank_opts* opts, int cmn, void* stream) {
  WSP_GUARD({
    const wsp::FbankConfig c = wsp::fbank_config(opts);
    WSP_CHECK(wav_dtype == WSP_DTYPE_F32 || wav_dtype == WSP_DTYPE_S16, "fbank: bad dtype");
    WSP_CHECK(B >= 0 && max_frames >= 0, "fbank: bad shape");
    if (B > 0 && max_frames > 0) {
      WSP_CHECK(wav && feats && sample_offsets && frame_offsets, "fbank: null pointer");
      wsp::launch_fbank(wav, wav_dtype, B, 0, 0, scale, feats, max_frames, cmn, wsp::fbank_plan_dev(c), S(stream),
                        sample_offsets, frame_offsets);
    }
  });
}

int wsp_fbank_segments(const void* wav, int wav_dtype, int B, const int32_t* sample_offsets,
                       const int32_t* frame_offsets, int max_frames, float scale, float* feats, int num_bins,
                       int sample_rate, int window_type, int cmn, void* stream) {
  wsp_fbank_opts o;
  wsp_fbank_opts_default(&o);
  o.num_mel_bins = num_bins;
  o.sample_rate = sample_rate;
  o.window_type = window_type;
  return wsp_fbank_segments_ex(wav, wav_dtype, B, sample_offsets, frame_offsets, max_frames, scale, feats, &o, cmn,
                               stream);
}

int wsp_model_create(const char* arch, int feat_dim, int embed_dim, int emb_bn, int two_emb_layer,
                     wsp_model** out) {
  WSP_GUARD({
    WSP_CHECK(arch && out, "null argument");
    auto* h = new wsp_model();
    try {
      h->m.create(arch, feat_dim, embed_dim, emb_bn != 0, two_emb_layer != 0);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int wsp_model_destroy(wsp_model* m) {
  delete m;
  return WSP_OK;
}

int wsp_model_num_params(const wsp_model* m) { return m ? m->m.num_params() : WSP_E_INVALID; }

int wsp_model_param_info(const wsp_model* m, int index, const char** name, int* ndim,
                         int64_t shape[4]) {
  WSP_GUARD({
    WSP_CHECK(m && name && ndim && shape, "null argument");
    m->m.param_info(index, name, ndim, shape);
  });
}

int wsp_model_set_param(wsp_model* m, int index, const float* host_data, int64_t numel) {
  WSP_GUARD({
    WSP_CHECK(m && (host_data || numel == 0), "null argument");
    m->m.set_param(index, host_data, numel);
  });
}

int wsp_model_finalize(wsp_model* m) {
  WSP_GUARD({
    WSP_CHECK(m, "null model");
    m->m.finalize();
  });
}

int wsp_model_embed_dim(const wsp_model* m) { return m ? m->m.embed_dim() : WSP_E_INVALID; }
int wsp_model_feat_dim(const wsp_model* m) { return m ? m->m.feat_dim() : WSP_E_INVALID; }

int wsp_model_workspace_bytes(const wsp_model* m, int B, int T, size_t* bytes) {
  WSP_GUARD({
    WSP_CHECK(m && bytes && B >= 0 && T >= 0, "bad argument");
    *bytes = m->m.workspace_bytes(B, T);
  });
}

int wsp_model_forward(wsp_model* m, const float* feats, int B, int T, float* embed, void* workspace,
                      size_t workspace_bytes, void* stream) {
  WSP_GUARD({
    WSP_CHECK(m && feats && embed && workspace, "null argument");
    m->m.forward(feats, B, T, embed, workspace, workspace_bytes, S(stream));
  });
}

int wsp_frontend_out_frames(const wsp_model* m, int num_samples, int* frames) {
  WSP_GUARD({
    WSP_CHECK(m && frames, "null argument");
    *frames = m->m.out_frames(num_samples);
  });
}

int wsp_frontend_workspace_bytes(const wsp_model* m, int B, int num_samples, size_t* bytes) {
  WSP_GUARD({
    WSP_CHECK(m && bytes, "null argument");
    *bytes = m->m.frontend_workspace_bytes(B, num_samples);
  });
}

int wsp_frontend_forward(wsp_model* m, const float* wav, int B, int num_samples, float* feats, int cmn,
                         void* workspace, size_t workspace_bytes, void* stream) {
  WSP_GUARD({
    WSP_CHECK(m && wav && feats && workspace, "null argument");
    m->m.forward_frontend(wav, B, num_samples, feats, cmn, workspace, workspace_bytes, S(stream));
  });
}

int wsp_model_workspace_bytes_segments(const wsp_model* m, int B, int total_frames, size_t* bytes) {
  WSP_GUARD({
    WSP_CHECK(m && bytes, "null argument");
    *bytes = m->m.workspace_bytes_segments(B, total_frames);
  });
}

int wsp_model_forward_segments(wsp_model* m, const float* feats, int B, const int32_t* frame_offsets,
                               int total_frames, float* embed, void* workspace, size_t workspace_bytes,
                               void* stream) {
  WSP_GUARD({
    WSP_CHECK(m && feats && frame_offsets && embed && workspace, "null argument");
    m->m.forward_segments(feats, B, frame_offsets, total_frames, embed, workspace, workspace_bytes, S(stream));
  });
}

int wsp_frontend_workspace_bytes_segments(const wsp_model* m, int B, const int32_t* num_samples, size_t* bytes) {
  WSP_GUARD({
    WSP_CHECK(m && num_samples && bytes, "null argument");
    *bytes = m->m.frontend_workspace_bytes_segments(B, num_samples);
  });
}

int wsp_frontend_forward_segments(wsp_model* m, const float* wav, int B, const int32_t* num_samples, float* feats,
                                  int32_t* frame_offsets, int cmn, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  WSP_GUARD({
    WSP_CHECK(m && wav && num_samples && feats && workspace, "null argument");
    m->m.forward_frontend_segments(wav, B, num_samples, feats, frame_offsets, cmn, workspace, workspace_bytes,
                                   S(stream));
  });
}

int wsp_model_set_option(wsp_model* m, const char* key, int value) {
  WSP_GUARD({
    WSP_CHECK(m && key, "null argument");
    m->m.set_option(key, value);
  });
}

int wsp_model_get_option(const wsp_model* m, const char* key, int* value) {
  WSP_GUARD({
    WSP_CHECK(m && key && value, "null argument");
    *value = m->m.get_option(key);
  });
}

int wsp_model_profile(wsp_model* m, int enable) {
  WSP_GUARD({
    WSP_CHECK(m, "null model");
    m->m.profile(enable != 0);
  });
}

int wsp_model_profile_query(wsp_model* m, const char* kernel_class, int* launches,
                            double* total_ms, double* flops_per_launch) {
  WSP_GUARD({
    WSP_CHECK(m && kernel_class && launches && total_ms && flops_per_launch, "null argument");
    m->m.profile_query(kernel_class, launches, total_ms, flops_per_launch);
  });
}

struct wsp_resampler {
  wsp::ResamplePlan plan;
  // device copy of the kernel table, made on the first wsp_resample call
  // (creation is host-only, like wsp_model_create)
  mutable std::mutex mu;
  mutable int device = -1;
  mutable float* kern = nullptr;
  mutable int* band = nullptr;
};

int wsp_resampler_create(int orig_freq, int new_freq, int lowpass_filter_width, float rolloff,
                         wsp_resampler** out) {
  WSP_GUARD({
    WSP_CHECK(out != nullptr, "bad argument");
    *out = nullptr;
    auto r = std::make_unique<wsp_resampler>();
    wsp::resample_plan(orig_freq, new_freq, lowpass_filter_width, rolloff, r->plan);
    *out = r.release();
  });
}

int wsp_resampler_destroy(wsp_resampler* r) {
  WSP_GUARD({
    if (r) {
      if (r->kern) (void)hipFree(r->kern);
      if (r->band) (void)hipFree(r->band);
      delete r;
    }
  });
}

int wsp_resampler_out_len(const wsp_resampler* r, int num_samples, int* out_len) {
  WSP_GUARD({
    WSP_CHECK(r && out_len && num_samples >= 0, "bad argument");
    const long long n = wsp::resample_out_len(r->plan, num_samples);
    WSP_CHECK(n < (1LL << 31), "output too long");
    *out_len = (int)n;
  });
}

int wsp_resampler_kernel(const wsp_resampler* r, int* reduced_orig, int* reduced_new, int* width, int* taps,
                         float* kernel) {
  WSP_GUARD({
    WSP_CHECK(r != nullptr, "bad argument");
    if (reduced_orig) *reduced_orig = r->plan.orig;
    if (reduced_new) *reduced_new = r->plan.nw;
    if (width) *width = r->plan.width;
    if (taps) *taps = r->plan.L;
    if (kernel && !r->plan.identity) std::copy(r->plan.kern.begin(), r->plan.kern.end(), kernel);
  });
}

int wsp_resample(const wsp_resampler* r, const float* x, int B, int num_samples, int ld, float* y, int ldy,
                 void* stream) {
  WSP_GUARD({
    WSP_CHECK(r && B >= 0 && num_samples >= 0 && (B == 0 || num_samples == 0 || (x && y)), "bad argument");
    int dev = -1;
    WSP_HIP(hipGetDevice(&dev));
    if (!r->plan.identity) {
      std::lock_guard<std::mutex> lk(r->mu);
      if (r->device < 0) {
        WSP_HIP(hipMalloc(&r->kern, r->plan.kern.size() * sizeof(float)));
        WSP_HIP(hipMalloc(&r->band, r->plan.band.size() * sizeof(int)));
        WSP_HIP(hipMemcpy(r->kern, r->plan.kern.data(), r->plan.kern.size() * sizeof(float),
                          hipMemcpyHostToDevice));
        WSP_HIP(hipMemcpy(r->band, r->plan.band.data(), r->plan.band.size() * sizeof(int), hipMemcpyHostToDevice));
        r->device = dev;
      }
      WSP_CHECK(dev == r->device, "resampler is bound to another device");
    }
    wsp::launch_resample(r->plan, r->kern, r->band, x, B, num_samples, ld, y, ldy, S(stream));
  });
}

int wsp_cmn(float* x, int B, int T, int D, void* stream) {
  WSP_GUARD({
    WSP_CHECK(B >= 0 && T > 0 && D > 0 && (B == 0 || x), "bad argument");
    if (B > 0) wsp::launch_cmn_rows(x, B, T, D, S(stream));
  });
}

int wsp_cmvn(float* x, int B, int T, int D, const int32_t* frame_offsets, int norm_mean, int norm_var,
             void* stream) {
  WSP_GUARD({
    WSP_CHECK(B >= 0 && D > 0 && (frame_offsets || T > 0) && (B == 0 || x), "bad argument");
    if (B > 0 && (norm_mean || norm_var))
      wsp::launch_cmvn_rows(x, B, T, D, norm_mean != 0, norm_var != 0, S(stream), frame_offsets);
  });
}

int wsp_l2_normalize(const float* x, const float* sub, float* y, int R, int D, void* stream) {
  WSP_GUARD({
    WSP_CHECK(R >= 0 && D > 0 && (R == 0 || (x && y)), "bad argument");
    wsp::launch_l2_normalize(x, sub, y, R, D, S(stream));
  });
}

int wsp_cosine_pairs(const float* E, int D, const int32_t* idx_a, const int32_t* idx_b, int P,
                     double* score, void* stream) {
  WSP_GUARD({
    WSP_CHECK(P >= 0 && D > 0 && (P == 0 || (E && idx_a && idx_b && score)), "bad argument");
    wsp::launch_cosine_pairs(E, D, idx_a, idx_b, P, score, S(stream));
  });
}

int wsp_asnorm_workspace_bytes(int Ne, int Nc, int D, size_t* bytes) {
  WSP_GUARD({
    WSP_CHECK(bytes && Ne >= 0 && Nc > 0 && D > 0, "bad argument");
    int a, b;
    wsp::asnorm_layout(Ne, Nc, D, &a, &b, bytes);
  });
}

int wsp_asnorm_stats(const float* E, int Ne, const float* C, int Nc, int D, int top_n, double* mu,
                     double* sd, void* workspace, size_t workspace_bytes, void* stream) {
  WSP_GUARD({
    WSP_CHECK(Ne >= 0 && Nc > 0 && D > 0, "bad argument");
    if (Ne == 0) return WSP_OK;
    int Ncp, Dp;
    size_t need;
    wsp::asnorm_layout(Ne, Nc, D, &Ncp, &Dp, &need);
    WSP_CHECK(workspace && workspace_bytes >= need, "asnorm: workspace too small");
    wsp::launch_asnorm_stats(E, Ne, C, Nc, D, top_n, mu, sd, static_cast<float*>(workspace),
                             S(stream));
  });
}

int wsp_row_mean_accum(const float* x, const int32_t* group, int R, int D, double* acc,
                       double* cnt, void* stream) {
  WSP_GUARD({
    WSP_CHECK(R >= 0 && D > 0 && (R == 0 || (x && group && acc && cnt)), "bad argument");
    wsp::launch_row_mean_accum(x, group, R, D, acc, cnt, S(stream));
  });
}

}  // extern "C"
