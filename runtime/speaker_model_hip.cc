// HipSpeakerModel / HipSpeakerEngine over the C-ABI (see speaker_model_hip.h).
#include "speaker_model_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>
#include <numeric>
#include <stdexcept>

namespace wespeaker {

namespace {

void Check(int status, const char* what) {
  if (status != WSP_OK) throw std::runtime_error(std::string(what) + ": " + wsp_last_error());
}
void CheckHip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// ---- tiny JSON reader for the safetensors header ({"name": {"dtype": "F32",
// "shape": [..], "data_offsets": [b, e]}, "__metadata__": {"k": "v"}}) ----
struct Json {
  const std::string& s;
  size_t i = 0;
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("safetensors header: ") + m); }
  void expect(char c) {
    ws();
    if (i >= s.size() || s[i] != c) fail("unexpected character");
    ++i;
  }
  bool peek(char c) {
    ws();
    return i < s.size() && s[i] == c;
  }
  std::string str() {
    expect('"');
    std::string out;
    while (i < s.size() && s[i] != '"') {
      if (s[i] == '\\') {
        if (++i >= s.size()) fail("bad escape");
        const char e = s[i];
        out += e == 'n' ? '\n' : e == 't' ? '\t' : e;  // names / metadata are plain ASCII
      } else {
        out += s[i];
      }
      ++i;
    }
    expect('"');
    return out;
  }
  long long num() {
    ws();
    size_t j = i;
    while (j < s.size() && (isdigit((unsigned char)s[j]) || s[j] == '-')) ++j;
    if (j == i) fail("number expected");
    const long long v = std::stoll(s.substr(i, j - i));
    i = j;
    return v;
  }
  std::vector<long long> nums() {
    std::vector<long long> v;
    expect('[');
    if (peek(']')) {
      ++i;
      return v;
    }
    for (;;) {
      v.push_back(num());
      if (peek(',')) {
        ++i;
        continue;
      }
      expect(']');
      return v;
    }
  }
};

}  // namespace

SafeTensors SafeTensors::Load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open model file " + path);
  uint64_t hlen = 0;
  f.read(reinterpret_cast<char*>(&hlen), 8);
  if (!f || hlen == 0 || hlen > (1u << 26)) throw std::runtime_error(path + ": not a safetensors file");
  std::string header(hlen, '\0');
  f.read(&header[0], (std::streamsize)hlen);
  SafeTensors st;
  st.data.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  Json j{header};
  j.expect('{');
  if (j.peek('}')) return st;
  for (;;) {
    const std::string key = j.str();
    j.expect(':');
    j.expect('{');
    if (key == "__metadata__") {
      if (!j.peek('}')) {
        for (;;) {
          const std::string k = j.str();
          j.expect(':');
          st.metadata[k] = j.str();
          if (j.peek(',')) {
            ++j.i;
            continue;
          }
          break;
        }
      }
      j.expect('}');
    } else {
      Tensor t;
      std::string dtype;
      std::vector<long long> offs;
      for (;;) {
        const std::string field = j.str();
        j.expect(':');
        if (field == "dtype") dtype = j.str();
        else if (field == "shape") for (long long d : j.nums()) t.shape.push_back(d);
        else if (field == "data_offsets") offs = j.nums();
        else j.fail("unknown tensor field");
        if (j.peek(',')) {
          ++j.i;
          continue;
        }
        break;
      }
      j.expect('}');
      if (dtype != "F32") throw std::runtime_error(path + ": tensor " + key + " is " + dtype + " (F32 expected)");
      if (offs.size() != 2 || offs[0] < 0 || offs[1] < offs[0] || (size_t)offs[1] > st.data.size())
        throw std::runtime_error(path + ": bad data_offsets for " + key);
      t.begin = (size_t)offs[0];
      t.end = (size_t)offs[1];
      st.tensors[key] = t;
    }
    if (j.peek(',')) {
      ++j.i;
      continue;
    }
    j.expect('}');
    break;
  }
  return st;
}

// ------------------------------------------------------------------ model --
HipSpeakerModel::HipSpeakerModel(const std::string& model_path, int device) : device_(device) {
  SafeTensors st = SafeTensors::Load(model_path);
  auto meta = [&](const char* k, const char* dflt) -> std::string {
    auto it = st.metadata.find(k);
    if (it != st.metadata.end()) return it->second;
    if (dflt) return dflt;
    throw std::runtime_error(model_path + ": metadata '" + k + "' missing (export with bin/export_hip)");
  };
  arch_ = meta("arch", nullptr);
  feat_dim_ = std::stoi(meta("feat_dim", nullptr));
  embed_dim_ = std::stoi(meta("embed_dim", nullptr));
  const int emb_bn = std::stoi(meta("emb_bn", "0"));
  const int two_emb = std::stoi(meta("two_emb_layer", "0"));
  CheckHip(hipSetDevice(device_), "hipSetDevice");
  Check(wsp_model_create(arch_.c_str(), feat_dim_, embed_dim_, emb_bn, two_emb, &model_), "wsp_model_create");
  const int n = wsp_model_num_params(model_);
  for (int i = 0; i < n; ++i) {
    const char* name = nullptr;
    int ndim = 0;
    int64_t shape[4] = {0, 0, 0, 0};
    Check(wsp_model_param_info(model_, i, &name, &ndim, shape), "wsp_model_param_info");
    const std::string key(name);
    if (key.size() >= 19 && key.compare(key.size() - 19, 19, "num_batches_tracked") == 0) continue;
    auto it = st.tensors.find(key);
    if (it == st.tensors.end()) throw std::runtime_error(model_path + ": missing tensor " + key);
    int64_t numel = 1;
    for (int d = 0; d < ndim; ++d) numel *= shape[d];
    const auto& t = it->second;
    if ((int64_t)t.shape.size() != ndim || !std::equal(t.shape.begin(), t.shape.end(), shape))
      throw std::runtime_error(model_path + ": shape mismatch for " + key);
    if ((int64_t)(t.end - t.begin) != numel * 4) throw std::runtime_error(model_path + ": size mismatch for " + key);
    std::vector<float> host((size_t)numel);
    std::memcpy(host.data(), st.data.data() + t.begin, (size_t)numel * 4);  // unaligned-safe copy
    Check(wsp_model_set_param(model_, i, host.data(), numel), "wsp_model_set_param");
  }
  Check(wsp_model_finalize(model_), "wsp_model_finalize");
  hipStream_t s;
  CheckHip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
}

HipSpeakerModel::~HipSpeakerModel() {
  (void)hipSetDevice(device_);
  if (d_feats_) (void)hipFree(d_feats_);
  if (d_emb_) (void)hipFree(d_emb_);
  if (d_ws_) (void)hipFree(d_ws_);
  if (stream_) (void)hipStreamDestroy(static_cast<hipStream_t>(stream_));
  if (model_) wsp_model_destroy(model_);
}

void HipSpeakerModel::Reserve(size_t feat_floats, size_t emb_floats, size_t ws_bytes) {
  auto grow = [](void** p, size_t* cap, size_t need, const char* what) {
    if (need <= *cap) return;
    if (*p) CheckHip(hipFree(*p), "hipFree");
    *p = nullptr;
    CheckHip(hipMalloc(p, need), what);
    *cap = need;
  };
  grow(reinterpret_cast<void**>(&d_feats_), &cap_feats_, feat_floats * 4, "hipMalloc feats");
  grow(reinterpret_cast<void**>(&d_emb_), &cap_emb_, emb_floats * 4, "hipMalloc embed");
  grow(&d_ws_, &cap_ws_, std::max<size_t>(ws_bytes, 256), "hipMalloc workspace");
}

void HipSpeakerModel::ExtractEmbeddingBatch(const float* feats, int B, int T, std::vector<float>* embeds) {
  if (B <= 0 || T <= 0) throw std::invalid_argument("ExtractEmbeddingBatch: empty batch");
  CheckHip(hipSetDevice(device_), "hipSetDevice");
  size_t ws = 0;
  Check(wsp_model_workspace_bytes(model_, B, T, &ws), "wsp_model_workspace_bytes");
  const size_t nf = (size_t)B * T * feat_dim_;
  Reserve(nf, (size_t)B * embed_dim_, ws);
  hipStream_t s = static_cast<hipStream_t>(stream_);
  CheckHip(hipMemcpyAsync(d_feats_, feats, nf * 4, hipMemcpyHostToDevice, s), "H2D feats");
  Check(wsp_model_forward(model_, d_feats_, B, T, d_emb_, d_ws_, cap_ws_, s), "wsp_model_forward");
  embeds->resize((size_t)B * embed_dim_);
  CheckHip(hipMemcpyAsync(embeds->data(), d_emb_, embeds->size() * 4, hipMemcpyDeviceToHost, s), "D2H embed");
  CheckHip(hipStreamSynchronize(s), "hipStreamSynchronize");
}

void HipSpeakerModel::ExtractEmbedding(const std::vector<std::vector<float>>& feats, std::vector<float>* embed) {
  if (feats.empty()) throw std::invalid_argument("ExtractEmbedding: no frames");
  const int T = (int)feats.size();
  std::vector<float> flat((size_t)T * feat_dim_);
  for (int t = 0; t < T; ++t) {
    if ((int)feats[t].size() != feat_dim_) throw std::invalid_argument("ExtractEmbedding: feature dim mismatch");
    std::copy(feats[t].begin(), feats[t].end(), flat.begin() + (size_t)t * feat_dim_);
  }
  std::vector<float> out;
  ExtractEmbeddingBatch(flat.data(), 1, T, &out);
  embed->assign(out.begin(), out.end());
}

// ----------------------------------------------------------------- engine --
HipSpeakerEngine::HipSpeakerEngine(const std::string& model_path, int feat_dim, int sample_rate,
                                   int embedding_size, int samples_per_chunk, int device)
    : feat_dim_(feat_dim), sample_rate_(sample_rate), per_chunk_samples_(samples_per_chunk) {
  // FeaturePipelineConfig(num_bins, sample_rate): 25 / 10 ms frames (feature_pipeline.h:35-39)
  wsp_fbank_opts o;
  wsp_fbank_opts_default(&o);
  o.num_mel_bins = feat_dim;
  o.sample_rate = sample_rate;
  Check(wsp_fbank_geometry(&o, &frame_len_, &frame_shift_, nullptr), "wsp_fbank_geometry");
  model_ = std::make_unique<HipSpeakerModel>(model_path, device);
  if (model_->FeatDim() != feat_dim) throw std::invalid_argument("HipSpeakerEngine: model feat_dim differs");
  embedding_size_ = model_->EmbedDim();
  if (embedding_size > 0 && embedding_size != embedding_size_)
    throw std::invalid_argument("HipSpeakerEngine: embedding_size differs from the model's");
  hipStream_t s;
  CheckHip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
}

void HipSpeakerEngine::ExtractFeature(const int16_t* data, int data_size,
                                      std::vector<std::vector<std::vector<float>>>* chunks_feat) {
  if (!data) throw std::invalid_argument("ExtractFeature: input is nullptr");
  const int T = wsp_fbank_num_frames(data_size, frame_len_, frame_shift_);
  if (T <= 0) throw std::invalid_argument("ExtractFeature: fewer samples than one frame");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  auto grow = [](void** p, size_t* cap, size_t need) {
    if (need <= *cap) return;
    if (*p) CheckHip(hipFree(*p), "hipFree");
    *p = nullptr;
    CheckHip(hipMalloc(p, need), "hipMalloc");
    *cap = need;
  };
  grow(&d_wav_, &cap_wav_, (size_t)data_size * 2);
  grow(reinterpret_cast<void**>(&d_fbank_), &cap_fbank_, (size_t)T * feat_dim_ * 4);
  CheckHip(hipMemcpyAsync(d_wav_, data, (size_t)data_size * 2, hipMemcpyHostToDevice, s), "H2D wav");
  Check(wsp_fbank(d_wav_, WSP_DTYPE_S16, 1, data_size, data_size, 1.0f, d_fbank_, feat_dim_, sample_rate_,
                  WSP_WINDOW_HAMMING, 0, s),
        "wsp_fbank");
  std::vector<float> fb((size_t)T * feat_dim_);
  CheckHip(hipMemcpyAsync(fb.data(), d_fbank_, fb.size() * 4, hipMemcpyDeviceToHost, s), "D2H fbank");
  CheckHip(hipStreamSynchronize(s), "hipStreamSynchronize");
  auto row = [&](int t) { return std::vector<float>(fb.begin() + (size_t)t * feat_dim_, fb.begin() + (size_t)(t + 1) * feat_dim_); };
  if (per_chunk_samples_ <= 0) {  // full mode
    std::vector<std::vector<float>> c;
    for (int t = 0; t < T; ++t) c.push_back(row(t));
    chunks_feat->push_back(std::move(c));
    return;
  }
  const int chunk = 1 + (per_chunk_samples_ - sample_rate_ / 1000 * 25) / (sample_rate_ / 1000 * 10);
  int t = 0;
  for (; t + chunk <= T; t += chunk) {
    std::vector<std::vector<float>> c;
    for (int k = 0; k < chunk; ++k) c.push_back(row(t + k));
    chunks_feat->push_back(std::move(c));
  }
  const int last = T - t;
  if (last > 0) {
    std::vector<std::vector<float>> c;
    for (int k = 0; k < last; ++k) c.push_back(row(t + k));
    if (chunks_feat->empty()) {  // utterance shorter than a chunk: repeat it, then top up
      const int reps = chunk / last;
      for (int r = 1; r < reps; ++r)
        for (int k = 0; k < last; ++k) {
          std::vector<float> v = c[k];
          c.push_back(std::move(v));
        }
      const size_t have = c.size();
      for (size_t k = 0; have + k < (size_t)chunk; ++k) {
        std::vector<float> v = c[k];
        c.push_back(std::move(v));
      }
    } else {  // tail: top up with the first chunk's leading frames
      const auto& first = (*chunks_feat)[0];
      for (size_t k = 0; c.size() < (size_t)chunk; ++k) c.push_back(first[k]);
    }
    chunks_feat->push_back(std::move(c));
  }
}

void HipSpeakerEngine::ExtractEmbedding(const int16_t* data, int data_size, std::vector<float>* avg_emb) {
  std::vector<std::vector<std::vector<float>>> chunks;
  ExtractFeature(data, data_size, &chunks);
  const int n = (int)chunks.size();
  const int T = (int)chunks[0].size();
  // per-chunk mean subtraction (speaker_engine.cc:64-75), then one batched forward
  std::vector<float> flat((size_t)n * T * feat_dim_);
  for (int c = 0; c < n; ++c) {
    std::vector<float> mean(feat_dim_, 0.f);
    for (const auto& fr : chunks[c])
      for (int d = 0; d < feat_dim_; ++d) mean[d] += fr[d];
    for (int d = 0; d < feat_dim_; ++d) mean[d] /= (float)chunks[c].size();
    for (int t = 0; t < T; ++t)
      for (int d = 0; d < feat_dim_; ++d)
        flat[((size_t)c * T + t) * feat_dim_ + d] = chunks[c][t][d] - mean[d];
  }
  std::vector<float> embs;
  model_->ExtractEmbeddingBatch(flat.data(), n, T, &embs);
  avg_emb->assign(embedding_size_, 0.f);
  for (int c = 0; c < n; ++c)
    for (int j = 0; j < embedding_size_; ++j) (*avg_emb)[j] += embs[(size_t)c * embedding_size_ + j];
  for (auto& v : *avg_emb) v /= (float)n;
}

float HipSpeakerEngine::CosineSimilarity(const std::vector<float>& emb1, const std::vector<float>& emb2) {
  if (emb1.size() != emb2.size()) throw std::invalid_argument("CosineSimilarity: size mismatch");
  float dot = std::inner_product(emb1.begin(), emb1.end(), emb2.begin(), 0.0);
  const float n1 = std::inner_product(emb1.begin(), emb1.end(), emb1.begin(), 0.0);
  const float n2 = std::inner_product(emb2.begin(), emb2.end(), emb2.begin(), 0.0);
  dot /= std::max(std::sqrt(n1) * std::sqrt(n2), std::numeric_limits<float>::epsilon());
  return (dot + 1.0f) / 2.0f;  // [-1, 1] -> [0, 1]
}

// -------------------------------------------------------------------- wav --
std::vector<int16_t> ReadWavPcm16(const std::string& path, int* sample_rate) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  auto u32 = [&](size_t o) { uint32_t v; std::memcpy(&v, b.data() + o, 4); return v; };
  auto u16 = [&](size_t o) { uint16_t v; std::memcpy(&v, b.data() + o, 2); return v; };
  if (b.size() < 12 || std::memcmp(b.data(), "RIFF", 4) || std::memcmp(b.data() + 8, "WAVE", 4))
    throw std::runtime_error(path + ": not a RIFF/WAVE file");
  size_t o = 12;
  int channels = 0, bits = 0;
  *sample_rate = 0;
  while (o + 8 <= b.size()) {
    const uint32_t sz = u32(o + 4);
    if (!std::memcmp(b.data() + o, "fmt ", 4) && o + 24 <= b.size()) {
      channels = u16(o + 10);
      *sample_rate = (int)u32(o + 12);
      bits = u16(o + 22);
    } else if (!std::memcmp(b.data() + o, "data", 4)) {
      if (channels != 1 || bits != 16) throw std::runtime_error(path + ": only 16-bit mono PCM is supported");
      const size_t n = std::min<size_t>(sz, b.size() - o - 8) / 2;
      std::vector<int16_t> pcm(n);
      std::memcpy(pcm.data(), b.data() + o + 8, n * 2);
      return pcm;
    }
    o += 8 + sz + (sz & 1);
  }
  throw std::runtime_error(path + ": no data chunk");
}

}  // namespace wespeaker
