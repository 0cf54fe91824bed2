// C++ runtime backend on the MI355X path: a `wespeaker::SpeakerModel`
// implementation over libwsp_hip.so (include/wespeaker_amd.h), sibling of the
// reference's ONNX / MNN backends behind runtime/core/speaker/speaker_model.h:25-32,
// and a chunk-averaging engine with the reference SpeakerEngine's contract
// (runtime/core/speaker/speaker_engine.h:26-54, speaker_engine.cc:77-159).
//
// Inside the reference tree, define WSP_HAVE_REFERENCE_SPEAKER_MODEL and include
// "speaker/speaker_model.h" first: HipSpeakerModel then derives from the
// reference's own base class.  Standalone (this repo), the same one-method
// interface is declared below.
//
// Model file: safetensors written by `python -m wespeaker_hubert_amd.bin.export_hip`
// (the reference checkpoint's state_dict names and f32 data, metadata "arch",
// "feat_dim", "embed_dim", "emb_bn", "two_emb_layer").
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../include/wespeaker_amd.h"

namespace wespeaker {

#ifndef WSP_HAVE_REFERENCE_SPEAKER_MODEL
class SpeakerModel {
 public:
  virtual ~SpeakerModel() = default;
  virtual void ExtractEmbedding(const std::vector<std::vector<float>>& feats, std::vector<float>* embed) {}
};
#endif

// Minimal safetensors reader (f32 tensors + string metadata).
struct SafeTensors {
  struct Tensor {
    std::vector<int64_t> shape;
    size_t begin = 0, end = 0;  // byte range in `data`
  };
  std::map<std::string, Tensor> tensors;
  std::map<std::string, std::string> metadata;
  std::vector<char> data;
  static SafeTensors Load(const std::string& path);  // throws std::runtime_error
};

class HipSpeakerModel : public SpeakerModel {
 public:
  // Loads the model file, packs the weights on HIP device `device`.
  explicit HipSpeakerModel(const std::string& model_path, int device = 0);
  ~HipSpeakerModel() override;
  HipSpeakerModel(const HipSpeakerModel&) = delete;
  HipSpeakerModel& operator=(const HipSpeakerModel&) = delete;

  // SpeakerModel: one utterance, feats [T][feat_dim] -> embed [embed_dim]
  // (the reference's ONNX backend contract, onnx_speaker_model.cc:79-112).
  void ExtractEmbedding(const std::vector<std::vector<float>>& feats, std::vector<float>* embed) override;
  // Equal-length batch: feats [B*T*feat_dim] -> embeds [B*embed_dim] in one forward.
  void ExtractEmbeddingBatch(const float* feats, int B, int T, std::vector<float>* embeds);

  int EmbedDim() const { return embed_dim_; }
  int FeatDim() const { return feat_dim_; }
  const std::string& Arch() const { return arch_; }

 private:
  void Reserve(size_t feat_floats, size_t emb_floats, size_t ws_bytes);
  wsp_model* model_ = nullptr;
  int device_ = 0;
  int feat_dim_ = 0, embed_dim_ = 0;
  std::string arch_;
  void* stream_ = nullptr;
  float* d_feats_ = nullptr;
  float* d_emb_ = nullptr;
  void* d_ws_ = nullptr;
  size_t cap_feats_ = 0, cap_emb_ = 0, cap_ws_ = 0;
};

// SpeakerEngine analogue: whole-utterance fbank on the device, the reference's
// chunking (samples_per_chunk <= 0: one chunk = whole utterance; else chunks
// of 1 + (samples_per_chunk - 400) / 160 frames, a short tail filled from the
// first chunk, a lone short utterance repeated), per-chunk CMN, embeddings of
// all chunks in ONE batched forward, averaged.
class HipSpeakerEngine {
 public:
  HipSpeakerEngine(const std::string& model_path, int feat_dim, int sample_rate, int embedding_size,
                   int samples_per_chunk, int device = 0);
  int EmbeddingSize() const { return embedding_size_; }
  void ExtractFeature(const int16_t* data, int data_size, std::vector<std::vector<std::vector<float>>>* chunks_feat);
  void ExtractEmbedding(const int16_t* data, int data_size, std::vector<float>* avg_emb);
  float CosineSimilarity(const std::vector<float>& emb1, const std::vector<float>& emb2);

 private:
  std::unique_ptr<HipSpeakerModel> model_;
  int feat_dim_ = 80, sample_rate_ = 16000, embedding_size_ = 0, per_chunk_samples_ = 32000;
  void* stream_ = nullptr;
  void* d_wav_ = nullptr;
  float* d_fbank_ = nullptr;
  int frame_len_ = 400, frame_shift_ = 160;  // samples (wsp_fbank_geometry)
  size_t cap_wav_ = 0, cap_fbank_ = 0;
};

// 16-bit PCM mono WAV reader (RIFF); returns samples, sets sample_rate.
std::vector<int16_t> ReadWavPcm16(const std::string& path, int* sample_rate);

}  // namespace wespeaker
