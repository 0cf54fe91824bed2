// Speaker model runtime object behind the wsp_model_* C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace wsp {

class Model {
 public:
  Model();
  ~Model();
  void create(const std::string& arch, int feat_dim, int embed_dim, bool emb_bn, bool two_emb);
  int num_params() const;
  void param_info(int i, const char** name, int* ndim, int64_t* shape) const;
  void set_param(int i, const float* data, int64_t numel);
  void finalize();
  int embed_dim() const;
  int feat_dim() const;
  size_t workspace_bytes(int B, int T) const;
  void forward(const float* feats, int B, int T, float* embed, void* ws, size_t ws_bytes,
               hipStream_t s);
  // HuBERT front end (arch "HuBERT_base"): wav [B][N] -> feats [B][out_frames(N)][768]
  bool is_frontend() const;
  int out_frames(int N) const;
  size_t frontend_workspace_bytes(int B, int N) const;
  void forward_frontend(const float* wav, int B, int N, float* feats, int cmn, void* ws, size_t ws_bytes,
                        hipStream_t s);
  // ragged batch: utterance b = lens[b] samples (host array) of the concatenated wav;
  // feats rows [frame_offsets[b], frame_offsets[b+1]) (host [B+1] out, may be null)
  size_t frontend_workspace_bytes_segments(int B, const int* lens) const;
  void forward_frontend_segments(const float* wav, int B, const int* lens, float* feats, int* frame_offsets, int cmn,
                                 void* ws, size_t ws_bytes, hipStream_t s);
  // Segmented (ragged) batch: utterance b = feats rows [seg[b], seg[b+1]) (device int32
  // [B+1]), M = seg[B] rows in total.  ECAPA-TDNN only.
  size_t workspace_bytes_segments(int B, int M) const;
  void forward_segments(const float* feats, int B, const int* seg, int M, float* embed, void* ws, size_t ws_bytes,
                        hipStream_t s);
  void profile(bool on);
  void set_option(const std::string& key, int value);
  int get_option(const std::string& key) const;
  void profile_query(const std::string& tag, int* launches, double* total_ms, double* flops);

  struct Impl;

 private:
  Impl* impl;
};

}  // namespace wsp
