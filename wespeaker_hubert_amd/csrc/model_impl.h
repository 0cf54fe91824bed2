// Internal: the Model::Impl runtime object shared by the ECAPA / ResNet
// (model.cpp) and HuBERT (hubert_model.cpp) translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "kernels.h"
#include "model.h"
#include "res2_chain.h"
#include "astp_fused.h"
#include "conv3x3_img.h"

namespace wsp {

namespace detail {

constexpr double kBnEps = 1e-5;

struct DevBuf {
  std::vector<void*> ptrs;
  ~DevBuf() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  void* upload_u16(const std::vector<uint16_t>& v) {
    void* p = nullptr;
    WSP_HIP(hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(uint16_t)));
    ptrs.push_back(p);
    if (!v.empty()) WSP_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    return p;
  }
  float* upload(const std::vector<float>& v) {
    void* p = nullptr;
    WSP_HIP(hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(float)));
    ptrs.push_back(p);
    if (!v.empty()) WSP_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
    return static_cast<float*>(p);
  }
};

struct ConvW {
  float* w = nullptr;
  void* whi = nullptr;  // bf16 hi / lo split images for the bf16x3 kernel
  void* wlo = nullptr;
  float* bias = nullptr;
  float* scale = nullptr;
  float* shift = nullptr;
  int N = 0, cin = 0, taps = 1, K = 0, Kp = 0;
  void* frag = nullptr;  // MFMA B-fragment order of a stride-1 3x3 conv with N = cin (conv3x3_img.hip)
};

struct LinW {  // small_linear weights, k-major
  float* wt = nullptr;
  float* bias = nullptr;
  int K = 0, N = 0;
};

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// fp32 -> bf16, round to nearest even (matches v_cvt_pk_bf16_f32 on finite values)
inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float bf2f(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

}  // namespace detail

using namespace detail;

// HuBERT batch plan (hubert_model.cpp): utterance ranges of the feature
// extractor, their row counts per conv level, and the int32 offset tables.
struct HubertChunk {
  int b0 = 0, b1 = 0;
  size_t off = 0;       // index of this chunk's tables in HubertPlan::offs
  size_t rows[7] = {};  // conv-level frame rows of the chunk
  size_t samples = 0, sample0 = 0, row6 = 0;
  size_t row3 = 0;  // the chunk's first row in the batch-wide level-3 rows (cnn_tail_batch)
  int maxT0 = 0;
};
struct HubertPlan {
  int B = 0;
  size_t M = 0, Mout = 0, maxA = 0, maxB = 0;
  // batch-wide rows of conv levels 3..5 and whether CNN layers 4..6 run once over the batch
  // (their global offsets follow seg6 | fseg in offs as seg3 | seg4 | seg5)
  size_t M3 = 0, M4 = 0, M5 = 0;
  bool tail_batch = false;
  int maxChunk = 0, maxT6 = 0;
  size_t maxStats = 0;  // doubles of conv0 partial moments (hubert_conv0_stats_doubles) of the largest chunk
  std::vector<HubertChunk> chunks;
  std::vector<int> offs;
};

struct Param {
  std::string name;
  std::vector<int64_t> shape;
  std::vector<float> host;
  bool set = false;
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

struct ProfEntry {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t used = 0;
  double flops = 0;
};

struct Model::Impl {
  std::string arch;
  bool ecapa = true;
  int C = 512;
  bool glob = false;
  int feat_dim = 80, embed_dim = 192;
  bool emb_bn = false, two_emb = false;
  std::vector<Param> params;
  std::map<std::string, int> idx;
  bool finalized = false;
  int device = 0;
  DevBuf dev;

  // ECAPA packed weights
  ConvW layer1;
  struct Block {
    ConvW c1, c3, res2[7];
    LinW se1, se2;
    // the 7 Res2Net convs packed for res2_chain.hip (one launch per block)
    void* r2w = nullptr;
    float *r2b = nullptr, *r2s = nullptr, *r2t = nullptr;
  } blk[3];
  int res2_fused = 1;  // 0: the 7-launch GEMM chain (A/B option "res2_fused")
  // ResNet stride-1 3x3 convs on conv3x3_img.hip (option "conv3x3_img"): 0 = off (implicit GEMM),
  // 1 = 32 / 64 channels, 2 = also 128 channels (4 x 32 tile), 3 = also 128 (2 x 32 tile)
  int conv3x3_img_on = 2;
  int res_prefetch = 1;  // ResNet 1x1 residual convs: residual loaded ahead of the last k-tiles (option "res_prefetch")
  // ResNet bottleneck conv2 + conv3 (+ residual) of stride-1 blocks with planes 32 / 64 / 128 in one
  // launch, y2 kept in registers (conv3x3_img.hip bottleneck_tail; option "res_tail"): 1 = also the
  // next block's conv1 on the tail's output while it is on chip (tail2_kernel: two position runs
  // per wave), 2 = the tail alone, 0 = off
  int res_tail = 1;
  // bottleneck conv3 + projection shortcut fused: bit 0 as one GEMM (RBlock::c3sc), bit 1 inside
  // the fused tail (RBlock::w3scx)
  int sc_fuse = 3;
  int c1_stage_fuse = 1;  // a stage's first conv1 (4C -> 2C) inside the previous stage's last tail
  bool img_ok(const ConvW& cw, int C) const { return cw.frag && conv3x3_img_on && (C <= 64 || conv3x3_img_on >= 2); }
  int res2_variant = 4;  // res2_chain.hip kernel variant (option "res2_variant"; 4 = halo-free strips, C2 1.48 -> 1.24 ms/step; c512 widths run 3)
  ConvW conv, pool1, pool2;
  // conv_cat on [out2, out3, g4 * h3_4]: out4 = out3 + g4 * h3_4, so W . [out2; out3; out4]
  // = W_a out2 + (W_b + W_c) out3 + W_c (g4 * h3_4) — the last SE block's residual pass
  // writes only g4 * h3_4 (no residual read) (option "cat_gate", default on)
  ConvW conv_g;
  int cat_gate = 1;
  void* pool2_frag = nullptr;  // pool.linear2 in MFMA B-fragment order for astp_fused.hip
  // 0: linear2 GEMM + separate pooling kernel; 1: astp_fused.hip (option "astp_fused"; 256 channels
  // per block, att chunks two ahead in an LDS-DMA ring, W2 in VGPRs: C2 0.465 -> 0.31 ms)
  int astp_fused_on = 1;
  LinW pool1_ctx;
  LinW head;

  // ResNet (resnet.py:110-260), NHWC activations [B][F][T][C]
  bool bottleneck = true;
  int nblocks[4] = {0, 0, 0, 0};
  int m_ch = 32;
  float* stem_w = nullptr;
  float* stem_b = nullptr;
  struct RBlock {
    ConvW c1, c2, c3, sc;
    // conv3 (bn3 folded) and the projection shortcut (its bn folded) as ONE 1x1 GEMM over
    // [y2 | strided x] (K = planes + in_planes, bias b3 + b_sc): the shortcut's output never goes
    // through HBM (option "sc_fuse"; bottleneck blocks off the fused-tail path, N % 256 == 0)
    ConvW c3sc;
    void* w3acc = nullptr;  // conv3 (bn3 folded) as pack_frag_acc B fragments for bottleneck_tail
    // [conv3 | shortcut] (both BN-folded) for the in-tail shortcut (BottleneckTailArgs::xsc) and its
    // summed bias: a stride-1 first block with in_planes == planes == 32
    void* w3scx = nullptr;
    float* b3scx = nullptr;
    void* w1frag = nullptr;  // conv1 (bn1 folded) as pack_frag B fragments: run inside the previous block's tail
    bool has_sc = false;
    int stride = 1, in_planes = 0, planes = 0, out_planes = 0;
  };
  std::vector<RBlock> rblocks;
  LinW seg1, seg2;  // seg2: two_emb_layer's seg_2 with the affine-free seg_bn_1 folded in

  // SimAM-ResNet (samresnet.py:20-166): basic blocks whose bn2 output passes
  // SimAM before the shortcut add, ASP pooling, `bottleneck` Linear.
  bool simam = false;
  ConvW asp1, asp2;
  LinW simam_head;

  // HuBERT-base front end (hubert_model.cpp), channels-last [B][T][C]
  bool hubert = false;
  float* h_conv0_w = nullptr;  // [512][10]
  float* h_gn_g = nullptr;
  float* h_gn_b = nullptr;
  ConvW h_conv[7];  // 1..6: strided feature-extractor convs (GELU epilogue)
  float* h_ln0_g = nullptr;
  float* h_ln0_b = nullptr;
  ConvW h_proj, h_pos;
  float* h_enc_g = nullptr;
  float* h_enc_b = nullptr;
  struct HLayer {
    ConvW qkv, out, fc1, fc2;
    float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
    // LayerNorm fold (option ln_fold): fc1 on the un-normalised rows with gamma1 folded into W
    // and W beta1 into the bias; fc1_cs[n] = sum_c W'[n][c] (of the bf16 hi + lo images)
    ConvW fc1f;
    float* fc1_cs = nullptr;
  };
  std::vector<HLayer> h_layers;
  std::vector<float> h_fw;  // featurizer weight per hidden state
  int h_layer_sel = -1;     // s3prl `layer` (-1: softmax-weighted sum of all 13)
  int attn_pipe = 1;        // attn.hip: 1 = persistent pipelined kernel, 0 = one block per (utterance, head)
  int pos_conv = 1;         // HuBERT pos_conv: 1 = direct grouped conv (pos_conv.hip), 0 = grouped implicit GEMM
  // HuBERT: 1 = the post-attention LayerNorm folded into out_proj / fc1 / fc2 (x3_variant 7); measured
  // neutral on C4 (A/B 4 234 / 4 223 vs 4 233 / 4 232 emb/s, profiles/r5g_ln_fold.txt): default off
  int ln_fold = 0;
  // HuBERT CNN layers 4-6 once over the whole batch when the feature extractor runs in several
  // utterance chunks (r5); 0 = per chunk (the tests compare the two)
  int tail_batch = 1;
  void build_hubert_params();
  void finalize_hubert();
  int hubert_cnn_frames(int N, int upto) const;
  HubertPlan hubert_plan(int B, const int* lens) const;
  size_t hubert_ws_floats(const HubertPlan& pl, size_t* offs) const;
  void forward_hubert(const float* wav, const HubertPlan& pl, float* feats, int cmn, float* ws, hipStream_t s);

  // segmented (ragged) forward in progress: device row offsets [cur_nseg + 1]
  const int* cur_seg = nullptr;
  int cur_nseg = 0;

  // 1 = bf16x3 split MFMA (default), 0 = exact f32 MFMA
  int precision = 1;
  // bf16x3 tile family (conv_gemm_x3.hip): 5 = 256 x 256 where N % 256 == 0, else 256 x 128;
  // 4 = 256 x 128; 3 = 128 x 128; 6 = 5 on 16x16x32 MFMAs; 7 = 6 with plain-epilogue GEMMs
  // staged by LDS-DMA (conv_gemm_x3_t6.hip) (option "x3_variant")
  int x3_variant = 5;

  // concurrent sub-batches (option "streams"): the batch's utterances are split
  // into `streams` contiguous ranges, each forwarded on its own HIP stream over its
  // own workspace slice, so one range's HBM-bound kernels run beside the other's
  // MFMA-bound GEMMs; the caller's stream forks to and joins them with events.
  int streams = 1;
  std::vector<hipStream_t> sub_st;  // streams 1.. (range 0 runs on the caller's stream)
  std::vector<hipEvent_t> sub_ev;   // [0] fork, [i] join of range i
  int nsub(int B) const { return std::max(1, std::min(streams, B)); }
  size_t ws_bytes_one(int B, int T) const;
  hipStream_t sub(hipStream_t s, int i) const { return i == 0 ? s : sub_st[i - 1]; }
  void fork(hipStream_t s, int ns) {
    while ((int)sub_st.size() < ns - 1) {
      hipStream_t t;
      WSP_HIP(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
      sub_st.push_back(t);
    }
    while ((int)sub_ev.size() < ns) {
      hipEvent_t e;
      WSP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      sub_ev.push_back(e);
    }
    WSP_HIP(hipEventRecord(sub_ev[0], s));
    for (int i = 1; i < ns; ++i) WSP_HIP(hipStreamWaitEvent(sub_st[i - 1], sub_ev[0], 0));
  }
  void join(hipStream_t s, int ns) {
    for (int i = 1; i < ns; ++i) {
      WSP_HIP(hipEventRecord(sub_ev[i], sub_st[i - 1]));
      WSP_HIP(hipStreamWaitEvent(s, sub_ev[i], 0));
    }
  }

  // profiling
  bool prof = false;
  std::map<std::string, ProfEntry> prof_map;

  void add(const std::string& n, std::vector<int64_t> shape) {
    idx[n] = (int)params.size();
    params.push_back(Param{n, std::move(shape), {}, false});
  }
  void add_bn(const std::string& p, int64_t c) {
    add(p + ".weight", {c});
    add(p + ".bias", {c});
    add(p + ".running_mean", {c});
    add(p + ".running_var", {c});
    add(p + ".num_batches_tracked", {});
  }
  const std::vector<float>& P(const std::string& n) const {
    auto it = idx.find(n);
    WSP_CHECK(it != idx.end(), "missing parameter " + n);
    const Param& p = params[it->second];
    WSP_CHECK(p.set || p.numel() == 0, "parameter not set: " + n);
    return p.host;
  }

  // eval BatchNorm as affine: y = x*scale + shift
  void bn_affine(const std::string& p, std::vector<double>& sc, std::vector<double>& sh) const {
    const auto& w = P(p + ".weight");
    const auto& b = P(p + ".bias");
    const auto& rm = P(p + ".running_mean");
    const auto& rv = P(p + ".running_var");
    sc.resize(w.size());
    sh.resize(w.size());
    for (size_t i = 0; i < w.size(); ++i) {
      sc[i] = (double)w[i] / std::sqrt((double)rv[i] + kBnEps);
      sh[i] = (double)b[i] - (double)rm[i] * sc[i];
    }
  }

  // Conv1d weight [N][cin][taps] -> packed [N][Kp], k = tap*cin + c.
  ConvW pack_conv(const std::vector<float>& w, int N, int cin, int taps, const float* bias,
                  const std::string& bn) {
    ConvW cw;
    cw.N = N;
    cw.cin = cin;
    cw.taps = taps;
    cw.K = cin * taps;
    cw.Kp = round_up(cw.K, 64);  // even number of 32-wide k-tiles (bf16x3 pipeline)
    std::vector<float> packed((size_t)N * cw.Kp, 0.f);
    for (int n = 0; n < N; ++n)
      for (int c = 0; c < cin; ++c)
        for (int j = 0; j < taps; ++j)
          packed[(size_t)n * cw.Kp + j * cin + c] = w[((size_t)n * cin + c) * taps + j];
    cw.w = dev.upload(packed);
    {
      std::vector<uint16_t> hi(packed.size()), lo(packed.size());
      for (size_t i = 0; i < packed.size(); ++i) {
        hi[i] = f2bf(packed[i]);
        lo[i] = f2bf(packed[i] - bf2f(hi[i]));
      }
      cw.whi = dev.upload_u16(hi);
      cw.wlo = dev.upload_u16(lo);
    }
    if (bias) cw.bias = dev.upload(std::vector<float>(bias, bias + N));
    if (!bn.empty()) {
      std::vector<double> sc, sh;
      bn_affine(bn, sc, sh);
      std::vector<float> s(N), t(N);
      for (int i = 0; i < N; ++i) {
        s[i] = (float)sc[i];
        t[i] = (float)sh[i];
      }
      cw.scale = dev.upload(s);
      cw.shift = dev.upload(t);
    }
    return cw;
  }

  // Linear / 1x1-conv weight [N][K] -> bf16 hi / lo in MFMA B-fragment order
  // [K/16 k-steps][2 planes][N/32 column tiles][64 lanes][8]: lane l of a
  // 32x32x16 MFMA holds W[n = 32 j + (l & 31)][k = 16 ks + 8 (l >> 5) + e].
  void* pack_frag(const std::vector<float>& w, int N, int K) {
    const int KS = K / 16, NT = N / 32;
    std::vector<uint16_t> pk((size_t)KS * 2 * NT * 64 * 8);
    for (int ks = 0; ks < KS; ++ks)
      for (int jt = 0; jt < NT; ++jt)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 8; ++e) {
            const float v = w[(size_t)(jt * 32 + (l & 31)) * K + ks * 16 + 8 * (l >> 5) + e];
            const uint16_t hi = f2bf(v), lo = f2bf(v - bf2f(hi));
            const size_t o = (((size_t)ks * 2 * NT + jt) * 64 + l) * 8 + e;
            pk[o] = hi;
            pk[o + (size_t)NT * 64 * 8] = lo;
          }
    return dev.upload_u16(pk);
  }

  // As pack_frag, but lane l, element e of k-step ks holds k = 16 ks + (e & 3) + 8 (e >> 2)
  // + 4 (l >> 5): the order in which a transposed 32x32 accumulator tile holds its 32 rows
  // (register r = (r & 3) + 8 (r >> 2) + 4 (l >> 5)), so such accumulators feed this
  // weight's MFMAs as the A operand without a shuffle (bottleneck_tail).
  // kacc >= 0: only the k-steps below kacc in that order, the rest in pack_frag's (the in-tail
  // shortcut's x fragments, BottleneckTailArgs::xsc)
  void* pack_frag_acc(const std::vector<float>& w, int N, int K, int kacc = -1) {
    const int KS = K / 16, NT = N / 32;
    std::vector<uint16_t> pk((size_t)KS * 2 * NT * 64 * 8);
    for (int ks = 0; ks < KS; ++ks)
      for (int jt = 0; jt < NT; ++jt)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 8; ++e) {
            const int k = kacc >= 0 && ks * 16 >= kacc ? ks * 16 + 8 * (l >> 5) + e
                                                        : ks * 16 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
            const float v = w[(size_t)(jt * 32 + (l & 31)) * K + k];
            const uint16_t hi = f2bf(v), lo = f2bf(v - bf2f(hi));
            const size_t o = (((size_t)ks * 2 * NT + jt) * 64 + l) * 8 + e;
            pk[o] = hi;
            pk[o + (size_t)NT * 64 * 8] = lo;
          }
    return dev.upload_u16(pk);
  }

  // Linear weight [N][K] (row-major, ldk) -> k-major [K][N]
  LinW pack_lin(const float* w, int N, int K, int ldk, const float* bias) {
    LinW lw;
    lw.N = N;
    lw.K = K;
    std::vector<float> t((size_t)K * N);
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < K; ++k) t[(size_t)k * N + n] = w[(size_t)n * ldk + k];
    lw.wt = dev.upload(t);
    if (bias) lw.bias = dev.upload(std::vector<float>(bias, bias + N));
    return lw;
  }

  void build_ecapa_params() {
    const int64_t C = this->C, w = C / 8;
    add("layer1.conv.weight", {C, feat_dim, 5});
    add("layer1.conv.bias", {C});
    add_bn("layer1.bn", C);
    for (int li = 2; li <= 4; ++li) {
      const std::string p = "layer" + std::to_string(li) + ".se_res2block";
      add(p + ".0.conv.weight", {C, C, 1});
      add(p + ".0.conv.bias", {C});
      add_bn(p + ".0.bn", C);
      for (int i = 0; i < 7; ++i) {
        add(p + ".1.convs." + std::to_string(i) + ".weight", {w, w, 3});
        add(p + ".1.convs." + std::to_string(i) + ".bias", {w});
      }
      for (int i = 0; i < 7; ++i) add_bn(p + ".1.bns." + std::to_string(i), w);
      add(p + ".2.conv.weight", {C, C, 1});
      add(p + ".2.conv.bias", {C});
      add_bn(p + ".2.bn", C);
      add(p + ".3.linear1.weight", {128, C});
      add(p + ".3.linear1.bias", {128});
      add(p + ".3.linear2.weight", {C, 128});
      add(p + ".3.linear2.bias", {C});
    }
    add("conv.weight", {1536, 3 * C, 1});
    add("conv.bias", {1536});
    add("pool.linear1.weight", {128, glob ? 4608 : 1536, 1});
    add("pool.linear1.bias", {128});
    add("pool.linear2.weight", {1536, 128, 1});
    add("pool.linear2.bias", {1536});
    add_bn("bn", 3072);
    add("linear.weight", {embed_dim, 3072});
    add("linear.bias", {embed_dim});
    if (emb_bn) add_bn("bn2", embed_dim);
  }

  void build_resnet_params() {
    const int exp = bottleneck ? 4 : 1;
    add("conv1.weight", {m_ch, 1, 3, 3});
    add_bn("bn1", m_ch);
    int in_planes = m_ch;
    for (int li = 0; li < 4; ++li) {
      const int planes = m_ch << li;
      for (int bi = 0; bi < nblocks[li]; ++bi) {
        const int stride = (li > 0 && bi == 0) ? 2 : 1;
        const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
        RBlock rb;
        rb.stride = stride;
        rb.in_planes = in_planes;
        rb.planes = planes;
        rb.out_planes = planes * exp;
        if (bottleneck) {
          add(p + ".conv1.weight", {planes, in_planes, 1, 1});
          add_bn(p + ".bn1", planes);
          add(p + ".conv2.weight", {planes, planes, 3, 3});
          add_bn(p + ".bn2", planes);
          add(p + ".conv3.weight", {planes * 4, planes, 1, 1});
          add_bn(p + ".bn3", planes * 4);
        } else {
          add(p + ".conv1.weight", {planes, in_planes, 3, 3});
          add_bn(p + ".bn1", planes);
          add(p + ".conv2.weight", {planes, planes, 3, 3});
          add_bn(p + ".bn2", planes);
        }
        if (stride != 1 || in_planes != exp * planes) {
          rb.has_sc = true;
          add(p + ".shortcut.0.weight", {exp * planes, in_planes, 1, 1});
          add_bn(p + ".shortcut.1", exp * planes);
        }
        rblocks.push_back(rb);
        in_planes = planes * exp;
      }
    }
    const int stats_dim = (feat_dim / 8) * m_ch * 8 * exp;
    add("seg_1.weight", {embed_dim, stats_dim * 2});
    add("seg_1.bias", {embed_dim});
    if (two_emb) {  // resnet.py:158-161: BatchNorm1d(affine=False) + seg_2
      add("seg_bn_1.running_mean", {embed_dim});
      add("seg_bn_1.running_var", {embed_dim});
      add("seg_bn_1.num_batches_tracked", {});
      add("seg_2.weight", {embed_dim, embed_dim});
      add("seg_2.bias", {embed_dim});
    }
  }

  // conv -> BN (eval) folded into the weights: W' = W * s[n], bias = shift.
  ConvW pack_conv_bn(const std::string& wname, const std::string& bn, int N, int cin, int taps,
                     void** acc_frag = nullptr, void** b_frag = nullptr) {
    std::vector<double> sc, sh;
    bn_affine(bn, sc, sh);
    std::vector<float> w = P(wname);
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < cin * taps; ++k) w[(size_t)n * cin * taps + k] = (float)(w[(size_t)n * cin * taps + k] * sc[n]);
    std::vector<float> b(N);
    for (int n = 0; n < N; ++n) b[n] = (float)sh[n];
    ConvW cw = pack_conv(w, N, cin, taps, b.data(), "");
    if (acc_frag) *acc_frag = pack_frag_acc(w, N, cin * taps);
    if (b_frag) *b_frag = pack_frag(w, N, cin * taps);
    if (taps == 9 && N == cin && conv3x3_img_supported(cin)) {
      // the same k = tap * cin + c order as the implicit GEMM's packed image
      std::vector<float> wk((size_t)N * 9 * cin);
      for (int n = 0; n < N; ++n)
        for (int c = 0; c < cin; ++c)
          for (int j = 0; j < 9; ++j) wk[(size_t)n * 9 * cin + j * cin + c] = w[((size_t)n * cin + c) * 9 + j];
      cw.frag = pack_frag(wk, N, 9 * cin);
    }
    return cw;
  }

  void finalize_resnet() {
    {
      std::vector<double> sc, sh;
      bn_affine("bn1", sc, sh);
      const auto& w = P("conv1.weight");
      std::vector<float> wf(m_ch * 9), bf(m_ch);
      for (int c = 0; c < m_ch; ++c) {
        for (int q = 0; q < 9; ++q) wf[c * 9 + q] = (float)(w[c * 9 + q] * sc[c]);
        bf[c] = (float)sh[c];
      }
      stem_w = dev.upload(wf);
      stem_b = dev.upload(bf);
    }
    int idx_b = 0;
    for (int li = 0; li < 4; ++li)
      for (int bi = 0; bi < nblocks[li]; ++bi) {
        RBlock& rb = rblocks[idx_b++];
        const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
        if (bottleneck) {
          // a stride-1 block whose input has 4 x its planes (every block after the first of a
          // stage) runs its conv1 inside the previous block's bottleneck_tail
          // ... and a stage's first block whose conv1 is 2C <- 4C of the previous stage's C = 32 / 64
          // planes runs it inside the previous stage's last tail (c1_stage_fuse)
          const bool c1_in_tail = (rb.stride == 1 && rb.in_planes == 4 * rb.planes && bi > 0 &&
                                   bottleneck_tail_supported(rb.planes)) ||
                                  (bi == 0 && li > 0 && rb.in_planes == 2 * rb.planes && rb.planes <= 128 &&
                                   bottleneck_tail_supported(rb.planes / 2));
          rb.c1 = pack_conv_bn(p + ".conv1.weight", p + ".bn1", rb.planes, rb.in_planes, 1, nullptr,
                               c1_in_tail ? &rb.w1frag : nullptr);
          rb.c2 = pack_conv_bn(p + ".conv2.weight", p + ".bn2", rb.planes, rb.planes, 9);
          rb.c3 = pack_conv_bn(p + ".conv3.weight", p + ".bn3", rb.out_planes, rb.planes, 1,
                               rb.stride == 1 && bottleneck_tail_supported(rb.planes) ? &rb.w3acc : nullptr);
        } else {
          rb.c1 = pack_conv_bn(p + ".conv1.weight", p + ".bn1", rb.planes, rb.in_planes, 9);
          rb.c2 = pack_conv_bn(p + ".conv2.weight", p + ".bn2", rb.planes, rb.planes, 9);
        }
        if (rb.has_sc) rb.sc = pack_conv_bn(p + ".shortcut.0.weight", p + ".shortcut.1", rb.out_planes, rb.in_planes, 1);
        if (bottleneck && rb.has_sc && rb.out_planes % 256 == 0 && rb.planes % 32 == 0 && rb.in_planes % 32 == 0) {
          std::vector<double> s3, h3, ss, hs;
          bn_affine(p + ".bn3", s3, h3);
          bn_affine(p + ".shortcut.1", ss, hs);
          const std::vector<float>& w3 = P(p + ".conv3.weight");
          const std::vector<float>& wsc = P(p + ".shortcut.0.weight");
          const int K = rb.planes + rb.in_planes, N = rb.out_planes;
          std::vector<float> wf((size_t)N * K), bf(N);
          for (int n = 0; n < N; ++n) {
            for (int k = 0; k < rb.planes; ++k) wf[(size_t)n * K + k] = (float)(w3[(size_t)n * rb.planes + k] * s3[n]);
            for (int k = 0; k < rb.in_planes; ++k)
              wf[(size_t)n * K + rb.planes + k] = (float)(wsc[(size_t)n * rb.in_planes + k] * ss[n]);
            bf[n] = (float)h3[n] + (float)hs[n];
          }
          rb.c3sc = pack_conv(wf, N, K, 1, bf.data(), "");
        }
        if (bottleneck && rb.has_sc && rb.stride == 1 && rb.in_planes == rb.planes && rb.planes == 32 && rb.w3acc) {
          std::vector<double> s3, h3, ss, hs;
          bn_affine(p + ".bn3", s3, h3);
          bn_affine(p + ".shortcut.1", ss, hs);
          const std::vector<float>& w3 = P(p + ".conv3.weight");
          const std::vector<float>& wsc = P(p + ".shortcut.0.weight");
          const int C = rb.planes, K = 2 * C, N = rb.out_planes;
          std::vector<float> wf((size_t)N * K), bf(N);
          for (int n = 0; n < N; ++n) {
            for (int k = 0; k < C; ++k) {
              wf[(size_t)n * K + k] = (float)(w3[(size_t)n * C + k] * s3[n]);
              wf[(size_t)n * K + C + k] = (float)(wsc[(size_t)n * C + k] * ss[n]);
            }
            bf[n] = (float)h3[n] + (float)hs[n];
          }
          rb.w3scx = pack_frag_acc(wf, N, K, C);
          rb.b3scx = dev.upload(bf);
        }
      }
    // seg_1 over TSTP stats; reference flatten index s*C*F4 + c*F4 + f, ours f*2C + s*C + c
    const int C4 = rblocks.back().out_planes, F4 = feat_dim / 8;
    const auto& W = P("seg_1.weight");
    const int K = 2 * C4 * F4;
    std::vector<float> wp((size_t)embed_dim * K);
    for (int n = 0; n < embed_dim; ++n)
      for (int f = 0; f < F4; ++f)
        for (int sidx = 0; sidx < 2; ++sidx)
          for (int c = 0; c < C4; ++c)
            wp[(size_t)n * K + f * 2 * C4 + sidx * C4 + c] = W[(size_t)n * K + sidx * C4 * F4 + c * F4 + f];
    seg1 = pack_lin(wp.data(), embed_dim, K, K, P("seg_1.bias").data());
    if (two_emb) {
      // embed_b = seg_2(BN(relu(embed_a))), BN without affine (resnet.py:196-200):
      // W2 ((r - rm) / sqrt(rv + eps)) + b2 = (W2 diag(s)) r + (b2 - W2 (rm s))
      const auto& rm = P("seg_bn_1.running_mean");
      const auto& rv = P("seg_bn_1.running_var");
      const auto& W2 = P("seg_2.weight");
      const auto& b2 = P("seg_2.bias");
      const int D = embed_dim;
      std::vector<float> w2((size_t)D * D), bb(D);
      for (int n = 0; n < D; ++n) {
        double acc = b2[n];
        for (int k = 0; k < D; ++k) {
          const double sk = 1.0 / std::sqrt((double)rv[k] + kBnEps);
          w2[(size_t)n * D + k] = (float)(W2[(size_t)n * D + k] * sk);
          acc -= (double)W2[(size_t)n * D + k] * rm[k] * sk;
        }
        bb[n] = (float)acc;
      }
      seg2 = pack_lin(w2.data(), D, D, D, bb.data());
    }
  }

  struct RShapes {
    size_t big = 0, y1 = 0, y2 = 0, sc = 0;  // floats per utterance
    int F4 = 0, T4 = 0, C4 = 0;
  };
  RShapes resnet_shapes(int T) const {
    RShapes r;
    int Fi = feat_dim, Ti = T;
    r.big = (size_t)Fi * Ti * m_ch;
    for (const RBlock& rb : rblocks) {
      const int Fo = (Fi - 1) / rb.stride + 1, To = (Ti - 1) / rb.stride + 1;
      r.big = std::max(r.big, (size_t)Fo * To * rb.out_planes);
      r.y1 = std::max(r.y1, (size_t)(bottleneck ? Fi * Ti : Fo * To) * rb.planes);
      r.y2 = std::max(r.y2, (size_t)Fo * To * rb.planes);
      // the buffers Y1 / Y2 alternate as a fused tail's input and its next-conv1 output, which at a
      // stage transition is the next stage's conv1 at this resolution
      if (bottleneck) r.y2 = std::max(r.y2, (size_t)Fi * Ti * rb.planes);
      if (rb.has_sc) r.sc = std::max(r.sc, (size_t)Fo * To * rb.out_planes);
      Fi = Fo;
      Ti = To;
    }
    r.F4 = Fi;
    r.T4 = Ti;
    r.C4 = rblocks.back().out_planes;
    return r;
  }
  // utterances per forward chunk: every activation operand must stay < 2 GiB
  // (32-bit buffer-load offsets).
  int resnet_chunk(int B, int T) const {
    const RShapes r = resnet_shapes(T);
    const size_t per = std::max(r.big, std::max(r.y1, std::max(r.y2, r.sc))) * sizeof(float);
    int bc = (int)std::max<size_t>(1, ((size_t)1 << 31) / 8 * 7 / per);
    bc = std::min(bc, B);
    const int chunks = (B + bc - 1) / bc;
    return (B + chunks - 1) / chunks;
  }
  size_t resnet_ws_floats(int B, int T, size_t* offs) const {
    const int bc = resnet_chunk(B, T);
    const RShapes r = resnet_shapes(T);
    const size_t sizes[] = {bc * r.big, bc * r.big, bc * r.y1, bc * r.y2, bc * std::max<size_t>(r.sc, 1),
                            (size_t)bc * r.F4 * 2 * r.C4};
    size_t o = 0;
    for (int i = 0; i < 6; ++i) {
      if (offs) offs[i] = o;
      o += (sizes[i] + 63) / 64 * 64;
    }
    return o;
  }

  void gemm2d(const char* tag, const ConvW& cw, const float* a0, int lda, float* out, int ldo, int B,
              int Fi, int Ti, int kw, int stride, int pad, int act, const float* res, int ldres,
              hipStream_t s) {
    ConvGemmArgs g{};
    g.a[0] = g.a[1] = g.a[2] = a0;
    g.lda[0] = g.lda[1] = g.lda[2] = lda;
    g.cseg[0] = 0;
    g.cseg[1] = g.cseg[2] = g.cseg[3] = cw.cin;
    const int Fo = (Fi + 2 * pad - kw) / stride + 1, To = (Ti + 2 * pad - kw) / stride + 1;
    const int M = B * Fo * To;
    fill(g, cw, M, M, 1, pad, out, ldo, act, nullptr, true);
    g.conv2d = 1;
    g.Fi = Fi;
    g.Ti = Ti;
    g.Fo = Fo;
    g.To = To;
    g.stride = stride;
    g.kw = kw;
    g.res = res;
    g.ldres = ldres;
    run(tag, 2.0 * M * cw.N * cw.K, s, [&] { launch_conv_gemm_x3(g, cw.whi, cw.wlo, x3_variant, s); });
  }
  void gemm1x1(const char* tag, const ConvW& cw, const float* a0, float* out, int M, int act, const float* res,
               hipStream_t s) {
    ConvGemmArgs g{};
    g.a[0] = g.a[1] = g.a[2] = a0;
    g.lda[0] = g.lda[1] = g.lda[2] = cw.cin;
    g.cseg[0] = 0;
    g.cseg[1] = g.cseg[2] = g.cseg[3] = cw.cin;
    fill(g, cw, M, M, 1, 0, out, cw.N, act, nullptr, true);
    g.res = res;
    g.ldres = cw.N;
    g.role = res && res_prefetch ? 2 : 0;
    run(tag, 2.0 * M * cw.N * cw.K, s, [&] { launch_conv_gemm_x3(g, cw.whi, cw.wlo, x3_variant, s); });
  }

  // bottleneck conv3 + projection shortcut as one GEMM (RBlock::c3sc, ConvGemmArgs::sc2d): A segment 0
  // = y2 [M][planes] (row m), segment 1 = the block input x [B][Fi][Ti][Ci] at the shortcut's
  // strided position of output row m
  void gemm_c3sc(const char* tag, const RBlock& rb, const float* y2, const float* x, int Ci, float* out, int B,
                 int Fi, int Ti, int Fo, int To, hipStream_t s) {
    const ConvW& cw = rb.c3sc;
    ConvGemmArgs g{};
    g.a[0] = y2;
    g.a[1] = g.a[2] = x;
    g.lda[0] = rb.planes;
    g.lda[1] = g.lda[2] = Ci;
    g.cseg[0] = 0;
    g.cseg[1] = rb.planes;
    g.cseg[2] = g.cseg[3] = cw.cin;
    const int M = B * Fo * To;
    fill(g, cw, M, M, 1, 0, out, cw.N, kActRelu, nullptr, true);
    g.sc2d = 1;
    g.Fi = Fi;
    g.Ti = Ti;
    g.Fo = Fo;
    g.To = To;
    g.stride = rb.stride;
    run(tag, 2.0 * M * cw.N * cw.K, s, [&] { launch_conv_gemm_x3(g, cw.whi, cw.wlo, x3_variant, s); });
  }

  void forward_resnet(const float* feats, int B, int T, float* embed, float* ws, hipStream_t s) {
    const int bc = resnet_chunk(B, T);
    size_t off[6];
    resnet_ws_floats(B, T, off);
    float* X = ws + off[0];
    float* O = ws + off[1];
    float* Y1 = ws + off[2];
    float* Y2 = ws + off[3];
    float* SC = ws + off[4];
    float* pooled = ws + off[5];
    for (int b0 = 0; b0 < B; b0 += bc) {
      const int nb = std::min(bc, B - b0);
      int Fi = feat_dim, Ti = T, Ci = m_ch;
      run("stem", 0, s, [&] {
        launch_resnet_stem(feats + (size_t)b0 * T * feat_dim, nb, T, feat_dim, m_ch, stem_w, stem_b, X, s);
      });
      float* x = X;
      float* o = O;
      // profiling sub-classes per stage: res_conv1x1.{c1,c3}.L<n>, res_conv3x3.L<n>
      static const char* kC1[4] = {"res_conv1x1.c1.L1", "res_conv1x1.c1.L2", "res_conv1x1.c1.L3",
                                   "res_conv1x1.c1.L4"};
      static const char* kC3[4] = {"res_conv1x1.c3.L1", "res_conv1x1.c3.L2", "res_conv1x1.c3.L3",
                                   "res_conv1x1.c3.L4"};
      static const char* kK3[4] = {"res_conv3x3.L1", "res_conv3x3.L2", "res_conv3x3.L3", "res_conv3x3.L4"};
      static const char* kTl[4] = {"res_tail.L1", "res_tail.L2", "res_tail.L3", "res_tail.L4"};
      int ib = 0;
      bool y1_ready = false;  // this block's conv1 output was written by the previous block's tail
      float* y1_next = nullptr;
      for (const RBlock& rb : rblocks) {
        int li = 0, acc = nblocks[0];
        while (li < 3 && ib >= acc) acc += nblocks[++li];
        ++ib;
        const int Fo = (Fi - 1) / rb.stride + 1, To = (Ti - 1) / rb.stride + 1;
        const float* res = x;
        const bool tail = bottleneck && rb.stride == 1 && res_tail && rb.w3acc && img_ok(rb.c2, rb.planes);
        const RBlock* nx = (size_t)ib < rblocks.size() ? &rblocks[ib] : nullptr;
        // the tail also runs the next block's conv1 on this block's output (res_tail 1; the next
        // block's conv2 reads y1 from either buffer); at a stage transition the next (first)
        // block's conv1 is 4C -> 2C at this stage's resolution (option c1_stage_fuse)
        const bool fuse1 =
            tail && res_tail == 1 && nx && nx->w1frag &&
            ((nx->planes == rb.planes && nx->w3acc && nx->stride == 1 && img_ok(nx->c2, nx->planes)) ||
             (c1_stage_fuse && nx->planes == 2 * rb.planes && nx->in_planes == rb.out_planes && rb.planes <= 64));
        // conv3 + shortcut in one GEMM on the non-tail path (sc_fuse): no SC round trip through HBM
        const bool fuse_sc = bottleneck && rb.has_sc && !tail && (sc_fuse & 1) && rb.c3sc.w && x3_variant == 7;
        // ... and inside the tail's conv3 for a stride-1 first block of 32 planes (w3scx)
        const bool tail_sc = fuse1 && (sc_fuse & 2) && rb.w3scx && nx->planes == rb.planes;
        if (rb.has_sc && !fuse_sc && !tail_sc) {
          gemm2d("shortcut", rb.sc, x, Ci, SC, rb.out_planes, nb, Fi, Ti, 1, rb.stride, 0, kActNone, nullptr, 0, s);
          res = SC;
        }
        if (bottleneck) {
          if (!y1_ready) gemm1x1(kC1[li], rb.c1, x, Y1, nb * Fi * Ti, kActRelu, nullptr, s);
          const float* y1 = y1_ready ? y1_next : Y1;
          y1_ready = false;
          if (tail) {
            // conv2 + conv3 + residual in one launch, y2 in registers (bottleneck_tail); with
            // fuse1 also the next block's conv1 on this block's output (into the buffer the tail
            // does not read)
            BottleneckTailArgs a{y1, res, o, nb, Fi, Ti, rb.c2.frag, rb.c2.bias, rb.w3acc, rb.c3.bias};
            float* y1n = y1 == Y1 ? Y2 : Y1;
            if (fuse1) {
              a.w1n = nx->w1frag;
              a.b1n = nx->c1.bias;
              a.y1n = y1n;
              a.c1n = nx->planes;
            }
            if (tail_sc) {
              a.res = nullptr;
              a.xsc = x;
              a.w3 = rb.w3scx;
              a.b3 = rb.b3scx;
            }
            const double pos = (double)nb * Fi * Ti;
            run(kTl[li],
                2.0 * pos *
                    (rb.c2.N * rb.c2.K + rb.c3.N * rb.c3.K + (fuse1 ? nx->c1.N * nx->c1.K : 0) +
                     (tail_sc ? rb.sc.N * rb.sc.K : 0)),
                s, [&] { launch_bottleneck_tail(a, rb.planes, s); });
            if (fuse1) {
              y1_ready = true;
              y1_next = y1n;
            }
          } else {
            // y1 is in Y1, or in Y2 when the previous block's tail computed this conv1
            float* y2 = y1 == Y2 ? Y1 : Y2;
            if (rb.stride == 1 && img_ok(rb.c2, rb.planes)) {
              const Conv3x3Args a{y1, y2, nb, Fi, Ti, rb.c2.frag, rb.c2.bias, rb.c2.scale, rb.c2.shift, nullptr, 1,
                                  conv3x3_img_on};
              run(kK3[li], 2.0 * nb * Fi * Ti * rb.c2.N * rb.c2.K, s, [&] { launch_conv3x3_img(a, rb.planes, s); });
            } else {
              gemm2d(kK3[li], rb.c2, y1, rb.planes, y2, rb.planes, nb, Fi, Ti, 3, rb.stride, 1, kActRelu, nullptr, 0,
                     s);
            }
            if (fuse_sc)
              gemm_c3sc(kC3[li], rb, y2, x, Ci, o, nb, Fi, Ti, Fo, To, s);
            else
              gemm1x1(kC3[li], rb.c3, y2, o, nb * Fo * To, kActRelu, res, s);
          }
        } else {
          if (rb.stride == 1 && img_ok(rb.c1, rb.planes)) {
            const Conv3x3Args a{x, Y1, nb, Fi, Ti, rb.c1.frag, rb.c1.bias, rb.c1.scale, rb.c1.shift, nullptr, 1, conv3x3_img_on};
            run(kK3[li], 2.0 * nb * Fi * Ti * rb.c1.N * rb.c1.K, s, [&] { launch_conv3x3_img(a, rb.planes, s); });
          } else {
            gemm2d(kK3[li], rb.c1, x, Ci, Y1, rb.planes, nb, Fi, Ti, 3, rb.stride, 1, kActRelu, nullptr, 0, s);
          }
          if (img_ok(rb.c2, rb.planes) && rb.out_planes == rb.planes) {
            const Conv3x3Args a{Y1, o, nb, Fo, To, rb.c2.frag, rb.c2.bias, rb.c2.scale, rb.c2.shift, res, 1, conv3x3_img_on};
            run(kK3[li], 2.0 * nb * Fo * To * rb.c2.N * rb.c2.K, s, [&] { launch_conv3x3_img(a, rb.planes, s); });
          } else {
            gemm2d(kK3[li], rb.c2, Y1, rb.planes, o, rb.out_planes, nb, Fo, To, 3, 1, 1, kActRelu, res,
                   rb.out_planes, s);
          }
        }
        std::swap(x, o);
        Fi = Fo;
        Ti = To;
        Ci = rb.out_planes;
      }
      // TSTP over frames for every (utterance, freq) row block, then seg_1
      run("tstp_head", 0, s, [&] {
        launch_frame_stats(x, Ci, nb * Fi, Ti, Ci, pooled, 2 * Ci, 1, Ci, s);
        float* e_out = embed + (size_t)b0 * embed_dim;
        // split-K partials of seg_1 (K = F/8 x 2 x C) in the free second conv1 buffer
        const size_t sk = off[4] - off[3];
        if (two_emb) {
          // relu(seg_1(stats)) into the free conv1 buffer, then the folded seg_bn_1 + seg_2
          launch_small_linear({pooled, Fi * 2 * Ci, seg1.wt, seg1.bias, Y1, embed_dim, nb, Fi * 2 * Ci, embed_dim, 1,
                               Y2, sk},
                              s);
          launch_small_linear({Y1, embed_dim, seg2.wt, seg2.bias, e_out, embed_dim, nb, embed_dim, embed_dim, 0}, s);
        } else {
          launch_small_linear({pooled, Fi * 2 * Ci, seg1.wt, seg1.bias, e_out, embed_dim, nb, Fi * 2 * Ci, embed_dim, 0,
                               Y2, sk},
                              s);
        }
      });
    }
  }

  // ------------------------------------------------------------ SimAM ---
  // state_dict of SimAM_ResNet{34,100}_ASP (samresnet.py:72-166): front.* backbone,
  // pooling.attention.{0,2,3} (ASP, pooling_layers.py:151-173), bottleneck.
  void build_simam_params() {
    params.clear();
    idx.clear();
    rblocks.clear();
    add("front.conv1.weight", {m_ch, 1, 3, 3});
    add_bn("front.bn1", m_ch);
    int in_planes = m_ch;
    for (int li = 0; li < 4; ++li) {
      const int planes = m_ch << li;
      for (int bi = 0; bi < nblocks[li]; ++bi) {
        const int stride = (li > 0 && bi == 0) ? 2 : 1;
        const std::string p = "front.layer" + std::to_string(li + 1) + "." + std::to_string(bi);
        RBlock rb;
        rb.stride = stride;
        rb.in_planes = in_planes;
        rb.planes = planes;
        rb.out_planes = planes;
        add(p + ".conv1.weight", {planes, in_planes, 3, 3});
        add_bn(p + ".bn1", planes);
        add(p + ".conv2.weight", {planes, planes, 3, 3});
        add_bn(p + ".bn2", planes);
        if (stride != 1 || in_planes != planes) {
          rb.has_sc = true;
          add(p + ".downsample.0.weight", {planes, in_planes, 1, 1});
          add_bn(p + ".downsample.1", planes);
        }
        rblocks.push_back(rb);
        in_planes = planes;
      }
    }
    const int CF = 8 * m_ch * (feat_dim / 8);  // ASP: in_planes * 8 * int(acoustic_dim / 8)
    add("pooling.attention.0.weight", {128, CF, 1});
    add("pooling.attention.0.bias", {128});
    add_bn("pooling.attention.2", 128);
    add("pooling.attention.3.weight", {CF, 128, 1});
    add("pooling.attention.3.bias", {CF});
    add("bottleneck.weight", {embed_dim, 2 * CF});
    add("bottleneck.bias", {embed_dim});
  }

  void finalize_simam() {
    {
      std::vector<double> sc, sh;
      bn_affine("front.bn1", sc, sh);
      const auto& w = P("front.conv1.weight");
      std::vector<float> wf(m_ch * 9), bf(m_ch);
      for (int c = 0; c < m_ch; ++c) {
        for (int q = 0; q < 9; ++q) wf[c * 9 + q] = (float)(w[c * 9 + q] * sc[c]);
        bf[c] = (float)sh[c];
      }
      stem_w = dev.upload(wf);
      stem_b = dev.upload(bf);
    }
    int ib = 0;
    for (int li = 0; li < 4; ++li)
      for (int bi = 0; bi < nblocks[li]; ++bi) {
        RBlock& rb = rblocks[ib++];
        const std::string p = "front.layer" + std::to_string(li + 1) + "." + std::to_string(bi);
        rb.c1 = pack_conv_bn(p + ".conv1.weight", p + ".bn1", rb.planes, rb.in_planes, 9);
        rb.c2 = pack_conv_bn(p + ".conv2.weight", p + ".bn2", rb.planes, rb.planes, 9);
        if (rb.has_sc)
          rb.sc = pack_conv_bn(p + ".downsample.0.weight", p + ".downsample.1", rb.planes, rb.in_planes, 1);
      }
    // reference channel index c*F4 + f of x.reshape(B, C*F, T); ours f*C4 + c (frame rows [T][F][C])
    const int C4 = rblocks.back().out_planes, F4 = feat_dim / 8, CF = C4 * F4;
    auto ref_ch = [&](int k) { return (k % C4) * F4 + k / C4; };
    {
      const auto& W = P("pooling.attention.0.weight");
      std::vector<float> wp((size_t)128 * CF);
      for (int n = 0; n < 128; ++n)
        for (int k = 0; k < CF; ++k) wp[(size_t)n * CF + k] = W[(size_t)n * CF + ref_ch(k)];
      asp1 = pack_conv(wp, 128, CF, 1, P("pooling.attention.0.bias").data(), "pooling.attention.2");
    }
    {
      const auto& W = P("pooling.attention.3.weight");
      const auto& bb = P("pooling.attention.3.bias");
      std::vector<float> wp((size_t)CF * 128), bp(CF);
      for (int n = 0; n < CF; ++n) {
        for (int k = 0; k < 128; ++k) wp[(size_t)n * 128 + k] = W[(size_t)ref_ch(n) * 128 + k];
        bp[n] = bb[ref_ch(n)];
      }
      asp2 = pack_conv(wp, CF, 128, 1, bp.data(), "");
    }
    {
      const auto& W = P("bottleneck.weight");
      const int K = 2 * CF;
      std::vector<float> wp((size_t)embed_dim * K);
      for (int n = 0; n < embed_dim; ++n)
        for (int sidx = 0; sidx < 2; ++sidx)
          for (int k = 0; k < CF; ++k)
            wp[(size_t)n * K + sidx * CF + k] = W[(size_t)n * K + sidx * CF + ref_ch(k)];
      simam_head = pack_lin(wp.data(), embed_dim, K, K, P("bottleneck.bias").data());
    }
  }

  size_t simam_ws_floats(int B, int T, size_t* offs) const {
    const int bc = resnet_chunk(B, T);
    const RShapes r = resnet_shapes(T);
    const size_t CF = (size_t)r.C4 * r.F4, cmax = (size_t)rblocks.back().out_planes;
    const size_t nchunk = (size_t)std::max(1, ceil_div(2048, bc));
    const size_t sizes[] = {bc * r.big, bc * r.big, bc * r.y1, bc * r.y2, bc * std::max<size_t>(r.sc, 1),
                            (size_t)bc * 2 * CF,
                            (size_t)bc * nchunk * 2 * cmax * 2,  // f64 moment partials
                            (size_t)bc * 2 * cmax,                // mean / 1/(4(v+l))
                            (size_t)bc * r.T4 * CF,               // frame rows [T][F*C]
                            (size_t)bc * r.T4 * 128,              // attention hidden
                            (size_t)bc * r.T4 * CF};              // attention logits
    size_t o = 0;
    for (int i = 0; i < 11; ++i) {
      if (offs) offs[i] = o;
      o += (sizes[i] + 63) / 64 * 64;
    }
    return o;
  }

  void forward_simam(const float* feats, int B, int T, float* embed, float* ws, hipStream_t s) {
    const int bc = resnet_chunk(B, T);
    size_t off[11];
    simam_ws_floats(B, T, off);
    float* X = ws + off[0];
    float* O = ws + off[1];
    float* Y1 = ws + off[2];
    float* Z = ws + off[3];
    float* SC = ws + off[4];
    float* pooled = ws + off[5];
    double* part = reinterpret_cast<double*>(ws + off[6]);
    float* coef = ws + off[7];
    float* Xt = ws + off[8];
    float* att = ws + off[9];
    float* logit = ws + off[10];
    for (int b0 = 0; b0 < B; b0 += bc) {
      const int nb = std::min(bc, B - b0);
      int Fi = feat_dim, Ti = T, Ci = m_ch;
      run("stem", 0, s, [&] {
        launch_resnet_stem(feats + (size_t)b0 * T * feat_dim, nb, T, feat_dim, m_ch, stem_w, stem_b, X, s);
      });
      float* x = X;
      float* o = O;
      for (const RBlock& rb : rblocks) {
        const int Fo = (Fi - 1) / rb.stride + 1, To = (Ti - 1) / rb.stride + 1;
        const float* res = x;
        if (rb.has_sc) {
          gemm2d("shortcut", rb.sc, x, Ci, SC, rb.planes, nb, Fi, Ti, 1, rb.stride, 0, kActNone, nullptr, 0, s);
          res = SC;
        }
        if (rb.stride == 1 && img_ok(rb.c1, rb.planes)) {
          const Conv3x3Args a{x, Y1, nb, Fi, Ti, rb.c1.frag, rb.c1.bias, rb.c1.scale, rb.c1.shift, nullptr, 1, conv3x3_img_on};
          run("res_conv3x3", 2.0 * nb * Fi * Ti * rb.c1.N * rb.c1.K, s, [&] { launch_conv3x3_img(a, rb.planes, s); });
        } else {
          gemm2d("res_conv3x3", rb.c1, x, Ci, Y1, rb.planes, nb, Fi, Ti, 3, rb.stride, 1, kActRelu, nullptr, 0, s);
        }
        if (img_ok(rb.c2, rb.planes)) {
          const Conv3x3Args a{Y1, Z, nb, Fo, To, rb.c2.frag, rb.c2.bias, rb.c2.scale, rb.c2.shift, nullptr, 0, conv3x3_img_on};
          run("res_conv3x3", 2.0 * nb * Fo * To * rb.c2.N * rb.c2.K, s, [&] { launch_conv3x3_img(a, rb.planes, s); });
        } else {
          gemm2d("res_conv3x3", rb.c2, Y1, rb.planes, Z, rb.planes, nb, Fo, To, 3, 1, 1, kActNone, nullptr, 0, s);
        }
        run("simam", 0, s, [&] { launch_simam(Z, res, o, nb, Fo * To, rb.planes, part, coef, s); });
        std::swap(x, o);
        Fi = Fo;
        Ti = To;
        Ci = rb.planes;
      }
      const int CF = Fi * Ci;
      run("asp_rows", 0, s, [&] { launch_nhwc_to_tfc(x, Xt, nb, Fi, Ti, Ci, s); });
      gemm("asp_linear1", asp1, Xt, CF, att, 128, nb * Ti, Ti, 1, 0, kActRelu, s);
      gemm("asp_linear2", asp2, att, 128, logit, CF, nb * Ti, Ti, 1, 0, kActNone, s);
      run("asp_pool_head", 0, s, [&] {
        launch_astp_pool(logit, Xt, nb, Ti, CF, pooled, s, nullptr, 1e-5f);
        // split-K partials in the free conv1 buffer
        launch_small_linear({pooled, 2 * CF, simam_head.wt, simam_head.bias, embed + (size_t)b0 * embed_dim,
                             embed_dim, nb, 2 * CF, embed_dim, 0, Y1, off[3] - off[2]},
                            s);
      });
    }
  }

  // Res2Net chain weights for res2_chain.hip: W_i [w][w][3] -> bf16 hi / lo in
  // MFMA B-fragment order [7][3w/16][2][w/32][64 lanes][8], k = tap * w + c;
  // conv bias and eval-BN affine per step [7][w].
  void pack_res2(Block& b, const std::string& p, int w) {
    const int KS = 3 * w / 16, NT = w / 32;
    std::vector<uint16_t> pk((size_t)7 * KS * 2 * NT * 64 * 8);
    std::vector<float> bias((size_t)7 * w), sc((size_t)7 * w), sh((size_t)7 * w);
    for (int i = 0; i < 7; ++i) {
      const std::string ci = p + ".1.convs." + std::to_string(i);
      const auto& W = P(ci + ".weight");
      const auto& bb = P(ci + ".bias");
      std::vector<double> s, t;
      bn_affine(p + ".1.bns." + std::to_string(i), s, t);
      for (int n = 0; n < w; ++n) {
        bias[(size_t)i * w + n] = bb[n];
        sc[(size_t)i * w + n] = (float)s[n];
        sh[(size_t)i * w + n] = (float)t[n];
      }
      for (int ks = 0; ks < KS; ++ks)
        for (int jt = 0; jt < NT; ++jt)
          for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) {
              const int n = jt * 32 + (l & 31), k = ks * 16 + 8 * (l >> 5) + e;
              const float v = W[((size_t)n * w + k % w) * 3 + k / w];
              const uint16_t hi = f2bf(v), lo = f2bf(v - bf2f(hi));
              const size_t o = ((((size_t)i * KS + ks) * 2) * NT + jt) * 64 + l;
              pk[o * 8 + e] = hi;
              pk[(o + (size_t)NT * 64) * 8 + e] = lo;
            }
    }
    b.r2w = dev.upload_u16(pk);
    b.r2b = dev.upload(bias);
    b.r2s = dev.upload(sc);
    b.r2t = dev.upload(sh);
  }

  void finalize_ecapa() {
    const int w = C / 8;
    layer1 = pack_conv(P("layer1.conv.weight"), C, feat_dim, 5, P("layer1.conv.bias").data(), "layer1.bn");
    for (int li = 0; li < 3; ++li) {
      const std::string p = "layer" + std::to_string(li + 2) + ".se_res2block";
      Block& b = blk[li];
      b.c1 = pack_conv(P(p + ".0.conv.weight"), C, C, 1, P(p + ".0.conv.bias").data(), p + ".0.bn");
      for (int i = 0; i < 7; ++i) {
        const std::string ci = p + ".1.convs." + std::to_string(i);
        b.res2[i] = pack_conv(P(ci + ".weight"), w, w, 3, P(ci + ".bias").data(),
                              p + ".1.bns." + std::to_string(i));
      }
      if (res2_chain_supported(w, li + 2)) pack_res2(b, p, w);
      b.c3 = pack_conv(P(p + ".2.conv.weight"), C, C, 1, P(p + ".2.conv.bias").data(), p + ".2.bn");
      b.se1 = pack_lin(P(p + ".3.linear1.weight").data(), 128, C, C, P(p + ".3.linear1.bias").data());
      b.se2 = pack_lin(P(p + ".3.linear2.weight").data(), C, 128, 128, P(p + ".3.linear2.bias").data());
    }
    conv = pack_conv(P("conv.weight"), 1536, 3 * C, 1, P("conv.bias").data(), "");
    {
      std::vector<float> wg = P("conv.weight");  // [1536][3C]
      for (int n = 0; n < 1536; ++n)
        for (int c = 0; c < C; ++c) {
          float* r = wg.data() + (size_t)n * 3 * C;
          r[C + c] = (float)((double)r[C + c] + (double)r[2 * C + c]);
        }
      conv_g = pack_conv(wg, 1536, 3 * C, 1, P("conv.bias").data(), "");
    }
    const auto& l1 = P("pool.linear1.weight");
    const int l1k = glob ? 4608 : 1536;
    {
      std::vector<float> wx((size_t)128 * 1536);
      for (int n = 0; n < 128; ++n)
        for (int k = 0; k < 1536; ++k) wx[(size_t)n * 1536 + k] = l1[(size_t)n * l1k + k];
      pool1 = pack_conv(wx, 128, 1536, 1, P("pool.linear1.bias").data(), "");
      if (glob) {
        // columns 1536..4607 multiply the (constant over T) mean/std context:
        // folded into a per-utterance bias computed by small_linear.
        pool1_ctx = pack_lin(l1.data() + 1536, 128, 3072, l1k, P("pool.linear1.bias").data());
      }
    }
    pool2 = pack_conv(P("pool.linear2.weight"), 1536, 128, 1, P("pool.linear2.bias").data(), "");
    pool2_frag = pack_frag(P("pool.linear2.weight"), 1536, 128);
    // head: y = Linear(BN(p)) [-> bn2] folded to y = W' p + b'
    {
      std::vector<double> s, t;
      bn_affine("bn", s, t);
      const auto& W = P("linear.weight");
      const auto& bb = P("linear.bias");
      const int D = embed_dim;
      std::vector<double> s2(D, 1.0), t2(D, 0.0);
      if (emb_bn) bn_affine("bn2", s2, t2);
      std::vector<float> wf((size_t)D * 3072), bf(D);
      for (int n = 0; n < D; ++n) {
        double acc = bb[n];
        for (int k = 0; k < 3072; ++k) {
          const double wv = W[(size_t)n * 3072 + k];
          wf[(size_t)n * 3072 + k] = (float)(s2[n] * wv * s[k]);
          acc += wv * t[k];
        }
        bf[n] = (float)(s2[n] * acc + t2[n]);
      }
      head = pack_lin(wf.data(), D, 3072, 3072, bf.data());
    }
  }

  // --------------------------------------------------------------- launch --
  template <typename F>
  void run(const char* tag, double flops, hipStream_t s, F&& f) {
    if (!prof) {
      f();
      return;
    }
    ProfEntry& e = prof_map[tag];
    if (e.used == e.ev.size()) {
      hipEvent_t a, b;
      WSP_HIP(hipEventCreate(&a));
      WSP_HIP(hipEventCreate(&b));
      e.ev.emplace_back(a, b);
    }
    auto& pr = e.ev[e.used++];
    e.flops += flops;  // summed; profile_query reports the mean per launch
    WSP_HIP(hipEventRecord(pr.first, s));
    f();
    WSP_HIP(hipEventRecord(pr.second, s));
  }

  void gemm(const char* tag, const ConvW& cw, const float* a0, int lda, float* out, int ldo, int M,
            int T, int dil, int pad, int act, hipStream_t s, const float* row_bias = nullptr,
            bool use_bias = true, int role = 0) {
    ConvGemmArgs g{};
    g.role = role;
    g.a[0] = g.a[1] = g.a[2] = a0;
    g.lda[0] = g.lda[1] = g.lda[2] = lda;
    g.cseg[0] = 0;
    g.cseg[1] = g.cseg[2] = g.cseg[3] = cw.cin;
    fill(g, cw, M, T, dil, pad, out, ldo, act, row_bias, use_bias);
    run(tag, 2.0 * M * cw.N * cw.K, s, [&] { launch(g, cw, s); });
  }
  void launch(const ConvGemmArgs& g, const ConvW& cw, hipStream_t s) {
    if (precision == 1)
      launch_conv_gemm_x3(g, cw.whi, cw.wlo, x3_variant, s);
    else
      launch_conv_gemm(g, s);
  }
  void fill(ConvGemmArgs& g, const ConvW& cw, int M, int T, int dil, int pad, float* out, int ldo,
            int act, const float* row_bias, bool use_bias) {
    g.cin = cw.cin;
    g.taps = cw.taps;
    g.dil = dil;
    g.pad = pad;
    g.M = M;
    g.T = T;
    g.N = cw.N;
    g.w = cw.w;
    g.K = cw.K;
    g.Kp = cw.Kp;
    g.bias = use_bias ? cw.bias : nullptr;
    g.row_bias = row_bias;
    g.scale = cw.scale;
    g.shift = cw.shift;
    g.out = out;
    g.ldo = ldo;
    g.act = act;
    g.seg = cur_seg;
    g.nseg = cur_nseg;
  }

  // M = frame rows of the batch (B * T, or the segment total)
  // utterances per ECAPA forward chunk (uniform batches): every activation operand, the widest
  // being the [M][1536] ASTP input / logits, must stay < 2 GiB (32-bit buffer offsets); larger
  // batches run as consecutive chunks over one chunk-sized workspace (as resnet_chunk)
  int ecapa_chunk(int B, int T) const {
    const size_t per = (size_t)T * std::max(C, 1536) * sizeof(float);
    int bc = (int)std::max<size_t>(1, ((size_t)1 << 31) / 8 * 7 / per);
    bc = std::min(bc, B);
    const int chunks = (B + bc - 1) / bc;
    return (B + chunks - 1) / chunks;
  }
  size_t ecapa_ws_floats(int B, size_t M, size_t* offs) const {
    const size_t sizes[] = {M * C, M * C, M * C, M * C,           // x1..x4
                            M * C, M * C, M * C,                   // h1..h3
                            (size_t)B * C, (size_t)B * 128, (size_t)B * C,  // gmean, ghid, gate
                            M * 1536, M * 128, M * 1536,           // xp, att, logit
                            (size_t)B * 3072, (size_t)B * 128, (size_t)B * 3072,  // gstats, rowb, pooled
                            ((M + 127) / 128) * 2 * (size_t)C * 2};  // SE column-sum partials (f64)
    size_t o = 0;
    for (int i = 0; i < 17; ++i) {
      if (offs) offs[i] = o;
      o += (sizes[i] + 63) / 64 * 64;  // 256-B alignment
    }
    return o;
  }

  // seg (device [B+1] row offsets) non-null: ragged batch of M rows; T unused by the
  // kernels then (per-utterance lengths come from seg).
  void forward_ecapa(const float* feats, int B, int T, float* embed, float* ws, hipStream_t s,
                     const int* seg = nullptr, int M_seg = 0) {
    const int M = seg ? M_seg : B * T, w = C / 8;
    cur_seg = seg;
    cur_nseg = B;
    size_t off[17];
    ecapa_ws_floats(B, M, off);
    float* x[5] = {nullptr, ws + off[0], ws + off[1], ws + off[2], ws + off[3]};
    float* h1 = ws + off[4];
    float* h2 = ws + off[5];
    float* h3 = ws + off[6];
    float* gmean = ws + off[7];
    float* ghid = ws + off[8];
    float* gate = ws + off[9];
    float* xp = ws + off[10];
    float* att = ws + off[11];
    float* logit = ws + off[12];
    float* gstats = ws + off[13];
    float* rowb = ws + off[14];
    float* pooled = ws + off[15];
    double* sesum = reinterpret_cast<double*>(ws + off[16]);
    // SE squeeze fused into conv3's epilogue (per-utterance f64 column sums) on the
    // bf16x3 path for uniform batches whose utterances span >= one block of rows
    const int se_bm = precision == 1 ? conv_gemm_x3_block_rows(ConvGemmArgs{.N = C}, x3_variant) : 0;
    const bool se_fused = precision == 1 && !seg && T >= se_bm;

    gemm("layer1", layer1, feats, feat_dim, x[1], C, M, T, 1, 2, kActRelu, s);
    for (int li = 0; li < 3; ++li) {
      const Block& b = blk[li];
      const int dil = li + 2;
      const float* xin = x[li + 1];
      gemm("conv1x1_CxC", b.c1, xin, C, h1, C, M, T, 1, 0, kActRelu, s, nullptr, true, 1);
      if (precision == 1 && res2_fused && b.r2w) {
        // the whole chain in one launch (res2_chain.hip)
        Res2Args r{};
        r.x = h1;
        r.out = h2;
        r.ldx = r.ldo = C;
        r.M = M;
        r.T = T;
        r.dil = dil;
        r.rout = res2_chain_rout(dil, w == 128 ? res2_variant : std::min(res2_variant, 3), M);
        r.seg = seg;
        r.nseg = B;
        r.w = b.r2w;
        r.bias = b.r2b;
        r.scale = b.r2s;
        r.shift = b.r2t;
        r.variant = w == 128 ? res2_variant : std::min(res2_variant, 3);
        run("res2_k3", 7 * 2.0 * M * w * 3 * w, s, [&] { launch_res2_chain(r, w, s); });
      }
      for (int i = 0; i < 7 && !(precision == 1 && res2_fused && b.r2w); ++i) {
        ConvGemmArgs g{};
        if (i == 0) {
          g.amode = kACat;
          g.a[0] = g.a[1] = g.a[2] = h1;
          g.lda[0] = g.lda[1] = g.lda[2] = C;
          g.cseg[0] = 0;
          g.cseg[1] = g.cseg[2] = g.cseg[3] = w;
        } else {
          g.amode = kAAdd;
          g.a[0] = h1 + i * w;
          g.a[1] = h2 + (i - 1) * w;
          g.a[2] = h1;
          g.lda[0] = g.lda[1] = g.lda[2] = C;
        }
        fill(g, b.res2[i], M, T, dil, dil, h2 + i * w, C, kActRelu, nullptr, true);
        run("res2_k3", 2.0 * M * w * 3 * w, s, [&] { launch(g, b.res2[i], s); });
      }
      {
        ConvGemmArgs g{};
        g.amode = kACat;
        g.a[0] = h2;
        g.a[1] = h1 + 7 * w;
        g.a[2] = h1;
        g.lda[0] = g.lda[1] = g.lda[2] = C;
        g.cseg[0] = 0;
        g.cseg[1] = 7 * w;
        g.cseg[2] = g.cseg[3] = C;
        fill(g, b.c3, M, T, 1, 0, h3, C, kActRelu, nullptr, true);
        g.role = 1;
        if (se_fused) g.colsum = sesum;
        run("conv1x1_CxC", 2.0 * M * C * C, s, [&] { launch(g, b.c3, s); });
      }
      run("se", 0, s, [&] {
        if (se_fused) launch_colsum_mean(sesum, se_bm, T, B, C, gmean, C, s);
        else launch_frame_stats(h3, C, B, T, C, gmean, C, 0, 0, s, seg);
        launch_small_linear({gmean, C, b.se1.wt, b.se1.bias, ghid, 128, B, C, 128, 1}, s);
        launch_small_linear({ghid, 128, b.se2.wt, b.se2.bias, gate, C, B, 128, C, 3}, s);
        // cat_gate: the last block stores only g4 * h3 (conv_cat adds out3 through its weights)
        launch_residual_scale(cat_gate && li == 2 ? nullptr : xin, h3, gate, x[li + 2], B, T, C, s, seg, M);
      });
    }
    {
      ConvGemmArgs g{};
      g.amode = kACat;
      g.a[0] = x[2];
      g.a[1] = x[3];
      g.a[2] = x[4];
      g.lda[0] = g.lda[1] = g.lda[2] = C;
      g.cseg[0] = 0;
      g.cseg[1] = C;
      g.cseg[2] = 2 * C;
      g.cseg[3] = 3 * C;
      const ConvW& cc = cat_gate ? conv_g : conv;
      fill(g, cc, M, T, 1, 0, xp, 1536, kActRelu, nullptr, true);
      run("conv_cat", 2.0 * M * 1536 * 3 * C, s, [&] { launch(g, cc, s); });
    }
    if (glob) {
      run("glob_ctx", 0, s, [&] {
        launch_frame_stats(xp, 1536, B, T, 1536, gstats, 3072, 1, 1536, s, seg);
        launch_small_linear({gstats, 3072, pool1_ctx.wt, pool1_ctx.bias, rowb, 128, B, 3072, 128, 0}, s);
      });
      gemm("pool_linear1", pool1, xp, 1536, att, 128, M, T, 1, 0, kActTanh, s, rowb, false);
    } else {
      gemm("pool_linear1", pool1, xp, 1536, att, 128, M, T, 1, 0, kActTanh, s);
    }
    if (precision == 1 && astp_fused_on) {
      // linear2 + softmax over frames + attentive mean / std in one pass (astp_fused.hip)
      AstpArgs a{att, xp, 1536, B, T, 1536, seg, pool2_frag, pool2.bias, 1e-7f, pooled};
      run("astp", 2.0 * M * 1536 * 128, s, [&] { launch_astp_fused(a, s); });
    } else {
      gemm("pool_linear2", pool2, att, 128, logit, 1536, M, T, 1, 0, kActNone, s);
      run("astp", 0, s, [&] { launch_astp_pool(logit, xp, B, T, 1536, pooled, s, seg); });
    }
    run("head", 0, s, [&] {
      launch_small_linear({pooled, 3072, head.wt, head.bias, embed, embed_dim, B, 3072, embed_dim, 0}, s);
    });
    cur_seg = nullptr;
    cur_nseg = 0;
  }
};

}  // namespace wsp
