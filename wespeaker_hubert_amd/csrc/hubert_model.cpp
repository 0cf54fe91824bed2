// HuBERT-base SSL front end runtime (arch "HuBERT_base").
//
// Replaces S3prlFrontend.forward (wespeaker/frontend/s3prl.py:80-93) with the
// s3prl `hubert` upstream (third party, restated in oracle/hubert_ref.py):
//   conv0 + GroupNorm + GELU           launch_hubert_conv0          [B][T0][512]
//   6 x strided conv + GELU            implicit GEMM (stride 2)     [B][T][512]
//   LayerNorm(512) -> Linear(512->768) layernorm + GEMM             x [B][T][768]
//   x + GELU(pos_conv(x)) -> LN        grouped GEMM (16 x 48 ch, k128) + layernorm
//   12 x post-LN transformer layer     GEMM qkv | mha | GEMM out(+x) | LN |
//                                      GEMM fc1 GELU | GEMM fc2(+x) | LN
//   Featurizer + length match          accumulated inside each hidden-state LN
// Parameters arrive under the reference checkpoint's names
// ("frontend.upstream.upstream.model." + fairseq names, "frontend.featurizer.weights").
#include "model_impl.h"

namespace wsp {

namespace {

constexpr int kConvDim = 512, kHidden = 768, kLayers = 12, kHeads = 12, kFfn = 3072;
constexpr int kPosK = 128, kPosGroups = 16, kPosGin = kHidden / kPosGroups, kPosGout = 64;
constexpr int kConvK[7] = {10, 3, 3, 3, 3, 2, 2};
constexpr int kConvS[7] = {5, 2, 2, 2, 2, 2, 2};
constexpr int kDownsample = 320;
const char* const kPre = "frontend.upstream.upstream.model.";

std::string hp(const std::string& n) { return std::string(kPre) + n; }

}  // namespace

void Model::Impl::build_hubert_params() {
  for (int i = 0; i < 7; ++i) {
    add(hp("feature_extractor.conv_layers." + std::to_string(i) + ".0.weight"),
        {kConvDim, i == 0 ? 1 : kConvDim, kConvK[i]});
    if (i == 0) {
      add(hp("feature_extractor.conv_layers.0.2.weight"), {kConvDim});
      add(hp("feature_extractor.conv_layers.0.2.bias"), {kConvDim});
    }
  }
  add(hp("layer_norm.weight"), {kConvDim});
  add(hp("layer_norm.bias"), {kConvDim});
  add(hp("post_extract_proj.weight"), {kHidden, kConvDim});
  add(hp("post_extract_proj.bias"), {kHidden});
  add(hp("encoder.pos_conv.0.bias"), {kHidden});
  add(hp("encoder.pos_conv.0.weight_g"), {1, 1, kPosK});
  add(hp("encoder.pos_conv.0.weight_v"), {kHidden, kPosGin, kPosK});
  add(hp("encoder.layer_norm.weight"), {kHidden});
  add(hp("encoder.layer_norm.bias"), {kHidden});
  for (int l = 0; l < kLayers; ++l) {
    const std::string p = "encoder.layers." + std::to_string(l) + ".";
    for (const char* proj : {"k_proj", "v_proj", "q_proj", "out_proj"}) {
      add(hp(p + "self_attn." + proj + ".weight"), {kHidden, kHidden});
      add(hp(p + "self_attn." + proj + ".bias"), {kHidden});
    }
    add(hp(p + "self_attn_layer_norm.weight"), {kHidden});
    add(hp(p + "self_attn_layer_norm.bias"), {kHidden});
    add(hp(p + "fc1.weight"), {kFfn, kHidden});
    add(hp(p + "fc1.bias"), {kFfn});
    add(hp(p + "fc2.weight"), {kHidden, kFfn});
    add(hp(p + "fc2.bias"), {kHidden});
    add(hp(p + "final_layer_norm.weight"), {kHidden});
    add(hp(p + "final_layer_norm.bias"), {kHidden});
  }
  add("frontend.featurizer.weights", {kLayers + 1});
}

void Model::Impl::finalize_hubert() {
  h_conv0_w = dev.upload(P(hp("feature_extractor.conv_layers.0.0.weight")));
  h_gn_g = dev.upload(P(hp("feature_extractor.conv_layers.0.2.weight")));
  h_gn_b = dev.upload(P(hp("feature_extractor.conv_layers.0.2.bias")));
  for (int i = 1; i < 7; ++i)
    h_conv[i] = pack_conv(P(hp("feature_extractor.conv_layers." + std::to_string(i) + ".0.weight")), kConvDim,
                          kConvDim, kConvK[i], nullptr, "");
  h_ln0_g = dev.upload(P(hp("layer_norm.weight")));
  h_ln0_b = dev.upload(P(hp("layer_norm.bias")));
  h_proj = pack_conv(P(hp("post_extract_proj.weight")), kHidden, kConvDim, 1, P(hp("post_extract_proj.bias")).data(),
                     "");
  {
    // weight_norm(dim=2): w[o][i][k] = g[k] * v[o][i][k] / ||v[:, :, k]||  (f64), then the
    // grouped layout: output column g*64 + o' (o' < 48 real, 48..63 zero) reading the
    // 48 input channels of group g.
    const auto& g = P(hp("encoder.pos_conv.0.weight_g"));
    const auto& v = P(hp("encoder.pos_conv.0.weight_v"));
    const auto& bias = P(hp("encoder.pos_conv.0.bias"));
    std::vector<double> nrm(kPosK, 0.0);
    for (int o = 0; o < kHidden; ++o)
      for (int i = 0; i < kPosGin; ++i)
        for (int k = 0; k < kPosK; ++k) {
          const double x = v[((size_t)o * kPosGin + i) * kPosK + k];
          nrm[k] += x * x;
        }
    const int Np = kPosGroups * kPosGout;
    std::vector<float> w((size_t)Np * kPosGin * kPosK, 0.f), b(Np, 0.f);
    for (int o = 0; o < kHidden; ++o) {
      const int col = (o / kPosGin) * kPosGout + o % kPosGin;
      b[col] = bias[o];
      for (int i = 0; i < kPosGin; ++i)
        for (int k = 0; k < kPosK; ++k)
          w[((size_t)col * kPosGin + i) * kPosK + k] =
              (float)(g[k] * (double)v[((size_t)o * kPosGin + i) * kPosK + k] / std::sqrt(nrm[k]));
    }
    h_pos = pack_conv(w, Np, kPosGin, kPosK, b.data(), "");
  }
  h_enc_g = dev.upload(P(hp("encoder.layer_norm.weight")));
  h_enc_b = dev.upload(P(hp("encoder.layer_norm.bias")));
  h_layers.assign(kLayers, HLayer{});
  for (int l = 0; l < kLayers; ++l) {
    const std::string p = "encoder.layers." + std::to_string(l) + ".";
    HLayer& L = h_layers[l];
    // fused [q | k | v] projection: rows 0..767 q, 768.. k, 1536.. v
    std::vector<float> w((size_t)3 * kHidden * kHidden), b(3 * kHidden);
    const char* order[3] = {"q_proj", "k_proj", "v_proj"};
    for (int j = 0; j < 3; ++j) {
      const auto& wj = P(hp(p + "self_attn." + order[j] + ".weight"));
      const auto& bj = P(hp(p + "self_attn." + order[j] + ".bias"));
      std::copy(wj.begin(), wj.end(), w.begin() + (size_t)j * kHidden * kHidden);
      std::copy(bj.begin(), bj.end(), b.begin() + j * kHidden);
    }
    L.qkv = pack_conv(w, 3 * kHidden, kHidden, 1, b.data(), "");
    L.out = pack_conv(P(hp(p + "self_attn.out_proj.weight")), kHidden, kHidden, 1,
                      P(hp(p + "self_attn.out_proj.bias")).data(), "");
    L.fc1 = pack_conv(P(hp(p + "fc1.weight")), kFfn, kHidden, 1, P(hp(p + "fc1.bias")).data(), "");
    L.fc2 = pack_conv(P(hp(p + "fc2.weight")), kHidden, kFfn, 1, P(hp(p + "fc2.bias")).data(), "");
    L.ln1_g = dev.upload(P(hp(p + "self_attn_layer_norm.weight")));
    L.ln1_b = dev.upload(P(hp(p + "self_attn_layer_norm.bias")));
    L.ln2_g = dev.upload(P(hp(p + "final_layer_norm.weight")));
    L.ln2_b = dev.upload(P(hp(p + "final_layer_norm.bias")));
  }
  // Featurizer weights: softmax over the 13 hidden states (s3prl Featurizer,
  // normalize=False), or a one-hot pick for `layer != -1` (s3prl.py:84-87).
  const auto& fw = P("frontend.featurizer.weights");
  h_fw.assign(kLayers + 1, 0.f);
  if (h_layer_sel >= 0) {
    h_fw[h_layer_sel] = 1.f;
  } else {
    double mx = fw[0], sum = 0.0;
    for (float x : fw) mx = std::max(mx, (double)x);
    for (float x : fw) sum += std::exp((double)x - mx);
    for (int i = 0; i <= kLayers; ++i) h_fw[i] = (float)(std::exp((double)fw[i] - mx) / sum);
  }
}

int Model::Impl::hubert_cnn_frames(int N, int upto) const {
  int t = N;
  for (int i = 0; i <= upto; ++i) t = (t - kConvK[i]) / kConvS[i] + 1;
  return t;
}

// Utterances per feature-extractor chunk: the conv0 output (33 MB per 5 s
// utterance) must stay below 2 GiB (32-bit buffer offsets).
int Model::Impl::hubert_chunk(int B, int N) const {
  const size_t per = (size_t)hubert_cnn_frames(N, 0) * kConvDim * sizeof(float);
  int bc = (int)std::max<size_t>(1, ((size_t)1 << 31) / 8 * 7 / per);
  bc = std::min(bc, B);
  const int chunks = (B + bc - 1) / bc;
  return (B + chunks - 1) / chunks;
}

size_t Model::Impl::hubert_ws_floats(int B, int N, size_t* offs) const {
  const int bc = hubert_chunk(B, N);
  const size_t T0 = hubert_cnn_frames(N, 0), T1 = hubert_cnn_frames(N, 1), T = hubert_cnn_frames(N, 6);
  const size_t M = (size_t)B * T;
  const size_t sizes[] = {bc * T0 * kConvDim, bc * T1 * kConvDim, (size_t)4 * bc * kConvDim,  // cnnA, cnnB, stats
                          M * kHidden,        M * kHidden,        M * 3 * kHidden,           // x, x1, qkv
                          M * kHidden,        M * kFfn};                                     // ao, ffn / pos
  size_t o = 0;
  for (int i = 0; i < 8; ++i) {
    if (offs) offs[i] = o;
    o += (sizes[i] + 63) / 64 * 64;
  }
  return o;
}

void Model::Impl::forward_hubert(const float* wav, int B, int N, float* feats, int cmn, float* ws, hipStream_t s) {
  size_t off[8];
  hubert_ws_floats(B, N, off);
  float* cnnA = ws + off[0];
  float* cnnB = ws + off[1];
  double* stats = reinterpret_cast<double*>(ws + off[2]);
  float* x = ws + off[3];
  float* x1 = ws + off[4];
  float* qkv = ws + off[5];
  float* ao = ws + off[6];
  float* ffn = ws + off[7];
  float* pc = ffn;  // the pos_conv output is consumed before fc1 writes
  const int T0 = hubert_cnn_frames(N, 0), T = hubert_cnn_frames(N, 6);
  const int Tout = (N + kDownsample - 1) / kDownsample;
  const int M = B * T;
  const int bc = hubert_chunk(B, N);

  auto conv = [&](const char* tag, const ConvW& cw, const float* a, int lda, float* out, int ldo, int rows, int Tt,
                  int Ti, int stride, int pad, int act, const float* res, bool bias, int gcols = 0, int gcin = 0) {
    ConvGemmArgs g{};
    g.a[0] = g.a[1] = g.a[2] = a;
    g.lda[0] = g.lda[1] = g.lda[2] = lda;
    g.cseg[0] = 0;
    g.cseg[1] = g.cseg[2] = g.cseg[3] = cw.cin;
    fill(g, cw, rows, Tt, 1, pad, out, ldo, act, nullptr, bias);
    g.stride = stride;
    g.Ti = Ti;
    g.res = res;
    g.ldres = res ? ldo : 0;
    g.gcols = gcols;
    g.gcin = gcin;
    run(tag, 2.0 * rows * (gcols ? (double)cw.N * kPosGin / kPosGout : cw.N) * cw.K, s, [&] { launch(g, cw, s); });
  };
  auto ln = [&](const char* tag, const float* in, const float* add, float* out, int rows, int D, const float* gm,
                const float* bt, int layer) {
    LayerNormArgs a{};
    a.x = in;
    a.ldx = D;
    a.add = add;
    a.ldadd = kPosGroups * kPosGout;
    a.gin = kPosGin;
    a.gout = kPosGout;
    a.gamma = gm;
    a.beta = bt;
    a.eps = 1e-5f;
    a.out = out;
    a.ldo = D;
    a.M = rows;
    a.D = D;
    if (layer >= 0 && (h_fw[layer] != 0.f || (h_layer_sel < 0 && layer == 0))) {
      // weighted mode initialises at hidden state 0; one-hot mode at the chosen one
      a.feat = feats;
      a.feat_w = h_fw[layer];
      a.feat_init = (h_layer_sel >= 0 || layer == 0) ? 1 : 0;
      a.T = T;
      a.Tout = Tout;
    }
    run(tag, 0, s, [&] { launch_layernorm(a, s); });
  };

  // ---- feature extractor, utterance chunks of bc
  for (int b0 = 0; b0 < B; b0 += bc) {
    const int nb = std::min(bc, B - b0);
    run("h_conv0", 2.0 * nb * T0 * kConvDim * 10, s, [&] {
      launch_hubert_conv0(wav + (size_t)b0 * N, nb, N, N, T0, h_conv0_w, h_gn_g, h_gn_b, stats, cnnA, s);
    });
    float* src = cnnA;
    float* dst = cnnB;
    int Ti = T0;
    for (int i = 1; i < 7; ++i) {
      const int To = (Ti - kConvK[i]) / kConvS[i] + 1;
      conv("h_cnn", h_conv[i], src, kConvDim, dst, kConvDim, nb * To, To, Ti, kConvS[i], 0, kActGelu, nullptr, false);
      std::swap(src, dst);
      Ti = To;
    }
    ln("h_ln", src, nullptr, src, nb * T, kConvDim, h_ln0_g, h_ln0_b, -1);
    conv("h_proj", h_proj, src, kConvDim, x + (size_t)b0 * T * kHidden, kHidden, nb * T, T, T, 1, 0, kActNone, nullptr,
         true);
  }
  // ---- encoder: x + GELU(pos_conv(x)) -> LN  (SamePad: pad 64, last output dropped)
  conv("h_pos_conv", h_pos, x, kHidden, pc, kPosGroups * kPosGout, M, T, T, 1, kPosK / 2, kActGelu, nullptr, true,
       kPosGout, kPosGin);
  ln("h_ln", x, pc, x, M, kHidden, h_enc_g, h_enc_b, 0);
  for (int l = 0; l < kLayers; ++l) {
    const HLayer& L = h_layers[l];
    conv("h_qkv", L.qkv, x, kHidden, qkv, 3 * kHidden, M, T, T, 1, 0, kActNone, nullptr, true);
    run("h_attn", 4.0 * B * kHeads * (double)T * T * (kHidden / kHeads), s,
        [&] { launch_mha(qkv, 3 * kHidden, ao, kHidden, B, T, kHeads, kHidden / kHeads, s); });
    conv("h_out_proj", L.out, ao, kHidden, x1, kHidden, M, T, T, 1, 0, kActNone, x, true);
    ln("h_ln", x1, nullptr, x, M, kHidden, L.ln1_g, L.ln1_b, -1);
    conv("h_fc1", L.fc1, x, kHidden, ffn, kFfn, M, T, T, 1, 0, kActGelu, nullptr, true);
    conv("h_fc2", L.fc2, ffn, kFfn, x1, kHidden, M, T, T, 1, 0, kActNone, x, true);
    ln("h_ln", x1, nullptr, x, M, kHidden, L.ln2_g, L.ln2_b, l + 1);
  }
  if (cmn) run("h_cmn", 0, s, [&] { launch_cmn_rows(feats, B, Tout, kHidden, s); });
}

// ------------------------------------------------------------ Model API ---
bool Model::is_frontend() const { return impl->hubert; }

int Model::out_frames(int N) const {
  WSP_CHECK(impl->hubert, "out_frames: not a front-end handle");
  WSP_CHECK(N >= 400, "HuBERT needs at least 400 samples");
  return (N + kDownsample - 1) / kDownsample;
}

size_t Model::frontend_workspace_bytes(int B, int N) const {
  WSP_CHECK(impl->hubert, "frontend_workspace_bytes: not a front-end handle");
  WSP_CHECK(B > 0 && N >= 400, "HuBERT needs B >= 1 and N >= 400 samples");
  return impl->hubert_ws_floats(B, N, nullptr) * sizeof(float) + 256;
}

void Model::forward_frontend(const float* wav, int B, int N, float* feats, int cmn, void* ws, size_t ws_bytes,
                             hipStream_t s) {
  Impl& m = *impl;
  WSP_CHECK(m.hubert, "forward_frontend: not a front-end handle");
  WSP_CHECK(m.finalized, "forward before finalize");
  WSP_CHECK(B > 0 && N >= 400, "HuBERT needs B >= 1 and N >= 400 samples");
  const size_t M = (size_t)B * m.hubert_cnn_frames(N, 6);
  WSP_CHECK(M * kFfn * sizeof(float) < ((size_t)1 << 31) - 64,
            "HuBERT batch too large for one call (B * frames * 3072 floats must stay below 2 GiB)");
  WSP_CHECK(ws_bytes >= frontend_workspace_bytes(B, N), "workspace too small");
  float* wsf = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  m.forward_hubert(wav, B, N, feats, cmn, wsf, s);
}

}  // namespace wsp
