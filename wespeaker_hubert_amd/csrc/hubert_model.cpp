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
#include <cstring>

#include "attn.h"
#include "model_impl.h"

namespace wsp {

namespace {

constexpr int kConvDim = 512, kHidden = 768, kLayers = 12, kHeads = 12, kFfn = 3072;
constexpr int kPosK = 128, kPosGroups = 16, kPosGin = kHidden / kPosGroups, kPosGout = 64;
constexpr int kConvK[7] = {10, 3, 3, 3, 3, 2, 2};
constexpr int kConvS[7] = {5, 2, 2, 2, 2, 2, 2};
constexpr int kDownsample = 320;
constexpr int kMinSamples = 800;  // s3prl MIN_SECOND (0.05 s) * 16 kHz
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
    {
      // fc1 on LN1's input u: fc1(LN1(u)) = (u W'^T - mu cs) rstd + b + W beta, W' = W diag(gamma)
      const auto& w1 = P(hp(p + "fc1.weight"));
      const auto& b1 = P(hp(p + "fc1.bias"));
      const auto& g1 = P(hp(p + "self_attn_layer_norm.weight"));
      const auto& be1 = P(hp(p + "self_attn_layer_norm.bias"));
      std::vector<float> wf(w1.size()), bf(kFfn), cs(kFfn);
      for (int n = 0; n < kFfn; ++n) {
        double bb = b1[n], c = 0.0;
        for (int k = 0; k < kHidden; ++k) {
          const float wv = w1[(size_t)n * kHidden + k];
          wf[(size_t)n * kHidden + k] = wv * g1[k];
          bb += (double)wv * be1[k];
          const float x = wf[(size_t)n * kHidden + k];
          const uint16_t h = f2bf(x);
          c += (double)bf2f(h) + (double)bf2f(f2bf(x - bf2f(h)));
        }
        bf[n] = (float)bb;
        cs[n] = (float)c;
      }
      L.fc1f = pack_conv(wf, kFfn, kHidden, 1, bf.data(), "");
      L.fc1_cs = dev.upload(cs);
    }
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

// Host-side plan of one (uniform or ragged) batch: frames per conv level,
// feature-extractor chunks whose conv0 output stays below 2 GiB (32-bit buffer
// offsets; 33 MB per 5 s utterance), and the int32 offset tables the kernels
// read (uploaded into the workspace).
HubertPlan Model::Impl::hubert_plan(int B, const int* lens) const {
  HubertPlan pl;
  pl.B = B;
  std::vector<int> T[7], Tout(B);
  for (int k = 0; k < 7; ++k) T[k].resize(B);
  for (int b = 0; b < B; ++b) {
    WSP_CHECK(lens[b] >= 1, "HuBERT needs at least 1 sample per utterance");
    // s3prl S3PRLUpstream.forward (MIN_SECOND = 0.05): an utterance shorter than
    // 800 samples runs zero-padded to 800 (conv0 reads zeros past the real
    // samples, and its GroupNorm statistics cover the padded frames); the
    // output keeps len(range(0, W, 320)) frames of the real length W (the
    // featurizer's length match trims the extra frame).
    int t = std::max(lens[b], kMinSamples);
    for (int k = 0; k < 7; ++k) T[k][b] = t = (t - kConvK[k]) / kConvS[k] + 1;
    Tout[b] = (lens[b] + kDownsample - 1) / kDownsample;
  }
  const size_t cap = ((size_t)1 << 31) / 8 * 7 / (kConvDim * sizeof(float));  // conv0 rows per chunk
  for (int b0 = 0; b0 < B;) {
    size_t rows = 0;
    int b1 = b0;
    while (b1 < B && (b1 == b0 || rows + T[0][b1] <= cap)) rows += T[0][b1++];
    pl.chunks.push_back({b0, b1});
    b0 = b1;
  }
  // offsets: global [seg6 | fseg | seg3 | seg4 | seg5], then per chunk [wseg | seg0 .. seg6] relative to the chunk
  auto prefix = [&](const std::vector<int>& v, int lo, int hi) {
    long long acc = 0;
    pl.offs.push_back(0);
    for (int b = lo; b < hi; ++b) {
      acc += v[b];
      WSP_CHECK(acc < (1LL << 31), "HuBERT batch too large");
      pl.offs.push_back((int)acc);
    }
    return (size_t)acc;
  };
  pl.M = prefix(T[6], 0, B);
  pl.Mout = prefix(Tout, 0, B);
  // CNN layers 4..6 run once over the whole batch when the level-3 rows fit a 2 GiB operand (r5:
  // the per-chunk launches of these short layers filled 112-446 of the 256 CUs)
  pl.M3 = prefix(T[3], 0, B);
  pl.M4 = prefix(T[4], 0, B);
  pl.M5 = prefix(T[5], 0, B);
  std::vector<int> lv(lens, lens + B);
  for (auto& c : pl.chunks) {
    c.off = pl.offs.size();
    c.samples = prefix(lv, c.b0, c.b1);
    for (int k = 0; k < 7; ++k) c.rows[k] = prefix(T[k], c.b0, c.b1);
    c.row6 = 0;
    for (int b = 0; b < c.b0; ++b) c.row6 += T[6][b];
    c.row3 = 0;
    for (int b = 0; b < c.b0; ++b) c.row3 += T[3][b];
    c.sample0 = 0;
    for (int b = 0; b < c.b0; ++b) c.sample0 += lens[b];
    c.maxT0 = *std::max_element(T[0].begin() + c.b0, T[0].begin() + c.b1);
    pl.maxA = std::max(pl.maxA, c.rows[0]);
    pl.maxB = std::max(pl.maxB, c.rows[1]);
    pl.maxChunk = std::max(pl.maxChunk, c.b1 - c.b0);
    pl.maxStats = std::max(pl.maxStats, hubert_conv0_stats_doubles(c.b1 - c.b0, c.maxT0));
  }
  pl.maxT6 = *std::max_element(T[6].begin(), T[6].end());
  // layers 4..6 batch-wide: more than one chunk, level-3 rows within a 2 GiB operand, and the
  // chunk buffers (free after the chunk loop) large enough for the level-4 / level-5 rows
  pl.tail_batch = tail_batch && pl.chunks.size() > 1 && pl.M3 * kConvDim * sizeof(float) < ((size_t)1 << 31) / 8 * 7 &&
                  pl.M4 <= pl.maxA && pl.M5 <= pl.maxB;
  WSP_CHECK(pl.M * kFfn * sizeof(float) < ((size_t)1 << 31) - 64,
            "HuBERT batch too large for one call (frames * 3072 floats must stay below 2 GiB)");
  return pl;
}

size_t Model::Impl::hubert_ws_floats(const HubertPlan& pl, size_t* offs) const {
  const size_t M = pl.M;
  const size_t sizes[] = {pl.maxA * kConvDim, pl.maxB * kConvDim, 2 * pl.maxStats,  // cnnA, cnnB, stats (f64)
                          M * kHidden,        M * kHidden,        M * 3 * kHidden,                     // x, x1, qkv
                          M * kHidden,        M * kFfn,                                                // ao, ffn / pos
                          pl.offs.size(),                                                              // int32 offsets
                          M * (kHidden / 128) * 2,                                                     // LN partials
                          pl.tail_batch ? pl.M3 * kConvDim : 0};                                       // level-3 rows
  size_t o = 0;
  for (int i = 0; i < 11; ++i) {
    if (offs) offs[i] = o;
    o += (sizes[i] + 63) / 64 * 64;
  }
  return o;
}

void Model::Impl::forward_hubert(const float* wav, const HubertPlan& pl, float* feats, int cmn, float* ws,
                                 hipStream_t s) {
  size_t off[11];
  hubert_ws_floats(pl, off);
  float* cnnA = ws + off[0];
  float* cnnB = ws + off[1];
  double* stats = reinterpret_cast<double*>(ws + off[2]);
  float* x = ws + off[3];
  float* x1 = ws + off[4];
  float* qkv = ws + off[5];
  float* ao = ws + off[6];
  float* ffn = ws + off[7];
  float* cnn6 = qkv;  // [M][512] CNN output of the whole batch; qkv is first written by layer 0
  float* pc = ffn;  // the pos_conv output is consumed before fc1 writes
  int* dseg = reinterpret_cast<int*>(ws + off[8]);
  float* lnst = ws + off[9];  // LN1 row statistics: [M][6] (mean, M2) of 128-column pieces
  // pageable source: the copy is staged before hipMemcpyAsync returns, so pl.offs may go away
  WSP_HIP(hipMemcpyAsync(dseg, pl.offs.data(), pl.offs.size() * sizeof(int), hipMemcpyHostToDevice, s));
  const int B = pl.B;
  const int M = (int)pl.M;
  const int* seg6 = dseg;           // [B+1] hidden-state rows per utterance
  const int* fseg = dseg + B + 1;   // [B+1] output feature rows per utterance
  const int* gseg3 = dseg + 2 * (B + 1);  // [B+1] batch-wide rows of conv levels 3, 4, 5
  const int* gseg4 = dseg + 3 * (B + 1);
  const int* gseg5 = dseg + 4 * (B + 1);
  float* cnn3 = ws + off[10];       // tail_batch: [M3][512] level-3 rows of the whole batch

  auto conv = [&](const char* tag, const ConvW& cw, const float* a, int lda, float* out, int ldo, int rows, int Ti,
                  int stride, int pad, int act, const float* res, bool bias, const int* oseg, const int* iseg, int nseg,
                  int gcols = 0, int gcin = 0, const ConvGemmArgs* lnf = nullptr) {
    ConvGemmArgs g{};
    if (lnf) {  // LayerNorm fold fields
      g.lnmode = lnf->lnmode;
      g.ln_out = lnf->ln_out;
      g.ln_in = lnf->ln_in;
      g.ln_parts = lnf->ln_parts;
      g.ln_cs = lnf->ln_cs;
      g.ln_g = lnf->ln_g;
      g.ln_b = lnf->ln_b;
      g.ln_eps = lnf->ln_eps;
    }
    g.a[0] = g.a[1] = g.a[2] = a;
    g.lda[0] = g.lda[1] = g.lda[2] = lda;
    g.cseg[0] = 0;
    g.cseg[1] = g.cseg[2] = g.cseg[3] = cw.cin;
    fill(g, cw, rows, 1, 1, pad, out, ldo, act, nullptr, bias);
    g.stride = stride;
    g.Ti = oseg ? Ti : 1;  // row-local (taps 1) GEMMs: uniform T = Ti = 1 so input row == output row
    g.res = res;
    g.ldres = res ? ldo : 0;
    g.gcols = gcols;
    g.gcin = gcin;
    g.seg = oseg;  // taps==1 projections pass null: row-local, no utterance structure needed
    g.iseg = iseg;
    g.nseg = nseg;
    // x3_variant 5 only: the long-K / GELU GEMMs (CNN, fc1, fc2) on the 16x16x32 form of the 256 x 256
    // tile (r3 A/B: CNN -2 %, fc1 -3 %, fc2 -6 % per launch), QKV / out_proj on 32x32.  Under the
    // default 7 (and 8) every one of these GEMMs (N % 256 == 0) takes the LDS-DMA 16x16x32 tile, which
    // is faster than the register-staged 16x16x32 tile for QKV and out_proj too (tools/gemm_check,
    // profiles/r5a_gemm_check.txt: qkv / out_proj / fc1 / fc2 / cnn.c1 per launch, families 6 vs 7)
    const bool mf16 = x3_variant == 5 && (std::strncmp(tag, "h_cnn", 5) == 0 || std::strcmp(tag, "h_fc1") == 0 ||
                                          std::strcmp(tag, "h_fc2") == 0);
    run(tag, 2.0 * rows * (gcols ? (double)cw.N * kPosGin / kPosGout : cw.N) * cw.K, s, [&] {
      if (precision == 1)
        launch_conv_gemm_x3(g, cw.whi, cw.wlo, mf16 ? 6 : x3_variant, s);
      else
        launch(g, cw, s);
    });
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
      a.seg = seg6;
      a.fseg = fseg;
      a.nseg = B;
    }
    run(tag, 0, s, [&] { launch_layernorm(a, s); });
  };

  // ---- feature extractor, utterance chunks
  for (const HubertChunk& c : pl.chunks) {
    const int nb = c.b1 - c.b0;
    const int* cs = dseg + c.off;  // [wseg | seg0 .. seg6], each nb+1, relative to the chunk
    auto lvl = [&](int k) { return cs + (size_t)(k + 1) * (nb + 1); };
    run("h_conv0", 2.0 * c.rows[0] * kConvDim * 10, s, [&] {
      launch_hubert_conv0(wav + c.sample0, nb, 0, 0, c.maxT0, h_conv0_w, h_gn_g, h_gn_b, stats, cnnA, s, cs, lvl(0));
    });
    float* src = cnnA;
    float* dst = cnnB;
    // profiling sub-classes per layer: h_cnn.c<i>
    static const char* kCnn[7] = {"", "h_cnn.c1", "h_cnn.c2", "h_cnn.c3", "h_cnn.c4", "h_cnn.c5", "h_cnn.c6"};
    const int last = pl.tail_batch ? 3 : 6;
    for (int i = 1; i <= last; ++i) {
      // the last layer writes this chunk's rows of the whole batch's level-`last` output
      float* o = i == 6 ? cnn6 + c.row6 * kConvDim : i == last ? cnn3 + c.row3 * kConvDim : dst;
      conv(kCnn[i], h_conv[i], src, kConvDim, o, kConvDim, (int)c.rows[i], (int)c.rows[i - 1], kConvS[i], 0,
           kActGelu, nullptr, false, lvl(i), lvl(i - 1), nb);
      std::swap(src, dst);
    }
  }
  if (pl.tail_batch) {
    // layers 4..6 once over the whole batch (the chunk buffers are free now): cnn3 -> cnnA -> cnnB -> cnn6
    static const char* kCnnT[3] = {"h_cnn.c4", "h_cnn.c5", "h_cnn.c6"};
    const int* gs[4] = {gseg3, gseg4, gseg5, seg6};
    const float* in = cnn3;
    float* outs[3] = {cnnA, cnnB, cnn6};
    const size_t rows[4] = {pl.M3, pl.M4, pl.M5, pl.M};
    for (int i = 4; i < 7; ++i) {
      conv(kCnnT[i - 4], h_conv[i], in, kConvDim, outs[i - 4], kConvDim, (int)rows[i - 3], (int)rows[i - 4], kConvS[i],
           0, kActGelu, nullptr, false, gs[i - 3], gs[i - 4], B);
      in = outs[i - 4];
    }
  }
  // LayerNorm + feature projection once over every chunk's rows (row-local: the same results as
  // per chunk, in one launch each instead of one per chunk with a few hundred blocks)
  ln("h_ln", cnn6, nullptr, cnn6, M, kConvDim, h_ln0_g, h_ln0_b, -1);
  conv("h_proj", h_proj, cnn6, kConvDim, x, kHidden, M, M, 1, 0, kActNone, nullptr, true, nullptr, nullptr, 0);
  // ---- encoder: x + GELU(pos_conv(x)) -> LN  (SamePad: pad 64, last output dropped)
  if (precision == 1 && pos_conv) {
    // direct grouped conv over the same packed weights (pos_conv.hip): 48 of 64 columns per group
    // computed, input patch split once per block
    run("h_pos_conv", 2.0 * M * kHidden * (double)h_pos.K, s, [&] {
      launch_hubert_pos_conv(x, kHidden, seg6, B, pl.maxT6, M, h_pos.whi, h_pos.wlo, h_pos.Kp, kPosGout, h_pos.bias,
                             pc, kPosGroups * kPosGout, s);
    });
  } else {
    conv("h_pos_conv", h_pos, x, kHidden, pc, kPosGroups * kPosGout, M, M, 1, kPosK / 2, kActGelu, nullptr, true,
         seg6, nullptr, B, kPosGout, kPosGin);
  }
  ln("h_ln", x, pc, x, M, kHidden, h_enc_g, h_enc_b, 0);
  // LayerNorm fold: the GEMMs it touches run on tile family 7 (x3_variant 7, bf16x3)
  const bool fold = ln_fold && precision == 1 && x3_variant == 7;
  for (int l = 0; l < kLayers; ++l) {
    const HLayer& L = h_layers[l];
    conv("h_qkv", L.qkv, x, kHidden, qkv, 3 * kHidden, M, M, 1, 0, kActNone, nullptr, true, nullptr, nullptr, 0);
    run("h_attn", 4.0 * B * kHeads * (double)pl.maxT6 * pl.maxT6 * (kHidden / kHeads), s,
        [&] { launch_attn(qkv, 3 * kHidden, ao, kHidden, B, pl.maxT6, kHeads, kHidden / kHeads, s, seg6, attn_pipe); });
    if (fold) {
      // LN1 folded: out_proj emits x1's row statistics, fc1 runs on x1 with gamma1 / beta1 in its
      // weights, fc2 normalises its residual x1 on the fly (in place: each element is read by the
      // lane that then overwrites it)
      ConvGemmArgs f{};
      f.ln_parts = kHidden / 128;
      f.ln_eps = 1e-5f;
      f.lnmode = 1;
      f.ln_out = lnst;
      conv("h_out_proj", L.out, ao, kHidden, x1, kHidden, M, M, 1, 0, kActNone, x, true, nullptr, nullptr, 0, 0, 0, &f);
      f.lnmode = 2;
      f.ln_out = nullptr;
      f.ln_in = lnst;
      f.ln_cs = L.fc1_cs;
      conv("h_fc1", L.fc1f, x1, kHidden, ffn, kFfn, M, M, 1, 0, kActGelu, nullptr, true, nullptr, nullptr, 0, 0, 0, &f);
      f.lnmode = 4;
      f.ln_cs = nullptr;
      f.ln_g = L.ln1_g;
      f.ln_b = L.ln1_b;
      conv("h_fc2", L.fc2, ffn, kFfn, x1, kHidden, M, M, 1, 0, kActNone, x1, true, nullptr, nullptr, 0, 0, 0, &f);
    } else {
      conv("h_out_proj", L.out, ao, kHidden, x1, kHidden, M, M, 1, 0, kActNone, x, true, nullptr, nullptr, 0);
      ln("h_ln", x1, nullptr, x, M, kHidden, L.ln1_g, L.ln1_b, -1);
      conv("h_fc1", L.fc1, x, kHidden, ffn, kFfn, M, M, 1, 0, kActGelu, nullptr, true, nullptr, nullptr, 0);
      conv("h_fc2", L.fc2, ffn, kFfn, x1, kHidden, M, M, 1, 0, kActNone, x, true, nullptr, nullptr, 0);
    }
    ln("h_ln", x1, nullptr, x, M, kHidden, L.ln2_g, L.ln2_b, l + 1);
  }
  if (cmn) run("h_cmn", 0, s, [&] { launch_cmn_rows(feats, B, 0, kHidden, s, fseg); });
}

// ------------------------------------------------------------ Model API ---
bool Model::is_frontend() const { return impl->hubert; }

int Model::out_frames(int N) const {
  WSP_CHECK(impl->hubert, "out_frames: not a front-end handle");
  WSP_CHECK(N >= 1, "HuBERT needs at least 1 sample");
  return (N + kDownsample - 1) / kDownsample;
}

size_t Model::frontend_workspace_bytes(int B, int N) const {
  WSP_CHECK(impl->hubert, "frontend_workspace_bytes: not a front-end handle");
  WSP_CHECK(B > 0 && N >= 1, "HuBERT needs B >= 1 and N >= 1 samples");
  const std::vector<int> lens(B, N);
  return frontend_workspace_bytes_segments(B, lens.data());
}

size_t Model::frontend_workspace_bytes_segments(int B, const int* lens) const {
  WSP_CHECK(impl->hubert, "frontend_workspace_bytes: not a front-end handle");
  WSP_CHECK(B > 0 && lens, "HuBERT needs B >= 1 utterances");
  const int ns = impl->nsub(B);
  size_t bytes = 256;
  for (int i = 0; i < ns; ++i) {
    const int b0 = B * i / ns, b1 = B * (i + 1) / ns;
    bytes += (impl->hubert_ws_floats(impl->hubert_plan(b1 - b0, lens + b0), nullptr) * sizeof(float) + 255) &
             ~size_t(255);
  }
  return bytes;
}

void Model::forward_frontend(const float* wav, int B, int N, float* feats, int cmn, void* ws, size_t ws_bytes,
                             hipStream_t s) {
  WSP_CHECK(B > 0 && N >= 1, "HuBERT needs B >= 1 and N >= 1 samples");
  const std::vector<int> lens(B, N);
  forward_frontend_segments(wav, B, lens.data(), feats, nullptr, cmn, ws, ws_bytes, s);
}

void Model::forward_frontend_segments(const float* wav, int B, const int* lens, float* feats, int* frame_offsets,
                                      int cmn, void* ws, size_t ws_bytes, hipStream_t s) {
  Impl& m = *impl;
  WSP_CHECK(m.hubert, "forward_frontend: not a front-end handle");
  WSP_CHECK(m.finalized, "forward before finalize");
  WSP_CHECK(B > 0 && lens, "HuBERT needs B >= 1 utterances");
  WSP_CHECK(ws_bytes >= frontend_workspace_bytes_segments(B, lens), "workspace too small");
  // utterance ranges on concurrent streams (option "streams"); each range's plan is
  // relative to its first sample / output frame
  const int ns = m.nsub(B);
  std::vector<HubertPlan> pls(ns);
  for (int i = 0; i < ns; ++i) {
    const int b0 = B * i / ns, b1 = B * (i + 1) / ns;
    pls[i] = m.hubert_plan(b1 - b0, lens + b0);
  }
  if (frame_offsets) {
    frame_offsets[0] = 0;
    int b = 0;
    for (int i = 0; i < ns; ++i) {
      const HubertPlan& pl = pls[i];
      const int base = frame_offsets[b];
      for (int j = 1; j <= pl.B; ++j) frame_offsets[b + j] = base + pl.offs[pl.B + 1 + j];
      b += pl.B;
    }
  }
  char* wsb = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  if (ns > 1) m.fork(s, ns);
  size_t sample0 = 0, frame0 = 0;
  for (int i = 0; i < ns; ++i) {
    const HubertPlan& pl = pls[i];
    m.forward_hubert(wav + sample0, pl, feats + frame0 * kHidden, cmn, reinterpret_cast<float*>(wsb), m.sub(s, i));
    wsb += (m.hubert_ws_floats(pl, nullptr) * sizeof(float) + 255) & ~size_t(255);
    for (int b = B * i / ns; b < B * (i + 1) / ns; ++b) sample0 += lens[b];
    frame0 += pl.Mout;
  }
  if (ns > 1) m.join(s, ns);
}

}  // namespace wsp
