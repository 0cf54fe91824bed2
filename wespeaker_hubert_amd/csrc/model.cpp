// Speaker-model runtime: parameter intake (reference state_dict order),
// BatchNorm folding + weight packing on the host in f64, device residency,
// and the forward schedule of HIP kernels over a caller-provided workspace.
//
// ECAPA-TDNN forward = wespeaker/models/ecapa_tdnn.py:208-234, channels-last:
//   layer1  Conv1dReluBn(F->C, k5)                        -> x1   [M][C]
//   layerL  SE_Res2Block(dil L):  c1 (1x1) -> h1
//           Res2 chain i=0..6: conv_k3(h1_i (+ h2_{i-1})) -> h2_i  (7 GEMMs)
//           c3 (1x1) over cat(h2_0..6, h1_7)             -> h3   (no copy)
//           SE: frame mean -> FC relu -> FC sigmoid -> x_{L} + h3 * g
//   conv    1x1 over cat(x2, x3, x4) (no copy), ReLU      -> xp   [M][1536]
//   ASTP    [GLOB: frame mean/std -> per-utterance bias]  -> tanh(W1 xp) -> W2
//           -> online-softmax attentive mean/std          -> [B][3072]
//   head    BN(3072) + Linear (+ bn2) folded into one GEMV -> embed [B][D]
#include "model_impl.h"

namespace wsp {

Model::Model() : impl(new Impl) {}
Model::~Model() {
  for (auto& kv : impl->prof_map)
    for (auto& e : kv.second.ev) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
  for (auto t : impl->sub_st) (void)hipStreamDestroy(t);
  for (auto e : impl->sub_ev) (void)hipEventDestroy(e);
  delete impl;
}

void Model::create(const std::string& arch, int feat_dim, int embed_dim, bool emb_bn, bool two_emb) {
  Impl& m = *impl;
  m.arch = arch;
  m.feat_dim = feat_dim;
  m.embed_dim = embed_dim;
  m.emb_bn = emb_bn;
  m.two_emb = two_emb;
  // Creation and parameter intake are host-only; the device is bound at
  // finalize (create's device when one was current).
  if (hipGetDevice(&m.device) != hipSuccess) {
    (void)hipGetLastError();
    m.device = -1;
  }
  if (arch == "ECAPA_TDNN_c512" || arch == "ECAPA_TDNN_GLOB_c512" || arch == "ECAPA_TDNN_c1024" ||
      arch == "ECAPA_TDNN_GLOB_c1024") {
    m.ecapa = true;
    m.x3_variant = 7;  // 6 (the 256 x 256 tile on 16x16x32 MFMAs, r3) with LDS-DMA staging (r4)
    m.C = (arch.find("c1024") != std::string::npos) ? 1024 : 512;
    m.glob = arch.find("GLOB") != std::string::npos;
    WSP_CHECK(feat_dim > 0 && feat_dim % 4 == 0, "ECAPA feat_dim must be a positive multiple of 4");
    WSP_CHECK(embed_dim > 0, "embed_dim must be positive");
    m.build_ecapa_params();
  } else if (arch.rfind("ResNet", 0) == 0) {
    static const std::map<std::string, std::pair<bool, std::vector<int>>> kRes = {
        {"ResNet18", {false, {2, 2, 2, 2}}},     {"ResNet34", {false, {3, 4, 6, 3}}},
        {"ResNet50", {true, {3, 4, 6, 3}}},      {"ResNet101", {true, {3, 4, 23, 3}}},
        {"ResNet152", {true, {3, 8, 36, 3}}},    {"ResNet221", {true, {6, 16, 48, 3}}},
        {"ResNet293", {true, {10, 20, 64, 3}}}};
    auto it = kRes.find(arch);
    WSP_CHECK(it != kRes.end(), "unsupported arch " + arch);
    // resnet.py:124 sizes the pooling for int(feat_dim / 8) frequency rows while stage 4 keeps
    // ceil(feat_dim / 8): the reference model only runs for multiples of 8
    WSP_CHECK(feat_dim >= 8 && feat_dim % 8 == 0, "ResNet feat_dim must be a positive multiple of 8");
    m.ecapa = false;
    // basic blocks: 256 x 128 swizzled (with the residual prefetch, ROLE 2: +1.3 % C3 over variant 3,
    // r2c); bottleneck ResNets: family 7 wherever it takes the operands (1x1 convs with N % 256 == 0),
    // family 6 elsewhere — ResNet293 C3 +0.2-0.4 % over 4 in three interleaved pairs (r6u)
    m.x3_variant = it->second.first ? 7 : 4;
    m.streams = 2;     // two utterance ranges in flight: ResNet293 C3 +8.6 %
    m.bottleneck = it->second.first;
    for (int i = 0; i < 4; ++i) m.nblocks[i] = it->second.second[i];
    m.build_resnet_params();
  } else if (arch == "SimAM_ResNet34_ASP" || arch == "SimAM_ResNet100_ASP") {
    // samresnet.py:124-166: in_planes 64 (option "in_planes" before the weights),
    // acoustic_dim = feat_dim, basic SimAM blocks [3,4,6,3] / [6,16,24,3]
    WSP_CHECK(!two_emb && !emb_bn, "SimAM-ResNet has no emb_bn / two_emb_layer");
    WSP_CHECK(feat_dim >= 8 && feat_dim % 8 == 0, "SimAM-ResNet acoustic_dim must be a multiple of 8");
    WSP_CHECK(embed_dim > 0, "embed_dim must be positive");
    m.ecapa = false;
    m.simam = true;
    m.bottleneck = false;
    m.x3_variant = 5;  // MFMA-bound 3x3 convs (K = 9C): wide tiles where N % 256 == 0 (+6 % over variant 3)
    m.streams = 2;     // SimAM-ResNet100 +3.8 %
    m.m_ch = 64;
    const int nb34[4] = {3, 4, 6, 3}, nb100[4] = {6, 16, 24, 3};
    for (int i = 0; i < 4; ++i) m.nblocks[i] = arch == "SimAM_ResNet34_ASP" ? nb34[i] : nb100[i];
    m.build_simam_params();
  } else if (arch == "HuBERT_base") {
    // s3prl HuBERT-base upstream + Featurizer (frontend/s3prl.py); input is
    // the waveform, output 768-dim frames (S3prlFrontend.output_size()).
    WSP_CHECK(embed_dim == 768, "HuBERT_base output size is 768");
    m.ecapa = false;
    m.hubert = true;
    m.feat_dim = 1;
    m.x3_variant = 7;  // every GEMM whose operands family 7 takes (r4), the rest on 6
    m.streams = 2;  // HuBERT + ECAPA C4 chain +2.6 %
    m.build_hubert_params();
  } else {
    throw InvalidArg{"unsupported arch " + arch};
  }
}

int Model::num_params() const { return (int)impl->params.size(); }

void Model::param_info(int i, const char** name, int* ndim, int64_t* shape) const {
  WSP_CHECK(i >= 0 && i < num_params(), "param index out of range");
  const Param& p = impl->params[i];
  *name = p.name.c_str();
  *ndim = (int)p.shape.size();
  for (size_t d = 0; d < p.shape.size() && d < 4; ++d) shape[d] = p.shape[d];
}

void Model::set_param(int i, const float* data, int64_t numel) {
  WSP_CHECK(i >= 0 && i < num_params(), "param index out of range");
  Param& p = impl->params[i];
  WSP_CHECK(numel == p.numel(), "numel mismatch for " + p.name);
  p.host.assign(data, data + numel);
  p.set = true;
}

void Model::finalize() {
  Impl& m = *impl;
  WSP_CHECK(!m.finalized, "model already finalized");
  int dev = 0;
  WSP_HIP(hipGetDevice(&dev));
  WSP_CHECK(m.device < 0 || dev == m.device, "finalize on a different device than create");
  m.device = dev;
  for (auto& p : m.params)
    WSP_CHECK(p.set || p.name.find("num_batches_tracked") != std::string::npos,
              "parameter not set: " + p.name);
  if (m.ecapa)
    m.finalize_ecapa();
  else if (m.simam)
    m.finalize_simam();
  else if (m.hubert)
    m.finalize_hubert();
  else
    m.finalize_resnet();
  for (auto& p : m.params) std::vector<float>().swap(p.host);
  m.finalized = true;
}

int Model::embed_dim() const { return impl->embed_dim; }
int Model::feat_dim() const { return impl->feat_dim; }

// workspace of one sub-batch of B utterances, 256-byte granules
size_t Model::Impl::ws_bytes_one(int B, int T) const {
  const int bc = ecapa ? ecapa_chunk(B, T) : B;
  const size_t f = ecapa   ? ecapa_ws_floats(bc, (size_t)bc * T, nullptr)
                   : simam ? simam_ws_floats(B, T, nullptr)
                           : resnet_ws_floats(B, T, nullptr);
  return (f * sizeof(float) + 255) & ~size_t(255);
}

size_t Model::workspace_bytes(int B, int T) const {
  WSP_CHECK(!impl->hubert, "HuBERT handle: use the front-end workspace query");
  const int ns = impl->nsub(B);
  size_t bytes = 256;
  for (int i = 0; i < ns; ++i) bytes += impl->ws_bytes_one(B * (i + 1) / ns - B * i / ns, T);
  return bytes;
}

void Model::forward(const float* feats, int B, int T, float* embed, void* ws, size_t ws_bytes,
                    hipStream_t s) {
  Impl& m = *impl;
  WSP_CHECK(!m.hubert, "HuBERT handle: use the front-end forward");
  WSP_CHECK(m.finalized, "forward before finalize");
  WSP_CHECK(B > 0 && T > 1, "forward needs B >= 1 and T >= 2 frames");
  WSP_CHECK((size_t)B * T < (1u << 31), "B*T too large");
  WSP_CHECK(ws_bytes >= workspace_bytes(B, T), "workspace too small");
  WSP_CHECK(m.ecapa || m.precision == 1, "ResNet runs on the bf16x3 kernels only (precision=1)");
  WSP_CHECK(!m.simam || (T + 7) / 8 >= 2, "SimAM-ResNet needs >= 2 frames after the three stride-2 stages");
  char* wsb = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  const int ns = m.nsub(B);
  if (ns > 1) m.fork(s, ns);
  for (int i = 0; i < ns; ++i) {
    const int b0 = B * i / ns, nb = B * (i + 1) / ns - b0;
    const float* f = feats + (size_t)b0 * T * m.feat_dim;
    float* e = embed + (size_t)b0 * m.embed_dim;
    float* wsf = reinterpret_cast<float*>(wsb);
    const hipStream_t si = m.sub(s, i);
    if (m.ecapa) {
      // consecutive utterance chunks whose operands stay < 2 GiB, over one chunk-sized workspace
      const int bc = m.ecapa_chunk(nb, T);
      for (int c0 = 0; c0 < nb; c0 += bc)
        m.forward_ecapa(f + (size_t)c0 * T * m.feat_dim, std::min(bc, nb - c0), T, e + (size_t)c0 * m.embed_dim, wsf,
                        si);
    } else if (m.simam)
      m.forward_simam(f, nb, T, e, wsf, si);
    else
      m.forward_resnet(f, nb, T, e, wsf, si);
    wsb += m.ws_bytes_one(nb, T);
  }
  if (ns > 1) m.join(s, ns);
}

size_t Model::workspace_bytes_segments(int B, int M) const {
  WSP_CHECK(impl->ecapa, "segmented batches are implemented for ECAPA-TDNN handles");
  WSP_CHECK(B > 0 && M >= B, "segmented batch needs B >= 1 and M >= B rows");
  return impl->ecapa_ws_floats(B, (size_t)M, nullptr) * sizeof(float) + 256;
}

void Model::forward_segments(const float* feats, int B, const int* seg, int M, float* embed, void* ws,
                             size_t ws_bytes, hipStream_t s) {
  Impl& m = *impl;
  WSP_CHECK(m.ecapa, "segmented batches are implemented for ECAPA-TDNN handles");
  WSP_CHECK(m.finalized, "forward before finalize");
  WSP_CHECK(seg != nullptr && B > 0 && M >= B, "segmented batch needs offsets, B >= 1 and M >= B rows");
  WSP_CHECK((size_t)M * 1536 < (1u << 31) / 4, "segmented batch too large");
  WSP_CHECK(ws_bytes >= workspace_bytes_segments(B, M), "workspace too small");
  float* wsf = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  m.forward_ecapa(feats, B, 1, embed, wsf, s, seg, M);  // T unused when segmented
}

void Model::profile(bool on) {
  if (on && !impl->prof)  // a new profiling window: drop the previous one's launches
    for (auto& kv : impl->prof_map) {
      kv.second.used = 0;
      kv.second.flops = 0;
    }
  impl->prof = on;
}

void Model::set_option(const std::string& key, int value) {
  if (key == "precision") {
    WSP_CHECK(value == 0 || value == 1, "precision must be 0 (f32) or 1 (bf16x3)");
    impl->precision = value;
  } else if (key == "layer") {
    WSP_CHECK(impl->hubert, "option 'layer' applies to the HuBERT front end");
    WSP_CHECK(!impl->finalized, "option 'layer' must be set before finalize");
    WSP_CHECK(value >= -1 && value <= 12, "layer must be -1 (weighted sum) or 0..12");
    impl->h_layer_sel = value;
  } else if (key == "in_planes") {
    WSP_CHECK(impl->simam, "option 'in_planes' applies to SimAM-ResNet handles");
    WSP_CHECK(!impl->finalized, "option 'in_planes' must be set before finalize");
    WSP_CHECK(value == 32 || value == 64, "in_planes must be 32 or 64");
    for (const auto& p : impl->params) WSP_CHECK(!p.set, "option 'in_planes' must be set before the weights");
    impl->m_ch = value;
    impl->build_simam_params();
  } else if (key == "res_prefetch") {
    WSP_CHECK(value == 0 || value == 1, "res_prefetch must be 0 or 1");
    impl->res_prefetch = value;
  } else if (key == "c1_stage_fuse") {
    WSP_CHECK(value == 0 || value == 1, "c1_stage_fuse must be 0 or 1");
    impl->c1_stage_fuse = value;
  } else if (key == "sc_fuse") {
    WSP_CHECK(value >= 0 && value <= 3, "sc_fuse must be 0 .. 3 (bit 0: one GEMM, bit 1: in the tail)");
    impl->sc_fuse = value;
  } else if (key == "res_tail") {
    WSP_CHECK(value >= 0 && value <= 2, "res_tail must be 0 (off), 1 (tail + next conv1) or 2 (tail alone)");
    impl->res_tail = value;
  } else if (key == "cat_gate") {
    WSP_CHECK(value == 0 || value == 1, "cat_gate must be 0 or 1");
    impl->cat_gate = value;
  } else if (key == "res2_fused") {
    WSP_CHECK(value == 0 || value == 1, "res2_fused must be 0 or 1");
    impl->res2_fused = value;
  } else if (key == "attn_pipe") {
    WSP_CHECK(value == 0 || value == 1, "attn_pipe must be 0 or 1");
    impl->attn_pipe = value;
  } else if (key == "pos_conv") {
    WSP_CHECK(value == 0 || value == 1, "pos_conv must be 0 (grouped implicit GEMM) or 1 (direct grouped conv)");
    impl->pos_conv = value;
  } else if (key == "ln_fold") {
    WSP_CHECK(value == 0 || value == 1, "ln_fold must be 0 (LayerNorm kernels) or 1 (folded into the GEMMs)");
    impl->ln_fold = value;
  } else if (key == "tail_batch") {
    WSP_CHECK(value == 0 || value == 1, "tail_batch must be 0 (CNN layers 4-6 per chunk) or 1 (batch-wide)");
    impl->tail_batch = value;
  } else if (key == "astp_fused") {
    WSP_CHECK(value >= 0 && value <= 3, "astp_fused must be 0 (linear2 GEMM + pooling kernel) or 1 (fused)");
    impl->astp_fused_on = value ? 1 : 0;  // 2 / 3: former fused variants (r3 pruned), deprecated aliases of 1
  } else if (key == "conv3x3_img") {
    WSP_CHECK(value >= 0 && value <= 3, "conv3x3_img must be 0 (off), 1 (32 / 64 channels) or 2 / 3 (also 128)");
    impl->conv3x3_img_on = value;
  } else if (key == "streams") {
    WSP_CHECK(value >= 1 && value <= 8, "streams must be 1..8");
    impl->streams = value;
  } else if (key == "res2_variant") {
    WSP_CHECK(value == 0 || value == 2 || value == 3 || value == 4,
              "res2_variant must be 0 (4 waves, 2 x 2), 2 (4 waves on N, 4 W k-steps in flight), 3 (8 waves) "
              "or 4 (halo-free strips, c1024 widths; else as 3)");
    impl->res2_variant = value;
  } else if (key == "x3_variant") {
    WSP_CHECK((value >= 0 && value <= 9),
              "x3_variant must be 3, 4, 5, 6 (5 on 16x16x32 MFMAs) or 7 (6 staged by LDS-DMA)");
    // 0 / 1 (unswizzled tiles), 2 / 9 (the r2 LDS-DMA tiles): pruned in r3; 8 (the r5 ping-pong form
    // of 7, bit-identical and slower): pruned in r5 — deprecated aliases of 5 / 7
    impl->x3_variant = value >= 3 && value <= 7 ? value : value == 8 ? 7 : 5;
  } else if (key == "attn_lds" || key == "conv1x1_rows") {
    // pruned in r3 (hubert.hip's streaming mha_kernel, conv1x1_rows.hip): accepted, no effect
  } else {
    throw InvalidArg{"unknown option " + key};
  }
}

int Model::get_option(const std::string& key) const {
  const Impl& m = *impl;
  if (key == "precision") return m.precision;
  if (key == "streams") return m.streams;
  if (key == "layer") return m.h_layer_sel;
  if (key == "in_planes") return m.m_ch;
  if (key == "res2_fused") return m.res2_fused;
  if (key == "cat_gate") return m.cat_gate;
  if (key == "res_prefetch") return m.res_prefetch;
  if (key == "res_tail") return m.res_tail;
  if (key == "sc_fuse") return m.sc_fuse;
  if (key == "c1_stage_fuse") return m.c1_stage_fuse;
  if (key == "astp_fused") return m.astp_fused_on;
  if (key == "attn_pipe") return m.attn_pipe;
  if (key == "pos_conv") return m.pos_conv;
  if (key == "ln_fold") return m.ln_fold;
  if (key == "tail_batch") return m.tail_batch;
  if (key == "res2_variant") return m.res2_variant;
  if (key == "x3_variant") return m.x3_variant;
  if (key == "conv3x3_img") return m.conv3x3_img_on;
  throw InvalidArg{"unknown option " + key};
}

void Model::profile_query(const std::string& tag, int* launches, double* total_ms, double* flops) {
  // `tag` names one kernel class or, as a prefix "tag.", every sub-class under it
  // (e.g. "res_conv1x1" = "res_conv1x1.c1.L1" + ...).  Launches of the current /
  // last profiling window.
  *launches = 0;
  *total_ms = 0;
  *flops = 0;
  double fl = 0;
  for (auto& kv : impl->prof_map) {
    const std::string& k = kv.first;
    if (k != tag && k.compare(0, tag.size() + 1, tag + ".") != 0) continue;
    ProfEntry& e = kv.second;
    for (size_t i = 0; i < e.used; ++i) {
      WSP_HIP(hipEventSynchronize(e.ev[i].second));
      float ms = 0;
      WSP_HIP(hipEventElapsedTime(&ms, e.ev[i].first, e.ev[i].second));
      *total_ms += ms;
    }
    *launches += (int)e.used;
    fl += e.flops;
  }
  *flops = *launches ? fl / (double)*launches : 0.0;
}

}  // namespace wsp
