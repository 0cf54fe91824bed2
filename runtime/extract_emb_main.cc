// Embedding extraction CLI on the HIP backend — same flags and output format as
// the reference's runtime/core/bin/extract_emb_main.cc (one line per utterance:
// "<key> <e0> <e1> ..."), with HipSpeakerEngine in place of the ONNX / MNN engine.
//   extract_emb_main --speaker_model_path model.safetensors (--wav_path x.wav | --wav_scp wav.scp)
//                    [--result out.txt] [--fbank_dim 80] [--sample_rate 16000]
//                    [--embedding_size 256] [--samples_per_chunk 32000]
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "flags.h"
#include "speaker_model_hip.h"

int main(int argc, char** argv) {
  Flags f(argc, argv);
  if (f.has("help") || argc == 1) {
    std::printf("usage: %s --speaker_model_path M (--wav_path W | --wav_scp S) [--result R]\n"
                "       [--fbank_dim 80] [--sample_rate 16000] [--embedding_size N] [--samples_per_chunk 32000]\n",
                argv[0]);
    return argc == 1 ? 1 : 0;
  }
  const std::string model = f.str("speaker_model_path", "");
  const std::string wav_path = f.str("wav_path", ""), wav_scp = f.str("wav_scp", "");
  if (model.empty() || (wav_path.empty() && wav_scp.empty())) {
    std::fprintf(stderr, "speaker_model_path and one of wav_path / wav_scp are required\n");
    return 1;
  }
  std::vector<std::pair<std::string, std::string>> waves;
  if (!wav_path.empty()) {
    waves.emplace_back("test", wav_path);
  } else {
    std::ifstream scp(wav_scp);
    std::string line;
    while (std::getline(scp, line)) {
      std::istringstream ss(line);
      std::string k, p;
      if (ss >> k >> p) waves.emplace_back(k, p);
    }
    if (waves.empty()) {
      std::fprintf(stderr, "empty wav scp\n");
      return 1;
    }
  }
  try {
    wespeaker::HipSpeakerEngine engine(model, f.integer("fbank_dim", 80), f.integer("sample_rate", 16000),
                                       f.integer("embedding_size", 0), f.integer("samples_per_chunk", 32000));
    std::ofstream res;
    const std::string result = f.str("result", "");
    if (!result.empty()) res.open(result);
    std::ostream& out = result.empty() ? std::cout : res;
    double total_audio = 0, total_time = 0;
    for (const auto& w : waves) {
      int sr = 0;
      std::vector<int16_t> pcm = wespeaker::ReadWavPcm16(w.second, &sr);
      // extract_emb_main.cc:52 CHECK_EQs 16000; here the engine's --sample_rate (default 16000)
      if (sr != f.integer("sample_rate", 16000))
        throw std::runtime_error(w.second + ": sample rate differs from --sample_rate");
      std::vector<float> emb;
      const auto t0 = std::chrono::steady_clock::now();
      engine.ExtractEmbedding(pcm.data(), (int)pcm.size(), &emb);
      total_time += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      total_audio += (double)pcm.size() / sr;
      out << w.first;
      char buf[32];
      for (float v : emb) {
        std::snprintf(buf, sizeof(buf), " %.9g", v);
        out << buf;
      }
      out << "\n";
    }
    std::fprintf(stderr, "extracted %zu embeddings, RTF %.5f\n", waves.size(),
                 total_audio > 0 ? total_time / total_audio : 0.0);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 2;
  }
  return 0;
}
