// Verification CLI on the HIP backend — flags of the reference's
// runtime/core/bin/asv_main.cc: cosine score of --enroll_wav vs --test_wav,
// mapped to [0, 1], compared with --threshold.
#include <cstdio>
#include <string>
#include <vector>

#include "flags.h"
#include "speaker_model_hip.h"

int main(int argc, char** argv) {
  Flags f(argc, argv);
  const std::string model = f.str("speaker_model_path", "");
  const std::string enroll = f.str("enroll_wav", ""), test = f.str("test_wav", "");
  if (f.has("help") || model.empty() || enroll.empty() || test.empty()) {
    std::printf("usage: %s --speaker_model_path M --enroll_wav A --test_wav B [--threshold 0.5]\n"
                "       [--fbank_dim 80] [--sample_rate 16000] [--embedding_size N] [--SamplesPerChunk 32000]\n",
                argv[0]);
    return f.has("help") ? 0 : 1;
  }
  try {
    wespeaker::HipSpeakerEngine engine(model, f.integer("fbank_dim", 80), f.integer("sample_rate", 16000),
                                       f.integer("embedding_size", 0), f.integer("SamplesPerChunk", 32000));
    std::vector<float> e1, e2;
    int sr = 0;
    std::vector<int16_t> a = wespeaker::ReadWavPcm16(enroll, &sr);
    engine.ExtractEmbedding(a.data(), (int)a.size(), &e1);
    std::vector<int16_t> b = wespeaker::ReadWavPcm16(test, &sr);
    engine.ExtractEmbedding(b.data(), (int)b.size(), &e2);
    const float score = engine.CosineSimilarity(e1, e2);
    std::printf("Cosine score: %.6f\n", score);
    std::printf(score >= f.real("threshold", 0.5) ? "It's the same speaker!\n" : "Warning! It's a different speaker.\n");
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 2;
  }
  return 0;
}
