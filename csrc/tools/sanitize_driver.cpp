// Host-side sanitizer harness: the C++ runtime pieces that parse and
// transform untrusted input - the GGUF parser, the planar repack and the CPU
// engine's forward / sampling loop - built with -fsanitize=address,undefined
// (tests/test_sanitizers.py builds and runs it; GPU sanitizers are not available
// on the target pool, so device code is covered by the numerics tests instead).
//
//   sanitize_driver parse <file.gguf>     parse only; exit 0 ok, 2 rejected cleanly
//   sanitize_driver run <file.gguf> <n>   parse + load + prefill + n sampled tokens
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <string>
#include <vector>

#include "cpu/cpu_backend.h"
#include "runtime/gguf.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s parse|run <file.gguf> [n_tokens]\n", argv[0]);
    return 64;
  }
  const std::string mode = argv[1], path = argv[2];
  try {
    if (mode == "parse") {
      lfk::GGUFFile f(path);
      size_t bytes = 0;
      for (const auto& t : f.tensors()) bytes += (size_t)t.n_elements();
      std::printf("ok tensors=%zu kv=%zu elements=%zu\n", f.tensors().size(), f.metadata().size(), bytes);
      return 0;
    }
    if (mode == "run") {
      const int n = argc > 3 ? std::atoi(argv[3]) : 8;
      lfk::CpuOptions o;
      o.n_ctx = 128;
      o.n_threads = 2;
      o.n_batch = 16;
      lfk::CpuEngine eng(path, o);
      std::vector<int> prompt;
      for (int i = 0; i < 20; ++i) prompt.push_back((i * 37 + 5) % eng.n_vocab());
      const std::vector<float> lg = eng.eval_logits(prompt, 0);
      for (float v : lg)
        if (!std::isfinite(v)) {
          std::fprintf(stderr, "non-finite logit\n");
          return 3;
        }
      lfk::CpuSampling sp;
      sp.seed = 7;
      sp.temp = 1.2f;
      sp.top_p = 0.9f;
      sp.freq_penalty = 0.7f;
      sp.presence_penalty = 0.8f;
      const lfk::CpuGenOut g = eng.generate(prompt, 0, n, sp, {}, [] { return false; }, [](int) {});
      std::printf("ok logits=%zu generated=%zu finish=%s\n", lg.size(), g.tokens.size(), g.finish.c_str());
      return 0;
    }
  } catch (const std::exception& e) {
    std::printf("rejected: %s\n", e.what());
    return 2;
  }
  std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
  return 64;
}
