// Host-sanitizer (ASan + UBSan) random-walk fuzz of the grammar engine.
//
//   grammar_fuzz <ir.json> <vocab.bin> <walks> <budget> <seed>
// vocab.bin: u32 count, then per token u32 length + bytes; eos ids are the zero-length tokens.
// Every walk samples uniformly among the tokens the mask allows, checks mask/can_accept_token/
// accept_token agreement, applies jump-forward prefixes, and must end in an accepting state
// within the character budget.  Exit code != 0 (or a sanitizer report) on any violation.
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../grammar.h"

using namespace vwa;

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s ir.json vocab.bin walks budget seed\n", argv[0]);
    return 2;
  }
  const std::string ir = slurp(argv[1]);
  const std::string vb = slurp(argv[2]);
  const int walks = std::atoi(argv[3]), budget = std::atoi(argv[4]);
  std::mt19937 rng((unsigned)std::atoi(argv[5]));
  size_t off = 0;
  auto rd32 = [&]() {
    uint32_t v;
    std::memcpy(&v, vb.data() + off, 4);
    off += 4;
    return v;
  };
  const uint32_t n = rd32();
  std::vector<std::string> toks(n);
  std::vector<int> eos;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t len = rd32();
    toks[i] = vb.substr(off, len);
    off += len;
    if (len == 0) eos.push_back((int)i);
  }
  auto g = std::make_shared<Grammar>(ir);
  auto v = std::make_shared<Vocab>(toks, eos);
  auto c = std::make_shared<Compiled>(g, v, 512);
  const int words = (int)((n + 31) / 32);
  std::vector<uint32_t> mask(words);
  int accepted = 0;
  for (int wk = 0; wk < walks; ++wk) {
    Matcher m(c, budget);
    std::string out;
    for (int step = 0; step < 4 * budget && !m.is_accept(); ++step) {
      const std::string fp = m.forced_prefix();
      if (!fp.empty()) {
        if (!m.accept_bytes(fp)) return 10;
        out += fp;
        if (m.is_accept()) break;
      }
      m.fill_mask(mask.data());
      std::vector<int> allowed;
      for (uint32_t t = 0; t < n; ++t)
        if ((mask[t >> 5] >> (t & 31)) & 1u) allowed.push_back((int)t);
      if (allowed.empty()) {
        std::fprintf(stderr, "walk %d: empty mask after %zu bytes: %s\n", wk, out.size(), out.c_str());
        return 11;
      }
      // every token the (cached) mask allows must be accepted from this exact state, and a sample
      // of the rejected ones must be rejected (a cache-key collision between two states shows up
      // here as an allowed token the state cannot take)
      for (int t : allowed) {
        if (!m.can_accept_token(t)) {
          std::fprintf(stderr, "walk %d: mask allows token %d the state rejects (after %zu bytes)\n", wk, t,
                       out.size());
          return 12;
        }
      }
      for (int k = 0; k < 64; ++k) {
        const int t = (int)(rng() % n);
        const bool in = (mask[t >> 5] >> (t & 31)) & 1u;
        if (in != m.can_accept_token(t)) {
          std::fprintf(stderr, "walk %d: mask/can_accept disagree on token %d\n", wk, t);
          return 12;
        }
      }
      const int t = allowed[rng() % allowed.size()];
      if (!m.accept_token(t)) return 13;
      out += toks[t];
      if (m.used() > budget) return 14;
    }
    if (!m.is_accept()) {
      std::fprintf(stderr, "walk %d: not accepted: %s\n", wk, out.c_str());
      return 15;
    }
    ++accepted;
  }
  std::printf("FUZZ_OK walks=%d accepted=%d cache_hits=%zu misses=%zu\n", walks, accepted, c->hits, c->misses);
  return 0;
}
