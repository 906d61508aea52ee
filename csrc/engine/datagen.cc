// Native generators of sorted map-output runs for the BASELINE configs (host side): fast enough
// to produce GBs for the CPU/bridge configs and the GPU generic-merge benchmark.
//   terasort  : Text(10 random bytes) -> Text(90 printable bytes)
//   wordcount : Text(word) -> IntWritable(1), Zipf vocabulary, hash-partitioned
//   secondary : Text(<skewed long common prefix><8 digits>) -> Text(0..120 random bytes)
#include "uda/datagen.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <cmath>
#include <cstring>
#include <random>
#include <thread>

#include "uda/compare.h"
#include "uda/ifile.h"

namespace uda {

namespace {
struct Rec {
  std::string key, val;
};

std::string text_bytes(const std::string& s) {
  uint8_t h[9];
  int n = vint_encode((int64_t)s.size(), h);
  return std::string((const char*)h, n) + s;
}

uint32_t hash_part(const std::string& k, int reducers) {
  uint32_t h = 0;
  for (unsigned char c : k) h = (h * 31 + c) & 0x7FFFFFFF;
  return h % (uint32_t)reducers;
}
}  // namespace

std::vector<std::vector<std::vector<uint8_t>>> generate_runs(const std::string& kind, int maps, int reducers,
                                                             int64_t rows_per_map, uint64_t seed) {
  std::vector<std::vector<std::vector<uint8_t>>> out((size_t)maps);
  const KeyKind kk = kind == "wordcount_int" ? KeyKind::kRaw : KeyKind::kText;
  std::vector<std::string> vocab;
  std::vector<double> cdf;
  if (kind == "wordcount") {
    const int V = 100000;
    double acc = 0;
    for (int i = 0; i < V; ++i) {
      char b[32];
      snprintf(b, sizeof(b), "w%07d", (i * 7919) % 10000000);
      vocab.emplace_back(b);
      acc += 1.0 / (i + 1);
      cdf.push_back(acc);
    }
    for (auto& c : cdf) c /= acc;
  }
  std::vector<std::string> prefixes;
  if (kind == "secondary") {
    std::mt19937_64 prng(seed ^ 0xABCDEF);
    for (int i = 0; i < 64; ++i) {
      char b[64];
      snprintf(b, sizeof(b), "user/%04d/session/", i);
      prefixes.push_back(std::string(b) + std::string(prng() % 41, 'x'));
    }
  }
  auto one_map = [&](int m) {
    std::mt19937_64 rng(seed * 1000003 + (uint64_t)m);
    std::vector<std::vector<Rec>> parts((size_t)reducers);
    for (int64_t i = 0; i < rows_per_map; ++i) {
      Rec r;
      int p = 0;
      if (kind == "terasort") {
        std::string k(10, '\0'), v(90, '\0');
        for (auto& c : k) c = (char)(rng() & 0xFF);
        for (auto& c : v) c = (char)('A' + rng() % 26);
        p = (int)((uint8_t)k[0] * (uint64_t)reducers / 256);
        r.key = text_bytes(k);
        r.val = text_bytes(v);
      } else if (kind == "wordcount") {
        const double u = std::uniform_real_distribution<double>(0, 1)(rng);
        const size_t w = std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin();
        const std::string& word = vocab[std::min(w, vocab.size() - 1)];
        p = (int)hash_part(word, reducers);
        r.key = text_bytes(word);
        r.val = std::string("\0\0\0\1", 4);
      } else if (kind == "secondary") {
        // Pareto-skewed prefix choice, and 60 % of the rows land on reducer 0 (partition skew)
        const double u = std::uniform_real_distribution<double>(1e-9, 1)(rng);
        int idx = (int)(std::pow(u, -1.0 / 1.2)) - 1;
        idx = std::min(std::max(idx, 0), 63);
        char d[16];
        snprintf(d, sizeof(d), "%08u", (unsigned)(rng() % 100000000));
        std::string k = prefixes[(size_t)idx] + d;
        std::string v((size_t)(rng() % 121), '\0');
        for (auto& c : v) c = (char)(rng() & 0xFF);
        p = (rng() % 10 < 6) ? 0 : (int)hash_part(k, reducers);
        r.key = text_bytes(k);
        r.val = text_bytes(v);
      } else {
        throw std::runtime_error("unknown generator kind " + kind);
      }
      parts[(size_t)p].push_back(std::move(r));
    }
    out[(size_t)m].resize((size_t)reducers);
    for (int p = 0; p < reducers; ++p) {
      auto& v = parts[(size_t)p];
      std::stable_sort(v.begin(), v.end(), [kk](const Rec& a, const Rec& b) {
        return key_compare(kk, (const uint8_t*)a.key.data(), (int)a.key.size(), (const uint8_t*)b.key.data(),
                           (int)b.key.size()) < 0;
      });
      std::vector<uint8_t> s;
      size_t total = 2;
      for (auto& r : v) total += (size_t)ifile_record_size((int64_t)r.key.size(), (int64_t)r.val.size());
      s.reserve(total);
      for (auto& r : v)
        ifile_append(&s, (const uint8_t*)r.key.data(), (int32_t)r.key.size(), (const uint8_t*)r.val.data(),
                     (int32_t)r.val.size());
      ifile_append_eof(&s);
      out[(size_t)m][(size_t)p] = std::move(s);
    }
  };
  const int nthreads = std::max(1, std::min<int>(maps, (int)std::thread::hardware_concurrency()));
  std::vector<std::thread> ts;
  std::atomic<int> next{0};
  std::exception_ptr err;
  std::mutex err_mu;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&] {
      for (int m; (m = next++) < maps;) {
        try {
          one_map(m);
        } catch (...) {
          std::lock_guard<std::mutex> g(err_mu);
          err = std::current_exception();
        }
      }
    });
  for (auto& t : ts) t.join();
  if (err) std::rethrow_exception(err);
  return out;
}

}  // namespace uda
