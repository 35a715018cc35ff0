#include "name_loader.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#include <fstream>
#include <stdexcept>

namespace gk {

namespace {
// the syllable tables of utils/data.py
const char* const kOnsets[] = {"",  "b",  "br", "c",  "ch", "d",  "dr", "f", "g", "gr", "h", "j", "k", "kr", "l",
                               "m", "n",  "p",  "r",  "s",  "sh", "st", "t", "th", "tr", "v", "w", "y", "z"};
const char* const kVowels[] = {"a", "e", "i", "o", "u", "ae", "ai", "ia", "io", "ou", "y", "ee"};
const char* const kCodas[] = {"", "", "", "n", "r", "l", "s", "th", "m", "nd", "x", "k"};
constexpr uint32_t kNO = sizeof(kOnsets) / sizeof(kOnsets[0]);
constexpr uint32_t kNV = sizeof(kVowels) / sizeof(kVowels[0]);
constexpr uint32_t kNC = sizeof(kCodas) / sizeof(kCodas[0]);

uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
}  // namespace

NameLoader::Rng::Rng(uint64_t seed) {
  uint64_t x = seed;
  for (auto& v : s) v = splitmix64(x);
}
uint64_t NameLoader::Rng::next() {
  const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
  s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
  s[2] ^= t; s[3] = rotl(s[3], 45);
  return r;
}

NameLoader::NameLoader(const LoaderCfg& c) : c_(c), rng_(c.seed * 0x9E3779B97F4A7C15ull + 0x1234567ull) {
  if (c_.B <= 0 || c_.T <= 0 || c_.prefetch <= 0) throw std::runtime_error("NameLoader: bad batch shape");
  if (!c_.path.empty()) {
    std::ifstream f(c_.path, std::ios::binary);
    if (!f) throw std::runtime_error("NameLoader: cannot open " + c_.path);
    std::string line;
    while (std::getline(f, line)) {
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (line.empty()) continue;
      if ((int)line.size() > c_.max_len - 1 && c_.max_len > 1) line.resize(c_.max_len - 1);
      file_names_.push_back(line);
    }
    if (file_names_.empty()) throw std::runtime_error("NameLoader: no names in " + c_.path);
    order_.resize(file_names_.size());
  }
  worker_ = std::thread([this] { run(); });
}

NameLoader::~NameLoader() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_space_.notify_all();
  if (worker_.joinable()) worker_.join();
}

void NameLoader::append_synth() {
  // SOS, 1-3 (onset vowel coda) syllables truncated to max_len-1 chars, first one upper-case, EOS
  const size_t cap = (size_t)std::max(1, c_.max_len - 1);
  stream_.push_back(c_.sos);
  const size_t start = stream_.size();
  const int syl = 1 + (int)rng_.below(3);
  for (int i = 0; i < syl; ++i) {
    const char* parts[3] = {kOnsets[rng_.below(kNO)], kVowels[rng_.below(kNV)], kCodas[rng_.below(kNC)]};
    for (const char* p : parts)
      for (; *p; ++p)
        if (stream_.size() - start < cap) stream_.push_back((int32_t)(unsigned char)*p);
  }
  if (stream_.size() > start) stream_[start] = std::toupper(stream_[start]);
  stream_.push_back(c_.eos);
}

void NameLoader::append_name(const std::string& nm) {
  stream_.push_back(c_.sos);
  for (unsigned char ch : nm) stream_.push_back((int32_t)ch);
  stream_.push_back(c_.eos);
}

void NameLoader::refill(size_t need) {
  // drop the consumed prefix, then append names until `need` ids are buffered
  if (stream_pos_) {
    stream_.erase(stream_.begin(), stream_.begin() + (long)stream_pos_);
    stream_pos_ = 0;
  }
  while (stream_.size() < need) {
    if (file_names_.empty()) {
      append_synth();
      continue;
    }
    if (cursor_ == 0) {   // new epoch: seeded Fisher-Yates reshuffle
      for (uint32_t i = 0; i < order_.size(); ++i) order_[i] = i;
      for (size_t i = order_.size(); i > 1; --i) std::swap(order_[i - 1], order_[rng_.below((uint32_t)i)]);
    }
    append_name(file_names_[order_[cursor_]]);
    if (++cursor_ == order_.size()) { cursor_ = 0; ++epoch_; }
  }
}

void NameLoader::make_batch(std::vector<int32_t>& xy) {
  const int B = c_.B, T = c_.T;
  const size_t need = (size_t)B * (T + 1);
  if (stream_.size() - stream_pos_ < need) refill(need);
  const int32_t* w = stream_.data() + stream_pos_;
  xy.resize((size_t)2 * B * T);
  int32_t* x = xy.data();
  int32_t* y = x + (size_t)B * T;
  for (int b = 0; b < B; ++b) {
    std::memcpy(x + (size_t)b * T, w + (size_t)b * (T + 1), (size_t)T * 4);
    std::memcpy(y + (size_t)b * T, w + (size_t)b * (T + 1) + 1, (size_t)T * 4);
  }
  stream_pos_ += need;
}

void NameLoader::run() {
  for (;;) {
    std::vector<int32_t> xy;
    make_batch(xy);
    std::unique_lock<std::mutex> g(mu_);
    cv_space_.wait(g, [this] { return stop_ || (int)ready_.size() < c_.prefetch; });
    if (stop_) return;
    ready_.push_back(std::move(xy));
    g.unlock();
    cv_ready_.notify_one();
  }
}

void NameLoader::next(int32_t* x, int32_t* y) {
  std::vector<int32_t> xy;
  {
    std::unique_lock<std::mutex> g(mu_);
    cv_ready_.wait(g, [this] { return !ready_.empty(); });
    xy = std::move(ready_.front());
    ready_.pop_front();
    ++served_;
  }
  cv_space_.notify_one();
  const size_t n = (size_t)c_.B * c_.T;
  std::memcpy(x, xy.data(), n * 4);
  std::memcpy(y, xy.data() + n, n * 4);
}

}  // namespace gk
