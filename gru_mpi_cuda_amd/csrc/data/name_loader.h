// Native training-data loader: packed character streams -> [B][T] (inputs, labels) int32 batches,
// produced by a background thread into a ring of ready batches so the step loop never waits on
// data generation (the Python syllable generator costs ~20 ms per 256 x 33 batch; one training
// step is 0.25 ms).
//
// Two sources, same packing (SOS name EOS SOS name EOS ... cut into windows of T+1 ids, every
// position a valid next-char target):
//   * synthetic: the seeded syllable generator of utils/data.py (same onset / vowel / coda
//     tables and capitalisation; its own xoshiro256** stream, so the exact names differ from the
//     numpy generator's but the distribution is the same);
//   * file: names, one per line (bytes = char ids, as NUM_CHAR = 256 in the reference,
//     namegensf.cu:862), reshuffled every epoch with the seeded generator.
// Rank r of a data-parallel job passes seed = base + r so ranks read different streams.
// No reference counterpart: the reference is inference-only.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace gk {

struct LoaderCfg {
  int B = 256, T = 32, sos = 0, eos = 0, max_len = 10;
  uint64_t seed = 0;
  int prefetch = 4;          // ready batches kept ahead of the consumer
  std::string path;          // empty: synthetic names; else a names file (one per line)
};

class NameLoader {
 public:
  explicit NameLoader(const LoaderCfg& c);
  ~NameLoader();
  NameLoader(const NameLoader&) = delete;
  NameLoader& operator=(const NameLoader&) = delete;

  // Blocks until a batch is ready; copies it to x[B*T], y[B*T] (row-major [B][T]).
  void next(int32_t* x, int32_t* y);
  long batches() const { return served_; }
  long names_in_file() const { return (long)file_names_.size(); }
  int epoch() const { return epoch_.load(); }

 private:
  struct Rng {   // xoshiro256**, seeded by splitmix64
    uint64_t s[4];
    explicit Rng(uint64_t seed);
    uint64_t next();
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
  };
  void run();
  void make_batch(std::vector<int32_t>& xy);
  void refill(size_t need);
  void append_name(const std::string& nm);
  void append_synth();

  LoaderCfg c_;
  Rng rng_;
  std::vector<std::string> file_names_;
  std::vector<uint32_t> order_;
  size_t cursor_ = 0;
  std::atomic<int> epoch_{0};
  std::vector<int32_t> stream_;   // packed ids not yet consumed, from stream_pos_
  size_t stream_pos_ = 0;

  std::mutex mu_;
  std::condition_variable cv_ready_, cv_space_;
  std::deque<std::vector<int32_t>> ready_;
  bool stop_ = false;
  long served_ = 0;
  std::thread worker_;
};

}  // namespace gk
