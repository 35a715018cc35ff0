// Host-only checkpoint inspector: reads a parameter blob with the same reader the C API uses
// (ckpt_reader.cpp) and prints one JSON line -- total floats and, per tensor, offset, count and
// fp64 sum.  build_ext links it a second time with AddressSanitizer + UBSan
// (bin/ckpt_check_asan): the reference's only failure handling was exit(1) on a CUDA error
// (namegensf.cu:11-19) and it had no sanitizer story; tests/test_host_asan.py runs
// this binary on good, truncated and oversized blobs.
//
//   ckpt_check <blob path>          dims from <path>.json or GK_* env (see ckpt_reader.h)
#include <cstdio>
#include <exception>
#include <algorithm>
#include <string>
#include <vector>
#include "ckpt_reader.h"

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s <checkpoint>\n", argv[0]);
    return 2;
  }
  try {
    const gk::CkptDims d = gk::ckpt_dims(argv[1]);
    long total = 0;
    const auto off = gk::ckpt_offsets(d, &total);
    const std::vector<float> blob = gk::ckpt_read(argv[1], d);
    // tensor extents from consecutive offsets (map is name-ordered: sort by offset first)
    std::vector<std::pair<long, std::string>> order;
    for (const auto& kv : off) order.push_back({kv.second, kv.first});
    std::sort(order.begin(), order.end());
    std::printf("{\"total\": %ld, \"V\": %d, \"E\": %d, \"H\": %d, \"L\": %d, \"tensors\": {", total, d.V, d.E,
                d.H, d.L);
    for (size_t i = 0; i < order.size(); ++i) {
      const long o = order[i].first, end = i + 1 < order.size() ? order[i + 1].first : total;
      double s = 0.0;
      for (long k = o; k < end; ++k) s += blob[k];
      std::printf("%s\"%s\": [%ld, %ld, %.9g]", i ? ", " : "", order[i].second.c_str(), o, end - o, s);
    }
    std::printf("}}\n");
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ckpt_check: %s\n", e.what());
    return 3;
  }
}
