// Native reader for the reference checkpoint layout: a headerless
// little-endian fp32 blob of 27 tensors (for L = 2) in the order of namegensf.cu:375-407,
// generalised to any L as emb, all W_i, all W_h, all b_i, all b_h, W_fc, b_fc.
#pragma once
#include <map>
#include <string>
#include <vector>

namespace gk {

struct CkptDims {
  int V = 256, E = 512, H = 1024, L = 2, max_len = 10, sos = 0, eos = 0;
};

// dims from "<path>.json" if it exists (generalised format), else env overrides / defaults
CkptDims ckpt_dims(const std::string& path);
// float offsets of every named tensor inside the blob (names as in models/params.py)
std::map<std::string, long> ckpt_offsets(const CkptDims& d, long* total_floats);
// reads and size-checks the blob (throws on mismatch)
std::vector<float> ckpt_read(const std::string& path, const CkptDims& d);

}  // namespace gk
