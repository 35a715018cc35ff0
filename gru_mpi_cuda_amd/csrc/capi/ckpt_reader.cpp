#include "ckpt_reader.h"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace gk {

static int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : dflt;
}

// minimal scan for `"key": <int>` in the sidecar (written by utils/ckpt.py)
static bool json_int(const std::string& s, const char* key, int* out) {
  const std::string k = std::string("\"") + key + "\"";
  size_t p = s.find(k);
  if (p == std::string::npos) return false;
  p = s.find(':', p + k.size());
  if (p == std::string::npos) return false;
  *out = std::atoi(s.c_str() + p + 1);
  return true;
}

CkptDims ckpt_dims(const std::string& path) {
  CkptDims d;
  d.V = env_int("GK_VOCAB", d.V); d.E = env_int("GK_EMBED", d.E); d.H = env_int("GK_HIDDEN", d.H);
  d.L = env_int("GK_LAYERS", d.L); d.max_len = env_int("GK_MAX_LEN", d.max_len);
  d.sos = env_int("GK_SOS", d.sos); d.eos = env_int("GK_EOS", d.eos);
  std::ifstream f(path + ".json");
  if (f) {
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    json_int(s, "vocab", &d.V); json_int(s, "embed", &d.E); json_int(s, "hidden", &d.H);
    json_int(s, "layers", &d.L); json_int(s, "max_len", &d.max_len);
    json_int(s, "sos", &d.sos); json_int(s, "eos", &d.eos);
  }
  return d;
}

std::map<std::string, long> ckpt_offsets(const CkptDims& d, long* total) {
  std::map<std::string, long> off;
  long o = 0;
  auto put = [&](const std::string& n, long sz) { off[n] = o; o += sz; };
  put("embedding", (long)d.V * d.E);
  for (int l = 0; l < d.L; ++l) put("weight_ih_l" + std::to_string(l), 3L * d.H * (l == 0 ? d.E : d.H));
  for (int l = 0; l < d.L; ++l) put("weight_hh_l" + std::to_string(l), 3L * d.H * d.H);
  for (int l = 0; l < d.L; ++l) put("bias_ih_l" + std::to_string(l), 3L * d.H);
  for (int l = 0; l < d.L; ++l) put("bias_hh_l" + std::to_string(l), 3L * d.H);
  put("fc.weight", (long)d.V * d.H);
  put("fc.bias", d.V);
  if (total) *total = o;
  return off;
}

std::vector<float> ckpt_read(const std::string& path, const CkptDims& d) {
  long total = 0;
  ckpt_offsets(d, &total);
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("namegen: cannot open parameter file " + path);
  std::fseek(f, 0, SEEK_END);
  const long bytes = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (bytes != total * 4) {
    std::fclose(f);
    throw std::runtime_error("namegen: " + path + " has " + std::to_string(bytes / 4) + " floats, dims (V=" +
                             std::to_string(d.V) + " E=" + std::to_string(d.E) + " H=" + std::to_string(d.H) +
                             " L=" + std::to_string(d.L) + ") need " + std::to_string(total));
  }
  std::vector<float> buf(total);
  const size_t got = std::fread(buf.data(), 4, total, f);
  std::fclose(f);
  if ((long)got != total) throw std::runtime_error("namegen: short read of " + path);
  return buf;
}

}  // namespace gk
