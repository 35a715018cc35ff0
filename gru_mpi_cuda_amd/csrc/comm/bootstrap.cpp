#include "bootstrap.h"

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <stdexcept>
#include <thread>
#include <unistd.h>

namespace gk {

static const char kMagic[8] = {'G', 'K', 'U', 'I', 'D', '0', '0', '1'};
static constexpr size_t kUidBytes = 128;

static const char* env_str(const char* k) {
  const char* v = std::getenv(k);
  return v && *v ? v : nullptr;
}

LaunchEnv launch_env() {
  struct Scheme { const char *rank, *world, *local, *name; };
  static const Scheme schemes[] = {
      {"RANK", "WORLD_SIZE", "LOCAL_RANK", "torchrun"},
      {"OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK", "openmpi"},
      {"PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID", "hydra"},
      {"SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID", "slurm"},
  };
  LaunchEnv e;
  for (const Scheme& sc : schemes) {
    const char* r = env_str(sc.rank);
    const char* w = env_str(sc.world);
    if (!r || !w) continue;
    e.rank = std::atoi(r);
    e.world = std::atoi(w);
    const char* l = env_str(sc.local);
    e.local = l ? std::atoi(l) : e.rank;
    e.launcher = sc.name;
    if (e.world < 1 || e.rank < 0 || e.rank >= e.world)
      throw std::runtime_error(std::string("launch_env: inconsistent ") + sc.rank + "/" + sc.world);
    return e;
  }
  return e;
}

std::string bootstrap_key() {
  if (const char* r = std::getenv("GK_RUN_ID"); r && *r) return std::string("run:") + r;
  if (const char* t = std::getenv("TORCHELASTIC_RUN_ID"); t && *t && std::strcmp(t, "none") != 0)
    return std::string("te:") + t;
  if (const char* p = env_str("PMIX_NAMESPACE")) return std::string("pmix:") + p;
  if (const char* o = env_str("OMPI_MCA_ess_base_jobid")) return std::string("ompi:") + o;
  if (const char* j = env_str("SLURM_JOB_ID")) {
    const char* st = env_str("SLURM_STEP_ID");
    return std::string("slurm:") + j + "." + (st ? st : "0");
  }
  const char* port = std::getenv("MASTER_PORT");
  return "ppid:" + std::to_string((long)getppid()) + ":" + (port ? port : "0");
}

std::string bootstrap_path(const std::string& key) {
  if (const char* f = std::getenv("GK_BOOTSTRAP_FILE"); f && *f) return f;
  char hex[17];
  std::snprintf(hex, sizeof(hex), "%016zx", std::hash<std::string>{}(key));
  return std::string("/tmp/gk_namegen_") + hex + ".uid";
}

static std::string payload(const std::string& key, const std::string& uid) {
  std::string p(kMagic, sizeof(kMagic));
  const uint32_t n = (uint32_t)key.size();
  p.append(reinterpret_cast<const char*>(&n), 4);
  p += key;
  p += uid;
  return p;
}

std::string file_exchange_uid(int rank, const std::string& path, const std::string& key, const std::string& uid,
                              int timeout_ms) {
  const std::string want_head = payload(key, "");
  if (rank == 0) {
    if (uid.size() != kUidBytes) throw std::runtime_error("bootstrap: bad unique id size");
    std::remove(path.c_str());   // a stale file of an earlier job must not outlive this publish
    const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
    {
      std::ofstream o(tmp, std::ios::binary);
      const std::string p = payload(key, uid);
      o.write(p.data(), (std::streamsize)p.size());
      if (!o) throw std::runtime_error("bootstrap: cannot write " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("bootstrap: cannot publish " + path);
    return uid;
  }
  const auto end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (std::chrono::steady_clock::now() < end) {
    std::ifstream in(path, std::ios::binary);
    if (in) {
      std::string got((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
      // a complete payload of THIS job only (an old job's file is ignored until rank 0 replaces it)
      if (got.size() == want_head.size() + kUidBytes && got.compare(0, want_head.size(), want_head) == 0)
        return got.substr(want_head.size());
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  throw std::runtime_error("bootstrap: rank " + std::to_string(rank) + " timed out waiting for " + path +
                           " (job key " + key + ")");
}

}  // namespace gk
