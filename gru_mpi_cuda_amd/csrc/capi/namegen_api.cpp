// Native implementation of the reference's 3-call API (see namegen_api.h).
//
// Reference behaviour kept: same signatures, rank-0 output layout N x (MAX_LEN+1) with the EOS
// char written and NUL padding (namegensf.cu:877-882), the global random index n*MAX_LEN+l
// (namegensf.cu:876), the rank hello line (namegensf.cu:365-366).  Reference defects NOT kept
// (SURVEY §2.7): N % P names are generated (remainder spread over the first ranks), each rank
// uses its own GPU (LOCAL_RANK), only rank 0 reads the file, no leaked buffers.
#include "namegen_api.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <unistd.h>

#include "../runtime/runtime.h"
#include "../engine/generator.h"
#include "../comm/rccl_comm.h"
#include "../comm/bootstrap.h"
#include "ckpt_reader.h"

namespace {

using namespace gk;

struct State {
  int rank = 0, world = 1, local = 0;
  CkptDims d;
  float* params = nullptr;
  long nparams = 0;
  std::unique_ptr<Generator> gen;
  std::unique_ptr<RcclComm> comm;
  hipStream_t s = nullptr;
  std::string uid_file;
};
std::unique_ptr<State> S;

void shard(int n, int rank, int world, int* start, int* count) {
  const int base = n / world, rem = n % world;
  *count = base + (rank < rem ? 1 : 0);
  *start = rank * base + (rank < rem ? rank : rem);
}

}  // namespace

static void init_impl(int N, int rng_seed, char* parameter_fname) {
  (void)rng_seed;   // unused, as in the reference (namegensf.cu:359)
  S.reset(new State());
  State& st = *S;
  const LaunchEnv le = launch_env();   // torchrun, mpirun (Open MPI / Hydra) or srun
  st.rank = le.rank;
  st.world = le.world;
  st.local = le.local;
  global_rank() = st.rank;
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  HIP_CHECK(hipSetDevice(ndev > 0 ? st.local % ndev : 0));
  HIP_CHECK(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking));
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  std::printf("(%s) Hello world, rank %d out of %d\n", host, st.rank, st.world);
  std::fflush(stdout);

  if (st.world > 1) {
    // job-unique file exchange of the ncclUniqueId (comm/bootstrap.h)
    const std::string key = bootstrap_key();
    st.uid_file = bootstrap_path(key);
    const std::string uid = st.rank == 0 ? RcclComm::unique_id() : std::string();
    st.comm.reset(new RcclComm(file_exchange_uid(st.rank, st.uid_file, key, uid), st.rank, st.world));
  }
  // dims: rank 0's view (sidecar / env / defaults), broadcast so every rank agrees
  int dims[8] = {0};
  if (st.rank == 0) {
    st.d = ckpt_dims(parameter_fname);
    int v[8] = {st.d.V, st.d.E, st.d.H, st.d.L, st.d.max_len, st.d.sos, st.d.eos, 0};
    std::memcpy(dims, v, sizeof(v));
  }
  if (st.comm) {
    float* dd = nullptr;
    HIP_CHECK(hipMalloc(&dd, sizeof(dims)));
    HIP_CHECK(hipMemcpy(dd, dims, sizeof(dims), hipMemcpyHostToDevice));
    st.comm->broadcast_f32(dd, 8, 0, st.s);   // 32-bit payload, bit-exact
    HIP_CHECK(hipStreamSynchronize(st.s));
    HIP_CHECK(hipMemcpy(dims, dd, sizeof(dims), hipMemcpyDeviceToHost));
    HIP_CHECK(hipFree(dd));
    st.d.V = dims[0]; st.d.E = dims[1]; st.d.H = dims[2]; st.d.L = dims[3];
    st.d.max_len = dims[4]; st.d.sos = dims[5]; st.d.eos = dims[6];
  }
  long total = 0;
  auto offsets = ckpt_offsets(st.d, &total);
  st.nparams = total;
  HIP_CHECK(hipMalloc(&st.params, (size_t)total * 4));
  if (st.rank == 0) {
    std::vector<float> blob = ckpt_read(parameter_fname, st.d);
    HIP_CHECK(hipMemcpy(st.params, blob.data(), (size_t)total * 4, hipMemcpyHostToDevice));
  }
  if (st.comm) st.comm->broadcast_f32(st.params, total, 0, st.s);
  GenDims g;
  g.V = st.d.V; g.E = st.d.E; g.H = st.d.H; g.L = st.d.L; g.max_len = st.d.max_len;
  g.sos = st.d.sos; g.eos = st.d.eos;
  g.max_batch = std::max(64, std::min(8192, (N + st.world - 1) / std::max(1, st.world)));
  // the reference's arithmetic is fp32 (namegensf.cu:233-242, 294-333).  Default: bf16x3 (split-bf16
  // products, fp32 everywhere else): the same names as the fp64 oracle as often as fp32 over 3 seeds
  // x 2 reference-shaped presets (profiles/r3_gen_default_decision.jsonl) at 1.9x its speed.
  // GK_GEN_PRECISION=fp32 selects plain fp32 products, bf16 the bf16 MFMA fast mode.
  const char* prec = std::getenv("GK_GEN_PRECISION");
  g.fp32 = !prec ? 2 : std::string(prec) == "bf16" ? 0 : std::string(prec) == "fp32" ? 1 : 2;
  st.gen.reset(new Generator(g, st.params, offsets));
  st.gen->refresh_weights(st.s);
  HIP_CHECK(hipStreamSynchronize(st.s));   // the reference's MPI_Barrier (namegensf.cu:615)
}

static void namegen_impl(int N, float* random_floats, char* output) {
  if (!S) throw std::runtime_error("namegen: call namegen_initialize first");
  State& st = *S;
  const int ML = st.d.max_len;
  int start = 0, count = 0;
  shard(N, st.rank, st.world, &start, &count);
  const int per = (N + st.world - 1) / st.world;
  float* rf = nullptr;
  unsigned char *slab = nullptr, *all = nullptr;
  HIP_CHECK(hipMalloc(&rf, (size_t)std::max(N, 1) * ML * 4));
  HIP_CHECK(hipMalloc(&slab, (size_t)std::max(per, 1) * (ML + 1)));
  HIP_CHECK(hipMemsetAsync(slab, 0, (size_t)std::max(per, 1) * (ML + 1), st.s));
  if (st.rank == 0) HIP_CHECK(hipMemcpyAsync(rf, random_floats, (size_t)N * ML * 4, hipMemcpyHostToDevice, st.s));
  if (st.comm) st.comm->broadcast_f32(rf, (long)N * ML, 0, st.s);   // replaces MPI_Scatter (cu:636)
  if (count > 0) st.gen->generate(rf + (size_t)start * ML, count, slab, st.s);
  std::vector<unsigned char> host((size_t)st.world * per * (ML + 1));
  if (st.comm) {                                                    // replaces MPI_Gather (cu:889)
    HIP_CHECK(hipMalloc(&all, host.size()));
    st.comm->allgather_u8(slab, all, (long)per * (ML + 1), st.s);
    HIP_CHECK(hipMemcpyAsync(host.data(), all, host.size(), hipMemcpyDeviceToHost, st.s));
  } else {
    HIP_CHECK(hipMemcpyAsync(host.data(), slab, (size_t)per * (ML + 1), hipMemcpyDeviceToHost, st.s));
  }
  HIP_CHECK(hipStreamSynchronize(st.s));
  if (st.rank == 0) {
    std::memset(output, 0, (size_t)N * (ML + 1));
    for (int r = 0; r < st.world; ++r) {
      int s0 = 0, c0 = 0;
      shard(N, r, st.world, &s0, &c0);
      std::memcpy(output + (size_t)s0 * (ML + 1), host.data() + (size_t)r * per * (ML + 1), (size_t)c0 * (ML + 1));
    }
  }
  (void)hipFree(rf);
  (void)hipFree(slab);
  if (all) (void)hipFree(all);
}

static void finalize_impl() {
  if (!S) return;
  State& st = *S;
  st.gen.reset();
  st.comm.reset();
  if (st.params) (void)hipFree(st.params);
  if (st.s) (void)hipStreamDestroy(st.s);
  if (st.rank == 0 && !st.uid_file.empty()) std::remove(st.uid_file.c_str());
  S.reset();
}

extern "C" int namegen_rank(void) { return S ? S->rank : launch_env().rank; }
extern "C" int namegen_world(void) { return S ? S->world : launch_env().world; }
extern "C" int namegen_max_len(void) { return S ? S->d.max_len : 0; }

// C boundary: like the reference's CUDA_CALL, report and exit instead of unwinding into C
static void fatal(const std::exception& e) {
  std::fprintf(stderr, "[rank %d] namegen: %s\n", namegen_rank(), e.what());
  std::exit(1);
}
extern "C" void namegen_initialize(int N, int rng_seed, char* parameter_fname) {
  try { init_impl(N, rng_seed, parameter_fname); } catch (const std::exception& e) { fatal(e); }
}
extern "C" void namegen(int N, float* random_floats, char* output) {
  try { namegen_impl(N, random_floats, output); } catch (const std::exception& e) { fatal(e); }
}
extern "C" void namegen_finalize(void) {
  try { finalize_impl(); } catch (const std::exception& e) { fatal(e); }
}
