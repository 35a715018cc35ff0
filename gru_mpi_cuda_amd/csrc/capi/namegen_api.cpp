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
  // device buffers kept across namegen() calls (grown, never shrunk): the uniforms (the root holds
  // all N * MAX_LEN, another rank its slice) and the output rows (the root all N, another rank its own)
  float* rf = nullptr;
  size_t rf_cap = 0;
  unsigned char* out = nullptr;
  size_t out_cap = 0;
  long allocs = 0;   // device allocations made by namegen() (tests: none after the first call)
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
  // the reference's arithmetic is fp32 (namegensf.cu:233-242, 294-333), and so is the default here.
  // GK_GEN_PRECISION=bf16x3 selects split-bf16 products (fp32 everywhere else, ~2^-16 relative error
  // per product, 1.9x faster at 4096 names; parity with fp32 on near-tie samples unpinned), bf16 the
  // bf16 MFMA fast mode.
  const char* prec = std::getenv("GK_GEN_PRECISION");
  g.fp32 = !prec ? 1 : std::string(prec) == "bf16" ? 0 : std::string(prec) == "bf16x3" ? 2 : 1;
  st.gen.reset(new Generator(g, st.params, offsets));
  st.gen->refresh_weights(st.s);
  HIP_CHECK(hipStreamSynchronize(st.s));   // the reference's MPI_Barrier (namegensf.cu:615)
}

template <class T>
static T* ensure(T*& p, size_t& cap, size_t n, long& allocs) {
  if (n > cap) {
    if (p) HIP_CHECK(hipFree(p));
    HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
    cap = n;
    ++allocs;
  }
  return p;
}

// namegensf.cu:627-890.  The root's uniforms reach every rank as that rank's slice only (grouped
// ncclSend / ncclRecv: MPI_Scatter at cu:636, with the uneven remainder counts), the generated
// rows come back to the root the same way (MPI_Gather at cu:889); the buffers persist across calls.
static void namegen_impl(int N, float* random_floats, char* output) {
  if (!S) throw std::runtime_error("namegen: call namegen_initialize first");
  State& st = *S;
  const int ML = st.d.max_len;
  const bool root = st.rank == 0;
  std::vector<long> cnt(st.world), dsp(st.world), ocnt(st.world), odsp(st.world);
  for (int r = 0; r < st.world; ++r) {
    int s0 = 0, c0 = 0;
    shard(N, r, st.world, &s0, &c0);
    cnt[r] = (long)c0 * ML; dsp[r] = (long)s0 * ML;
    ocnt[r] = (long)c0 * (ML + 1); odsp[r] = (long)s0 * (ML + 1);
  }
  const int me = st.rank;
  const long my_names = cnt[me] / std::max(ML, 1);
  float* rf = ensure(st.rf, st.rf_cap, std::max<size_t>(1, root ? (size_t)N * ML : (size_t)cnt[me]), st.allocs);
  unsigned char* out = ensure(st.out, st.out_cap, std::max<size_t>(1, root ? (size_t)N * (ML + 1) : (size_t)ocnt[me]),
                              st.allocs);
  if (root && N > 0) HIP_CHECK(hipMemcpyAsync(rf, random_floats, (size_t)N * ML * 4, hipMemcpyHostToDevice, st.s));
  if (st.comm) st.comm->scatterv_f32(rf, cnt.data(), dsp.data(), rf, 0, st.s);
  // the root's slice sits at its displacement of the full buffer; another rank's at offset 0
  const size_t in_off = root ? (size_t)dsp[me] : 0, out_off = root ? (size_t)odsp[me] : 0;
  st.gen->set_global_names(N);   // the same precision path at every world size
  if (my_names > 0) st.gen->generate(rf + in_off, (int)my_names, out + out_off, st.s);
  if (st.comm) st.comm->gatherv_u8(out, ocnt.data(), odsp.data(), out, 0, st.s);
  if (root && N > 0) HIP_CHECK(hipMemcpyAsync(output, out, (size_t)N * (ML + 1), hipMemcpyDeviceToHost, st.s));
  HIP_CHECK(hipStreamSynchronize(st.s));
}

static void finalize_impl() {
  if (!S) return;
  State& st = *S;
  st.gen.reset();
  st.comm.reset();
  if (st.params) (void)hipFree(st.params);
  if (st.rf) (void)hipFree(st.rf);
  if (st.out) (void)hipFree(st.out);
  if (st.s) (void)hipStreamDestroy(st.s);
  if (st.rank == 0 && !st.uid_file.empty()) std::remove(st.uid_file.c_str());
  S.reset();
}

extern "C" int namegen_rank(void) { return S ? S->rank : launch_env().rank; }
extern "C" int namegen_world(void) { return S ? S->world : launch_env().world; }
extern "C" int namegen_max_len(void) { return S ? S->d.max_len : 0; }
extern "C" long namegen_device_allocs(void) { return S ? S->allocs : 0; }

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
