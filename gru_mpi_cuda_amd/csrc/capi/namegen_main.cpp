// Native driver for the 3-call API -- the role of the reference's missing main.cpp
// (MPI_Init -> random floats -> namegen_initialize / namegen / namegen_finalize).
//
//   namegen <parameter_file> <output_file> <N> [rng_seed]
//
// One process per GPU under torchrun / parallel.launch (RANK, WORLD_SIZE, LOCAL_RANK), Open MPI or
// MPICH `mpirun -np P`, or Slurm `srun` -- the reference's launch line works unchanged (the rank
// variables of each are read by comm/bootstrap.cpp launch_env; the RCCL unique id travels through a
// job-unique file).  Rank 0 draws
// N*MAX_LEN uniforms in [0,1) from rng_seed (splitmix64; the reference's generator is not in
// its repo), writes one name per line to output_file and prints the generation throughput.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "namegen_api.h"

static uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <parameter_file> <output_file> <N> [rng_seed]\n", argv[0]);
    return 2;
  }
  const char* param = argv[1];
  const char* outf = argv[2];
  const int N = std::atoi(argv[3]);
  const int seed = argc > 4 ? std::atoi(argv[4]) : 0;

  auto t0 = std::chrono::steady_clock::now();
  namegen_initialize(N, seed, const_cast<char*>(param));
  const int ML = namegen_max_len();
  std::vector<float> rf((size_t)N * ML);
  uint64_t s = (uint64_t)seed;
  for (auto& v : rf) v = (float)((splitmix64(s) >> 40) * (1.0 / 16777216.0));   // 24-bit uniform [0,1)
  std::vector<char> out((size_t)N * (ML + 1), 0);
  auto t1 = std::chrono::steady_clock::now();
  namegen(N, rf.data(), out.data());
  auto t2 = std::chrono::steady_clock::now();
  if (namegen_rank() == 0) {
    FILE* f = std::fopen(outf, "w");
    if (!f) { std::perror(outf); return 1; }
    for (int n = 0; n < N; ++n) std::fprintf(f, "%s\n", out.data() + (size_t)n * (ML + 1));
    std::fclose(f);
    const double gen_s = std::chrono::duration<double>(t2 - t1).count();
    const double init_s = std::chrono::duration<double>(t1 - t0).count();
    std::printf("{\"names\": %d, \"ranks\": %d, \"init_s\": %.4f, \"generate_s\": %.6f, \"names_per_s\": %.1f}\n",
                N, namegen_world(), init_s, gen_s, N / (gen_s > 0 ? gen_s : 1e-9));
  }
  namegen_finalize();
  return 0;
}
