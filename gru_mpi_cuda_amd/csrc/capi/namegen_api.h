/* The reference's engine API, same signatures (/root/reference/namegensf.cu:359, 627, 897),
 * implemented natively on the MI355X engine (csrc/engine/generator.cpp) with RCCL instead of MPI.
 *
 *   namegen_initialize(N, rng_seed, parameter_fname)
 *       reads the fp32 parameter blob (reference OFFSET layout; dims from `<fname>.json` when
 *       present, else GK_VOCAB/GK_EMBED/GK_HIDDEN/GK_LAYERS/GK_MAX_LEN/GK_SOS/GK_EOS or the
 *       reference defaults V=256 E=512 H=1024 L=2 MAX_LEN=10 SOS=EOS=0); rank 0 reads, the
 *       weights are broadcast over RCCL.  rng_seed is accepted and unused (as in the reference).
 *   namegen(N, random_floats, output)
 *       random_floats[N*MAX_LEN] (rank 0), output[N*(MAX_LEN+1)] filled on rank 0.  Name n
 *       uses random_floats[n*MAX_LEN + l] at step l on whichever rank generates it.
 *   namegen_finalize()
 *
 * Process model: one process per GPU, RANK / WORLD_SIZE / LOCAL_RANK from the environment
 * (any launcher); rank 0's ncclUniqueId is exchanged through the file GK_BOOTSTRAP_FILE
 * (default /tmp/gk_namegen_<MASTER_PORT>.uid).  WORLD_SIZE unset = single process.
 */
#ifndef GK_NAMEGEN_API_H
#define GK_NAMEGEN_API_H
#ifdef __cplusplus
extern "C" {
#endif

void namegen_initialize(int N, int rng_seed, char* parameter_fname);
void namegen(int N, float* random_floats, char* output);
void namegen_finalize(void);

/* extras */
int namegen_rank(void);
int namegen_world(void);
int namegen_max_len(void);
long namegen_device_allocs(void);   /* device allocations made by namegen() so far (buffers persist) */

#ifdef __cplusplus
}
#endif
#endif
