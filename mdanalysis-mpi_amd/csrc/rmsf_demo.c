/*
 * rmsf_demo.c -- a plain-C host of the context ABI (no Python, no torch):
 * RMSF.py's script (RMSF.py:53-146) for P "ranks" that are P contexts of one
 * process, exchanging through rmsf_multi_* (RCCL with --rccl, else the
 * in-process fold).
 *
 *   rmsf_demo FRAMES.f32 N_FRAMES N_ATOMS SEL.i64|- N_SEL P MODE OUT.f64 [--rccl] [--device]
 *
 * FRAMES.f32: float32 [N_FRAMES][N_ATOMS][3]; SEL.i64: int64 [N_SEL] atom
 * indices ("-" = atoms 0..N_SEL-1); MODE: none | frame0 | average | exact
 * (exact: RMSF.py:120-146 with the script's own arithmetic -- RMSF_PUSH_EXACT
 * per block, the blocks reduced in mpi4py's comm.reduce order by
 * rmsf_multi_chan_merge_exact, device to device);
 * OUT.f64: the RMSF, float64 [N_SEL].  Every context gets its RMSF.py:65-69
 * frame block (rmsf_block_range) and pushes it from host memory in two
 * halves (exercising the stager and the running Chan fold).  --device: each
 * block is first copied into its context's HBM and the contexts run the
 * one-process step -- rmsf_multi_push_frames (one host thread per context,
 * frame 0 as the reference or the merge shift) and the reduce to context 0
 * (rmsf_multi_chan_merge_root, RMSF.py:143).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rmsf_hip.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ != RMSF_OK) {                                                     \
      fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, rmsf_last_error());    \
      return 1;                                                               \
    }                                                                         \
  } while (0)

static void *slurp(const char *path, size_t bytes) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  void *p = malloc(bytes);
  if (p && fread(p, 1, bytes, f) != bytes) {
    free(p);
    p = NULL;
  }
  fclose(f);
  return p;
}

int main(int argc, char **argv) {
  if (argc < 9) {
    fprintf(stderr, "usage: %s FRAMES N_FRAMES N_ATOMS SEL|- N_SEL P none|frame0|average OUT [--rccl]\n", argv[0]);
    return 2;
  }
  const int64_t n_frames = atoll(argv[2]), n_atoms = atoll(argv[3]), n_sel = atoll(argv[5]);
  const int P = atoi(argv[6]);
  const char *mode = argv[7];
  int use_rccl = 0, on_device = 0;
  for (int a = 9; a < argc; ++a) {
    use_rccl |= strcmp(argv[a], "--rccl") == 0;
    on_device |= strcmp(argv[a], "--device") == 0;
  }
  const int exact = strcmp(mode, "exact") == 0;
  const int align = strcmp(mode, "none") != 0 && !exact, average = strcmp(mode, "average") == 0;
  if (P < 1 || P > 64 || n_frames < 1) return 2;

  float *xyz = (float *)slurp(argv[1], sizeof(float) * 3 * (size_t)(n_frames * n_atoms));
  int64_t *sel = strcmp(argv[4], "-") ? (int64_t *)slurp(argv[4], sizeof(int64_t) * (size_t)n_sel) : NULL;
  if (!xyz || (strcmp(argv[4], "-") && !sel)) {
    fprintf(stderr, "cannot read inputs\n");
    return 1;
  }
  int ndev = 0;
  CHECK(rmsf_device_count(&ndev));
  rmsf_ctx *ctx[64];
  int64_t b0[64], b1[64];
  for (int r = 0; r < P; ++r) {
    CHECK(rmsf_ctx_create(r % ndev, n_atoms, n_sel, sel, NULL, 0, &ctx[r]));
    CHECK(rmsf_block_range(n_frames, P, r, &b0[r], &b1[r]));
    printf("Process:%3d --> Frames: %10lld -- %10lld\n", r, (long long)b0[r], (long long)b1[r]);
  }
  if (use_rccl) CHECK(rmsf_multi_init_all(ctx, P));
  const size_t fsz = 3 * (size_t)n_atoms;
  double *rmsf = (double *)malloc(sizeof(double) * (size_t)n_sel);
  if (exact) {
    for (int r = 0; r < P; ++r) { /* RMSF.py:120-138, the recurrence continued across the halves */
      const int64_t n = b1[r] - b0[r], h = n / 2;
      CHECK(rmsf_push_frames(ctx[r], xyz + b0[r] * fsz, h, 0, RMSF_PUSH_EXACT, 0));
      CHECK(rmsf_push_frames(ctx[r], xyz + (b0[r] + h) * fsz, n - h, 0, RMSF_PUSH_EXACT, 0));
    }
    CHECK(rmsf_multi_chan_merge_exact(ctx, P, 0, RMSF_MERGE_MPI4PY)); /* RMSF.py:140-143 */
    CHECK(rmsf_get_rmsf(ctx[0], rmsf));                               /* RMSF.py:145-146 */
  } else if (on_device) {
    /* every block (and frame 0) in its context's HBM, then the one-process
     * step with no host synchronisation until the result */
    const float *d_block[64], *d_frame0[64];
    int64_t nf[64];
    void *mem[128];
    for (int r = 0; r < P; ++r) {
      nf[r] = b1[r] - b0[r];
      CHECK(rmsf_set_device(r % ndev));
      CHECK(rmsf_malloc(&mem[2 * r], sizeof(float) * fsz * (size_t)(nf[r] > 0 ? nf[r] : 1)));
      CHECK(rmsf_malloc(&mem[2 * r + 1], sizeof(float) * fsz));
      if (nf[r] > 0) CHECK(rmsf_memcpy_h2d(mem[2 * r], xyz + b0[r] * fsz, sizeof(float) * fsz * nf[r], NULL));
      CHECK(rmsf_memcpy_h2d(mem[2 * r + 1], xyz, sizeof(float) * fsz, NULL));
      CHECK(rmsf_stream_synchronize(NULL));
      d_block[r] = (const float *)mem[2 * r];
      d_frame0[r] = (const float *)mem[2 * r + 1];
    }
    if (average) {
      CHECK(rmsf_multi_push_frames(ctx, P, d_block, nf, 0, RMSF_PUSH_ALIGN_SUM, RMSF_MULTI_RESET, d_frame0, NULL,
                                   0));                                             /* RMSF.py:80-105 */
      CHECK(rmsf_multi_allreduce_sum(ctx, P));                                      /* RMSF.py:107-110 */
      for (int r = 0; r < P; ++r) CHECK(rmsf_set_reference_average(ctx[r]));      /* RMSF.py:111-118 */
      CHECK(rmsf_multi_push_frames(ctx, P, d_block, nf, 0, RMSF_PUSH_ALIGN_WELFORD, RMSF_MULTI_RESET, NULL, NULL, 0));
    } else {
      CHECK(rmsf_multi_push_frames(ctx, P, d_block, nf, 0, align ? RMSF_PUSH_ALIGN_WELFORD : RMSF_PUSH_WELFORD,
                                   RMSF_MULTI_RESET, align ? d_frame0 : NULL, align ? NULL : d_frame0, 0));
    }
    CHECK(rmsf_multi_chan_merge_root(ctx, P, 0)); /* RMSF.py:140-143: comm.reduce(root=0) */
    CHECK(rmsf_get_rmsf(ctx[0], rmsf));           /* RMSF.py:145-146, on the root */
    for (int r = 0; r < P; ++r) CHECK(rmsf_ctx_synchronize(ctx[r]));
    for (int r = 0; r < 2 * P; ++r) CHECK(rmsf_free(mem[r]));
  } else {
    if (align)
      for (int r = 0; r < P; ++r) CHECK(rmsf_set_reference_frame(ctx[r], xyz, 0)); /* RMSF.py:80-87 */
    if (average) {
      for (int r = 0; r < P; ++r) { /* sweep 1, RMSF.py:89-105 */
        const int64_t n = b1[r] - b0[r], h = n / 2;
        CHECK(rmsf_push_frames(ctx[r], xyz + b0[r] * fsz, h, 0, RMSF_PUSH_ALIGN_SUM, 0));
        CHECK(rmsf_push_frames(ctx[r], xyz + (b0[r] + h) * fsz, n - h, 0, RMSF_PUSH_ALIGN_SUM, 0));
      }
      CHECK(rmsf_multi_allreduce_sum(ctx, P));                                     /* RMSF.py:107-110 */
      for (int r = 0; r < P; ++r) CHECK(rmsf_set_reference_average(ctx[r]));     /* RMSF.py:111-118 */
    }
    const int push = align ? RMSF_PUSH_ALIGN_WELFORD : RMSF_PUSH_WELFORD;
    for (int r = 0; r < P; ++r) { /* RMSF.py:120-138 */
      const int64_t n = b1[r] - b0[r], h = n / 2;
      CHECK(rmsf_push_frames(ctx[r], xyz + b0[r] * fsz, h, 0, push, 0));
      CHECK(rmsf_push_frames(ctx[r], xyz + (b0[r] + h) * fsz, n - h, 0, push, 0));
    }
    CHECK(rmsf_multi_chan_merge(ctx, P)); /* RMSF.py:140-143 */
    CHECK(rmsf_get_rmsf(ctx[0], rmsf)); /* RMSF.py:145-146 */
  }
  FILE *o = fopen(argv[8], "wb");
  if (!o || fwrite(rmsf, sizeof(double), (size_t)n_sel, o) != (size_t)n_sel) return 1;
  fclose(o);
  for (int r = 0; r < P; ++r) CHECK(rmsf_ctx_destroy(ctx[r]));
  free(rmsf);
  free(xyz);
  free(sel);
  return 0;
}
