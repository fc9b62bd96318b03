/*
 * rmsf_hip.h -- C ABI of the MI355X (gfx950) frame-parallel RMSF path.
 *
 * This is the drop-in boundary for the hot path of i2nico/MDAnalysis-MPI
 * `RMSF.py` (the whole reference is that one file).  The reference has no
 * native FFI of its own: its per-frame loops call numpy, MDAnalysis
 * `lib.qcprot` (Cython) and mpi4py.  Every entry point below replaces one of
 * those call sites; the citation `RMSF.py:N` is /root/reference/RMSF.py line N.
 *
 * Conventions (all entry points):
 *   - Plain pointers and sizes only.  `d_` = device pointer (HBM, caller
 *     owned), `h_` = host pointer.  Coordinates are float32 `fac` layout
 *     (frame, atom, xyz); statistics are float64.
 *   - Every call returns an int status: 0 = ok, < 0 = error (see RMSF_E*).
 *     rmsf_last_error() returns a thread-local message for the last failure.
 *     No C++ exception crosses the ABI.
 *   - Device work is enqueued asynchronously on `stream` (a hipStream_t, NULL
 *     = the legacy default stream).  Nothing synchronises unless stated.
 *   - `sel` (int32 atom indices into a frame) may be NULL, meaning atoms
 *     0..n_sel-1 of each frame (the contiguous fast path).
 *   - `frame_stride` is the distance between consecutive frames in floats
 *     (>= 3*n_atoms of the frame; a multiple of it implements `step`).
 */
#ifndef RMSF_HIP_H
#define RMSF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMSF_ABI_VERSION 1

#define RMSF_OK 0
#define RMSF_EINVAL (-1)   /* bad argument (shape, null pointer, size)      */
#define RMSF_EHIP (-2)     /* HIP runtime error                             */
#define RMSF_ENOMEM (-3)   /* allocation failed / workspace too small       */
#define RMSF_EEMPTY (-4)   /* no frames to reduce (RMSF.py:39 would raise   */
                           /* ZeroDivisionError)                            */

/* accumulate modes for rmsf_accumulate() */
#define RMSF_MODE_WELFORD 0 /* n/mean/M2 per coordinate   (RMSF.py:137-138) */
#define RMSF_MODE_SUM 1     /* f64 sum of positions        (RMSF.py:103)     */

/* Size of one per-frame transform record written by rmsf_superpose():
 * R[9] (row-major, applied as x @ R, RMSF.py:100), mobile COM[3], rmsd, pad[3] */
#define RMSF_XFORM_DOUBLES 16
/* longest frame tile one rmsf_accumulate split may hold (Welford
 * coefficient table); n_splits >= ceil(n_frames / RMSF_MAX_SPLIT_FRAMES)    */
#define RMSF_MAX_SPLIT_FRAMES 4096
/* Size of the reference record written by rmsf_reference_setup():
 * [0..15]  ref_com[3], sum_r[3] (= sum of centred ref coords),
 *          G_ref (= sum |r|^2), total mass, n_sel, pad[7]
 * [16..]   scratch for the setup's fixed-order block reductions             */
#define RMSF_REFINFO_DOUBLES 2064

/* ---- library / device helpers (for callers without their own allocator) */
int rmsf_abi_version(void);
const char *rmsf_last_error(void);
int rmsf_device_count(int *n);
int rmsf_set_device(int dev);
int rmsf_malloc(void **d_ptr, size_t bytes);
int rmsf_free(void *d_ptr);
int rmsf_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes, void *stream);
int rmsf_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes, void *stream);
/* Strided device->device copy of `height` rows of `width` bytes (pitches in
 * bytes), asynchronous on `stream`: fills the HBM frame cache that lets the
 * second sweep (RMSF.py:124) read the frames the first (RMSF.py:92) staged. */
int rmsf_memcpy2d_d2d(void *d_dst, size_t dpitch, const void *d_src, size_t spitch,
                      size_t width, size_t height, void *stream);
int rmsf_stream_synchronize(void *stream);

/* ---- frame-block decomposition: RMSF.py:63-72 ----------------------------
 * per = n_frames // size; ranks 0..size-2 get [r*per, (r+1)*per); the last
 * rank gets [(size-1)*per, n_frames).  Pure integer, bit-exact.            */
int rmsf_block_range(int64_t n_frames, int size, int rank, int64_t *start,
                     int64_t *stop);

/* ---- reference structure: RMSF.py:80-87 (frame `ref_frame`, float32) and
 * RMSF.py:113-118 (the all-reduced float64 average) -------------------------
 * Exactly one of d_frame (float32 frame, atoms addressed via sel) or d_avg
 * (float64 [n_sel*3], already the selection) is non-NULL.
 * ref_com = sum(m x)/sum(m) in f64 (center_of_mass, RMSF.py:84,117);
 * d_ref[n_sel*3] = x - ref_com (f64, RMSF.py:85,118); d_refinfo as above.  */
int rmsf_reference_setup(const float *d_frame, const double *d_avg,
                         int64_t n_sel, const int32_t *d_sel,
                         const double *d_masses, double *d_ref,
                         double *d_refinfo, void *stream);

/* ---- RMSF.py:111 + 113-118 in one call: the sweep-1 average
 * d_avg[n_sel*3] = d_sum / n_frames (f64) and the reference setup from it, as
 * rmsf_divide() followed by rmsf_reference_setup(NULL, d_avg, ...) would
 * write them, bit for bit.  Up to 1,024 selected atoms this is ONE launch
 * (the division done as the sums are read); otherwise the same launches as
 * the two calls.                                                            */
int rmsf_reference_setup_mean(const double *d_sum, double n_frames,
                              int64_t n_sel, const double *d_masses,
                              double *d_avg, double *d_ref, double *d_refinfo,
                              void *stream);

/* ---- superposition: RMSF.py:94-97,127-131 + get_rotation_matrix RMSF.py:43-51
 * For every frame f of the block: mobile COM (mass-weighted, f64), the 3x3
 * inner product A = sum (x-com) (x) ref and E0 against the centred reference
 * (qcprot InnerProduct), then the QCP rotation (qcprot FastCalcRMSDAndRotation,
 * Theobald 2005 / Liu 2010) -> d_xform[f*RMSF_XFORM_DOUBLES + ...].
 * Two launches: a (frame, atom-chunk) covariance reduction and a per-frame
 * QCP solve.  d_work must hold rmsf_superpose_workspace_bytes() bytes.     */
size_t rmsf_superpose_workspace_bytes(int64_t n_sel, int64_t n_frames);
int rmsf_superpose(const float *d_xyz, int64_t frame_stride, int64_t n_frames,
                   int64_t n_sel, const int32_t *d_sel,
                   const double *d_masses, const double *d_ref,
                   const double *d_refinfo, double *d_xform, void *d_work,
                   size_t work_bytes, void *stream);

/* rmsf_superpose over a gathered selection (d_sel != NULL, rows) that also
 * COMPACTS it: every frame's selected rows, as the covariance pass stages
 * them, go out to d_dense_out + f * dense_stride as [n_sel][3] (f32, an exact
 * copy; dense_stride >= 3 n_sel floats, 0 = 3 n_sel), so the passes after it
 * -- the accumulate of this sweep, and with the whole block kept resident
 * every pass of RMSF.py's second sweep -- read n_sel dense rows (d_sel =
 * NULL, frame_stride = dense_stride) instead of gathering them again from
 * the full frames.  Same records, same bits as rmsf_superpose.  A gathered
 * row read costs every 128-B line holding a selected atom -- at CA-like
 * densities (1 in 10) nearly all of the frame -- so each avoided gather saves
 * up to ~10x the selected bytes ("Sparse selections").   */
int rmsf_superpose_compact(const float *d_xyz, int64_t frame_stride,
                           int64_t n_frames, int64_t n_sel, const int32_t *d_sel,
                           const double *d_masses, const double *d_ref,
                           const double *d_refinfo, double *d_xform,
                           void *d_work, size_t work_bytes, float *d_dense_out,
                           int64_t dense_stride, void *stream);

/* The same for frames stored as coordinate planes (SoA): atom a's x, y and
 * z of frame f at d_xyz + f*frame_stride + a (or d_sel[a]) + {0, 1, 2} *
 * plane_stride floats (frame_stride >= 3*plane_stride).  Same workspace,
 * same records, same arithmetic: the planes are read in place.           */
int rmsf_superpose_planes(const float *d_xyz, int64_t frame_stride,
                          int64_t plane_stride, int64_t n_frames,
                          int64_t n_sel, const int32_t *d_sel,
                          const double *d_masses, const double *d_ref,
                          const double *d_refinfo, double *d_xform,
                          void *d_work, size_t work_bytes, void *stream);

/* ---- streaming accumulator: RMSF.py:99-103 (SUM) and RMSF.py:133-138 (WELFORD)
 * For each frame: if d_xform != NULL apply the f32-faithful transform of
 * RMSF.py:99-101 / 133-135
 *     p = f32(f64(p) - com_f); p = f32(f64(p) @ R_f); p = f32(f64(p) + ref_com)
 * (ref_com from d_refinfo), then x = f64(p) feeds
 *   WELFORD: M2 += k/(k+1) (x-mean)^2 ; mean = (k mean + x)/(k+1)
 *   SUM:     sum += x
 * Frames are cut into n_splits contiguous splits (frame tiles); split s
 * holds frames [n_frames*s/n_splits, n_frames*(s+1)/n_splits) and writes
 * d_out0[s*3*n_sel + j] (mean or sum) and, for WELFORD, d_out1 (M2).
 * n_splits <= 0 picks one (see rmsf_accumulate_splits()).  The partials are
 * folded by rmsf_chan_merge() / rmsf_sum_splits().                          */
int rmsf_accumulate_splits(int64_t n_sel, int64_t n_frames, int aligned);
int rmsf_accumulate(const float *d_xyz, int64_t frame_stride, int64_t n_frames,
                    int64_t n_sel, const int32_t *d_sel,
                    const double *d_xform, const double *d_refinfo, int mode,
                    int n_splits, double *d_out0, double *d_out1,
                    void *stream);

/* split s of rmsf_accumulate() holds this many frames */
int64_t rmsf_split_count(int64_t n_frames, int n_splits, int s);

/* ---- balanced streaming accumulator (the default product path) ------------
 * Same arithmetic as rmsf_accumulate(), different work decomposition: the
 * batch's (256-lane chunk, frame) space is cut into n_groups equal contiguous
 * ranges, one per workgroup (n_groups <= 0: a per-kernel multiple of the
 * CU count -- 3 for the float4 Welford, 2 per atom lane, 32 with the
 * transform -- fewer for small batches), so every workgroup streams the same
 * bytes and no tail wave is left.  The partials and a plan header go to d_work
 * (rmsf_accumulate_balanced_workspace_bytes() bytes, 16-B aligned; the
 * bound covers every layout and mode for these n_sel/n_frames/n_groups).
 * rmsf_fold_balanced() then folds them, in frame order, into a running
 * result that already holds acc_n frames (acc_n = 0: d_acc* are
 * overwritten): Chan's merge (RMSF.py:36-41) into d_acc0 = mean,
 * d_acc1 = M2 for WELFORD; d_acc0 += sum for SUM.  n_coord = 3*n_sel.
 * d_work must not be reused between the two calls.                        */
size_t rmsf_accumulate_balanced_workspace_bytes(int64_t n_sel, int64_t n_frames,
                                                int n_groups);
int rmsf_accumulate_balanced(const float *d_xyz, int64_t frame_stride,
                             int64_t n_frames, int64_t n_sel,
                             const int32_t *d_sel, const double *d_xform,
                             const double *d_refinfo, int mode, int n_groups,
                             void *d_work, size_t work_bytes, void *stream);
int rmsf_fold_balanced(const void *d_work, int64_t n_coord, int mode,
                       int64_t acc_n, double *d_acc0, double *d_acc1,
                       void *stream);
/* rmsf_fold_balanced (WELFORD) of the last batch + the finalise of
 * RMSF.py:146 (d_rmsf[n_sel] over n_total frames), bit-identical to
 * rmsf_fold_balanced + rmsf_finalize, for every plan the accumulate can
 * write.  An atom plan (the aligned sweep, a gathered selection, planes: one
 * atom per lane) finalises inside the fold (one launch); the flat plan of an
 * unaligned contiguous selection (an atom's coordinates span two lanes) is
 * finalised by a second launch.  The plan is read from the workspace's own
 * header on the device (the host keeps no record of workspaces).          */
int rmsf_fold_balanced_finalize(const void *d_work, int64_t n_coord,
                                int64_t acc_n, double *d_acc0, double *d_acc1,
                                int64_t n_total, double *d_rmsf, void *stream);
/* The accumulate (RMSF.py:99-103 / 133-138 with d_xform, else the raw
 * frames) over frames stored as coordinate planes (see
 * rmsf_superpose_planes), read in place, one atom per lane; partials, header
 * and fold as rmsf_accumulate_balanced's.  (Without a selection, the
 * unaligned sweep can also read contiguous planes as rows of 3n floats on
 * the float4 stream and permute its statistics with rmsf_planes_to_rows.)  */
int rmsf_accumulate_balanced_planes(const float *d_xyz, int64_t frame_stride,
                                    int64_t plane_stride, int64_t n_frames,
                                    int64_t n_sel, const int32_t *d_sel,
                                    const double *d_xform,
                                    const double *d_refinfo, int mode,
                                    int n_groups, void *d_work,
                                    size_t work_bytes, void *stream);

/* ---- Chan merge: second_order_moments, RMSF.py:36-41 ------------------------
 * op(S1, S2): T = n1+n2, mu = (n1 mu1 + n2 mu2)/T, M = M1+M2+(n1 n2/T)(mu2-mu1)^2,
 * with RMSF.py's operations in its order (no FP contraction; n1 n2 / T as
 * Python's exact int product and one rounded division, exact for
 * n1 n2 < 2^53), so every value RMSF.py produces is reproduced bit for bit.
 * An empty partial (count 0) is RMSF.py:119-121's (0, zeros, zeros) -- its
 * memory is not read -- and enters op like any other (op((0,0,0), S) is not
 * S bit for bit, as in RMSF.py).  op of two empty partials (T = 0), where
 * RMSF.py:39 raises ZeroDivisionError, is skipped: the result stays empty.
 * RMSF_EEMPTY when every partial is empty.
 *
 * rmsf_chan_merge folds n_parts partials of n_coord coordinates in order:
 * res = part 0, res = op(res, part i) for i = 1..n_parts-1 (mpi4py's naive
 * reduce, RMSF_MERGE_RANK below).  h_counts: host array of n_parts counts. */
int rmsf_chan_merge(const double *d_mean_parts, const double *d_m2_parts,
                    const int64_t *h_counts, int n_parts, int64_t n_coord,
                    double *d_mean, double *d_m2, void *stream);

/* The order RMSF.py:143's comm.reduce(S, root=0, op=second_order_moments)
 * applies op in (mpi4py's lowercase object reduce; upstream, not vendored):
 *   RMSF_MERGE_MPI4PY  mpi4py's default (rc.fast_reduce): a binomial tree,
 *                      for mask = 1, 2, 4, ...: rank r, r % (2 mask) == 0,
 *                      computes op(S_r, S_{r+mask}) -- at 4 ranks
 *                      op(op(S0,S1), op(S2,S3)), at 5 op(op(op(S0,S1),
 *                      op(S2,S3)), S4).  Equal to RANK up to 3 ranks.
 *   RMSF_MERGE_RANK    rc.fast_reduce = False: op folded in rank order.   */
#define RMSF_MERGE_RANK 0
#define RMSF_MERGE_MPI4PY 1
/* The schedule as (dst, src) steps S[dst] = op(S[dst], S[src]), S[0] the
 * result: returns the step count (n_parts - 1) and, when h_dst/h_src are
 * non-NULL, writes up to `capacity` steps.                                   */
int rmsf_chan_reduce_steps(int n_parts, int order, int *h_dst, int *h_src,
                           int capacity);
/* comm.reduce's result over n_parts partials (the ranks' S of RMSF.py:140,
 * in rank order) in the given order, written to d_mean / d_m2.  The parts
 * are the schedule's working storage (each rank's `result`, as in mpi4py)
 * and are overwritten.                                                      */
int rmsf_chan_reduce(double *d_mean_parts, double *d_m2_parts,
                     const int64_t *h_counts, int n_parts, int64_t n_coord,
                     int order, double *d_mean, double *d_m2, void *stream);
/* One step S1 = op(S1, S2) in place (S2 in separate buffers: the partial
 * another rank or device just sent) -- a distributed reduction's building
 * block.  RMSF_EEMPTY when n1 = n2 = 0.                                    */
int rmsf_chan_merge_pair(double *d_mean1, double *d_m21, int64_t n1,
                         const double *d_mean2, const double *d_m22,
                         int64_t n2, int64_t n_coord, void *stream);

/* sum of split partial sums (sweep 1, RMSF.py:103,105) */
int rmsf_sum_splits(const double *d_parts, int n_parts, int64_t n_coord,
                    double *d_sum, void *stream);

/* y = x / divisor  (average structure, RMSF.py:111) */
int rmsf_divide(const double *d_x, double divisor, int64_t n, double *d_y,
                void *stream);

/* Exact k-way Chan across ranks as two all-reduce(SUM) passes (replaces the
 * pickle comm.reduce of RMSF.py:143):
 *   pass 1 input: d_out = w * mean_k            (w = n_k / n)
 *   pass 2 input: d_out = M2_k + n_k (mean_k - mean)^2                      */
int rmsf_chan_weight(const double *d_mean_k, double w, int64_t n,
                     double *d_out, void *stream);
int rmsf_chan_deviation(const double *d_mean_k, const double *d_m2_k,
                        const double *d_mean, double n_k, int64_t n,
                        double *d_out, void *stream);

/* One-collective form of the same merge (RMSF.py:140-143 + 146): moments
 * about a shift c held by every rank (c[j] = shift[j] + off3[j % 3]; shift
 * f64, or f32 when shift_is_f32; off3 may be NULL):
 *   pack:   d_t[0:n] = n_k (mean_k - c),  d_t[n:2n] = M2_k + n_k (mean_k - c)^2
 *   -- one all-reduce(SUM) of d_t[0:2n] over the ranks --
 *   finish: mean = c + T1/n,  M2 = max(T2 - T1^2/n, 0),  rmsf = sqrt(sum M2 / n)
 * (d_rmsf may be NULL; n = 3 n_sel coordinates).                           */
int rmsf_chan_shift_pack(const double *d_mean_k, const double *d_m2_k,
                         const void *d_shift, int shift_is_f32,
                         const double *d_off3, double n_k, int64_t n,
                         double *d_t, void *stream);
int rmsf_chan_shift_finish(const double *d_t, const void *d_shift,
                           int shift_is_f32, const double *d_off3,
                           int64_t n_sel, int64_t n_frames, double *d_mean,
                           double *d_m2, double *d_rmsf, void *stream);

/* rmsf_fold_balanced (WELFORD) and rmsf_chan_shift_pack in ONE launch, for a
 * rank's last batch before the cross-rank merge: the fold as above, then
 * d_t as the pack writes it, with n_k = acc_n + the batch's frames --
 * bit-identical to the two calls (RMSF.py:36-41 + 140-143).                */
int rmsf_fold_balanced_shift(const void *d_work, int64_t n_coord,
                             int64_t acc_n, double *d_acc0, double *d_acc1,
                             const void *d_shift, int shift_is_f32,
                             const double *d_off3, double *d_t, void *stream);

/* The reduce-scatter form of the merge (RMSF.py:140-143 with :146 on each
 * rank's atom slice, then only the RMSF gathered to the root): the same
 * T1/T2 in the ATOM-SLICED layout -- for slice_coords = 3 x atoms per rank,
 * slice r = j / slice_coords holds [T1 | T2] of its slice_coords
 * coordinates at d_t + 2 r slice_coords (T2 slice_coords after T1), so a
 * reduce-scatter of equal chunks gives rank r its slice; coordinates past n
 * in the last slice are not written (the caller zeroes that padding).
 * rmsf_chan_shift_finish_slice unpacks one reduced slice [T1 | T2] of width
 * slice_coords for its n_sel atoms (d_shift, d_mean, d_m2, d_rmsf point at
 * the slice's first atom).  Bit-identical per coordinate to the plain
 * layout's pack and finish.                                                 */
int rmsf_fold_balanced_shift_sliced(const void *d_work, int64_t n_coord,
                                    int64_t acc_n, double *d_acc0,
                                    double *d_acc1, const void *d_shift,
                                    int shift_is_f32, const double *d_off3,
                                    int64_t slice_coords, double *d_t,
                                    void *stream);
int rmsf_chan_shift_pack_sliced(const double *d_mean_k, const double *d_m2_k,
                                const void *d_shift, int shift_is_f32,
                                const double *d_off3, double n_k, int64_t n,
                                int64_t slice_coords, double *d_t,
                                void *stream);
int rmsf_chan_shift_finish_slice(const double *d_t, int64_t slice_coords,
                                 const void *d_shift, int shift_is_f32,
                                 const double *d_off3, int64_t n_sel,
                                 int64_t n_frames, double *d_mean, double *d_m2,
                                 double *d_rmsf, void *stream);

/* Atom slabs of the flat WELFORD plan (no selection, no transform, 16-B
 * aligned float4 columns), so a rank's cross-rank merge can start on the
 * first slab while the next one streams (large n_sel; RMSF.py:140-143).
 * rmsf_balanced_slab_chunks: *h_chunks = the plan's chunk count C (256
 * lanes of 4 coordinates = 1024 coordinates each) when the plan is
 * chunk-aligned, else 0 (no slabs).  rmsf_accumulate_balanced_slab runs
 * the whole plan's ranges of chunks [c0, c1) -- the same segments, so the
 * slab's partials equal the whole launch's -- into the same d_work;
 * rmsf_fold_balanced_shift_slab folds those chunks into d_acc* (global
 * coordinates) and writes the slab's [T1 | T2] (2 (j1 - j0) doubles,
 * j0 = 1024 c0, j1 = min(1024 c1, n_coord)) to d_t.  Bit-identical to the
 * whole-selection calls for every coordinate.  Slab bounds that are a
 * multiple of 3 chunks keep whole atoms together (rmsf_chan_shift_finish
 * per slab).                                                               */
int rmsf_balanced_slab_chunks(const float *d_xyz, int64_t frame_stride,
                              int64_t n_frames, int64_t n_sel,
                              int64_t *h_chunks);
int rmsf_accumulate_balanced_slab(const float *d_xyz, int64_t frame_stride,
                                  int64_t n_frames, int64_t n_sel, int64_t c0,
                                  int64_t c1, void *d_work, size_t work_bytes,
                                  void *stream);
int rmsf_fold_balanced_shift_slab(const void *d_work, int64_t n_coord,
                                  int64_t acc_n, double *d_acc0,
                                  double *d_acc1, const void *d_shift,
                                  int shift_is_f32, const double *d_off3,
                                  double *d_t, int64_t c0, int64_t c1,
                                  void *stream);

/* ---- RMSF.py:137-138 as written: the sequential Welford ---------------------
 * For every selected coordinate (atom d_sel[a], or a, when d_sel is NULL;
 * f32 rows d_xyz[f * frame_stride + 3 atom + c], no transform), the frames
 * f = 0 .. n_frames-1 in order with k = k0 + f:
 *   sumsquares += (k / (k + 1.0)) * (x - mean)**2 ;  mean = (k*mean + x)/(k+1)
 * in numpy's operations and roundings, so d_mean / d_sumsquares (f64
 * [3 n_sel], the running state after k0 frames; k0 = 0: start from zeros,
 * inputs ignored) end as the reference recurrence's own values bit for bit
 * -- a rank's S of RMSF.py:140, which rmsf_chan_merge then combines as
 * RMSF.py:143 does, also bit for bit.  Parallel over coordinates only (one
 * lane per coordinate through every frame; one lane per atom for a d_sel of
 * >= 49,152 atoms -- same bits); rmsf_accumulate_balanced is the
 * reassociated, frame-parallel form (faster, equal to ~1e-13).
 * d_work: rmsf_welford_sequential_workspace_bytes(n_frames) bytes (the
 * per-frame coefficients).  Replaces RMSF.py:120-138's loop for one rank.
 * Domain of the bit-for-bit claim: any float32 coordinates (zeros and
 * infinities included; NaN wherever the reference has NaN, payload bits
 * aside) and any running state they can produce; a caller-made state with
 * |mean| beyond ~1e270 would need the full division sequence.              */
size_t rmsf_welford_sequential_workspace_bytes(int64_t n_frames);
int rmsf_welford_sequential(const float *d_xyz, int64_t frame_stride,
                            int64_t n_frames, int64_t n_sel,
                            const int32_t *d_sel, int64_t k0, double *d_mean,
                            double *d_sumsquares, void *d_work,
                            size_t work_bytes, void *stream);

/* ---- exact=True on the ALIGNED path: RMSF.py:80-146 in the reference's own
 * summation orders -----------------------------------------------------------
 * The frame-parallel kernels above (rmsf_reference_setup, rmsf_superpose,
 * rmsf_accumulate*) reassociate the per-frame sums; their rotations then
 * differ from the script's in the last bits, which now and then flips an
 * f32 rounding point of an aligned coordinate (RMSF.py:99-101) -- a few
 * e-8 A at 100 frames, but up to ~ulp/2 = 2e-6 A at 2 frames.  These three
 * entry points remove every such source: each sum runs atom by atom or
 * frame by frame exactly as the reference runs it, so the transform records,
 * the sweep-1 sums, the average and the Welford state equal the script's
 * bit for bit.  The orders of the absent upstream dependencies are the
 * published ones, restated (oracle/rmsf_oracle.py; upstream, unverified):
 *   AtomGroup.center_of_mass(): einsum('ij,ij->j', x, m[:, None]) / m.sum()
 *     -- a sequential sum over the atoms of f64(x) * m, divided by
 *     mass_total = the caller's numpy ``masses.sum()`` (numpy sums pairwise;
 *     n_sel when d_masses is NULL, i.e. unit masses);
 *   qcprot InnerProduct: one pass over the atoms, A[3a+b] += mob_a ref_b,
 *     G1 += x*x + y*y + z*z per atom, E0 = (G1 + G2) * 0.5.
 *
 * rmsf_reference_setup_sequential: RMSF.py:84-85 (d_frame, f32, atoms via
 * d_sel) or RMSF.py:111 + 117-118 (d_avg = the all-reduced f64 sweep-1 sums,
 * divided by avg_divisor = n_frames as they are read and written to
 * d_avg_out when non-NULL; d_sel must be NULL): ref_com, d_ref = x - ref_com,
 * and the refinfo record (ref_com, sum r, G2 of qcprot's loop, mass_total,
 * n_sel).  Each sum is one wave's in-order add chain (two chain phases,
 * ~0.2 ms each per 100k atoms); below 16,384 atoms one launch, from there
 * the fill and the centring as grid-wide launches around the chains.      */
int rmsf_reference_setup_sequential(const float *d_frame, const double *d_avg,
                                    double avg_divisor, int64_t n_sel,
                                    const int32_t *d_sel, const double *d_masses,
                                    double mass_total, double *d_avg_out,
                                    double *d_ref, double *d_refinfo,
                                    void *stream);
/* The two halves of rmsf_reference_setup_sequential, same bits and the same
 * arguments: rmsf_reference_centre_sequential writes d_ref (centred) and
 * d_refinfo[0..2] (ref_com) -- all an InnerProduct needs;
 * rmsf_reference_sums_sequential writes the rest of the record from the
 * centred d_ref (sum r, G2, mass_total, n_sel).  Only the QCP reads G2, so the
 * sums may run on another stream beside rmsf_inner_product_sequential.    */
int rmsf_reference_centre_sequential(const float *d_frame, const double *d_avg,
                                     double avg_divisor, int64_t n_sel,
                                     const int32_t *d_sel, const double *d_masses,
                                     double mass_total, double *d_avg_out,
                                     double *d_ref, double *d_refinfo,
                                     void *stream);
int rmsf_reference_sums_sequential(int64_t n_sel, double mass_total,
                                   const double *d_ref, double *d_refinfo,
                                   void *stream);
/* rmsf_superpose_sequential: RMSF.py:94-97 / 127-131 + get_rotation_matrix
 * for every frame: mobile COM atom by atom, centred coordinates f64(x) - com,
 * InnerProduct against d_ref (G2 from d_refinfo[6], i.e. a record of
 * rmsf_reference_setup_sequential), QCP -> d_xform[f * RMSF_XFORM_DOUBLES]
 * as rmsf_superpose writes it (COM absolute).  Rows only (frame, atom, xyz).
 * Three launches: the COM (one wave per frame and axis), the InnerProduct
 * (one wave per frame and sum: A[0..8], G1) and the QCP (one lane per
 * frame); d_xform holds the COM and the sums in between.  Each sum is an
 * in-order add chain over the atoms, so the cost grows with n_sel, not the
 * frames: ~0.7 ms per 100k atoms ("Few frames").       */
int rmsf_superpose_sequential(const float *d_xyz, int64_t frame_stride,
                              int64_t n_frames, int64_t n_sel,
                              const int32_t *d_sel, const double *d_masses,
                              double mass_total, const double *d_ref,
                              const double *d_refinfo, double *d_xform,
                              void *stream);
/* The two halves of rmsf_superpose_sequential, same bits:
 * rmsf_frame_com_sequential writes every frame's mobile COM (RMSF.py:94 /
 * 127) to d_xform[f * RMSF_XFORM_DOUBLES + 9..11]; it needs no reference, so
 * it may run on another stream beside rmsf_reference_setup_sequential.
 * rmsf_superpose_sequential_from_com then runs the InnerProduct and the QCP
 * from those COMs (it keeps [9..11] and rewrites the rest of the record).
 * It is in turn rmsf_inner_product_sequential (A[0..8] and G1 into the
 * record's [0..8] and [13]; needs the centred d_ref only) followed by
 * rmsf_superpose_sequential_qcp (E0 = (G1 + d_refinfo[6]) * 0.5 and the QCP:
 * R in [0..8], rmsd in [12], [13..15] zero).                                */
int rmsf_frame_com_sequential(const float *d_xyz, int64_t frame_stride,
                              int64_t n_frames, int64_t n_sel,
                              const int32_t *d_sel, const double *d_masses,
                              double mass_total, double *d_xform, void *stream);
int rmsf_superpose_sequential_from_com(const float *d_xyz, int64_t frame_stride,
                                       int64_t n_frames, int64_t n_sel,
                                       const int32_t *d_sel, const double *d_ref,
                                       const double *d_refinfo, double *d_xform,
                                       void *stream);
int rmsf_inner_product_sequential(const float *d_xyz, int64_t frame_stride,
                                  int64_t n_frames, int64_t n_sel,
                                  const int32_t *d_sel, const double *d_ref,
                                  double *d_xform, void *stream);
int rmsf_superpose_sequential_qcp(int64_t n_frames, int64_t n_sel,
                                  const double *d_refinfo, double *d_xform,
                                  void *stream);
/* rmsf_accumulate_sequential: the frames in order for every selected atom
 * (one lane per atom), k = k0 + f, each frame transformed first when d_xform
 * (+ d_refinfo) is given (RMSF.py:99-101 / 133-135, the same f32-faithful
 * transform as rmsf_accumulate), then
 *   RMSF_MODE_SUM:     d_acc0 += x                          (RMSF.py:103)
 *   RMSF_MODE_WELFORD: rmsf_welford_sequential's recurrence (RMSF.py:137-138)
 *                      on (d_acc0 = mean, d_acc1 = sumsquares)
 * continuing the running state after k0 frames (k0 = 0: from zeros).  The
 * WELFORD mode needs d_work of rmsf_welford_sequential_workspace_bytes
 * (n_frames) bytes; SUM needs none.  Rows only.                            */
int rmsf_accumulate_sequential(const float *d_xyz, int64_t frame_stride,
                               int64_t n_frames, int64_t n_sel,
                               const int32_t *d_sel, const double *d_xform,
                               const double *d_refinfo, int mode, int64_t k0,
                               double *d_acc0, double *d_acc1, void *d_work,
                               size_t work_bytes, void *stream);

/* ---- finalise: RMSF.py:146  rmsf = sqrt(M2.sum(axis=1) / n) ---------------*/
int rmsf_finalize(const double *d_m2, int64_t n_sel, int64_t n_frames,
                  double *d_rmsf, void *stream);

/* ---- qcprot.CalcRMSDRotationalMatrix (RMSF.py:48) --------------------------
 * Batched QCP on device: A[n][9], E0[n], atom counts N[n] -> rot[n][9],
 * rmsd[n].  Exposed for the upstream known-answer test.                      */
int rmsf_qcp_batch(const double *d_A, const double *d_E0, const double *d_N,
                   int64_t n, double *d_rot, double *d_rmsd, void *stream);

/* Host-pointer form with the signature of
 * MDAnalysis.lib.qcprot.CalcRMSDRotationalMatrix(ref, conf, N, rot, weights)
 * (called at RMSF.py:48): ref/conf f64 [N][3] (already centred by the
 * caller), rot f64[9] out, weights NULL or f64[N].  Runs on the current
 * device, synchronous.  *rmsd_out receives the rmsd.                        */
int rmsf_calc_rmsd_rotational_matrix(const double *h_ref, const double *h_conf,
                                     int64_t N, double *h_rot,
                                     const double *h_weights,
                                     double *rmsd_out);

/* ---- scattered frames (RMSF.run(frames=...), RMSF.py:92,124 frame source) --
 * Compact batch d_dst[k][j][3] (k < n_frames <= 65535, j < n_sel) of the
 * frames at d_src + d_frames[k]*frame_stride (device int64 indices), the
 * selection d_sel (NULL = atoms 0..n_sel-1) gathered: one launch per batch
 * of a scattered frame list instead of kernel launches per frame.           */
int rmsf_gather_frames(const float *d_src, int64_t frame_stride,
                       const int64_t *d_frames, int64_t n_frames, int64_t n_sel,
                       const int32_t *d_sel, float *d_dst, void *stream);

/* The same compact batch from HBM-resident frames stored as coordinate
 * planes (SoA): frame k's x[n_atoms], y and z at d_src + d_frames[k] *
 * frame_stride + {0, 1, 2} * plane_stride floats (frame_stride >=
 * 3 * plane_stride).  The selection is gathered from each plane and
 * interleaved into d_dst's [n_frames][n_sel][3] rows for the kernels above
 * (an extra read and write of the selected bytes: a convenience path for
 * data that already lives in HBM as planes).                               */
int rmsf_gather_planes(const float *d_src, int64_t frame_stride,
                       int64_t plane_stride, const int64_t *d_frames,
                       int64_t n_frames, int64_t n_sel, const int32_t *d_sel,
                       float *d_dst, void *stream);

/* Per-coordinate f64 statistics in plane order (x[n], y[n], z[n]) to
 * (atom, xyz) order, d_dst[3a + c] = d_src[c*n + a] (d_dst != d_src): the
 * unaligned accumulate reads contiguous coordinate planes in place, as it
 * reads rows (its statistics are per coordinate), and its mean / M2 come
 * out in plane order.                                                      */
int rmsf_planes_to_rows(const double *d_src, int64_t n, double *d_dst,
                        void *stream);

/* ---- synthetic trajectories -------------------------------
 * out[f*frame_stride + 3*a + c] for frames [f0, f0+nf) of n_atoms atoms:
 *   base(a,c) ~ U[0,100), sigma(a) ~ U[0.2,2.0), g ~ triangular, unit var,
 *   p = base + sigma*g ; optional rigid motion from d_motion[f][12]
 *   (R[9] row-major, t[3]):  p' = ((p-50) @ R) + t ; out = f32(p').
 * Counter-based (splitmix64 of seed/frame/atom/axis) with every float op
 * explicitly rounded, so the CPU regenerates any slice bit-identically.     */
int rmsf_synth_frames(float *d_out, int64_t frame_stride, int64_t n_atoms,
                      int64_t f0, int64_t nf, uint64_t seed,
                      const double *d_motion, void *stream);
/* The generator's noise scale sigma(a) of atoms a0..a0+n-1 (f64, device):
 * an unaligned synthetic atom's population RMSF is sqrt(3) sigma(a) -- the
 * reference value of the bench's per-mode sanity figure.                    */
int rmsf_synth_sigma(double *d_sigma, int64_t a0, int64_t n, uint64_t seed,
                     void *stream);

/* ---- host -> device frame stager (north star subsystem 1) ---
 * Pinned-host, multi-buffered hipMemcpyAsync stager.  Frames arrive as host
 * float32 arrays of n_atoms_frame atoms; the selection (h_sel, NULL = first
 * n_sel atoms) is gathered on the host into a pinned slot by a thread pool,
 * the slot is copied on the stager's own copy stream, and the consumer
 * stream is made to wait on the copy event.  A slot is reused only after
 * the consumer released it (an event recorded on the consumer stream).     */
typedef struct rmsf_stager rmsf_stager;
int rmsf_stager_create(int64_t n_atoms_frame, int64_t n_sel,
                       const int32_t *h_sel, int64_t batch_frames,
                       int n_slots, int n_threads, rmsf_stager **out);
int rmsf_stager_destroy(rmsf_stager *st);
/* Stage n_frames (<= batch_frames) host frames (stride h_frame_stride
 * floats) into the next slot.  Returns the slot index and its device
 * pointer (compact [n_frames][n_sel][3] layout, frame_stride = 3*n_sel).
 * `consumer_stream` waits on the copy before any later work it runs.       */
int rmsf_stager_stage(rmsf_stager *st, const float *h_frames,
                      int64_t h_frame_stride, int64_t n_frames,
                      void *consumer_stream, int *slot, float **d_batch);
/* Stage frames given as an array of n_frames host pointers (one per frame,
 * each n_atoms_frame*3 floats) -- the per-Timestep MDAnalysis path.        */
int rmsf_stager_stage_ptrs(rmsf_stager *st, const float *const *h_frame_ptrs,
                           int64_t n_frames, void *consumer_stream, int *slot,
                           float **d_batch);
/* Stage frames stored as coordinate planes (SoA): frame f's x[n_atoms_frame],
 * y and z at h_frame_ptrs[f], + h_plane_stride and + 2*h_plane_stride floats
 * (h_plane_stride >= n_atoms_frame) -- a synthetic [F][3][n] array, or a DCD
 * frame's X/Y/Z records in place (RMSF.py:92,124's reader interleaves them
 * per frame).  The selection is gathered and interleaved on the host into
 * the same compact [n_frames][n_sel][3] device batch as rmsf_stager_stage().*/
int rmsf_stager_stage_planes(rmsf_stager *st, const float *const *h_frame_ptrs,
                             int64_t h_plane_stride, int64_t n_frames,
                             void *consumer_stream, int *slot, float **d_batch);
/* Decode XTC frames f0, f0+step, ... (n_frames of them) frame-parallel
 * straight into the next pinned slot (selection applied), then DMA it. */
typedef struct rmsf_xtc rmsf_xtc;
int rmsf_stager_stage_xtc(rmsf_stager *st, const rmsf_xtc *x, int64_t f0,
                          int64_t n_frames, int64_t step,
                          void *consumer_stream, int *slot, float **d_batch);
/* Mark the slot free once the work queued so far on consumer_stream ends. */
int rmsf_stager_release(rmsf_stager *st, int slot, void *consumer_stream);
/* Wait until every copy issued by the stager has completed. */
int rmsf_stager_synchronize(rmsf_stager *st);

/* ---- GROMACS XTC trajectories ---------------------------
 * Host reader/writer replacing libxdrfile behind MDAnalysis' XTCReader, the
 * frame source of RMSF.py:56,92,124 (GRO/XTC input, RMSF.py:34).  Published
 * xdrfile format (magic 1995, xdr3dfcoord compression).  Positions are in
 * Angstrom, rounded as MDAnalysis does: f32(f32(int * f32(1/prec)) * 10).
 * Host-only code: no HIP calls.                                             */
int rmsf_xtc_open(const char *path, rmsf_xtc **out, int64_t *n_atoms,
                  int64_t *n_frames);
int rmsf_xtc_close(rmsf_xtc *x);
int rmsf_xtc_frame_info(const rmsf_xtc *x, int64_t frame, int32_t *step,
                        float *time, float *box9);
/* Decode frames f0, f0+step, ... (n) into h_out[n][rows][3] (rows = n_sel
 * when h_sel != NULL, else n_atoms), frame-parallel on n_threads threads. */
int rmsf_xtc_read(const rmsf_xtc *x, int64_t f0, int64_t n, int64_t step,
                  const int32_t *h_sel, int64_t n_sel, float *h_out,
                  int n_threads);
/* Write (append != 0: append) n_frames frames given in Angstrom. */
int rmsf_xtc_write(const char *path, const float *h_xyz, int64_t n_frames,
                   int64_t n_atoms, float precision, const float *h_box9,
                   int append);
/* Byte offset (a multiple of 4) and length of frame f's XDR record. */
int rmsf_xtc_frame_record(const rmsf_xtc *x, int64_t frame, int64_t *offset,
                          int64_t *bytes);

/* ---- XTC decompression on the GPU (config C5) -------------------------------
 * The same decoder on the device: the compressed frame records (about 1/6
 * of the decoded bytes) are read into a pinned slot (pread, n_threads host
 * threads), copied to HBM on the slot's own stream and decompressed there,
 * one wave per frame (the xdr3dfcoord stream of a frame is sequential;
 * frames run in parallel), into float32 [n][n_atoms][3] Angstrom frames,
 * bit-identical to rmsf_xtc_read().  The selection is applied downstream
 * (rmsf_accumulate / rmsf_superpose gather it in-kernel).  Replaces the
 * libxdrfile decode behind trajectory[frame] (RMSF.py:92,124).           */
typedef struct rmsf_xtcdec rmsf_xtcdec;
int rmsf_xtcdec_create(const rmsf_xtc *x, int64_t batch_frames, int n_slots,
                       int n_threads, rmsf_xtcdec **out);
int rmsf_xtcdec_destroy(rmsf_xtcdec *d);
/* Decode frames f0, f0+step, ... (n_frames <= batch_frames) into the next
 * slot; *d_frames = its device frames (frame stride 3*n_atoms floats).
 * consumer_stream waits for the decode.  Per-frame errors (corrupt data:
 * the frame is filled with NaN) are reported when the slot is next used or
 * by rmsf_xtcdec_synchronize().                                             */
int rmsf_xtcdec_decode(rmsf_xtcdec *d, int64_t f0, int64_t n_frames,
                       int64_t step, void *consumer_stream, int *slot,
                       float **d_frames);
/* Decode the n_frames frames h_frames[0..n) (any order, repeats allowed;
 * n_frames <= batch_frames) into the next slot, frame k of the list at
 * *d_frames + k*3*n_atoms: a run(frames=...) list of scattered frames costs
 * one batched read + decode instead of one per frame.                      */
int rmsf_xtcdec_decode_list(rmsf_xtcdec *d, const int64_t *h_frames,
                            int64_t n_frames, void *consumer_stream, int *slot,
                            float **d_frames);
/* The same into the caller's device buffer: frame k of the batch at
 * d_out + k*out_stride floats (e.g. a trajectory kept resident in HBM). */
int rmsf_xtcdec_decode_into(rmsf_xtcdec *d, int64_t f0, int64_t n_frames,
                            int64_t step, float *d_out, int64_t out_stride,
                            void *consumer_stream, int *slot);
/* The slot may be reused once the work queued so far on consumer_stream ends. */
int rmsf_xtcdec_release(rmsf_xtcdec *d, int slot, void *consumer_stream);
/* Wait for every outstanding decode; first per-frame error, if any. */
int rmsf_xtcdec_synchronize(rmsf_xtcdec *d);
/* Kernel level: decode n_frames XDR frame records (each starting at its
 * magic word) held in device memory at 32-bit word offsets d_rec_off with
 * lengths d_rec_len (words); d_status[f] = 0 or a per-frame error code.   */
int rmsf_xtc_decode_records(const void *d_records, const int64_t *d_rec_off,
                            const int64_t *d_rec_len, int64_t n_frames,
                            int64_t n_atoms, float *d_out, int64_t out_stride,
                            int32_t *d_status, void *stream);
/* The device decoder's code run on the host (tests; no HIP calls). */
int rmsf_xtc_decode_records_host(const void *h_records,
                                 const int64_t *h_rec_off,
                                 const int64_t *h_rec_len, int64_t n_frames,
                                 int64_t n_atoms, float *h_out,
                                 int64_t out_stride, int32_t *h_status);

/* ---- RMSF context: the whole per-rank loop behind one opaque handle -------
 * SURVEY.md 8(b)'s minimal export set, for hosts that bring neither torch
 * nor their own device allocator (a C/C++ program, an MPI code, ctypes).
 * A context owns, on one device: the selection and masses, the centred
 * reference, the running Welford (n, mean, M2) and sweep-1 sum partials,
 * workspaces, a host stager and a non-blocking stream.  Calls on one context
 * are not re-entrant; different contexts may be driven from different host
 * threads.  Every call makes the context's device current for its duration
 * and restores the caller's device.  Work is asynchronous on the context
 * stream; rmsf_get_* synchronise.
 *
 * RMSF.py's per-rank loop (RMSF.py:80-146) in these terms:
 *   rmsf_ctx_create(dev, n_atoms, n_sel, ca_indices, masses, 0, &c);
 *   rmsf_set_reference_frame(c, frame0, is_dev);            RMSF.py:80-87
 *   rmsf_push_frames(c, block, n, 0, RMSF_PUSH_ALIGN_SUM, is_dev);  :89-105
 *   rmsf_multi_allreduce_sum(&c, 1)   (or the callback form)  :107-110
 *   rmsf_set_reference_average(c);                           :111-118
 *   rmsf_push_frames(c, block, n, 0, RMSF_PUSH_ALIGN_WELFORD, is_dev); :120-138
 *   rmsf_multi_chan_merge(&c, 1)      (or the callback form)  :140-143
 *   rmsf_get_rmsf(c, h_rmsf);                                 :145-146    */
typedef struct rmsf_ctx rmsf_ctx;

/* push modes for rmsf_push_frames() / rmsf_push_xtc() */
#define RMSF_PUSH_WELFORD 0       /* Welford on the raw frames (rms.RMSF)     */
#define RMSF_PUSH_ALIGN_SUM 1     /* superpose, f64 sum      (RMSF.py:91-105) */
#define RMSF_PUSH_ALIGN_WELFORD 2 /* superpose, Welford      (RMSF.py:123-138)*/
#define RMSF_PUSH_SUM 3           /* f64 sum of the raw frames                */
/* RMSF.py:137-138 as written on the raw frames (rmsf_welford_sequential):
 * the running Welford state continued frame by frame with the reference's
 * own arithmetic, so rmsf_get_partial returns a rank's S of RMSF.py:140 bit
 * for bit.  rmsf_multi_chan_merge_exact reduces such contexts with
 * second_order_moments in comm.reduce's order (RMSF_MERGE_MPI4PY), device to
 * device: the script's result bit for bit.  (rmsf_multi_chan_merge combines
 * them too, to rounding.)                                                   */
#define RMSF_PUSH_EXACT 4

/* h_sel: n_sel int64 atom indices (MDAnalysis AtomGroup.indices; copied),
 * NULL = atoms 0..n_sel-1.  h_masses: n_sel f64 (copied) or NULL = uniform
 * (RMSF.py:84 center_of_mass).  flags must be 0.      */
int rmsf_ctx_create(int device, int64_t n_atoms, int64_t n_sel,
                    const int64_t *h_sel, const double *h_masses, int flags,
                    rmsf_ctx **out);
int rmsf_ctx_destroy(rmsf_ctx *ctx);
/* the context's hipStream_t (order producer work of device frames on it) */
int rmsf_ctx_stream(rmsf_ctx *ctx, void **stream);
int rmsf_ctx_synchronize(rmsf_ctx *ctx);
/* Host-frame staging: frames per pinned slot (<= 0: ~64 MiB worth), slots
 * (>= 1) and gather threads.  Takes effect at the next host push.           */
int rmsf_ctx_set_staging(rmsf_ctx *ctx, int64_t batch_frames, int n_slots,
                         int n_threads);
/* Measurement: with timing on, every superpose and accumulate launch the
 * context makes is bracketed by HIP events on its stream.
 * rmsf_ctx_kernel_time() synchronises and returns, for one kernel family,
 * the number of launches, their summed duration (ms) and the atom-frames
 * they processed (x 12 B = algorithmic bytes), then clears
 * that family's record.  Note: a push recorded for atom slabs
 * (rmsf_multi_push_frames with merge_slabs > 1) is run whole before the
 * timings are read, so reading them between that push and
 * rmsf_multi_chan_merge_root makes the merge take its non-overlapped form
 * (same bits; only the slab overlap is lost).  Read timings after the
 * merge to keep the overlap.                                                 */
#define RMSF_TIME_ACCUMULATE 0 /* rmsf_accumulate_balanced (RMSF.py:99-103,133-138) */
#define RMSF_TIME_SUPERPOSE 1  /* rmsf_superpose (RMSF.py:94-97 + qcprot, :43-51)  */
/* the cross-context merge, per context: from its packed moments to its
 * finished result on its stream (collective, waits for the slowest context,
 * unpack/finalise; with atom slabs the part after the last slab's pack);
 * atom_frames = 0                                                           */
#define RMSF_TIME_MERGE 2
int rmsf_ctx_set_timing(rmsf_ctx *ctx, int on);
int rmsf_ctx_kernel_time(rmsf_ctx *ctx, int which, int64_t *launches,
                         double *ms, double *atom_frames);
/* Per-frame QCP rmsd (the value RMSF.py:48 discards; AlignTraj's
 * results.rmsd): with collection on, every RMSF_PUSH_ALIGN_WELFORD push
 * appends its frames' rmsd, in push order, to a device list the context
 * keeps (cleared by turning collection on and by rmsf_ctx_reset(what & 1)).
 * rmsf_get_rmsd synchronises; *n = frames collected, h_rmsd (capacity
 * doubles, may be NULL to query n) receives them.                          */
int rmsf_ctx_collect_rmsd(rmsf_ctx *ctx, int on);
int rmsf_get_rmsd(rmsf_ctx *ctx, int64_t *n, double *h_rmsd, int64_t capacity);
/* Zero the running Welford (what & 1) and/or sweep-1 sum (what & 2) state. */
int rmsf_ctx_reset(rmsf_ctx *ctx, int what);

/* Reference given directly: h_ref_centered f64 [n_sel][3], h_ref_com f64[3]
 * (RMSF.py:85-86 ref_ca / ref_com).                                         */
int rmsf_set_reference(rmsf_ctx *ctx, const double *h_ref_centered,
                       const double *h_ref_com);
/* Reference from a float32 frame of n_atoms atoms (RMSF.py:80-87). */
int rmsf_set_reference_frame(rmsf_ctx *ctx, const float *xyz,
                             int is_device_ptr);
/* Reference = the context's sweep-1 average sum/n (RMSF.py:111-118);
 * RMSF_EEMPTY when no frame was summed.                                      */
int rmsf_set_reference_average(rmsf_ctx *ctx);

/* exact=True for the context (RMSF.py:80-146 with the reference's own
 * summation orders, the sequential entry points above): with on != 0 the
 * reference setters run rmsf_reference_setup_sequential, RMSF_PUSH_ALIGN_SUM
 * / RMSF_PUSH_ALIGN_WELFORD run rmsf_superpose_sequential +
 * rmsf_accumulate_sequential (RMSF_PUSH_WELFORD the sequential Welford, as
 * RMSF_PUSH_EXACT), and rmsf_multi_allreduce_sum over contexts of this
 * process adds the sums in rank order.  mass_total = numpy's masses.sum()
 * of the selection (pairwise; n_sel for unit masses), the centre of mass's
 * divisor.  Set it before the reference (an earlier reference is refused by
 * the aligned pushes); merge the Welford states with
 * rmsf_multi_chan_merge_exact.                                              */
int rmsf_ctx_set_exact(rmsf_ctx *ctx, int on, double mass_total);

/* Push n_frames float32 frames of n_atoms atoms (frame_stride floats apart,
 * 0 = 3*n_atoms; a multiple of it implements `step`).  is_device_ptr != 0:
 * the frames are in HBM and must stay valid and unmodified until the
 * context is synchronised; otherwise they are host memory, gathered to the
 * selection and streamed through the context's pinned stager (the host
 * buffer may be reused when the call returns).                               */
int rmsf_push_frames(rmsf_ctx *ctx, const float *xyz, int64_t n_frames,
                     int64_t frame_stride, int mode, int is_device_ptr);
/* Push XTC frames f0, f0+step, ... (n_frames) of an open file (RMSF.py:92,124
 * frame source): the compressed records are decompressed on the GPU (the
 * context keeps an rmsf_xtcdec for the file, up to 3 batches in flight).
 * Synchronises at the end to report corrupt frames.                          */
int rmsf_push_xtc(rmsf_ctx *ctx, const rmsf_xtc *x, int64_t f0,
                  int64_t n_frames, int64_t step, int mode);

/* Push the XTC frames h_frames[0..n) (a frame list, e.g. run(frames=...)):
 * decoded on the GPU in batches of scattered records, one wait at the end. */
int rmsf_push_xtc_frames(rmsf_ctx *ctx, const rmsf_xtc *x, const int64_t *h_frames,
                         int64_t n_frames, int mode);
/* Push n_frames host frames given as one pointer per frame (n_atoms float32
 * atoms each; e.g. the rows of a frame list, or per-Timestep buffers): the
 * stager gathers the selection from every frame into its pinned slots.      */
int rmsf_push_frame_ptrs(rmsf_ctx *ctx, const float *const *h_ptrs,
                         int64_t n_frames, int mode);
/* The same for host frames stored as coordinate planes (SoA; see
 * rmsf_stager_stage_planes): x, y, z of frame f at h_ptrs[f] + {0, 1, 2} *
 * plane_stride floats.                                                      */
int rmsf_push_frame_planes(rmsf_ctx *ctx, const float *const *h_ptrs,
                           int64_t plane_stride, int64_t n_frames, int mode);

/* Running Welford partial (RMSF.py:120-121,137-138): *n frames, mean and M2
 * f64 [n_sel][3] (any output may be NULL).  Synchronises.                    */
int rmsf_get_partial(rmsf_ctx *ctx, int64_t *n, double *h_mean, double *h_m2);
/* Sweep-1 sum (RMSF.py:103,105): *n frames and f64 [n_sel][3]. */
int rmsf_get_sum(rmsf_ctx *ctx, int64_t *n, double *h_sum);
/* Average structure sum/n (RMSF.py:111; AverageStructure.results.positions). */
int rmsf_get_average(rmsf_ctx *ctx, double *h_avg);
/* rmsf = sqrt(M2.sum(axis=1)/n) (RMSF.py:146), f64 [n_sel]. */
int rmsf_get_rmsf(rmsf_ctx *ctx, double *h_rmsf);
/* Replace the running Welford state (checkpoint restore / external merge). */
int rmsf_set_partial(rmsf_ctx *ctx, int64_t n, const double *h_mean,
                     const double *h_m2);

/* ---- cross-rank exchange (RMSF.py:107-110 all-reduce, :140-143 reduce) -----
 * Each exchange leaves the GLOBAL result in every participating context:
 *   allreduce_sum: sweep-1 sum and frame count summed over ranks;
 *   chan_merge:    exact k-way Chan of the Welford partials, as three
 *                  all-reduce(SUM) steps -- n, sum w_k mean_k (w_k=n_k/n),
 *                  sum M2_k + n_k (mean_k - mean)^2.  Empty ranks contribute
 *                  nothing; RMSF_EEMPTY if n == 0.
 * Three transports, the same arithmetic:
 *   (1) a caller callback -- fn sums the device buffer d_buf[0..count) in
 *       place over all ranks (MPI, gloo, ...) and returns 0.  d_buf is
 *       produced by work queued on `stream` (the context's): fn orders its
 *       reduction after it (enqueues on `stream`, or synchronises it first),
 *       and the sum is complete when fn returns or is queued on `stream`;
 *   (2) RCCL communicators (rmsf_multi_init / rmsf_multi_init_all);
 *   (3) neither: the n contexts of this process are reduced among themselves
 *       on the host, in context order (one process, any devices).          */
typedef int (*rmsf_allreduce_fn)(double *d_buf, int64_t count, void *stream,
                                 void *user);
int rmsf_ctx_allreduce_sum(rmsf_ctx *ctx, rmsf_allreduce_fn fn, void *user);
int rmsf_ctx_chan_merge(rmsf_ctx *ctx, rmsf_allreduce_fn fn, void *user);
/* The same merge with ONE data all-reduce (2*3*n_sel doubles, plus the
 * frame-count exchange): moments about the context's reference structure
 * (rmsf_chan_shift_pack / _finish).  Precondition, as in RMSF.py: every rank
 * holds the SAME reference (rmsf_ctx_set_reference_frame on the same frame,
 * or rmsf_ctx_set_reference_average after rmsf_ctx_allreduce_sum); every rank
 * must call this form (the buffer sizes differ from the two-pass form).
 * rmsf_multi_chan_merge uses it by itself when all ranks are contexts of the
 * calling process and each holds a reference.                              */
int rmsf_ctx_chan_merge_shifted(rmsf_ctx *ctx, rmsf_allreduce_fn fn, void *user);

/* RCCL (librccl.so.1, loaded on first use).  One process per GPU:
 * rank 0 calls rmsf_multi_unique_id, the host broadcasts the 128 bytes, each
 * rank calls rmsf_multi_init.  One process, many GPUs: rmsf_multi_init_all
 * (ncclCommInitAll over the contexts' devices).                              */
#define RMSF_UNIQUE_ID_BYTES 128
int rmsf_multi_unique_id(void *id_out);
int rmsf_multi_init(rmsf_ctx *ctx, const void *id, int nranks, int rank);
int rmsf_multi_init_all(rmsf_ctx **ctxs, int n);
int rmsf_multi_allreduce_sum(rmsf_ctx **ctxs, int n);
int rmsf_multi_chan_merge(rmsf_ctx **ctxs, int n);

/* ---- one process, several contexts: the torchrun rank step's shape --------
 * The merge's shift for UNALIGNED Welford state (RMSF.py:141-143 as one
 * collective of moments about a shift every rank holds; aligned state uses
 * the reference): frame 0 of the frame list, n_atoms float32 atoms, host or
 * device pointer; the context keeps its selected rows (f32) and a digest.
 * rmsf_multi_chan_merge[_root] merges unaligned contexts in one collective
 * when all hold the same shift frame, else in the two-pass form.           */
int rmsf_set_merge_shift_frame(rmsf_ctx *ctx, const float *xyz,
                               int is_device_ptr);
/* rmsf_multi_chan_merge with RMSF.py:143's shape: root >= 0 reduces the
 * moments to context `root` only (half the link bytes of an all-reduce);
 * the other contexts then refuse rmsf_get_rmsf / rmsf_get_partial with
 * RMSF_EINVAL until they are reset.  root = -1: every context gets the
 * result (rmsf_multi_chan_merge).  Only the one-collective (shifted) merge
 * can reduce to a root; the two-pass form leaves the result everywhere.
 * Replaces RMSF.py:140-143 (comm.Barrier + comm.reduce(root=0)).           */
int rmsf_multi_chan_merge_root(rmsf_ctx **ctxs, int n, int root);
/* RMSF.py:141-143 as the script computes it: the contexts' Welford states
 * (each a rank's S of RMSF.py:140, context i = rank i) reduced with
 * second_order_moments in `order` (RMSF_MERGE_MPI4PY: comm.reduce's
 * binomial tree; RMSF_MERGE_RANK: rank order) -- each step copies the
 * source context's state to the destination's device (peer copy over xGMI,
 * or a device copy) and merges it there (rmsf_chan_merge_pair), the steps of
 * one tree level on their own streams at once.  The result is context 0's,
 * then forwarded to `root` (the others refuse getters with RMSF_EINVAL until
 * reset) or, root = -1, to every context.  Bit for bit with RMSF.py:143 on
 * RMSF_PUSH_EXACT states.  Contexts of this process only (a communicator
 * spanning processes: RMSF_EINVAL).                                        */
int rmsf_multi_chan_merge_exact(rmsf_ctx **ctxs, int n, int root, int order);
/* Push each context's HBM frames d_frames[i] (n_frames[i] frames,
 * frame_stride floats apart, 0 = 3*n_atoms) in `mode`, the n contexts'
 * launches enqueued from one host thread per device (asynchronous: the
 * frames must stay valid until the contexts are synchronised).  Per context,
 * first: flags & RMSF_MULTI_RESET resets the state `mode` accumulates into;
 * d_ref_frames[i] (device frame, may be NULL) sets the reference
 * (rmsf_set_reference_frame); d_shift_frames[i] the merge shift frame.
 * merge_slabs (unaligned Welford, no selection, one launch group whose flat
 * plan is chunk-aligned, a shift frame set, fresh state): 0 = auto (2 slabs
 * from 1M atoms, as the torchrun pipeline), 1 = off, k >= 2 = k slabs -- the
 * push is then recorded, and the next rmsf_multi_chan_merge_root streams it
 * slab by slab with each slab's collective (on a communicator stream, RCCL)
 * beside the next slab's accumulate; any other call runs it whole.          */
#define RMSF_MULTI_RESET 1
int rmsf_multi_push_frames(rmsf_ctx **ctxs, int n, const float *const *d_frames,
                           const int64_t *n_frames, int64_t frame_stride,
                           int mode, int flags, const float *const *d_ref_frames,
                           const float *const *d_shift_frames, int merge_slabs);
/* Transport of the contexts' exchanges: AUTO = RCCL when every context has a
 * communicator, else the in-process host fold; NOOP = a timing rehearsal of
 * N contexts on fewer devices -- the exchanges move no data, so the merged
 * statistics are NOT the global ones (measurement only).                    */
#define RMSF_TRANSPORT_AUTO 0
#define RMSF_TRANSPORT_NOOP 1
int rmsf_multi_set_transport(rmsf_ctx **ctxs, int n, int transport);

#ifdef __cplusplus
}
#endif
#endif /* RMSF_HIP_H */
