/*
 * brd.h -- C ABI of the MI355X-native two-stage bidiagonal reduction
 * (libbrd_hip.so, built from svdsolver_amd/csrc/).
 *
 * Plain pointers and sizes; no exceptions, no C++ or torch types cross this
 * boundary.  Every entry point returns BRD_OK (0) or a negative brd_status;
 * brd_last_error() gives a human-readable message for the calling thread.
 *
 * Storage: row-major (the layout of csc586::gpu::Matrix<T>::flatten(),
 * matrix_gpu.h:223), element (i,j) at A[i*lda + j].
 *
 * Which reference interface each entry point replaces:
 *   brd_ge2band_*   csc586::gpu::cuda_brd_p1(Matrix<float>& A, size_t b)
 *                   (reference svd_cuda_2.cu:1117; svd_cuda_1.cu:750) and the
 *                   CPU csc586::parallel::brd_p1<T>(Matrix<T>&, size_t)
 *                   (svd_parallel.h:411).  Dense N x N -> upper band with b
 *                   super-diagonals, in place.  Unlike the reference GPU path
 *                   it is not fp32-only.
 *   brd_band2bd_*   csc586::parallel::brd_p2<T>(Matrix<T>&, size_t b)
 *                   (svd_parallel.h:640; twin gpu::brd_p2, svd_cpu.h:631) --
 *                   band -> bidiagonal, in place, returning d and e like the
 *                   reference's Bidiagonal{d, e} (svd_parallel.h:691).
 *   brd_dist_*,     new (the reference has no multi-GPU path):
 *   brd_ge2band_dist_*  block-cyclic column-sharded stage 1 over RCCL / xGMI.
 */
#ifndef BRD_H_
#define BRD_H_

#ifdef __cplusplus
extern "C" {
#endif

enum brd_status {
    BRD_OK = 0,
    BRD_EINVAL = -1,      /* bad argument (sizes, band width, null pointer)        */
    BRD_EHIP = -2,        /* HIP runtime error (message in brd_last_error)         */
    BRD_ENOMEM = -3,      /* device allocation failed                              */
    BRD_ERCCL = -4,       /* RCCL error                                            */
    BRD_EUNSUPPORTED = -5 /* valid request this build does not implement           */
};

/* flags */
#define BRD_DEVICE_PTR 0x1u   /* A, d, e are device pointers (else host; staged)   */
#define BRD_ASYNC      0x2u   /* device pointers only: return without syncing      */
#define BRD_COMPAT     0x0u   /* stage 2: the reference's window geometry (default)*/
#define BRD_EXACT_ORDER 0x4u  /* stage 2 compat, evaluated in the reference's exact
                                 operation order (bit-identical to the reference's
                                 CPU code; slow, for verification)                 */
#define BRD_NO_EXTRACT 0x8u   /* stage 2: do not write d/e (may pass NULL)         */
#define BRD_SIGMA      0x10u  /* stage 2: sigma-preserving geometry -- the reference's
                                 windows plus the final window pair each sweep
                                 needs, so the result is orthogonally equivalent
                                 to the band (not in the reference; combines
                                 with BRD_EXACT_ORDER)                            */

/* Stage 1: dense m x n (m >= n) -> upper band, bandwidth b (1 <= b <= 32).
 * On return A holds the band matrix: entries (i,j) with 0 <= j-i <= b, and
 * exact zeros elsewhere.  ngpus must be 1 (multi-GPU: brd_ge2band_dist_*). */
int brd_ge2band_f64(double *A, int m, int n, int lda, int b, int ngpus, unsigned flags);
int brd_ge2band_f32(float *A, int m, int n, int lda, int b, int ngpus, unsigned flags);

/* Stage 2: n x n band (bandwidth b) -> bidiagonal, in place, with the
 * reference's window geometry (BRD_COMPAT) or the sigma-preserving one
 * (BRD_SIGMA).  d (n) and e (n-1) receive the diagonal and super-diagonal
 * (same memory kind as A; e may be NULL when n = 1). */
int brd_band2bd_f64(double *A, int n, int lda, int b, double *d, double *e, unsigned flags);
int brd_band2bd_f32(float *A, int n, int lda, int b, float *d, float *e, unsigned flags);

/* Singular values of the upper bidiagonal (d (n), e (n-1)), host memory, in
 * descending order into sv (n): Golub-Kahan QR with Wilkinson shifts, values
 * only (replaces the reference's serial::qrd, svd_serial.h:368).  After
 * brd_band2bd_* with BRD_SIGMA these are the singular values of the matrix
 * stage 1 started from. */
int brd_bdsvd_f64(const double *d, const double *e, int n, double *sv);
int brd_bdsvd_f32(const float *d, const float *e, int n, float *sv);

/* The same on the GPU: d (n), e (n-1) and sv (n) are DEVICE pointers; the
 * values (descending) are bracketed by multisection on the Golub-Kahan
 * tridiagonal (every value independently, G lanes each), to the host QR's
 * accuracy (|sigma_i - exact| ~ eps sigma_max).  Runs on the library stream;
 * BRD_ASYNC returns without waiting.  e may be NULL when n = 1. */
int brd_bdsvd_dev_f64(const double *d, const double *e, int n, double *sv, unsigned flags);
int brd_bdsvd_dev_f32(const float *d, const float *e, int n, float *sv, unsigned flags);

/* Stream used by subsequent calls (hipStream_t; NULL = the legacy default
 * stream).  Until the first call the library uses a stream of its own;
 * brd_use_own_stream() reverts to it. */
int brd_set_stream(void *hip_stream);
int brd_use_own_stream(void);

/* Two reductions side by side (a stream of matrices): stage 2 of matrix i on
 * one stream while stage 1 of matrix i+1 runs on another.  s2_cus > 0 runs
 * every stage-2 sweep on that many workgroups (one per CU; the bundle chain
 * keeps fewer than ~64 busy at N <= 16384) and sizes stage-1 launches for the
 * remaining CUs; 0 restores the defaults (each stage on the whole chip).
 * No reference counterpart (the reference runs one reduction at a time,
 * svd_cuda_2.cu:1387 / timing.h:55). */
int brd_set_overlap(int s2_cus);   /* 0 <= s2_cus < device CUs, else BRD_EINVAL */

/* Drains every stream the library has launched on and reports failures of
 * asynchronous (BRD_ASYNC) calls: a stage-2 sweep whose bounded spin gave up
 * (its output is then invalid) or a pending HIP error.  The stage-2 error
 * word of a stream is sticky: no launch resets it; a synchronous band2bd on
 * that stream or this call reads and clears it.  Call it after a batch of
 * asynchronous work before trusting the results. */
int brd_check_errors(void);

/* Drain hip_stream (NULL: the library's current stream) and free the
 * library's per-stream state for it: stage-1/stage-2 workspaces, the cached
 * HBM staging buffer of host-pointer calls, the stage-2 error word (read
 * first: BRD_EHIP if it was set).  brd_check_errors() visits every stream the
 * library has launched on, so call this before destroying such a stream.
 * Host-pointer calls keep their staging buffer until then (with
 * BRD_STAGE_KEEP_MB set, one larger than that many MiB is freed on return). */
int brd_release_stream(void *hip_stream);

/* Per-kernel device timing for roofline reporting.  While enabled, the library
 * brackets every launch of the named kernel class with HIP events on the
 * launch stream.  kernel: "s1_apply", "s1_factor", "s2_sweep".  Returns the
 * number of launches, their total device time in ms and the algorithmic flops
 * and bytes those launches were credited with. */
int brd_profile_enable(int enable);
int brd_profile_reset(void);
int brd_profile_query(const char *kernel, long long *launches, double *total_ms,
                      double *flops, double *bytes);

/* ---- Multi-GPU stage 1 (one process per GPU) ------------------------------
 * Layout: 1-D block-cyclic over column panels of width b -- global panel p
 * (columns [p b, p b + b)) lives on rank p mod P as local panel p / P.  A
 * rank's shard is m x n_loc (n_loc = brd_dist_local_cols), row-major with
 * leading dimension lda_loc, in device memory.  The stage-2 input is
 * assembled on one rank with brd_dist_gather_band.
 * Collectives go to RCCL over xGMI (brd_dist_init, with an id from
 * brd_dist_unique_id on one rank, shared out of band) or to a host callback
 * (brd_dist_init_host: the library drains its stream, then calls fn, which
 * must complete the collective on the device buffers before returning).
 * A communicator belongs to the library stream current at its init
 * (brd_set_stream); the first one is also the default for streams without
 * their own.  Calls on a stream use that stream's communicator and a
 * workspace of that stream, so several matrices' distributed reductions can
 * run at once, one stream (and communicator) each; every rank must issue a
 * communicator's calls in the same order.  brd_dist_finalize releases all. */
enum brd_coll_op {
    BRD_COLL_BCAST = 0,         /* recv (== send) broadcast from root, count elems */
    BRD_COLL_ALLGATHER = 1,     /* send: count elems; recv: count * nranks elems    */
    BRD_COLL_ALLREDUCE_SUM = 2  /* in place (send == recv), count elems             */
};
enum brd_dtype { BRD_DT_BYTE = 0, BRD_DT_F32 = 1, BRD_DT_F64 = 2 };
typedef int (*brd_coll_fn)(int op, const void *send, void *recv, unsigned long count, int dtype, int root,
                           void *user);

int brd_dist_unique_id(void *id_out, int id_bytes);      /* id_bytes >= 128 */
int brd_dist_init(int rank, int nranks, const void *id, int id_bytes);
int brd_dist_init_host(int rank, int nranks, brd_coll_fn fn, void *user);
int brd_dist_finalize(void);
int brd_dist_local_cols(int n, int b, int nranks, int rank);   /* n_loc of a rank (>= 0) */
/* Stage 1 on the sharded matrix (every rank calls; BRD_DEVICE_PTR required). */
int brd_ge2band_dist_f64(double *A_loc, int m, int n, int lda_loc, int b, unsigned flags);
int brd_ge2band_dist_f32(float *A_loc, int m, int n, int lda_loc, int b, unsigned flags);
/* Assemble the band (diagonals 0..b) on rank root into the dense m x n matrix
 * B (device, ldb >= n; zero outside the band).  B is ignored on other ranks. */
int brd_dist_gather_band_f64(const double *A_loc, int m, int n, int lda_loc, int b, double *B, int ldb, int root,
                             unsigned flags);
int brd_dist_gather_band_f32(const float *A_loc, int m, int n, int lda_loc, int b, float *B, int ldb, int root,
                             unsigned flags);

const char *brd_last_error(void);
int brd_version(void);

#ifdef __cplusplus
}
#endif

#endif /* BRD_H_ */
