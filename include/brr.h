/*
 * brr.h -- C ABI of the MI355X BayesR / BayesRR / Horseshoe Gibbs sampler (libbrr.so).
 *
 * Drop-in boundary: the four one-shot entry points take exactly the arguments of the
 * reference's Rcpp-exported C++ functions (plain pointers + sizes instead of Eigen/Rcpp
 * types) and produce the same output file.  A maintainer binds them from the Rcpp glue
 * (r_shim/RcppExports.cpp) in place of the reference bodies:
 *
 *   brr_BayesRSamplerV2        replaces BayesRSamplerV2        src/BayesRv2.cpp:60
 *                                       (.Call glue src/RcppExports.cpp:39-59)
 *   brr_BayesRSamplerV2Groups  replaces BayesRSamplerV2Groups  src/BayesRv2Groups.cpp:75
 *                                       (.Call glue src/RcppExports.cpp:61-84)
 *   brr_BRV2Grstart            replaces BRV2Grstart            src/BRv2Grstart.cpp:77
 *                                       (.Call glue src/RcppExports.cpp:10-37)
 *   brr_HorseshoeR             replaces HorseshoeR             src/HorseshoeR.cpp:109
 *                                       (.Call glue src/RcppExports.cpp:86-108)
 *
 * Matrices are column-major with leading dimension = rows (R's storage), borrowed and
 * read-only; the library never copies X on the host (it uploads once, f64 -> f32).
 *
 * Return codes: 0 ok; 1 validation abort with the reference's semantics (message through
 * the log callback, file left as the reference leaves it); < 0 device / IO / argument error
 * (message through the log callback and brr_last_error()).  No C++ exception crosses the ABI.
 *
 * The session API underneath (brr_session_*) is what the one-shot calls, tests and the
 * benchmark use: device-resident data, explicit sweeps, state read-back and the
 * column-sharded multi-GPU protocol (one process per GPU, E residual exchanges per sweep).
 */
#ifndef BRR_H
#define BRR_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BRR_ABI_VERSION 4

enum brr_model { BRR_MODEL_V2 = 0, BRR_MODEL_GROUPS = 1, BRR_MODEL_RESTART = 2, BRR_MODEL_HORSESHOE = 3 };

/* Visit order of the markers within a sweep.
 *  BLOCKED   (default) fixed column blocks of size block_size; block order and the order
 *            inside each block are Philox permutations redrawn every sweep.  Block Gram
 *            matrices are computed once, so this is the fast path.
 *  REFERENCE the reference's own order: libstdc++ std::random_shuffle driven by glibc
 *            rand() from a fresh-process state (BayesRv2.cpp:182), persisting across
 *            sweeps; Gram blocks are recomputed every sweep (slow; for parity / replay).
 *            Column shards shuffle the permutation of all M_total markers and visit their own
 *            columns in its order; row shards visit every marker in it.
 *  IDENTITY  markers 0..P-1 in index order every sweep (debugging). */
enum brr_order { BRR_ORDER_BLOCKED = 0, BRR_ORDER_REFERENCE = 1, BRR_ORDER_IDENTITY = 2 };

/* Device storage of the genotype matrix (no reference counterpart: the reference
 * keeps a dense f64 Eigen copy, src/BayesRv2.cpp:60).
 *  F32   dense f32 column-major: any matrix (4 N M bytes, streamed once per sweep).
 *  2BIT  2-bit codes + a 4-entry f32 value table per column (N M / 4 bytes): for genotype-coded
 *        columns (at most 3 distinct non-zero values, e.g. scale()d 0/1/2 dosages).  Decoded
 *        values equal the F32 storage's bit for bit, so a chain is identical under both. */
enum brr_x_storage { BRR_X_F32 = 0, BRR_X_2BIT = 1 };

typedef void (*brr_log_fn)(const char *msg, void *userdata);

typedef struct brr_options {
  int32_t abi_version;     /* BRR_ABI_VERSION */
  int32_t device;          /* HIP device ordinal (default 0) */
  int32_t block_size;      /* marker block B: 64, 128, 256 or 512; 0 (default) = automatic:
                              512 for V2 / restart, 128 for Groups and the Horseshoe */
  int32_t order_mode;      /* enum brr_order (default BLOCKED) */
  int32_t shard_rank;      /* column shard of this process (default 0) */
  int32_t shard_count;     /* number of column shards / processes (default 1) */
  int32_t verbose;         /* 1 = progress lines "iteration: i" like the reference */
  int32_t x_storage;       /* enum brr_x_storage (default F32) */
  brr_log_fn log;          /* NULL = stderr */
  void *log_userdata;
  /* exact row-sharded mode (ABI 2): this session holds rows
   * [row_offset, row_offset + N) of an N_total-row cohort and ALL markers; per marker block the
   * partial dots x_j . eps are summed across the row shards before the (replicated, identical)
   * block solve, so every shard runs the single-GPU chain exactly.  Exchanges go through RCCL
   * (brr_session_comm_init, one process per GPU) or an in-process brr_group. */
  int32_t row_shard_rank;  /* default 0 */
  int32_t row_shard_count; /* default 1 (no row sharding) */
  int64_t row_offset;      /* first global row of this shard */
  int64_t N_total;         /* rows of the whole cohort (0 = N) */
  /* column shards (ABI 3): residual exchanges per sweep E.  Each shard's block positions split into
   * E segments of whole blocks (segment e = blocks [nb e / E, nb (e + 1) / E)); after every segment
   * the residual deltas are summed across the shards, so a shard sees the other shards' changes at
   * most one segment late instead of one sweep (stale-residual bias).
   * 0 (default) = automatic: E = 8, capped at ceil(M_total / B) / shard_count -- a shard then sees
   * less than 1/8 of a sweep's changes of the others late, and the 8-shard chain matches the 1-shard
   * chain within Monte-Carlo error.  1 = north_star's single exchange per sweep (measurably biased
   * from 2 shards on).  Every shard must use the same E.
   * Ignored without column shards.
   * 0 is automatic for every abi_version (as ABI 3 documented it; ABI 1 / 2 structs have no such
   * field and get the default).  A caller that drives sweep_local / exchange / sweep_finish itself
   * queries brr_session_exchanges_per_sweep() and runs E rounds per sweep, as brr_session_sweep and
   * distributed.HostExchange do; E = 1 keeps one round per sweep. */
  int32_t exchanges_per_sweep;
} brr_options;

void brr_options_default(brr_options *opt);
/* the options the library uses for a caller's struct (defaults for a NULL pointer, the ABI-version
 * upgrade of an older struct applied) */
void brr_options_effective(const brr_options *in, brr_options *out);
const char *brr_last_error(void);
int brr_device_count(void);
/* free and total device memory of a HIP device in bytes (a caller sizing its shards; a session whose
 * buffers do not fit fails at brr_session_create with the sizes in brr_last_error()) */
int brr_device_memory(int32_t device, int64_t *free_bytes, int64_t *total_bytes);

/* ---------------- one-shot drop-in entry points (reference signatures) ---------------- */
int brr_BayesRSamplerV2(const char *outputFile, int seed, int max_iterations, int burn_in,
                        int thinning, const double *X, int64_t N, int64_t M, const double *Y,
                        double sigma0, double v0E, double s02E, double v0G, double s02G,
                        const double *cva, int32_t n_cva, const brr_options *opt);

int brr_BayesRSamplerV2Groups(const char *outputFile, int seed, int max_iterations, int burn_in,
                              int thinning, const double *X, int64_t N, int64_t M,
                              const double *Y, double sigma0, double v0E, double s02E,
                              double v0G, double s02G, const double *cva /* groups x n_cva */,
                              int32_t n_cva, int groups, const int32_t *gAssign /* M */,
                              const double *fixed /* N x F */, int64_t F,
                              const brr_options *opt);

int brr_BRV2Grstart(const char *outputFile, int seed, int max_iterations, int burn_in,
                    int thinning, double mu, const double *beta /* M */, double sigmaE,
                    const double *sigmaGG /* groups */, const double *X, int64_t N, int64_t M,
                    const double *epsilon /* N */, const double *components /* M */,
                    double sigma0, double v0E, double s02E, double v0G, double s02G,
                    const double *cva, int32_t n_cva, int groups, const int32_t *gAssign,
                    const brr_options *opt);

int brr_HorseshoeR(const char *outputFile, int seed, int max_iterations, int burn_in,
                   int thinning, const double *X, int64_t N, int64_t M, const double *Y,
                   double A, double v0E, double s02E, double vL, double vT, double c2,
                   double vC, double sC, const brr_options *opt);

/* ---------------- session API ---------------- */
typedef struct brr_session brr_session;

/* N rows; M = markers of THIS shard (columns of the X given to upload) ; M_total = all
 * markers; col_offset = global index of this shard's first marker (multiple of block_size
 * when shard_count > 1).  K = mixture components incl. zero (n_cva + 1; Horseshoe: 1). */
brr_session *brr_session_create(int32_t model, int64_t N, int64_t M, int64_t M_total,
                                int64_t col_offset, int32_t K, int32_t groups, int64_t F,
                                const brr_options *opt);
void brr_session_destroy(brr_session *s);

/* X: host column-major N x M (this shard), f64 or f32.  With x_storage = BRR_X_2BIT every
 * column must hold at most 3 distinct non-zero values (error otherwise). */
int brr_session_upload_x_f64(brr_session *s, const double *X, int64_t ldx);
int brr_session_upload_x_f32(brr_session *s, const float *X, int64_t ldx);
/* PLINK .bed body (SNP-major, without the 3 magic bytes) for this shard's M markers,
 * bytes_per_col >= ceil(N/4) bytes each: genotype = copies of allele 1 (00 -> 2, 10 -> 1, 11 -> 0,
 * 01 = missing), standardised per column as R's scale() after mean imputation; missing -> 0.
 * Either storage; with BRR_X_2BIT the codes are stored as they come (no decode on the host). */
int brr_session_upload_bed(brr_session *s, const uint8_t *bed, int64_t bytes_per_col);
/* On-device synthetic cohort (DESIGN.md "synthetic data spec"): standardised Binomial(2,f)
 * genotypes for this shard's global columns; Y = standardised X beta + noise computed over
 * all M_total columns' causal set.  Requires shard_count == 1 for Y (else use set_y). */
int brr_session_synthesize(brr_session *s, uint64_t data_seed, double h2, int64_t n_causal);
/* sharded synthetic Y: Y = scale(sum over shards of X_c beta_c + noise).  Each process reads
 * its shard's genetic values, the caller sums them across processes, then every process
 * calls brr_session_synth_y with the sum (identical Y everywhere).  Row shards: every shard
 * holds all markers, so its partial values are final for its rows; the caller concatenates them
 * in row order (N_total values) and every shard calls brr_session_synth_y with that vector (Y is
 * standardised over all N_total rows; each shard keeps its own rows). */
int brr_session_synth_partial_y(brr_session *s, double *out /* N */);
int brr_session_synth_y(brr_session *s, const double *genetic_sum /* N */, uint64_t data_seed,
                        double h2);
int brr_session_set_y(brr_session *s, const double *Y);
int brr_session_set_fixed(brr_session *s, const double *fixed /* N x F */);
int brr_session_set_bayesr(brr_session *s, double sigma0, double v0E, double s02E, double v0G,
                           double s02G, const double *cva /* groups x (K-1) col-major */,
                           const int32_t *gAssign /* M (this shard) or NULL */);
int brr_session_set_horseshoe(brr_session *s, double A, double v0E, double s02E, double vL,
                              double vT, double c2, double vC, double sC);
/* BRV2Grstart state (src/BRv2Grstart.cpp:77): beta/components for this shard's markers */
int brr_session_set_restart(brr_session *s, double mu, const double *beta, double sigmaE,
                            const double *sigmaGG, const double *epsilon,
                            const double *components);
/* optional override of the initial mixture proportions pi (groups x K, row-major) */
int brr_session_set_pi(brr_session *s, const double *pi);
/* reference init block (draws keyed by seed) + Gram precompute */
int brr_session_init(brr_session *s, int32_t seed);
/* n full sweeps on this device (shard_count must be 1, or an exchange callback set) */
int brr_session_sweep(brr_session *s, int32_t n);

/* column-sharded protocol, one process per GPU:
 *   brr_session_sweep_local(s)  -> mu, fixed effects, this shard's markers against the
 *                                  local residual; writes dEps (N doubles) and the partial
 *                                  statistics into the exchange buffers;
 *   caller all-reduces (sum) the exchange buffers across processes (RCCL / gloo);
 *   brr_session_sweep_finish(s) -> eps = eps_start + sum dEps, hyper-parameter draws
 *                                  (redundant and identical on every process).
 * With exchanges_per_sweep = E > 1 a sweep is E such rounds: local covers one segment of the
 * shard's blocks (mu and fixed effects in the first only, the statistics in the last only --
 * zeros before), finish sets eps = eps_segment_start + sum dEps and, after the last segment, draws
 * the hyper-parameters.  brr_session_exchanges_per_sweep() returns E.
 * Exchange buffers are device memory owned by the caller (e.g. torch tensors), sizes from
 * brr_session_exchange_sizes().  sweep_local returns after the device work (the exchange buffers
 * are complete) and, like brr_session_sweep, -3 with brr_last_error() when a device pipeline wait
 * timed out or the fused sweep could not be made resident (the sweep's later segments and sweeps
 * then use the per-block kernels; a caller of the protocol still takes part in that round's exchange
 * and may go on, or abort every rank together).  With a failed census the failed segment's markers
 * keep their values this sweep (the state stays consistent). */
int brr_session_exchange_sizes(brr_session *s, int64_t *n_eps, int64_t *n_stats);
int brr_session_set_exchange(brr_session *s, double *dev_eps, double *dev_stats);
/* session-owned exchange buffers (allocated on first use; the statistics directly follow the N
 * residual deltas, so brr_session_sweep's exchange is one all-reduce); host copies for gloo / tests:
 * dir 0 = device -> host, 1 = host -> device */
int brr_session_exchange_buffers(brr_session *s, double **dev_eps, double **dev_stats);
int brr_session_exchange_copy(brr_session *s, int32_t dir, double *host_eps, double *host_stats);
int brr_session_sweep_local(brr_session *s);
int brr_session_sweep_finish(brr_session *s);
int32_t brr_session_exchanges_per_sweep(brr_session *s);
/* the same split for init, needed by the restart model only (its pi init counts every
 * marker's component, src/BRv2Grstart.cpp:157-165): brr_session_init_local(s, seed) leaves
 * this shard's counts in the exchange statistics; the caller sums them across shards (as for a
 * sweep) and calls brr_session_init_finish(s).  For every other model init_local is a complete
 * init and init_finish a no-op.  With a communicator, brr_session_init does all of it. */
int brr_session_init_local(brr_session *s, int32_t seed);
int brr_session_init_finish(brr_session *s);

/* native multi-GPU: RCCL over xGMI, one process per GPU.  Rank 0 creates the 128-byte id,
 * the caller broadcasts it (MPI, a file, torch.distributed/gloo ...), every rank calls
 * brr_session_comm_init; brr_session_sweep then runs, E times per sweep, local segment ->
 * ncclAllReduce(sum) of the exchange buffers on the session stream (N + NS doubles after the last
 * segment, N before) -> finish, with no host round trip.
 * Row-sharded sessions (row_shard_count > 1) take nranks = row_shard_count, rank =
 * row_shard_rank and must call it BEFORE brr_session_init (the Gram blocks are summed there);
 * their sweeps then all-reduce B partial dots per marker block (exact chain). */
int brr_comm_unique_id(void *out /* 128 bytes */);
int brr_session_comm_init(brr_session *s, const void *unique_id, int32_t nranks, int32_t rank);

/* exact row shards in ONE process: the sessions (created with row_shard_rank
 * 0..n-1, same model / M / options, on one device or on peer-accessible devices) are driven in
 * lock step; the per-block partial dots, the residual sums, the fixed-effect dots and, at init,
 * the Gram blocks are summed across the members on the device (rank order) instead of by RCCL.
 * Setters (upload, set_y, set_bayesr ...) stay per session; init and sweeps go through the group.
 * The group borrows the sessions (destroy the group first). */
typedef struct brr_group brr_group;
brr_group *brr_group_create(brr_session *const *members, int32_t n);
int brr_group_init(brr_group *g, int32_t seed);
int brr_group_sweep(brr_group *g, int32_t n);
void brr_group_destroy(brr_group *g);

/* sample output for callers that drive sweeps themselves: the one-shots' pipeline
 * (a device snapshot per kept sweep, an asynchronous copy into a ring of ring_depth pinned host
 * slots, a writer thread formatting the reference's CSV row; the caller blocks only when the
 * writer is ring_depth rows behind).  model/N/M/groups/F select the reference's row and header
 * layout (header = 0: none, as BRV2Grstart).  close drains every queued row; max_rows_in_flight
 * (may be NULL) reports the most slots ever in use. */
int brr_session_output_open(brr_session *s, const char *path, int32_t model, int64_t N, int64_t M,
                            int32_t groups, int64_t F, int32_t header, int32_t ring_depth);
int brr_session_output_sample(brr_session *s, int32_t iteration);
int brr_session_output_close(brr_session *s, int32_t *max_rows_in_flight);

/* state read-back (host buffers) */
enum brr_scalar { BRR_MU = 0, BRR_SIGMAE, BRR_SIGMAG, BRR_SIGMAF, BRR_TAU, BRR_ETA, BRR_C2,
                  BRR_SUMSQ_BETA, BRR_N_SCALARS };
enum brr_vector { BRR_BETA = 0, BRR_COMP, BRR_EPS, BRR_SIGMAGG, BRR_PI, BRR_ALPHA, BRR_LAMBDA,
                  BRR_XSQ, BRR_ORDER, BRR_VCOUNT, BRR_BETAACUM, BRR_HSV };
int brr_session_get_scalar(brr_session *s, int32_t which, double *out);
int64_t brr_session_get_vector(brr_session *s, int32_t which, double *out /* may be NULL */);
int brr_session_set_vector(brr_session *s, int32_t which, const double *in);
int brr_session_set_scalar(brr_session *s, int32_t which, double v);
int32_t brr_session_iteration(brr_session *s);
/* validation read-back: out[i] = sum_j X[i,j] beta_j + sum_c fixed[i,c] alpha_c over this shard's
 * markers (N doubles), computed by a plain row kernel independent of the sweep kernels; used by
 * the full-size residual invariant eps = Y - mu - X beta - F alpha */
int brr_session_linear_predictor(brr_session *s, double *out /* N */);

/* instrumentation: per-launch HIP-event timing of the streaming kernel (dots + residual
 * update), accumulated over the sweeps run while enabled. */
int brr_session_set_timing(brr_session *s, int32_t on);
int brr_session_timing(brr_session *s, double *stream_ms_total, int64_t *stream_launches,
                       double *solve_ms_total, int64_t *solve_launches);
/* algorithmic bytes of one streaming launch = 4 * N * block_size */
int64_t brr_session_block_size(brr_session *s);
int brr_session_synchronize(brr_session *s);

#ifdef __cplusplus
}
#endif
#endif
