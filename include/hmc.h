/*
 * hmc.h — C ABI of libhmc.so, the MI355X-native many-chain HMC engine.
 *
 * Drop-in boundary for the hot path of jaekor91/understanding-HMC (samplers.py).
 * The reference has no FFI of its own (pure NumPy); each entry
 * point below names the reference function whose behaviour it replaces, so a
 * maintainer can bind it from the reference's Python side with ctypes
 * (INTEGRATION.md shows the stub).
 *
 * Conventions
 *  - Plain C types only: pointers, sizes, POD structs.  No torch types.
 *  - Every array argument is a DEVICE pointer (hipMalloc'd or a torch tensor's
 *    data_ptr()) unless stated otherwise; fp64 throughout; row-major.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Calls
 *    are stream-ordered and asynchronous; the library allocates nothing on the
 *    hot call and never synchronises the device (graph-capturable).
 *  - Errors: integer status (hmc_status).  hmc_last_error() returns a message
 *    for the last failing call on this host thread.  The Python mirror maps
 *    HMC_EINVAL -> AssertionError (the reference validates with `assert`,
 *    samplers.py:331-348, :396), HMC_EINDEX -> IndexError (samplers.py:471, Q5),
 *    HMC_EDMAX -> AssertionError (samplers.py:596-598).
 */
#ifndef HMC_AMD_HMC_H
#define HMC_AMD_HMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum hmc_status {
  HMC_OK = 0,
  HMC_EINVAL = 1,   /* bad argument (reference: AssertionError) */
  HMC_EDMAX = 2,    /* NUTS doubling exceeded d_max (samplers.py:596-598) */
  HMC_EHIP = 3,     /* HIP runtime error */
  HMC_EINDEX = 4,   /* q_chain row out of range during warm-up (samplers.py:471, Q5) */
  HMC_ENOTSUP = 5   /* shape/feature outside what the kernels support */
} hmc_status;

enum { HMC_TARGET_DIAG = 0, HMC_TARGET_DENSE = 1 };
enum { HMC_RNG_REPLAY = 0, HMC_RNG_PHILOX = 1 };
enum { HMC_MODE_EXACT = 0, HMC_MODE_FAST = 1 };

/* counters[] slots (unsigned long long, device, accumulated with atomics) */
enum {
  HMC_CNT_ACCEPT = 0,        /* accepted proposals, i >= warm_up (samplers.py:467)          */
  HMC_CNT_ACCEPT_WU = 1,     /* accepted proposals, i <  warm_up (samplers.py:469)          */
  HMC_CNT_LEAPFROG = 2,      /* sum of L actually integrated (the metric's unit of work)     */
  HMC_CNT_LEAPFROG_SQ = 3,   /* Random: sum of L^2 (N_total_steps, Q13); NUTS: steps of the
                                kernel's scheduling unit (see hmc_nuts_iters)                 */
  HMC_CNT_OOB_REJECT = 4,    /* rejections whose warm-up row index is < -L_chain (Q5)        */
  HMC_CNT_UNSTABLE = 5,      /* NUTS |E-E0| > 1000 sub-tree rejections (samplers.py:647)     */
  HMC_CNT_DMAX = 6,          /* NUTS chain-iterations that hit d_max                         */
  HMC_CNT_ENERGY_EVALS = 7,  /* NUTS energy evaluations (N_total_steps accounting)           */
  HMC_CNT_HANDOFF_GIVEUP = 8,/* NUTS chain hand-offs between work-queue slots given up (a
                                launch error: must stay 0; the Python layer raises)           */
  HMC_NCOUNTERS = 9,
  /* counters are spread over HMC_COUNTER_SLOTS rows ([slot][HMC_NCOUNTERS]) so that the
   * per-wave atomics of a launch do not serialise on one address; totals = sum over slots */
  HMC_COUNTER_SLOTS = 4096
};

/* MVN target: V(q) = 0.5*(logdet_const + (q-q0)^T P (q-q0)), dV/dq = P (q-q0).
 * Replaces the driver closures V/dVdq (case1-script.py:39-49) + utils.normal_lnL
 * (utils.py:213-218); P = inv(cov0) (case1-script.py:36). */
typedef struct hmc_target {
  int32_t D;
  int32_t kind;            /* HMC_TARGET_DIAG or HMC_TARGET_DENSE                       */
  const double* q0;        /* [D] mean, NULL => 0                                        */
  const double* prec;      /* DIAG: [D] diagonal of P, NULL => identity; DENSE: [D*D]    */
  double logdet_const;     /* D*log(2*pi) + log det(cov0)  (scipy logpdf constant, Q15)  */
} hmc_target;

/* Kinetic part and integrator step.  Replaces HMC_sampler.cov_p/inv_cov_p/dt
 * (samplers.py:333, :352-356) as used by K, p_sample and leap_frog (:811-839). */
typedef struct hmc_kinetic {
  const double* minv;      /* [D] diagonal of inv(cov_p), NULL => identity (Q3)          */
  const double* p_scale;   /* [D] sqrt(diag(cov_p)) for in-kernel draws, NULL => 1        */
  const double* dt_vec;    /* [D] per-dimension step (global_dt=False), NULL => dt        */
  double dt;               /* scalar step                                                 */
  /* Dense (non-diagonal) mass matrix, samplers.py:352-356 with a full cov_p (Q3 semantics:
   * K = p.inv(cov_p).p/2, kick by inv(cov_p).dVdq, drift by p).  All NULL => diagonal/identity
   * via minv/p_scale above (which must then be NULL).  Dense targets (pass prec dense), any D,
   * Random and NUTS samplers (NUTS reads minv_full and kick; p_chol_t for Philox draws).  */
  const double* minv_full; /* [D*D] inv(cov_p), row-major (symmetric)                     */
  const double* p_chol_t;  /* [D*D] transpose of the lower Cholesky factor C of cov_p:
                              Philox momentum p = C z, z ~ N(0, I)                        */
  const double* kick;      /* [D*D] inv(cov_p) . prec, row-major: the kick matrix          */
} hmc_kinetic;

/* Run schedule of gen_sample_random / gen_sample_NUTS (samplers.py:387, :495). */
typedef struct hmc_schedule {
  int64_t n_chains;        /* chains handled by this call (this shard)                    */
  int64_t chain_offset;    /* global id of the first chain: RNG key, so results do not
                              depend on the number of GPUs or the launch geometry         */
  int32_t n_iter;          /* Niter                                                        */
  int32_t warm_up;         /* warm_up_num                                                  */
  int32_t thin;            /* thin_rate                                                    */
  int32_t L_chain;         /* 1 + (Niter - warm_up)//thin   (samplers.py:31)              */
  int32_t L_low, L_high;   /* Random: L ~ U{L_low .. L_high-1} (samplers.py:441, Q1)      */
  int32_t iter_begin;      /* first iteration i (1-based) of this call                     */
  int32_t iter_end;        /* one past the last iteration of this call                     */
  int32_t rng_mode;        /* HMC_RNG_REPLAY or HMC_RNG_PHILOX                             */
  int32_t fp_mode;         /* HMC_MODE_EXACT (no FMA contraction: bit-identical to the
                              NumPy reference for diagonal targets) or HMC_MODE_FAST     */
  int32_t d_max;           /* NUTS max doublings (samplers.py:306, :596)                  */
  int32_t on_dmax;         /* NUTS: 0 = flag HMC_EDMAX (reference aborts), 1 = count and
                              keep the current sample                                      */
  uint64_t seed;           /* Philox4x32-10 key                                             */
} hmc_schedule;

/* Host-replayed random streams (RNG_REPLAY): the draws the reference would
 * consume from the global legacy np.random, in its order (Q7). */
typedef struct hmc_replay {
  const double* p0;        /* [n_chains][D]        initial momentum (samplers.py:415, Q4) */
  const double* p;         /* [n_chains][n_iter][D] momentum of iterations 1..Niter (:431) */
  const int32_t* L;        /* [n_chains][n_iter]    trajectory lengths (:441)              */
  const double* lnu;       /* [n_chains][n_iter]    log-uniforms (:461)                    */
  const double* tape;      /* NUTS: [n_chains][tape_stride] directions/uniforms in order  */
  int64_t tape_stride;
} hmc_replay;

/* Chain state and outputs (all device).  Result attributes of HMC_sampler
 * (samplers.py:31-50, :359-360). */
typedef struct hmc_state {
  double* q;               /* [n_chains][D] current position (in/out)                     */
  double* E_prev;          /* [n_chains] E_initial of the previous iteration (Q14)         */
  double* q_chain;         /* [n_chains][L_chain][D] or NULL (no sample storage)          */
  double* E_chain;         /* [n_chains][L_chain] or NULL                                  */
  double* dE_chain;        /* [n_chains][L_chain] or NULL                                  */
  unsigned long long* counters; /* [HMC_COUNTER_SLOTS][HMC_NCOUNTERS], zero-initialised       */
  /* Trajectory capture of global chain 0 for the first n_save iterations (make_movie input;
   * samplers.py:397-400, :442-475): traj_q[n_save][traj_stride][2] = q[:2] after each step,
   * traj_len[n_save] = L+1, decision[n_save] = accepted.  NULL / 0 disables capture. */
  double* traj_q;
  int32_t* traj_len;
  int32_t* decision;
  int32_t n_save;
  int32_t traj_stride;     /* >= L_high (Random)                                              */
  /* q_chain as a circular window (streaming diagnostics): the buffer holds qc_rows rows per
   * chain, chain row r >= qc_row0 is stored at row r % qc_rows; rows < qc_row0 are not stored.
   * 0, 0 = the whole chain. */
  int64_t qc_rows;
  int64_t qc_row0;
  /* Dense targets, Random sampler: scratch of hmc_random_workspace_size() bytes for L-ordered
   * tiles (each iteration, chains are counting-sorted by trajectory length so that the 16
   * chains sharing an MFMA tile integrate the same number of steps; results are unchanged) and
   * a per-chain cache of the gradient at q (reused instead of recomputed at the start of each
   * iteration; bit-identical).  hmc_chain_init invalidates the cache: a caller that writes q
   * itself must call hmc_chain_init again.  NULL = tiles in chain order (several iterations
   * fused per launch), no cache.  Ignored for DIAG. */
  int32_t* order;
} hmc_state;

const char* hmc_version(void);
const char* hmc_last_error(void);

/* Chain initialisation: q_chain[:,0] = q_start, E_chain[:,0] = E(q_start, p0),
 * dE_chain[:,0] = 0, q = q_start, E_prev = E_chain[:,0].
 * Replaces samplers.py:413-420 (Random) and :548-555 (NUTS). */
hmc_status hmc_chain_init(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s,
                          const hmc_replay* r /* NULL for Philox */, const double* q_start,
                          hmc_state* st, void* stream);

/* Iterations [iter_begin, iter_end) of the Random-trajectory sampler for all chains:
 * fused momentum resample -> E0 -> L leapfrogs -> E1 -> Metropolis test -> store.
 * Replaces HMC_sampler.gen_sample_random, samplers.py:428-475 (+ :811-839). */
hmc_status hmc_random_iters(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s,
                            const hmc_replay* r /* NULL for Philox */, hmc_state* st, void* stream);

/* The same two calls with the size of hmc_state.order (bytes) passed alongside: HMC_EINVAL when
 * it is smaller than this call reads or writes (hmc_random_workspace_size_ex), before any kernel
 * runs.  The size is also recorded for the buffer, so that the unsized forms above refuse it later
 * if a call needs more (as they refuse any buffer recorded by hmc_workspace_register). */
hmc_status hmc_chain_init_ws(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s,
                             const hmc_replay* r, const double* q_start, hmc_state* st,
                             int64_t order_bytes, void* stream);
hmc_status hmc_random_iters_ws(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s,
                               const hmc_replay* r, hmc_state* st, int64_t order_bytes, void* stream);

/* Record the size of a scratch buffer (hmc_state.order or a NUTS workspace) for the unsized entry
 * points: a later call that would need more than `bytes` returns HMC_EINVAL instead of writing past
 * the end.  bytes = 0 forgets the buffer; a record stays until the pointer is registered again, so
 * register (or use a sized form) again after reallocating.  Host-side bookkeeping only (no device
 * access). */
hmc_status hmc_workspace_register(const void* workspace, int64_t bytes);

/* Bytes of the optional hmc_state.order scratch for hmc_random_iters on this target
 * (0 for diagonal targets, which need none): the tile order plus the gradient cache.  Large-D
 * targets (dense D > 128, diagonal D > 2048) keep their chain state there and need it, also for
 * hmc_chain_init of a NUTS run.  hmc_random_workspace_size covers either cov_p; the _ex form sizes
 * for the given kinetic part (two [n][D] vectors fewer without a full cov_p). */
int64_t hmc_random_workspace_size(const hmc_target* t, int64_t n_chains);
int64_t hmc_random_workspace_size_ex(const hmc_target* t, const hmc_kinetic* k, int64_t n_chains);
/* Bytes of device workspace hmc_nuts_iters needs for n_chains chains: tree vectors (live points,
 * both boundaries, d_max+1 save slots), replay-tape cursors, the launch's work queue and, for
 * Philox runs with a diagonal cov_p (philox_momenta != 0), the momenta drawn ahead of the tree
 * kernel: n_chains x min(32, iters_per_call) x 16*ceil(D/16) doubles (iters_per_call = the largest
 * iter_end - iter_begin the caller will pass).  philox_momenta = 0 (replay tapes, or a full cov_p,
 * whose momenta the kernels draw in place, and whose lockstep blocks keep the inv(cov_p) products
 * of their chains) sizes for those runs.  0 if unsupported.
 * hmc_nuts_workspace_size(D, n, d_max): enough for any call (iters_per_call 32, either kind). */
int64_t hmc_nuts_workspace_size_ex(int32_t D, int64_t n_chains, int32_t d_max, int32_t iters_per_call,
                                   int32_t philox_momenta);
int64_t hmc_nuts_workspace_size(int32_t D, int64_t n_chains, int32_t d_max);

/* Iterations [iter_begin, iter_end) of the No-U-Turn sampler for all chains: momentum
 * resample -> E0 -> tree doubling until both ends U-turn (sub-tree U-turn checks against the
 * saved odd points, progressive sampling, biased sub-tree acceptance) -> store.
 * Replaces HMC_sampler.gen_sample_NUTS, samplers.py:563-791 (+ utils.py:222-385).
 * Dense precision only (pass diagonal targets as dense), any D, 1 <= d_max <= 30 (the reference
 * takes any d_max; 30 = up to 2^30 - 1 leapfrogs per tree), diagonal or
 * full cov_p (minv_full) at any D:
 *   D <= 128              the 16-chain MFMA tree kernel (hmc_nuts.hip; a full cov_p adds its
 *                         momentum and kinetic products on the same tiles);
 *   128 < D <= 320        16 chains per block in lockstep sharing one MFMA GEMM per leapfrog
 *                         (hmc_nuts_lock.hip; a full cov_p adds the inv(cov_p) and Cholesky
 *                         products as block GEMMs on the same fragments, round 6);
 *   otherwise (D > 320)   one wave per chain (hmc_nuts_big.hip; a full cov_p as three GEMVs per
 *                         leapfrog).
 * `workspace` (hmc_nuts_workspace_size bytes, or hmc_nuts_workspace_size_ex sized for the calls
 * made) must be zeroed before the first call of a run and kept between calls; hmc_nuts_iters_ws
 * also takes the workspace's size and refuses (HMC_EINVAL) a call that needs more.  Counters:
 * LEAPFROG (= ENERGY_EVALS), UNSTABLE (|E-E0| > 1000 rejections, :647), DMAX (chain-iterations
 * that reached d_max; the reference aborts there, on_dmax selects whether the caller raises),
 * OOB_REJECT (replay tape exhausted: an error), LEAPFROG_SQ = steps of the kernel's scheduling
 * unit, whose meaning depends on the path: wave steps of the 16-chain tree kernel and block steps
 * of the lockstep kernel (16 chain slots each: lane utilisation = LEAPFROG / (16 x LEAPFROG_SQ)),
 * wave steps of the per-chain kernel (one chain per wave: equal to LEAPFROG). */
hmc_status hmc_nuts_iters(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s,
                          const hmc_replay* r /* NULL for Philox */, hmc_state* st, void* workspace,
                          void* stream);
/* hmc_nuts_iters_ws: the sized form (records workspace_bytes for the buffer; the unsized form then
 * refuses it for any call that needs more, as for hmc_workspace_register). */
hmc_status hmc_nuts_iters_ws(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s,
                             const hmc_replay* r /* NULL for Philox */, hmc_state* st, void* workspace,
                             int64_t workspace_bytes, void* stream);

/* Batched single leapfrog step (n independent (p, q) rows).
 * Replaces HMC_sampler.leap_frog(p_old, q_old), samplers.py:831-839. */
hmc_status hmc_leapfrog(const hmc_target* t, const hmc_kinetic* k, int64_t n, const double* p,
                        const double* q, double* p_out, double* q_out, int32_t fp_mode,
                        void* stream);

/* Batched total energy E(q, p) = V(q) + K(p) of n rows.
 * Replaces HMC_sampler.E / K (samplers.py:811-823) with V of utils.py:213-218. */
hmc_status hmc_energy(const hmc_target* t, const hmc_kinetic* k, int64_t n, const double* q,
                      const double* p, double* E_out, void* stream);

/* The standard normals the Philox mode draws for (chain, iteration): out[n][2*npairs].
 * Debug/verification entry (statistical tests of the in-kernel generator). */
hmc_status hmc_rng_normals(uint64_t seed, int64_t chain0, int64_t n, int32_t iteration,
                           int32_t npairs, double* out, void* stream);

/* Raw Philox4x32-10 blocks: out[n][4] = philox(ctr = {x0 + i, x1, x2, x3}, key). */
hmc_status hmc_philox(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t k0,
                      uint32_t k1, int64_t n, uint32_t* out, void* stream);

/* ---------------------------------------------------------------- diagnostics
 * Split-chain R-hat / ESS building blocks (utils.py:77-179) and the per-dimension
 * mean/std of plot_samples (samplers.py:213, :246).  Chains are read in place:
 * element (chain m, sample s, dim d) = x[base + m*chain_stride + s*sample_stride + d].
 * All sums are deterministic (fixed-order two-stage reductions); `work` is caller-owned
 * scratch of the size the *_work_size query returns (doubles).
 * Lag passes (hmc_variogram, hmc_convergence_sums, hmc_half_sums) address a chain's samples with
 * 32-bit buffer offsets: one chain's span (about 3 x chain_stride doubles) must stay within 1 GiB,
 * e.g. D = 1000 up to ~40,000 stored samples per chain; larger views return HMC_ENOTSUP (pass a
 * contiguous copy of fewer dimensions; hmc_amd.diagnostics does so by itself). */

/* Per split chain j (= 2m + half; half h covers samples [h*n, h*n+n)): mean and std
 * (ddof=1) of every dimension -> mean_out/std_out [2*n_chains][D].  utils.py:88-119. */
hmc_status hmc_split_moments(const double* x, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                             int64_t base, int32_t n, int32_t D, double* mean_out, double* std_out, void* stream);

/* out[d] = sum over rows (o, i) of x[base + o*outer_stride + i*inner_stride + d], or of
 * (x - center[d])^2 when center != NULL.  Used for W, B (utils.py:112-120) and mean/std. */
int64_t hmc_rowsum_work_size(int64_t rows, int32_t D);
hmc_status hmc_rowsum(const double* x, int64_t n_outer, int64_t outer_stride, int64_t n_inner,
                      int64_t inner_stride, int64_t base, int32_t D, const double* center, double* work,
                      double* out, void* stream);

/* Variogram sums out[t - t0][d] = sum_j sum_s (x_j[s+t] - x_j[s])^2 over split chains,
 * lags t in [t0, t1), 1 <= t1 - t0 <= 2^20 (one read of the samples for any lag count; work grows
 * with it).  utils.py:161-179 (before its division by m*(n-t)). */
int64_t hmc_variogram_work_size(int64_t n_chains, int32_t D, int32_t nlags);
hmc_status hmc_variogram(const double* x, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                         int64_t base, int32_t n, int32_t D, int32_t t0, int32_t t1, double* work, double* out,
                         void* stream);

/* Everything convergence_stats needs from the samples in ONE pass (utils.py:88-126, :161-179):
 * out[(4 + tmax)][D] =
 *   row 0        sum_j std_j (ddof=1)                       (W, utils.py:109-112)
 *   row 1        sum_j (mean_j - S_d)                       (mean_all, :116-119)
 *   row 2        sum_j (mean_j - S_d)^2                     (B, :120, after re-centring)
 *   row 2 + t    sum_j sum_s (x_j[s+t] - x_j[s])^2, t = 1..tmax (variogram, :161-179; 0 for t >= n)
 *   row 3 + tmax sum_j (x_j[n-1] - x_j[0])^2: the variogram of lag n - 1, the last lag the ESS loop
 *                reads (:139-150), whatever tmax (0 for n < 2)
 * over the 2*n_chains split chains j (same strided view as hmc_split_moments), S_d = x[base + d]
 * (the view's first sample: a common shift so that B needs no second pass).  1 <= tmax <= 2^20:
 * the window is read once whatever tmax (ramp-skipping lag kernel); tmax >= n - 2 gives every lag
 * the ESS loop can read (the last few in difference form); more lags later for a subset of dims:
 * hmc_variogram.  Complete passes (tmax >= n - 2) of 96 <= n <= 208 run on the f64 matrix cores
 * (lag products as Hankel-tile MFMAs; split means from partial sums in a fixed order, within a few
 * ulps of np.mean's sequential sum).  Deterministic (fixed-order two-stage sums). */
int64_t hmc_convergence_work_size(int64_t n_chains, int32_t D, int32_t tmax);
hmc_status hmc_convergence_sums(const double* x, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                                int64_t base, int32_t n, int32_t D, int32_t tmax, double* work, double* out,
                                void* stream);

/* hmc_convergence_sums for ONE completed split half of every chain, read in place from a circular
 * streaming window: sample s (0 <= s < n) of chain c, dim d at window[c*chain_stride +
 * ((slot0 + s) % wrap)*sample_stride + d] (wrap 0: row slot0 + s).  Same output layout over the
 * n_chains series (one per chain) with S_d = chain 0's sample 0; additive over halves and ranks
 * after re-centring (hmc_amd.diagnostics.StreamingDiagnostics): the streaming run's R-hat and ESS
 * then use every lag 1 .. n-1, exactly as convergence_stats on the stored q_chain (utils.py:77-179).
 * work: hmc_convergence_work_size(n_chains, D, tmax) doubles. */
hmc_status hmc_half_sums(const double* window, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                         int32_t D, int32_t wrap, int32_t slot0, int32_t n, int32_t tmax, double* work, double* out,
                         void* stream);

/* Streaming (windowed) split-chain statistics for runs whose q_chain does not fit: feed the
 * samples segment by segment.  Positions p index q_chain[:, 1:, :] (Q16); p lies in split half
 * h = p / n_half.  `window` is circular with `wrap` rows per chain (element [c*chain_stride +
 * r*sample_stride + d]): the k-th sample from position pos0 - carry sits in row (slot0 + k) % wrap;
 * the last `rows` of the carry + rows samples are new.  carry >= min(tmax, pos0) keeps every
 * variogram lag t <= tmax exact.  Accumulates per chain/half/dim shift (first sample), s1 =
 * sum (x - shift), s2 = sum (x - shift)^2 ([n_chains][2][D], zero-initialised) and
 * vsum[t-1][d] += sum over chains of sum (x[p] - x[p-t])^2 for lags t = 1..tmax (tmax in {8,16,32,64};
 * a half adds its sums once complete; rows of lags t >= n_half are not variogram sums).
 * Replaces the q_chain-wide passes of utils.py:88-126 and :161-179. */
int64_t hmc_stream_work_size(int64_t n_chains, int32_t D, int32_t tmax);
hmc_status hmc_stream_accumulate(const double* window, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                                 int32_t D, int32_t wrap, int32_t slot0, int32_t carry, int32_t rows, int64_t pos0,
                                 int32_t n_half, double* shift, double* s1, double* s2, int32_t tmax, double* work,
                                 double* vsum, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HMC_AMD_HMC_H */
