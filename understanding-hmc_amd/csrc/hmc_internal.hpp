// hmc_internal.hpp — host-side kernel argument blocks and launchers (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hmc.h"

namespace hmc {

constexpr int kStampWords = 16;   // debug phase-timer words per wave (HMC_DEBUG_STAMPS)

// Lane-group layout of one chain inside a wave64 (see hmc_device.hpp).
struct Layout {
  int K;       // coordinate pairs per lane
  int lpc;     // lanes per chain
  int cpw;     // chains per wave
  int npairs;  // ceil(D/2)
};

// Arguments of the diagonal-target Random-trajectory kernels (init + iterations).
struct RandArgs {
  int64_t n;             // chains in this call
  int64_t chain_offset;  // global id of chain 0 (Philox key)
  int D, npairs, lpc, cpw;
  int niter, wu, thin, Lc, L_low, L_high, it0, it1, i_oob;
  uint32_t k0, k1;       // Philox key (seed)
  double dt, h, logc;    // step, dt/2, V constant
  const double* q0;      // [D] or null
  const double* prec;    // [D] or null
  const double* minv;    // [D] or null
  const double* pscale;  // [D] or null
  const double* dtv;     // [D] or null
  const double* minvf;   // dense mass: [D*D] inv(cov_p) (symmetric) or null
  const double* cholt;   // dense mass: [D*D] transpose of chol(cov_p) (Philox draws)
  const double* kick;    // dense mass: [D*D] inv(cov_p) . prec (staged in LDS instead of prec)
  const double* rp0;     // replay streams
  const double* rp;
  const double* rlnu;
  const int32_t* rL;
  const double* qstart;  // init only
  double* q;
  double* Eprev;
  double* qc;
  double* Ec;
  double* dEc;
  unsigned long long* cnt;
  double* traj_q;        // chain-0 trajectory capture (or null)
  int32_t* traj_len;
  int32_t* decision;
  int n_save, traj_stride;
  int Lq, q_row0;        // q_chain buffer: rows per chain (row r at r % Lq) and the first row stored
  int d_max, on_dmax;    // NUTS (hmc_nuts.hip)
  uint64_t wait_cap;     // NUTS: wave steps a slot waits for a chain hand-off before giving up
  int nuts_kb;           // NUTS: iterations of the launch's chain-affine block units (0: tree units only)
  double* ws;            // NUTS per-chain workspace (vectors: live points, boundaries, save slots)
  const double* tape;    // NUTS replay tape [n][tape_stride] (directions / uniforms in consumption order)
  int64_t tape_stride;
  int dbg;               // ablation flags (HMC_DEBUG_ABLATE env; 0 in normal runs)
  int dbgL;              // forced trajectory length (HMC_DEBUG_L env; -1 in normal runs)
  unsigned long long* stamps;  // diagnostic phase timers (HMC_DEBUG_STAMPS env; null in normal runs),
                               // kStampWords per wave
  const int32_t* order;  // dense: tile slot -> chain (L-ordered tiles) or null (slot = chain)
  double* gcache;        // dense: per-chain gradient at q [n][D] (in the order workspace) or null
  const int32_t* gvalid; // dense: nonzero once gcache holds the gradient of every chain's q
  int64_t ntiles;        // dense: 16-chain tiles
};

// Dense-precision (correlated MVN) kernels take the same argument block; `prec` is then the
// row-major D x D precision.  dense_tiles(D) = 16-dim output tiles per chain (0: unsupported).
using DenseArgs = RandArgs;
int dense_tiles(int D);
// NUTS: the largest d_max the kernels take (samplers.py:306 takes any; a tree of 2^30 - 1 leapfrogs
// per iteration is far past any practical run; the save slots are d_max + 1 vectors per chain)
constexpr int kNutsDmaxMax = 30;
int64_t nuts_ws_doubles(int64_t n, int D, int d_max, int mom_iters);   // mom_iters: Philox momenta drawn ahead
hipError_t launch_nuts_iters(const RandArgs& a, bool exact, bool replay, hipStream_t s);
// NUTS for dense D > 128 (hmc_nuts_big.hip): one wave per chain, tree vectors in the workspace.
int64_t nuts_big_ws_doubles(int64_t n, int D, int d_max);
// NUTS for 128 < D <= 320 in lockstep 16-chain blocks (hmc_nuts_lock.hip): one MFMA GEMM per block
// step gives every chain its gradient
bool nuts_lock_path(int D);
int64_t nuts_lock_ws_doubles(int64_t n, int D, int d_max, bool mass);
hipError_t launch_nuts_lock(const RandArgs& a, bool exact, bool replay, hipStream_t s);
hipError_t launch_nuts_big(const RandArgs& a, bool exact, bool replay, hipStream_t s);

Layout choose_layout(int D, int L_low, int L_high);

hipError_t launch_random_init(const RandArgs& a, const Layout& lay, bool gen, bool replay, hipStream_t s);
hipError_t launch_random_iters(const RandArgs& a, const Layout& lay, bool exact, bool gen, bool replay,
                               hipStream_t s);
hipError_t launch_wave_iters(const RandArgs& a, int K, bool exact, bool gen, bool replay, hipStream_t s);
hipError_t launch_dense_init(const DenseArgs& a, bool replay, hipStream_t s);
hipError_t launch_dense_iters(const DenseArgs& a, bool exact, bool replay, hipStream_t s);
int64_t dense_order_ints(int64_t n);   // int32 scratch of the L-ordering (order[n] + histograms)
// gradient cache inside the order workspace: validity word, then [n][D] doubles
int64_t dense_gcache_offset_bytes(int64_t n);
int64_t dense_workspace_bytes(int64_t n, int D);
bool dense_order_ok(const DenseArgs& a);
hipError_t launch_dense_order(const DenseArgs& a, int it, bool replay, int32_t* ws, hipStream_t s);
int device_cus();


// Large-D Random sampler (hmc_big.hip): dense D > 128, diagonal D > 2048; chain state in HBM,
// one iteration = begin, per leapfrog step (kick + drift, gradient, kick), end.
struct BigArgs {
  RandArgs a;
  double* p;     // [n][D] momentum
  double* g;     // [n][D] gradient at q (dense targets)
  double* qi;    // [n][D] q at the start of the iteration (restored on rejection)
  double* gi;    // [n][D] its gradient (dense targets)
  double* kv;    // [n][D] full cov_p: the kick inv_cov_p g
  double* u;     // [n][D] full cov_p: inv_cov_p p, or the momentum's z
  const double* gk;   // the kick vector the leapfrog reads: g, or kv with a full cov_p
  int32_t* L;    // [n] trajectory length of the current iteration
  double* lnu;   // [n] log u of the current iteration
  double* E0;    // [n] energy at the start of the current iteration
};
bool big_path(int kind_dense, int D);
int64_t big_workspace_bytes(int64_t n, int D, bool dense, bool full_mass);
BigArgs big_args(const RandArgs& a, void* ws, bool dense);
hipError_t launch_big_init(const BigArgs& b, bool dense, bool replay, hipStream_t s);
hipError_t launch_big_iters(const BigArgs& b, bool dense, bool exact, bool replay, hipStream_t s);

// Row-wise API kernels (hmc_api_kernels.hip).
struct RowArgs {
  int64_t n;
  int D;
  int dense;
  const double* q0;
  const double* prec;
  const double* minv;
  const double* dtv;
  const double* minvf;   // dense mass matrix inv(cov_p) [D*D] or null
  double dt, logc;
  const double* p;
  const double* q;
  double* po;
  double* qo;
  double* E;
};
hipError_t launch_leapfrog_rows(const RowArgs& a, bool exact, hipStream_t s);
hipError_t launch_energy_rows(const RowArgs& a, hipStream_t s);
hipError_t launch_philox(uint4 c, uint32_t k0, uint32_t k1, int64_t n, uint32_t* out, hipStream_t s);
hipError_t launch_rng_normals(uint32_t k0, uint32_t k1, int64_t chain0, int64_t n, int it, int npairs,
                              double* out, hipStream_t s);

// Diagnostics (hmc_diag.hip).
int64_t diag_rowsum_work(int64_t rows, int D);
// whether the lag kernel's 32-bit buffer offsets cover a strided view (hmc_diag.hip lag_view_ok)
bool diag_view_ok(int64_t n_chains, int64_t cs, int64_t ss, int n, int D, int halves, int wrap, int slot0);
int64_t diag_variogram_work(int64_t n_chains, int D, int nlags);
int64_t diag_stream_groups(int64_t n_chains);
int64_t diag_conv_work(int64_t n_chains, int D, int T);
hipError_t launch_conv_fused(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n, int D,
                             int T, double* work, double* out, hipStream_t st);
hipError_t launch_half_sums(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int D, int wrap, int slot0,
                            int n, int T, double* work, double* out, hipStream_t st);
hipError_t launch_stream_accum(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int D, int wrap, int slot0,
                               int carry, int rows, int64_t pos0, int n, double* shift, double* s1, double* s2, int T,
                               double* vpart, double* vsum, hipStream_t st);
hipError_t launch_split_moments(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n,
                                int D, double* mean_out, double* std_out, hipStream_t st);
hipError_t launch_rowsum(const double* x, int64_t n_outer, int64_t os, int64_t n_inner, int64_t is, int64_t base,
                         int D, const double* center, double* work, double* out, hipStream_t st);
hipError_t launch_variogram(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n, int D,
                            int t0, int t1, double* work, double* out, hipStream_t st);

}  // namespace hmc
