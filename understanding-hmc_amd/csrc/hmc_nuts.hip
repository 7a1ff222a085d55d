// hmc_nuts.hip — the reference's NUTS engine (samplers.py:495-808, utils.py:222-385) for many chains.
//
// Semantics follow gen_sample_NUTS exactly (quirks Q10-Q12 of SURVEY §8-Q): doubling until BOTH
// ends U-turn, sub-tree U-turn checks against the saved odd points named by check_points(m)
// with release_fast bookkeeping, progressive multinomial sampling inside the new sub-tree,
// biased sub-tree acceptance exp(-(Emax_new-Emax_old))*pi_old/pi_new, |E - E0| > 1000 guard.
//
// Execution model: 16 chains per wave share the f64-MFMA gradient tile of hmc_dense_ops.hpp.
// NUTS trees diverge per chain (7 ... 1023 leapfrogs per iteration), so each chain runs its own
// state machine and the wave advances in *steps*: every step all chains that are inside a
// sub-tree take exactly one leapfrog (one MFMA pass for the tile), then each chain processes its
// new point; chains between trees (iteration end / start, sub-tree start) do their transition
// work first.  A launch ends when every chain of the wave finished its iterations.
// Per-chain vectors that trees keep (live points, both boundaries, the d_max+1 save slots) live
// in a workspace in HBM (`ws`, hmc_nuts_workspace_size), chain-contiguous and zero padded so
// lanes never branch on the dimension and chains that sit out a branch move no bytes.  The tail of the workspace holds the per-chain replay-tape cursors (zeroed by the
// host before the first launch of a run).  All cross-lane reductions run in converged control flow.
#include <algorithm>

#include "hmc_dense_ops.hpp"
#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {

namespace {


// Waves per block (one block per CU: the LDS copy of P), one per SIMD with the whole register file.
// 8 (two waves per SIMD, 256 registers each) was measured at 0.42x: the step spills ~560 B per lane
// to scratch and the queue's tail grows (lane utilisation 0.80 -> 0.66).
#ifndef HMC_NUTS_WAVES
#define HMC_NUTS_WAVES 4
#endif
constexpr int kNutsWaves = HMC_NUTS_WAVES;

// Chain affinity (work queue below): a launch's first K - kNutsTail iterations of every chain run in
// units of kNutsBlock consecutive iterations (a slot keeps its chain from tree to tree inside a unit:
// no write-back, drain, publish, poll or state loads between them), queued block-major so a chain's
// next block waits behind the whole grid's current one; its last kNutsTail iterations run as one unit
// per (chain, iteration), which keeps the launch's tail at one tree per slot.  kNutsBlock 1 gives the
// per-tree units only.
// (round 6, with the release/acquire hand-off: blocks of 12 beat 8 by 1.0%, 10 and 14 lost 0.3% and
// 3%, 16 lost 2.5%: profiles/r06s_nuts_block_ab.txt)
#ifndef HMC_NUTS_BLOCK
#define HMC_NUTS_BLOCK 12
#endif
#ifndef HMC_NUTS_TAIL
#define HMC_NUTS_TAIL 4
#endif
constexpr int kNutsBlock = HMC_NUTS_BLOCK;
constexpr int kNutsTail = HMC_NUTS_TAIL;

// S_FETCH: the chain slot hands its chain back and takes the next (chain, iteration) unit of the
// launch from the queue (or retires); S_WAIT: the unit's chain is still finishing its previous
// iteration in another slot; S_GRAD: a fetched chain waits one wave step for the MFMA gradient at
// its start point.  (A doubling towards the other end starts from that end's q, p, g, loaded at
// the previous sub-tree's end for the termination check: no load state.)
enum : int { S_ITER_START = 0, S_READY = 2, S_ITER_END = 3, S_DONE = 4, S_FETCH = 5, S_GRAD = 6,
             S_WAIT = 8 };

// Chain hand-off between slots (any CU, any XCD) inside a launch: the chain's state (q, E_prev, tape
// cursor) is stored with relaxed agent-scope atomic stores (write-through, sc1) and drained
// (vmcnt(0)); then, following the HIP memory model, one agent-scope RELEASE fence per wave step
// that publishes orders those stores before the relaxed store of the chain's iteration count; the
// taking slot polls that word with relaxed loads and, in the step a poll succeeds, issues one
// agent-scope ACQUIRE fence before its (sc1) state loads: fence-fence synchronisation, so the
// hand-off holds on any memory system the model covers, not only on today's gfx950 caches.  With
// chain affinity (hand-offs once per kNutsBlock trees) it costs 2.5% against the relaxed sc1 +
// vmcnt protocol alone (1.934e9 vs 1.982e9 lf/s, same box; -5 to -6% with a hand-off per tree);
// that protocol stays as the dev A/B variant HMC_NUTS_RELAXED.
// Reserving the next unit at tree start and polling its chain during the tree (so that a tree's
// end costs one round trip) measured 1.77e9 -> 1.52e9 lf/s: those loads sit in the in-order vmcnt
// queue ahead of the U-turn checks' loads, which then wait for them.
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_wt(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt_d(double* p, double x) {
  st_wt(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, x));
}
__device__ __forceinline__ double ld_wt_d(const double* p) {
  return __builtin_bit_cast(double, ld_wt(reinterpret_cast<const unsigned long long*>(p)));
}

// Wave steps a slot may wait for a chain's previous iteration before the launch gives up (the
// holder always advances, so this is only a guard against a broken hand-off).  Units of one chain
// are handed out n apart, so at most ceil(slots / n) + 1 iterations of a chain are in flight and
// each holder finishes within one tree, 2^(d_max+1) steps plus its transitions; a step of the
// waiting wave costs about what a step of the holder's does (both run the MFMA gradient), and
// the factor 4 covers the difference.  A holder can still be slowed far more than that (clock or
// XCD variation, several ranks sharing one GPU), so the cap never drops below 2^20 wave steps: a
// give-up is a hard error and only a broken hand-off may trip it.
// 64-bit counter and cap (advisor r05): at d_max >= 27 a block of 8 legitimate deep trees exceeds
// 2^31 wave steps, and a 32-bit clamp would turn a slow but healthy hand-off into a give-up.
inline uint64_t nuts_wait_cap(int64_t slots, int64_t n, int d_max, int kb) {
  const int64_t inflight = (slots + n - 1) / std::max<int64_t>(n, 1) + 1;
  // a block unit holds its chain for kb trees (wait: the chain's previous unit)
  const int64_t trees = std::max(kb, 1);
  return (uint64_t)std::max<int64_t>(4 * inflight * trees * ((int64_t(1) << (d_max + 1)) + 64), int64_t(1) << 20);
}

// workspace vector ids (per chain).  The live points old/new (:577, :623, :750, :775) are two
// buffers, 0 and 2 (1 and 3 are unused since the per-tree queue: no gradient is kept with them):
// `old2` (0 or 2, per chain) names the old one and the other is new, so accepting a sub-tree's
// point swaps the names instead of copying a vector.
enum : int { V_OLD_Q = 0, V_OLD_G = 1, V_NEW_Q = 2, V_NEW_G = 3, V_LEFT_Q = 4, V_LEFT_P = 5, V_LEFT_G = 6,
             V_RIGHT_Q = 7, V_RIGHT_P = 8, V_RIGHT_G = 9, V_SLOTS = 10 };

__device__ __forceinline__ int nuts_nvec(int d_max) { return V_SLOTS + 2 * (d_max + 1); }

// Phase timers of the debug build (make debug; HMC_DEBUG_STAMPS): wave-uniform s_memtime deltas per
// part of a wave step, summed over the launch: 0 transitions, 1 half kick + drift, 2 gradient
// (MFMA), 3 half kick + energies, 4 new-point bookkeeping / saves, 5 loaded U-turn checks,
// 6 progressive sampling, 7 sub-tree end; inside 0: 8 tree end (live point, row), 9 write-back +
// drain + publish, 10 queue reservation, 11 poll + state loads, 12 momentum + tree start; 13 counts
// the wave steps with a tree end.  The release library compiles none of it.
#ifdef HMC_DEBUG_HOOKS
#define NUTS_PHASE(i)                                        \
  do {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - t_ph;                                      \
    t_ph = t_;                                               \
  } while (0)
#else
#define NUTS_PHASE(i) \
  do {                \
  } while (0)
#endif
#ifdef HMC_DEBUG_HOOKS
#define NUTS_SUBPHASE(i)                                     \
  do {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - t_sub;                                     \
    t_sub = t_;                                              \
  } while (0)
#else
#define NUTS_SUBPHASE(i) \
  do {                   \
  } while (0)
#endif

// bytes of the work queue block, zeroed before every launch: head, a spare word, done[n] (u32),
// padded to a multiple of 16
__host__ __device__ inline size_t nuts_queue_bytes(int64_t n) { return (size_t)((16 + 4 * n + 15) / 16 * 16); }

// Philox momenta are drawn ahead of the tree kernel (k_nuts_momenta) for up to kNutsMomIters
// iterations per launch into the workspace tail: a tree start then costs a 16-byte load per lane
// pair, issued with the chain's state loads, instead of ~23k clocks of Philox + Box-Muller that
// the whole wave waited for at every tree end (profiles/r03_c5_nuts_phases.json), and the tree
// kernel needs no Box-Muller tables in LDS.  Longer ranges run as several launches.
constexpr int kNutsMomIters = 32;
__host__ __device__ inline int64_t nuts_mom_doubles(int64_t n, int MT, int iters) {
  return n * (iters < kNutsMomIters ? iters : kNutsMomIters) * 4 * MT * 4;
}

// Workspace: per chain slot, nvec vectors of Dp = 4M doubles (dims, zero padded), slot-contiguous,
// the 16 slots of a wave in one block addressed through a wave-uniform buffer descriptor (SGPR
// base, 32-bit lane offset: no 64-bit addresses kept live).  Inside a vector, lane (c, h) keeps
// its dims h + 4m in pairs (m, m+1) at byte (m/2)*64 + h*16: one chain's part of an access is
// 64 contiguous bytes moved by 16-byte lane accesses (half the instructions and twice the
// contiguous span of an 8-byte-per-lane layout).  Lanes of chains that sit out a branch move
// no bytes.  `vl` is a per-lane extra vector index (the save slot of this chain), 0 for fixed
// vectors.
struct WaveWS {
  __amdgpu_buffer_rsrc_t r;
  int lane_off;   // (lane & 15) * nvec * Dp * 8 + h * 16
};

__device__ __forceinline__ constexpr int ws_elem(int m) { return (m >> 1) * 64 + (m & 1) * 8; }

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// N (even, <= M): the vector's slots that can hold a dimension (the rest stay zero untouched)
template <int M, int N = M>
__device__ __forceinline__ void vstore(const WaveWS& w, int v, int vl, const double (&x)[M]) {
  const int vo = w.lane_off + vl * (4 * M * 8);
#pragma unroll
  for (int m = 0; m < N; m += 2) {
    const u32x2 lo = __builtin_bit_cast(u32x2, x[m]), hi = __builtin_bit_cast(u32x2, x[m + 1]);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo.x, lo.y, hi.x, hi.y}, w.r, vo, v * (4 * M * 8) + ws_elem(m), 0);
  }
}

// x * sg (sg = +-1: exact) into vector v + vl
template <int M, int N = M>
__device__ __forceinline__ void vstore_sg(const WaveWS& w, int v, int vl, const double (&x)[M], double sg) {
  const int vo = w.lane_off + vl * (4 * M * 8);
#pragma unroll
  for (int m = 0; m < N; m += 2) {
    const u32x2 lo = __builtin_bit_cast(u32x2, x[m] * sg), hi = __builtin_bit_cast(u32x2, x[m + 1] * sg);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo.x, lo.y, hi.x, hi.y}, w.r, vo, v * (4 * M * 8) + ws_elem(m), 0);
  }
}

template <int M>
__device__ __forceinline__ void vput(const WaveWS& w, int v, int m, double x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), w.r, w.lane_off, v * (4 * M * 8) + ws_elem(m), 0);
}

template <int M>
__device__ __forceinline__ double vget(const WaveWS& w, int v, int vl, int m) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(w.r, w.lane_off + vl * (4 * M * 8),
                                                                         v * (4 * M * 8) + ws_elem(m), 0));
}

template <int M>
__device__ __forceinline__ void vput2(const WaveWS& w, int v, int m, double x0, double x1) {
  const u32x2 lo = __builtin_bit_cast(u32x2, x0), hi = __builtin_bit_cast(u32x2, x1);
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo.x, lo.y, hi.x, hi.y}, w.r, w.lane_off, v * (4 * M * 8) + ws_elem(m), 0);
}

// dims m and m+1 (m even) in one 16-byte access
template <int M>
__device__ __forceinline__ void vget2(const WaveWS& w, int v, int vl, int m, double& x0, double& x1) {
  const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(w.r, w.lane_off + vl * (4 * M * 8), v * (4 * M * 8) + ws_elem(m), 0);
  x0 = __builtin_bit_cast(double, u32x2{r.x, r.y});
  x1 = __builtin_bit_cast(double, u32x2{r.z, r.w});
}

template <int M, int N = M>
__device__ __forceinline__ void vload(const WaveWS& w, int v, int vl, double (&x)[M]) {
#pragma unroll
  for (int m = 0; m < N; m += 2) vget2<M>(w, v, vl, m, x[m], x[m + 1]);
}

template <int MT, int N = 4 * MT>
__device__ __forceinline__ void gstore(const WaveWS& w, int v, int vl, const d4 (&acc)[MT]) {
  double x[4 * MT];
#pragma unroll
  for (int m = 0; m < 4 * MT; ++m) x[m] = acc[m >> 2][m & 3];
  vstore<4 * MT, N>(w, v, vl, x);
}

template <int MT, int N = 4 * MT>
__device__ __forceinline__ void gload(const WaveWS& w, int v, int vl, d4 (&acc)[MT]) {
#pragma unroll
  for (int m = 0; m < N; m += 2) {
    double x0, x1;
    vget2<4 * MT>(w, v, vl, m, x0, x1);
    acc[m >> 2][m & 3] = x0;
    acc[m >> 2][(m & 3) + 1] = x1;
  }
}

// Save slot of odd point l of a sub-tree.  The reference keeps the saved odd points in a table
// (find_next / retrieve_save_index / release_fast, utils.py:222-385) and looks them up by value.
// A saved point l is only ever checked as the first point of an aligned block of size s | (l - 1)
// ending at an even point m <= l + lowbit(l - 1) - 1, so two points with the same level
// ctz(l - 1) are never needed at the same time: slot = ctz(l - 1) (point 1, the start of every
// block, gets slot d_max) holds exactly the points the table would hold when they are checked,
// with no search and no releases.
__device__ __forceinline__ int save_slot(int l, int d_max) { return l == 1 ? d_max : __builtin_ctz(l - 1); }

// closed forms of utils.py check_points / release_fast (integer bit logic)
__device__ __forceinline__ int cp_r(int m) {   // r of check_points(m): strip leading bits until pow2 or <= 2
  int r = m;
  while ((r & (r - 1)) != 0 && r > 2) r -= 1 << (31 - __builtin_clz(r));
  return r;
}
__device__ __forceinline__ int cp_count(int m) {   // number of check points of even m
  const int r = cp_r(m);
  int cnt = 1, half = r;
  while (half > 2) {
    half >>= 1;
    ++cnt;
  }
  return cnt;
}
__device__ __forceinline__ bool release_fast(int m, int l) {   // utils.py:367-385
  int rm = m, rl = l;
  while ((rm & (rm - 1)) != 0 && rm > 4) {
    const int top = 1 << (31 - __builtin_clz(rm));
    rm -= top;
    rl -= top;
  }
  return (rm >= 4) && (rl > 1);
}

// acc + x*y: the reference's separate multiply and add in EXACT mode, one FMA in FAST mode (the
// per-step dot products and energy sums: ~150 VALU per wave step).
template <bool EXACT>
__device__ __forceinline__ double mac(double acc, double x, double y) {
  if constexpr (EXACT) return acc + x * y;
  else return __builtin_fma(x, y, acc);
}

// Momenta of iterations [it0, it1) (K = it1 - it0 <= kNutsMomIters) for every chain: p ~ N(0, cov_p)
// with a diagonal cov_p (samplers.py:565, :829), exactly the tree kernel's former in-kernel draws
// (pair slot h + 4m -> dims h + 4m and h + 4m + 4, table Box-Muller, pscale, zero padding).
// Layout: per (chain, iteration) one 4M-double vector, chain-major (c * K + it - it0; the buffer holds
// min(kNutsMomIters, iterations per call) iterations, hmc_nuts_workspace_size_ex), in the
// workspace's pair layout (ws_elem):
// 16-byte slot s = 4j + h holds dims (h + 8j, h + 8j + 4), so slot s sits at doubles 2s..2s+1 and
// consecutive threads write consecutive 16-byte slots.
template <int MT, bool GEN>
__global__ __launch_bounds__(256) void k_nuts_momenta(RandArgs a, double* __restrict__ pm) {
  constexpr int M = 4 * MT;
  __shared__ double s_ntab[kNormalTableDoubles];
  init_normal_tables(s_ntab);
  __syncthreads();
  const int K = a.it1 - a.it0;
  const int64_t total = a.n * K * (2 * M);
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < total; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t vec = s / (2 * M);
    const int r = (int)(s - vec * (2 * M));
    const int64_t c = vec / K;
    const int it = a.it0 + (int)(vec - c * K);
    const int h = r & 3, m = 2 * (r >> 2);
    double z0, z1;
    normal_pair_tab(draw_block((uint32_t)(h + 4 * m), (uint32_t)it, (uint64_t)(a.chain_offset + c), a.k0, a.k1),
                    s_ntab, z0, z1);
    const int d0 = h + 4 * m, d1 = d0 + 4;
    if (GEN && a.pscale) {
      z0 *= a.pscale[min(d0, a.D - 1)];
      z1 *= a.pscale[min(d1, a.D - 1)];
    }
    z0 = d0 < a.D ? z0 : 0.0;
    z1 = d1 < a.D ? z1 : 0.0;
    *reinterpret_cast<double2*>(pm + (c * K + (vec - c * K)) * (4 * M) + 2 * r) = make_double2(z0, z1);
  }
}

// MASS: full (non-diagonal) cov_p (implies GEN): LDS holds the kick matrix inv(cov_p).P
// (stage_precision), p = C z, and every energy takes P x and inv(cov_p) p from two L2 products
// (matvec_global) in converged code.  Its own instantiation, like the dense Random kernel's.
// SHORT: the gradient's short-last-tile form (hmc_dense_ops.hpp), compiled in (kShortAlways) for
// the plain instances at D = 97..100.
template <int MT, bool EXACT, bool GEN, bool REPLAY, bool MASS = false, int SHORT = kShortNever>
__global__ __launch_bounds__(64 * kNutsWaves) __attribute__((amdgpu_waves_per_eu(kNutsWaves / 4, kNutsWaves / 4)))
void k_nuts_iters(RandArgs a) {
  constexpr int M = 4 * MT;
  // ME: the slots that can hold a dimension.  The instance compiled for D = 16(MT-1)+1 .. +4
  // (kShortAlways) needs m <= 4(MT-1) (dims h + 4m < D), rounded up to the 16-byte pairs; every
  // per-slot loop stops there and the slots past it stay zero (D = 100: 26 of 28)
  constexpr int ME = SHORT == kShortAlways ? 4 * (MT - 1) + 2 : M;
  // PG: Philox momenta drawn ahead by k_nuts_momenta (all but the dense-mass instances, whose
  // p = C z needs the tile's MFMA product and keeps the in-kernel draws and their tables)
  constexpr bool PG = !REPLAY && !MASS;
  extern __shared__ double sP[];
  __shared__ double s_ntab[(REPLAY || PG) ? 2 : kNormalTableDoubles];   // Box–Muller tables (MASS momentum)
  if constexpr (!REPLAY && !PG) init_normal_tables(s_ntab);             // synchronised by stage_precision
  stage_precision<MT, SHORT>(a, sP);

  const int lane = threadIdx.x & (kWave - 1);
  const int h = lane >> 4;
  // Persistent waves with a work queue: each of the 16 chain slots of a wave takes (chain,
  // iteration) units from a launch-wide counter, unit u = iteration it0 + u / n of chain u % n, and
  // hands the chain back after that one iteration (one tree).  Slots idle only while the last
  // trees of the launch finish, not the last chains' remaining iterations (lane utilisation).
  // Draws are keyed by (chain, iteration), so results do not depend on which slot or wave runs a
  // tree.  The tree vectors are per slot (W), the tape cursors and hand-off words per chain.
  const int64_t wv = (int64_t)blockIdx.x * kNutsWaves + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t wave_doubles = (int64_t)nuts_nvec(a.d_max) * M * kWave;
  const int64_t n_waves = (a.n + 15) / 16;
  const WaveWS W{__builtin_amdgcn_make_buffer_rsrc(a.ws + wv * wave_doubles, 0, (int)(wave_doubles * 8), 0x00020000),
                 (lane & 15) * nuts_nvec(a.d_max) * (4 * M * 8) + h * 16};
  int64_t* const tcur = reinterpret_cast<int64_t*>(a.ws + n_waves * wave_doubles);
  unsigned long long* const queue = reinterpret_cast<unsigned long long*>(tcur + n_waves * 16);   // zeroed per launch
  unsigned* const done = reinterpret_cast<unsigned*>(queue + 2);    // per chain: iterations done (zeroed per launch)
  const double* const pm = reinterpret_cast<const double*>(queue) + nuts_queue_bytes(a.n) / 8;   // k_nuts_momenta
  const int n_blk = (a.nuts_kb + kNutsBlock - 1) / kNutsBlock;   // block units per chain
  const unsigned long long nb = (unsigned long long)a.n * (unsigned long long)n_blk;
  const unsigned long long n_units = nb + (unsigned long long)a.n * (unsigned long long)(a.it1 - a.it0 - a.nuts_kb);
  uint64_t waited = 0;
  int it_last = 0;                                      // the current unit's last iteration
  int64_t c = 0;
  bool live = false;
  uint64_t gc = 0;

  double q[M], p[M];
  d4 acc[MT];
#pragma unroll
  for (int m = 0; m < M; ++m) q[m] = p[m] = 0.0;
#pragma unroll
  for (int nt = 0; nt < MT; ++nt) acc[nt] = d4{0.0, 0.0, 0.0, 0.0};
  double Eprev = 0.0;
  double maha_old = 0.0, maha_new = 0.0;    // x.g of live_old / live_new points

  int state = (a.it0 < a.it1 && wv < n_waves) ? S_FETCH : S_DONE;   // workspace has n_waves slot blocks
  int it = a.it0;
  int d = 0, k = 0, Lsub = 1, udir = 0, ndraw = 0;
  bool lterm = false, rterm = false;
  double E_init = 0.0, E_max_now = 0.0, E_max_old = 0.0, pi_new = 1.0, pi_old = 1.0;
  int64_t tpos = 0;                                     // replay tape cursor (persists across launches)
  int old2 = 0;                                         // vector offset of the live_point_old pair
  unsigned long long n_lf = 0, n_unst = 0, n_dmax = 0, n_tape = 0, n_steps = 0, n_giveup = 0;
#ifdef HMC_DEBUG_HOOKS
  unsigned long long ph[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_ph = __builtin_amdgcn_s_memtime(), t_sub = t_ph;
#endif

  auto draw = [&](bool direction) -> double {           // next random number of this chain (reference order)
    if constexpr (REPLAY) {
      if (tpos >= a.tape_stride) {                     // exhausted tape: flagged, host raises
        ++n_tape;
        return direction ? 0.0 : 2.0;
      }
      return a.tape[c * a.tape_stride + (tpos++)];
    } else {
      const uint4 r = draw_block(kDrawSlot + (uint32_t)(ndraw++), (uint32_t)it, gc, a.k0, a.k1);
      return direction ? (double)(r.x & 1u) : u53(r.z, r.w);
    }
  };
  auto write_row_of = [&](int i) { return i >= a.wu && ((i == a.niter) || ((i - a.wu + 1) % a.thin == 0)); };

  while (true) {
    // ================= transitions (ITER_END -> ITER_START -> first doubling), converged reductions
    {
      const bool at_end = state == S_ITER_END;
#ifdef HMC_DEBUG_HOOKS
      t_sub = __builtin_amdgcn_s_memtime();
      if (__builtin_amdgcn_ballot_w64(at_end)) ++ph[13];
#endif
      if (at_end) {                                     // samplers.py:786-791: q = live_point_q_old
        vload<M, ME>(W, V_OLD_Q, old2, q);                  // its gradient: recomputed by the slot that
                                                        // takes the chain next (S_GRAD), so the live
                                                        // points keep no gradient vector
        const int qrow = (it - a.wu) / a.thin;
        if (write_row_of(it) && a.qc && qrow >= a.q_row0) {
          double* rowp = a.qc + (c * (int64_t)a.Lq + qrow % a.Lq) * a.D;
#pragma unroll
          for (int m = 0; m < ME; ++m)
            if (h + 4 * m < a.D) rowp[h + 4 * m] = q[m];
        }
        Eprev = E_init;
        if (it < it_last) {                             // a block unit: the same chain's next tree,
          ++it;                                         // no hand-off (q, E_prev and the tape cursor
          if constexpr (PG) {                           // stay in registers), its momentum loaded
            const double* pv = pm + (c * (a.it1 - a.it0) + (it - a.it0)) * (4 * M) + 2 * h;
#pragma unroll
            for (int m = 0; m < ME; m += 2) {
              const double2 z = *reinterpret_cast<const double2*>(pv + 4 * m);
              p[m] = z.x;
              p[m + 1] = z.y;
            }
          }
          state = S_GRAD;                               // gradient at q in the next wave step
        } else {
          state = S_FETCH;                              // hand the chain back after its unit
        }
      }
      NUTS_SUBPHASE(8);
      if (state == S_FETCH && live) {                   // tree done: write the chain's state through
#pragma unroll
        for (int m = 0; m < ME; ++m) {
          const int dd = h + 4 * m;
          if (dd < a.D) st_wt_d(a.q + c * a.D + dd, q[m]);
        }
        if (h == 0) st_wt_d(a.Eprev + c, Eprev);
        if (REPLAY && h == 0) st_wt(tcur + c, tpos);
      }
      if (__builtin_amdgcn_ballot_w64(state == S_FETCH && live)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the state has reached L2/memory ...
#ifndef HMC_NUTS_RELAXED
        // one agent-scope release fence per wave step that publishes (an L2 write-back across
        // XCDs), then relaxed atomic publishes
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (state == S_FETCH && live && h == 0)
          __hip_atomic_store(done + c, (unsigned)(it + 1 - a.it0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
        if (state == S_FETCH && live && h == 0) st_wt(done + c, (unsigned)(it + 1 - a.it0));   // ... then publish
#endif
        if (state == S_FETCH) live = false;
      }
      NUTS_SUBPHASE(9);
      if (__builtin_amdgcn_ballot_w64(state == S_FETCH)) {   // next unit from the queue (converged shuffle;
        const bool fetching = state == S_FETCH;              // skipped in the steps where no slot fetches)
        unsigned long long u = (fetching && h == 0) ? atomicAdd(queue, 1ull) : 0ull;
        u = __shfl(u, lane & 15, kWave);
        if (fetching) {
          if (u < n_units) {
            // units 0 .. nb-1: block b = u / n of chain u % n, kNutsBlock iterations run back to
            // back by this slot (chain affinity); then one unit per (chain, iteration) of the
            // launch's last iterations, iteration-major, so the launch's tail is one tree per slot
            if (u < nb) {
              const int b = (int)(u / (unsigned long long)a.n);
              c = (int64_t)(u % (unsigned long long)a.n);
              it = a.it0 + b * kNutsBlock;
              it_last = a.it0 + min((b + 1) * kNutsBlock, a.nuts_kb) - 1;
            } else {
              const unsigned long long ut = u - nb;
              c = (int64_t)(ut % (unsigned long long)a.n);
              it = a.it0 + a.nuts_kb + (int)(ut / (unsigned long long)a.n);
              it_last = it;
            }
            gc = (uint64_t)(a.chain_offset + c);
            waited = 0;
            state = S_WAIT;
          } else {
            state = S_DONE;
          }
        }
      }
      NUTS_SUBPHASE(10);
      if (state == S_WAIT) {                            // the chain's previous iteration published?
        const unsigned need = (unsigned)(it - a.it0);
        bool ready = need == 0;
        if (!ready) {
#ifndef HMC_NUTS_RELAXED
          // relaxed polls; the acquire fence (an L1 invalidate) once, in the step a poll succeeds
          ready = __hip_atomic_load(done + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need;
          if (__builtin_amdgcn_ballot_w64(ready)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#else
          ready = ld_wt(done + c) >= need;
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the state loads below the poll
#endif
          if (!ready && ++waited > a.wait_cap) {   // broken hand-off: flag it and retire the slot
            ++n_giveup;
            state = S_DONE;
          }
        }
        if (ready) {
          live = true;
#pragma unroll
          for (int m = 0; m < ME; ++m) {
            const int dd = h + 4 * m;
            q[m] = dd < a.D ? ld_wt_d(a.q + c * a.D + dd) : 0.0;
          }
          Eprev = ld_wt_d(a.Eprev + c);
          tpos = REPLAY ? ld_wt(tcur + c) : 0;
          if constexpr (PG) {                           // this iteration's momentum, with the state
            const double* pv = pm + (c * (a.it1 - a.it0) + (it - a.it0)) * (4 * M) + 2 * h;
#pragma unroll
            for (int m = 0; m < ME; m += 2) {
              const double2 z = *reinterpret_cast<const double2*>(pv + 4 * m);
              p[m] = z.x;
              p[m + 1] = z.y;
            }
          }
          state = S_GRAD;                               // gradient at q in the next wave step
        }
      }
      NUTS_SUBPHASE(11);
      const bool starting = state == S_ITER_START;
      double kin = 0.0;
      if (starting) {   // momentum (:565), dims h+4m, streamed to the boundaries: right = p, left = -p (:581-584)
        if constexpr (REPLAY) {
          const double* row = a.rp + (c * (int64_t)a.niter + (it - 1)) * a.D;
#pragma unroll
          for (int m = 0; m < ME; ++m) {
            const double z = (h + 4 * m < a.D) ? row[h + 4 * m] : 0.0;
            p[m] = z;
            if constexpr (MASS) continue;               // K after the products below
            kin += z * (dim_minv<MT, GEN>(a, h + 4 * m) * z);
          }
        } else if constexpr (PG) {                     // p loaded with the chain's state (S_WAIT)
#pragma unroll
          for (int m = 0; m < ME; m += 2) {
            const double z0 = p[m], z1 = p[m + 1];
            kin += z0 * (dim_minv<MT, GEN>(a, h + 4 * m) * z0);
            kin += z1 * (dim_minv<MT, GEN>(a, h + 4 * m + 4) * z1);
          }
        } else {
#pragma unroll
          for (int m = 0; m < ME; m += 2) {
            double z0, z1;
            normal_pair_tab(draw_block((uint32_t)(h + 4 * m), (uint32_t)it, gc, a.k0, a.k1), s_ntab, z0, z1);
            const int d0 = h + 4 * m, d1 = d0 + 4;
            if (GEN && a.pscale) {
              z0 *= a.pscale[min(d0, a.D - 1)];
              z1 *= a.pscale[min(d1, a.D - 1)];
            }
            z0 = d0 < a.D ? z0 : 0.0;
            z1 = d1 < a.D ? z1 : 0.0;
            p[m] = z0;
            p[m + 1] = z1;
            if constexpr (!MASS) {
              kin += z0 * (dim_minv<MT, GEN>(a, d0) * z0);
              kin += z1 * (dim_minv<MT, GEN>(a, d1) * z1);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      if constexpr (MASS) {                             // converged: the products need every lane
        if (__builtin_amdgcn_ballot_w64(starting)) {
          d4 t[MT];
          double pc[M];
          if constexpr (!REPLAY) {                      // p = C z ~ N(0, cov_p) (samplers.py:829)
            matvec_global<MT>(a.cholt, a.D, lane, p, t);
#pragma unroll
            for (int m = 0; m < ME; ++m) pc[m] = (h + 4 * m < a.D) ? gval<MT>(t, m) : 0.0;
          } else {
#pragma unroll
            for (int m = 0; m < ME; ++m) pc[m] = p[m];
          }
          matvec_global<MT>(a.minvf, a.D, lane, pc, t);
          double kk = 0.0;
#pragma unroll
          for (int m = 0; m < ME; ++m) kk = mac<EXACT>(kk, pc[m], gval<MT>(t, m));
          if (starting) {
            kin = kk;
#pragma unroll
            for (int m = 0; m < ME; ++m) p[m] = pc[m];
          }
        }
      }
      kin = chain_sum4(kin);
      if (starting) {                                   // E_initial (:569), E/dE storage (:571-573)
        E_init = 0.5 * (a.logc + (maha_old + kin));
        if (write_row_of(it) && h == 0) {
          const int64_t row = c * (int64_t)a.Lc + (it - a.wu) / a.thin;
          if (a.Ec) a.Ec[row] = E_init;
          if (a.dEc) a.dEc[row] = E_init - Eprev;
        }
        vstore<M, ME>(W, V_OLD_Q, old2, q);                 // live_point_q_old = q (:577)
        E_max_old = E_init;
        pi_old = 1.0;
        d = 0;
        lterm = rterm = false;
        ndraw = 0;
        // first doubling (:595-626), d = 0: its direction (:608) first, so that only the end it
        // does not extend is stored (left = (q, -p), right = (q, p), :581-584); the end it extends
        // is written at the sub-tree's end, before anything reads it
        Lsub = 1;
        udir = (int)draw(true);
        const int o = udir == 0 ? V_LEFT_Q : V_RIGHT_Q;
        vstore<M, ME>(W, 0, o, q);
        vstore_sg<M, ME>(W, 1, o, p, udir == 0 ? -1.0 : 1.0);
        gstore<MT, ME>(W, 2, o, acc);
        if (udir != 0) {                                // the doubling runs from (q, -p)
#pragma unroll
          for (int m = 0; m < ME; ++m) p[m] = -p[m];
        }
        k = 0;
        state = S_READY;
      }
      NUTS_SUBPHASE(12);
    }
    if (!__builtin_amdgcn_ballot_w64(state != S_DONE)) break;
    NUTS_PHASE(0);

    // ================= one leapfrog for every chain inside a sub-tree (:612-614, :639)
    // chains outside a sub-tree are frozen by the EXEC mask of a divergent block (no per-dim
    // selects); the MFMAs and the reductions run with all lanes
    // The last U-turn check of an even point m is against point m - 1 (check_points(m) ends with
    // m - 1), which is the point in registers before this leapfrog: dq = q_m - q_{m-1} (the same
    // subtraction the saved-vector check would do) and B = dq.p_{m-1} are formed here, A = dq.p_m
    // after the second half kick, so that check loads nothing and points l = 3 (mod 4), which
    // check_points only names at m = l + 1, are never saved.
    const bool act = state == S_READY;
    // FAST: dq = q_m - q_{m-1} is dt p_half up to the rounding of q, and the U-turn tests read only
    // the signs of the dots, so regB = dt (p_half . p_{m-1}) and regA = dt (p_half . p_m) are formed
    // inside the two half kicks: no dq vector lives across the gradient (56 registers at D = 100).
    // EXACT keeps the reference's subtraction.
    constexpr bool DQV = EXACT;
    const bool dtv = GEN && a.dtv;                      // per-dimension dt: scale each term
    double dq[DQV ? M : 1], regB = 0.0, regA = 0.0;
#pragma unroll
    for (int m = 0; m < (DQV ? M : 1); ++m) dq[m] = 0.0;
    if (act) {
#pragma unroll
      for (int m = 0; m < ME; ++m) {
        const int dd = h + 4 * m;
        const double dt = dim_dt<MT, GEN>(a, dd), mi = dim_minv<MT, GEN>(a, dd);
        const double pk = p[m], qk = q[m];
        if constexpr (EXACT) {
          p[m] = p[m] - (dt * (mi * gval<MT>(acc, m))) * 0.5;
          q[m] = q[m] + dt * p[m];
          dq[m] = q[m] - qk;
          regB = mac<EXACT>(regB, dq[m], pk);
        } else {
          p[m] = __builtin_fma(-0.5 * dt * mi, gval<MT>(acc, m), p[m]);
          q[m] = __builtin_fma(dt, p[m], q[m]);
          regB = __builtin_fma(dtv ? dt * p[m] : p[m], pk, regB);
        }
        if ((m & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
    }
    NUTS_PHASE(1);
    gradient<MT, GEN, true, SHORT>(a, sP, lane, h, q, acc);
    NUTS_PHASE(2);
    if (act) {
#pragma unroll
      for (int m = 0; m < ME; ++m) {
        const int dd = h + 4 * m;
        const double dt = dim_dt<MT, GEN>(a, dd), mi = dim_minv<MT, GEN>(a, dd);
        if constexpr (EXACT) {
          p[m] = p[m] - (dt * (mi * gval<MT>(acc, m))) * 0.5;
        } else {
          const double ph = p[m];
          p[m] = __builtin_fma(-0.5 * dt * mi, gval<MT>(acc, m), ph);
          regA = __builtin_fma(dtv ? dt * ph : ph, p[m], regA);
        }
        if ((m & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
    }
    double mp1 = 0.0, kp1 = 0.0;
    if constexpr (DQV) {
#pragma unroll
      for (int m = 0; m < ME; ++m) regA = mac<EXACT>(regA, dq[m], p[m]);
    } else if (!dtv) {
      regA *= a.dt;
      regB *= a.dt;
    }
    if constexpr (MASS) {                               // x.P.x and p.inv(cov_p).p (acc holds the kick)
      double xv[M];
      d4 t[MT];
#pragma unroll
      for (int m = 0; m < ME; ++m) xv[m] = a.q0 ? q[m] - a.q0[min(h + 4 * m, a.D - 1)] : q[m];
      matvec_global<MT>(a.prec, a.D, lane, xv, t);
#pragma unroll
      for (int m = 0; m < ME; ++m) mp1 = mac<EXACT>(mp1, xv[m], gval<MT>(t, m));
      matvec_global<MT>(a.minvf, a.D, lane, p, t);
#pragma unroll
      for (int m = 0; m < ME; ++m) kp1 = mac<EXACT>(kp1, p[m], gval<MT>(t, m));
    } else {
#pragma unroll
      for (int m = 0; m < ME; ++m) {
        const int dd = h + 4 * m;
        const double mi = dim_minv<MT, GEN>(a, dd);
        mp1 = mac<EXACT>(mp1, (GEN && a.q0) ? q[m] - a.q0[min(dd, a.D - 1)] : q[m], gval<MT>(acc, m));
        kp1 = mac<EXACT>(kp1, p[m], mi * p[m]);
        if ((m & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
    }
    const double maha_pt = chain_sum4(mp1);
    const double E_tmp = 0.5 * (a.logc + (maha_pt + chain_sum4(kp1)));   // E (:618 / :643)
    if (state == S_GRAD) {                              // fetched chain: acc = gradient at its q
      maha_old = maha_pt;
      state = S_ITER_START;
    }
    if (act && h == 0) ++n_lf;
    ++n_steps;
    NUTS_PHASE(3);

    // ================= process the new point
    bool reject = false, sub_end = false;
    const int mpt = k + 1;                              // point number within the sub-tree
    const bool first = act && k == 0, later = act && k > 0;
    if (first) {                                        // first point (:617-626)
      vstore<M, ME>(W, V_OLD_Q, 2 - old2, q);               // live_point_new (the other buffer pair)
      maha_new = maha_pt;
      E_max_now = E_tmp;
      pi_new = 1.0;
      vstore<M, ME>(W, V_SLOTS, 2 * a.d_max, q);            // point 1: save_slot(1)
      vstore<M, ME>(W, V_SLOTS + 1, 2 * a.d_max, p);
      k = 1;
      sub_end = Lsub == 1;
    } else if (later) {
      if (fabs(E_tmp - E_init) > 1000.0) {              // :647-651
        reject = true;
        if (h == 0) ++n_unst;
      } else if ((mpt & 3) == 1) {                      // odd point: save (:654-658); 3 (mod 4): see dq
        const int s = save_slot(mpt, a.d_max);
        vstore<M, ME>(W, V_SLOTS, 2 * s, q);
        vstore<M, ME>(W, V_SLOTS + 1, 2 * s, p);
      }
    }
    NUTS_PHASE(4);
    // even point: sub-tree U-turn checks against check_points(mpt) (:699-736), converged loop
    const bool checking = later && !reject && (mpt & 1) == 0;
    {                                                   // the check against point mpt - 1, from registers
      const double r_dot = chain_sum4(udir == 0 ? regA : regB);
      const double l_dot = chain_sum4(udir == 0 ? regB : regA);
      if (checking && l_dot < 0.0 && r_dot < 0.0) reject = true;
    }
    const int ncheck = checking && !reject ? cp_count(mpt) - 1 : 0;   // the saved check points
    const int ncheck_w = wave_max_i32(ncheck);
    bool alive_chk = ncheck > 0;
    // check points of mpt, incrementally (cp_point): mpt - r + 1, then + r/2, + r/4, ...
    int cp_half = checking ? cp_r(mpt) : 2;
    int cp_pt = mpt - cp_half + 1;
    for (int ci = 0; ci < ncheck_w; ++ci) {
      const bool doit = alive_chk && ci < ncheck;
      if (ci > 0) {
        cp_half >>= 1;
        cp_pt += cp_half;
      }
      const int l = doit ? cp_pt : 1;
      const int s = save_slot(l, a.d_max);              // retrieve_save_index (:715)
      double r_dot = 0.0, l_dot = 0.0;
      if (doit) {
        double qcv[M], pcv[M];
        vload<M, ME>(W, V_SLOTS, 2 * s, qcv);
        vload<M, ME>(W, V_SLOTS + 1, 2 * s, pcv);
        // forward: left = (q_check, -p_check), right = (q, p); backward: left = (q, p),
        // right = (q_check, -p_check).  Both directions reduce to A = (q - qc).p and
        // B = (q - qc).p_check (every sign flip is exact): r_dot, l_dot = (A, B) forward, (B, A)
        // backward, term for term the reference's products.
        double A = 0.0, B = 0.0;
#pragma unroll
        for (int m = 0; m < ME; ++m) {
          const double Dq = q[m] - qcv[m];
          A = mac<EXACT>(A, Dq, p[m]);
          B = mac<EXACT>(B, Dq, pcv[m]);
        }
        r_dot = udir == 0 ? A : B;
        l_dot = udir == 0 ? B : A;
      }
      r_dot = chain_sum4(r_dot);
      l_dot = chain_sum4(l_dot);
      if (doit) {
        if (l_dot < 0.0 && r_dot < 0.0) {               // :727-732
          reject = true;
          alive_chk = false;
        }                                               // (release, :735-736: nothing to free)
      }
    }
    NUTS_PHASE(5);
    if (later && !reject) {                             // progressive sampling (:743-751)
      const double E_max_prev = E_max_now;
      E_max_now = fmax(E_max_prev, E_tmp);
      // exp(-(E_tmp - E_max_now)) and exp(E_max_now - E_max_prev): one argument is exactly 0
      // (E_max_now is one of E_tmp, E_max_prev), so one exp and exp(0) = 1, as the reference
      // (NaN energies give the same NaN r as the two exps)
      const bool up = E_max_now != E_max_prev;
      const double e = exp(up ? E_max_now - E_max_prev : -(E_tmp - E_max_now));
      const double num = up ? 1.0 : e;
      pi_new = num + (up ? e : 1.0) * pi_new;
      const double r = num / pi_new;
      if (draw(false) < r) {
        vstore<M, ME>(W, V_OLD_Q, 2 - old2, q);
        maha_new = maha_pt;
      }
      ++k;
      sub_end = k == Lsub;
    }
    if (act && reject) state = S_ITER_END;               // q = live_point_q_old (:649, :731)
    NUTS_PHASE(6);

    // ================= sub-tree end: boundary, biased acceptance, termination (:757-784)
    // The other end (q, p, g) is loaded here for the termination dots; a next doubling towards it
    // starts from these registers (no separate boundary-load step).  The chain sums run inside
    // this divergent block: v_permlane16/32_swap pair lanes c, c^16, c^32 of the same chain, which
    // are active together.
    if (sub_end) {
      double oqv[M], opv[M];
      d4 og[MT];
      const int b = udir == 0 ? V_RIGHT_Q : V_LEFT_Q;    // this end <- (q, p)
      const int o = udir == 0 ? V_LEFT_Q : V_RIGHT_Q;   // the other end
      // the other end's loads first: the stores behind them in the in-order vmcnt queue do not
      // delay the wait for the loads (b != o, so the order changes nothing else)
      vload<M, ME>(W, 0, o, oqv);
      vload<M, ME>(W, 1, o, opv);
      gload<MT, ME>(W, 2, o, og);
      vstore<M, ME>(W, 0, b, q);
      vstore<M, ME>(W, 1, b, p);
      gstore<MT, ME>(W, 2, b, acc);
      const double r = exp(-(E_max_now - E_max_old)) * pi_old / pi_new;   // :766 (Q11)
      const double E_max_old_prev = E_max_old;
      E_max_old = fmax(E_max_old_prev, E_max_now);
      pi_old = exp(-(E_max_now - E_max_old)) * pi_new + exp(-(E_max_old_prev - E_max_old)) * pi_old;
      const double A = fmin(1.0, r);
      if (draw(false) < A) {                            // :773-775: old <- new, as a buffer swap
        old2 = 2 - old2;
        maha_old = maha_new;
      }
      // A = (q - q_other).p, B = (q - q_other).p_other; (tr, tl) = (A, -B) forward, (-B, A)
      // backward: the reference's terms up to exact sign flips
      double tA = 0.0, tB = 0.0;
#pragma unroll
      for (int m = 0; m < ME; ++m) {
        const double Dq = q[m] - oqv[m];
        tA = mac<EXACT>(tA, Dq, p[m]);
        tB = mac<EXACT>(tB, Dq, opv[m]);
      }
      const double tr = chain_sum4(udir == 0 ? tA : -tB);
      const double tl = chain_sum4(udir == 0 ? -tB : tA);
      // :779-784 (Q10: stop when BOTH ends turn)
      rterm = tr < 0.0;
      lterm = tl < 0.0;
      ++d;
      if (lterm && rterm) {
        state = S_ITER_END;
      } else if (d > a.d_max - 1) {                     // :596-598 (the reference aborts the run)
        ++n_dmax;
        state = S_ITER_END;
      } else {                                          // next doubling: its direction (:608) now
        Lsub = 1 << d;
        const int nd = (int)draw(true);
        if (nd != udir) {                               // the other end, loaded above
          udir = nd;
#pragma unroll
          for (int m = 0; m < ME; ++m) {
            q[m] = oqv[m];
            p[m] = opv[m];
          }
#pragma unroll
          for (int nt = 0; nt < MT; ++nt) acc[nt] = og[nt];
        }                                               // (same end: (q, p, acc) in registers)
        k = 0;
        state = S_READY;
      }
    }
    NUTS_PHASE(7);
  }
#ifdef HMC_DEBUG_HOOKS
  if (a.stamps && lane == 0 && wv < n_waves) {   // g_stamps has one row per workspace wave
#pragma unroll
    for (int i = 0; i < 14; ++i) a.stamps[wv * kStampWords + i] = ph[i];
  }
#endif

  // counters (every chain's state was written back when its slot fetched the next one)
  n_lf = wave_sum_u64(n_lf);
  n_unst = wave_sum_u64(n_unst);
  n_dmax = wave_sum_u64(h == 0 ? n_dmax : 0ull);
  n_tape = wave_sum_u64(h == 0 ? n_tape : 0ull);
  n_giveup = wave_sum_u64(h == 0 ? n_giveup : 0ull);
  if (lane == 0 && a.cnt) {
    unsigned long long* cs = a.cnt + (wv & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
    if (n_lf) {
      atomicAdd(cs + HMC_CNT_LEAPFROG, n_lf);
      atomicAdd(cs + HMC_CNT_ENERGY_EVALS, n_lf);
    }
    if (n_unst) atomicAdd(cs + HMC_CNT_UNSTABLE, n_unst);
    if (n_dmax) atomicAdd(cs + HMC_CNT_DMAX, n_dmax);
    if (n_tape) atomicAdd(cs + HMC_CNT_OOB_REJECT, n_tape);   // NUTS: replay tape exhausted
    if (n_giveup) atomicAdd(cs + HMC_CNT_HANDOFF_GIVEUP, n_giveup);   // broken chain hand-offs (must be 0)
    atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, n_steps);               // NUTS: wave steps (lane utilisation)
  }
}

template <int MT, bool EXACT>
hipError_t launch_nuts_mt3(const RandArgs& args, bool gen, bool replay, hipStream_t s);

// Launches of at most kNutsMomIters iterations, each after its momenta (Philox, diagonal cov_p).
template <int MT, bool EXACT>
hipError_t launch_nuts_mt2(const RandArgs& args, bool gen, bool replay, hipStream_t s) {
  if (replay || args.minvf) return launch_nuts_mt3<MT, EXACT>(args, gen, replay, s);
  const int64_t n_waves = (args.n + 15) / 16;
  const int64_t wave_doubles = (int64_t)(V_SLOTS + 2 * (args.d_max + 1)) * 4 * MT * kWave;
  double* pm = args.ws + n_waves * wave_doubles + n_waves * 16 + nuts_queue_bytes(args.n) / 8;
  for (int i0 = args.it0; i0 < args.it1; i0 += kNutsMomIters) {
    RandArgs a = args;
    a.it0 = i0;
    a.it1 = std::min(args.it1, i0 + kNutsMomIters);
    const int64_t slots = a.n * (a.it1 - a.it0) * (8 * MT);
    const dim3 mgrid((unsigned)std::max<int64_t>(1, std::min<int64_t>((slots + 255) / 256, (int64_t)device_cus() * 8)));
#ifndef HMC_NUTS_DEV_C5
    if (gen) k_nuts_momenta<MT, true><<<mgrid, 256, 0, s>>>(a, pm);
    else
#endif
      k_nuts_momenta<MT, false><<<mgrid, 256, 0, s>>>(a, pm);
    if (hipError_t e = hipGetLastError()) return e;
    if (hipError_t e = launch_nuts_mt3<MT, EXACT>(a, gen, replay, s)) return e;
  }
  return hipSuccess;
}

template <int MT, bool EXACT>
hipError_t launch_nuts_mt3(const RandArgs& args, bool gen, bool replay, hipStream_t s) {
  RandArgs a = args;
  // persistent: one block per CU (LDS: P + index tables), chains handed out by the queue
  const int64_t blocks = (a.n + 16 * kNutsWaves - 1) / (16 * kNutsWaves);
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)device_cus())));
  const int64_t n_waves = (a.n + 15) / 16;
  const int64_t wave_doubles = (int64_t)(V_SLOTS + 2 * (a.d_max + 1)) * 4 * MT * kWave;
  double* queue = a.ws + n_waves * wave_doubles + n_waves * 16;   // queue head, (unused), done[n]
  if (hipError_t e = hipMemsetAsync(queue, 0, nuts_queue_bytes(a.n), s)) return e;
  // chain affinity: all but the launch's last kNutsTail iterations run in kNutsBlock-tree units
  a.nuts_kb = kNutsBlock > 1 ? std::max(0, (a.it1 - a.it0) - kNutsTail) : 0;
  a.wait_cap = nuts_wait_cap((int64_t)grid.x * kNutsWaves * 16, a.n, a.d_max, std::min(a.nuts_kb, kNutsBlock));
  const size_t lds = (size_t)MT * 4 * MT * kWave * sizeof(double);
#ifdef HMC_NUTS_DEV_C5
  if constexpr (MT == 7 && !EXACT) k_nuts_iters<MT, EXACT, false, false, false, kShortAlways><<<grid, 64 * kNutsWaves, lds, s>>>(a);
  return hipGetLastError();
#endif
  if (a.minvf) {
    if (replay) k_nuts_iters<MT, EXACT, true, true, true><<<grid, 64 * kNutsWaves, lds, s>>>(a);
    else k_nuts_iters<MT, EXACT, true, false, true><<<grid, 64 * kNutsWaves, lds, s>>>(a);
  } else if (gen) {
    if (replay) k_nuts_iters<MT, EXACT, true, true><<<grid, 64 * kNutsWaves, lds, s>>>(a);
    else k_nuts_iters<MT, EXACT, true, false><<<grid, 64 * kNutsWaves, lds, s>>>(a);
  } else {
    bool done = false;
    if constexpr (MT == 7) {
      if (a.D <= 16 * (MT - 1) + 4) {                   // D = 97..100 (c5: D = 100)
        if (replay) k_nuts_iters<MT, EXACT, false, true, false, kShortAlways><<<grid, 64 * kNutsWaves, lds, s>>>(a);
        else k_nuts_iters<MT, EXACT, false, false, false, kShortAlways><<<grid, 64 * kNutsWaves, lds, s>>>(a);
        done = true;
      }
    }
    if (!done) {
      if (replay) k_nuts_iters<MT, EXACT, false, true><<<grid, 64 * kNutsWaves, lds, s>>>(a);
      else k_nuts_iters<MT, EXACT, false, false><<<grid, 64 * kNutsWaves, lds, s>>>(a);
    }
  }
  return hipGetLastError();
}

template <int MT>
hipError_t launch_nuts_mt(const RandArgs& a, bool exact, bool gen, bool replay, hipStream_t s) {
  return exact ? launch_nuts_mt2<MT, true>(a, gen, replay, s) : launch_nuts_mt2<MT, false>(a, gen, replay, s);
}

}  // namespace

int64_t nuts_ws_doubles(int64_t n, int D, int d_max, int mom_iters) {
  const int MT = dense_tiles(D);
  const int64_t waves = (n + 15) / 16;
  // vectors + tape cursors + work queue (head, spare, per-chain iterations done) + the Philox
  // momenta drawn ahead (diagonal cov_p only) for min(32, iterations per call) iterations
  return waves * (int64_t)(V_SLOTS + 2 * (d_max + 1)) * 4 * MT * kWave + waves * 16 + nuts_queue_bytes(n) / 8 +
         nuts_mom_doubles(n, MT, mom_iters);
}

#ifdef HMC_NUTS_DEV_C5
// dev-only build of the c5 instance alone (seconds instead of minutes per A/B compile): objdump /
// register checks; not a usable library
hipError_t launch_nuts_iters(const RandArgs& a, bool, bool, hipStream_t s) { return launch_nuts_mt2<7, false>(a, false, false, s); }
#else
hipError_t launch_nuts_iters(const RandArgs& a, bool exact, bool replay, hipStream_t s) {
  const bool gen = a.q0 || a.minv || a.pscale || a.dtv || a.minvf;
  switch (dense_tiles(a.D)) {
    case 1: return launch_nuts_mt<1>(a, exact, gen, replay, s);
    case 2: return launch_nuts_mt<2>(a, exact, gen, replay, s);
    case 4: return launch_nuts_mt<4>(a, exact, gen, replay, s);
    case 7: return launch_nuts_mt<7>(a, exact, gen, replay, s);
    case 8: return launch_nuts_mt<8>(a, exact, gen, replay, s);
  }
  return hipErrorInvalidValue;
}
#endif

}  // namespace hmc
