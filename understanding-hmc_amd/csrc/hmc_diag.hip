// hmc_diag.hip — convergence diagnostics on the device (utils.py:77-179; samplers.py:213, :246).
//
// The reference's convergence_stats splits every chain into two halves
// (utils.py:88-104), then needs, per dimension:
//   * per split chain j: mean_j and std_j (ddof=1)             -> k_split_moments
//   * sums over j of std_j, mean_j, (mean_j - mean_all)^2        -> k_rowsum (two-stage, deterministic)
//   * variogram sums  sum_j sum_s (x_j[s+t] - x_j[s])^2, t = lags -> k_variogram (two-stage)
// Everything is additive over chains, so on several GPUs each rank reduces its own
// chains and one small all-reduce combines the per-dimension sums.
// Chains are read in place through strides: element (chain m, sample s, dim d) sits at
//   x[base + m*chain_stride + s*sample_stride + d]
// which covers q_chain[:, 1:, :], warm-up offsets and thinning without copies.
#include <type_traits>
#include <utility>

#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {

namespace {

constexpr int kRowChunk = 256;   // rows per partial-sum block
constexpr int kDimTile = 64;     // dims per block (lane = dim: coalesced row reads)

struct Src {
  const double* x;
  int64_t chain_stride, sample_stride, base;
  int64_t n_chains;
  int n, D;
  // series per chain: 2 = the split chains j = 2m + h of convergence_stats (half h starts h*n
  // samples in); 1 = one series per chain (a completed half of a streaming window: series j =
  // chain j, its sample s in window row (slot0 + s) % wrap, wrap 0 = row s)
  int halves = 2;
  int wrap = 0, slot0 = 0;
};

__host__ __device__ __forceinline__ int64_t n_series(const Src& s) { return s.halves * s.n_chains; }

__device__ __forceinline__ const double* split_ptr(const Src& s, int64_t j, int smp) {
  if (s.halves == 1) return s.x + s.base + j * s.chain_stride + (int64_t)smp * s.sample_stride;
  const int64_t m = j >> 1;
  const int h = (int)(j & 1);
  return s.x + s.base + m * s.chain_stride + (int64_t)(h * s.n + smp) * s.sample_stride;
}

// One thread per (split chain j, dim d): two-pass mean and std (ddof = 1, numpy np.std(ddof=1)).
__global__ __launch_bounds__(256) void k_split_moments(Src s, double* mean_out, double* std_out) {
  const int d = blockIdx.y * kDimTile + (threadIdx.x & (kDimTile - 1));
  const int64_t j = (int64_t)blockIdx.x * (256 / kDimTile) + (threadIdx.x / kDimTile);
  if (d >= s.D || j >= 2 * s.n_chains) return;
  double sum = 0.0;
  for (int t = 0; t < s.n; ++t) sum += split_ptr(s, j, t)[d];
  const double mean = sum / s.n;
  double m2 = 0.0;
  for (int t = 0; t < s.n; ++t) {
    const double e = split_ptr(s, j, t)[d] - mean;
    m2 += e * e;
  }
  mean_out[j * s.D + d] = mean;
  std_out[j * s.D + d] = sqrt(m2 / (s.n - 1));
}

struct Rows {
  const double* x;
  int64_t n_outer, outer_stride, n_inner, inner_stride, base;
  int D;
  const double* center;  // null: plain sum; else sum of (x - center_d)^2
};

// partial[chunk][d] = sum over the chunk's rows.  Block = 4 row-lanes x 64 dims.
__global__ __launch_bounds__(256) void k_rowsum_partial(Rows r, double* partial) {
  __shared__ double red[4][kDimTile];
  const int dl = threadIdx.x & (kDimTile - 1);
  const int rl = threadIdx.x / kDimTile;
  const int d = blockIdx.y * kDimTile + dl;
  const int64_t rows = r.n_outer * r.n_inner;
  const int64_t r0 = (int64_t)blockIdx.x * kRowChunk;
  double acc = 0.0;
  if (d < r.D) {
    const double c = r.center ? r.center[d] : 0.0;
    for (int i = rl; i < kRowChunk; i += 4) {
      const int64_t row = r0 + i;
      if (row >= rows) break;
      const int64_t o = row / r.n_inner, in = row - o * r.n_inner;
      const double v = r.x[r.base + o * r.outer_stride + in * r.inner_stride + d];
      if (r.center) {
        const double e = v - c;
        acc += e * e;
      } else {
        acc += v;
      }
    }
  }
  red[rl][dl] = acc;
  __syncthreads();
  if (rl == 0 && d < r.D)
    partial[(int64_t)blockIdx.x * r.D + d] = ((red[0][dl] + red[1][dl]) + red[2][dl]) + red[3][dl];
}

// out[c] = sum_k partial[k][c] for c < ncols (fixed order: deterministic).
__global__ __launch_bounds__(256) void k_colsum_final(const double* partial, int64_t nchunks, int64_t ncols,
                                                      double* out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  double acc = 0.0;
  for (int64_t k = 0; k < nchunks; ++k) acc += partial[k * ncols + c];
  out[c] = acc;
}

// out[c] += sum_k partial[k][c] (fixed order: deterministic; accumulates across calls).
__global__ __launch_bounds__(256) void k_colsum_acc(const double* partial, int64_t nchunks, int64_t ncols,
                                                    double* out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  double acc = 0.0;
  for (int64_t k = 0; k < nchunks; ++k) acc += partial[k * ncols + c];
  out[c] += acc;
}

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)x >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)x));
}
template <class T>
__device__ __forceinline__ T* uni(T* p) {
  return reinterpret_cast<T*>(uni((int64_t)(uintptr_t)p));
}

// f(std::integral_constant<int, r>) for the runtime r in [0, N): a uniform branch to one of N
// statically indexed bodies
template <class F, int... I>
__device__ __forceinline__ void static_dispatch_(int r, F& f, std::integer_sequence<int, I...>) {
  ((r == I ? f(std::integral_constant<int, I>{}) : void()), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_dispatch(int r, F& f) {
  static_dispatch_(r, f, std::make_integer_sequence<int, N>{});
}
// f(std::integral_constant<int, i>) for i = 0 .. N-1 in order: a source-level unroll (bodies too
// large for the loop unroller's pragma threshold)
template <class F, int... I>
__device__ __forceinline__ void static_for_(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F& f) {
  static_for_(f, std::make_integer_sequence<int, N>{});
}

// ---- The variogram lag sums and split-chain moments of convergence_stats (utils.py:88-126,
// :161-179) in ONE read of the samples, for any lag range.
//
// A *series* is one dimension d of one split chain j (n samples), flattened e = j*D + d; a wave
// owns 64 consecutive series (a tile: every lane busy whatever D; rows of a split chain are
// contiguous, so a wave's row load is one or two coalesced segments) and walks their n samples
// once.  Per series, with y = x - x_j[0] (shifted: well-conditioned sums),
//   V_t = sum_{s=t}^{n-1} (y_s - y_{s-t})^2 = 2 S2 - P(t) - Q(t) - 2 C_t,
//   C_t = sum_s y_s y_{s-t},  P(t) = sum_{s<t} y_s^2,  Q(t) = sum_{s>=n-t} y_s^2,
// so a lag costs ONE FMA per sample against a register ring of TL delayed samples.  A wave takes
// the TL lags t = gofs + 1 .. gofs + TL (lag group g: gofs = L0 + g*TL); its ring is fed by the
// sample stream delayed by gofs (the stream itself for gofs = 0).  Rows run in unrolled chunks of
// TL from row gofs, so ring slots are static registers:
//   * chunk 0 is the ramp: lag k of row i only meets the slots already written (k < i), so the
//     products with samples before the series start are never issued -- the pass costs the
//     triangle sum_t (n - t) of the reference's loop, not n*T -- and row i's running S2 is P(t);
//   * the delayed stream's squares over the run are P(n - gofs), from which Q(t) follows with the
//     ring's final contents (the last TL delayed samples);
//   * rows 0 .. gofs - 1 (lag groups with gofs > 0) only add their squares to S2.
// Lag group 0 of a first pass (L0 = 0) also sums the moments (mean_j: the samples added in order
// without FMA, NumPy's np.mean over axis 0 bit for bit; std_j (ddof 1) from S2 and s1) and the
// lag n - 1 the ESS loop reads last.
// Determinism: a wave owns the tiles tau = c + C (r + R i) of one class c (C = D / gcd(D, 64): lane
// l of every such tile holds dimension (64 c + l) mod D) and sums them in order in its lanes;
// k_lag_classes / k_lag_dims add the waves' lanes per dimension in a fixed order.  Wave ids are
// XCD-major (blocks b, b + 8, ... share an XCD): the lag groups of one (class, replica) run on the
// same XCD, so the rows one group reads are L2 hits for the others.
#ifndef HMC_LAG_TL
#define HMC_LAG_TL 48
#endif
#ifndef HMC_LAG_PF
#define HMC_LAG_PF 16
#endif
#ifndef HMC_LAG_WPE
#define HMC_LAG_WPE 1
#endif
// Lags per wave, rows in flight per stream and waves per SIMD.  One wave per SIMD with the whole
// register file, 48 lags (n = 50, the bench window, needs lags 1..48 + n - 1: one wave per tile) and
// 16 rows in flight measured best on the bench window (29 ms; 32 lags at two waves per SIMD: 65 ms,
// 53 ms with the ragged rows masked instead of branched; 48 lags at two waves per SIMD spill).
constexpr int kLagTL = HMC_LAG_TL;
constexpr int kLagPF = HMC_LAG_PF;   // divides kLagTL
// Tail lags: a first pass (mom) also sums the last `tail` <= kLagTail lags n - k, k = 1 .. tail, in
// difference form, V_{n-k} = sum_{i<k} (y_{n-k+i} - y_i)^2 (k terms each: rows 0 .. tail-1 and the
// last tail rows).  A complete pass then needs the lag groups only for lags 1 .. n - 1 - tail:
// n = 99 (c4's halves) takes two groups of 48 and a tail of 2 instead of a third group that would
// read every row again for one lag.
constexpr int kLagTail = 8;
// partial rows per wave: std, mean - S, (mean - S)^2, the tail lags n-1 .. n-kLagTail, the lag group
constexpr int kLagRows = kLagTL + 3 + kLagTail;
constexpr int kLagWaves = 8192;        // target waves per pass (4 rounds of 2 waves per SIMD)
constexpr int kLagOOB = 0x40000000;    // buffer bound: lanes past the last series read zeros

struct LagArgs {
  Src s;
  int L0;          // lags L0 + 1 .. L0 + T (L0 a multiple of kLagPF)
  int T;           // lags of this pass
  int G;           // lag groups, ceil(T / TL)
  int C, R;        // classes, replicas per class
  int mom;         // group 0 sums the moments and the tail lags (first pass)
  int tail;        // mom: tail lags n-1 .. n-tail (1 <= tail <= kLagTail)
  int64_t NT;      // tiles of 64 series
  int rowb;        // bytes between samples (sample_stride * 8)
};

__host__ __device__ inline int lag_gcd(int a, int b) {
  while (b) {
    const int t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// The tiles of one wave.  Z: the lag group starts at lag 1 (gofs = 0: the ring is fed by the
// stream itself; also the moments), else gofs > 0 (a second, delayed stream).  The two forms are
// separate non-inlined functions so that each gets its own register allocation (one kernel
// holding both spilled at 256 registers).
// WR: one series per chain in a circular window (Src::halves == 1, wrap > 0): sample s of every
// series sits in window row (slot0 + s) % wrap, so row offsets wrap (scalar arithmetic per load);
// the tile's buffer descriptor is based at the chain's window row 0.
template <int TL, int PF, bool Z, bool WR>
__device__ __forceinline__ void lag_wave(const LagArgs& a_, int W_, int g_, int c_, int r_, double* partial_) {
  // a function's arguments arrive in VGPRs: make every launch constant uniform again (SGPRs), so
  // that row and chunk tests stay scalar branches
  LagArgs a;
  a.s.x = uni(a_.s.x);
  a.s.chain_stride = uni(a_.s.chain_stride);
  a.s.sample_stride = uni(a_.s.sample_stride);
  a.s.base = uni(a_.s.base);
  a.s.n_chains = uni(a_.s.n_chains);
  a.s.n = uni(a_.s.n);
  a.s.D = uni(a_.s.D);
  a.s.halves = WR ? 1 : uni(a_.s.halves);
  a.s.wrap = WR ? uni(a_.s.wrap) : 0;
  a.s.slot0 = WR ? uni(a_.s.slot0) : 0;
  a.L0 = uni(a_.L0);
  a.T = uni(a_.T);
  a.G = uni(a_.G);
  a.C = uni(a_.C);
  a.R = uni(a_.R);
  a.mom = uni(a_.mom);
  a.tail = uni(a_.tail);
  a.NT = uni(a_.NT);
  a.rowb = uni(a_.rowb);
  const int W = uni(W_), g = uni(g_), c = uni(c_), r = uni(r_);
  double* const partial = uni(partial_);
  const int lane = threadIdx.x;
  const Src& s = a.s;
  const int n = s.n, D = s.D;
  const int gofs = a.L0 + g * TL;
  const bool mom = Z && a.mom;                     // wave-uniform (Z: gofs == 0, group 0)
  const int64_t m2 = n_series(s);
  // byte offset of sample `row` from a series' first window row (WR) or first sample
  auto rowoff = [&](int row) -> int {
    if constexpr (WR) {
      int p = row + s.slot0;
      p = p >= s.wrap ? p - s.wrap : p;
      return p * a.rowb;
    } else {
      return row * a.rowb;
    }
  };
  // lane -> (split chain jj past the tile's first, dim d): the same for every tile of the class
  const int per = 64 / lag_gcd(D, 64);             // split chains per class period (64 C / D)
  const int d0 = (int)((64 * (int64_t)c) % D);
  const int jj = (d0 + lane) / D;
  const int d = d0 + lane - jj * D;
  int64_t j0 = (64 * (int64_t)c) / D + (int64_t)per * r;
  const int64_t jstep = (int64_t)per * a.R;

  double v[TL];
#pragma unroll
  for (int k = 0; k < TL; ++k) v[k] = 0.0;
  double a_std = 0.0, a_m = 0.0, a_m2 = 0.0;
  double a_tail[kLagTail];
#pragma unroll
  for (int k = 0; k < kLagTail; ++k) a_tail[k] = 0.0;
  // shift of rows 1-2: the view's first sample
  const double Sd = s.x[s.base + (WR ? (int64_t)s.slot0 * s.sample_stride : 0) + d];
  if (gofs + 1 < n || mom) {
    // a tile's buffer descriptor and lane offset: split chain j0's first sample (wave-uniform) is the
    // base; lane offsets in bytes (host-checked below kLagOOB); lanes past the last series read
    // zeros (out of the buffer's range)
    auto tile_rsrc = [&](int64_t jt, int& vo) {
      const int64_t j = jt + jj;
      const double* tb = split_ptr(s, jt, 0);
      tb = reinterpret_cast<const double*>(
          ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)tb >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)tb));
      vo = j < m2 ? (int)((split_ptr(s, j, 0) + d - tb) * 8) : kLagOOB + 64;
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(tb), 0, kLagOOB, 0x00020000);
    };
    // the first PF rows of the NEXT tile are loaded a whole tile ahead (a tile's first rows used to
    // wait a full memory latency: one wave per SIMD has nothing else to run meanwhile)
    double xn[PF];
    int voff_n = 0;
    __amdgpu_buffer_rsrc_t rs_n = tile_rsrc(j0, voff_n);
    const int64_t tau0 = c + (int64_t)a.C * r;
    if (tau0 < a.NT) {
#pragma unroll
      for (int p = 0; p < PF; ++p)
        xn[p] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs_n, voff_n, rowoff(p < n ? p : n - 1), 0));
    }
    for (int64_t tau = tau0; tau < a.NT; tau += (int64_t)a.C * a.R, j0 += jstep) {
      const bool valid = j0 + jj < m2;
      const __amdgpu_buffer_rsrc_t rs = rs_n;
      const int voff = voff_n;
      double xq[PF], xdq[PF];
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        xq[p] = xn[p];
        if constexpr (!Z) xdq[p] = xn[p];            // loop B's delayed rows 0 .. PF-1 (PF <= gofs)
      }
      if (tau + (int64_t)a.C * a.R < a.NT) {         // the next tile's first rows
        rs_n = tile_rsrc(j0 + jstep, voff_n);
#pragma unroll
        for (int p = 0; p < PF; ++p)
          xn[p] = __builtin_bit_cast(double,
                                     __builtin_amdgcn_raw_buffer_load_b64(rs_n, voff_n, rowoff(p < n ? p : n - 1), 0));
      }
      auto ldb = [&](int boff) -> double {         // sample at byte offset boff of the series
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, boff, 0));
      };
      auto ld = [&](int row) -> double { return ldb(rowoff(row)); };
      // the rolling prefetch's next row, as a running byte offset (a scalar the compiler may not
      // precompute per unrolled row: those products spilled the scalar file), clamped to row n - 1;
      // WR: a running row number, clamped, then wrapped (and the delayed stream's row wrapped apart)
      const int last_off = (n - 1) * a.rowb;
      const int dly_off = gofs * a.rowb;
      int nxt = PF * a.rowb;
      int nxr = PF;
      int dly_o = 0;                               // WR: the delayed row's offset of the last next_off()
      auto next_off = [&]() {
        if constexpr (WR) {
          int rw = nxr < n - 1 ? nxr : n - 1;
          asm volatile("" : "+s"(rw));
          ++nxr;
          asm volatile("" : "+s"(nxr));
          if constexpr (!Z) dly_o = rowoff(rw - gofs);
          return rowoff(rw);
        } else {
          int o = nxt < last_off ? nxt : last_off;
          asm volatile("" : "+s"(o));
          nxt += a.rowb;
          asm volatile("" : "+s"(nxt));
          return o;
        }
      };
      auto dly_of = [&](int o) -> int {            // offset of the delayed stream's row
        if constexpr (WR) return dly_o;
        else return o - dly_off;
      };
      const double sh = xq[0];                      // row 0
      const double sh2 = 2.0 * sh;
      double ring[TL];
#pragma unroll
      for (int k = 0; k < TL; ++k) ring[k] = 0.0;
      double s1 = 0.0, s2 = 0.0, r1 = 0.0, q4 = 0.0;
      if constexpr (!Z) {
        // rows 0 .. gofs - 1 (gofs >= PF, a multiple of PF): squares only; the rolling prefetch
        // runs on into loop B's first rows (slot = row % PF = (row - gofs) % PF)
        for (int s0 = 0; s0 < gofs; s0 += PF) {
#pragma unroll
          for (int p = 0; p < PF; ++p) {
            const double y = xq[p] - sh;
            s2 = __builtin_fma(y, y, s2);
            xq[p] = ldb(next_off());                 // row s0 + p + PF
          }
        }
      }
      const int nrow = n - gofs;                   // rows of loop B (>= 2)
      // TL rows from row gofs + ci TL.  FIRST: chunk 0 (ramp, P events); MOM: moments; DLY: the
      // delayed stream is a second load; RAG: fewer than TL rows left (uniform row tests)
      auto chunk = [&](auto first_c, auto mom_c, auto dly_c, auto rag_c, int ci) {
        constexpr bool FIRST = decltype(first_c)::value, MOM = decltype(mom_c)::value;
        constexpr bool DLY = decltype(dly_c)::value, RAG = decltype(rag_c)::value;
        const int s0 = gofs + ci * TL;
        const int rem = n - s0;
        auto row = [&](auto i_c) {
          constexpr int i = decltype(i_c)::value;
          // the loads are unconditional (rows past n re-read row n - 1): a load inside the ragged
          // rows' branch made its register a phi whose copy waited for vmcnt(0) every row
          const double x = xq[i % PF];
          const double xd = DLY ? xdq[i % PF] : x;
          {
            const int o = next_off();                // row min(s0 + i + PF, n - 1)
            xq[i % PF] = ldb(o);
            if (DLY) xdq[i % PF] = ldb(dly_of(o));
          }
          // ragged rows past n: a uniform branch over the arithmetic only (the loads above are
          // unconditional, so no load result is a phi: the waitcnt pass keeps its counts)
          if (!RAG || i < rem) {
            const double y = x - sh;
            if constexpr (MOM) {
              r1 += x;
              s1 += y;
            }
            s2 = __builtin_fma(y, y, s2);
#pragma unroll
            for (int k = 0; k < TL; ++k) {
              if (FIRST && k >= i) continue;       // the ramp: slot (i - 1 - k) not written yet
              v[k] = __builtin_fma(y, ring[(i - 1 - k + TL) % TL], v[k]);
            }
            if constexpr (FIRST) v[i] -= s2;       // P(gofs + 1 + i)
            const double rv = __builtin_fma(-2.0, xd, sh2);   // -2 (xd - sh): exact scaling
            if constexpr (DLY) q4 = __builtin_fma(rv, rv, q4);   // 4 x the delayed stream's squares
            ring[i] = rv;
          }
          // rows stay in program order: hoisting later rows' loads (the scheduler's choice in a
          // straight-line chunk) holds their results in registers and spills the ring
          __builtin_amdgcn_sched_barrier(0);
        };
        static_for<TL>(row);
      };
      auto run = [&](auto mom_c, auto dly_c) {
        if (nrow < TL) chunk(std::true_type{}, mom_c, dly_c, std::true_type{}, 0);
        else chunk(std::true_type{}, mom_c, dly_c, std::false_type{}, 0);
        int ci = 1;
        for (; (ci + 1) * TL <= nrow; ++ci) chunk(std::false_type{}, mom_c, dly_c, std::false_type{}, ci);
        if (ci * TL < nrow) chunk(std::false_type{}, mom_c, dly_c, std::true_type{}, ci);
      };
      if constexpr (Z) run(std::true_type{}, std::false_type{});   // (moments unused unless mom)
      else run(std::false_type{}, std::true_type{});
      // Q(t) = S2 - P(n - t), t = gofs + 1 + k: 4 (S2 - P(n - gofs)) (0 for gofs = 0), plus the
      // squares of the last k + 1 delayed samples, slot (n - 1 - gofs - k') mod TL, k' <= k
      double q = Z ? 0.0 : 4.0 * s2 - q4;
      const double s2x2 = 2.0 * s2;
      auto fin = [&](auto rl_c) {
        constexpr int RL = decltype(rl_c)::value;
#pragma unroll
        for (int k = 0; k < TL; ++k) {
          const double rk = ring[(RL - k + TL) % TL];
          q = __builtin_fma(rk, rk, q);            // 4 Q(gofs + 1 + k)
          v[k] += __builtin_fma(-0.25, q, s2x2);
        }
      };
      static_dispatch<TL>((n - 1 - gofs) % TL, fin);
      if (mom && valid) {
        const double dn = n;
        const double mean = r1 / dn;
        const double dm = mean - sh;
        const double mm2 = (s2 - 2.0 * dm * s1) + dn * (dm * dm);
        a_std += sqrt(mm2 > 0.0 ? mm2 / (dn - 1.0) : 0.0);
        const double e = mean - Sd;
        a_m += e;
        a_m2 = __builtin_fma(e, e, a_m2);
        // the tail lags n - k, k = 1 .. tail, in difference form: y_0 = 0 (the shift), y_1 .. y_{tail-1}
        // and the last tail samples, loaded together (clamped rows; unused values are masked)
        const int K = a.tail;
        double yl[kLagTail], yf[kLagTail];
#pragma unroll
        for (int j = 0; j < kLagTail; ++j) {
          const int rl = n - 1 - j;
          yl[j] = ld(j < K && rl > 0 ? rl : 0);     // y_{n-1-j} (+ sh)
          yf[j] = ld(j < K ? j : 0);               // y_j (+ sh)
        }
#pragma unroll
        for (int j = 0; j < kLagTail; ++j) {
          yl[j] -= sh;
          yf[j] -= sh;
        }
#pragma unroll
        for (int k = 1; k <= kLagTail; ++k) {
          if (k <= K) {                            // uniform
            // V_{n-k} = sum_{i<k} (y_{n-k+i} - y_i)^2, y_{n-k+i} = yl[k-1-i]
            double acc = 0.0;
#pragma unroll
            for (int i = 0; i < k; ++i) {
              const double df = yl[k - 1 - i] - yf[i];
              acc = __builtin_fma(df, df, acc);
            }
            a_tail[k - 1] += acc;
          }
        }
      }
    }
  }
  double* out = partial + (int64_t)W * kLagRows * 64 + lane;
  out[0] = a_std;
  out[64] = a_m;
  out[128] = a_m2;
#pragma unroll
  for (int k = 0; k < kLagTail; ++k) out[(3 + k) * 64] = a_tail[k];
#pragma unroll
  for (int k = 0; k < TL; ++k) out[(3 + kLagTail + k) * 64] = v[k];
}

template <int TL, int PF, bool WR>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HMC_LAG_WPE, HMC_LAG_WPE))) void k_conv_series(LagArgs a,
                                                                                               double* partial) {
  const int W = blockIdx.x;
  const int u = W >> 3;
  const int g = u % a.G;
  const int cr = (u / a.G) * 8 + (W & 7);
  const int c = cr % a.C, r = cr / a.C;
  if (r >= a.R) return;                            // grid padding (never reduced)
  if (a.L0 + g * TL == 0) lag_wave<TL, PF, true, WR>(a, W, g, c, r, partial);
  else lag_wave<TL, PF, false, WR>(a, W, g, c, r, partial);
}

// inter[(c * G + g) * kLagRows + row][l] = sum over the replicas r (in order) of the waves' lanes
__global__ __launch_bounds__(256) void k_lag_classes(LagArgs a, const double* __restrict__ partial,
                                                     double* __restrict__ inter) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)a.C * a.G * kLagRows * 64;
  if (i >= tot) return;
  const int l = (int)(i & 63);
  const int64_t cgr = i >> 6;
  const int row = (int)(cgr % kLagRows);
  const int64_t cg = cgr / kLagRows;
  const int g = (int)(cg % a.G), c = (int)(cg / a.G);
  double acc = 0.0;
  for (int r = 0; r < a.R; ++r) {
    const int cr = r * a.C + c;
    const int64_t W = 8 * (g + (int64_t)a.G * (cr / 8)) + (cr & 7);
    acc += partial[(W * kLagRows + row) * 64 + l];
  }
  inter[i] = acc;
}

// out[orow][d]: conv layout (conv != 0: rows std, mean - S, (mean - S)^2, lags L0 + 1 + skip ..,
// lag n - 1; nlag lags) or lags only; lags t >= n are 0.  Sums the classes' lanes that hold
// dimension d, in a fixed order.
__global__ __launch_bounds__(256) void k_lag_dims(LagArgs a, const double* __restrict__ inter, int conv, int skip,
                                                  int nlag, double* __restrict__ out) {
  const int D = a.s.D;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nrow = conv ? nlag + 4 : nlag;
  if (i >= (int64_t)nrow * D) return;
  const int orow = (int)(i / D), d = (int)(i - (int64_t)orow * D);
  int g = 0, prow;
  int t = 0;                                       // lag (0: a moment row)
  if (conv && orow < 3) prow = orow;
  else {
    t = (conv && orow == nlag + 3) ? a.s.n - 1 : a.L0 + 1 + skip + orow - (conv ? 3 : 0);
    if (a.mom && t >= a.s.n - a.tail) {            // a tail lag (difference form, group 0)
      prow = 3 + (a.s.n - 1 - t);
    } else {
      const int k = t - a.L0 - 1;                  // lag index inside the pass
      g = k / kLagTL;
      prow = 3 + kLagTail + k % kLagTL;
    }
  }
  double acc = 0.0;
  if (t < a.s.n && t >= 0 && g < a.G && !(conv && orow == nlag + 3 && a.s.n < 2)) {
    for (int c = 0; c < a.C; ++c) {
      int l = (int)(((int64_t)d - 64 * (int64_t)c) % D);
      if (l < 0) l += D;
      for (; l < 64; l += D) acc += inter[(((int64_t)c * a.G + g) * kLagRows + prow) * 64 + l];
    }
  }
  out[i] = acc;
}

// ---- The same one-read sums on the matrix cores (complete passes, 96 <= n <= 208: c3's
// n = 200).  The lag products are GEMM-shaped once the series is laid out as Hankel slices:
// v_mfma_f64_16x16x4_f64 with A[t'][k] = y_k[b + T + t'] and B[k][s] = y_k[b - s] (k = four split
// chains of ONE dimension, the contraction index) adds y_k[i] y_k[i + L] to entry (t', s) of tile T,
// L = T + t' + s, anchor i = b - s.  Tiles T = -16, 0, 16, .. and anchor steps b = 0, 16, ..: a lag
// L = 16 q + r gets s <= r from tile 16 q and s > r from tile 16 q - 16, so over all b every product
// y_i y_{i+L} (0 <= i, i + L < n; rows outside [0, n) are zeros in LDS) is added exactly once, and a
// tile only runs the anchor steps that still meet lags < n (the triangle, at 16-row granularity).
// V_t = sum_{s>=t} sq_s + sum_{s<=n-1-t} sq_s - 2 C_t with sq_s = sum_j y_{j,s}^2 (no cancellation
// in the square terms), y = x - x_j[0] per series as in lag_wave.
// Workgroup = 4 waves = 4 dimensions x a range of split chains (two workgroups per CU, so one's
// staging runs beside the other's matrix work): the waves stage each group of four split chains
// into LDS together (lanes across the 4 dims: 32-B row segments; each row's other segments are read
// by the neighbouring dimension groups on the same XCD), then each wave runs its dimension's tiles,
// accumulating across the range in registers (tiles x 4 doubles per lane).  Split means and stds come
// from the same A slices (partial sums over rows t' mod 16, reduced in a fixed order: deterministic,
// within a few ulps of np.mean's sequential sum).
constexpr int kMfmaNT = 16;                      // tiles T = -16 .. 16 (kMfmaNT - 2)
constexpr int kMfmaMaxN = 16 * (kMfmaNT - 3);    // 208 samples per split chain (NTM = 14)
#ifndef HMC_MFMA_MIN_N
#define HMC_MFMA_MIN_N 96
#endif
constexpr int kMfmaMinN = HMC_MFMA_MIN_N;
constexpr int kMfmaDims = 4;                     // waves (dimensions) per workgroup
constexpr int kMfmaThreads = 64 * kMfmaDims;
constexpr int kMfmaSer = 4 * kMfmaDims;          // series staged per chain group
constexpr int kMfmaSlack = 320;                  // doubles past the last series (read-ahead)
constexpr int kSqStride = 272;                   // sq rows per lane group (2176 B: bank-spread)
constexpr int kMfmaPW = kMfmaNT * 256 + 256 + 4; // partial doubles per wave: tiles, sq rows, moments

struct MfmaArgs {
  Src s;
  int P;            // LDS doubles between dims' series (rows -16 .. n + 29; 8 mod 32)
  int PK;           // between chains' (4 P + 16: 16 mod 32)
  int NT, NB;       // tiles and anchor steps used
  int G;            // dimension groups ceil(D / kMfmaDims)
  int R;            // split-chain ranges (a multiple of 8)
  int64_t per;      // split chains per range (a multiple of 4)
};

// W3: the small instance (NTM = 8, c4's halves) at three waves per SIMD (168 VGPRs: the B column
// read a step ahead instead of up front; three workgroups' double buffers in 141 KB of LDS):
// 41.40 -> 41.07 ms per c4 half (same box, alternating runs); more waves hide little here, the
// pass is not latency-bound the way that would
#ifndef HMC_MFMA_W2
constexpr bool kMfmaW3 = true;
#else
constexpr bool kMfmaW3 = false;
#endif
// VT >= 0 (NTM = 8 with 97 <= n <= 111, NTM = 14 with 193 <= n <= 207: VT = NTM - 2 = n / 16 and
// NT = NTM): the tile bound and the tile count are compile-time,
// so the triangle is static (no per-MFMA branches, no merges of accumulator tuples).  E4 (1..3,
// with VT): n % 16 < 12, and each anchor step's last tile runs as E4 v_mfma_f64_4x4x4 on the row
// groups that meet rows below n (a quarter of a 16x16x4's cycles each) instead of a whole tile.
template <int NTM, int E4 = 0, int VT = -1>
__global__ __launch_bounds__(kMfmaThreads) __attribute__((amdgpu_waves_per_eu((kMfmaW3 && NTM <= 8) ? 3 : 2, (kMfmaW3 && NTM <= 8) ? 3 : 2))) void k_conv_mfma(MfmaArgs a,
                                                                                             double* partial) {
  // capacity of this instance: NTM tiles, NTM - 1 anchor steps, n <= 16 (NTM - 1)
  constexpr int kNB = NTM - 1, kRows = NTM - 1;
  // the host takes this instance for 16 (NTM - 3) < n <= 16 (NTM - 1) (launch_conv_mfma): slices
  // q <= kQAll always hold a row below n, and staging rows 16 i + 15 < n for i < kQAll (NTM = 6, below
  // the matrix-core range's lower bound, keeps every test)
  constexpr int kQAll = NTM == 6 ? -1 : NTM - 3;
  // LDS: [4 chains][dims] series of the group at k PK + w P (bank-spread for both the staging writes
  // and the matrix waves' slice reads), x0[16], slack, sq rows [dims][4 chain lanes][272]
  extern __shared__ double lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  // XCD-major: the G dimension groups of one chain range run on one XCD (blocks id, id + 8, ..
  // share an XCD), so a row's segments are fetched into that L2 once
  const int id = blockIdx.x;
  const int local = id >> 3;
  const int r = (local / a.G) * 8 + (id & 7), g = local % a.G;
  const Src& s = a.s;
  const int n = s.n, D = s.D, P = a.P, PK = a.PK;
  // PIPE (n <= 144, where two sample buffers fit beside the other workgroup's): the staged group
  // g + 1 is written to the other LDS buffer while group g's matrix work runs from registers, and
  // group g + 1's operands are read into registers right after the group's one barrier -- no LDS
  // wait in front of the MFMAs and one barrier per group instead of two (c4's halves: 45.6 -> see
  // DESIGN.md §3.5).  (Two staged groups per pair of barriers: 48.1 -> 50.5 ms; a second
  // staging register set two groups ahead: 48.1 -> 48.3 ms.  Neither is kept.)
  constexpr bool PIPE = NTM <= 10;
  constexpr int NBUF = PIPE ? 2 : 1;
  constexpr bool SQR_LDS = NTM > 10;               // the sq rows live in LDS (else in registers)
  const int SB = 4 * PK;
  double* const x0l = lds + NBUF * SB;
  double* const sqb = x0l + NBUF * kMfmaSer + kMfmaSlack;
  const int64_t m2 = n_series(s);
  const int64_t jlo = (int64_t)r * a.per;
  const int64_t jhi = jlo + a.per < m2 ? jlo + a.per : m2;
  // split chains of this range (< 2^31), the group loop in 32-bit offsets o from jlo: its bounds
  // are scalar compares (int64 compares of wave-uniform values run on the VALU)
  const int nrem = jhi > jlo ? (int)(jhi - jlo) : 0;
  for (int i = tid; i < NBUF * (SB + kMfmaSer) + kMfmaSlack + (SQR_LDS ? kMfmaSer * kSqStride : 0); i += kMfmaThreads)
    lds[i] = 0.0;
  // staging role: wave = chain sk of the group, lane = (dim sw, row phase rho); rows rho + 16 i
  // (sk wave-uniform in an SGPR: the chain's base offset is scalar arithmetic)
  const int sk = uni(wv), sw = lane & 3, rho = lane >> 2;
  const int sd = g * kMfmaDims + sw;
  // staged rows of the next chain group (loads in flight under a group of matrix work)
  double xsa[kRows];
  double x0a = 0.0;
  // buffer loads based at the group's first split chain (uniform): one 32-bit lane offset (host-
  // checked below kLagOOB) plus 16 i rows (in the vector offset: the range check covers it); the
  // buffer ends with the view's last sample, so lanes past the range or the dims (offset kLagOOB)
  // and rows past the last chain's end read zeros (y = 0 - 0)
  const int rowb = (int)(s.sample_stride * 8);
  const double* const vend = split_ptr(s, m2 - 1, n - 1) + D;
  auto stage_load = [&](int o, double (&xs)[kRows], double& x0s) {
    const int64_t jg = jlo + o, j = jg + sk;
    const double* b = uni(split_ptr(s, jg, 0));
    const int64_t span = (vend - b) * 8;
    const int nrec = span < kLagOOB ? (int)span : kLagOOB;
    const int lo = (sd < D && o + sk < nrem) ? (int)((split_ptr(s, j, 0) - b) + sd) * 8 + rho * rowb : kLagOOB + 64;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(b), 0, nrec, 0x00020000);
    x0s = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lo - rho * rowb, 0, 0));
#pragma unroll
    for (int i = 0; i < kRows; ++i)
      xs[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lo + 16 * i * rowb, 0, 0));
  };
  // x0l holds x0 - S_d of each staged series (0 for chains past the range: their rows are zeros,
  // so their moments add nothing)
  const double Ssd = sd < D ? s.x[s.base + sd] : 0.0;
  auto stage_store = [&](int nn, const double (&xs)[kRows], double x0s, int buf, bool valid) {
    double* dst = lds + buf * SB + sk * PK + sw * P + 16 + rho;
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      if (i < kQAll || 16 * i + 15 < nn) dst[16 * i] = xs[i] - x0s;      // whole 16-row phase
      else if (16 * i < nn && rho + 16 * i < nn) dst[16 * i] = xs[i] - x0s;   // rows >= n stay zero
    }
    if (rho == 0) x0l[buf * kMfmaSer + sk * 4 + sw] = valid ? x0s - Ssd : 0.0;
  };
  // matrix role: wave wv = dimension d; lane = (chain k = lane >> 4, t' or s = lane & 15)
  const int d = g * kMfmaDims + sk;
  const int k = lane >> 4, c16 = lane & 15;
  typedef double v4d __attribute__((ext_vector_type(4)));
  v4d acc[NTM];
#pragma unroll
  for (int t = 0; t < NTM; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
  double* const sqa = sqb + (wv * 4 + k) * kSqStride;   // sq rows of this wave's chain lane group k
  // the small instances keep the sq rows in registers instead (they have the room: no LDS
  // read-modify-write per group)
  constexpr bool SQR = NTM <= 10;
  double sqr[SQR ? NTM : 1];
#pragma unroll
  for (int q = 0; q < (SQR ? NTM : 1); ++q) sqr[q] = 0.0;
  double a_std = 0.0, a_m = 0.0, a_m2 = 0.0;
  const int NT = a.NT;
  const double dn = n;
  const double rn = 1.0 / dn, rn1 = 1.0 / (dn - 1.0);
  // split moments, four groups at a time: after the row scans a group's totals (chain k: lane
  // 16 k + 15) are parked by one DPP row_shl:4 per value (lanes 3, 7, 11 take the previous three
  // groups' totals; lanes 12-15 the new ones), and the std/mean arithmetic runs once per four
  // groups on lanes 3, 7, 11, 15 of each row (the other lanes' results are never read)
  double pk1 = 0.0, pk2 = 0.0, pkx = 0.0;
  int gi = 0;                                     // groups parked (wave-uniform)
  auto park = [](double b, double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(b), 0x104, 0xF, 0x7, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(b), 0x104, 0xF, 0x7, false);
    return __hiloint2double(hi, lo);
  };
  auto flush = [&]() {
    const double mm2 = pk2 - pk1 * (pk1 * rn);
    a_std += sqrt(mm2 > 0.0 ? mm2 * rn1 : 0.0);
    const double e = pkx + pk1 * rn;
    a_m += e;
    a_m2 = __builtin_fma(e, e, a_m2);
  };
  // the matrix operands of a group: A slices q = 0 .. NTM (rows 16 (q - 1) + 15 + t') and the B
  // column of every anchor step (PIPE; else one step ahead, read inside matrix)
  constexpr bool BBALL = PIPE && !(kMfmaW3 && NTM <= 8);   // every step's B column up front
  double sl[NTM + 1], bb[BBALL ? kNB : 1];
  auto ops_ptr = [&](int buf) {
    int zo = buf * SB + k * PK + wv * P + 16;     // (an opaque integer offset keeps sr an LDS pointer)
    asm volatile("" : "+v"(zo));
    return (const double*)(lds + zo);
  };
  auto read_ops = [&](int buf) {
    const double* sr = ops_ptr(buf);
#pragma unroll
    for (int q = 0; q <= NTM; ++q) sl[q] = sr[16 * (q - 1) + 15 + c16];
#pragma unroll
    for (int bi = 0; bi < (BBALL ? kNB : 1); ++bi) bb[bi] = sr[16 * bi + 15 - c16];
  };
  auto matrix = [&](int nn, int buf) {
    if (d < D) {
      const double* sr = ops_ptr(buf);
      // Anchor steps b = 16 bi + 15 (anchors b - 15 .. b: step 0 starts at anchor 0).  Every
      // product of tile ti (T = 16 (ti - 1)) at step bi pairs an anchor with row b + T + t' >=
      // 16 (bi + ti) - 1, so the tile meets a row below n only while 16 (bi + ti) <= n:
      // ti <= tl(bi) = n / 16 - bi (round 6: the bound was (n - 1) / 16 + 1 - bi, one tile per step
      // of LDS-zero rows unless 16 | n: 7 of 35 MFMAs per group at n = 99, 13 of 104 at
      // n = 200).  Steps bi <= v = (n - 1) / 16.  Step-major: a step's tiles are
      // independent accumulators back to back (a tile's own chain of dependent MFMAs ran 20-40 %
      // slower).  Tile ti at step bi reads A slice q = bi + ti (rows 16 (q - 1) + 15 + t'): the
      // slices q = 0 .. NTM are read once, up front, into registers; B of the next step is read a
      // step ahead.  Reads past row n + 29 land in the next series or the LDS slack, feed no MFMA.
      const int vt = nn >> 4;                     // tiles ti <= vt - bi meet rows below n
      if constexpr (!PIPE) read_ops(buf);
      double bcur = bb[0];
      auto bstep = [&](auto bi_c) {
        constexpr int bi = decltype(bi_c)::value;
        const int tl = min(NT - 1, vt - bi);
        double bnx = 0.0;
        if constexpr (BBALL) bnx = bi + 1 < kNB ? bb[bi + 1 < kNB ? bi + 1 : 0] : 0.0;
        else bnx = bi + 1 < kNB ? sr[16 * (bi + 1) + 15 - c16] : 0.0;
        auto tile = [&](auto ti_c) {
          constexpr int ti = decltype(ti_c)::value;
          if constexpr (bi + ti <= NTM) {
            constexpr int tls = VT - bi;          // (VT >= 0: the static bound)
            if (VT >= 0 ? (E4 > 0 ? ti < tls : ti <= tls) : ti <= tl) {
#ifdef HMC_MFMA_DEV_NOLDS                         // dev timing variant: no LDS operands
              acc[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(dn, dn, acc[ti], 0, 0, 0);
#else
              acc[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(sl[bi + ti], bcur, acc[ti], 0, 0, 0);
#endif
            }
            else if (VT >= 0 && E4 > 0 && ti == tls) {
              // the step's edge tile: rows 16 (bi + ti) - 1 + t' < n only for t' <= n % 16, i.e.
              // accumulator components g < e4 (rows 4 g .. 4 g + 3).  Each takes one
              // v_mfma_f64_4x4x4f64 (a quarter of the 16x16x4 cost): its four blocks share the A
              // rows (A lane (k, blk, i) = y_k[row 4 g + i]), B is the 16x16x4 operand as it is
              // (lane (k, s)), and its result lane (i, blk, j) is entry (4 g + i, 4 blk + j) --
              // the lane and component g where the 16x16x4 layout keeps that entry.
#pragma unroll
              for (int g = 0; g < (E4 > 0 ? E4 : 1); ++g) {
                if constexpr (E4 > 0) {
                  const double a4 = sr[16 * (bi + ti - 1) + 15 + 4 * g + (c16 & 3)];
                  acc[ti][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(a4, bcur, acc[ti][g], 0, 0, 0);
                }
              }
            }
          }
        };
        static_for<NTM>(tile);
        bcur = bnx;
      };
      static_for<kNB>(bstep);
      // split moments of chain k and the sq rows from the slices q = 0 .. kRows (rows
      // 16 (q - 1) + 15 + t': every row once; row -1 and rows >= n are zeros or masked), the 16 row
      // phases reduced in a fixed xor order
      double ps1, ps2;
      double sv[kRows + 1];
#pragma unroll
      for (int q = 0; q <= kRows; ++q) sv[q] = SQR ? 0.0 : sqa[16 * q + c16];
      const int qn = nn >> 4;                     // slices past q = n / 16 hold rows >= n only
#pragma unroll
      for (int q = 0; q <= kRows; ++q) {
        // (rows n .. n + 29 of slice qn are LDS zeros; later slices may read the next series).
        // Only the last slices of an instance can lie past qn (kQAll): one select there, instead of
        // a guarded update per slice that the compiler turned into six v_cndmask per slice
        double y = sl[q];
        if (q > kQAll) y = q <= qn ? y : 0.0;
        if (q == 0) {                             // (no add to a zero start)
          ps1 = y;
          ps2 = y * y;
        } else {
          ps1 += y;
          ps2 = __builtin_fma(y, y, ps2);
        }
        if constexpr (SQR) sqr[q] = __builtin_fma(y, y, sqr[q]);
        else if (q <= kQAll || q <= qn) sqa[16 * q + c16] = __builtin_fma(y, y, sv[q]);   // sq row 16 q + t' - 1
      }
      // the 16 row phases of chain k summed by a DPP row_shr scan: the total lands in the row's
      // lane 15 (other lanes keep partial sums, accumulate into moments that are never read)
      ps1 += dpp_u<0x111>(ps1);
      ps2 += dpp_u<0x111>(ps2);
      ps1 += dpp_u<0x112>(ps1);
      ps2 += dpp_u<0x112>(ps2);
      ps1 += dpp_u<0x114>(ps1);
      ps2 += dpp_u<0x114>(ps2);
      ps1 += dpp_u<0x118>(ps1);
      ps2 += dpp_u<0x118>(ps2);
      pk1 = park(pk1, ps1);
      pk2 = park(pk2, ps2);
      pkx = park(pkx, x0l[buf * kMfmaSer + k * 4 + wv]);
      if ((gi & 3) == 3) flush();
      ++gi;
    }
  };
  if (nrem > 0) stage_load(0, xsa, x0a);
  if constexpr (PIPE) {
    // group jg in buffer buf: its operands are in registers when the iteration starts; the group
    // jg + 4 is stored into buf ^ 1 (last read before the previous iteration's barrier) and read
    // back after this iteration's barrier; the loads of group jg + 8 are issued before the matrix
    // work and waited for before the barrier
    if (nrem > 0) {
      __syncthreads();                            // the zeroed LDS
      stage_store(n, xsa, x0a, 0, sk < nrem);
      if (4 < nrem) stage_load(4, xsa, x0a);
      __syncthreads();
      if (d < D) read_ops(0);
    }
    int buf = 0;
    for (int o = 0; o < nrem; o += 4) {
      int nn = n;                                 // opaque per group: bounds recomputed, not hoisted
      asm volatile("" : "+s"(nn));
      if (o + 4 < nrem) {
        stage_store(nn, xsa, x0a, buf ^ 1, o + 4 + sk < nrem);
        if (o + 8 < nrem) stage_load(o + 8, xsa, x0a);
      }
      matrix(nn, buf);
      // the loads just issued land before the barrier: the workgroups that read one row's 128-B
      // lines stay in step and share them in L2.  FETCH_SIZE at c4's halves: 2.5x the samples
      // without this wait (44.9 ms), 1.3x with it (43.2 ms); loads three groups ahead in two
      // register sets with a wait for the older set: 2.0x, 44.1 ms
#ifndef HMC_MFMA_NO_THROTTLE
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      __syncthreads();                            // group jg + 4 stored, group jg read
      buf ^= 1;
      if (o + 4 < nrem && d < D) read_ops(buf);
    }
  } else {
    for (int o = 0; o < nrem; o += 4) {
      int nn = n;                                 // opaque per group: bounds recomputed, not hoisted
      asm volatile("" : "+s"(nn));
      __syncthreads();                            // the previous group's slices are read
      stage_store(nn, xsa, x0a, 0, o + sk < nrem);
      __syncthreads();
      if (o + 4 < nrem) stage_load(o + 4, xsa, x0a);    // in flight under this group's matrix work
      matrix(nn, 0);
    }
  }
  if (d < D && (gi & 3) != 0) {                   // the last groups: zero-padded to four
    while ((gi & 3) != 0) {
      pk1 = park(pk1, 0.0);
      pk2 = park(pk2, 0.0);
      pkx = park(pkx, 0.0);
      ++gi;
    }
    flush();
  }
  // partial of this wave: tiles (entry t' * 16 + s), sq rows (summed over the 4 chain lanes; LDS
  // entry i holds row i - 1), moments
  double* out = partial + ((int64_t)id * kMfmaDims + wv) * kMfmaPW;
#pragma unroll
  for (int t = 0; t < NTM; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) out[t * 256 + q * 64 + lane] = acc[t][q];
  if constexpr (SQR) {                            // rows 16 q + t' - 1, summed over the 4 lane groups
#pragma unroll
    for (int q = 0; q <= kRows; ++q) {
      double v = sqr[q];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int row = 16 * q + c16 - 1;
      if (lane < 16 && row >= 0) out[kMfmaNT * 256 + row] = v;
    }
  } else {
    const double* sw4 = sqb + wv * 4 * kSqStride;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 64 * i + lane;              // output row; LDS entry row + 1
      double v = 0.0;
      if (row < 255)
        v = ((sw4[row + 1] + sw4[kSqStride + row + 1]) + sw4[2 * kSqStride + row + 1]) + sw4[3 * kSqStride + row + 1];
      out[kMfmaNT * 256 + row] = v;
    }
  }
  // moments: lanes 3, 7, 11, 15 of each row (the parked slots)
  auto slots = [&](double v) {
    v = (c16 & 3) == 3 ? v : 0.0;
#pragma unroll
    for (int m = 4; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
    return v;
  };
  a_std = slots(a_std);
  a_m = slots(a_m);
  a_m2 = slots(a_m2);
  if (lane == 63) {
    out[kMfmaNT * 256 + 256] = a_std;
    out[kMfmaNT * 256 + 257] = a_m;
    out[kMfmaNT * 256 + 258] = a_m2;
  }
}

// red[d][e] = sum over the chain ranges (in order) of the partial entry e of dimension d's wave
__global__ __launch_bounds__(256) void k_mfma_ranges(MfmaArgs a, const double* __restrict__ partial,
                                                     double* __restrict__ red) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.s.D * kMfmaPW) return;
  const int d = (int)(i / kMfmaPW), e = (int)(i - (int64_t)d * kMfmaPW);
  const int g = d / kMfmaDims, w = d - g * kMfmaDims;
  double acc = 0.0;
  // entries k_mfma_dims never reads (tiles past NT, sq rows past n): not summed (half the reads
  // at n = 99, 8 of 16 tiles)
  if ((e >= a.NT * 256 && e < kMfmaNT * 256) || (e >= kMfmaNT * 256 + a.s.n && e < kMfmaNT * 256 + 256)) {
    red[i] = 0.0;
    return;
  }
  for (int r = 0; r < a.R; ++r) {
    const int id = ((r >> 3) * a.G + g) * 8 + (r & 7);   // inverse of k_conv_mfma's block map
    acc += partial[((int64_t)id * kMfmaDims + w) * kMfmaPW + e];
  }
  red[i] = acc;
}

// out in the conv layout of k_lag_dims (std, mean - S, (mean - S)^2, lags 1 .. nlag, lag n - 1)
__global__ __launch_bounds__(256) void k_mfma_dims(MfmaArgs a, const double* __restrict__ red, int nlag,
                                                   double* __restrict__ out) {
  const int D = a.s.D, n = a.s.n;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)(nlag + 4) * D) return;
  const int orow = (int)(i / D), d = (int)(i - (int64_t)orow * D);
  const double* rd = red + (int64_t)d * kMfmaPW;
  const double* sq = rd + kMfmaNT * 256;
  if (orow < 3) {
    out[i] = sq[256 + orow];
    return;
  }
  const int t = orow == nlag + 3 ? n - 1 : orow - 2;
  double v = 0.0;
  if (t >= 1 && t < n) {
    const int q = t >> 4, rr = t & 15;
    double c = 0.0;                               // C_t: tile 16 q (s <= r), tile 16 q - 16 (s > r)
    for (int sc = 0; sc <= rr; ++sc) c += rd[(q + 1) * 256 + (rr - sc) * 16 + sc];
    for (int sc = rr + 1; sc < 16; ++sc) c += rd[q * 256 + (rr + 16 - sc) * 16 + sc];
    double suf = 0.0, pre = 0.0;
    for (int r2 = t; r2 < n; ++r2) suf += sq[r2];
    for (int r2 = 0; r2 <= n - 1 - t; ++r2) pre += sq[r2];
    v = (suf + pre) - 2.0 * c;
  }
  out[i] = v;
}

// ---- streaming (windowed) split-chain statistics: q_chain never has to be stored whole.
// Sample position p (0-based over q_chain[:, 1:, :]) lies in split half h = p / n at offset
// s = p - h*n (positions >= 2n are not part of any split chain, utils.py:102-104).  A call
// consumes `rows` new samples (positions pos0 ...) from a circular window of `wrap` rows per
// chain: the k-th sample from position pos0 - carry sits in window row (slot0 + k) % wrap.
// carry >= min(T, pos0) keeps every lag t <= T exact.
struct StreamArgs {
  const double* x;
  int64_t n_chains, chain_stride, sample_stride;
  int D, wrap, slot0, carry, rows, n;
  int64_t pos0;
  double* shift;  // [n_chains][2][D] first sample of each half (variance shift)
  double* s1;     // [n_chains][2][D] sum (x - shift)
  double* s2;     // [n_chains][2][D] sum (x - shift)^2
  double* vpart;  // [groups][T][D] partial variogram sums over this block's chains
  int groups;
};

constexpr int kStreamChunk = 8;   // window rows loaded together (memory-level parallelism)
#ifndef HMC_STREAM_PF
#define HMC_STREAM_PF 8              // rows in flight per wave in k_stream_prod (rolling prefetch)
#endif

// Block = 4 chain lanes x 64 dims (lane = dim: coalesced rows).  Each thread walks its chains'
// new rows once, with the last T samples in a register ring.  Two forms of the lag sums:
//  * PROD (halves of n >= T samples): the product form of k_conv_lags, ONE FMA per lag and row,
//    V_t = 2 S2 - H_t - T_t - 2 C_t over shifted samples y = x - shift.  The ring is zeroed when a
//    half starts (so no product crosses halves) and the other terms are three per-half events,
//    all at static register indices: at position T-1 the ring holds y[T-1..0] (H_t), at n-1 it
//    holds the half's last T samples (T_t), and 2 S2 is added once the half is complete.  vsum
//    thus holds the sums of every completed half.
//  * difference form (short halves): per lag and row (x - x_{-t})^2 under a same-half mask.
// T <= 16 capped at 168 registers: three waves per SIMD keep enough rows in flight.
template <int T, bool PROD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(T <= 16 ? 3 : 1))) void k_stream_accum(StreamArgs a) {
  __shared__ double red[4][kDimTile];
  const int dl = threadIdx.x & (kDimTile - 1);
  const int rl = threadIdx.x / kDimTile;
  const int d = blockIdx.y * kDimTile + dl;
  const int64_t left = 2 * (int64_t)a.n - a.pos0;
  const int rows = (int)(left < a.rows ? (left > 0 ? left : 0) : a.rows);
  double v[T];
#pragma unroll
  for (int t = 0; t < T; ++t) v[t] = 0.0;
  if (d < a.D) {
    for (int64_t c = (int64_t)blockIdx.x * 4 + rl; c < a.n_chains; c += (int64_t)a.groups * 4) {
      const double* xc = a.x + c * a.chain_stride + d;
      auto at = [&](int k) {             // k-th window sample (k < carry + rows)
        int sl = a.slot0 + k;
        sl = sl >= a.wrap ? sl - a.wrap : sl;
        return xc[(int64_t)sl * a.sample_stride];
      };
      const int64_t o = c * 2 * a.D + d;
      double sh[2] = {a.shift[o], a.shift[o + a.D]};
      double m1[2] = {a.s1[o], a.s1[o + a.D]};
      double m2[2] = {a.s2[o], a.s2[o + a.D]};
      // first new row's half and position: carry rows of the same half enter the ring (as y for
      // PROD), older ones are zero
      const int hc = a.pos0 >= a.n ? 1 : 0;
      const int sidx0 = (int)(a.pos0 - (int64_t)hc * a.n);
      double ring[T];
#pragma unroll
      for (int k = 0; k < T; ++k) {
        if constexpr (PROD) ring[k] = (k < a.carry && k < sidx0) ? at(a.carry - 1 - k) - sh[hc] : 0.0;
        else ring[k] = (k < a.carry) ? at(a.carry - 1 - k) : 0.0;
      }
      for (int i0 = 0; i0 < rows; i0 += kStreamChunk) {
        double xs[kStreamChunk];
#pragma unroll
        for (int j = 0; j < kStreamChunk; ++j) xs[j] = (i0 + j < rows) ? at(a.carry + i0 + j) : 0.0;
        if constexpr (PROD) {
#pragma unroll
          for (int j = 0; j < kStreamChunk; ++j) {
            if (i0 + j < rows) {                  // uniform
              const int64_t p = a.pos0 + i0 + j;
              const int h = p >= a.n ? 1 : 0;
              const int sidx = (int)(p - (int64_t)h * a.n);
              if (sidx == 0) {                    // a half starts: its shift, an empty ring
                sh[h] = xs[j];
#pragma unroll
                for (int k = 0; k < T; ++k) ring[k] = 0.0;
              }
              const double y = xs[j] - sh[h];
              m1[h] += y;
              m2[h] = __builtin_fma(y, y, m2[h]);
              const double ym2 = -2.0 * y;
#pragma unroll
              for (int t = 0; t < T; ++t) v[t] = __builtin_fma(ym2, ring[t], v[t]);   // -2 C_t
#pragma unroll
              for (int k = T - 1; k > 0; --k) ring[k] = ring[k - 1];
              ring[0] = y;
              if (sidx == T - 1) {                // ring = y[T-1 .. 0]: H_t = sum_{s<t} y^2
                double q = 0.0;
#pragma unroll
                for (int t = 0; t < T; ++t) {
                  q = __builtin_fma(ring[T - 1 - t], ring[T - 1 - t], q);
                  v[t] -= q;
                }
              }
              if (sidx == a.n - 1) {              // ring = the last T samples: T_t; then + 2 S2
                double q = 0.0;
                const double s2x2 = 2.0 * m2[h];
#pragma unroll
                for (int t = 0; t < T; ++t) {
                  q = __builtin_fma(ring[t], ring[t], q);
                  v[t] += s2x2 - q;
                }
              }
            }
          }
          continue;
        }
        // difference form.  Whole chunk inside one split half with every lag <= T available
        // (uniform over the block): no same-half selects.  Same operations as the general path.
        const int64_t p0 = a.pos0 + i0;
        const int h0 = p0 >= a.n ? 1 : 0;
        const int64_t s0 = p0 - (int64_t)h0 * a.n;
        if (i0 + kStreamChunk <= rows && s0 >= T && s0 + kStreamChunk <= a.n) {
#pragma unroll
          for (int j = 0; j < kStreamChunk; ++j) {
            const double x = xs[j];
            const double e = x - sh[h0];
            m1[h0] += e;
            m2[h0] = __builtin_fma(e, e, m2[h0]);
#pragma unroll
            for (int t = 0; t < T; ++t) {
              const double df = x - ring[t];
              v[t] = __builtin_fma(df, df, v[t]);
            }
#pragma unroll
            for (int k = T - 1; k > 0; --k) ring[k] = ring[k - 1];
            ring[0] = x;
          }
          continue;
        }
#pragma unroll
        for (int j = 0; j < kStreamChunk; ++j) {
          if (i0 + j >= rows) break;
          const double x = xs[j];
          const int64_t p = a.pos0 + i0 + j;
          const int h = p >= a.n ? 1 : 0;
          const int sidx = (int)(p - (int64_t)h * a.n);
          if (sidx == 0) sh[h] = x;
          const double e = x - sh[h];
          m1[h] += e;
          m2[h] = __builtin_fma(e, e, m2[h]);
#pragma unroll
          for (int t = 0; t < T; ++t) {
            const double df = x - ring[t];
            v[t] = (t < sidx) ? __builtin_fma(df, df, v[t]) : v[t];   // lag t+1 inside the same half
          }
#pragma unroll
          for (int k = T - 1; k > 0; --k) ring[k] = ring[k - 1];
          ring[0] = x;
        }
      }
      a.shift[o] = sh[0];
      a.shift[o + a.D] = sh[1];
      a.s1[o] = m1[0];
      a.s1[o + a.D] = m1[1];
      a.s2[o] = m2[0];
      a.s2[o + a.D] = m2[1];
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    red[rl][dl] = v[t];
    __syncthreads();
    if (rl == 0 && d < a.D)
      a.vpart[((int64_t)blockIdx.x * T + t) * a.D + d] = ((red[0][dl] + red[1][dl]) + red[2][dl]) + red[3][dl];
    __syncthreads();
  }
}

// The product form (halves of n >= T samples) as its own kernel, T rows per unrolled chunk so that
// every ring slot is a static register: position p lives in slot p mod T (chunks start at
// multiples of T), so the lag products, the ring update and both per-half events (H_t at half
// position T-1, T_t at n-1) index the ring statically -- no ring shifts (T moves per row before).
// Rows arrive by a rolling prefetch (slot p mod PF; the load of row p + PF is issued as row p is
// consumed), so PF rows per wave are always in flight instead of one chunk at a time; a wave's rows
// are one chain's (buffer descriptor on the chain, row offsets in the scalar offset).  Same sums
// in the same order as the difference-form kernel's PROD path had: bit-identical results.
template <int T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(T <= 16 ? 3 : 1))) void k_stream_prod(StreamArgs a) {
  constexpr int PF = T < HMC_STREAM_PF ? T : HMC_STREAM_PF;
  static_assert(T % PF == 0, "prefetch slots repeat per chunk");
  __shared__ double red[4][kDimTile];
  const int dl = threadIdx.x & (kDimTile - 1);
  const int rl = __builtin_amdgcn_readfirstlane(threadIdx.x / kDimTile);   // wave-uniform: one chain per wave
  const int d = blockIdx.y * kDimTile + dl;
  const int dd = d < a.D ? d : a.D - 1;            // lanes past D load a valid element, write nothing
  const int64_t left = 2 * (int64_t)a.n - a.pos0;
  const int rows = (int)(left < a.rows ? (left > 0 ? left : 0) : a.rows);
  const int64_t pos0 = a.pos0, pend = a.pos0 + rows;
  double v[T];
#pragma unroll
  for (int t = 0; t < T; ++t) v[t] = 0.0;
  for (int64_t c = (int64_t)blockIdx.x * 4 + rl; c < a.n_chains; c += (int64_t)a.groups * 4) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double*>(a.x + c * a.chain_stride), 0, -1, 0x00020000);
    auto at = [&](int k) -> double {                // k-th window sample (k < carry + rows)
      int sl = a.slot0 + k;
      sl = sl >= a.wrap ? sl - a.wrap : sl;
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                            rs, dd * 8, (int)(sl * a.sample_stride * 8), 0));
    };
    auto kpos = [&](int64_t p) { return (int)(a.carry + (p - pos0)); };
    const int64_t o = c * 2 * a.D + dd;
    const int hc = pos0 >= a.n ? 1 : 0;
    // the current half's shift and sums; the other half's as stored
    double csh = a.shift[o + hc * a.D], cm1 = a.s1[o + hc * a.D], cm2 = a.s2[o + hc * a.D];
    double sh0 = a.shift[o], m10 = a.s1[o], m20 = a.s2[o];
    const double sh1s = a.shift[o + a.D], m11s = a.s1[o + a.D], m21s = a.s2[o + a.D];
    const int sidx0 = (int)(pos0 - (int64_t)hc * a.n);
    // ring: carry samples of the same half, slot = position mod T
    const int lim = a.carry < sidx0 ? a.carry : sidx0;
    double ring[T];
#pragma unroll
    for (int sl = 0; sl < T; ++sl) {
      const int k = (int)(((pos0 - 1 - sl) % T + T) % T);   // pos0 - 1 - k = position in slot sl
      const int kk = a.carry - 1 - k;
      ring[sl] = at(kk > 0 ? kk : 0);               // unconditional, all issued before any use
    }
    __builtin_amdgcn_sched_barrier(0);              // (the scheduler serialised load -> use pairs)
#pragma unroll
    for (int sl = 0; sl < T; ++sl) {
      const int k = (int)(((pos0 - 1 - sl) % T + T) % T);
      ring[sl] = k < lim ? ring[sl] - csh : 0.0;
    }
    double xs[PF];
#pragma unroll
    for (int sl = 0; sl < PF; ++sl) {
      const int64_t p = pos0 + (((sl - pos0) % PF) + PF) % PF;   // the first row with p = sl mod PF
      xs[sl] = at(kpos(p < pend ? p : pos0));       // (unconditional: rows past the end are unused)
    }
    int nsl = (a.slot0 + kpos(pos0 + PF)) % a.wrap;   // window slot of the next row to prefetch
    const int64_t P0 = pos0 - ((pos0 % T) + T) % T;
    for (int64_t pc = P0; pc < pend; pc += T) {
      auto row = [&](auto j_c) {
        constexpr int j = decltype(j_c)::value;
        const int64_t p = pc + j;
        if (p >= pos0 && p < pend) {                  // uniform
          const double x = xs[j % PF];
          if (p + PF < pend) {                        // row p + PF: a running window slot (scalar;
            int sl = nsl;                             // precomputed per unrolled row they spilled)
            asm volatile("" : "+s"(sl));
            xs[j % PF] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                       rs, dd * 8, (int)(sl * a.sample_stride * 8), 0));
            nsl = sl + 1 == a.wrap ? 0 : sl + 1;
          }
          if (p == a.n) {                            // the call crosses into half 1
            sh0 = csh;
            m10 = cm1;
            m20 = cm2;
            csh = sh1s;
            cm1 = m11s;
            cm2 = m21s;
          }
          const int sidx = (int)(p < a.n ? p : p - a.n);
          if (sidx == 0) {                           // a half starts: its shift, an empty ring
            csh = x;
#pragma unroll
            for (int k = 0; k < T; ++k) ring[k] = 0.0;
          }
          const double y = x - csh;
          cm1 += y;
          cm2 = __builtin_fma(y, y, cm2);
          const double ym2 = -2.0 * y;
#pragma unroll
          for (int t = 0; t < T; ++t) v[t] = __builtin_fma(ym2, ring[(j - 1 - t + 2 * T) % T], v[t]);   // -2 C_t
          ring[j] = y;
          if (sidx == T - 1) {                       // the half's first T samples: H_t = sum_{s<t} y^2
            double q = 0.0;
#pragma unroll
            for (int t = 0; t < T; ++t) {
              const double r = ring[(j - (T - 1) + t + T) % T];
              q = __builtin_fma(r, r, q);
              v[t] -= q;
            }
          }
          if (sidx == a.n - 1) {                     // its last T samples: T_t; then + 2 S2
            double q = 0.0;
            const double s2x2 = 2.0 * cm2;
#pragma unroll
            for (int t = 0; t < T; ++t) {
              const double r = ring[(j - t + T) % T];
              q = __builtin_fma(r, r, q);
              v[t] += s2x2 - q;
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<T>(row);
    }
    if (d < a.D) {
      const bool crossed = pos0 < a.n && pend > a.n;
      if (hc == 1 || crossed) {
        a.shift[o + a.D] = csh;
        a.s1[o + a.D] = cm1;
        a.s2[o + a.D] = cm2;
      }
      if (hc == 0) {
        a.shift[o] = crossed ? sh0 : csh;
        a.s1[o] = crossed ? m10 : cm1;
        a.s2[o] = crossed ? m20 : cm2;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    red[rl][dl] = v[t];
    __syncthreads();
    if (rl == 0 && d < a.D)
      a.vpart[((int64_t)blockIdx.x * T + t) * a.D + d] = ((red[0][dl] + red[1][dl]) + red[2][dl]) + red[3][dl];
    __syncthreads();
  }
}

int64_t rows_chunks(int64_t rows) { return (rows + kRowChunk - 1) / kRowChunk; }

// The matrix-core pass's geometry: ranges R (a multiple of 8) picked so that R x G workgroups (8 waves
// per CU at a time) end in as full a last round as possible, at least 4 rounds.
MfmaArgs mfma_args(const Src& s) {
  MfmaArgs a{};
  a.s = s;
  const int n = s.n;
  a.P = 32 * ((n + 46 - 8 + 31) / 32) + 8;
  a.PK = 4 * a.P + 16;
  a.NT = (n - 1) / 16 + 2;
  a.NB = (n + 14) / 16 + 1;
  a.G = (s.D + kMfmaDims - 1) / kMfmaDims;
  const int64_t m2 = n_series(s);
  const int64_t groups = (m2 + 3) / 4;
  // workgroups resident at a time, as two per CU for every instance: the range count must not
  // depend on n, because diag_conv_work sizes the partials at n = kMfmaMinN for any n (a W3-aware
  // count, 3 per CU below n = 113, made a c3 pass at n = 200 write past a work buffer sized at a
  // different R)
  const int cus = device_cus() * 2;
  int best = 8;
  double best_eff = -1.0;
  for (int x = 1; x <= 64; ++x) {
    const int64_t R = 8 * x;
    if (R > groups) break;
    const int64_t wgs = R * a.G;
    const int64_t rounds = (wgs + cus - 1) / cus;
    double eff = (double)wgs / (double)(rounds * cus);
    if (rounds < 4) eff *= 0.5;                   // too few workgroups per CU to balance
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = (int)R;
    }
  }
  a.R = best;
  a.per = ((groups + a.R - 1) / a.R) * 4;
  return a;
}

// Stored split chains (halves 2) or completed halves of a streaming window that do not wrap
// (halves 1, wrap 0).  The staging's 32-bit lane offsets span a group's four series: two chains'
// rows (split chains) or four chains' (halves).
bool mfma_ok(const Src& s, int T) {
  const int64_t rows = (int64_t)s.n * s.sample_stride;
  const int64_t span = (s.halves == 2 ? 2 * s.chain_stride + 2 * rows : 3 * s.chain_stride + rows) + s.D;
  return (s.halves == 2 || s.halves == 1) && s.wrap == 0 && s.n >= kMfmaMinN && s.n <= kMfmaMaxN &&
         T >= s.n - 2 && n_series(s) >= 4 && s.chain_stride >= rows && span * 8 < kLagOOB;
}

// the samples, x0, the slack for the read-ahead past the last series, the sq rows
size_t mfma_lds(const MfmaArgs& a) {
  // k_conv_mfma<NTM <= 10> (n <= 144) keeps the sq rows in registers (no LDS for them) and
  // double-buffers the samples and x0 (PIPE)
  const bool small = a.s.n <= 16 * 9;
  const size_t buf = (size_t)(4 * a.PK + kMfmaSer);
  return ((small ? 2 : 1) * buf + kMfmaSlack + (small ? 0 : kMfmaSer * kSqStride)) * sizeof(double);
}

int64_t mfma_work(const MfmaArgs& a) {
  return (int64_t)a.R * a.G * kMfmaDims * kMfmaPW + (int64_t)a.s.D * kMfmaPW;
}

// the matrix-core partials' bound that diag_conv_work reserves (the geometry at n = kMfmaMinN,
// either series layout): every launch checks its own geometry against it
int64_t mfma_work_bound(int64_t n_chains, int D) {
  int64_t w = 0;
  for (int halves = 1; halves <= 2; ++halves) {
    Src s{nullptr, 0, 0, 0, n_chains, kMfmaMinN, D, halves};
    w = std::max(w, mfma_work(mfma_args(s)));
  }
  return w;
}

hipError_t launch_conv_mfma(const Src& s, int nlag, double* work, double* out, hipStream_t st) {
  const MfmaArgs a = mfma_args(s);
  if (mfma_work(a) > mfma_work_bound(s.n_chains, s.D)) return hipErrorInvalidValue;   // never past the work
  double* partial = work;
  double* red = work + (int64_t)a.R * a.G * kMfmaDims * kMfmaPW;
  const unsigned grid = (unsigned)(a.R * a.G);
  if (s.n <= 16 * 5) k_conv_mfma<6><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
  else if (s.n <= 16 * 7) {
    const int e4 = ((s.n & 15) >> 2) + 1;         // row groups of the steps' last tiles
    if (s.n < 97 || s.n > 111) k_conv_mfma<8><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else if (e4 == 1) k_conv_mfma<8, 1, 6><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else if (e4 == 2) k_conv_mfma<8, 2, 6><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else if (e4 == 3) k_conv_mfma<8, 3, 6><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else k_conv_mfma<8, 0, 6><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
  }
  else if (s.n <= 16 * 9) k_conv_mfma<10><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
  else if (s.n <= 16 * 11) k_conv_mfma<12><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
  else if (s.n < 193 || s.n > 207) k_conv_mfma<14><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
  else {                                          // c3's n = 200: E4 = 3
    const int e4 = ((s.n & 15) >> 2) + 1;
    if (e4 == 1) k_conv_mfma<14, 1, 12><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else if (e4 == 2) k_conv_mfma<14, 2, 12><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else if (e4 == 3) k_conv_mfma<14, 3, 12><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
    else k_conv_mfma<14, 0, 12><<<grid, kMfmaThreads, mfma_lds(a), st>>>(a, partial);
  }
  if (hipError_t e = hipGetLastError()) return e;
  const int64_t nr = (int64_t)s.D * kMfmaPW;
  k_mfma_ranges<<<(unsigned)((nr + 255) / 256), 256, 0, st>>>(a, partial, red);
  if (hipError_t e = hipGetLastError()) return e;
  const int64_t no = (int64_t)(nlag + 4) * s.D;
  k_mfma_dims<<<(unsigned)((no + 255) / 256), 256, 0, st>>>(a, red, nlag, out);
  return hipGetLastError();
}

// G lag groups (and the tail) of a pass over lags L0 + 1 .. L0 + T.  A first pass (mom) asking for
// every lag (T >= n - 2; lag n - 1 always comes from the tail) runs the groups up to lag
// n - 1 - tail only and sums the rest, tail <= kLagTail lags, in difference form.
LagArgs lag_args(const Src& s, int L0, int T, int mom) {
  LagArgs a{};
  a.s = s;
  a.L0 = L0;
  a.T = T;
  a.G = (T + kLagTL - 1) / kLagTL;
  a.mom = mom;
  a.tail = mom ? 1 : 0;
  if (mom && L0 == 0 && T >= s.n - 2 && s.n >= 2) {
    const int need = s.n - 1 - kLagTail;           // lags the groups must cover at least
    const int G = need > 0 ? (need + kLagTL - 1) / kLagTL : 1;
    const int Tg = std::min(G * kLagTL, s.n - 2);
    a.G = G;
    a.T = Tg > 0 ? Tg : 0;
    a.tail = s.n - 1 - a.T;
  }
  a.C = s.D / lag_gcd(s.D, 64);
  a.NT = (n_series(s) * (int64_t)s.D + 63) / 64;
  const int64_t per_class = (a.NT + a.C - 1) / a.C;
  const int64_t R = (kLagWaves + (int64_t)a.C * a.G - 1) / ((int64_t)a.C * a.G);
  a.R = (int)(R < per_class ? (R < 1 ? 1 : R) : per_class);
  a.rowb = (int)(s.sample_stride * 8);
  return a;
}

int64_t lag_grid(const LagArgs& a) { return 8 * (int64_t)a.G * (((int64_t)a.C * a.R + 7) / 8); }
int64_t lag_work(const LagArgs& a) {
  return lag_grid(a) * kLagRows * 64 + (int64_t)a.C * a.G * kLagRows * 64;
}

// Work (doubles) that any pass of at most T lags (L0 = 0, n unknown: a complete first pass may take
// fewer groups than ceil(T / TL)) over n_chains chains of D dims needs: the largest over the group
// counts it could run.
int64_t lag_work_bound(int64_t n_chains, int D, int T, int mom) {
  int64_t w = 0;
  const int Gmax = (T + kLagTL - 1) / kLagTL;
  for (int G = 1; G <= Gmax; ++G) {
    Src s{nullptr, 0, 0, 0, n_chains, 2, D};
    LagArgs a = lag_args(s, 0, G * kLagTL, 0);   // geometry of G groups (pairs: the most series)
    a.mom = mom;
    w = std::max(w, lag_work(a));
  }
  return w;
}

// One read of the samples: lags L0 + 1 .. L0 + T (group 0 also the moments when mom), reduced into
// out (conv layout or lags only, from lag L0 + 1 + skip, nlag lags).
// Lane offsets (bytes from a tile's first series) and row offsets must stay inside the buffer
// bound kLagOOB (1 GiB): a tile spans at most 64 / D + 2 series; the second half of a chain starts
// n * sample_stride after its first (chain_stride >= that for every q_chain view).  So one chain's
// samples (its stride) must stay well within 1 GiB: e.g. D = 1000 up to ~40,000 stored samples per
// chain, D = 100 up to ~400,000 (hmc_amd.diagnostics splits larger views by dimension).
bool lag_view_ok(const Src& s) {
  const int64_t cs = s.chain_stride, ss = s.sample_stride;
  if (ss < 1 || ss * 8 > 0x7FFFFFFF || s.D < 1) return false;
  if (s.halves == 2) {
    if (cs < (int64_t)s.n * ss) return false;
    const int64_t span = ((64 / s.D + 2) / 2 + 1) * cs + (int64_t)s.n * ss + s.D;   // doubles
    return (span + (int64_t)s.n * ss) * 8 < kLagOOB;
  }
  // one series per chain: a tile spans at most 64 / D + 2 chains; rows up to the window's last
  const bool wr = s.wrap > 0;
  const int64_t rows = wr ? (int64_t)s.wrap : (int64_t)s.n;
  if (wr && (s.slot0 < 0 || s.slot0 >= s.wrap || s.n > s.wrap)) return false;
  const int64_t span = (64 / s.D + 2) * cs + s.D;
  return (span + rows * ss) * 8 < kLagOOB;
}

hipError_t launch_lags(const Src& s, int L0, int T, int mom, int conv, int skip, int nlag, double* work, double* out,
                       hipStream_t st) {
  if (T < 1 || L0 < 0 || L0 % kLagPF != 0) return hipErrorInvalidValue;
  if (!lag_view_ok(s)) return hipErrorInvalidValue;
  const bool wr = s.halves == 1 && s.wrap > 0;
  const LagArgs a = lag_args(s, L0, T, mom);
  const int64_t grid = lag_grid(a);
  double* partial = work;
  double* inter = work + grid * kLagRows * 64;
  if (wr) k_conv_series<kLagTL, kLagPF, true><<<(unsigned)grid, 64, 0, st>>>(a, partial);
  else k_conv_series<kLagTL, kLagPF, false><<<(unsigned)grid, 64, 0, st>>>(a, partial);
  if (hipError_t e = hipGetLastError()) return e;
  const int64_t ni = (int64_t)a.C * a.G * kLagRows * 64;
  k_lag_classes<<<(unsigned)((ni + 255) / 256), 256, 0, st>>>(a, partial, inter);
  if (hipError_t e = hipGetLastError()) return e;
  const int64_t no = (int64_t)(conv ? nlag + 4 : nlag) * s.D;
  k_lag_dims<<<(unsigned)((no + 255) / 256), 256, 0, st>>>(a, inter, conv, skip, nlag, out);
  return hipGetLastError();
}

}  // namespace

int64_t diag_rowsum_work(int64_t rows, int D) { return rows_chunks(rows) * D; }

bool diag_view_ok(int64_t n_chains, int64_t cs, int64_t ss, int n, int D, int halves, int wrap, int slot0) {
  Src s{nullptr, cs, ss, 0, n_chains, n, D, halves, wrap, slot0};
  return lag_view_ok(s);
}

int64_t diag_variogram_work(int64_t n_chains, int D, int nlags) {
  Src s{nullptr, 0, 0, 0, n_chains, 2, D};
  return lag_work(lag_args(s, 0, nlags + kLagPF - 1, 0));   // the lag range may start up to PF-1 lower
}

hipError_t launch_split_moments(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n,
                                int D, double* mean_out, double* std_out, hipStream_t st) {
  Src s{x, cs, ss, base, n_chains, n, D};
  const int64_t m2 = 2 * n_chains;
  dim3 grid((unsigned)((m2 + 3) / 4), (unsigned)((D + kDimTile - 1) / kDimTile));
  k_split_moments<<<grid, 256, 0, st>>>(s, mean_out, std_out);
  return hipGetLastError();
}

hipError_t launch_rowsum(const double* x, int64_t n_outer, int64_t os, int64_t n_inner, int64_t is, int64_t base,
                         int D, const double* center, double* work, double* out, hipStream_t st) {
  Rows r{x, n_outer, os, n_inner, is, base, D, center};
  const int64_t nch = rows_chunks(n_outer * n_inner);
  dim3 grid((unsigned)nch, (unsigned)((D + kDimTile - 1) / kDimTile));
  k_rowsum_partial<<<grid, 256, 0, st>>>(r, work);
  if (hipError_t e = hipGetLastError()) return e;
  k_colsum_final<<<(unsigned)((D + 255) / 256), 256, 0, st>>>(work, nch, D, out);
  return hipGetLastError();
}

int64_t diag_conv_work(int64_t n_chains, int D, int T) {
  int64_t w = lag_work_bound(n_chains, D, T, 1);
  // a complete pass of split chains of kMfmaMinN .. T + 2 samples may take the matrix cores (their
  // geometry depends on the chains and dims only)
  if (T + 2 >= kMfmaMinN) w = std::max(w, mfma_work_bound(n_chains, D));   // stored split chains or halves
  return w;
}

hipError_t launch_conv_fused(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n, int D,
                             int T, double* work, double* out, hipStream_t st) {
  Src s{x, cs, ss, base, n_chains, n, D};
#ifndef HMC_LAG_NO_MFMA
  if (mfma_ok(s, T)) return launch_conv_mfma(s, T, work, out, st);
#endif
  return launch_lags(s, 0, T, 1, 1, 0, T, work, out, st);
}

hipError_t launch_half_sums(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int D, int wrap, int slot0,
                            int n, int T, double* work, double* out, hipStream_t st) {
  // a half that does not reach the window's end reads plain strided rows (no per-row wrap)
  if (wrap > 0 && slot0 + n <= wrap) wrap = 0;
  Src s{x, cs, ss, 0, n_chains, n, D, 1, wrap, slot0};
  if (wrap <= 0) s.base = (int64_t)slot0 * ss;   // no wrap: sample s in row slot0 + s
#ifndef HMC_LAG_NO_MFMA
  if (mfma_ok(s, T)) return launch_conv_mfma(s, T, work, out, st);
#endif
  return launch_lags(s, 0, T, 1, 1, 0, T, work, out, st);
}

int64_t diag_stream_groups(int64_t n_chains) {
  const int64_t g = (n_chains + 3) / 4;
  return g < 1024 ? (g < 1 ? 1 : g) : 1024;
}

hipError_t launch_stream_accum(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int D, int wrap, int slot0,
                               int carry, int rows, int64_t pos0, int n, double* shift, double* s1, double* s2, int T,
                               double* vpart, double* vsum, hipStream_t st) {
  if ((int64_t)wrap * ss * 8 >= 0x7FFFFFFF) return hipErrorInvalidValue;   // row offsets: 32-bit scalar offsets
  const int64_t groups = diag_stream_groups(n_chains);
  StreamArgs a{x, n_chains, cs, ss, D, wrap, slot0, carry, rows, n, pos0, shift, s1, s2, vpart, (int)groups};
  dim3 grid((unsigned)groups, (unsigned)((D + kDimTile - 1) / kDimTile));
  // the product form needs every half to reach position T-1 (its H_t event); both forms give the
  // same sums of every completed half, and a run keeps one form (n and T are fixed per run)
  const bool prod = n >= T;
  auto go = [&](auto t_c) {
    constexpr int TT = decltype(t_c)::value;
    if (prod) k_stream_prod<TT><<<grid, 256, 0, st>>>(a);
    else k_stream_accum<TT, false><<<grid, 256, 0, st>>>(a);
  };
  switch (T) {
    case 8: go(std::integral_constant<int, 8>{}); break;
    case 16: go(std::integral_constant<int, 16>{}); break;
    case 32: go(std::integral_constant<int, 32>{}); break;
    case 64: go(std::integral_constant<int, 64>{}); break;
    default: return hipErrorInvalidValue;
  }
  if (hipError_t e = hipGetLastError()) return e;
  const int64_t ncols = (int64_t)T * D;   // vsum[t][d] += sum over groups (accumulated across calls)
  k_colsum_acc<<<(unsigned)((ncols + 255) / 256), 256, 0, st>>>(vpart, groups, ncols, vsum);
  return hipGetLastError();
}

hipError_t launch_variogram(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n, int D,
                            int t0, int t1, double* work, double* out, hipStream_t st) {
  Src s{x, cs, ss, base, n_chains, n, D};
  const int L0 = (t0 - 1) / kLagPF * kLagPF;   // the pass starts at a prefetch-aligned lag
  return launch_lags(s, L0, t1 - 1 - L0, 0, 0, t0 - 1 - L0, t1 - t0, work, out, st);
}

}  // namespace hmc
