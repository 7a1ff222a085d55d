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
};

__device__ __forceinline__ const double* split_ptr(const Src& s, int64_t j, int smp) {
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

// partial[chunk][k][d] = sum over the chunk's split chains j of sum_s (x_j[s+t]-x_j[s])^2 for the lags
// t = t0 + k, k < nt <= T.  ONE pass over the samples (round 1 re-read the chain once per lag):
// each thread walks its chains' samples s = t0 .. n-1 with a register ring holding
// x[s-t0], x[s-t0-1], ..., x[s-t0-T+1]; per sample it reads x[s] and the delayed x[s-t0] (the same
// value for t0 = 1, a second, cache-friendly stream otherwise).  Lane = dim: coalesced rows.
template <int T>
__global__ __launch_bounds__(256) void k_variogram_ring(Src s, int t0, int nt, int64_t jchunk, double* partial) {
  __shared__ double red[4][kDimTile];
  const int dl = threadIdx.x & (kDimTile - 1);
  const int rl = threadIdx.x / kDimTile;
  const int d = blockIdx.y * kDimTile + dl;
  const int64_t j0 = (int64_t)blockIdx.x * jchunk;
  const int64_t j1 = min(j0 + jchunk, 2 * s.n_chains);
  const int64_t ss = s.sample_stride;
  double v[T];
#pragma unroll
  for (int k = 0; k < T; ++k) v[k] = 0.0;
  if (d < s.D) {
    for (int64_t j = j0 + rl; j < j1; j += 4) {
      const double* b = split_ptr(s, j, 0) + d;
      double ring[T];
#pragma unroll
      for (int k = 0; k < T; ++k) ring[k] = 0.0;
      int i = t0;
      // fill: ring slot k is valid once i - t0 >= k
      for (; i < s.n && i - t0 < T - 1; ++i) {
#pragma unroll
        for (int k = T - 1; k > 0; --k) ring[k] = ring[k - 1];
        ring[0] = b[(int64_t)(i - t0) * ss];
        const double x = b[(int64_t)i * ss];
#pragma unroll
        for (int k = 0; k < T; ++k) {
          const double e = x - ring[k];
          v[k] = (k <= i - t0) ? __builtin_fma(e, e, v[k]) : v[k];
        }
      }
      for (; i < s.n; ++i) {
#pragma unroll
        for (int k = T - 1; k > 0; --k) ring[k] = ring[k - 1];
        ring[0] = b[(int64_t)(i - t0) * ss];
        const double x = b[(int64_t)i * ss];
#pragma unroll
        for (int k = 0; k < T; ++k) {
          const double e = x - ring[k];
          v[k] = __builtin_fma(e, e, v[k]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < T; ++k) {
    if (k < nt) {
      red[rl][dl] = v[k];
      __syncthreads();
      if (rl == 0 && d < s.D)
        partial[((int64_t)blockIdx.x * nt + k) * s.D + d] = ((red[0][dl] + red[1][dl]) + red[2][dl]) + red[3][dl];
      __syncthreads();
    }
  }
}

// ---- ONE pass for convergence_stats (utils.py:88-126 and :161-179).  Per split chain j (n samples)
// and dim d, with y = x - x_j[0] (shifted: the sums stay well conditioned):
//   mean_j = (x[0] + x[1] + ... + x[n-1]) / n, summed in sample order without FMA: NumPy's np.mean
//   over axis 0 bit for bit (np.std(ddof=1) at utils.py:109-112 starts from it);
//   s1 = sum y, S2 = sum y^2, delta = mean_j - x_j[0]:
//   sum (x - mean_j)^2 = S2 - 2 delta s1 + n delta^2 (NumPy's second pass, up to rounding: for a chain
//   that never moved, e.g. every proposal rejected, it is n delta^2 with NumPy's own delta, so
//   W = mean std_j keeps the reference's rounding-level value instead of an exact 0)
//   V_t,j = sum_{s<n-t} (y[s+t] - y[s])^2 = 2 S2 - H_t - T_t - 2 C_t,  C_t = sum_s y[s] y[s-t],
//   H_t = sum_{s<t} y^2 (the first t samples), T_t = sum_{s>=n-t} y^2 (the last t)
// so a lag costs ONE FMA per sample (v += (-2 y[s]) y[s-t] against a register ring) instead of a
// subtraction and an FMA.  The lags are split over G waves (lag group g: lags gTW+1 .. gTW+TW, a
// ring fed by the sample stream delayed by gTW), so T = G*TW lags fit the register file:
//   * samples run in chunks of TW; chunk g is exactly the positions whose running S2 is H_t of
//     this wave's lags (static register index inside the unrolled chunk);
//   * at the end the ring holds y[n-1-gTW-k], so T_t = (S2 - S2 through position n-1-gTW) +
//     cumulative squares of the ring.
// Sums over the block's split chains:
//   row 0: sum_j std_j, row 1: sum_j (mean_j - S_d), row 2: sum_j (mean_j - S_d)^2,
//   row 3 + t - 1: sum_j V_t,j for lags t = 1..T (valid for t < n), S_d = x[base + d].
// Block = 4 waves = 4/G split chains at a time x G lag groups, lane = dim (coalesced rows).  The dim
// tiles of one chain group run on the same XCD (block b on XCD b % 8), so a row's line shared by
// two tiles is fetched from HBM once.
template <int TW, int G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_conv_lags(Src s, int groups,
                                                                                             int ntiles,
                                                                                             double* partial) {
  constexpr int SL = 4 / G;             // split chains per block at a time
  constexpr int T = TW * G;
  __shared__ double red[4][kDimTile];
  const int dl = threadIdx.x & (kDimTile - 1);
  const int w = threadIdx.x / kDimTile;
  const int slot = w / G, g = w % G;    // wave-uniform
  const int gofs = g * TW;              // this wave's lags: gofs + 1 .. gofs + TW
  const int b = blockIdx.x;             // XCD-aware: tiles of a group 8 blocks apart
  const int tile = (b >> 3) % ntiles;
  const int grp = (b & 7) + 8 * ((b >> 3) / ntiles);
  const int d = tile * kDimTile + dl;
  const int64_t m2 = 2 * s.n_chains;
  const int64_t ss = s.sample_stride;
  const int n = s.n;
  double v[TW];
#pragma unroll
  for (int k = 0; k < TW; ++k) v[k] = 0.0;
  double a_std = 0.0, a_m = 0.0, a_m2 = 0.0, a_last = 0.0;
  if (d < s.D && grp < groups && slot < SL) {   // (G = 3: the fourth wave idles)
    const double S = s.x[s.base + d];
    const int pos_suf = n - gofs - 1;   // T_t needs S2 through this position
    for (int64_t j = (int64_t)grp * SL + slot; j < m2; j += (int64_t)groups * SL) {
      const double* bp = split_ptr(s, j, 0) + d;
      const double sh = bp[0];
      double ring[TW];
#pragma unroll
      for (int k = 0; k < TW; ++k) ring[k] = 0.0;
      double s1 = 0.0, s2 = 0.0, r1 = 0.0, sufb = 0.0;
      for (int c0 = 0; c0 < n; c0 += TW) {
        double xc[TW], xd[TW];
#pragma unroll
        for (int i = 0; i < TW; ++i) {
          const int sp = c0 + i, sq = sp - gofs;
          xc[i] = sp < n ? bp[(int64_t)sp * ss] : 0.0;
          xd[i] = (sq >= 0 && sq < n) ? bp[(int64_t)sq * ss] : sh;   // delayed stream (y = 0 before 0)
        }
        const bool hwin = c0 == gofs;   // uniform: this chunk's running S2 gives H_t of our lags
#pragma unroll
        for (int i = 0; i < TW; ++i) {
          const int sp = c0 + i;
          if (sp < n) {                 // uniform
            r1 += xc[i];
            const double y = xc[i] - sh;
            s1 += y;
            s2 = __builtin_fma(y, y, s2);
            const double ym2 = -2.0 * y;
#pragma unroll
            for (int k = 0; k < TW; ++k) v[k] = __builtin_fma(ym2, ring[k], v[k]);
            if (hwin) v[i] -= s2;       // H_t, t = gofs + 1 + i
            if (sp == pos_suf) sufb = s2;
#pragma unroll
            for (int k = TW - 1; k > 0; --k) ring[k] = ring[k - 1];
            ring[0] = xd[i] - sh;       // y[sp - gofs]
          }
        }
      }
      // ring[k] = y[n-1-gofs-k]: T_t = (S2 - S2 through n-1-gofs) + sum_{k' <= k} ring[k']^2
      double q = pos_suf >= 0 ? s2 - sufb : s2;
      const double s2x2 = 2.0 * s2;
#pragma unroll
      for (int k = 0; k < TW; ++k) {
        q = __builtin_fma(ring[k], ring[k], q);
        v[k] += s2x2 - q;
      }
      const double mean = r1 / n;
      const double dm = mean - sh;
      const double mm2 = (s2 - 2.0 * dm * s1) + n * (dm * dm);
      a_std += sqrt(mm2 > 0.0 ? mm2 / (n - 1) : 0.0);
      const double e = mean - S;
      a_m += e;
      a_m2 = __builtin_fma(e, e, a_m2);
      const double yl = bp[(int64_t)(n - 1) * ss] - sh;   // lag n - 1: (x[n-1] - x[0])^2
      a_last = __builtin_fma(yl, yl, a_last);
    }
  }
  auto put = [&](int row, double x) {
    red[w][dl] = x;
    __syncthreads();
    if (w == 0 && d < s.D && grp < groups)
      partial[((int64_t)grp * (T + 4) + row) * s.D + d] = ((red[0][dl] + red[1][dl]) + red[2][dl]) + red[3][dl];
    __syncthreads();
  };
  put(0, g == 0 ? a_std : 0.0);
  put(1, g == 0 ? a_m : 0.0);
  put(2, g == 0 ? a_m2 : 0.0);
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
#pragma unroll
    for (int k = 0; k < TW; ++k) put(3 + gg * TW + k, g == gg && gg * TW + k + 1 < s.n ? v[k] : 0.0);   // lags t >= n: 0
  }
  put(3 + T, g == 0 && s.n >= 2 ? a_last : 0.0);  // lag n - 1 (the ESS loop's last), whatever T
}

// The same sums with the series staged through LDS: each block runs SL = 4/G split chains at a time
// (G waves each, one per lag group, as k_conv_lags) through a per-slot LDS ring of rows (lane = dim).
// The G waves of a slot bring the slot's next rows in with direct-to-LDS loads
// (global_load_lds_dwordx4: 16 B per lane, two 512-B rows per wave-instruction, no registers),
// PD chunks of TW rows ahead, and every wave reads its current row and its delayed row (gTW back)
// from the ring: one HBM read per element, no load buffers in registers, and the loads of PD
// chunks in flight behind the lag products (the register-staged k_conv_lags is latency-bound).
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

// this lane's id in its wave, recomputed where it is used (volatile: never kept live across a
// loop, which costs two VALU instead of a register or a scratch reload)
__device__ __forceinline__ int lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// waves per block, and waves per SIMD (the launch bound: registers) of k_conv_lds<TW, G, 2>; the
// LDS ring allows 4 / 3 / 2 / 1 / 3 blocks per CU for G = 3 / 4 / 2 / 1 (TW 16) / 1 (TW 8)
constexpr int conv_waves(int G) { return G == 3 ? 3 : 4; }
constexpr int conv_wpe(int TW, int G) { return G >= 3 ? 3 : G == 2 ? 2 : TW == 16 ? 1 : 3; }

template <int TW, int G, int PD>
__global__ __launch_bounds__(64 * conv_waves(G), conv_wpe(TW, G)) void k_conv_lds(Src s, int groups, int ntiles,
                                                                                  double* partial) {
  constexpr int NW = conv_waves(G);               // waves per block
  constexpr int SL = NW / G;                      // split chains per block at a time
  constexpr int T = TW * G;
  constexpr int RB = (G + PD) * TW;               // ring rows per slot (multiple of TW)
  constexpr int NP = TW / 2;                      // DMA instructions per chunk (2 rows each)
  static_assert(SL * G == NW && TW % 2 == 0 && (TW & (TW - 1)) == 0, "layout");
  __shared__ double ring_x[SL * RB * kDimTile];   // (the final reduction reuses it)
  const int lane = threadIdx.x & (kDimTile - 1);
  const int dl = lane;
  const int w = threadIdx.x / kDimTile;
  const int slot = w / G, g = w % G;
  const int gofs = g * TW;
  const int b = blockIdx.x;                       // XCD-aware: tiles of a group 8 blocks apart
  const int tile = (b >> 3) % ntiles;
  const int grp = (b & 7) + 8 * ((b >> 3) / ntiles);
  const int d = tile * kDimTile + dl;
  const int64_t m2 = 2 * s.n_chains;
  const int n = s.n;
  const int nch = (n + TW - 1) / TW;              // chunks per split chain
  const int64_t stride = (int64_t)groups * SL;
  const int64_t j0 = (int64_t)grp * SL;
  const int K = grp < groups ? (int)((m2 - j0 + stride - 1) / stride) : 0;   // split chains per slot (max)
  const int F = K * nch;                          // (split chain, chunk) items, the same for all slots
  double* const my = ring_x + slot * RB * kDimTile;
  // DMA of item f into ring rows (f TW) % RB ...: wave g moves row pairs g, g + G, ... of the chunk
  constexpr int NI = (NP + G - 1) / G;            // DMA instructions per wave and chunk (G = 3: the
                                                  // last wave repeats pair NP - 1: same bytes, same place)
  const int dcol = (lane & 31) * 2;               // this lane's dim pair (and row lane >> 5 of 2)
  // per-lane part of a DMA address: this lane's dim pair (pair 0 for the dims past D: loaded,
  // never read), and rows clamped into the split chain (rows past n are loaded, never read)
  const int dofs = tile * kDimTile + dcol < s.D ? tile * kDimTile + dcol : 0;
  auto issue = [&](int f) {
    const int64_t j = j0 + slot + (int64_t)(f / nch) * stride;
    const int cc = f % nch;
    const double* rb = split_ptr(s, j < m2 ? j : m2 - 1, 0);   // wave-uniform
    rb = reinterpret_cast<const double*>(
        ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)rb >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)rb));
    const int r0 = (f * TW) % RB;
#pragma unroll
    for (int e = 0; e < NI; ++e) {
      const int rr = 2 * min(g + G * e, NP - 1);  // row pair inside the chunk
      const int row = min(cc * TW + rr + (lane_id() >> 5), n - 1);
      const double* src = rb + (int64_t)row * s.sample_stride + dofs;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(my + (r0 + rr) * kDimTile),
                                       16, 0, 0);
    }
  };
  double v[TW];
#pragma unroll
  for (int k = 0; k < TW; ++k) v[k] = 0.0;
  double a_std = 0.0, a_m = 0.0, a_m2 = 0.0, a_last = 0.0;
  const double S = d < s.D ? s.x[s.base + d] : 0.0;
  asm volatile("" ::"v"(S));                      // landed before the ring's loads are in flight: a
                                                  // later first use would wait for vmcnt(0)
  // ring slot i holds -2 (x_delayed - shift) of chunk row i (the chunks are TW-aligned), so at row
  // i lag gofs + 1 + k reads slot (i - 1 - k) mod TW: static registers, no ring shifts, and the
  // lag product is one FMA (-2 y x_d: scaling by -2 is exact)
  double ring[TW];
  double sh = 0.0, sh2 = 0.0, s1 = 0.0, s2 = 0.0, r1 = 0.0, sufb = 0.0;
  const int pos_suf = n - gofs - 1;
  for (int f = 0; f < PD && f < F; ++f) issue(f);
  for (int f = 0; f < F; ++f) {
    // item f's rows have landed (PD - 1 newer items may still fly), and every wave is past item f-1
    if (f + PD - 1 < F) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((PD - 1) * NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (f + PD < F) issue(f + PD);
    const int64_t j = j0 + slot + (int64_t)(f / nch) * stride;
    const int cc = f % nch;
    const int rc = (f * TW) % RB;                 // ring row of this chunk's first row
    const int rd = (rc - gofs + RB) % RB;         // ... of the delayed stream's
    if (j < m2 && d < s.D) {
      if (cc == 0) {                              // a split chain starts
        sh = my[rc * kDimTile + lane_id()];
        sh2 = 2.0 * sh;
#pragma unroll
        for (int k = 0; k < TW; ++k) ring[k] = 0.0;
        s1 = s2 = r1 = sufb = 0.0;
      }
      const int rem = n - cc * TW;                // rows of this chunk
      const bool hwin = cc * TW == gofs;          // this chunk's running S2 gives H_t of our lags
      const bool dly = cc * TW >= gofs;           // the delayed rows exist (gofs is a multiple of TW)
      const int isuf = pos_suf - cc * TW;         // suffix mark (T_t terms), if inside this chunk
      auto rows = [&](auto plain_c, auto mom_c, auto dly_c, auto ev_c) {
        constexpr bool PLAIN = decltype(plain_c)::value;   // whole chunk, no H_t / suffix event
        constexpr bool MOM = decltype(mom_c)::value;       // lag group 0 also sums the moments
        constexpr bool DLY = decltype(dly_c)::value;       // the delayed rows exist (else: the shift)
        constexpr int EV = decltype(ev_c)::value;          // events in this chunk: 1 H_t, 2 suffix mark
        // rows one ahead: row i + 1's two LDS reads are issued before row i's FMAs, and no later
        // read moves above them (compiler fence), so at most two rows' values are live: a spill
        // reload here would wait for vmcnt(0), i.e. for the ring's in-flight loads
        const int ll = lane_id();                 // (recomputed: not worth a register)
        double xn = my[rc * kDimTile + ll];
        double xdn = DLY ? my[rd * kDimTile + ll] : sh;
#pragma unroll
        for (int i = 0; i < TW; ++i) {
          const double x = xn, xd = xdn;
          if (i + 1 < TW && (PLAIN || i + 1 < rem)) {
            xn = my[(rc + i + 1) * kDimTile + ll];
            xdn = DLY ? my[(rd + i + 1) * kDimTile + ll] : sh;
          }
          asm volatile("" ::: "memory");
          if (PLAIN || i < rem) {
            const double y = x - sh;
            if constexpr (MOM) {
              r1 += x;
              s1 += y;
            }
            s2 = __builtin_fma(y, y, s2);
#pragma unroll
            for (int k = 0; k < TW; ++k) v[k] = __builtin_fma(y, ring[(i - 1 - k) & (TW - 1)], v[k]);
            if constexpr (EV & 1) v[i] -= s2;
            if constexpr (EV & 2) {
              if (i == isuf) sufb = s2;
            }
            ring[i] = __builtin_fma(-2.0, xd, sh2);   // -2 (xd - sh), one rounding: exact scaling
          }
        }
      };
      const bool suf = isuf >= 0 && isuf < TW;
      const bool plain = rem >= TW && !hwin && !suf;
      // dly and the chunk's events as template arguments: g is not wave-uniform to the compiler,
      // so runtime flags made every delayed read an exec-masked branch (a default move and mask
      // saves per row) and every row of an event chunk two selects
      auto go = [&](auto mom_c, auto dly_c) {
        if (plain) {
          rows(std::true_type{}, mom_c, dly_c, std::integral_constant<int, 0>{});
        } else {
          auto f = [&](auto ev_c) { rows(std::false_type{}, mom_c, dly_c, ev_c); };
          static_dispatch<4>((hwin ? 1 : 0) | (suf ? 2 : 0), f);
        }
      };
      if (g == 0) go(std::true_type{}, std::true_type{});   // g = 0: dly always
      else if (dly) go(std::false_type{}, std::true_type{});
      else go(std::false_type{}, std::false_type{});
      if (cc == nch - 1) {                        // the split chain is complete
        // q4 = 4 (S2 - S2 through n-1-gofs) + sum of the ring's (-2 y)^2: 4x the T_t suffix sums,
        // exactly (power-of-2 scalings commute with rounding)
        double q4 = 4.0 * (pos_suf >= 0 ? s2 - sufb : s2);
        const double s2x2 = 2.0 * s2;
        // the k-th latest delayed value sits in slot (n - 1 - k) mod TW: one static rotation per n
        auto fin = [&](auto rl_c) {
          constexpr int RL = decltype(rl_c)::value;
#pragma unroll
          for (int k = 0; k < TW; ++k) {
            const double rk = ring[(RL - k) & (TW - 1)];
            q4 = __builtin_fma(rk, rk, q4);
            v[k] += __builtin_fma(-0.25, q4, s2x2);
          }
        };
        static_dispatch<TW>((n - 1) & (TW - 1), fin);
        if (g == 0) {
          int nn = n;
          asm volatile("" : "+s"(nn));            // n's doubles: converted here, not kept in registers
          const double dn = nn;
          const double mean = r1 / dn;
          const double dm = mean - sh;
          const double mm2 = (s2 - 2.0 * dm * s1) + dn * (dm * dm);
          a_std += sqrt(mm2 > 0.0 ? mm2 / (dn - 1.0) : 0.0);
          const double e = mean - S;
          a_m += e;
          a_m2 = __builtin_fma(e, e, a_m2);
          const double yl = my[(rc + rem - 1) * kDimTile + lane_id()] - sh;   // lag n - 1: (x[n-1] - x[0])^2
          a_last = __builtin_fma(yl, yl, a_last);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                // every wave is done with the ring
  double* const red = ring_x;                     // [NW][kDimTile]
  auto put = [&](int row, double x) {
    red[w * kDimTile + dl] = x;
    __syncthreads();
    if (w == 0 && d < s.D && grp < groups) {
      double acc = red[dl];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) acc += red[ww * kDimTile + dl];
      partial[((int64_t)grp * (T + 4) + row) * s.D + d] = acc;
    }
    __syncthreads();
  };
  put(0, g == 0 ? a_std : 0.0);
  put(1, g == 0 ? a_m : 0.0);
  put(2, g == 0 ? a_m2 : 0.0);
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
#pragma unroll
    for (int k = 0; k < TW; ++k) put(3 + gg * TW + k, g == gg && gg * TW + k + 1 < s.n ? v[k] : 0.0);   // lags t >= n: 0
  }
  put(3 + T, g == 0 && s.n >= 2 ? a_last : 0.0);  // lag n - 1 (the ESS loop's last), whatever T
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

int64_t rows_chunks(int64_t rows) { return (rows + kRowChunk - 1) / kRowChunk; }

// Blocks resident per CU for the lag kernel of T lags (LDS ring and VGPRs; see the launch switch).
#ifdef HMC_CONV48_BPC3   // A/B: 48-lag grid sized for 3 blocks per CU
constexpr int conv_blocks_per_cu(int T) { return T == 16 ? 1 : T == 32 ? 2 : 3; }
#else
constexpr int conv_blocks_per_cu(int T) { return T == 16 ? 1 : T == 32 ? 2 : T == 48 ? 4 : 3; }
#endif

// Block groups of the lag pass: one resident wave of blocks over all dim tiles (no tail wave).
int64_t conv_groups(int64_t n_chains, int D, int T) {
  const int64_t g = (2 * n_chains + 3) / 4;       // 4 split chains per block row set
  const int ntiles = (D + kDimTile - 1) / kDimTile;
  int64_t cap = (int64_t)256 * conv_blocks_per_cu(T) / ntiles;
  cap = cap >= 8 ? cap / 8 * 8 : 8;
  return g < cap ? (g < 1 ? 1 : g) : cap;
}

int64_t vario_jchunk(int64_t m2) {
  // ~4096 blocks at most; at least 16 split chains per block
  int64_t c = (m2 + 4095) / 4096;
  return c < 16 ? 16 : c;
}

}  // namespace

int64_t diag_rowsum_work(int64_t rows, int D) { return rows_chunks(rows) * D; }

int64_t diag_variogram_work(int64_t n_chains, int D, int nlags) {
  const int64_t m2 = 2 * n_chains;
  const int64_t jc = vario_jchunk(m2);
  return ((m2 + jc - 1) / jc) * (int64_t)nlags * D;
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

int64_t diag_conv_work(int64_t n_chains, int D, int T) { return conv_groups(n_chains, D, T) * (int64_t)(T + 4) * D; }

hipError_t launch_conv_fused(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int64_t base, int n, int D,
                             int T, double* work, double* out, hipStream_t st) {
  Src s{x, cs, ss, base, n_chains, n, D};
  const int64_t groups = conv_groups(n_chains, D, T);
  const int ntiles = (D + kDimTile - 1) / kDimTile;
  // blocks: 8 groups x ntiles per 8 * ntiles consecutive block ids (XCD-aware order, see kernel)
  const int64_t gpad = (groups + 7) / 8 * 8;
  const dim3 grid((unsigned)(gpad * ntiles));
  // the direct-to-LDS loads move dim pairs of 16 B: rows must start 16-B aligned and hold whole pairs
  if (((D | cs | ss | base) & 1) || (reinterpret_cast<uintptr_t>(x) & 15)) {
    switch (T) {
      case 8: k_conv_lags<8, 1><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
      case 16: k_conv_lags<16, 1><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
      case 32: k_conv_lags<16, 2><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
      case 48: k_conv_lags<16, 3><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
      case 64: k_conv_lags<16, 4><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
      default: return hipErrorInvalidValue;
    }
  } else switch (T) {   // T = TW x G lags; rows staged through LDS by direct-to-LDS loads, 2 chunks ahead
    case 8: k_conv_lds<8, 1, 2><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
    case 16: k_conv_lds<16, 1, 2><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
    case 32: k_conv_lds<16, 2, 2><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
    case 48: k_conv_lds<16, 3, 2><<<grid, 192, 0, st>>>(s, (int)groups, ntiles, work); break;
    case 64: k_conv_lds<16, 4, 2><<<grid, 256, 0, st>>>(s, (int)groups, ntiles, work); break;
    default: return hipErrorInvalidValue;
  }
  if (hipError_t e = hipGetLastError()) return e;
  const int64_t ncols = (int64_t)(T + 4) * D;
  k_colsum_final<<<(unsigned)((ncols + 255) / 256), 256, 0, st>>>(work, groups, ncols, out);
  return hipGetLastError();
}

int64_t diag_stream_groups(int64_t n_chains) {
  const int64_t g = (n_chains + 3) / 4;
  return g < 1024 ? (g < 1 ? 1 : g) : 1024;
}

hipError_t launch_stream_accum(const double* x, int64_t n_chains, int64_t cs, int64_t ss, int D, int wrap, int slot0,
                               int carry, int rows, int64_t pos0, int n, double* shift, double* s1, double* s2, int T,
                               double* vpart, double* vsum, hipStream_t st) {
  const int64_t groups = diag_stream_groups(n_chains);
  StreamArgs a{x, n_chains, cs, ss, D, wrap, slot0, carry, rows, n, pos0, shift, s1, s2, vpart, (int)groups};
  dim3 grid((unsigned)groups, (unsigned)((D + kDimTile - 1) / kDimTile));
  // the product form needs every half to reach position T-1 (its H_t event); both forms give the
  // same sums of every completed half, and a run keeps one form (n and T are fixed per run)
  const bool prod = n >= T;
  auto go = [&](auto t_c) {
    constexpr int TT = decltype(t_c)::value;
    if (prod) k_stream_accum<TT, true><<<grid, 256, 0, st>>>(a);
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
  const int64_t m2 = 2 * n_chains;
  const int64_t jc = vario_jchunk(m2);
  const int64_t nch = (m2 + jc - 1) / jc;
  dim3 grid((unsigned)nch, (unsigned)((D + kDimTile - 1) / kDimTile));
  // lags in blocks of <= 32 per pass; work holds [nch][t1 - t0][D] partials
  for (int a = t0; a < t1; a += 32) {
    const int nt = t1 - a < 32 ? t1 - a : 32;
    double* part = work + (int64_t)nch * (a - t0) * D;
    if (nt <= 8) k_variogram_ring<8><<<grid, 256, 0, st>>>(s, a, nt, jc, part);
    else if (nt <= 16) k_variogram_ring<16><<<grid, 256, 0, st>>>(s, a, nt, jc, part);
    else k_variogram_ring<32><<<grid, 256, 0, st>>>(s, a, nt, jc, part);
    if (hipError_t e = hipGetLastError()) return e;
    const int64_t ncols = (int64_t)nt * D;
    k_colsum_final<<<(unsigned)((ncols + 255) / 256), 256, 0, st>>>(part, nch, ncols, out + (int64_t)(a - t0) * D);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

}  // namespace hmc
