// hmc_nuts_lock.hip — the reference's NUTS engine (samplers.py:495-808, utils.py:222-385) for dense
// targets with 128 < D <= kLockDmax, 16 chains per block in lockstep so that one f64-MFMA GEMM per
// block step gives all 16 chains their gradient (hmc_nuts_big.hip re-read the D x D precision from
// L2 once per chain and leapfrog).
//
// Block = 16 waves, one chain slot per wave.  A wave runs its chain's tree as a state machine that
// advances one leapfrog per block step (or, at an iteration start, computes the gradient at the
// start point), with the chain's current point (q, p, g) in registers (lane l owns coordinates
// d = l + 64 j) and every other tree vector (both ends, the two live points, the d_max + 1 save
// slots) in the slot's workspace, lane-owned as in hmc_nuts_big.hip (a lane reads back only what it
// wrote: no fences inside a tree).  Each block step:
//   1. every wave half-kicks and drifts its point and writes x = q - q0 into the LDS tile X[d][chain];
//   2. barrier; the 16 waves split the GEMM G = P X (NT x KS f64 16x16x4 MFMAs over the precision's
//      fragments, prepared once per launch in the workspace, lane-linear: coalesced L2 reads) into
//      contiguous fragment ranges and write their partial output tiles into LDS;
//   3. barrier; each wave sums its chain's gradient rows from the partial tiles (fixed order) and
//      finishes the step: second half kick, energy, the new point's bookkeeping (saves at slot
//      ctz(l - 1), U-turn checks against check_points, progressive sampling), the sub-tree end
//      (biased acceptance, termination).
// A full cov_p (MASS, samplers.py:352-356, :811-839; round 6) adds block GEMMs on the same fragment
// machinery, as the reference writes the products: the kick kv = inv_cov_p (P x) (a second GEMM on
// the 16 gradients), K = p.inv_cov_p.p (a GEMM on the 16 momenta after the second half kick) and,
// when a chain of the block starts an iteration in Philox mode, p = C z (C = chol(cov_p)); the tree
// ends then keep kv in their g slot (a doubling restarted from an end kicks with it).
// Chains come from a launch-wide queue; a slot runs all of a chain's iterations of the launch, then
// writes the chain back and takes the next one, so no chain changes slots inside a launch.
// Draws are the ones hmc_nuts_big.hip makes (replay tape / Philox keyed (slot, iteration, chain)),
// in the reference's order, so results equal the per-chain kernel's up to the gradient's summation
// order.
#include <algorithm>

#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {

namespace {

constexpr int kLockW = 16;        // chain slots (waves) per block
constexpr int kLockJ = 5;         // coordinates per lane: D <= 64 * kLockJ
constexpr int kLockDmax = 64 * kLockJ;
constexpr int kLockXS = 17;       // LDS row stride (doubles) of X[k][chain] and the partial tiles
constexpr int kLockSegMax = 40;   // partial output tiles per block step (<= NT + 15)
constexpr int kLockPF = 4;        // precision fragments in flight per wave

// slot vectors: left end (q, p, g), right end (q, p, g), live points, then save slot s: q, p
enum : int { LV_LEFT = 0, LV_RIGHT = 3, LV_LIVE = 6, LV_SAVE = 8 };
__host__ __device__ inline int lock_nvec(int d_max) { return LV_SAVE + 2 * (d_max + 1); }

enum : int { LS_FETCH = 0, LS_GRAD = 1, LS_LEAP = 2, LS_DONE = 3 };

struct LockGeom {
  int NT, KS, F;                  // output tiles (16 rows), k-steps (4), fragments NT * KS
  const double* pf;               // precision fragments [F][64]
  const double* mf;               // MASS: inv_cov_p fragments [F][64]
  const double* cf;               // MASS, Philox: chol(cov_p) fragments [F][64]
  double* slots;                  // per slot: lock_nvec vectors of 64 * kLockJ doubles
  unsigned long long* queue;      // next chain of the launch (zeroed per launch)
  int64_t* tcur;                  // per chain replay-tape cursor (persists across launches)
};

// fragment f = nt * KS + ks of the precision, lane l: P[16 nt + (l & 15)][4 ks + (l >> 4)] (zero
// padded): the A operand of v_mfma_f64_16x16x4f64, one coalesced 512-B row per fragment
// (trans: the matrix is passed transposed, as hmc_kinetic.p_chol_t = C^T)
__global__ __launch_bounds__(256) void k_lock_pfrag(const double* __restrict__ prec, int D, int KS, int64_t F,
                                                    double* __restrict__ pf, int trans) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < F * 64; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = i >> 6;
    const int l = (int)(i & 63);
    const int nt = (int)(f / KS), ks = (int)(f - (int64_t)nt * KS);
    const int row = 16 * nt + (l & 15), col = 4 * ks + (l >> 4);
    pf[i] = (row < D && col < D) ? prec[trans ? (int64_t)col * D + row : (int64_t)row * D + col] : 0.0;
  }
}

__device__ __forceinline__ int lock_f0(int w, int F) { return (int)(((int64_t)w * F) / kLockW); }

typedef unsigned u32x2l __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int save_slot_l(int l, int d_max) { return l == 1 ? d_max : __builtin_ctz(l - 1); }

// J: coordinates per lane (D <= 64 J): instances J = 3 (D <= 192) and kLockJ, so that the
// per-chain work of a smaller D issues no fully masked slots (and holds fewer registers)
template <bool EXACT, bool REPLAY, int J, bool MASS>
__global__ __launch_bounds__(64 * kLockW) void k_nuts_lock(RandArgs a, LockGeom G) {
  __shared__ double sX[kLockDmax * kLockXS];                 // x of the 16 chains, [k][chain]
  __shared__ double sSeg[kLockSegMax * 16 * kLockXS];        // partial output tiles, [row][chain]
  __shared__ double tab[REPLAY ? 2 : kNormalTableDoubles];   // Box-Muller tables (Philox momenta)
  __shared__ int sAlive[kLockW];
  __shared__ int sGrad[kLockW];                              // MASS: slots at an iteration start
  if constexpr (!REPLAY) init_normal_tables(tab);
  const int lane = threadIdx.x & (kWave - 1);
  const int w = uniform_i(threadIdx.x / kWave);
  const int D = a.D, d_max = a.d_max;
  const int KS = G.KS, F = G.F;
  const int Dp = 64 * J;
  // every per-lane access goes through a buffer descriptor (scalar base) with the lane offset
  // lane * 8 and a constant 512 j: no 64-bit address per (array, j) kept live (the 128-register
  // budget of 16 waves per block spilled them)
  double* const ws = G.slots + ((int64_t)blockIdx.x * kLockW + w) * (int64_t)lock_nvec(d_max) * Dp;
  const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc(ws, 0, lock_nvec(d_max) * Dp * 8, 0x00020000);
  const int lo8 = lane * 8;
  const __amdgpu_buffer_rsrc_t rpf = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(G.pf), 0, G.F * 512,
                                                                      0x00020000);
  const __amdgpu_buffer_rsrc_t rmf = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(MASS ? G.mf : G.pf), 0,
                                                                      G.F * 512, 0x00020000);
  const __amdgpu_buffer_rsrc_t rcf = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>((MASS && G.cf) ? G.cf : G.pf),
                                                                      0, G.F * 512, 0x00020000);
  auto wget = [&](int id, int j) -> double {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rws, lo8 + 512 * j, id * Dp * 8, 0));
  };
  auto wput = [&](int id, int j, double x) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2l, x), rws, lo8 + 512 * j, id * Dp * 8, 0);
  };
  // per-dimension constants (zero past D: out of the descriptor's range)
  auto mk = [&](const double* arr) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(arr), 0, D * 8, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rq0 = mk(a.q0), rmi = mk(a.minv), rdt = mk(a.dtv), rps = mk(a.pscale);
  auto dget = [&](__amdgpu_buffer_rsrc_t r, int j) -> double {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lo8 + 512 * j, 0, 0));
  };
  // this wave's share of the GEMM: fragments [f0, f1); its first partial tile's index
  const int f0 = lock_f0(w, F), f1 = lock_f0(w + 1, F);
  int seg0 = 0;
  for (int v = 0; v < w; ++v) {
    const int a0 = lock_f0(v, F), a1 = lock_f0(v + 1, F);
    if (a1 > a0) seg0 += (a1 - 1) / KS - a0 / KS + 1;
  }
  // the partial tiles holding this lane's gradient rows d = lane + 64 j: the tile's first segment
  // (segments of one tile are consecutive) and their count
  int gseg[J], gcnt[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int d = lane + 64 * j;
    const int nt = d < D ? d / 16 : 0;
    int first = -1, cnt = 0, sb = 0;
    for (int v = 0; v < kLockW; ++v) {
      const int a0 = lock_f0(v, F), a1 = lock_f0(v + 1, F);
      if (a1 > a0) {
        const int t0 = a0 / KS, t1 = (a1 - 1) / KS;
        if (nt >= t0 && nt <= t1) {
          if (first < 0) first = sb + (nt - t0);
          ++cnt;
        }
        sb += t1 - t0 + 1;
      }
    }
    gseg[j] = first;
    gcnt[j] = d < D ? cnt : 0;
  }
  __syncthreads();                                          // tables

  auto dq0 = [&](int j) { return a.q0 ? dget(rq0, j) : 0.0; };
  auto dminv = [&](int j) { return a.minv ? dget(rmi, j) : 1.0; };
  auto ddt = [&](int j) { return a.dtv ? dget(rdt, j) : a.dt; };
  auto dps = [&](int j) { return a.pscale ? dget(rps, j) : 1.0; };
  auto wsum = [&](double s) { return wave_sum_dpp(s); };

  // g = P x; MASS: kv = inv_cov_p g (the kick), and the tree ends keep kv in their g slot
  // (MASS: the gradient and inv_cov_p p are step-local -- their energy terms are summed as they are
  // gathered -- so only kv is carried between steps: 20 VGPRs fewer at J = 5)
  double q[J], p[J], g[MASS ? 1 : J], kv[MASS ? J : 1];
  double maha_l = 0.0, kin_l = 0.0;                 // MASS: this step's energy partials (lane, d order)
#pragma unroll
  for (int j = 0; j < J; ++j) q[j] = p[j] = 0.0;
#pragma unroll
  for (int j = 0; j < (MASS ? 1 : J); ++j) g[j] = 0.0;
#pragma unroll
  for (int j = 0; j < (MASS ? J : 1); ++j) kv[j] = 0.0;
  int state = LS_FETCH;
  int64_t c = 0;
  uint64_t gc = 0;
  int it = 0;
  int64_t tpos = 0;
  uint32_t ndraw = 0;
  double Eprev = 0.0, E_init = 0.0, E_max_now = 0.0, E_max_old = 0.0, pi_new = 1.0, pi_old = 1.0;
  int d = 0, k = 0, Lsub = 1, udir = 0, lo = LV_LIVE;       // lo: the live_old vector (the other is new)
  unsigned long long n_lf = 0, n_unst = 0, n_dmax = 0, n_tape = 0, n_steps = 0;

  auto draw = [&](bool direction) -> double {               // next tree draw of this chain (reference order)
    if constexpr (REPLAY) {
      if (tpos >= a.tape_stride) {                          // exhausted tape: flagged, the host raises
        ++n_tape;
        return direction ? 0.0 : 2.0;
      }
      return a.tape[c * a.tape_stride + (tpos++)];
    } else {
      const uint4 r = draw_block(kDrawSlot + (ndraw++), (uint32_t)it, gc, a.k0, a.k1);
      return direction ? (double)(r.x & 1u) : u53(r.z, r.w);
    }
  };
  auto write_row_of = [&](int i) { return i >= a.wu && ((i == a.niter) || ((i - a.wu + 1) % a.thin == 0)); };
  auto vstore = [&](int id, const double (&x)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) wput(id, j, x[j]);
  };
  auto vload = [&](int id, double (&x)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) x[j] = wget(id, j);
  };
  // sum over d of (r - l) . v (samplers.py:720-722 / :779-781), lanes' partial sums in d order
  auto span_dot = [&](const double (&r)[J], const double (&l)[J], const double (&v)[J]) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < J; ++j) s += (r[j] - l[j]) * v[j];
    return wsum(s);
  };
  // E = V + K = 0.5 (logc + (q - q0).g + p.(minv p))  (samplers.py:811-823)
  auto energy = [&]() {
    if constexpr (MASS) return 0.5 * (a.logc + (wsum(maha_l) + wsum(kin_l)));   // p . (inv_cov_p p)
    double maha = 0.0, kin = 0.0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int dd = lane + 64 * j;
      if (dd < D) {
        maha += (q[j] - dq0(j)) * g[j];
        kin += p[j] * (dminv(j) * p[j]);
      }
    }
    return 0.5 * (a.logc + (wsum(maha) + wsum(kin)));
  };
  // the "g" slot of a tree end: the kick vector (MASS) or the gradient
  auto gslot = [&]() -> double (&)[J] {
    if constexpr (MASS) return kv;
    else return g;
  };

  while (true) {
    // ================= chain fetch (a slot runs all of a chain's iterations of the launch)
    if (state == LS_FETCH) {
      unsigned long long u = 0;
      if (lane == 0) u = atomicAdd(G.queue, 1ull);
      u = __builtin_amdgcn_readfirstlane((unsigned)u);
      if ((int64_t)u < a.n && a.it0 < a.it1) {
        c = (int64_t)u;
        gc = (uint64_t)(a.chain_offset + c);
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          q[j] = dd < D ? a.q[c * D + dd] : 0.0;
        }
        Eprev = a.Eprev[c];
        tpos = REPLAY ? G.tcur[c] : 0;
        it = a.it0;
        state = LS_GRAD;                                    // gradient at the start point
      } else {
        state = LS_DONE;
      }
    }
    // ================= pre-gradient: half kick + drift (:831-835), x = q - q0 into the block tile
    if (state == LS_LEAP) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int dd = lane + 64 * j;
        if (dd < D) {
          const double dt = ddt(j);
          if constexpr (MASS) {                               // kick by inv_cov_p dVdq (Q3)
            p[j] = EXACT ? p[j] - (dt * kv[j]) * 0.5 : __builtin_fma(-0.5 * dt, kv[j], p[j]);
          } else {
            const double mi = dminv(j);
            p[j] = EXACT ? p[j] - (dt * (mi * g[j])) * 0.5 : __builtin_fma(-0.5 * dt * mi, g[j], p[j]);
          }
          q[j] = EXACT ? q[j] + dt * p[j] : __builtin_fma(dt, p[j], q[j]);
        }
      }
    }
    const bool busy = state == LS_LEAP || state == LS_GRAD;
    if (busy) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int dd = lane + 64 * j;
        if (dd < 4 * KS) sX[dd * kLockXS + w] = dd < D ? q[j] - dq0(j) : 0.0;
      }
    }
    if (lane == 0) {
      sAlive[w] = state != LS_DONE;
      if constexpr (MASS) sGrad[w] = state == LS_GRAD;
    }
    __syncthreads();
    int alive = 0, any_grad = 0;
#pragma unroll
    for (int v = 0; v < kLockW; ++v) {
      alive |= sAlive[v];
      if constexpr (MASS) any_grad |= sGrad[v];
    }
    if (!alive) break;                                      // (uniform over the block)
    if (w == 0) ++n_steps;

    // ================= the block's GEMM: fragments [f0, f1) of M X (M = P, or with MASS inv_cov_p /
    // C), partial tiles to LDS.  Scalar k-step counter and a running LDS address (no division per
    // MFMA); A fragments through a buffer descriptor with the fragment's offset in the scalar offset.
    auto gemm = [&](const __amdgpu_buffer_rsrc_t& rm) {
      typedef double d4 __attribute__((ext_vector_type(4)));
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      const int ch = lane & 15, kh = lane >> 4;
      int seg = seg0;
      int ks = f0 - (f0 / KS) * KS;
      const int xb = kh * kLockXS + ch;
      int xa = xb + ks * 4 * kLockXS;
      auto flush = [&]() {
        double* t = sSeg + seg * (16 * kLockXS);
#pragma unroll
        for (int v = 0; v < 4; ++v) t[(4 * v + kh) * kLockXS + ch] = acc[v];
      };
      auto frag = [&](int f) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rm, lo8 + f * 512, 0, 0));
      };
      // four fragments in flight in a static register ring (unrolled by four). Every load is issued
      // on every path (past f1: a fragment the wave does not use, or zeros past the buffer), and the
      // ring is complete at the loop entry (the loop header then merges "nothing outstanding" with
      // the back edge's four in order), so the waitcnt pass keeps three loads outstanding at each
      // MFMA; a conditional load, a register rotation or a partly loaded ring at the entry made it
      // drain them all before the MFMAs
      double af[kLockPF];
#pragma unroll
      for (int i = 0; i < kLockPF; ++i) af[i] = frag(f0 + i);
#pragma unroll
      for (int i = 0; i < kLockPF; ++i) asm volatile("" ::"v"(af[i]));   // in hand at the loop entry, so
      double xc = sX[xa];                                   // B of the current fragment, read one ahead
      for (int fb = f0; fb < f1; fb += kLockPF) {
#pragma unroll
        for (int i = 0; i < kLockPF; ++i) {
          const int f = fb + i;
          const bool in = f < f1;
          const bool last_k = ks + 1 == KS;
          const int xan = last_k ? xb : xa + 4 * kLockXS;
          const double xn = sX[xan];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(in ? af[i] : 0.0, xc, acc, 0, 0, 0);
          af[i] = frag(f + kLockPF);
          if (in) {
            if (last_k) {
              flush();
              acc = d4{0.0, 0.0, 0.0, 0.0};
              ++seg;
              ks = 0;
            } else {
              ++ks;
            }
          }
          xa = xan;
          xc = xn;
        }
      }
      if (ks != 0) flush();                                 // a tile the range ends inside
    };
    // this chain's rows of the product, segments in order
    auto gather = [&](double (&y)[J]) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int dd = lane + 64 * j;
        double sacc = 0.0;
        for (int t = 0; t < gcnt[j]; ++t) sacc += sSeg[(gseg[j] + t) * (16 * kLockXS) + (dd & 15) * kLockXS + w];
        y[j] = sacc;
      }
    };
    // one more block product: this wave's column x (zero past D) into the tile, the GEMM, its rows
    auto product = [&](const __amdgpu_buffer_rsrc_t& rm, const double (&x)[J], double (&y)[J], bool put, bool get) {
      if (put) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          if (dd < 4 * KS) sX[dd * kLockXS + w] = dd < D ? x[j] : 0.0;
        }
      }
      __syncthreads();                                      // columns written, the last gather done
      gemm(rm);
      __syncthreads();
      if (get) gather(y);
    };
    gemm(rpf);
    __syncthreads();
    if constexpr (!MASS) {
      if (busy) gather(g);                                  // g = P (q - q0)
    }
    if constexpr (MASS) {
      double gl[J];                                         // g = P (q - q0), this step only
      maha_l = 0.0;
      kin_l = 0.0;
      if (busy) {
        gather(gl);
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          if (dd < D) maha_l += (q[j] - dq0(j)) * gl[j];
        }
      }
      product(rmf, gl, kv, busy, busy);                     // the kick inv_cov_p dVdq (:835-837)
      if (state == LS_GRAD) {                               // iteration start: p ~ N(0, cov_p) (:565, :829)
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          double pd = 0.0;
          if (dd < D) {
            if constexpr (REPLAY) {
              pd = a.rp[(c * (int64_t)a.niter + (it - 1)) * D + dd];
            } else {                                      // z, then p = C z below
              const int h = dd & 3, jj = dd >> 3;
              double z0, z1;
              normal_pair_tab(draw_block((uint32_t)(8 * jj + h), (uint32_t)it, gc, a.k0, a.k1), tab, z0, z1);
              pd = (dd >> 2) & 1 ? z1 : z0;
            }
          }
          p[j] = pd;
        }
      }
      if constexpr (!REPLAY) {
        if (any_grad) product(rcf, p, p, state == LS_GRAD, state == LS_GRAD);   // p = C z
      }
      if (state == LS_LEAP) {                               // second half kick (:837-839)
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          if (dd < D) {
            const double dt = ddt(j);
            p[j] = EXACT ? p[j] - (dt * kv[j]) * 0.5 : __builtin_fma(-0.5 * dt, kv[j], p[j]);
          }
        }
      }
      // inv_cov_p p for K (:823), summed against p as its rows are gathered
      if (busy) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          if (dd < 4 * KS) sX[dd * kLockXS + w] = dd < D ? p[j] : 0.0;
        }
      }
      __syncthreads();
      gemm(rmf);
      __syncthreads();
      if (busy) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int dd = lane + 64 * j;
          double sacc = 0.0;
          for (int t = 0; t < gcnt[j]; ++t) sacc += sSeg[(gseg[j] + t) * (16 * kLockXS) + (dd & 15) * kLockXS + w];
          if (dd < D) kin_l += p[j] * sacc;
        }
      }
    }

    // ================= post-gradient
    if (state == LS_GRAD) {                                 // iteration start (:563-584)
#pragma unroll
      for (int j = 0; j < J; ++j) {
        if constexpr (MASS) break;                          // p drawn above (C z / the replay draw)
        const int dd = lane + 64 * j;
        double pd = 0.0;
        if (dd < D) {
          if constexpr (REPLAY) {
            pd = a.rp[(c * (int64_t)a.niter + (it - 1)) * D + dd];
          } else {
            const int h = dd & 3, jj = dd >> 3;
            double z0, z1;
            normal_pair_tab(draw_block((uint32_t)(8 * jj + h), (uint32_t)it, gc, a.k0, a.k1), tab, z0, z1);
            pd = ((dd >> 2) & 1 ? z1 : z0) * dps(j);
          }
        }
        p[j] = pd;
      }
      E_init = energy();                                    // :569
      if (write_row_of(it) && lane == 0) {                  // :571-573
        const int64_t row = c * (int64_t)a.Lc + (it - a.wu) / a.thin;
        if (a.Ec) a.Ec[row] = E_init;
        if (a.dEc) a.dEc[row] = E_init - Eprev;
      }
      double mp[J];
#pragma unroll
      for (int j = 0; j < J; ++j) mp[j] = -p[j];
      vstore(LV_RIGHT, q);                                  // right = (q, p, g), left = (q, -p, g)
      vstore(LV_RIGHT + 1, p);
      vstore(LV_RIGHT + 2, gslot());
      vstore(LV_LEFT, q);
      vstore(LV_LEFT + 1, mp);
      vstore(LV_LEFT + 2, gslot());
      lo = LV_LIVE;
      vstore(lo, q);                                        // live_point_q_old (:577)
      E_max_old = E_init;
      pi_old = 1.0;
      d = 0;
      ndraw = 0;
      udir = (int)draw(true);                               // :608 (first doubling)
      if (udir != 0) {
#pragma unroll
        for (int j = 0; j < J; ++j) p[j] = -p[j];           // start from the left end (q, -p, g)
      }
      Lsub = 1;
      k = 0;
      state = LS_LEAP;
      continue;
    }
    if (state != LS_LEAP) continue;
    if constexpr (!MASS) {                                  // second half kick (:837-839; MASS: above)
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int dd = lane + 64 * j;
        if (dd < D) {
          const double dt = ddt(j), mi = dminv(j);
          p[j] = EXACT ? p[j] - (dt * (mi * g[j])) * 0.5 : __builtin_fma(-0.5 * dt * mi, g[j], p[j]);
        }
      }
    }
    ++n_lf;
    const double E_tmp = energy();                          // :618 / :643
    bool reject = false, sub_end = false;
    const int m = k + 1;                                    // point number within the sub-tree
    if (k == 0) {                                           // first point (:617-626)
      vstore(LV_LIVE + LV_LIVE + 1 - lo, q);                // live_point_new
      E_max_now = E_tmp;
      pi_new = 1.0;
      vstore(LV_SAVE + 2 * save_slot_l(1, d_max), q);
      vstore(LV_SAVE + 2 * save_slot_l(1, d_max) + 1, p);
      k = 1;
      sub_end = Lsub == 1;
    } else {
      if (fabs(E_tmp - E_init) > 1000.0) {                  // :647-651
        reject = true;
        ++n_unst;
      } else if (m & 1) {                                   // odd point: save (:654-658)
        const int s = save_slot_l(m, d_max);
        vstore(LV_SAVE + 2 * s, q);
        vstore(LV_SAVE + 2 * s + 1, p);
      } else {                                              // even point: U-turn checks (:699-736)
        int r = m;
        while ((r & (r - 1)) != 0 && r > 2) r -= 1 << (31 - __builtin_clz(r));
        int pt = m - r + 1, half = r;
        while (true) {
          const int s = save_slot_l(pt, d_max);
          double qc[J], pc[J];
          vload(LV_SAVE + 2 * s, qc);
          vload(LV_SAVE + 2 * s + 1, pc);
          double rdot, ldot;
          if (udir == 0) {                                  // left = (q_chk, -p_chk), right = current
            rdot = span_dot(q, qc, p);
            ldot = span_dot(q, qc, pc);
          } else {                                          // left = current, right = (q_chk, -p_chk)
            rdot = -span_dot(qc, q, pc);
            ldot = -span_dot(qc, q, p);
          }
          if (ldot < 0.0 && rdot < 0.0) {                   // :727-732
            reject = true;
            break;
          }
          if (half <= 2) break;
          half >>= 1;
          pt += half;
        }
      }
      if (!reject) {                                        // progressive sampling (:743-751)
        const double E_max_prev = E_max_now;
        E_max_now = fmax(E_max_prev, E_tmp);
        const double num = exp(-(E_tmp - E_max_now));
        pi_new = num + exp(E_max_now - E_max_prev) * pi_new;
        const double r_ = num / pi_new;
        if (draw(false) < r_) vstore(LV_LIVE + LV_LIVE + 1 - lo, q);
        ++k;
        sub_end = k == Lsub;
      }
    }
    bool iter_end = reject;                                 // q = live_point_q_old (:649, :731)
    if (sub_end) {                                          // sub-tree end (:757-784)
      const int b = udir == 0 ? LV_RIGHT : LV_LEFT;         // this end <- (q, p, g)
      const int o = udir == 0 ? LV_LEFT : LV_RIGHT;
      double oq[J], op[J];
      vload(o, oq);
      vload(o + 1, op);
      vstore(b, q);
      vstore(b + 1, p);
      vstore(b + 2, gslot());
      const double r_ = exp(-(E_max_now - E_max_old)) * pi_old / pi_new;   // :766 (Q11)
      const double E_max_old_prev = E_max_old;
      E_max_old = fmax(E_max_old_prev, E_max_now);
      pi_old = exp(-(E_max_now - E_max_old)) * pi_new + exp(-(E_max_old_prev - E_max_old)) * pi_old;   // :771
      const double A = fmin(1.0, r_);
      if (draw(false) < A) lo = LV_LIVE + LV_LIVE + 1 - lo; // :773-775 (names swap)
      bool rterm, lterm;                                    // :779-784 (Q10: both ends)
      if (udir == 0) {                                      // right = current
        rterm = span_dot(q, oq, p) < 0.0;
        lterm = -span_dot(q, oq, op) < 0.0;
      } else {                                              // left = current
        rterm = span_dot(oq, q, op) < 0.0;
        lterm = -span_dot(oq, q, p) < 0.0;
      }
      ++d;
      if (lterm && rterm) {
        iter_end = true;
      } else if (d > d_max - 1) {                           // :596-598 (the reference aborts)
        ++n_dmax;
        iter_end = true;
      } else {
        Lsub = 1 << d;
        const int nd = (int)draw(true);                     // :608, next doubling
        if (nd != udir) {                                   // from the other end
#pragma unroll
          for (int j = 0; j < J; ++j) {
            q[j] = oq[j];
            p[j] = op[j];
          }
          vload(o + 2, gslot());
          udir = nd;
        }
        k = 0;
      }
    }
    if (iter_end) {                                         // iteration end (:786-791)
      vload(lo, q);
      Eprev = E_init;
      const int qrow = (it - a.wu) / a.thin;
      if (write_row_of(it) && a.qc && qrow >= a.q_row0) {
        double* rowp = a.qc + (c * (int64_t)a.Lq + qrow % a.Lq) * D;
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (lane + 64 * j < D) rowp[lane + 64 * j] = q[j];
      }
      ++it;
      if (it < a.it1) {
        state = LS_GRAD;
      } else {                                              // the chain's launch is done: write it back
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (lane + 64 * j < D) a.q[c * D + lane + 64 * j] = q[j];
        if (lane == 0) {
          a.Eprev[c] = Eprev;
          if (REPLAY) G.tcur[c] = tpos;
        }
        state = LS_FETCH;
      }
    }
  }
  if (lane == 0 && a.cnt) {
    unsigned long long* cs = a.cnt + (((int64_t)blockIdx.x * kLockW + w) & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
    if (n_lf) {
      atomicAdd(cs + HMC_CNT_LEAPFROG, n_lf);
      atomicAdd(cs + HMC_CNT_ENERGY_EVALS, n_lf);
    }
    if (n_steps) atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, n_steps);   // NUTS: block steps (16 chain slots each)
    if (n_unst) atomicAdd(cs + HMC_CNT_UNSTABLE, n_unst);
    if (n_dmax) atomicAdd(cs + HMC_CNT_DMAX, n_dmax);
    if (n_tape) atomicAdd(cs + HMC_CNT_OOB_REJECT, n_tape);
  }
}

// blocks of a launch: two chains per slot on average (small runs exercise the queue), at most one
// block per CU (the LDS tiles)
int64_t lock_blocks(int64_t n) {
  const int64_t b = (n + 2 * kLockW - 1) / (2 * kLockW);
  const int64_t cap = device_cus();
  return b < cap ? (b < 1 ? 1 : b) : cap;
}

}  // namespace

bool nuts_lock_path(int D) { return D > 128 && D <= kLockDmax; }

// workspace: slot vectors (blocks x 16 slots), precision fragments, queue word, tape cursors
// (mass: the inv_cov_p and chol(cov_p) fragments too)
int64_t nuts_lock_ws_doubles(int64_t n, int D, int d_max, bool mass) {
  const int NT = (D + 15) / 16, KS = (D + 3) / 4;
  const int64_t blocks = (n + kLockW - 1) / kLockW < 1024 ? (n + kLockW - 1) / kLockW : 1024;
  return (blocks < 1 ? 1 : blocks) * kLockW * (int64_t)lock_nvec(d_max) * 64 * kLockJ +
         (int64_t)NT * KS * 64 * (mass ? 3 : 1) + 2 + n;
}

hipError_t launch_nuts_lock(const RandArgs& a, bool exact, bool replay, hipStream_t s) {
  LockGeom g{};
  g.NT = (a.D + 15) / 16;
  g.KS = (a.D + 3) / 4;
  g.F = g.NT * g.KS;
  int64_t blocks = lock_blocks(a.n);
  const int64_t cap = (a.n + kLockW - 1) / kLockW < 1024 ? (a.n + kLockW - 1) / kLockW : 1024;
  if (blocks > cap) blocks = cap < 1 ? 1 : cap;             // (the workspace holds this many slots)
  const int64_t slot_doubles = (cap < 1 ? 1 : cap) * kLockW * (int64_t)lock_nvec(a.d_max) * 64 * kLockJ;
  g.slots = a.ws;
  double* pf = a.ws + slot_doubles;
  g.pf = pf;
  const bool mass = a.minvf != nullptr;
  double* const after = pf + (int64_t)g.F * 64 * (mass ? 3 : 1);
  g.mf = mass ? pf + (int64_t)g.F * 64 : nullptr;
  g.cf = (mass && !replay) ? pf + 2 * (int64_t)g.F * 64 : nullptr;
  g.queue = reinterpret_cast<unsigned long long*>(after);
  g.tcur = reinterpret_cast<int64_t*>(after + 2);
  // the partial tiles of one block step: NT plus one per wave boundary inside a tile
  if (g.NT + kLockW - 1 > kLockSegMax || a.D > kLockDmax) return hipErrorInvalidValue;
  if (hipError_t e = hipMemsetAsync(g.queue, 0, sizeof(unsigned long long), s)) return e;
  const unsigned fgrid = (unsigned)std::min<int64_t>(((int64_t)g.F * 64 + 255) / 256, 4096);
  k_lock_pfrag<<<fgrid, 256, 0, s>>>(a.prec, a.D, g.KS, g.F, pf, 0);
  if (mass) {
    k_lock_pfrag<<<fgrid, 256, 0, s>>>(a.minvf, a.D, g.KS, g.F, const_cast<double*>(g.mf), 0);
    if (!replay) k_lock_pfrag<<<fgrid, 256, 0, s>>>(a.cholt, a.D, g.KS, g.F, const_cast<double*>(g.cf), 1);
  }
  if (hipError_t e = hipGetLastError()) return e;
  const dim3 grid((unsigned)blocks);
  auto go = [&](auto jc, auto mc) {
    constexpr int J = decltype(jc)::value;
    constexpr bool M = decltype(mc)::value;
    if (exact) {
      if (replay) k_nuts_lock<true, true, J, M><<<grid, 64 * kLockW, 0, s>>>(a, g);
      else k_nuts_lock<true, false, J, M><<<grid, 64 * kLockW, 0, s>>>(a, g);
    } else {
      if (replay) k_nuts_lock<false, true, J, M><<<grid, 64 * kLockW, 0, s>>>(a, g);
      else k_nuts_lock<false, false, J, M><<<grid, 64 * kLockW, 0, s>>>(a, g);
    }
  };
  if (mass) {
    if (a.D <= 64 * 3) go(std::integral_constant<int, 3>{}, std::true_type{});
    else go(std::integral_constant<int, kLockJ>{}, std::true_type{});
  } else {
    if (a.D <= 64 * 3) go(std::integral_constant<int, 3>{}, std::false_type{});
    else go(std::integral_constant<int, kLockJ>{}, std::false_type{});
  }
  return hipGetLastError();
}

}  // namespace hmc
