// hmc_nuts_big.hip — the reference's NUTS engine (samplers.py:495-808, utils.py:222-385) for
// dense-precision targets beyond the MFMA tree kernel's register budget (D > 128), where the
// reference's np.dot takes any D (samplers.py:835-837).
//
// One wave per chain runs the reference's per-chain loop as written (the chain loop :545 is the
// grid): every tree vector lives in the workspace, chain-contiguous, and lane l owns the
// coordinates d = l (mod 64) of every vector, so a lane only ever reads back what it wrote itself
// and no barrier or fence is needed between the steps of a tree.  The gradient P (q - q0) is a
// wave GEMV: lanes over output rows, P read as the symmetric P[k][row] (coalesced, L2-resident at
// these sizes), the 64 x values of a k-chunk broadcast by v_readlane.  Control flow (directions,
// U-turn checks, progressive sampling) is uniform per wave, so all reductions run converged.
// Vector names instead of copies: the current point, the left and the right end are three (q, p,
// g) triples whose roles rotate when a sub-tree ends (:758-761), and the two live points swap
// names when a sub-tree's point is accepted (:773-775).
//
// Draws: replay (momenta per iteration, a per-chain tape of directions / uniforms in consumption
// order) or Philox keyed (slot, iteration, global chain) exactly as hmc_nuts.hip: momentum pair
// slot 8j + h (h < 4) holds dims (8j + h, 8j + h + 4) through the table Box-Muller, tree draw n of
// an iteration is block kDrawSlot + n (direction = bit 0 of x, uniform = u53(z, w)).
// This is a shape-range path (the c5 workload is D = 100, hmc_nuts.hip): per leapfrog it reads P
// once per chain from L2 (D^2 * 8 bytes) instead of sharing it across a 16-chain MFMA tile.
// 128 < D <= 320 with a diagonal cov_p runs the lockstep kernel (hmc_nuts_lock.hip) instead.
//
// A full cov_p (MASS, samplers.py:352-356, :811-839) takes the reference's products as written:
// p = C z (Philox; replay momenta are the reference's own N(0, cov_p) draws), the kick
// inv_cov_p . (P x) as two GEMVs, K = p . (inv_cov_p p) with a third, and V from the P x product.
// The triples then hold the kick vector in their g slot; P x lives in a per-chain scratch vector.
#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {

namespace {

// per-chain vector ids: three (q, p, g) triples (current point, left end, right end), two live
// points (old / new, :577 / :617), the d_max + 1 save slots' q and p (:623-626, :654-658), then
// two scratch vectors of the full-cov_p products (P x of the newest point; inv_cov_p p or z)
constexpr int kTriples = 3, kLive0 = 3 * kTriples, kSave0 = kLive0 + 2;
__host__ __device__ constexpr int scratch0(int d_max) { return kSave0 + 2 * (d_max + 1); }

__device__ __forceinline__ double q0_of(const RandArgs& a, int d) { return a.q0 ? a.q0[d] : 0.0; }
__device__ __forceinline__ double minv_of(const RandArgs& a, int d) { return a.minv ? a.minv[d] : 1.0; }
__device__ __forceinline__ double dt_of(const RandArgs& a, int d) { return a.dtv ? a.dtv[d] : a.dt; }
__device__ __forceinline__ double ps_of(const RandArgs& a, int d) { return a.pscale ? a.pscale[d] : 1.0; }

struct ChainVecs {
  double* base;   // vector 0 of this chain
  int Dp;         // padded vector length (multiple of 64)
  __device__ double* v(int id) const { return base + (int64_t)id * Dp; }
};

// y = M (x - shift) for one chain, M row-major [D][D] read as M[k][row]: symmetric matrices
// (P, inv_cov_p) or a pre-transposed one (cholt = C^T gives C[row][k])
__device__ void wave_gemv(int D, const double* __restrict__ M, const double* __restrict__ x,
                          const double* __restrict__ shift, double* __restrict__ y, int lane) {
  for (int r0 = 0; r0 < D; r0 += kWave) {
    const int row = r0 + lane;
    const int rc = row < D ? row : D - 1;
    double acc = 0.0;
    for (int k0 = 0; k0 < D; k0 += kWave) {
      const int kk = k0 + lane;
      const double xv = kk < D ? x[kk] - (shift ? shift[kk] : 0.0) : 0.0;
      const int kn = min(kWave, D - k0);
      const double* pk = M + (int64_t)k0 * D + rc;
      int j = 0;
      for (; j + 4 <= kn; j += 4) {
        const double p0 = pk[(int64_t)j * D], p1 = pk[(int64_t)(j + 1) * D];
        const double p2 = pk[(int64_t)(j + 2) * D], p3 = pk[(int64_t)(j + 3) * D];
        acc = __builtin_fma(p0, readlane_d(xv, j), acc);
        acc = __builtin_fma(p1, readlane_d(xv, j + 1), acc);
        acc = __builtin_fma(p2, readlane_d(xv, j + 2), acc);
        acc = __builtin_fma(p3, readlane_d(xv, j + 3), acc);
      }
      for (; j < kn; ++j) acc = __builtin_fma(pk[(int64_t)j * D], readlane_d(xv, j), acc);
    }
    if (row < D) y[row] = acc;
  }
}

// the kick vector at q into g: P (q - q0) (samplers.py:835-837 dVdq), and with a full cov_p
// inv_cov_p . (P x) with P x kept in gs
template <bool MASS>
__device__ void wave_grad(const RandArgs& a, const double* __restrict__ q, double* __restrict__ g,
                          double* __restrict__ gs, int lane) {
  if constexpr (MASS) {
    wave_gemv(a.D, a.prec, q, a.q0, gs, lane);
    wave_gemv(a.D, a.minvf, gs, nullptr, g, lane);
  } else {
    wave_gemv(a.D, a.prec, q, a.q0, g, lane);
  }
}

// E = V + K = 0.5 (logc + (q - q0).P x + p.(minv p))  (samplers.py:811-823); P x is g (gs with a
// full cov_p, whose K takes the product inv_cov_p p into us)
template <bool MASS>
__device__ double wave_energy(const RandArgs& a, const double* q, const double* p, const double* g,
                              const double* gs, double* us, int lane) {
  double maha = 0.0, kin = 0.0;
  if constexpr (MASS) wave_gemv(a.D, a.minvf, p, nullptr, us, lane);
  for (int d = lane; d < a.D; d += kWave) {
    maha += (q[d] - q0_of(a, d)) * (MASS ? gs[d] : g[d]);
    kin += MASS ? p[d] * us[d] : p[d] * (minv_of(a, d) * p[d]);
  }
  return 0.5 * (a.logc + (wave_sum_dpp(maha) + wave_sum_dpp(kin)));
}

// one leapfrog step (samplers.py:831-839) from (sq, sp, sg) into (q, p, g); may run in place
template <bool EXACT, bool MASS>
__device__ void wave_leapfrog(const RandArgs& a, const double* sq, const double* sp, const double* sg, double* q,
                              double* p, double* g, double* gs, int lane) {
  for (int d = lane; d < a.D; d += kWave) {
    const double dt = dt_of(a, d), mi = MASS ? 1.0 : minv_of(a, d);
    double pd = sp[d];
    pd = EXACT ? pd - (dt * (mi * sg[d])) * 0.5 : __builtin_fma(-0.5 * dt * mi, sg[d], pd);
    const double qd = EXACT ? sq[d] + dt * pd : __builtin_fma(dt, pd, sq[d]);
    p[d] = pd;
    q[d] = qd;
  }
  wave_grad<MASS>(a, q, g, gs, lane);
  for (int d = lane; d < a.D; d += kWave) {
    const double dt = dt_of(a, d), mi = MASS ? 1.0 : minv_of(a, d);
    const double pd = p[d];
    p[d] = EXACT ? pd - (dt * (mi * g[d])) * 0.5 : __builtin_fma(-0.5 * dt * mi, g[d], pd);
  }
}

// sum over d of (rq - lq) . v, the U-turn dots of samplers.py:720-722 / :779-781
__device__ double wave_span_dot(int D, const double* rq, const double* lq, const double* v, int lane) {
  double s = 0.0;
  for (int d = lane; d < D; d += kWave) s += (rq[d] - lq[d]) * v[d];
  return wave_sum_dpp(s);
}

__device__ __forceinline__ void wave_copy(int D, const double* src, double* dst, int lane) {
  for (int d = lane; d < D; d += kWave) dst[d] = src[d];
}

// utils.py:246-283 check_points(m) for even m as an iterator: the first point of every aligned
// power-of-two sub-tree (size >= 2) ending at m, smallest start first
struct CheckPoints {
  int pt, half;
  __device__ explicit CheckPoints(int m) {
    int r = m;
    while ((r & (r - 1)) != 0 && r > 2) r -= 1 << (31 - __builtin_clz(r));
    pt = m - r + 1;
    half = r;
  }
  __device__ bool next() {   // advance; false when done
    if (half <= 2) return false;
    half >>= 1;
    pt += half;
    return true;
  }
};

// utils.py:367-385 release_fast(m, l)
__device__ __forceinline__ bool release_fast(int m, int l) {
  while ((m & (m - 1)) != 0 && m > 4) {
    const int top = 1 << (31 - __builtin_clz(m));
    m -= top;
    l -= top;
  }
  return m >= 4 && l > 1;
}

template <bool EXACT, bool REPLAY, bool MASS>
__global__ __launch_bounds__(256) void k_nuts_big(RandArgs a, int Dp, int nv) {
  __shared__ double tab[REPLAY ? 2 : kNormalTableDoubles];
  if constexpr (!REPLAY) {
    init_normal_tables(tab);
    __syncthreads();
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  if (c >= a.n) return;
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  const int D = a.D, d_max = a.d_max;
  const ChainVecs W{a.ws + c * (int64_t)nv * Dp, Dp};
  double* gs = W.v(scratch0(a.d_max));       // P x of the newest point (full cov_p)
  double* us = W.v(scratch0(a.d_max) + 1);   // inv_cov_p p, or the momentum's z (full cov_p)
  int64_t* tcur = reinterpret_cast<int64_t*>(a.ws + a.n * (int64_t)nv * Dp);
  int64_t tpos = REPLAY ? tcur[c] : 0;
  double* qs = a.q + c * (int64_t)D;
  double Eprev = a.Eprev[c];
  unsigned long long n_lf = 0, n_unst = 0, n_dmax = 0, n_tape = 0;
  int it = 0;
  uint32_t ndraw = 0;

  auto draw = [&](bool direction) -> double {          // next tree draw of this chain (reference order)
    if constexpr (REPLAY) {
      if (tpos >= a.tape_stride) {                      // exhausted tape: flagged, the host raises
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

  for (it = a.it0; it < a.it1; ++it) {
    // ---- iteration start (:563-584): p, E_initial, both ends (q, -p) / (q, p), live_q_old = q
    int cur = 0, lft = 1, rgt = 2, old = kLive0, nw = kLive0 + 1;
    auto tq = [&](int t) { return W.v(3 * t); };
    auto tp = [&](int t) { return W.v(3 * t + 1); };
    auto tg = [&](int t) { return W.v(3 * t + 2); };
    for (int d = lane; d < D; d += kWave) {
      double pd;
      if constexpr (REPLAY) {
        pd = a.rp[(c * (int64_t)a.niter + (it - 1)) * D + d];
      } else {
        const int h = d & 3, j = d >> 3;
        double z0, z1;
        normal_pair_tab(draw_block((uint32_t)(8 * j + h), (uint32_t)it, gc, a.k0, a.k1), tab, z0, z1);
        pd = ((d >> 2) & 1 ? z1 : z0) * ps_of(a, d);
      }
      const double qd = qs[d];
      tq(rgt)[d] = qd;
      if (MASS && !REPLAY) {
        us[d] = pd;                                                            // z; p = C z below
      } else {
        tp(rgt)[d] = pd;
        tp(lft)[d] = -pd;
      }
      tq(lft)[d] = qd;
      W.v(old)[d] = qd;
    }
    if constexpr (MASS && !REPLAY) {                                           // p ~ N(0, cov_p) (:829)
      wave_gemv(D, a.cholt, us, nullptr, tp(rgt), lane);
      for (int d = lane; d < D; d += kWave) tp(lft)[d] = -tp(rgt)[d];
    }
    wave_grad<MASS>(a, tq(rgt), tg(rgt), gs, lane);
    wave_copy(D, tg(rgt), tg(lft), lane);
    const double E_init = wave_energy<MASS>(a, tq(rgt), tp(rgt), tg(rgt), gs, us, lane);   // :569
    if (write_row_of(it) && lane == 0) {                                       // :571-573
      const int64_t row = c * (int64_t)a.Lc + (it - a.wu) / a.thin;
      if (a.Ec) a.Ec[row] = E_init;
      if (a.dEc) a.dEc[row] = E_init - Eprev;
    }
    double E_max_old = E_init, pi_old = 1.0;
    bool lterm = false, rterm = false;
    ndraw = 0;
    for (int d = 0; !lterm || !rterm; ++d) {                                   // :595 (Q10)
      if (d > d_max - 1) {                                                     // :596-598 (Q12)
        ++n_dmax;
        break;
      }
      int table[kNutsDmaxMax + 1];                                             // :601 save-slot table
#pragma unroll
      for (int s = 0; s <= kNutsDmaxMax; ++s) table[s] = -1;
      auto find_next = [&]() {                                                 // utils.py:222-228
        int f = -1;
#pragma unroll
        for (int s = kNutsDmaxMax; s >= 0; --s)
          if (s <= d_max && table[s] == -1) f = s;
        return f;
      };
      auto set_slot = [&](int s, int v) {
#pragma unroll
        for (int i = 0; i <= kNutsDmaxMax; ++i)
          if (i == s) table[i] = v;
      };
      auto save = [&](int v) {                                                 // q_save / p_save (:623-626)
        const int s = find_next();
        wave_copy(D, tq(cur), W.v(kSave0 + 2 * s), lane);
        wave_copy(D, tp(cur), W.v(kSave0 + 2 * s + 1), lane);
        set_slot(s, v);
      };
      const int L_new = 1 << d;
      const int udir = (int)draw(true);                                        // :608
      const int from = udir == 0 ? rgt : lft;
      wave_leapfrog<EXACT, MASS>(a, tq(from), tp(from), tg(from), tq(cur), tp(cur), tg(cur), gs, lane);   // :611-614
      ++n_lf;
      wave_copy(D, tq(cur), W.v(nw), lane);                                    // live_q_new (:617)
      double E_max_now = wave_energy<MASS>(a, tq(cur), tp(cur), tg(cur), gs, us, lane);   // :618
      double pi_new = 1.0;
      save(1);
      bool reject = false;
      for (int k = 1; k < L_new; ++k) {                                        // :637
        wave_leapfrog<EXACT, MASS>(a, tq(cur), tp(cur), tg(cur), tq(cur), tp(cur), tg(cur), gs, lane);
        ++n_lf;
        const double E_tmp = wave_energy<MASS>(a, tq(cur), tp(cur), tg(cur), gs, us, lane);   // :643
        if (fabs(E_tmp - E_init) > 1000.0) {                                   // :647-651
          reject = true;
          ++n_unst;
          break;
        }
        if (((k + 1) & 1) == 1) {                                              // :654-658
          save(k + 1);
        } else {                                                               // :699-736
          CheckPoints cp(k + 1);
          do {
            const int l = cp.pt;
            int s = 0;
#pragma unroll
            for (int i = kNutsDmaxMax; i >= 0; --i)                            // retrieve_save_index
              if (table[i] == l) s = i;
            const double* q_chk = W.v(kSave0 + 2 * s);
            const double* p_chk = W.v(kSave0 + 2 * s + 1);
            // udir 0: left = (q_chk, -p_chk), right = current; udir 1: left = current, right = (q_chk, -p_chk)
            double rdot, ldot;   // Dq.rp and -Dq.lp with Dq = rq - lq
            if (udir == 0) {
              rdot = wave_span_dot(D, tq(cur), q_chk, tp(cur), lane);
              ldot = wave_span_dot(D, tq(cur), q_chk, p_chk, lane);            // -Dq.(-p_chk)
            } else {
              rdot = -wave_span_dot(D, q_chk, tq(cur), p_chk, lane);           // Dq.(-p_chk)
              ldot = -wave_span_dot(D, q_chk, tq(cur), tp(cur), lane);         // -Dq.p
            }
            if (ldot < 0.0 && rdot < 0.0) {
              reject = true;
              break;
            }
            if (l > 1 && release_fast(k + 1, l)) set_slot(s, -1);
          } while (cp.next());
          if (reject) break;
        }
        const double E_max_prev = E_max_now;                                   // :743-751
        E_max_now = fmax(E_max_prev, E_tmp);
        const double num = exp(-(E_tmp - E_max_now));
        pi_new = num + exp(E_max_now - E_max_prev) * pi_new;
        const double r_ = num / pi_new;
        if (draw(false) < r_) wave_copy(D, tq(cur), W.v(nw), lane);
      }
      if (reject) break;                                                       // :754-755
      if (udir == 0) {                                                         // :758-761
        const int t = rgt;
        rgt = cur;
        cur = t;
      } else {
        const int t = lft;
        lft = cur;
        cur = t;
      }
      const double r_ = exp(-(E_max_now - E_max_old)) * pi_old / pi_new;       // :766 (Q11)
      const double E_max_old_prev = E_max_old;
      E_max_old = fmax(E_max_old_prev, E_max_now);
      pi_old = exp(-(E_max_now - E_max_old)) * pi_new + exp(-(E_max_old_prev - E_max_old)) * pi_old;   // :771
      const double A = fmin(1.0, r_);
      if (draw(false) < A) {                                                   // :773-775
        const int t = old;
        old = nw;
        nw = t;
      }
      rterm = wave_span_dot(D, tq(rgt), tq(lft), tp(rgt), lane) < 0.0;          // :779-781
      lterm = -wave_span_dot(D, tq(rgt), tq(lft), tp(lft), lane) < 0.0;
    }
    // ---- iteration end (:786-791): q = live_point_q_old, sample row
    Eprev = E_init;
    const double* qf = W.v(old);
    const int qrow = (it - a.wu) / a.thin;
    double* rowp = (write_row_of(it) && a.qc && qrow >= a.q_row0) ? a.qc + (c * (int64_t)a.Lq + qrow % a.Lq) * D
                                                                  : nullptr;
    for (int d = lane; d < D; d += kWave) {
      const double qd = qf[d];
      qs[d] = qd;
      if (rowp) rowp[d] = qd;
    }
  }
  if (lane == 0) {
    a.Eprev[c] = Eprev;
    if (REPLAY) tcur[c] = tpos;
    if (a.cnt) {
      unsigned long long* cs = a.cnt + (c & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
      if (n_lf) {
        atomicAdd(cs + HMC_CNT_LEAPFROG, n_lf);
        atomicAdd(cs + HMC_CNT_ENERGY_EVALS, n_lf);
        atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, n_lf);   // NUTS: wave steps (one chain per wave here)
      }
      if (n_unst) atomicAdd(cs + HMC_CNT_UNSTABLE, n_unst);
      if (n_dmax) atomicAdd(cs + HMC_CNT_DMAX, n_dmax);
      if (n_tape) atomicAdd(cs + HMC_CNT_OOB_REJECT, n_tape);
    }
  }
}

int nuts_big_vectors(int d_max) { return scratch0(d_max) + 2; }
int nuts_big_padded(int D) { return (D + kWave - 1) / kWave * kWave; }

}  // namespace

int64_t nuts_big_ws_doubles(int64_t n, int D, int d_max) {
  return n * (int64_t)nuts_big_vectors(d_max) * nuts_big_padded(D) + n;   // vectors + tape cursors
}

hipError_t launch_nuts_big(const RandArgs& a, bool exact, bool replay, hipStream_t s) {
  const int Dp = nuts_big_padded(a.D), nv = nuts_big_vectors(a.d_max);
  const dim3 grid((unsigned)((a.n + 3) / 4));
  if (a.minvf) {
    if (exact) {
      if (replay) k_nuts_big<true, true, true><<<grid, 256, 0, s>>>(a, Dp, nv);
      else k_nuts_big<true, false, true><<<grid, 256, 0, s>>>(a, Dp, nv);
    } else {
      if (replay) k_nuts_big<false, true, true><<<grid, 256, 0, s>>>(a, Dp, nv);
      else k_nuts_big<false, false, true><<<grid, 256, 0, s>>>(a, Dp, nv);
    }
  } else if (exact) {
    if (replay) k_nuts_big<true, true, false><<<grid, 256, 0, s>>>(a, Dp, nv);
    else k_nuts_big<true, false, false><<<grid, 256, 0, s>>>(a, Dp, nv);
  } else {
    if (replay) k_nuts_big<false, true, false><<<grid, 256, 0, s>>>(a, Dp, nv);
    else k_nuts_big<false, false, false><<<grid, 256, 0, s>>>(a, Dp, nv);
  }
  return hipGetLastError();
}

}  // namespace hmc
