// hmc_random.hip — fused Random-trajectory HMC iterations for diagonal-precision MVN targets.
//
// Replaces the hot triple loop of HMC_sampler.gen_sample_random (samplers.py:410 -> :428 -> :448)
// and its primitives K / E / p_sample / leap_frog (samplers.py:811-839) for targets whose
// precision inv(cov0) is diagonal (identity in BASELINE configs 1, 2, 4).
//
// One launch runs iterations [it0, it1) of every chain: state q stays in registers across
// iterations, each iteration does
//     p ~ N(0, cov_p)                      (replay stream or in-kernel Philox + Box–Muller)
//     E0 = V(q) + K(p)                     -> E_chain / dE_chain row            (Q14)
//     L  ~ U{L_low..L_high-1}              (Q1)
//     L x leap_frog with the gradient of q_new reused as the next step's q_old (bit-identical)
//     E1, dE = E1 - E0, accept iff dE < 0 or log u < -dE
//     store q_chain row (i - warm_up)//thin  (last write of a thinned row wins, as in Python)
// HBM traffic per chain-iteration: one q_chain row (8D B) + E + dE (16 B); q is read/written
// once per launch.  The arithmetic is fp64 VALU; EXACT mode keeps the reference's operation
// order with no FMA contraction (built with -ffp-contract=off), so for diagonal targets the
// sampled states are bit-identical to the NumPy reference on replayed streams.
#include <cstdlib>

#include "hmc_device.hpp"
#include "hmc_internal.hpp"
#include "hmc_target_ops.hpp"

namespace hmc {

namespace {

__device__ __forceinline__ unsigned long long stamp(bool on) {
  return on ? __builtin_amdgcn_s_memtime() : 0ull;
}

struct Lane {
  int lane, g, s, base;
  int64_t c;       // local chain index
  bool active;     // lane belongs to a live chain
  bool leader;     // first lane of a live chain's group
};

__device__ __forceinline__ Lane lane_info(const RandArgs& a) {
  Lane L;
  L.lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  L.g = L.lane / a.lpc;
  L.s = L.lane - L.g * a.lpc;
  L.base = L.g * a.lpc;
  L.c = wave * a.cpw + L.g;
  L.active = (L.g < a.cpw) && (L.c < a.n);
  L.leader = L.active && (L.s == 0);
  return L;
}

template <int K, bool GEN>
__device__ __forceinline__ double chain_energy(const RandArgs& a, const Lane& ln, const int (&kk)[K],
                                               const bool (&pv)[K], const double (&q)[2 * K],
                                               const double (&p)[2 * K]) {
  // E = V + K = 0.5*(logdet_const + (q-q0)^T P (q-q0)) + p^T Minv p / 2  (utils.py:218, samplers.py:817),
  // summed as one group reduction of the per-coordinate terms.
  double maha = 0.0, kin = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (pv[j]) {
      const int d = 2 * kk[j];
      energy_terms<GEN>(dim_const<GEN>(a, d), q[2 * j], p[2 * j], maha, kin);
      if (d + 1 < a.D) energy_terms<GEN>(dim_const<GEN>(a, d + 1), q[2 * j + 1], p[2 * j + 1], maha, kin);
    }
  }
  const double tot = group_sum(maha + kin, ln.s, a.lpc, ln.base);
  return 0.5 * (a.logc + tot);
}

template <int K, bool GEN, bool REPLAY>
__device__ __forceinline__ void draw_momentum(const RandArgs& a, const Lane& ln, int it, const int (&kk)[K],
                                              const bool (&pv)[K], double (&p)[2 * K]) {
  const bool even = (a.D & 1) == 0;
  const uint64_t gc = (uint64_t)(a.chain_offset + ln.c);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    p[2 * j] = 0.0;
    p[2 * j + 1] = 0.0;
    if (pv[j]) {
      const int d = 2 * kk[j];
      if constexpr (REPLAY) {
        const double* row = (it == 0) ? a.rp0 + ln.c * (int64_t)a.D
                                      : a.rp + (ln.c * (int64_t)a.niter + (it - 1)) * a.D;
        load_pair(row, kk[j], even, d + 1 < a.D, p[2 * j], p[2 * j + 1]);
      } else {
        normal_pair(draw_block((uint32_t)kk[j], (uint32_t)it, gc, a.k0, a.k1), p[2 * j], p[2 * j + 1]);
        if (GEN && a.pscale) {
          p[2 * j] *= a.pscale[d];
          if (d + 1 < a.D) p[2 * j + 1] *= a.pscale[d + 1];
        }
      }
      if (d + 1 >= a.D) p[2 * j + 1] = 0.0;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Chain initialisation (samplers.py:413-420): q_chain[:,0] = q_start, E_chain[:,0] = E(q, p0).
template <int K, bool GEN, bool REPLAY>
__global__ __launch_bounds__(256) void k_random_init(RandArgs a) {
  const Lane ln = lane_info(a);
  const bool even = (a.D & 1) == 0;
  int kk[K];
  bool pv[K];
  double q[2 * K], p[2 * K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    kk[j] = ln.s + a.lpc * j;
    pv[j] = ln.active && kk[j] < a.npairs;
    q[2 * j] = q[2 * j + 1] = 0.0;
    if (pv[j]) load_pair(a.qstart + ln.c * (int64_t)a.D, kk[j], even, 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
  }
  draw_momentum<K, GEN, REPLAY>(a, ln, 0, kk, pv, p);
  const double E0 = chain_energy<K, GEN>(a, ln, kk, pv, q, p);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (pv[j]) {
      const bool v1 = 2 * kk[j] + 1 < a.D;
      store_pair(a.q + ln.c * (int64_t)a.D, kk[j], even, v1, q[2 * j], q[2 * j + 1]);
      if (a.qc && a.q_row0 == 0) store_pair(a.qc + ln.c * (int64_t)a.Lq * a.D, kk[j], even, v1, q[2 * j], q[2 * j + 1]);
    }
  }
  if (ln.leader) {
    a.Eprev[ln.c] = E0;
    if (a.Ec) a.Ec[ln.c * (int64_t)a.Lc] = E0;
    if (a.dEc) a.dEc[ln.c * (int64_t)a.Lc] = 0.0;
  }
}

// ------------------------------------------------------------------------------------------
// Iterations [it0, it1) (samplers.py:428-475).
template <int K, bool EXACT, bool GEN, bool REPLAY>
__global__ __launch_bounds__(256) void k_random_iters(RandArgs a) {
  const unsigned long long t_start = stamp(a.stamps != nullptr);
  const Lane ln = lane_info(a);
  const bool even = (a.D & 1) == 0;
  const uint64_t gc = (uint64_t)(a.chain_offset + ln.c);
  int kk[K];
  bool pv[K];
  double q[2 * K], p[2 * K], qi[2 * K], t[2 * K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    kk[j] = ln.s + a.lpc * j;
    pv[j] = ln.active && kk[j] < a.npairs;
    q[2 * j] = q[2 * j + 1] = 0.0;
    if (pv[j]) load_pair(a.q + ln.c * (int64_t)a.D, kk[j], even, 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
  }
  double Eprev = ln.active ? a.Eprev[ln.c] : 0.0;
  unsigned long long n_acc = 0, n_acc_wu = 0, n_lf = 0, n_lf2 = 0, n_oob = 0;
  int it_base = a.it0 - a.lpc, draw_L = 0;     // cached (L, log u) draws (Philox mode)
  double draw_lnu = 0.0;
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};   // diagnostic phase timers (stamps build path)
  // Retire the state loads here: the wait-count pass otherwise sees them pending at the loop
  // header and emits vmcnt(0) inside the loop, which (loads and stores share one in-order
  // counter on gfx950) stalls every iteration on the previous iteration's sample stores.
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) only

  for (int it = a.it0; it < a.it1; ++it) {
    // ---- momentum resample (samplers.py:431) and initial energy (:434)
    const bool st_on = a.stamps != nullptr;
    unsigned long long t_0 = stamp(st_on);
    if (!(a.dbg & 1)) {
      draw_momentum<K, GEN, REPLAY>(a, ln, it, kk, pv, p);
    } else {
#pragma unroll
      for (int e = 0; e < 2 * K; ++e) p[e] = 0.3;
    }
    unsigned long long t_1 = stamp(st_on);
    const double E0 = (a.dbg & 2) ? 0.0 : chain_energy<K, GEN>(a, ln, kk, pv, q, p);
    unsigned long long t_2 = stamp(st_on);
    const bool post = it >= a.wu;
    const bool write_row = post && ((it == a.niter) || ((it - a.wu + 1) % a.thin == 0));
    const int64_t row = post ? (int64_t)((it - a.wu) / a.thin) : 0;
    if (ln.leader && write_row && !(a.dbg & 8)) {       // :436-438 (Q14)
      __builtin_nontemporal_store(E0, a.Ec + ln.c * (int64_t)a.Lc + row);
      __builtin_nontemporal_store(E0 - Eprev, a.dEc + ln.c * (int64_t)a.Lc + row);
    }
    Eprev = E0;                                          // :460

    // ---- trajectory length (:441) and log-uniform for the MH test (:461)
    int L;
    double lnu;
    if constexpr (REPLAY) {
      L = ln.active ? a.rL[ln.c * (int64_t)a.niter + (it - 1)] : 0;
      lnu = ln.active ? a.rlnu[ln.c * (int64_t)a.niter + (it - 1)] : 0.0;
    } else {
      // lane s of the group draws (L, u) of iteration it_base + s once per LPC iterations;
      // iteration it reads them from lane base + (it - it_base)
      if (it - it_base >= a.lpc) {
        it_base = it;
        const uint4 r = draw_block(kDrawSlot, (uint32_t)(it + ln.s), gc, a.k0, a.k1);
        draw_L = uniform_int(r.x, a.L_low, a.L_high);
        const double u = u53(r.z, r.w);
        draw_lnu = u > 0.0 ? fast_log(u) : -__builtin_inf();   // log(random()), :461
      }
      L = __shfl(draw_L, ln.base + (it - it_base), kWave);
      lnu = __shfl(draw_lnu, ln.base + (it - it_base), kWave);
      if (a.dbg & 16) L = 12;
      if (a.dbg & 4) L = 0;
      if (!ln.active) L = 0;
    }

    unsigned long long t_3 = stamp(st_on);
    // ---- chain-0 trajectory capture (samplers.py:442-452): lane holding dims 0,1 records q[:2]
    const bool cap = a.traj_q && (gc == 0) && (it <= a.n_save) && ln.leader;
    double* capp = cap ? a.traj_q + (int64_t)(it - 1) * a.traj_stride * 2 : nullptr;
    if (cap) {
      capp[0] = q[0];
      capp[1] = a.D > 1 ? q[1] : q[0];
    }

    // ---- L leapfrog steps (:448-450 -> :831-839)
#pragma unroll
    for (int e = 0; e < 2 * K; ++e) qi[e] = q[e];
    if constexpr (EXACT) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int h = 0; h < 2; ++h) t[2 * j + h] = kick<GEN>(slot_const<GEN>(a, kk[j], h, pv[j]), q[2 * j + h]);
      }
      for (int l = 0; l < L; ++l) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = 2 * j + h;
            const DimConst c = slot_const<GEN>(a, kk[j], h, pv[j]);
            const double ph = p[e] - t[e];              // p_half = p_old - dt*(M^-1 dVdq(q_old))/2
            q[e] = q[e] + c.dt * ph;                    // q_new  = q_old + dt*p_half
            t[e] = kick<GEN>(c, q[e]);                  // dt*(M^-1 dVdq(q_new))/2, reused next step
            p[e] = ph - t[e];                           // p_new  = p_half - ...
          }
        }
        if (cap) {
          capp[2 * (l + 1)] = q[0];
          capp[2 * (l + 1) + 1] = a.D > 1 ? q[1] : q[0];
        }
      }
    } else {
      for (int l = 0; l < L; ++l) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = 2 * j + h;
            const DimConst c = slot_const<GEN>(a, kk[j], h, pv[j]);
            const double cc = GEN ? c.hd * (c.minv * c.prec) : c.hd;
            const double ph = __builtin_fma(-cc, q[e] - c.q0, p[e]);
            q[e] = __builtin_fma(c.dt, ph, q[e]);
            p[e] = __builtin_fma(-cc, q[e] - c.q0, ph);
          }
        }
        if (cap) {
          capp[2 * (l + 1)] = q[0];
          capp[2 * (l + 1) + 1] = a.D > 1 ? q[1] : q[0];
        }
      }
    }
    // lanes whose slot is past D carry zeros; keep them zero
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (!pv[j] || 2 * kk[j] + 1 >= a.D) {
        q[2 * j + 1] = 0.0;
        p[2 * j + 1] = 0.0;
        if (!pv[j]) q[2 * j] = p[2 * j] = 0.0;
      }
    }

    unsigned long long t_4 = stamp(st_on);
    // ---- final energy and Metropolis test (:455-472)
    const double E1 = (a.dbg & 2) ? 0.0 : chain_energy<K, GEN>(a, ln, kk, pv, q, p);
    unsigned long long t_5 = stamp(st_on);
    const double dE = E1 - E0;
    const bool accept = (dE < 0.0) || (lnu < -dE);
    if (!accept) {
#pragma unroll
      for (int e = 0; e < 2 * K; ++e) q[e] = qi[e];
    }
    if (write_row && a.qc && !(a.dbg & 8) && row >= a.q_row0) {
      double* rowp = a.qc + (ln.c * (int64_t)a.Lq + row % a.Lq) * a.D;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (pv[j]) store_pair(rowp, kk[j], even, 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
    }
    if (cap) {
      a.traj_len[it - 1] = (L > 0 ? L : 0) + 1;
      a.decision[it - 1] = accept ? 1 : 0;
    }
    if (ln.leader) {
      if (accept) {
        if (post) ++n_acc; else ++n_acc_wu;
      } else if (it < a.i_oob) {
        ++n_oob;                                         // reference would raise IndexError (Q5)
      }
      const unsigned long long Lp = L > 0 ? (unsigned long long)L : 0ull;  // xrange(1, L+1) is empty for L <= 0
      n_lf += Lp;
      n_lf2 += Lp * Lp;
    }
    if (st_on) {
      const unsigned long long t_6 = stamp(true);
      ph[0] += t_1 - t_0;   // momentum draw
      ph[1] += t_2 - t_1;   // E0
      ph[2] += t_3 - t_2;   // row bookkeeping + L/u draw
      ph[3] += t_4 - t_3;   // leapfrog loop
      ph[4] += t_5 - t_4;   // E1
      ph[5] += t_6 - t_5;   // MH + stores
    }
  }

  // ---- state write-back and counters
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (pv[j]) store_pair(a.q + ln.c * (int64_t)a.D, kk[j], even, 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
  if (ln.leader) a.Eprev[ln.c] = Eprev;
  if (a.stamps && ln.lane == 0) {
    const int64_t wv = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
#pragma unroll
    for (int i = 0; i < 6; ++i) a.stamps[wv * kStampWords + i] = ph[i];
    a.stamps[wv * kStampWords + 6] = t_start;
    a.stamps[wv * kStampWords + 7] = stamp(true);
    // hardware placement: HW_ID (wave/simd/cu/sh/se) in the high word of slot 5's neighbour
    const unsigned hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    a.stamps[wv * kStampWords + 5] = ((unsigned long long)hwid << 32) | ((unsigned long long)(xcc & 0xffff) << 16) |
                           (a.stamps[wv * kStampWords + 5] & 0xffffull);
  }
  n_acc = wave_sum_u64(n_acc);
  n_acc_wu = wave_sum_u64(n_acc_wu);
  n_lf = wave_sum_u64(n_lf);
  n_lf2 = wave_sum_u64(n_lf2);
  n_oob = wave_sum_u64(n_oob);
  if (ln.lane == 0 && a.cnt) {   // per-wave counts into one of HMC_COUNTER_SLOTS rows
    const int64_t wv = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    unsigned long long* cs = a.cnt + (wv & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
    if (n_acc) atomicAdd(cs + HMC_CNT_ACCEPT, n_acc);
    if (n_acc_wu) atomicAdd(cs + HMC_CNT_ACCEPT_WU, n_acc_wu);
    if (n_lf) atomicAdd(cs + HMC_CNT_LEAPFROG, n_lf);
    if (n_lf2) atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, n_lf2);
    if (n_oob) atomicAdd(cs + HMC_CNT_OOB_REJECT, n_oob);
  }
}

template <int K>
hipError_t launch_init_k(const RandArgs& a, bool gen, bool replay, dim3 grid, hipStream_t s) {
  if (gen) {
    if (replay) k_random_init<K, true, true><<<grid, 256, 0, s>>>(a);
    else k_random_init<K, true, false><<<grid, 256, 0, s>>>(a);
  } else {
    if (replay) k_random_init<K, false, true><<<grid, 256, 0, s>>>(a);
    else k_random_init<K, false, false><<<grid, 256, 0, s>>>(a);
  }
  return hipGetLastError();
}

template <int K, bool EXACT>
hipError_t launch_iters_k2(const RandArgs& a, bool gen, bool replay, dim3 grid, hipStream_t s) {
  if (gen) {
    if (replay) k_random_iters<K, EXACT, true, true><<<grid, 256, 0, s>>>(a);
    else k_random_iters<K, EXACT, true, false><<<grid, 256, 0, s>>>(a);
  } else {
    if (replay) k_random_iters<K, EXACT, false, true><<<grid, 256, 0, s>>>(a);
    else k_random_iters<K, EXACT, false, false><<<grid, 256, 0, s>>>(a);
  }
  return hipGetLastError();
}

template <int K>
hipError_t launch_iters_k(const RandArgs& a, bool exact, bool gen, bool replay, dim3 grid, hipStream_t s) {
  return exact ? launch_iters_k2<K, true>(a, gen, replay, grid, s)
               : launch_iters_k2<K, false>(a, gen, replay, grid, s);
}

dim3 grid_for(const RandArgs& a) {
  const int64_t waves = (a.n + a.cpw - 1) / a.cpw;
  return dim3((unsigned)((waves + 3) / 4));
}

}  // namespace

// E[max of c iid U{lo..hi-1}] — the wave runs as long as its longest trajectory.
static double expected_max(int lo, int hi, int c) {
  const int n = hi - lo;
  if (n <= 1 || c <= 1) return 0.5 * (lo + hi - 1);
  double e = 0.0, prev = 0.0;
  for (int x = lo; x < hi; ++x) {
    const double F = pow((double)(x - lo + 1) / n, c);
    e += x * (F - prev);
    prev = F;
  }
  return e;
}

Layout choose_layout(int D, int L_low, int L_high) {
  static const int Ks[] = {1, 2, 4, 5, 8, 16};
  Layout best{0, 0, 0, (D + 1) / 2};
#ifdef HMC_DEBUG_HOOKS
  if (const char* fk = getenv("HMC_FORCE_K")) {   // experiments: force the pairs-per-lane template
    const int K = atoi(fk);
    const int lpc = (best.npairs + K - 1) / K;
    for (int k : Ks)
      if (k == K && lpc <= kWave) return Layout{K, lpc, kWave / lpc, best.npairs};
  }
#endif
  // D > 64: one wavefront per chain (hmc_wave.hip): no trajectory-length divergence inside a
  // wave, wave-uniform control flow; K pairs per lane.
  if (best.npairs > kWave / 2) {
    for (int K : {1, 2, 4, 8, 16})
      if (K * kWave >= best.npairs) return Layout{K, kWave, 1, best.npairs};
    return best;  // K = 0: unsupported
  }
  // small D: several chains per wave (lane groups); pick K by lane utilisation discounted by the
  // expected trajectory-length divergence between the chains sharing a wave
  double best_score = -1.0;
  const double mean = 0.5 * (L_low + L_high - 1);
  for (int K : Ks) {
    const int lpc = (best.npairs + K - 1) / K;
    if (lpc > kWave) continue;
    const int cpw = kWave / lpc;
    const double util = (double)best.npairs * cpw / (kWave * (double)K);
    const double emax = expected_max(L_low, L_high, cpw);
    const double score = util * (emax > 0 ? mean / emax : 1.0);
    if (score > best_score + 1e-9) {
      best_score = score;
      best.K = K;
      best.lpc = lpc;
      best.cpw = cpw;
    }
  }
  return best;
}

hipError_t launch_random_init(const RandArgs& a, const Layout& lay, bool gen, bool replay, hipStream_t s) {
  const dim3 grid = grid_for(a);
  switch (lay.K) {
    case 1: return launch_init_k<1>(a, gen, replay, grid, s);
    case 2: return launch_init_k<2>(a, gen, replay, grid, s);
    case 4: return launch_init_k<4>(a, gen, replay, grid, s);
    case 5: return launch_init_k<5>(a, gen, replay, grid, s);
    case 8: return launch_init_k<8>(a, gen, replay, grid, s);
    case 16: return launch_init_k<16>(a, gen, replay, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_random_iters(const RandArgs& a, const Layout& lay, bool exact, bool gen, bool replay,
                               hipStream_t s) {
#ifdef HMC_DEBUG_HOOKS
  const char* kern = getenv("HMC_KERNEL");       // experiments: "group" forces the lane-group kernel
  const bool force_group = kern && kern[0] == 'g';
#else
  const bool force_group = false;
#endif
  if (lay.cpw == 1 && !force_group && (lay.K == 1 || lay.K == 2 || lay.K == 4 || lay.K == 8 || lay.K == 16))
    return launch_wave_iters(a, lay.K, exact, gen, replay, s);
  const dim3 grid = grid_for(a);
  switch (lay.K) {
    case 1: return launch_iters_k<1>(a, exact, gen, replay, grid, s);
    case 2: return launch_iters_k<2>(a, exact, gen, replay, grid, s);
    case 4: return launch_iters_k<4>(a, exact, gen, replay, grid, s);
    case 5: return launch_iters_k<5>(a, exact, gen, replay, grid, s);
    case 8: return launch_iters_k<8>(a, exact, gen, replay, grid, s);
    case 16: return launch_iters_k<16>(a, exact, gen, replay, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace hmc
