// hmc_dense.hip — Random-trajectory HMC for correlated MVN targets (dense precision P = inv(cov0)).
//
// Replaces gen_sample_random (samplers.py:428-475) with the dense dVdq closure of the driver
// scripts, dVdq(q) = inv_cov0 (q - q0) (case3-script.py:45-49, BASELINE config 3: D=100, rho=0.95).
//
// The gradient of 16 chains is one GEMM tile G^T = P . X^T on v_mfma_f64_16x16x4_f64:
//   A = P fragment (16 dims x 4 k), read from LDS where the whole P sits as lane-linear
//       fragments (D padded to 16*MT; MT = 7 -> 112 x 112 x 8 B = 98 KiB per block);
//   B = X^T fragment: lane l supplies x[chain l&15][dim 4ks + (l>>4)];
//   C = 16x16 f64 tile: lane l receives g[chain l&15][dim 16nt + (l>>4) + 4r], r < 4.
// Lane (c = l&15, h = l>>4) therefore owns dims d = h + 4m (m < 4*MT) of chain c in BOTH the
// accumulator and the B-operand layout: the gradient feeds the next step's B operand and the
// elementwise kick/drift with no lane movement and no transpose (cdna_hip_programming.md §3,
// "an accumulator tile as the next MFMA's operand").  The energy V = 0.5*(c + x.g) reuses the
// gradient; the 4 lanes of a chain reduce with two xor-shuffles.
// Chains of one wave can have different trajectory lengths L: the wave runs max L and
// finished chains are masked (their gradient is recomputed at an unchanged q, bit-identical).
#include <algorithm>

#include "hmc_device.hpp"
#include "hmc_internal.hpp"
#include "hmc_dense_ops.hpp"

// Waves per block (one block per CU: the LDS copy of P).  8 = two waves per SIMD at 256 registers:
// the kernel spills ~88 B per lane, but one wave's MFMA gradient overlaps the other's RNG,
// kick/drift and load latency: +9.5% over one wave per SIMD (MFMA busy was 68%).
#ifndef HMC_DENSE_WAVES
#define HMC_DENSE_WAVES 8
#endif

namespace hmc {

namespace {

// WAVES waves per block, one block per CU (the LDS copy of P); WAVES = 4: one wave per SIMD
// with the whole 512-register file.
#ifndef HMC_DENSE_DB
#define HMC_DENSE_DB 0
#endif
// fragment double buffering only with one wave per SIMD (HMC_DENSE_DB=1 forces it: A/B)
template <int WAVES>
constexpr bool kDenseDB = WAVES <= 4 || HMC_DENSE_DB;

// MASS: dense (non-diagonal) mass matrix (implies GEN): its own instantiation, so the extra
// products' registers never touch the diagonal-mass kernels.
// SHORT: the gradient's short-last-tile form (hmc_dense_ops.hpp): compiled in (kShortAlways) for
// the plain instances at D = 97..100, tested per launch (kShortRuntime) in the others.
template <int MT, bool EXACT, bool GEN, bool REPLAY, int WAVES, bool MASS = false, int SHORT = kShortRuntime>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4, WAVES / 4)))
void k_dense_iters(DenseArgs a) {
  constexpr int M = 4 * MT;
  // ME: the slots that can hold a dimension.  The instance compiled for D = 16(MT-1)+1 .. +4
  // (kShortAlways) needs m <= 4(MT-1), rounded up to a pair; the per-slot loops stop there and
  // the slots past it stay zero (D = 100: 26 of 28)
  constexpr int ME = SHORT == kShortAlways ? 4 * (MT - 1) + 2 : M;
  extern __shared__ double sP[];
  __shared__ double s_ntab[REPLAY ? 2 : kNormalTableDoubles];   // Box–Muller tables (Philox momentum)
  if constexpr (!REPLAY) init_normal_tables(s_ntab);             // synchronised by stage_precision
  stage_precision<MT, SHORT>(a, sP);

  const int lane = threadIdx.x & (kWave - 1);
  const int h = lane >> 4;
  unsigned long long n_acc = 0, n_acc_wu = 0, n_lf = 0, n_lf2 = 0, n_oob = 0;
  // Persistent waves: P is staged into LDS once per block and the block's waves stride over the
  // 16-chain tiles.  With a.order (L-ordered tiles, one iteration per launch) tile t holds the
  // chains order[16t .. 16t+15], which share (up to bucket edges) one trajectory length, so no
  // lane idles through another chain's longer trajectory.
  const int64_t wave_id = (int64_t)blockIdx.x * WAVES + (threadIdx.x / kWave);
  const int64_t n_waves = (int64_t)gridDim.x * WAVES;
  for (int64_t tile = wave_id; tile < a.ntiles; tile += n_waves) {
  const int64_t slot = tile * 16 + (lane & 15);
  const bool live = slot < a.n;
  const int64_t c = a.order ? (live ? (int64_t)a.order[slot] : 0) : slot;
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  // a.q keeps the chain's state at the start of the current iteration (written back on every
  // acceptance), so a rejection reloads it instead of holding a copy in registers
  double q[M], p[M];
  d4 acc[MT];
  double* const qrow = a.q + c * a.D;
  double* const qh = qrow + h;           // dims h + 4m: constant offsets 32m from one base
  // dim h + 4m < D  <=>  m < mfull, or m == mfull and h < D % 4: a scalar test for all but one m
  // (a per-lane compare for every m is loop-invariant and gets hoisted into 28 SGPR-pair masks)
  const int mfull = uniform_i(a.D >> 2), mrem = a.D & 3;
  auto dim_ok = [&](int m) -> bool { return m < mfull || (m == mfull && h < mrem); };
#pragma unroll
  for (int m = 0; m < M; ++m) {
    q[m] = (live && dim_ok(m)) ? qh[4 * m] : 0.0;
    p[m] = 0.0;                                          // (slots past ME are never written)
  }
  double Eprev = live ? a.Eprev[c] : 0.0;
  double* const qcb = a.qc ? a.qc + c * (int64_t)a.Lq * a.D : nullptr;
  // gradient cache (L-ordered launches, one iteration each): the gradient at q is read with q
  // instead of recomputed (13 -> 12 gradients per 12 leapfrogs); it is the value the MFMA tile
  // computed at that q, so results are bit-identical.  Other launches keep it up to date.
  double* const gch = a.gcache ? a.gcache + c * a.D + h : nullptr;
  const bool g_read = a.gcache && a.order && a.gvalid && uniform_i(*a.gvalid) != 0;
  if (g_read) {
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m >> 2][m & 3] = (live && dim_ok(m)) ? gch[4 * m] : 0.0;
  }
  // chain-0 trajectory capture (samplers.py:442-452): the wave holding global chain 0 (lane 0;
  // capture runs never use a.order)
  const bool cap_wave = a.traj_q && uniform_i((int)(__builtin_amdgcn_readfirstlane((int)(gc & 0xffffffff)) == 0 &&
                                                    __builtin_amdgcn_readfirstlane((int)(gc >> 32)) == 0));

  for (int it = a.it0; it < a.it1; ++it) {
    // ---- momentum (samplers.py:431): dims h+4m; Philox pairs (m, m+1) keyed by slot h + 8*(m/2)
    if constexpr (REPLAY) {
      const double* row = a.rp + (c * (int64_t)a.niter + (it - 1)) * a.D + h;
#pragma unroll
      for (int m = 0; m < ME; ++m) {
        p[m] = (live && dim_ok(m)) ? row[4 * m] : 0.0;
      }
    } else {
#pragma unroll
      for (int m = 0; m < ME; m += 2) {
        double z0 = 0.0, z1 = 0.0;
        if (m < mfull || (m == mfull && mrem > 0)) {   // uniform: pairs wholly in the padding are not drawn
          normal_pair_tab(draw_block(opaque_u32((uint32_t)(h + 4 * m)), (uint32_t)it, gc, a.k0, a.k1), s_ntab, z0,
                          z1);
          const int d0 = h + 4 * m, d1 = d0 + 4;
          if (GEN && a.pscale) {
            z0 *= a.pscale[min(d0, a.D - 1)];
            z1 *= a.pscale[min(d1, a.D - 1)];
          }
        }
        p[m] = dim_ok(m) ? z0 : 0.0;
        p[m + 1] = dim_ok(m + 1) ? z1 : 0.0;
        if ((m & 6) == 6) __builtin_amdgcn_sched_barrier(0);   // bound the RNG chains in flight (registers)
      }
      if constexpr (MASS) {   // dense mass matrix: p = C z ~ N(0, cov_p) (samplers.py:829)
        d4 cz[MT];
        matvec_global<MT>(a.cholt, a.D, lane, p, cz);
#pragma unroll
        for (int m = 0; m < ME; ++m) p[m] = dim_ok(m) ? gval<MT>(cz, m) : 0.0;
      }
    }
    // ---- gradient at q and E0 = V(q) + K(p)  (:434)
    if (!g_read || it != a.it0) {
      gradient<MT, GEN, kDenseDB<WAVES>, SHORT>(a, sP, lane, h, q, acc);
      if (gch && live) {              // keep the cache valid for rejections (q stays, so does g)
#pragma unroll
        for (int m = 0; m < ME; ++m)
          if (dim_ok(m)) gch[4 * m] = gval<MT>(acc, m);
      }
    }
    double maha = 0.0, kin = 0.0;
    // (x . P x, p . Minv p) of this lane's dims.  Diagonal/identity mass: P x is the gradient
    // tile.  Dense mass: the tile holds Minv P x (the kick), so P x and Minv p are two more
    // products (samplers.py:811-823 with a full inv_cov_p).
    auto energy_terms = [&](double& mh, double& kn) {
      if constexpr (MASS) {
        double xv[M];
#pragma unroll
        for (int m = 0; m < ME; ++m) xv[m] = a.q0 ? q[m] - a.q0[min(h + 4 * m, a.D - 1)] : q[m];
        d4 t[MT];
        matvec_global<MT>(a.prec, a.D, lane, xv, t);
#pragma unroll
        for (int m = 0; m < ME; ++m) mh += xv[m] * gval<MT>(t, m);
        matvec_global<MT>(a.minvf, a.D, lane, p, t);
#pragma unroll
        for (int m = 0; m < ME; ++m) kn += p[m] * gval<MT>(t, m);
        return;
      }
#pragma unroll
      for (int m = 0; m < ME; ++m) {       // padded dims contribute exact zeros (g = p = 0)
        const int d = h + 4 * m;
        const double x = (GEN && a.q0) ? q[m] - a.q0[min(d, a.D - 1)] : q[m];
        mh += x * gval<MT>(acc, m);
        kn += p[m] * (dim_minv<MT, GEN>(a, d) * p[m]);
      }
    };
    energy_terms(maha, kin);
    const double E0 = 0.5 * (a.logc + chain_sum4(maha + kin));
    const bool post = it >= a.wu;
    const bool write_row = post && ((it == a.niter) || ((it - a.wu + 1) % a.thin == 0));
    const int64_t row = post ? (int64_t)((it - a.wu) / a.thin) : 0;
    if (live && h == 0 && write_row) {
      if (a.Ec) a.Ec[c * (int64_t)a.Lc + row] = E0;
      if (a.dEc) a.dEc[c * (int64_t)a.Lc + row] = E0 - Eprev;
    }
    Eprev = E0;
    // ---- L (:441) and log u (:461), per chain
    int L;
    double lnu;
    if constexpr (REPLAY) {
      L = live ? a.rL[c * (int64_t)a.niter + (it - 1)] : 0;
      lnu = live ? a.rlnu[c * (int64_t)a.niter + (it - 1)] : 0.0;
    } else {
      const uint4 r = draw_block(kDrawSlot, (uint32_t)it, gc, a.k0, a.k1);
      L = live ? uniform_int(r.x, a.L_low, a.L_high) : 0;
      const double u = u53(r.z, r.w);
      lnu = u > 0.0 ? fast_log(u) : -__builtin_inf();   // log(random()), :461 (ocml log keeps its
                                                        // constants in VGPRs across the loop)
    }
    int Lmax = L;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) Lmax = max(Lmax, __shfl_xor(Lmax, off, kWave));
    Lmax = uniform_i(Lmax);
    // ---- leapfrog (:448 -> :831-839); chains with l >= L are frozen
    const bool cap = cap_wave && it <= a.n_save;
    double* capp = cap ? a.traj_q + (int64_t)(it - 1) * a.traj_stride * 2 : nullptr;
    if (cap) {   // dims 0 and 1 of chain 0 live in lanes 0 (h=0) and 16 (h=1)
      const double q1 = __shfl(q[0], 16, kWave);
      if (lane == 0) {
        capp[0] = q[0];
        capp[1] = a.D > 1 ? q1 : q[0];
      }
    }
    for (int l = 0; l < Lmax; ++l) {
      // chains with l >= L are frozen by the EXEC mask of a divergent block (no per-dim selects;
      // with L-ordered tiles the mask is nearly always full).  The MFMAs run with all lanes.
      const bool act = l < L;
      if (act) {
#pragma unroll
        for (int m = 0; m < ME; ++m) {
          const int d = h + 4 * m;
          const double dt = dim_dt<MT, GEN>(a, d);
          const double mi = dim_minv<MT, GEN>(a, d);
          if constexpr (EXACT) {
            p[m] = p[m] - (dt * (mi * gval<MT>(acc, m))) * 0.5;
            q[m] = q[m] + dt * p[m];
          } else {
            p[m] = __builtin_fma(-0.5 * dt * mi, gval<MT>(acc, m), p[m]);
            q[m] = __builtin_fma(dt, p[m], q[m]);
          }
          if ((m & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
      }
      gradient<MT, GEN, kDenseDB<WAVES>, SHORT>(a, sP, lane, h, q, acc);
      if (act) {
#pragma unroll
        for (int m = 0; m < ME; ++m) {
          const int d = h + 4 * m;
          const double dt = dim_dt<MT, GEN>(a, d);
          const double mi = dim_minv<MT, GEN>(a, d);
          if constexpr (EXACT) p[m] = p[m] - (dt * (mi * gval<MT>(acc, m))) * 0.5;
          else p[m] = __builtin_fma(-0.5 * dt * mi, gval<MT>(acc, m), p[m]);
          if ((m & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (cap) {
        const double q1 = __shfl(q[0], 16, kWave);
        if (lane == 0 && l < L) {
          capp[2 * (l + 1)] = q[0];
          capp[2 * (l + 1) + 1] = a.D > 1 ? q1 : q[0];
        }
      }
    }
    // ---- E1 with the gradient of the final q, Metropolis test (:455-472)
    maha = 0.0;
    kin = 0.0;
    energy_terms(maha, kin);
    const double E1 = 0.5 * (a.logc + chain_sum4(maha + kin));
    const double dE = E1 - E0;
    const bool accept = (dE < 0.0) || (lnu < -dE);
#pragma unroll
    for (int m = 0; m < ME; ++m) {
      if (live && dim_ok(m)) {
        if (accept) qh[4 * m] = q[m];
        else q[m] = qh[4 * m];
      }
    }
    if (gch && live && accept) {      // the gradient at the new q (a rejection keeps the cached one)
#pragma unroll
      for (int m = 0; m < ME; ++m)
        if (dim_ok(m)) gch[4 * m] = gval<MT>(acc, m);
    }
    if (live && write_row && qcb && row >= a.q_row0) {
      double* rowp = qcb + (row % a.Lq) * a.D + h;
#pragma unroll
      for (int m = 0; m < ME; ++m) {
        if (dim_ok(m)) __builtin_nontemporal_store(q[m], rowp + 4 * m);   // sample row: written once
      }
    }
    if (cap && lane == 0) {
      a.traj_len[it - 1] = (L > 0 ? L : 0) + 1;
      a.decision[it - 1] = accept ? 1 : 0;
    }
    if (live && h == 0) {
      if (accept) {
        if (post) ++n_acc; else ++n_acc_wu;
      } else if (it < a.i_oob) {
        ++n_oob;
      }
      const unsigned long long Lp = L > 0 ? (unsigned long long)L : 0ull;
      n_lf += Lp;
      n_lf2 += Lp * Lp;
    }
  }
  if (live && h == 0) a.Eprev[c] = Eprev;
  }   // tile loop
  n_acc = wave_sum_u64(n_acc);
  n_acc_wu = wave_sum_u64(n_acc_wu);
  n_lf = wave_sum_u64(n_lf);
  n_lf2 = wave_sum_u64(n_lf2);
  n_oob = wave_sum_u64(n_oob);
  if (lane == 0 && a.cnt) {
    unsigned long long* cs = a.cnt + (wave_id & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
    if (n_acc) atomicAdd(cs + HMC_CNT_ACCEPT, n_acc);
    if (n_acc_wu) atomicAdd(cs + HMC_CNT_ACCEPT_WU, n_acc_wu);
    if (n_lf) atomicAdd(cs + HMC_CNT_LEAPFROG, n_lf);
    if (n_lf2) atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, n_lf2);
    if (n_oob) atomicAdd(cs + HMC_CNT_OOB_REJECT, n_oob);
  }
}

// p0 . inv(cov_p) . p0 of the initial momentum with a dense mass matrix (samplers.py:415-416):
// p0 = C z with z in the dims' Philox mapping (or the replayed p0).  One thread per chain, O(D^2).
template <bool REPLAY>
__device__ double dense_mass_kinetic0(const DenseArgs& a, int64_t c, uint64_t gc, int MT) {
  const int D = a.D;
  double p0[128];   // D <= 128 (dense_tiles)
  for (int d = 0; d < D; ++d) p0[d] = 0.0;
  if constexpr (REPLAY) {
    for (int d = 0; d < D; ++d) p0[d] = a.rp0[c * D + d];
  } else {
    double z[128];
    const int M = 4 * MT;
    for (int h = 0; h < 4; ++h)
      for (int m = 0; m < M; m += 2) {
        const int d0 = h + 4 * m, d1 = d0 + 4;
        double z0, z1;
        normal_pair(draw_block((uint32_t)(h + 4 * m), 0u, gc, a.k0, a.k1), z0, z1);
        if (d0 < D) z[d0] = z0;
        if (d1 < D) z[d1] = z1;
      }
    for (int r = 0; r < D; ++r) {
      double acc = 0.0;
      for (int k = 0; k <= r; ++k) acc = __builtin_fma(a.cholt[(int64_t)k * D + r], z[k], acc);   // C[r][k]
      p0[r] = acc;
    }
  }
  double kin = 0.0;
  for (int r = 0; r < D; ++r) {
    double mp = 0.0;
    for (int k = 0; k < D; ++k) mp = __builtin_fma(a.minvf[(int64_t)r * D + k], p0[k], mp);
    kin += p0[r] * mp;
  }
  return kin;
}

// Chain initialisation for dense targets (samplers.py:413-420), one thread per chain.
template <bool REPLAY>
__global__ __launch_bounds__(256) void k_dense_init(DenseArgs a, int MT) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n) return;
  const double* qs = a.qstart + c * a.D;
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  double maha = 0.0, kin = 0.0;
  for (int n = 0; n < a.D; ++n) {
    double g = 0.0;
    for (int k = 0; k < a.D; ++k) g = __builtin_fma(a.prec[(int64_t)n * a.D + k], qs[k] - (a.q0 ? a.q0[k] : 0.0), g);
    maha += (qs[n] - (a.q0 ? a.q0[n] : 0.0)) * g;
  }
  // momentum p0 with the dense kernel's Philox mapping (dims h + 4m, pair slot h + 4m, m even)
  const int M = 4 * MT;
  for (int h = 0; h < 4; ++h) {
    for (int m = 0; m < M; m += 2) {
      const int d0 = h + 4 * m, d1 = d0 + 4;
      double z0, z1;
      if constexpr (REPLAY) {
        z0 = d0 < a.D ? a.rp0[c * a.D + d0] : 0.0;
        z1 = d1 < a.D ? a.rp0[c * a.D + d1] : 0.0;
      } else {
        normal_pair(draw_block((uint32_t)(h + 4 * m), 0u, gc, a.k0, a.k1), z0, z1);
        if (a.pscale) {
          z0 = d0 < a.D ? z0 * a.pscale[d0] : 0.0;
          z1 = d1 < a.D ? z1 * a.pscale[d1] : 0.0;
        }
      }
      if (a.minvf) continue;   // dense mass: K from the whole vector below
      if (d0 < a.D) kin += z0 * ((a.minv ? a.minv[d0] : 1.0) * z0);
      if (d1 < a.D && m + 1 < M) kin += z1 * ((a.minv ? a.minv[d1] : 1.0) * z1);
    }
  }
  if (a.minvf) kin = dense_mass_kinetic0<REPLAY>(a, c, gc, MT);
  const double E0 = 0.5 * (a.logc + (maha + kin));
  for (int d = 0; d < a.D; ++d) {
    a.q[c * a.D + d] = qs[d];
    if (a.qc && a.q_row0 == 0) a.qc[c * (int64_t)a.Lq * a.D + d] = qs[d];
  }
  a.Eprev[c] = E0;
  if (a.Ec) a.Ec[c * (int64_t)a.Lc] = E0;
  if (a.dEc) a.dEc[c * (int64_t)a.Lc] = 0.0;
}

// ---- L-ordered tiles (one iteration per launch): counting sort of the chains by this
// iteration's trajectory length, so each 16-chain tile runs (nearly) one L.  The draws are the
// ones k_dense_iters makes (samplers.py:441); the order only decides which lanes a chain
// occupies, never a value it computes.
constexpr int kOrderBins = 256;

__device__ __forceinline__ int dense_bin(const DenseArgs& a, int64_t c, int it, bool replay) {
  int L;
  if (replay) {
    L = a.rL[c * (int64_t)a.niter + (it - 1)];
  } else {
    const uint4 r = draw_block(kDrawSlot, (uint32_t)it, (uint64_t)(a.chain_offset + c), a.k0, a.k1);
    L = uniform_int(r.x, a.L_low, a.L_high);
  }
  return min(max(L - a.L_low, 0), a.L_high - a.L_low - 1);
}

__global__ __launch_bounds__(256) void k_order_hist(DenseArgs a, int it, bool replay, int32_t* hist) {
  __shared__ int cnt[kOrderBins];
  const int nb = a.L_high - a.L_low;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < a.n) atomicAdd(&cnt[dense_bin(a, c, it, replay)], 1);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (cnt[b]) atomicAdd(&hist[b], cnt[b]);
}

__global__ __launch_bounds__(256) void k_order_scatter(DenseArgs a, int it, bool replay, const int32_t* hist,
                                                       int32_t* cursor, int32_t* order) {
  __shared__ int cnt[kOrderBins], base[kOrderBins];
  const int nb = a.L_high - a.L_low;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int bin = 0, rank = 0;
  if (c < a.n) {
    bin = dense_bin(a, c, it, replay);
    rank = atomicAdd(&cnt[bin], 1);
  }
  if (threadIdx.x == 0) {            // exclusive prefix of the global histogram
    int run = 0;
    for (int b = 0; b < nb; ++b) {
      base[b] = run;
      run += hist[b];
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (cnt[b]) base[b] += atomicAdd(&cursor[b], cnt[b]);
  __syncthreads();
  if (c < a.n) order[base[bin] + rank] = (int32_t)c;
}


template <int MT, bool EXACT, int WAVES>
void launch_dense_w(const DenseArgs& a, bool gen, bool replay, hipStream_t s) {
  // one block per CU (the LDS copy of P limits residency to one), persistent over the tiles
  const int64_t blocks = (a.ntiles + WAVES - 1) / WAVES;
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)device_cus())));
  const size_t lds = (size_t)MT * 4 * MT * kWave * sizeof(double);
  if (a.minvf) {
    if (replay) k_dense_iters<MT, EXACT, true, true, WAVES, true><<<grid, 64 * WAVES, lds, s>>>(a);
    else k_dense_iters<MT, EXACT, true, false, WAVES, true><<<grid, 64 * WAVES, lds, s>>>(a);
  } else if (gen) {
    if (replay) k_dense_iters<MT, EXACT, true, true, WAVES><<<grid, 64 * WAVES, lds, s>>>(a);
    else k_dense_iters<MT, EXACT, true, false, WAVES><<<grid, 64 * WAVES, lds, s>>>(a);
  } else {
    bool done = false;
    if constexpr (MT == 7) {
      if (a.D <= 16 * (MT - 1) + 4) {                   // D = 97..100 (c3: D = 100)
        if (replay) k_dense_iters<MT, EXACT, false, true, WAVES, false, kShortAlways><<<grid, 64 * WAVES, lds, s>>>(a);
        else k_dense_iters<MT, EXACT, false, false, WAVES, false, kShortAlways><<<grid, 64 * WAVES, lds, s>>>(a);
        done = true;
      }
    }
    if (!done) {
      if (replay) k_dense_iters<MT, EXACT, false, true, WAVES, false, kShortNever><<<grid, 64 * WAVES, lds, s>>>(a);
      else k_dense_iters<MT, EXACT, false, false, WAVES, false, kShortNever><<<grid, 64 * WAVES, lds, s>>>(a);
    }
  }
}

template <int MT, bool EXACT>
hipError_t launch_dense_mt2(const DenseArgs& a, bool gen, bool replay, hipStream_t s) {
  launch_dense_w<MT, EXACT, HMC_DENSE_WAVES>(a, gen, replay, s);
  return hipGetLastError();
}

template <int MT>
hipError_t launch_dense_mt(const DenseArgs& a, bool exact, bool gen, bool replay, hipStream_t s) {
  return exact ? launch_dense_mt2<MT, true>(a, gen, replay, s) : launch_dense_mt2<MT, false>(a, gen, replay, s);
}

}  // namespace

int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int v = 0;
    cache[dev] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v
                                                                                                                : 256;
  }
  return cache[dev];
}

int dense_tiles(int D) {
  const int mt = (D + 15) / 16;
  if (mt <= 1) return 1;
  if (mt <= 2) return 2;
  if (mt <= 4) return 4;
  if (mt <= 7) return 7;
  if (mt <= 8) return 8;
  return 0;
}

hipError_t launch_dense_init(const DenseArgs& a, bool replay, hipStream_t s) {
  const dim3 grid((unsigned)((a.n + 255) / 256));
  const int MT = dense_tiles(a.D);
  if (replay) k_dense_init<true><<<grid, 256, 0, s>>>(a, MT);
  else k_dense_init<false><<<grid, 256, 0, s>>>(a, MT);
  return hipGetLastError();
}

int64_t dense_order_ints(int64_t n) { return n + 2 * kOrderBins; }
int64_t dense_gcache_offset_bytes(int64_t n) { return ((dense_order_ints(n) * 4 + 15) / 16) * 16 + 16; }
int64_t dense_workspace_bytes(int64_t n, int D) { return dense_gcache_offset_bytes(n) + n * (int64_t)D * 8; }

bool dense_order_ok(const DenseArgs& a) { return a.L_high - a.L_low <= kOrderBins && a.n < (1ll << 31); }

hipError_t launch_dense_order(const DenseArgs& a, int it, bool replay, int32_t* ws, hipStream_t s) {
  int32_t* hist = ws + a.n;
  int32_t* cursor = hist + kOrderBins;
  if (hipError_t e = hipMemsetAsync(hist, 0, 2 * kOrderBins * sizeof(int32_t), s)) return e;
  const dim3 grid((unsigned)((a.n + 255) / 256));
  k_order_hist<<<grid, 256, 0, s>>>(a, it, replay, hist);
  k_order_scatter<<<grid, 256, 0, s>>>(a, it, replay, hist, cursor, ws);
  return hipGetLastError();
}

hipError_t launch_dense_iters(const DenseArgs& a, bool exact, bool replay, hipStream_t s) {
  const bool gen = a.q0 || a.minv || a.pscale || a.dtv || a.minvf;
  switch (dense_tiles(a.D)) {
    case 1: return launch_dense_mt<1>(a, exact, gen, replay, s);
    case 2: return launch_dense_mt<2>(a, exact, gen, replay, s);
    case 4: return launch_dense_mt<4>(a, exact, gen, replay, s);
    case 7: return launch_dense_mt<7>(a, exact, gen, replay, s);
    case 8: return launch_dense_mt<8>(a, exact, gen, replay, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace hmc
