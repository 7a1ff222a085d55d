// hmc_wave.hip — wave-per-chain Random-trajectory HMC kernel (diagonal-precision MVN, D > 64).
//
// Same semantics as k_random_iters (hmc_random.hip; samplers.py:428-475) with the layout the
// north star asks for: ONE wavefront per chain.  Lane l owns coordinate pairs l + 64*j.
// Everything that is per chain is wave-uniform, which the kernel exploits:
//   * trajectory length L and the MH log-uniform are SGPR values, so the leapfrog loop is a
//     scalar loop (no EXEC juggling) and the accept/reject is a scalar branch;
//   * energies are full-wave DPP reductions (row_shr/row_bcast, no LDS), read back with
//     v_readlane as SGPRs;
//   * one reduction per iteration: the final energy E1 of iteration i is reduced together
//     with the kinetic energy of iteration i+1's momentum (drawn before the MH test, its
//     draw is keyed by i+1 so the order of work does not change any value), and the potential
//     part of E0(i+1) is V(q) already known from E1 (accepted) or E0 (rejected);
//   * E_chain / dE_chain values of up to 64 iterations are parked one per lane and written
//     as one coalesced store (rows of a chain are contiguous).
// HBM traffic per chain-iteration: one q_chain row (8D B) + E + dE (16 B).
#include "hmc_device.hpp"
#include "hmc_internal.hpp"
#include "hmc_target_ops.hpp"

namespace hmc {

namespace {

template <int K, bool GEN>
__device__ __forceinline__ void wave_partials(const RandArgs& a, const int (&kk)[K], const bool (&pv)[K],
                                              const double (&q)[2 * K], const double (&p)[2 * K], double& maha,
                                              double& kin) {
  maha = 0.0;
  kin = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if constexpr (!GEN) {   // padding slots hold q = p = 0 (loads, draws and the integrator keep
                            // them zero), so they add exact zeros: no masks
      energy_terms<GEN>(DimConst{}, q[2 * j], p[2 * j], maha, kin);
      energy_terms<GEN>(DimConst{}, q[2 * j + 1], p[2 * j + 1], maha, kin);
    } else if (pv[j]) {
      const int d = 2 * kk[j];
      energy_terms<GEN>(dim_const<GEN>(a, d), q[2 * j], p[2 * j], maha, kin);
      if (d + 1 < a.D) energy_terms<GEN>(dim_const<GEN>(a, d + 1), q[2 * j + 1], p[2 * j + 1], maha, kin);
    }
  }
}

// FAST (non-EXACT) diagonal-identity partials as FMA chains: x.x and x.x + p.p of this lane's
// coordinates (the reference sums V and K separately; FAST only promises agreement to 1e-10).
template <int K>
__device__ __forceinline__ void wave_partials_fma(const double (&q)[2 * K], const double (&p)[2 * K], double& maha,
                                                  double& tot) {
  maha = q[1] * q[1];
  maha = __builtin_fma(q[0], q[0], maha);
#pragma unroll
  for (int j = 1; j < K; ++j) {
    maha = __builtin_fma(q[2 * j], q[2 * j], maha);
    maha = __builtin_fma(q[2 * j + 1], q[2 * j + 1], maha);
  }
  tot = maha;
#pragma unroll
  for (int e = 0; e < 2 * K; ++e) tot = __builtin_fma(p[e], p[e], tot);
}

template <int K, bool GEN>
__device__ __forceinline__ double kin_partial(const RandArgs& a, const int (&kk)[K], const bool (&pv)[K],
                                              const double (&p)[2 * K]) {
  double kin = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if constexpr (!GEN) {   // zero padding slots, as in wave_partials
      kin += p[2 * j] * p[2 * j];
      kin += p[2 * j + 1] * p[2 * j + 1];
    } else if (pv[j]) {
      const int d = 2 * kk[j];
      const DimConst c0 = dim_const<GEN>(a, d);
      kin += GEN ? p[2 * j] * (c0.minv * p[2 * j]) : p[2 * j] * p[2 * j];
      if (d + 1 < a.D) {
        const DimConst c1 = dim_const<GEN>(a, d + 1);
        kin += GEN ? p[2 * j + 1] * (c1.minv * p[2 * j + 1]) : p[2 * j + 1] * p[2 * j + 1];
      }
    }
  }
  return kin;
}

template <int K, bool GEN, bool REPLAY>
__device__ __forceinline__ void wave_momentum(const RandArgs& a, int64_t c, uint64_t gc, int it, const int (&kk)[K],
                                              const bool (&pv)[K], double (&p)[2 * K], const double* tab) {
  const bool even = (a.D & 1) == 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    p[2 * j] = 0.0;
    p[2 * j + 1] = 0.0;
    if (pv[j]) {
      const int d = 2 * kk[j];
      if constexpr (REPLAY) {
        const double* row = a.rp + (c * (int64_t)a.niter + (it - 1)) * a.D;
        load_pair(row, kk[j], even, d + 1 < a.D, p[2 * j], p[2 * j + 1]);
      } else {
        normal_pair_tab(draw_block_uc((uint32_t)kk[j], (uint32_t)it, gc, a.k0, a.k1), tab, p[2 * j], p[2 * j + 1]);
        if (GEN && a.pscale) {
          p[2 * j] *= a.pscale[d];
          if (d + 1 < a.D) p[2 * j + 1] *= a.pscale[d + 1];
        }
      }
      if (d + 1 >= a.D) p[2 * j + 1] = 0.0;
    }
  }
}

// K = 1 blocks hold 16 waves (16 chains): the Box–Muller tables are built once per 16 chains
// and a launch dispatches a quarter of the workgroups.
constexpr int kK1Block = 1024;

// Momentum ring (K = 1, Philox): at D <= 128 a chain's npairs = ceil(D/2) coordinate pairs leave
// 64 - npairs lanes idle (14 of 64 at D = 100), and the momentum draws (Philox4x32-10 +
// Box–Muller, ~95 VALU per pass) are the largest part of an iteration.  The wave instead draws
// 64 consecutive pairs per pass on ALL lanes into a per-wave LDS ring (pair g of the launch in
// slot g % kRingPairs) and every iteration reads its npairs pairs back: npairs/64 passes per
// iteration instead of one.  Pair k of iteration it is still keyed (k, it, chain), so every value
// is the one the per-lane scheme draws (independent of launch splits and of the ring).
constexpr int kRingPairs = 128;

// FULL: chain-0 trajectory capture and the ablation/debug hooks compiled in.  The production
// variant (FULL = false) drops them: their pointers and flags are live across the iteration loop
// and pushed the SGPR demand past the 8-waves/SIMD budget (spills to VGPR lanes cost one
// v_readlane/v_writelane VALU slot each, ~45 per iteration).
// ODD: D is odd (the ring zeroes the missing coordinate of the last pair); a template parameter so
// that the common even-D kernel carries no per-pass test.
template <int K, bool EXACT, bool GEN, bool REPLAY, bool FULL, bool ODD = false>
__device__ __forceinline__ void wave_iters(const RandArgs& a) {
#ifdef HMC_NO_RING
  constexpr bool RING = false;
#else
  constexpr bool RING = K == 1 && !REPLAY;
#endif
  __shared__ double s_ntab[REPLAY ? 2 : kNormalTableDoubles];   // Box–Muller tables (Philox mode)
  // per wave: kRingPairs ring slots (2 KB, 2 KB-aligned: a slot's byte address is the wave's base
  // OR'd with 16 * slot)
  __shared__ __attribute__((aligned(2048))) double s_ring[RING ? (kK1Block / kWave) * 2 * kRingPairs : 2];
  if constexpr (!REPLAY) {
    init_normal_tables(s_ntab);
    __syncthreads();
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave));
  if (c >= a.n) return;                                  // whole wave, uniform
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  const uint32_t ring_off = RING ? (threadIdx.x / kWave) * (16 * kRingPairs) : 0;   // bytes, 2 KB multiple
  char* const ring_b = reinterpret_cast<char*>(s_ring);
  char* const ring_lane = ring_b + ring_off + 16 * lane;   // this lane's slot in a pass's half
  // Generator position: pairs drawn so far (wave-uniform) and this lane's (pair, iteration) for the
  // next pass.  npairs is in (32, 64] for the wave kernel, so one pass of 64 pairs advances a lane
  // by one or two whole iterations: the position is kept incrementally instead of re-derived.
  int gen_n = 0;
  uint32_t gk = lane, git = a.it0;
  if (gk >= (uint32_t)a.npairs) { gk -= a.npairs; ++git; }
  const uint32_t gadv = kWave - a.npairs;                // uniform: a pass moves a lane 64 pairs on
  // momentum of iteration `it` through the ring: at most one 64-pair pass is due (the pairs drawn
  // so far cover every earlier iteration and npairs <= 64), and the ring never holds more than
  // npairs + 64 <= kRingPairs pairs that are not consumed yet
  auto ring_momentum = [&](int it, double (&pp)[2 * K]) {
    const int base = (it - a.it0) * a.npairs;
    if (gen_n < base + a.npairs) {                       // wave-uniform
      double z0, z1;
      normal_pair_tab(draw_block_uc(gk, git, gc, a.k0, a.k1), s_ntab, z0, z1);
      if constexpr (ODD) z1 = gk == (uint32_t)a.npairs - 1 ? 0.0 : z1;   // dimension D does not exist
      // pass slots gen_n + lane (mod 128) = lane + (gen_n & 64): gen_n is a multiple of 64
      *reinterpret_cast<double2*>(ring_lane + 16 * (gen_n & kWave)) = make_double2(z0, z1);
      __builtin_amdgcn_wave_barrier();
      gen_n += kWave;
      // next pass: gk += 64 - npairs, then one more wrap (git + 2) or none (git + 1); four VALU:
      // the borrow of gk - npairs picks both the new gk and git's increment
      uint64_t bo;
      uint32_t t;
      asm("v_add_u32_e32 %0, %4, %0\n\t"
          "v_subrev_co_u32_e32 %2, vcc, %5, %0\n\t"
          "v_subb_co_u32_e64 %1, %3, %1, -2, vcc\n\t"
          "v_cndmask_b32_e32 %0, %2, %0, vcc"
          : "+v"(gk), "+v"(git), "=&v"(t), "=&s"(bo)
          : "s"(gadv), "s"(a.npairs)
          : "vcc");
    }
    // lanes past npairs sit the read out (EXEC off): their p is never written and stays 0
    if (lane < a.npairs) {
      const uint32_t slot_b = (((uint32_t)(base + lane) << 4) & (16 * kRingPairs - 1)) | ring_off;
      const double2 z = *reinterpret_cast<const double2*>(ring_b + slot_b);
      pp[0] = z.x;
      pp[1] = z.y;
      if (GEN && a.pscale) {
        const int d = 2 * lane;
        pp[0] *= a.pscale[d];
        if (d + 1 < a.D) pp[1] *= a.pscale[d + 1];
      }
    }
  };
  // the ring (Philox, K = 1) kernels are specialised on the parity of D: `even` is then a
  // compile-time constant and the row stores need no masks (SGPR pressure: no spilled flags)
  const bool even = RING ? !ODD : (a.D & 1) == 0;
  int kk[K];
  bool pv[K];
  double q[2 * K], p[2 * K], qi[2 * K], pn[2 * K];
  double* const qrow = a.q + c * (int64_t)a.D;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    kk[j] = lane + kWave * j;
    pv[j] = kk[j] < a.npairs;
    q[2 * j] = q[2 * j + 1] = 0.0;
    p[2 * j] = p[2 * j + 1] = 0.0;      // the ring leaves lanes past npairs at p = 0
    pn[2 * j] = pn[2 * j + 1] = 0.0;
    if (pv[j]) load_pair(qrow, kk[j], even, 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
  }
  double Eprev = a.Eprev[c];
  __builtin_amdgcn_s_waitcnt(0x0F70);                    // retire state loads before the loop (vmcnt(0))

  // momentum and energy of the first iteration of this launch
  if constexpr (RING) ring_momentum(a.it0, p);
  else wave_momentum<K, GEN, REPLAY>(a, c, gc, a.it0, kk, pv, p, s_ntab);
  // FASTID: FAST integrator on an identity-precision target (the headline instantiation): FMA
  // energy partials and ONE reduction per iteration.  The lane's part of 2 E0 - logc (e0l, known
  // when the iteration starts) and of 2 (E1 - E0) (its q.q + p.p after the leapfrog minus e0l)
  // are summed together by wave_sum2_dpp: lane 31 holds 2 dE for the Metropolis test, lane 63
  // 2 E0 - logc for E_chain.  E = fma(sum, 1/2, logc/2); dE is summed directly (no cancellation
  // of two ~D-sized energies), which FAST mode's 1e-10 contract allows.
  constexpr bool FASTID = !EXACT && !GEN;
  const double hlogc = 0.5 * a.logc;
  double m0, k0, m0l;   // m0l: this lane's part of the potential of q (FAST mode bookkeeping)
  double e0l = 0.0;     // FASTID: this lane's part of q.q + p.p at the iteration start
  if constexpr (FASTID) {
    wave_partials_fma<K>(q, p, m0l, e0l);
    m0 = m0l;
    k0 = 0.0;
  } else {
    wave_partials<K, GEN>(a, kk, pv, q, p, m0, k0);
    m0l = m0;
  }
  if constexpr (EXACT) {   // reference grouping: V and K summed separately
    m0 = wave_sum_dpp(m0);
    k0 = wave_sum_dpp(k0);
  } else if constexpr (!FASTID) {   // one reduction of V + K
    k0 = wave_sum_dpp(m0 + k0);
  }
  // (FASTID: E0 of an iteration is formed inside it, by that iteration's one reduction)
  double E0 = EXACT ? 0.5 * (a.logc + (m0 + k0)) : (FASTID ? 0.0 : 0.5 * (a.logc + k0));

  // thinning bookkeeping without divisions: row = (it - wu)//thin, phase = (it - wu) % thin
  int row = 0, phase = 0;
  if (a.it0 >= a.wu) {
    row = (a.it0 - a.wu) / a.thin;
    phase = (a.it0 - a.wu) - row * a.thin;
  }
  int qslot = row % a.Lq;                                // q_chain buffer row of `row` (circular window)
  double Ebuf = 0.0, dEbuf = 0.0;
  int row_first = 0, nbuf = 0;
  const bool thin1 = a.thin == 1;
  const int bp63 = (int)opaque_u32((kWave - 1) * 4);     // park_lane's source lane (byte address)
  double* const Ec = a.Ec ? a.Ec + c * (int64_t)a.Lc : nullptr;
  double* const dEc = a.dEc ? a.dEc + c * (int64_t)a.Lc : nullptr;
  double* const qcb = a.qc ? a.qc + c * (int64_t)a.Lq * a.D : nullptr;
  auto flush_E = [&](int n) {          // rows row_first .. row_first + n - 1 from lanes 0 .. n-1
    double dE = dEbuf;
    if (thin1) {
      const double before = __shfl_up(Ebuf, 1, kWave);
      dE = lane == 0 ? dEbuf : Ebuf - before;   // lane 0: parked when the block began
    }
    if (lane < n) {
      if (Ec) __builtin_nontemporal_store(Ebuf, Ec + row_first + lane);
      if (dEc) __builtin_nontemporal_store(dE, dEc + row_first + lane);
    }
  };
  const bool cap_chain = FULL && a.traj_q && gc == 0 && !(a.dbg & 32);
  // per-launch tallies of one chain: (it1 - it0) <= 2^31 / L_high^2 is checked on the host, so
  // 32-bit counters cannot wrap (half the SGPRs of 64-bit ones)
  uint32_t n_acc = 0, n_acc_wu = 0, n_lf = 0, n_lf2 = 0, n_oob = 0;
  int it_base = a.it0 - kWave, draw_L = 0;
  double draw_lnu = 0.0;

  // One iteration; POST (it >= warm_up) is a compile-time constant: the launch runs the warm-up
  // iterations and the sampling iterations as two loops, so the per-iteration tests of `post`
  // (row writes, tallies, thinning) fold away.
  auto iteration = [&](auto post_c, int it) {
    constexpr bool post = decltype(post_c)::value;
    const bool write_row = post && ((it == a.niter) || (phase == a.thin - 1));
    // E_chain / dE_chain of this iteration parked in lane nbuf (flushed every 64 or at the end);
    // E (and Eprev) need only be valid in lane 63, where the DPP reductions leave them.
    // Parked rows are consecutive (row_first + lane).  With thin = 1 they are also consecutive
    // iterations, so dE = E(lane) - E(lane - 1) is formed at the flush (lane 0: the E before the
    // block) and only E is parked; otherwise dE is parked too.
    // Eprev (the E of the previous iteration) is only needed for a block's first row when
    // thin = 1: it is then refreshed at each flush instead of every iteration.
    // (the empty asm statements keep these uniform conditions as branches, not per-lane selects)
    // FASTID parks after the iteration's reduction has formed E0; the other modes know E0 here.
    auto park_row = [&]() {
      if (write_row) {
        if (nbuf == 0) {
          asm volatile("" ::: "memory");
          row_first = row;
          // thin = 1: the block's first dE (its E minus the E before the block) in lane 0 of
          // dEbuf; the flush forms the others from consecutive parked E
          if (thin1) dEbuf = park_lane(dEbuf, E0 - Eprev, 0, bp63);
        }
        Ebuf = park_lane(Ebuf, E0, nbuf, bp63);
        if (!thin1) {
          asm volatile("" ::: "memory");
          dEbuf = park_lane(dEbuf, E0 - Eprev, nbuf, bp63);
        }
        if (++nbuf == kWave) {
          flush_E(kWave);
          nbuf = 0;
          if (thin1) Eprev = E0;
        }
        if (!thin1) {
          asm volatile("" ::: "memory");
          Eprev = E0;
        }
      } else {
        Eprev = E0;
      }
    };
    if constexpr (!FASTID) park_row();

    // trajectory length (:441) and MH log-uniform (:461): wave-uniform
    int L;
    double lnu;
    if constexpr (REPLAY) {
      L = a.rL[c * (int64_t)a.niter + (it - 1)];
      lnu = a.rlnu[c * (int64_t)a.niter + (it - 1)];
      if constexpr (FASTID) lnu *= 2.0;                  // compared with 2 dE (exact scaling)
    } else {
      if (it - it_base >= kWave) {                       // lane l draws (L, u) of iteration it + l
        it_base = it;
        const uint4 r = draw_block_uc(kDrawSlot, (uint32_t)(it + lane), gc, a.k0, a.k1);
        draw_L = uniform_int(r.x, a.L_low, a.L_high);
        const double u = u53(r.z, r.w);
        draw_lnu = u > 0.0 ? fast_log(u) : -__builtin_inf();   // log(random()), :461
        if constexpr (FASTID) draw_lnu *= 2.0;           // compared with 2 dE (exact scaling)
      }
      L = __builtin_amdgcn_readlane(draw_L, it - it_base);
      lnu = readlane_d(draw_lnu, it - it_base);
    }
    if (FULL && a.dbgL >= 0) L = a.dbgL;                          // diagnostics: forced trajectory length
    L = uniform_i(L);

    // chain-0 trajectory capture (samplers.py:442-452)
    const bool cap = cap_chain && it <= a.n_save;
    double* capp = cap ? a.traj_q + (int64_t)(it - 1) * a.traj_stride * 2 : nullptr;
    if (cap && lane == 0) {
      capp[0] = q[0];
      capp[1] = a.D > 1 ? q[1] : q[0];
    }

    // L leapfrog steps (samplers.py:448 -> :831-839), scalar loop
    // the start point's copy as an opaque move: the integrated q (not the copy) is then the value
    // carried to the next iteration, and the back edge needs no moves
#pragma unroll
    for (int e = 0; e < 2 * K; ++e) asm("v_mov_b64 %0, %1" : "=v"(qi[e]) : "v"(q[e]));
    if constexpr (EXACT) {
      double t[2 * K];
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
            const DimConst cc = slot_const<GEN>(a, kk[j], h, pv[j]);
            const double ph = p[e] - t[e];
            q[e] = q[e] + cc.dt * ph;
            t[e] = kick<GEN>(cc, q[e]);
            p[e] = ph - t[e];
          }
        }
        if (cap && lane == 0) {
          capp[2 * (l + 1)] = q[0];
          capp[2 * (l + 1) + 1] = a.D > 1 ? q[1] : q[0];
        }
      }
    } else if (L > 0 && (K > 1 || lane < a.npairs)) {
      // (K = 1: lanes past npairs hold q = p = 0 and sit the integration out with EXEC off --
      // the kernel runs at the board power cap, and idle FP64 lanes cost power, not time)
      // FAST: consecutive half kicks merged into one full kick, in shifted coordinates
      // u = q - q0 (2 FMA per coordinate per step instead of 3; same integrator, other rounding)
      // (without q0 the shift is the identity: integrate q in place, no copies in and out)
      double ubuf[GEN ? 2 * K : 1], dtc[2 * K], kh[2 * K], kfull[2 * K];
      double (&u)[2 * K] = *reinterpret_cast<double(*)[2 * K]>(GEN ? ubuf : q);
#pragma unroll
      for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * j + h;
          const DimConst cc = slot_const<GEN>(a, kk[j], h, pv[j]);
          kh[e] = -(GEN ? cc.hd * (cc.minv * cc.prec) : cc.hd);
          kfull[e] = 2.0 * kh[e];
          dtc[e] = cc.dt;
          if constexpr (GEN) u[e] = q[e] - cc.q0;
          p[e] = __builtin_fma(kh[e], u[e], p[e]);          // first half kick
        }
      }
      auto capture = [&](int l) {
        if (cap && lane == 0) {
          const double x0 = GEN ? u[0] + slot_const<GEN>(a, 0, 0, true).q0 : u[0];
          const double x1 = a.D > 1 ? (GEN ? u[1] + slot_const<GEN>(a, 0, 1, true).q0 : u[1]) : x0;
          capp[2 * (l + 1)] = x0;
          capp[2 * (l + 1) + 1] = x1;
        }
      };
      for (int l = 0; l + 1 < L; ++l) {
#pragma unroll
        for (int e = 0; e < 2 * K; ++e) {
          u[e] = __builtin_fma(dtc[e], p[e], u[e]);         // drift
          p[e] = __builtin_fma(kfull[e], u[e], p[e]);       // two half kicks merged
        }
        capture(l);
      }
#pragma unroll
      for (int e = 0; e < 2 * K; ++e) {
        u[e] = __builtin_fma(dtc[e], p[e], u[e]);           // last drift
        p[e] = __builtin_fma(kh[e], u[e], p[e]);            // last half kick
      }
      capture(L - 1);
      if constexpr (GEN) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = 2 * j + h;
            q[e] = u[e] + slot_const<GEN>(a, kk[j], h, pv[j]).q0;
          }
        }
      }
    }

    // FASTID: E1's partials and the iteration's one reduction first; p is then dead, so the next
    // momentum is drawn into p itself (no copy at the end of the iteration)
    double m1 = 0.0, k1 = 0.0, m1l = 0.0, s2 = 0.0;
    if constexpr (FASTID) {
      wave_partials_fma<K>(q, p, m1l, k1);
      m1 = m1l;
      s2 = wave_sum2_dpp(k1 - e0l, e0l);   // lane 31: 2 (E1 - E0); lane 63: 2 E0 - logc
      E0 = __builtin_fma(s2, 0.5, hlogc);  // E0 of this iteration (lane 63)
      park_row();
    }
    // next iteration's momentum (keyed by it+1) so its kinetic energy joins this reduction
    const bool more = it + 1 < a.it1;
    double kn = 0.0;
    double (&pnext)[2 * K] = FASTID ? p : pn;
    if (more && !(FULL && (a.dbg & 256))) {
      if constexpr (RING) ring_momentum(it + 1, pnext);
      else wave_momentum<K, GEN, REPLAY>(a, c, gc, it + 1, kk, pv, pnext, s_ntab);
      if constexpr (!FASTID) kn = kin_partial<K, GEN>(a, kk, pv, pnext);
    }
    bool accept;
    uint32_t acc1 = 0;   // accept as 0/1 in an SGPR (FASTID), for the tallies
    if constexpr (FASTID) {
      // the test in lane 31 (samplers.py:459-462): dE < 0  <=>  2 dE < 0, and
      // log u < -dE  <=>  2 log u < -2 dE (lnu holds 2 log u here; both scalings are exact)
      acc1 = lane31(__builtin_amdgcn_ballot_w64(s2 < 0.0) | __builtin_amdgcn_ballot_w64(lnu < -s2));
      accept = acc1 != 0;
    } else {
      wave_partials<K, GEN>(a, kk, pv, q, p, m1, k1);
      m1l = m1;
      if constexpr (EXACT) {
        m1 = wave_sum_dpp(m1);
        k1 = wave_sum_dpp(k1);
        kn = wave_sum_dpp(kn);
      } else {
        k1 = wave_sum_dpp(m1 + k1);
      }
      const double E1 = EXACT ? 0.5 * (a.logc + (m1 + k1)) : 0.5 * (a.logc + k1);
      const double dE = E1 - E0;                          // samplers.py:459
      accept = (dE < 0.0) || (lnu < -dE);                 // :462
    }
    if (!accept && !(FULL && (a.dbg & 128))) {
#ifndef HMC_AB_SELECT
      asm volatile("" ::: "memory");   // keep a (uniform) branch: no per-iteration selects on accept
#endif
#pragma unroll
      for (int e = 0; e < 2 * K; ++e) q[e] = qi[e];
    }
    if (write_row && qcb && !(FULL && (a.dbg & 64)) && row >= a.q_row0) {
      double* rowp = qcb + (int64_t)qslot * a.D;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (pv[j]) store_pair_nt(rowp, kk[j], even, even || 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
    }
    if (cap && lane == 0) {
      a.traj_len[it - 1] = (L > 0 ? L : 0) + 1;
      a.decision[it - 1] = accept ? 1 : 0;
    }
    // tallies as scalar adds of the (uniform) decision: as `if (accept) ++n` the compiler merged
    // the increments through a pointer select and kept the counters in scratch (a load, a
    // vmcnt(0) wait behind the row store, and a store per iteration)
    if constexpr (!FASTID) acc1 = accept ? 1u : 0u;
    if (post) n_acc += acc1; else n_acc_wu += acc1;
    n_oob += (acc1 ^ 1u) & s_lt_i32(it, a.i_oob);
    const uint32_t Lp = L > 0 ? (uint32_t)L : 0u;
    n_lf += Lp;
    n_lf2 += Lp * Lp;
    // advance (FASTID: the next e0l unconditionally, so the one this iteration reduced is dead
    // after the reduction and the permlane swap may take its register)
    if constexpr (FASTID) {
      if (accept) {
        asm volatile("" ::: "memory");
        m0l = m1l;
      }
      e0l = __builtin_fma(p[1], p[1], m0l);   // V + K partial of the next iteration's start
      e0l = __builtin_fma(p[0], p[0], e0l);
#pragma unroll
      for (int e = 2; e < 2 * K; ++e) e0l = __builtin_fma(p[e], p[e], e0l);
    } else if (more) {
      if constexpr (!FASTID) {
#pragma unroll
        for (int e = 0; e < 2 * K; ++e) p[e] = pn[e];
      }
      if constexpr (EXACT) {
        m0 = accept ? m1 : m0;
        E0 = 0.5 * (a.logc + (m0 + kn));
      } else {                                            // V(q_next) + K(p_next) in one reduction
        if (accept) {
#ifndef HMC_AB_SELECT
          asm volatile("" ::: "memory");
#endif
          m0l = m1l;
        }
        E0 = 0.5 * (a.logc + wave_sum_dpp(m0l + kn));
      }
    }
    if (post && ++phase == a.thin) {
      phase = 0;
      ++row;
      if (++qslot == a.Lq) qslot = 0;
    }
  };
  const int it_mid = min(max(a.wu, a.it0), a.it1);
  for (int it = a.it0; it < it_mid; ++it) iteration(std::false_type{}, it);
  for (int it = it_mid; it < a.it1; ++it) iteration(std::true_type{}, it);
  // E of the launch's last iteration (E0 is not advanced past it)
  if (a.it1 > a.it0) Eprev = E0;

  // flush parked E/dE, write back state and counters
  if (nbuf > 0) flush_E(nbuf);
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (pv[j]) store_pair(qrow, kk[j], even, 2 * kk[j] + 1 < a.D, q[2 * j], q[2 * j + 1]);
  if (lane == kWave - 1) a.Eprev[c] = Eprev;          // lane 63: where FASTID keeps E
  if (lane == 0) {
    if (a.cnt) {   // per-wave counts into one of HMC_COUNTER_SLOTS rows (no single-address hot spot)
      unsigned long long* cs = a.cnt + (c & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
      if (n_acc) atomicAdd(cs + HMC_CNT_ACCEPT, (unsigned long long)n_acc);
      if (n_acc_wu) atomicAdd(cs + HMC_CNT_ACCEPT_WU, (unsigned long long)n_acc_wu);
      if (n_lf) atomicAdd(cs + HMC_CNT_LEAPFROG, (unsigned long long)n_lf);
      if (n_lf2) atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, (unsigned long long)n_lf2);
      if (n_oob) atomicAdd(cs + HMC_CNT_OOB_REJECT, (unsigned long long)n_oob);
    }
  }
}

// K = 1 (D <= 128, the headline shape) fits 64 VGPRs without spills: 8 waves per SIMD hide the
// dependent-latency part of the loop (+4%); wider K keep the compiler's register budget.
template <int K, bool EXACT, bool GEN, bool REPLAY, bool FULL>
__global__ __launch_bounds__(256) void k_wave_iters(RandArgs a) {
  wave_iters<K, EXACT, GEN, REPLAY, FULL>(a);
}

template <bool EXACT, bool GEN, bool REPLAY, bool FULL, bool ODD>
__global__ __launch_bounds__(kK1Block) __attribute__((amdgpu_waves_per_eu(8))) void k_wave_iters_k1(RandArgs a) {
  wave_iters<1, EXACT, GEN, REPLAY, FULL, ODD>(a);
}

template <int K, bool EXACT, bool GEN, bool REPLAY>
void launch_wave_one(const RandArgs& a, dim3 grid, hipStream_t s) {
  const bool full = a.traj_q != nullptr || a.dbg != 0 || a.dbgL >= 0;
  if constexpr (K == 1) {
    const dim3 g1((unsigned)((a.n + kK1Block / kWave - 1) / (kK1Block / kWave)));
    const bool odd = (a.D & 1) != 0 && !REPLAY;   // only the ring (Philox) path specialises on odd D
    if (full) {
      if (odd) k_wave_iters_k1<EXACT, GEN, REPLAY, true, !REPLAY><<<g1, kK1Block, 0, s>>>(a);
      else k_wave_iters_k1<EXACT, GEN, REPLAY, true, false><<<g1, kK1Block, 0, s>>>(a);
    } else {
      if (odd) k_wave_iters_k1<EXACT, GEN, REPLAY, false, !REPLAY><<<g1, kK1Block, 0, s>>>(a);
      else k_wave_iters_k1<EXACT, GEN, REPLAY, false, false><<<g1, kK1Block, 0, s>>>(a);
    }
  } else {
    if (full) k_wave_iters<K, EXACT, GEN, REPLAY, true><<<grid, 256, 0, s>>>(a);
    else k_wave_iters<K, EXACT, GEN, REPLAY, false><<<grid, 256, 0, s>>>(a);
  }
}

template <int K, bool EXACT>
hipError_t launch_wave_k2(const RandArgs& a, bool gen, bool replay, dim3 grid, hipStream_t s) {
  if (gen) {
    if (replay) launch_wave_one<K, EXACT, true, true>(a, grid, s);
    else launch_wave_one<K, EXACT, true, false>(a, grid, s);
  } else {
    if (replay) launch_wave_one<K, EXACT, false, true>(a, grid, s);
    else launch_wave_one<K, EXACT, false, false>(a, grid, s);
  }
  return hipGetLastError();
}

template <int K>
hipError_t launch_wave_k(const RandArgs& a, bool exact, bool gen, bool replay, dim3 grid, hipStream_t s) {
  return exact ? launch_wave_k2<K, true>(a, gen, replay, grid, s) : launch_wave_k2<K, false>(a, gen, replay, grid, s);
}

}  // namespace

hipError_t launch_wave_iters(const RandArgs& a, int K, bool exact, bool gen, bool replay, hipStream_t s) {
#ifdef HMC_WAVE_PROD_ONLY   // dev: ISA inspection of the headline instance only (seconds to compile)
  if (K == 1 && !exact && !gen && !replay) {
    launch_wave_one<1, false, false, false>(a, dim3(1), s);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
#endif
  const dim3 grid((unsigned)((a.n + 3) / 4));
  switch (K) {
    case 1: return launch_wave_k<1>(a, exact, gen, replay, grid, s);
    case 2: return launch_wave_k<2>(a, exact, gen, replay, grid, s);
    case 4: return launch_wave_k<4>(a, exact, gen, replay, grid, s);
    case 8: return launch_wave_k<8>(a, exact, gen, replay, grid, s);
    case 16: return launch_wave_k<16>(a, exact, gen, replay, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace hmc
