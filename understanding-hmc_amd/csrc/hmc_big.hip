// hmc_big.hip — the Random-trajectory sampler for targets beyond the fused kernels' register
// budget: dense precision with D > 128 and diagonal precision with D > 2048 (samplers.py:428-475
// with the reference's any-D dgemv, :835-837).
//
// The fused kernels keep a chain's q and p in registers for a whole launch; at these sizes they do
// not fit, so the chain state moves to HBM and one iteration becomes a short, stream-ordered
// sequence of kernels:
//   begin (wave per chain): momentum (samplers.py:431), E0 (:434), L (:441), log u (:461), and
//     the copies a rejection restores (q, and for dense targets the gradient at q);
//   per leapfrog step l, for the chains with l < L: half kick + drift (elementwise), the gradient
//     at the new q (dense: f64-MFMA GEMM tiles, 16 chains x 64 dims, P read from L2 with the same
//     k-ordered MFMA sums as the fused kernel; diagonal: elementwise, inline), half kick;
//   end (wave per chain): E1, the Metropolis test (:455-472), restore on rejection, sample row.
// Draws use the diagonal wave kernel's Philox mapping (pair k = dims 2k, 2k+1 in slot k), so the
// host restatement of the parity tests regenerates them unchanged.
//
// A full cov_p (dense targets, samplers.py:352-356, :811-839) keeps the reference's products: the
// kick inv_cov_p . (P x) is a second GEMM on the gradient (kv), K = p . (inv_cov_p p) a GEMM on p
// at the iteration's two energies (u), and the Philox momentum p = C z a GEMM on z (u, then p);
// replay momenta are the reference's own N(0, cov_p) draws.  The energies then run in their own
// wave-per-chain kernel after those products.
#include "hmc_device.hpp"
#include "hmc_internal.hpp"
#include "hmc_dense_ops.hpp"

namespace hmc {

namespace {

__device__ __forceinline__ double q0_of(const RandArgs& a, int d) { return a.q0 ? a.q0[d] : 0.0; }
__device__ __forceinline__ double minv_of(const RandArgs& a, int d) { return a.minv ? a.minv[d] : 1.0; }
__device__ __forceinline__ double dt_of(const RandArgs& a, int d) { return a.dtv ? a.dtv[d] : a.dt; }
__device__ __forceinline__ double ps_of(const RandArgs& a, int d) { return a.pscale ? a.pscale[d] : 1.0; }

// P x of coordinate d at q[d]: the cached dense product, or P_dd (q - q0) for diagonal targets
template <bool DENSE>
__device__ __forceinline__ double grad_at(const BigArgs& b, int64_t i, int d, double qd) {
  if constexpr (DENSE) return b.g[i];
  const RandArgs& a = b.a;
  const double x = qd - q0_of(a, d);
  return a.prec ? a.prec[d] * x : x;
}

__device__ __forceinline__ bool write_row_of(const RandArgs& a, int it) {
  return it >= a.wu && ((it == a.niter) || ((it - a.wu + 1) % a.thin == 0));
}

// chain-0 trajectory capture (samplers.py:442-452, :463-475; make_movie's input): global chain 0
// in iterations 1 .. n_save writes q[:2] at the start and after every leapfrog step, L + 1 and
// the Metropolis decision, as the fused kernels do
__device__ __forceinline__ double* cap_row(const RandArgs& a, uint64_t gc, int it) {
  return (a.traj_q && gc == 0 && it >= 1 && it <= a.n_save) ? a.traj_q + (int64_t)(it - 1) * a.traj_stride * 2
                                                           : nullptr;
}

// ---- iteration start: one wave per chain, lanes over the coordinate pairs
template <bool DENSE, bool REPLAY, bool MASS = false>
__global__ __launch_bounds__(256) void k_big_begin(BigArgs b, int it) {
  __shared__ double tab[REPLAY ? 2 : kNormalTableDoubles];
  if constexpr (!REPLAY) {
    init_normal_tables(tab);
    __syncthreads();
  }
  const RandArgs& a = b.a;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  if (c >= a.n) return;
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  const int D = a.D, npairs = (D + 1) / 2;
  const int64_t base = c * (int64_t)D;
  double maha = 0.0, kin = 0.0;
  for (int k = lane; k < npairs; k += kWave) {
    double z[2];
    if constexpr (REPLAY) {
      const double* row = a.rp + (c * (int64_t)a.niter + (it - 1)) * D;
      z[0] = row[2 * k];
      z[1] = 2 * k + 1 < D ? row[2 * k + 1] : 0.0;
    } else {
      normal_pair_tab(draw_block((uint32_t)k, (uint32_t)it, gc, a.k0, a.k1), tab, z[0], z[1]);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int d = 2 * k + e;
      if (d >= D) break;
      const double pd = REPLAY ? z[e] : z[e] * ps_of(a, d);
      const int64_t i = base + d;
      if (MASS && !REPLAY) b.u[i] = pd;                                  // z: p = C z follows
      else b.p[i] = pd;
      kin += pd * (minv_of(a, d) * pd);
      const double qd = a.q[i];
      b.qi[i] = qd;
      const double gd = grad_at<DENSE>(b, i, d, qd);
      if constexpr (DENSE) b.gi[i] = gd;
      maha += (qd - q0_of(a, d)) * gd;
    }
  }
  maha = wave_sum_dpp(maha);
  kin = wave_sum_dpp(kin);
  const double E0 = 0.5 * (a.logc + (maha + kin));
  if (lane == 0) {
    if (!MASS && write_row_of(a, it)) {                             // (full cov_p: k_big_energy)
      const int64_t row = c * (int64_t)a.Lc + (it - a.wu) / a.thin;
      if (a.Ec) a.Ec[row] = E0;
      if (a.dEc) a.dEc[row] = E0 - a.Eprev[c];
    }
    if constexpr (!MASS) {
      a.Eprev[c] = E0;
      b.E0[c] = E0;
    }
    int L;
    double lnu;
    if constexpr (REPLAY) {
      L = a.rL[c * (int64_t)a.niter + (it - 1)];
      lnu = a.rlnu[c * (int64_t)a.niter + (it - 1)];
    } else {
      const uint4 r = draw_block(kDrawSlot, (uint32_t)it, gc, a.k0, a.k1);
      L = uniform_int(r.x, a.L_low, a.L_high);
      const double u = u53(r.z, r.w);
      lnu = u > 0.0 ? fast_log(u) : -__builtin_inf();
    }
    b.L[c] = L;
    b.lnu[c] = lnu;
    if (double* cp = cap_row(a, gc, it)) {                        // phi_q_tmp[0] = q[:2] (:444-446)
      cp[0] = a.q[base];
      cp[1] = a.q[base + (D > 1 ? 1 : 0)];
      a.traj_len[it - 1] = (L > 0 ? L : 0) + 1;
    }
  }
}

// ---- leapfrog pieces (samplers.py:831-839), elementwise over (chain, dim) for chains with l < L
template <bool EXACT, bool DENSE, bool DRIFT>
__global__ __launch_bounds__(256) void k_big_kick(BigArgs b, int l, int it) {
  const RandArgs& a = b.a;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n * (int64_t)a.D) return;
  const int64_t c = i / a.D;
  const int d = (int)(i - c * a.D);
  if (l >= b.L[c]) return;
  const double dt = dt_of(a, d), mi = minv_of(a, d);
  double qd = a.q[i];
  const double g = DENSE ? b.gk[i] : grad_at<false>(b, i, d, qd);    // the kick vector
  double pd = b.p[i];
  if constexpr (EXACT) pd = pd - (dt * (mi * g)) * 0.5;
  else pd = __builtin_fma(-0.5 * dt * mi, g, pd);
  b.p[i] = pd;
  if constexpr (DRIFT) {
    qd = EXACT ? qd + dt * pd : __builtin_fma(dt, pd, qd);
    a.q[i] = qd;
    if (d < 2)                                                    // phi_q_tmp[l] = q[:2] (:448-452)
      if (double* cp = cap_row(a, (uint64_t)(a.chain_offset + c), it)) cp[2 * (l + 1) + d] = qd;
  }
}

// ---- dense products y = M (x - shift) for the chains with l < L (all chains when l < 0): the
// gradient g = P (q - q0), and with a full cov_p inv_cov_p g, inv_cov_p p and C z.  A wave per
// (16-chain tile, 64-dim block), v_mfma_f64_16x16x4_f64 in the fused kernel's lane layout
// (A: M[row][k] read as M[k][row]: symmetric, or the transpose passed (cholt = C^T); coalesced;
// B: x[chain][k]; C: y[chain][row]).
constexpr int kBigDims = 64;   // output dims per wave (4 MFMA tiles)

struct BigGemm {
  const double* m;   // [D][D], read as m[k][row]
  const double* x;   // [n][D]
  bool shift;        // subtract q0 from x
  double* y;         // [n][D]
};

__global__ __launch_bounds__(256) void k_big_gemm(BigArgs b, BigGemm G, int l) {
  const RandArgs& a = b.a;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t w = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  const int D = a.D;
  const int nblk = (D + kBigDims - 1) / kBigDims;
  const int64_t tile = w / nblk;
  const int blk = (int)(w - tile * nblk);
  if (tile * 16 >= a.n) return;
  const int cl = lane & 15, h = lane >> 4;
  const int64_t chain = tile * 16 + cl;
  const bool live = chain < a.n;
  const bool active = live && (l < 0 || l < b.L[chain]);
  if (!__builtin_amdgcn_ballot_w64(active)) return;                 // whole tile frozen
  const double* qrow = G.x + (live ? chain : 0) * (int64_t)D;
  d4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = d4{0.0, 0.0, 0.0, 0.0};
  const int ks_end = (D + 3) >> 2;
  for (int ks = 0; ks < ks_end; ++ks) {
    const int k = 4 * ks + h;
    const int kc = k < D ? k : D - 1;
    const double xv = qrow[kc] - (G.shift ? q0_of(a, kc) : 0.0);
    const double x = (live && k < D) ? xv : 0.0;
    const double* prow = G.m + (int64_t)kc * D;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int row = blk * kBigDims + 16 * nt + cl;
      const double pv = prow[row < D ? row : D - 1];
      const double av = (row < D && k < D) ? pv : 0.0;
      acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, x, acc[nt], 0, 0, 0);
    }
  }
  if (!active) return;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = blk * kBigDims + 16 * nt + h + 4 * r;
      if (row < D) G.y[chain * (int64_t)D + row] = acc[nt][r];
    }
  }
}

// ---- iteration end: E1, Metropolis test, restore on rejection, sample row, tallies
template <bool DENSE, bool MASS = false>
__global__ __launch_bounds__(256) void k_big_end(BigArgs b, int it) {
  const RandArgs& a = b.a;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  if (c >= a.n) return;
  const int D = a.D;
  const int64_t base = c * (int64_t)D;
  double maha = 0.0, kin = 0.0;
  for (int d = lane; d < D; d += kWave) {
    const int64_t i = base + d;
    const double qd = a.q[i], pd = b.p[i];
    maha += (qd - q0_of(a, d)) * grad_at<DENSE>(b, i, d, qd);
    kin += MASS ? pd * b.u[i] : pd * (minv_of(a, d) * pd);         // (full cov_p: u = inv_cov_p p)
  }
  maha = wave_sum_dpp(maha);
  kin = wave_sum_dpp(kin);
  const double E1 = 0.5 * (a.logc + (maha + kin));
  const double dE = E1 - b.E0[c];                                    // samplers.py:459
  const double lnu = b.lnu[c];
  const bool accept = (dE < 0.0) || (lnu < -dE);                    // :462
  const bool post = it >= a.wu;
  const bool write_row = write_row_of(a, it);
  const int64_t row = post ? (int64_t)((it - a.wu) / a.thin) : 0;
  const bool store = write_row && a.qc && row >= a.q_row0;
  double* rowp = store ? a.qc + c * (int64_t)a.Lq * D + (row % a.Lq) * D : nullptr;
  for (int d = lane; d < D; d += kWave) {
    const int64_t i = base + d;
    double qd;
    if (accept) {
      qd = a.q[i];
    } else {
      qd = b.qi[i];
      a.q[i] = qd;
      if constexpr (DENSE) b.g[i] = b.gi[i];
    }
    if (store) __builtin_nontemporal_store(qd, rowp + d);
  }
  if (lane == 0 && cap_row(a, (uint64_t)(a.chain_offset + c), it)) a.decision[it - 1] = accept ? 1 : 0;   // :463-466
  if (lane == 0 && a.cnt) {
    unsigned long long* cs = a.cnt + (c & (HMC_COUNTER_SLOTS - 1)) * HMC_NCOUNTERS;
    if (accept) atomicAdd(cs + (post ? HMC_CNT_ACCEPT : HMC_CNT_ACCEPT_WU), 1ull);
    else if (it < a.i_oob) atomicAdd(cs + HMC_CNT_OOB_REJECT, 1ull);
    const unsigned long long Lp = b.L[c] > 0 ? (unsigned long long)b.L[c] : 0ull;
    if (Lp) {
      atomicAdd(cs + HMC_CNT_LEAPFROG, Lp);
      atomicAdd(cs + HMC_CNT_LEAPFROG_SQ, Lp * Lp);
    }
  }
}

// ---- full cov_p: E = V + K after the products (g = P x, u = inv_cov_p p) at iteration it's start
// (it > 0: row of E/dE, Eprev, E0) or at chain initialisation (it = 0: row 0, dE 0)
__global__ __launch_bounds__(256) void k_big_energy(BigArgs b, int it) {
  const RandArgs& a = b.a;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  if (c >= a.n) return;
  const int64_t base = c * (int64_t)a.D;
  double maha = 0.0, kin = 0.0;
  for (int d = lane; d < a.D; d += kWave) {
    const int64_t i = base + d;
    maha += (a.q[i] - q0_of(a, d)) * b.g[i];
    kin += b.p[i] * b.u[i];
  }
  maha = wave_sum_dpp(maha);
  kin = wave_sum_dpp(kin);
  if (lane != 0) return;
  const double E0 = 0.5 * (a.logc + (maha + kin));
  if (it == 0) {
    if (a.Ec) a.Ec[c * (int64_t)a.Lc] = E0;
    if (a.dEc) a.dEc[c * (int64_t)a.Lc] = 0.0;
  } else {
    if (write_row_of(a, it)) {
      const int64_t row = c * (int64_t)a.Lc + (it - a.wu) / a.thin;
      if (a.Ec) a.Ec[row] = E0;
      if (a.dEc) a.dEc[row] = E0 - a.Eprev[c];
    }
    b.E0[c] = E0;
  }
  a.Eprev[c] = E0;
}

// ---- full cov_p, chain initialisation: the iteration-0 momentum (replay p0, or z for p = C z)
template <bool REPLAY>
__global__ __launch_bounds__(256) void k_big_mass_p0(BigArgs b) {
  const RandArgs& a = b.a;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  if (c >= a.n) return;
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  const int D = a.D, npairs = (D + 1) / 2;
  const int64_t base = c * (int64_t)D;
  for (int k = lane; k < npairs; k += kWave) {
    double z[2];
    if constexpr (REPLAY) {
      z[0] = a.rp0[base + 2 * k];
      z[1] = 2 * k + 1 < D ? a.rp0[base + 2 * k + 1] : 0.0;
    } else {
      normal_pair(draw_block((uint32_t)k, 0u, gc, a.k0, a.k1), z[0], z[1]);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int d = 2 * k + e;
      if (d >= D) break;
      (REPLAY ? b.p : b.u)[base + d] = z[e];
      if (a.qc && a.q_row0 == 0) a.qc[c * (int64_t)a.Lq * D + d] = a.q[base + d];
    }
  }
}

// ---- chain initialisation (samplers.py:413-420): E of (q_start, p0) with the iteration-0
// momentum of the same mapping (libm-free Box-Muller, as every kernel's p0)
template <bool DENSE, bool REPLAY>
__global__ __launch_bounds__(256) void k_big_init(BigArgs b) {
  const RandArgs& a = b.a;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = uniform_i(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
  if (c >= a.n) return;
  const uint64_t gc = (uint64_t)(a.chain_offset + c);
  const int D = a.D, npairs = (D + 1) / 2;
  const int64_t base = c * (int64_t)D;
  double maha = 0.0, kin = 0.0;
  for (int k = lane; k < npairs; k += kWave) {
    double z[2];
    if constexpr (REPLAY) {
      z[0] = a.rp0[base + 2 * k];
      z[1] = 2 * k + 1 < D ? a.rp0[base + 2 * k + 1] : 0.0;
    } else {
      normal_pair(draw_block((uint32_t)k, 0u, gc, a.k0, a.k1), z[0], z[1]);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int d = 2 * k + e;
      if (d >= D) break;
      const double pd = REPLAY ? z[e] : z[e] * ps_of(a, d);
      kin += pd * (minv_of(a, d) * pd);
      const double qd = a.q[base + d];
      maha += (qd - q0_of(a, d)) * grad_at<DENSE>(b, base + d, d, qd);
      if (a.qc && a.q_row0 == 0) a.qc[c * (int64_t)a.Lq * D + d] = qd;
    }
  }
  maha = wave_sum_dpp(maha);
  kin = wave_sum_dpp(kin);
  if (lane == 0) {
    const double E0 = 0.5 * (a.logc + (maha + kin));
    a.Eprev[c] = E0;
    if (a.Ec) a.Ec[c * (int64_t)a.Lc] = E0;
    if (a.dEc) a.dEc[c * (int64_t)a.Lc] = 0.0;
  }
}

dim3 waves_grid(int64_t waves) { return dim3((unsigned)((waves + 3) / 4)); }
dim3 elems_grid(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t gemm_all(const BigArgs& b, const BigGemm& G, int l, hipStream_t s) {
  const int64_t waves = ((b.a.n + 15) / 16) * ((b.a.D + kBigDims - 1) / kBigDims);
  k_big_gemm<<<waves_grid(waves), 256, 0, s>>>(b, G, l);
  return hipGetLastError();
}

// g = P (q - q0), and with a full cov_p the kick kv = inv_cov_p g
hipError_t grad_all(const BigArgs& b, int l, hipStream_t s) {
  if (hipError_t e = gemm_all(b, BigGemm{b.a.prec, b.a.q, true, b.g}, l, s)) return e;
  if (b.a.minvf) return gemm_all(b, BigGemm{b.a.minvf, b.g, false, b.kv}, l, s);
  return hipSuccess;
}

// full cov_p: p = C z (Philox: z in u) and u = inv_cov_p p, for every chain
hipError_t mass_momentum(const BigArgs& b, bool replay, hipStream_t s) {
  if (!replay)
    if (hipError_t e = gemm_all(b, BigGemm{b.a.cholt, b.u, false, b.p}, -1, s)) return e;
  return gemm_all(b, BigGemm{b.a.minvf, b.p, false, b.u}, -1, s);
}

}  // namespace

bool big_path(int kind_dense, int D) { return kind_dense ? dense_tiles(D) == 0 : (D + 1) / 2 > 16 * kWave; }

// vectors: p, qi; dense targets also g, gi and, with a full cov_p, its products kv, u
static int big_vectors(bool dense, bool full_mass) { return dense ? (full_mass ? 6 : 4) : 2; }

int64_t big_workspace_bytes(int64_t n, int D, bool dense, bool full_mass) {
  const int64_t v = ((n * (int64_t)D * 8 + 255) / 256) * 256;
  const int64_t s = ((n * 8 + 255) / 256) * 256;
  return v * big_vectors(dense, full_mass) + 3 * s;
}

BigArgs big_args(const RandArgs& a, void* ws, bool dense) {
  BigArgs b{};
  b.a = a;
  char* p = static_cast<char*>(ws);
  const int64_t v = ((a.n * (int64_t)a.D * 8 + 255) / 256) * 256;
  const int64_t s = ((a.n * 8 + 255) / 256) * 256;
  b.p = reinterpret_cast<double*>(p);
  b.qi = reinterpret_cast<double*>(p + v);
  if (dense) {
    b.g = reinterpret_cast<double*>(p + 2 * v);
    b.gi = reinterpret_cast<double*>(p + 3 * v);
    if (a.minvf) {
      b.kv = reinterpret_cast<double*>(p + 4 * v);
      b.u = reinterpret_cast<double*>(p + 5 * v);
    }
    b.gk = a.minvf ? b.kv : b.g;
  }
  char* t = p + v * big_vectors(dense, a.minvf != nullptr);
  b.L = reinterpret_cast<int32_t*>(t);
  b.lnu = reinterpret_cast<double*>(t + s);
  b.E0 = reinterpret_cast<double*>(t + 2 * s);
  return b;
}

hipError_t launch_big_init(const BigArgs& b, bool dense, bool replay, hipStream_t s) {
  const RandArgs& a = b.a;
  if (hipError_t e = hipMemcpyAsync(a.q, a.qstart, a.n * (int64_t)a.D * sizeof(double), hipMemcpyDeviceToDevice, s))
    return e;
  if (dense)
    if (hipError_t e = grad_all(b, -1, s)) return e;
  const dim3 g = waves_grid(a.n);
  if (a.minvf) {                                          // full cov_p: E after the products
    if (replay) k_big_mass_p0<true><<<g, 256, 0, s>>>(b);
    else k_big_mass_p0<false><<<g, 256, 0, s>>>(b);
    if (hipError_t e = mass_momentum(b, replay, s)) return e;
    k_big_energy<<<g, 256, 0, s>>>(b, 0);
  } else if (dense) {
    if (replay) k_big_init<true, true><<<g, 256, 0, s>>>(b);
    else k_big_init<true, false><<<g, 256, 0, s>>>(b);
  } else {
    if (replay) k_big_init<false, true><<<g, 256, 0, s>>>(b);
    else k_big_init<false, false><<<g, 256, 0, s>>>(b);
  }
  return hipGetLastError();
}

template <bool EXACT, bool DENSE>
hipError_t big_iterations(const BigArgs& b, bool replay, hipStream_t s) {
  const RandArgs& a = b.a;
  const dim3 gw = waves_grid(a.n), ge = elems_grid(a.n * (int64_t)a.D);
  const int lmax = a.L_high > 1 ? a.L_high - 1 : 0;       // L < L_high (randint, Q1)
  const bool mass = DENSE && a.minvf;
  for (int it = a.it0; it < a.it1; ++it) {
    if (mass) {                                           // full cov_p: products, then E0
      if (replay) k_big_begin<DENSE, true, true><<<gw, 256, 0, s>>>(b, it);
      else k_big_begin<DENSE, false, true><<<gw, 256, 0, s>>>(b, it);
      if (hipError_t e = mass_momentum(b, replay, s)) return e;
      if (hipError_t e = gemm_all(b, BigGemm{a.minvf, b.g, false, b.kv}, -1, s)) return e;   // kick at q
      k_big_energy<<<gw, 256, 0, s>>>(b, it);
    } else if (replay) {
      k_big_begin<DENSE, true><<<gw, 256, 0, s>>>(b, it);
    } else {
      k_big_begin<DENSE, false><<<gw, 256, 0, s>>>(b, it);
    }
    for (int l = 0; l < lmax; ++l) {
      k_big_kick<EXACT, DENSE, true><<<ge, 256, 0, s>>>(b, l, it);
      if (DENSE)
        if (hipError_t e = grad_all(b, l, s)) return e;
      k_big_kick<EXACT, DENSE, false><<<ge, 256, 0, s>>>(b, l, it);
    }
    if (mass) {
      if (hipError_t e = gemm_all(b, BigGemm{a.minvf, b.p, false, b.u}, -1, s)) return e;
      k_big_end<DENSE, true><<<gw, 256, 0, s>>>(b, it);
    } else {
      k_big_end<DENSE><<<gw, 256, 0, s>>>(b, it);
    }
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

hipError_t launch_big_iters(const BigArgs& b, bool dense, bool exact, bool replay, hipStream_t s) {
  if (exact) return dense ? big_iterations<true, true>(b, replay, s) : big_iterations<true, false>(b, replay, s);
  return dense ? big_iterations<false, true>(b, replay, s) : big_iterations<false, false>(b, replay, s);
}

}  // namespace hmc
