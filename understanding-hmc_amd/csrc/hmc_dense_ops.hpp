// hmc_dense_ops.hpp — shared pieces of the dense-precision kernels (Random: hmc_dense.hip,
// NUTS: hmc_nuts.hip): the f64-MFMA gradient of a 16-chain tile and its lane layout.
// Lane l = (chain c = l & 15, h = l >> 4) owns dims d = h + 4m, m < 4*MT, of chain c.
#pragma once
#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kDenseWaves = 4;   // waves per block: one block per CU (one P copy in LDS), one wave per SIMD with the full 512-register file

// Sum over lanes c, c+16, c+32, c+48 with gfx950's row swaps (v_permlane16_swap /
// v_permlane32_swap: VALU lane exchanges, no LDS round trip).  Swapping a register with itself
// leaves, in the two results, each lane's own value and its xor-16 (xor-32) partner in some order,
// so r0 + r1 is v[l] + v[l ^ 16] (then ^ 32): the same two-level sum as shuffles, bit for bit.
__device__ __forceinline__ double xor_sum_16(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double xor_sum_32(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double chain_sum4(double v) {   // sum over lanes c, c+16, c+32, c+48
  return xor_sum_32(xor_sum_16(v));
}

typedef __attribute__((address_space(3))) const double lds_cf64;

// P-fragment reader.  ds_read_b64 carries a 16-bit byte offset, so fragments past 64 KiB (P is
// up to 128 KiB) are read from a second base 64 KiB up.  That base is hidden from constant
// folding: otherwise the compiler materialises one address register per fragment past 64 KiB
// and, at 256 registers per wave, spills them.
struct FragReader {
  lds_cf64* lo;
  lds_cf64* hi;
  __device__ __forceinline__ FragReader(const double* sP, int lane) {
    lo = (lds_cf64*)sP + lane;
    uint32_t b = (uint32_t)(uintptr_t)(lo + 8192);
    asm volatile("" : "+v"(b));
    hi = (lds_cf64*)(uintptr_t)b;
  }
  // fragment f (compile-time constant after unrolling): f * 64 doubles from the lane's base
  __device__ __forceinline__ double operator()(int f) const { return f < 128 ? lo[f * kWave] : hi[(f - 128) * kWave]; }
};

// Short last tile: when the last 16-row output tile holds at most 4 dims (D = 97..100 at MT = 7),
// its rows are computed by v_mfma_f64_4x4x4f64 (4 blocks, a quarter of the 16x16x4 cost) instead
// of a 16x16x4 MFMA that is 3/4 zero rows.  Lane maps of the 4-block instruction (probed on
// gfx950, scripts/ubench/mfma_f64_4x4_layout.hip): A lane l = (k = l>>4, block = (l>>2)&3,
// i = l&3), B lane l = (k = l>>4, block = (l>>2)&3, j = l&3), D lane l = (i = l>>4,
// block = (l>>2)&3, j = l&3).  With block b = chains 4b..4b+3, B is the tile's usual x operand
// (lane (c, h) holds dim 4ks + h of chain c), A is P[16(MT-1) + (l&3)][4ks + (l>>4)] (staged that
// way, replicated over the blocks), and lane (c, h) receives row 16(MT-1) + h of chain c: the
// element the 16x16x4 layout puts in acc[MT-1][0].
// SHORT: kShortNever keeps the 16x16x4 form, kShortRuntime tests D per launch (one uniform branch
// per k-step: +3% on the dense Random kernel, -2.6% on NUTS), kShortAlways is an instance compiled
// for D = 16(MT-1)+1 .. 16(MT-1)+4 (no branch).
enum : int { kShortNever = 0, kShortRuntime = 1, kShortAlways = 2 };
template <int MT, int SHORT = kShortRuntime>
__device__ __forceinline__ bool short_last_tile(int D) {
  return SHORT == kShortAlways || (SHORT == kShortRuntime && D <= 16 * (MT - 1) + 4);
}

// DB: fragments of the next k-step read while this one's MFMAs run (one wave per SIMD must hide
// the LDS latency itself); without it the reads sit right before their MFMAs and a second wave
// on the SIMD covers the latency, for MT fewer live registers.
template <int MT, bool GEN, bool DB = true, int SHORT = kShortRuntime>
__device__ __forceinline__ void gradient(const DenseArgs& a, const double* __restrict__ sP, int lane, int h,
                                         const double (&q)[4 * MT], d4 (&acc)[MT]) {
  // k-step ks: MT MFMAs (one per 16-dim output tile) with the P fragments of ks, while the
  // fragments of ks+1 are read from LDS.  sched_barrier keeps the compiler from hoisting all
  // 4*MT*MT fragment reads to the top (which needs hundreds of VGPRs and spills).
  constexpr int KS = 4 * MT;
  // k-steps past ceil(D/4) multiply zero columns of P by zero (padded) coordinates: skipped
  // (D = 100: 25 of 28 k-steps, 11% fewer MFMAs).  Uniform bound, so the exit is a scalar branch.
  // k-steps past ceil(D/4) multiply zero columns of P by zero (padded) coordinates and are
  // skipped (D = 100: 25 of 28 k-steps).  Only the last three k-steps can be padding, so only
  // they carry the (scalar) exit test.
  const int ks_end = __builtin_amdgcn_readfirstlane((a.D + 3) >> 2);
  const bool sl = short_last_tile<MT, SHORT>(a.D);      // uniform
  double a4 = 0.0;                                      // the short last tile's accumulator
  const FragReader frag(sP, lane);
  auto mfma = [&](int nt, double af, double x) {
    if (nt == MT - 1 && sl) a4 = __builtin_amdgcn_mfma_f64_4x4x4f64(af, x, a4, 0, 0, 0);
    else acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, x, acc[nt], 0, 0, 0);
  };
  if constexpr (!DB) {
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) acc[nt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks >= KS - 3 && ks >= ks_end) break;
      double af[MT];
#pragma unroll
      for (int nt = 0; nt < MT; ++nt) af[nt] = frag(nt * KS + ks);
      const double x = (GEN && a.q0) ? q[ks] - a.q0[min(h + 4 * ks, a.D - 1)] : q[ks];
#pragma unroll
      for (int nt = 0; nt < MT; ++nt) mfma(nt, af[nt], x);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (sl) acc[MT - 1] = d4{a4, 0.0, 0.0, 0.0};
    return;
  }
  double af[MT], an[MT];
#pragma unroll
  for (int nt = 0; nt < MT; ++nt) {
    acc[nt] = d4{0.0, 0.0, 0.0, 0.0};
    af[nt] = frag(nt * KS);
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks >= KS - 3 && ks >= ks_end) break;
    if (ks + 1 < KS) {
#pragma unroll
      for (int nt = 0; nt < MT; ++nt) an[nt] = frag(nt * KS + ks + 1);
    }
    // keep the next k-step's fragment reads ahead of this k-step's MFMAs: scheduled after them
    // (the compiler's choice without this barrier) the reads issued only once the 7 MFMAs had
    // queued and the next k-step waited on their LDS latency
    __builtin_amdgcn_sched_barrier(0);
    // padded dims (d >= D) meet zero columns of P, so no guard is needed here
    const double x = (GEN && a.q0) ? q[ks] - a.q0[min(h + 4 * ks, a.D - 1)] : q[ks];
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) mfma(nt, af[nt], x);
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) af[nt] = an[nt];
    __builtin_amdgcn_sched_barrier(0);
  }
  if (sl) acc[MT - 1] = d4{a4, 0.0, 0.0, 0.0};
}

// y = M x for a symmetric (or pre-transposed) row-major D x D matrix in global memory (L2-resident),
// in the gradient's lane layout: the A-operand element (row 16nt + c, col 4ks + h) is read as
// src[(4ks + h) * D + 16nt + c], 16 consecutive doubles per (ks, h): 4 x 128 B per fragment.
// For symmetric M this is M[row][col]; pass the transpose of a non-symmetric matrix.  Used by the
// dense-mass-matrix path only (3-5 products per iteration against 13 LDS gradients), so the
// fragments come from L2 with a PF-deep prefetch instead of taking the LDS the kick matrix holds.
template <int MT>
__device__ __forceinline__ void matvec_global(const double* __restrict__ src, int D, int lane,
                                              const double (&x)[4 * MT], d4 (&acc)[MT]) {
  constexpr int KS = 4 * MT;
  constexpr int PF = 4;
  const int c = lane & 15, h = lane >> 4;
  const int ks_end = __builtin_amdgcn_readfirstlane((D + 3) >> 2);
  auto load = [&](int nt, int ks) -> double {
    const int row = 16 * nt + c, col = 4 * ks + h;
    const double v = src[(int64_t)min(col, D - 1) * D + min(row, D - 1)];
    return (row < D && col < D) ? v : 0.0;
  };
  double buf[PF][MT];
#pragma unroll
  for (int nt = 0; nt < MT; ++nt) acc[nt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < PF; ++j) {
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) buf[j][nt] = j < KS ? load(nt, j) : 0.0;
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks >= KS - 3 && ks >= ks_end) break;   // only the last 3 k-steps can be all padding
    double cur[MT];
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) cur[nt] = buf[ks % PF][nt];
    if (ks + PF < KS) {
#pragma unroll
      for (int nt = 0; nt < MT; ++nt) buf[ks % PF][nt] = load(nt, ks + PF);
    }
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(cur[nt], x[ks], acc[nt], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int MT>
__device__ __forceinline__ double gval(const d4 (&acc)[MT], int m) {
  return acc[m >> 2][m & 3];
}

// Per-dimension constants; the index is clamped so padded dims (whose p, q, g are all zero and
// stay zero) never branch.
template <int MT, bool GEN>
__device__ __forceinline__ double dim_minv(const DenseArgs& a, int d) {
  return (GEN && a.minv) ? a.minv[min(d, a.D - 1)] : 1.0;
}

template <int MT, bool GEN>
__device__ __forceinline__ double dim_dt(const DenseArgs& a, int d) {
  return (GEN && a.dtv) ? a.dtv[min(d, a.D - 1)] : a.dt;
}


// P fragments -> LDS (zero padded): fragment (nt, ks) lane l holds P[16nt + (l&15)][4ks + (l>>4)],
// stored lane-linear so every MFMA A-operand read is one conflict-free ds_read_b64.  A short last
// tile (short_last_tile) holds P[16nt + (l&3)][4ks + (l>>4)] instead: the 4x4x4 A operand.
// With a dense mass matrix the staged matrix is the kick matrix inv(cov_p).prec (a.kick).
template <int MT, int SHORT = kShortRuntime>
__device__ __forceinline__ void stage_precision(const DenseArgs& a, double* sP) {
  constexpr int KS = 4 * MT;
  const double* src = a.kick ? a.kick : a.prec;
  for (int f = threadIdx.x; f < MT * KS * kWave; f += blockDim.x) {
    const int l = f & (kWave - 1), t = f / kWave;
    const int nt = t / KS, ks = t - nt * KS;
    const int n = 16 * nt + ((nt == MT - 1 && short_last_tile<MT, SHORT>(a.D)) ? (l & 3) : (l & 15)), k = 4 * ks + (l >> 4);
    sP[f] = (n < a.D && k < a.D) ? src[(int64_t)n * a.D + k] : 0.0;
  }
  __syncthreads();
}

}  // namespace hmc
