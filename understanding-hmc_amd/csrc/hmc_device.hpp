// hmc_device.hpp — device-side building blocks shared by the HMC kernels (gfx950).
//
//  * Philox4x32-10 counter-based generator (Salmon et al., SC'11), keyed by
//    (seed) with counter (slot, iteration, global chain id): every draw is a pure
//    function of (seed, chain, iteration, slot), so results do not depend on the
//    launch geometry or on how chains are sharded over GPUs.
//  * fp64 Box–Muller from 53-bit uniforms (momentum draws, replaces
//    np.random.multivariate_normal at samplers.py:829).
//  * Lane-group layout: a chain's D coordinates live in one "group" of LPC
//    consecutive lanes of a wave64; lane s of the group owns coordinate pairs
//    k = s + LPC*j (j < K).  CPW = 64/LPC chains share a wave.  Group sums use
//    ds_bpermute shuffles (no LDS, no barriers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hmc {

constexpr int kWave = 64;
constexpr uint32_t kDrawSlot = 0x80000000u;  // counter.x for non-momentum draws (L, u, NUTS draws)

// a ^ b ^ k in one VALU instruction: gfx950's three-input v_bitop3_b32 with truth table 0x96.
// The key must be wave-uniform (every caller passes the seed from the kernel arguments): it is
// an SGPR operand.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}

template <int ROUNDS>
__device__ __forceinline__ uint4 philox_rounds(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    // one v_mad_u64_u32 per 32x32->64 product (lo and hi words together), one v_bitop3 per xor pair
    const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u;
    const uint64_t p1 = (uint64_t)c.z * 0xCD9E8D57u;
    c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, k0), (uint32_t)p1, xor3((uint32_t)(p0 >> 32), c.w, k1),
                   (uint32_t)p0);
    // key schedule on the SALU at the point of use: hoisted out of the chain loop it would hold
    // 20 SGPRs and be spilled (v_readlane per round)
    asm volatile("s_add_u32 %0, %0, 0x9E3779B9" : "+s"(k0) : : "scc");
    asm volatile("s_add_u32 %0, %0, 0xBB67AE85" : "+s"(k1) : : "scc");
  }
  return c;
}

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) { return philox_rounds<10>(c, k0, k1); }

// Loop-invariant value made opaque to the optimiser at its point of use (keeps a hoisted
// first Philox round of every draw slot from occupying registers across a whole loop).
__device__ __forceinline__ uint32_t opaque_u32(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
// A constant kept in an SGPR operand (the compiler would otherwise split the instruction that
// reads it back into a shift and an or).
__device__ __forceinline__ uint32_t opaque_s32(uint32_t v) {
  asm("" : "+s"(v));
  return v;
}

__device__ __forceinline__ uint4 draw_block(uint32_t slot, uint32_t iter, uint64_t gchain, uint32_t k0,
                                            uint32_t k1) {
  return philox4x32_10(make_uint4(slot, iter, (uint32_t)gchain, (uint32_t)(gchain >> 32)), k0, k1);
}

// draw_block when the chain (counter words z, w) is wave-uniform, as in the one-chain-per-wave
// kernel: the first two rounds are written out so the products and xors of uniform words run on
// the SALU (the asm xor3 of the generic round takes one SGPR operand only).  Same function.
__device__ __forceinline__ uint4 draw_block_uc(uint32_t slot, uint32_t iter, uint64_t gchain, uint32_t k0,
                                               uint32_t k1) {
  const uint32_t glo = (uint32_t)gchain, ghi = (uint32_t)(gchain >> 32);
  const uint64_t p0 = (uint64_t)slot * 0xD2511F53u;
  const uint64_t p1 = (uint64_t)glo * 0xCD9E8D57u;                      // uniform
  // (ghi ^ k1) pinned in an SGPR: reassociated, the xor with the lane's word took two VALU
  uint4 c = make_uint4(iter ^ ((uint32_t)(p1 >> 32) ^ k0), (uint32_t)p1, (uint32_t)(p0 >> 32) ^ opaque_s32(ghi ^ k1),
                       (uint32_t)p0);
  k0 += 0x9E3779B9u;
  k1 += 0xBB67AE85u;
  const uint64_t r0 = (uint64_t)c.x * 0xD2511F53u;
  const uint64_t r1 = (uint64_t)c.z * 0xCD9E8D57u;
  c = make_uint4((uint32_t)(r1 >> 32) ^ (c.y ^ k0), (uint32_t)r1, xor3((uint32_t)(r0 >> 32), c.w, k1), (uint32_t)r0);
  k0 += 0x9E3779B9u;
  k1 += 0xBB67AE85u;
  return philox_rounds<8>(c, k0, k1);
}

// 53-bit uniform in [0, 1) from two words.
__device__ __forceinline__ double u53(uint32_t lo, uint32_t hi) {
  return (double)((((uint64_t)hi) << 21) | (lo >> 11)) * 0x1p-53;
}
// 53-bit uniform in (0, 1].
__device__ __forceinline__ double u53_open0(uint32_t lo, uint32_t hi) {
  return ((double)((((uint64_t)hi) << 21) | (lo >> 11)) + 1.0) * 0x1p-53;
}

// ---- fp64 elementary functions for Box–Muller: ~1 ulp, straight-line (no double-double
// intermediate like the libm/ocml versions, which cost ~3x more).  Algorithms: fdlibm
// e_log.c (Lg1..Lg7 minimax on s = f/(2+f)) and k_sin.c / k_cos.c (|a| <= pi/4).

// 1/d: v_rcp_f64 seed + two Newton steps.
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}

// x*y + c with a compile-time constant c as an SGPR-pair operand of one v_fma_f64 (the compiler
// otherwise copies each constant into the destination VGPRs and uses v_fmac: two instructions).
__device__ __forceinline__ double fmac_k(double x, double y, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "s"(c));
  return r;
}

// log(x) for finite x > 0 (fdlibm e_log.c reduction; polynomials as Horner chains of
// v_fma_f64 with the coefficients as SGPR operands).
__device__ __forceinline__ double fast_log(double x) {
  int k = __builtin_amdgcn_frexp_exp(x);
  double m = __builtin_amdgcn_frexp_mant(x);       // [0.5, 1)
  const bool lo = m < 0.70710678118654752440;       // -> [sqrt(1/2), sqrt(2))
  m = lo ? 2.0 * m : m;
  k = lo ? k - 1 : k;
  const double f = m - 1.0;
  const double s = f * rcp_nr(2.0 + f);
  const double z = s * s, w = z * z;
  double t1 = fmac_k(w, 1.531383769920937332e-01, 2.222219843214978396e-01);   // Lg6, Lg4
  t1 = fmac_k(w, t1, 3.999999999940941908e-01);                                   // Lg2
  double t2 = fmac_k(w, 1.479819860511658591e-01, 1.818357216161805012e-01);    // Lg7, Lg5
  t2 = fmac_k(w, t2, 2.857142874366239149e-01);                                   // Lg3
  t2 = fmac_k(w, t2, 6.666666666666735130e-01);                                   // Lg1
  const double R = __builtin_fma(z, t2, w * t1);
  const double hfsq = (0.5 * f) * f;
  const double dk = (double)k;
  const double inner = __builtin_fma(s, hfsq + R, dk * 1.90821492927058770002e-10);
  return __builtin_fma(dk, 6.93147180369123816490e-01, -((hfsq - inner) - f));
}

// sqrt(x) for x >= 0: v_rsq_f64 seed + one Goldschmidt/Newton refinement.
__device__ __forceinline__ double fast_sqrt(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  const double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return x > 0.0 ? g : 0.0;
}

// sin(pi x), cos(pi x) for x in [0, 2] (fdlibm k_sin.c / k_cos.c kernels on |a| <= pi/4;
// Horner chains of v_fma_f64 with SGPR coefficients).
__device__ __forceinline__ void fast_sincospi(double x, double& sn, double& cs) {
  const double n = __builtin_rint(2.0 * x);
  const double r = __builtin_fma(-0.5, n, x);                    // exact, |r| <= 1/4
  const double a = __builtin_fma(r, 3.14159265358979311600e+00, r * 1.22464679914735317720e-16);
  const double z = a * a;
  const double v = z * a;
  double sr = fmac_k(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);   // S6, S5
  sr = fmac_k(z, sr, 2.75573137070700676789e-06);                                     // S4
  sr = fmac_k(z, sr, -1.98412698298579493134e-04);                                    // S3
  sr = fmac_k(z, sr, 8.33333333332248946124e-03);                                     // S2
  const double sa = __builtin_fma(v, fmac_k(z, sr, -1.66666666666666324348e-01), a);  // S1
  double cr = fmac_k(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);    // C6, C5
  cr = fmac_k(z, cr, -2.75573143513906633035e-07);                                    // C4
  cr = fmac_k(z, cr, 2.48015872894767294178e-05);                                     // C3
  cr = fmac_k(z, cr, -1.38888888888741095749e-03);                                    // C2
  cr = fmac_k(z, cr, 4.16666666666666019037e-02);                                     // C1
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double ca = w + __builtin_fma(z * z, cr, (1.0 - w) - hz);
  const int q = ((int)n) & 3;                        // pi x = q*pi/2 + a
  const double s0 = (q & 1) ? ca : sa;
  const double c0 = (q & 1) ? sa : ca;
  sn = (q & 2) ? -s0 : s0;
  cs = ((q + 1) & 2) ? -c0 : c0;
}

// [1, 2) with the top 52 bits of (hi:lo) as mantissa: two v_alignbit, no conversion.
__device__ __forceinline__ double one_to_two(uint32_t lo, uint32_t hi) {
  const uint32_t mlo = __builtin_amdgcn_alignbit(hi, lo, 12);   // low word of (hi:lo) >> 12
  // (0x3FF:hi) >> 12 = (hi >> 12) | 0x3FF00000, the exponent of [1, 2) shifted in with the bits
  const uint32_t mhi = __builtin_amdgcn_alignbit(opaque_s32(0x3FFu), hi, 12);
  return __builtin_bit_cast(double, ((uint64_t)mhi << 32) | mlo);
}

// Two independent N(0,1) from one Philox block (fp64 Box–Muller on 52-bit uniforms:
// u1 = 2 - d1 in (0, 1], angle 2*pi*(d2 - 1) in [0, 2*pi), all conversions exact).
__device__ __forceinline__ void normal_pair(uint4 r, double& z0, double& z1) {
  const double u1 = 2.0 - one_to_two(r.x, r.y);
  const double x2 = __builtin_fma(2.0, one_to_two(r.z, r.w), -2.0);
  const double rad = fast_sqrt(-2.0 * fast_log(u1));
  double s, c;
  fast_sincospi(x2, s, c);
  z0 = rad * c;
  z1 = rad * s;
}

// ---- table-driven Box–Muller (the wave kernel's momentum draws).  Per block, two small LDS
// tables built once with the ~1-ulp kernels above:
//   trig[i] = (cos, sin)(2*pi*i/1024), i < 1024          (16 KB)
//   logt[j] = (1/c_j, -log(1/c_j)), c_j = centre of the j-th of 1024 buckets of [0.5, 1)
//             (the last bucket uses c = 1: log is then log1p(m - 1), relative-accurate near 1)
// so that log and sincos reduce to short Horner chains around a table point (1024 entries: two
// fewer terms in each series than 256/128 entries, for 16 KB more LDS per block).
#ifdef HMC_SMALL_TABLES
constexpr int kTrigN = 256, kLogN = 128;
#else
constexpr int kTrigN = 1024, kLogN = 1024;
#endif
constexpr int kLogShift = kLogN == 1024 ? 10 : 13, kTrigShift = kTrigN == 1024 ? 10 : 12;
constexpr int kNormalTableDoubles = 2 * kTrigN + 2 * kLogN;

// Every thread of the block calls this, then the block synchronises.
__device__ __forceinline__ void init_normal_tables(double* tab) {
  for (int i = threadIdx.x; i < kTrigN; i += blockDim.x) {
    double sn, cs;
    fast_sincospi((double)i * (2.0 / kTrigN), sn, cs);
    tab[2 * i] = cs;
    tab[2 * i + 1] = sn;
  }
  for (int j = threadIdx.x; j < kLogN; j += blockDim.x) {
    const double c = j == kLogN - 1 ? 1.0 : 0.5 + ((double)j + 0.5) * (0.5 / kLogN);
    const double ic = j == kLogN - 1 ? 1.0 : rcp_nr(c);
    tab[2 * kTrigN + 2 * j] = ic;
    tab[2 * kTrigN + 2 * j + 1] = j == kLogN - 1 ? 0.0 : -fast_log(ic);
  }
}

__device__ __forceinline__ double2 lds_pair(const double* p) { return *reinterpret_cast<const double2*>(p); }

// log(u) for u in (0, 1] from the tables: u = 2^k m, m in [0.5, 1); bucket j = top 10 mantissa
// bits; log m = L_j + log1p(m / c_j - 1) with |r| <= 2^-11 (series to r^5; r^6/6 < 2^-68).
__device__ __forceinline__ double table_log(double u, const double* tab) {
  const int k = __builtin_amdgcn_frexp_exp(u);
  const double m = __builtin_amdgcn_frexp_mant(u);
  const uint32_t mhi = (uint32_t)(__builtin_bit_cast(uint64_t, m) >> 32);
  // byte offset 16 j of bucket j = (mhi >> kLogShift) & (kLogN - 1): one shift, one and
  const uint32_t j16 = (mhi >> (kLogShift - 4)) & ((kLogN - 1) << 4);
  const double2 e = lds_pair(reinterpret_cast<const double*>(reinterpret_cast<const char*>(tab + 2 * kTrigN) + j16));
  const double r = __builtin_fma(m, e.x, -1.0);
#ifdef HMC_SMALL_TABLES
  double pl = fmac_k(r, 1.0 / 7.0, -1.0 / 6.0);
  pl = fmac_k(r, pl, 1.0 / 5.0);
  pl = fmac_k(r, pl, -1.0 / 4.0);
#else
  // (an output-modifier form, (0.4 r - 0.5) with div:2, measured wrong on gfx950: omod is not
  // applied to this f64 FMA; test_table_normals_match_kernel caught it)
  double pl = fmac_k(r, 1.0 / 5.0, -1.0 / 4.0);
#endif
  pl = fmac_k(r, pl, 1.0 / 3.0);
  pl = __builtin_fma(r, pl, -0.5);                                      // inline constant
  const double l1p = __builtin_fma(r * r, pl, r);                       // log1p(r)
  const double dk = (double)k;
  return __builtin_fma(dk, 6.93147180369123816490e-01, e.y + __builtin_fma(dk, 1.90821492927058770002e-10, l1p));
}

// (cos, sin)(2*pi*(d - 1)) for d in [1, 2) holding 52 random mantissa bits: table point from the
// top 10 bits, the rest delta in [0, 2*pi/1024) by Taylor series (sin to delta^5, cos to delta^6:
// the next terms are below 2^-60 relative).
__device__ __forceinline__ void table_cossin(double d, const double* tab, double& cs, double& sn) {
  const uint64_t bits = __builtin_bit_cast(uint64_t, d);
  const uint32_t hi = (uint32_t)(bits >> 32);
  const uint32_t i16 = (hi >> (kTrigShift - 4)) & ((kTrigN - 1) << 4);   // byte offset of entry i
  const double f = __builtin_bit_cast(double, bits & ~((uint64_t)(kTrigN - 1) << (32 + kTrigShift))) - 1.0;  // exact
  // delta = 2 pi f rounded once: delta < 2 pi / 1024, so the low part of 2 pi (2.4e-16 relative)
  // would move the final (cos, sin) by < 1e-19, far below their ulp
  const double dl = f * 6.28318530717958623200e+00;
  const double z = dl * dl;
#ifdef HMC_SMALL_TABLES
  double ps = fmac_k(z, -1.0 / 5040.0, 1.0 / 120.0);
  ps = fmac_k(z, ps, -1.0 / 6.0);
  const double sd = __builtin_fma(dl * z, ps, dl);                       // sin(delta)
  double pc = fmac_k(z, 1.0 / 40320.0, -1.0 / 720.0);
  pc = fmac_k(z, pc, 1.0 / 24.0);
  pc = fmac_k(z, pc, -0.5);
#else
  const double ps = fmac_k(z, 1.0 / 120.0, -1.0 / 6.0);
  const double sd = __builtin_fma(dl * z, ps, dl);                       // sin(delta)
  // cos to delta^4: delta^6/720 < 7.5e-17 < ulp(1)/2 for delta < 2 pi/1024
  double pc;
  asm("v_fma_f64 %0, %1, %2, -0.5" : "=v"(pc) : "v"(z), "s"(1.0 / 24.0));
#endif
  const double cd = __builtin_fma(z, pc, 1.0);                          // cos(delta)
  const double2 t = lds_pair(reinterpret_cast<const double*>(reinterpret_cast<const char*>(tab) + i16));  // (cos, sin)(theta_i)
  cs = __builtin_fma(t.x, cd, -(t.y * sd));
  sn = __builtin_fma(t.y, cd, t.x * sd);
}

// Two independent N(0,1) from one Philox block, table-driven Box–Muller (same uniforms as
// normal_pair: u1 = 2 - d1 in (0, 1], angle 2*pi*(d2 - 1)).
// sqrt(t) for the Box-Muller radius: t = -2 log u1 >= 0 up to the table log's rounding at u1 = 1
// (probability 2^-52), so one v_max against a tiny floor replaces fast_sqrt's zero test and its
// two selects (radius 2^-500 instead of 0 there).
__device__ __forceinline__ double bm_sqrt(double t) {
  t = __builtin_fmax(t, 0x1p-1000);
  const double y = __builtin_amdgcn_rsq(t);
  double g = t * y, h = 0.5 * y;
  const double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  const double d = __builtin_fma(-g, g, t);
  return __builtin_fma(d, h, g);
}

__device__ __forceinline__ void normal_pair_tab(uint4 r, const double* tab, double& z0, double& z1) {
  const double u1 = 2.0 - one_to_two(r.x, r.y);
  const double rad = bm_sqrt(-2.0 * table_log(u1, tab));
  double c, s;
  table_cossin(one_to_two(r.z, r.w), tab, c, s);
  z0 = rad * c;
  z1 = rad * s;
}

// Uniform integer in [lo, hi) from one word (multiply-shift; bias <= (hi-lo)/2^32).
__device__ __forceinline__ int uniform_int(uint32_t w, int lo, int hi) {
  return lo + (int)(((uint64_t)w * (uint32_t)(hi - lo)) >> 32);
}

// Sum over the LPC lanes of a group; every lane of the group receives the total.
// `s` = lane index inside the group, `base` = wave lane of the group's first lane.
__device__ __forceinline__ double group_sum(double v, int s, int lpc, int base) {
  for (int off = 1; off < lpc; off <<= 1) {
    const double o = __shfl_down(v, off, kWave);
    if (s + off < lpc) v += o;
  }
  return __shfl(v, base, kWave);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Load / store coordinate pair k of a row (16-B vector access when D is even).
__device__ __forceinline__ void load_pair(const double* __restrict__ row, int k, bool even, bool v1,
                                          double& a, double& b) {
  if (even) {
    const double2 x = *reinterpret_cast<const double2*>(row + 2 * k);
    a = x.x;
    b = x.y;
  } else {
    a = row[2 * k];
    b = v1 ? row[2 * k + 1] : 0.0;
  }
}

__device__ __forceinline__ void store_pair(double* __restrict__ row, int k, bool even, bool v1, double a,
                                           double b) {
  if (even) {
    *reinterpret_cast<double2*>(row + 2 * k) = make_double2(a, b);
  } else {
    row[2 * k] = a;
    if (v1) row[2 * k + 1] = b;
  }
}

// Same as store_pair with non-temporal stores (q_chain sample rows: written once, read back only
// by the diagnostics after the run, so they should not displace cached lines).
__device__ __forceinline__ void store_pair_nt(double* __restrict__ row, int k, bool even, bool v1, double a,
                                              double b) {
  if (even) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(d2v{a, b}, reinterpret_cast<d2v*>(row + 2 * k));
  } else {
    __builtin_nontemporal_store(a, row + 2 * k);
    if (v1) __builtin_nontemporal_store(b, row + 2 * k + 1);
  }
}

// ---- full-wave fp64 sum with DPP (no LDS traffic): row_shr 1/2/4/8 prefix inside each
// 16-lane row, then row_bcast15 / row_bcast31 fold the rows; lane 63 holds the total, which
// v_readlane turns into a wave-uniform (SGPR) value.  EXEC must be all ones at the call.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp0(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xF, true);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// DPP move with an undefined old value: lanes a masked row leaves unwritten hold garbage.  Only
// lane 63 is read at the end, and every step writes it, so no zero-initialising moves are needed
// before the two row_bcast steps (4 VALU per reduction).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_u(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, ROW_MASK, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, ROW_MASK, 0xF, true);
  return __hiloint2double(hi, lo);
}

// The DPP chain alone: lane 63 holds the full-wave sum, other lanes partial sums.  Callers that
// only compare the total (the Metropolis test) finish the arithmetic in lane 63 and read the
// decision from the compare mask, with no readlane / v_mov round trip.
__device__ __forceinline__ double wave_sum_dpp_l63(double v) {
  v += dpp_u<0x111>(v);        // row_shr:1 (bound_ctrl: lanes shifted in from outside the row read 0)
  v += dpp_u<0x112>(v);        // row_shr:2
  v += dpp_u<0x114>(v);        // row_shr:4
  v += dpp_u<0x118>(v);        // row_shr:8
  v += dpp_u<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
  v += dpp_u<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ __forceinline__ double wave_sum_dpp(double v) { return readlane_d(wave_sum_dpp_l63(v), 63); }

// Two full-wave sums for the price of one (18 VALU instead of 36): one v_permlane32_swap per
// 32-bit half puts lanes 0-31 of `a` and of `b` side by side (and lanes 32-63 in the other
// result), so one add leaves a's pair sums in lanes 0-31 and b's in lanes 32-63; the row_shr
// prefix steps and one row_bcast:15 (into rows 1 and 3 only) then finish both halves at once.
// Lane 31 holds sum(a), lane 63 holds sum(b); other lanes hold partial sums.  EXEC all ones.
__device__ __forceinline__ double wave_sum2_dpp(double a, double b) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  double v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  v += dpp_u<0x111>(v);        // row_shr:1
  v += dpp_u<0x112>(v);        // row_shr:2
  v += dpp_u<0x114>(v);        // row_shr:4
  v += dpp_u<0x118>(v);        // row_shr:8
  v += dpp_u<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
  return v;
}

// Lane 63's bit of a compare mask as a wave-uniform bool (EXEC must be all ones): the sign of the
// mask's bit 63, tested on the SALU (written in C the compiler emits a VALU 64-bit compare of the
// SGPR pair for it and for its negation).
__device__ __forceinline__ bool lane63(uint64_t mask) {
  int r;
  asm("s_bitcmp1_b64 %1, 63\n\ts_cselect_b32 %0, 1, 0" : "=s"(r) : "s"(mask) : "scc");
  return r != 0;
}
// Lane 31's bit (where wave_sum2_dpp leaves its first sum) as 0/1 in an SGPR, on the SALU as
// lane63 (callers count it with scalar adds: a C bool -> int conversion compiles to v_cndmask).
__device__ __forceinline__ uint32_t lane31(uint64_t mask) {
  uint32_t r;
  asm("s_bitcmp1_b64 %1, 31\n\ts_cselect_b32 %0, 1, 0" : "=s"(r) : "s"(mask) : "scc");
  return r;
}

// Parks v (valid in lane 63, where a DPP reduction leaves its total) in lane n of buf: two
// ds_bpermute reads broadcast lane 63 over the LDS crossbar and the lane mask 1 << n is formed on
// the SALU, so the park costs two v_cndmask (VALU) instead of two v_readlane plus a compare and
// two selects.  (gfx950 has no wave-wide DPP rotate: wave_ror assembles but moves nothing.)
// bp63: the byte address of lane 63, (kWave - 1) * 4, made opaque once outside the loop (a
// literal lets the compiler turn the permute back into v_readlane + v_mov).
__device__ __forceinline__ double park_lane(double buf, double v, int n, int bp63) {
  const int src = bp63;
  const uint32_t vlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)__double2loint(v));
  const uint32_t vhi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)__double2hiint(v));
  uint64_t m;
  asm("s_lshl_b64 %0, 1, %1" : "=s"(m) : "s"(n) : "scc");
  uint32_t lo = __double2loint(buf), hi = __double2hiint(buf);
  asm("v_cndmask_b32_e64 %0, %0, %2, %4\n\tv_cndmask_b32_e64 %1, %1, %3, %4"
      : "+v"(lo), "+v"(hi)
      : "v"(vlo), "v"(vhi), "s"(m));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

// (a < b) as 0/1 in an SGPR for wave-uniform a, b (the C form goes through v_cndmask + readfirstlane).
__device__ __forceinline__ uint32_t s_lt_i32(int a, int b) {
  uint32_t r;
  asm("s_cmp_lt_i32 %1, %2\n\ts_cselect_b32 %0, 1, 0" : "=s"(r) : "s"(a), "s"(b) : "scc");
  return r;
}

// Wave-uniform max of an int: DPP row_shr 1/2/4/8 then row_bcast 15/31 (each step one VALU max
// with the DPP source; lanes without a source keep their value), lane 63 read back.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_max_step(int v) {
  return max(v, __builtin_amdgcn_update_dpp(v, v, CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ int wave_max_i32(int v) {
  v = dpp_max_step<0x111>(v);
  v = dpp_max_step<0x112>(v);
  v = dpp_max_step<0x114>(v);
  v = dpp_max_step<0x118>(v);
  v = dpp_max_step<0x142, 0xA>(v);
  v = dpp_max_step<0x143, 0xC>(v);
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ double uniform_d(double v) { return readlane_d(v, 0); }

}  // namespace hmc
