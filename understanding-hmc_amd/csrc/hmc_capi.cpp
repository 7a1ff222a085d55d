// hmc_capi.cpp — extern "C" entry points of libhmc.so (declared in include/hmc.h).
//
// Validation mirrors the reference's asserts (samplers.py:331-348, :396) and returns
// HMC_EINVAL instead of raising; the Python mirror re-raises AssertionError.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>

#include "hmc.h"
#include "hmc_internal.hpp"

namespace {

thread_local std::string g_err;
#ifdef HMC_DEBUG_HOOKS
unsigned long long* g_stamps = nullptr;   // HMC_DEBUG_STAMPS diagnostic buffer
int64_t g_stamp_waves = 0;
#endif

hmc_status fail(hmc_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

hmc_status hip_status(hipError_t e, const char* where) {
  if (e == hipSuccess) return HMC_OK;
  return fail(HMC_EHIP, "%s: %s", where, hipGetErrorString(e));
}

// Python floor division (the reference computes (i - warm_up)//thin with Python ints).
int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

hmc_status check_schedule(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, bool random) {
  if (!t || !k || !s) return fail(HMC_EINVAL, "null target/kinetic/schedule");
  if (t->D < 1) return fail(HMC_EINVAL, "D must be >= 1");
  if (t->kind != HMC_TARGET_DIAG && t->kind != HMC_TARGET_DENSE) return fail(HMC_EINVAL, "bad target kind");
  if (t->kind == HMC_TARGET_DENSE && !t->prec) return fail(HMC_EINVAL, "dense target needs prec");
  if (s->n_chains < 0) return fail(HMC_EINVAL, "n_chains < 0");
  if (s->n_iter < 1 || s->thin < 1 || s->warm_up < 0) return fail(HMC_EINVAL, "bad Niter/thin/warm_up");
  const int64_t Lc = 1 + floordiv(s->n_iter - s->warm_up, s->thin);  // samplers.py:31
  if (Lc < 1 || Lc != s->L_chain) return fail(HMC_EINVAL, "L_chain must be 1+(Niter-warm_up)//thin >= 1");
  if (!(std::isfinite(k->dt)) && !k->dt_vec) return fail(HMC_EINVAL, "dt must be set (samplers.py:332)");
  if (random && s->L_high <= s->L_low) return fail(HMC_EINVAL, "L_low must be < L_high (randint)");
  if (random && s->rng_mode == HMC_RNG_PHILOX && s->L_low < 0) return fail(HMC_EINVAL, "L_low < 0");
  if (s->rng_mode != HMC_RNG_REPLAY && s->rng_mode != HMC_RNG_PHILOX) return fail(HMC_EINVAL, "bad rng_mode");
  if (s->fp_mode != HMC_MODE_EXACT && s->fp_mode != HMC_MODE_FAST) return fail(HMC_EINVAL, "bad fp_mode");
  return HMC_OK;
}

// q_chain buffer geometry shared by the Random and NUTS kernels: the kernels index one chain's
// rows with 32-bit row numbers (row % Lq), so a chain's rows must stay within 2 GiB.
hmc_status check_window(const hmc_target* t, const hmc_schedule* s, const hmc_state* st) {
  if (st->qc_rows < 0 || st->qc_row0 < 0) return fail(HMC_EINVAL, "qc_rows, qc_row0 must be >= 0");
  if (st->qc_rows > 0x7FFFFFFFll || st->qc_row0 > 0x7FFFFFFFll) return fail(HMC_EINVAL, "qc_rows/qc_row0 too large");
  if ((st->qc_rows > 0 ? st->qc_rows : (int64_t)s->L_chain) * t->D * 8 > 0x7FFFFFFFll)
    return fail(HMC_ENOTSUP, "one chain's q_chain rows exceed 2 GiB (use a streaming window)");
  return HMC_OK;
}

// Dense mass matrix (full cov_p, samplers.py:352-356): only the dense-target Random kernels take it.
hmc_status check_mass(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s) {
  if (!k->minv_full && !k->p_chol_t && !k->kick) return HMC_OK;
  if (!k->minv_full || !k->kick) return fail(HMC_EINVAL, "dense mass matrix needs minv_full and kick");
  if (k->minv || k->p_scale) return fail(HMC_EINVAL, "dense mass matrix: minv/p_scale must be NULL");
  if (t->kind != HMC_TARGET_DENSE) return fail(HMC_ENOTSUP, "dense mass matrix needs a dense target (pass prec dense)");
  if (s && s->rng_mode == HMC_RNG_PHILOX && !k->p_chol_t)
    return fail(HMC_EINVAL, "dense mass matrix with Philox draws needs p_chol_t");
  return HMC_OK;
}

hmc::RandArgs rand_args(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                        hmc_state* st, const hmc::Layout& lay) {
  hmc::RandArgs a{};
  a.n = s->n_chains;
  a.chain_offset = s->chain_offset;
  a.D = t->D;
  a.npairs = lay.npairs;
  a.lpc = lay.lpc;
  a.cpw = lay.cpw;
  a.niter = s->n_iter;
  a.wu = s->warm_up;
  a.thin = s->thin;
  a.Lc = s->L_chain;
  a.L_low = s->L_low;
  a.L_high = s->L_high;
  a.it0 = s->iter_begin;
  a.it1 = s->iter_end;
  a.ntiles = (s->n_chains + 15) / 16;
  a.i_oob = (int)(s->warm_up - (int64_t)s->L_chain * s->thin);  // rejections at i < i_oob index < -L_chain
  a.k0 = (uint32_t)s->seed;
  a.k1 = (uint32_t)(s->seed >> 32);
  a.dt = k->dt;
  a.h = k->dt * 0.5;
  a.logc = t->logdet_const;
  a.q0 = t->q0;
  a.prec = t->prec;
  a.minv = k->minv;
  a.pscale = k->p_scale;
  a.dtv = k->dt_vec;
  a.minvf = k->minv_full;
  a.cholt = k->p_chol_t;
  a.kick = k->kick;
  if (r) {
    a.rp0 = r->p0;
    a.rp = r->p;
    a.rlnu = r->lnu;
    a.rL = r->L;
  }
  a.q = st->q;
  a.Eprev = st->E_prev;
  a.qc = st->q_chain;
  a.Lq = st->qc_rows > 0 ? (int)st->qc_rows : s->L_chain;
  a.q_row0 = (int)st->qc_row0;
  a.Ec = st->E_chain;
  a.dEc = st->dE_chain;
  a.cnt = st->counters;
  a.dbgL = -1;
#ifdef HMC_DEBUG_HOOKS
  // Profiling experiments only: compiled into the separate debug build (make debug ->
  // lib/libhmc_debug.so), never into the release libhmc.so the product and bench.py load.
  if (const char* ab = getenv("HMC_DEBUG_ABLATE")) a.dbg = atoi(ab);
  if (const char* dl = getenv("HMC_DEBUG_L")) a.dbgL = atoi(dl);
  if (getenv("HMC_DEBUG_STAMPS")) {                                     // diagnostic phase timers
    const int cpw = lay.cpw > 0 ? lay.cpw : 16;   // dense / NUTS layouts: 16 chains per wave
    const int64_t waves = (s->n_chains + cpw - 1) / cpw;
    if (g_stamps) (void)hipFree(g_stamps);
    g_stamps = nullptr;
    g_stamp_waves = waves;
    if (hipMalloc(&g_stamps, waves * hmc::kStampWords * sizeof(unsigned long long)) == hipSuccess) a.stamps = g_stamps;
  }
#endif
  if (st->traj_q && st->traj_len && st->decision && st->n_save > 0) {
    a.traj_q = st->traj_q;
    a.traj_len = st->traj_len;
    a.decision = st->decision;
    a.n_save = st->n_save;
    a.traj_stride = st->traj_stride;
  }
  return a;
}

bool general_diag(const hmc_target* t, const hmc_kinetic* k) {
  return t->q0 || t->prec || k->minv || k->p_scale || k->dt_vec;
}

constexpr int32_t kMaxLags = 1 << 20;   // lag passes of the diagnostics (any n the samples allow)

// Host-side record of the scratch buffers' sizes (device pointer -> bytes): the sized entries
// (*_ws) record what they were given, hmc_workspace_register records a caller's buffer, and every
// entry that takes scratch refuses (HMC_EINVAL) a buffer recorded as smaller than the call needs,
// before any kernel could write past its end.  No device access: the check stays graph-capturable.
std::mutex g_ws_mu;
std::unordered_map<const void*, int64_t> g_ws_bytes;

void ws_record(const void* p, int64_t bytes) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  if (bytes > 0) g_ws_bytes[p] = bytes;
  else g_ws_bytes.erase(p);
}

hmc_status ws_check(const void* p, int64_t need, const char* what) {
  if (!p || need <= 0) return HMC_OK;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  const auto it = g_ws_bytes.find(p);
  if (it != g_ws_bytes.end() && it->second < need)
    return fail(HMC_EINVAL, "%s: scratch buffer of %lld bytes, this call needs %lld", what, (long long)it->second,
                (long long)need);
  return HMC_OK;
}

// Bytes of hmc_state.order this Random-sampler call reads or writes (0: none).
int64_t order_need(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_state* st) {
  if (!st->order || s->n_chains == 0) return 0;
  const bool dense = t->kind == HMC_TARGET_DENSE;
  if (hmc::big_path(dense, t->D)) return hmc::big_workspace_bytes(s->n_chains, t->D, dense, k->minv_full != nullptr);
  return dense ? hmc::dense_workspace_bytes(s->n_chains, t->D) : 0;
}

hmc_status view_too_large(const char* what) {
  return fail(HMC_ENOTSUP,
              "%s: one chain's samples span more than the lag kernel's 1 GiB buffer offsets; pass fewer "
              "dimensions per call (the Python layer splits such views by dimension)", what);
}

}  // namespace

extern "C" {

#ifdef HMC_DEBUG_HOOKS
// Diagnostic: copy the per-wave phase timers of the last HMC_DEBUG_STAMPS launch (debug build only).
int64_t hmc_debug_stamps(unsigned long long* host, int64_t cap_words) {
  if (!g_stamps) return 0;
  const int64_t words = g_stamp_waves * hmc::kStampWords < cap_words ? g_stamp_waves * hmc::kStampWords : cap_words;
  if (hipDeviceSynchronize() != hipSuccess) return 0;
  if (hipMemcpy(host, g_stamps, words * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return words;
}
#endif

const char* hmc_version(void) { return "hmc_amd 0.1.0 gfx950 (diag random kernels, C ABI v1)"; }

const char* hmc_last_error(void) { return g_err.c_str(); }

hmc_status hmc_chain_init(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                          const double* q_start, hmc_state* st, void* stream) {
  if (hmc_status e = check_schedule(t, k, s, false)) return e;
  if (!st) return fail(HMC_EINVAL, "null state");
  if (hmc_status e = check_mass(t, k, s)) return e;
  if (s->n_chains == 0) return HMC_OK;   // empty batch: zero-size buffers may be NULL
  if (!st->q || !st->E_prev || !q_start) return fail(HMC_EINVAL, "null state/q_start");
  const bool replay = s->rng_mode == HMC_RNG_REPLAY;
  if (replay && (!r || !r->p0)) return fail(HMC_EINVAL, "replay mode needs p0");
  if (hmc_status e = ws_check(st->order, order_need(t, k, s, st), "hmc_chain_init: state.order")) return e;
  const bool dense = t->kind == HMC_TARGET_DENSE;
  if (hmc::big_path(dense, t->D)) {   // large D: chain state in the workspace (hmc_big.hip)
    if (!st->order) return fail(HMC_EINVAL, "D=%d needs hmc_random_workspace_size() bytes in state.order", t->D);
    const hmc::Layout lay{0, 0, 0, (t->D + 1) / 2};
    hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
    a.qstart = q_start;
    return hip_status(hmc::launch_big_init(hmc::big_args(a, st->order, dense), dense, replay, (hipStream_t)stream),
                      "hmc_chain_init(large D)");
  }
  if (t->kind == HMC_TARGET_DENSE) {
    const hmc::Layout lay{0, 0, 0, (t->D + 1) / 2};
    hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
    a.qstart = q_start;
    if (st->order) {   // the gradient cache no longer matches q: the next launch recomputes it
      int32_t* valid = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(st->order) +
                                                  hmc::dense_gcache_offset_bytes(s->n_chains) - 16);
      if (hmc_status e = hip_status(hipMemsetAsync(valid, 0, sizeof(int32_t), (hipStream_t)stream), "hmc_chain_init"))
        return e;
    }
    return hip_status(hmc::launch_dense_init(a, replay, (hipStream_t)stream), "hmc_chain_init(dense)");
  }
  const int L_lo = s->L_high > s->L_low ? s->L_low : 5, L_hi = s->L_high > s->L_low ? s->L_high : 20;
  const hmc::Layout lay = hmc::choose_layout(t->D, L_lo, L_hi);
  if (lay.K == 0) return fail(HMC_ENOTSUP, "D=%d too large for the diagonal kernels", t->D);
  hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
  a.qstart = q_start;
  return hip_status(hmc::launch_random_init(a, lay, general_diag(t, k), replay, (hipStream_t)stream),
                    "hmc_chain_init");
}

hmc_status hmc_random_iters(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                            hmc_state* st, void* stream) {
  if (hmc_status e = check_schedule(t, k, s, true)) return e;
  if (!st) return fail(HMC_EINVAL, "null state");
  if (hmc_status e = check_window(t, s, st)) return e;
  if (hmc_status e = check_mass(t, k, s)) return e;
  if (s->iter_begin < 1 || s->iter_end < s->iter_begin || s->iter_end > s->n_iter + 1)
    return fail(HMC_EINVAL, "iteration range must satisfy 1 <= begin <= end <= Niter+1");
  if (s->n_chains == 0) return HMC_OK;   // empty batch: zero-size buffers may be NULL
  if (!st->q || !st->E_prev) return fail(HMC_EINVAL, "null state");
  const bool replay = s->rng_mode == HMC_RNG_REPLAY;
  if (replay && (!r || !r->p || !r->L || !r->lnu)) return fail(HMC_EINVAL, "replay mode needs p, L, lnu");
  if (s->n_chains == 0 || s->iter_end == s->iter_begin) return HMC_OK;
  if (st->n_save > 0 && st->traj_q && st->traj_stride < s->L_high)
    return fail(HMC_EINVAL, "traj_stride must be >= L_high");
  if (hmc_status e = ws_check(st->order, order_need(t, k, s, st), "hmc_random_iters: state.order")) return e;
  const bool dense = t->kind == HMC_TARGET_DENSE;
  if (hmc::big_path(dense, t->D)) {   // large D (hmc_big.hip)
    if (!st->order) return fail(HMC_EINVAL, "D=%d needs hmc_random_workspace_size() bytes in state.order", t->D);
    const hmc::Layout lay{0, 0, 0, (t->D + 1) / 2};
    hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
    return hip_status(hmc::launch_big_iters(hmc::big_args(a, st->order, dense), dense,
                                            s->fp_mode == HMC_MODE_EXACT, replay, (hipStream_t)stream),
                      "hmc_random_iters(large D)");
  }
  if (t->kind == HMC_TARGET_DENSE) {
    const hmc::Layout lay{0, 0, 0, (t->D + 1) / 2};
    hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
    const bool exact = s->fp_mode == HMC_MODE_EXACT;
    int32_t* gvalid = nullptr;
    if (st->order) {   // gradient cache in the workspace (hmc_random_workspace_size)
      char* base = reinterpret_cast<char*>(st->order);
      gvalid = reinterpret_cast<int32_t*>(base + hmc::dense_gcache_offset_bytes(s->n_chains) - 16);
      a.gcache = reinterpret_cast<double*>(base + hmc::dense_gcache_offset_bytes(s->n_chains));
      a.gvalid = gvalid;
    }
    // every launch leaves the cache holding the gradient at each chain's q
    auto mark_valid = [&]() -> hmc_status {
      return gvalid ? hip_status(hipMemsetAsync(gvalid, 1, 1, (hipStream_t)stream), "hmc_random_iters") : HMC_OK;
    };
    if (!st->order || a.traj_q || !hmc::dense_order_ok(a)) {
      if (hmc_status e = hip_status(hmc::launch_dense_iters(a, exact, replay, (hipStream_t)stream),
                                    "hmc_random_iters(dense)"))
        return e;
      return mark_valid();
    }
    // L-ordered tiles: one launch per iteration, chains counting-sorted by that iteration's L
    for (int it = s->iter_begin; it < s->iter_end; ++it) {
      if (hmc_status e = hip_status(hmc::launch_dense_order(a, it, replay, st->order, (hipStream_t)stream),
                                    "hmc_random_iters(dense order)"))
        return e;
      a.it0 = it;
      a.it1 = it + 1;
      a.order = st->order;
      if (hmc_status e = hip_status(hmc::launch_dense_iters(a, exact, replay, (hipStream_t)stream),
                                    "hmc_random_iters(dense)"))
        return e;
      if (hmc_status e = mark_valid()) return e;
    }
    return HMC_OK;
  }
  const hmc::Layout lay = hmc::choose_layout(t->D, s->L_low, s->L_high);
  if (lay.K == 0) return fail(HMC_ENOTSUP, "D=%d too large for the diagonal kernels", t->D);
  hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
  // the kernels keep per-launch tallies in 32 bits: Sum L^2 over one launch must stay < 2^31
  // (only very long trajectories, e.g. L_high = 200, with thousands of iterations split here)
  const int64_t lmax = std::max<int64_t>(std::max(s->L_high, 1), a.dbgL > 0 ? a.dbgL : 1);
  const int64_t chunk = std::max<int64_t>(1, 0x7FFFFFFFll / (lmax * lmax));
  for (int it = s->iter_begin; it < s->iter_end;) {
    const int end = (int)std::min<int64_t>(s->iter_end, it + chunk);
    a.it0 = it;
    a.it1 = end;
    if (hmc_status e = hip_status(hmc::launch_random_iters(a, lay, s->fp_mode == HMC_MODE_EXACT, general_diag(t, k),
                                                           replay, (hipStream_t)stream),
                                  "hmc_random_iters"))
      return e;
    it = end;
  }
  return HMC_OK;
}

int64_t hmc_random_workspace_size_ex(const hmc_target* t, const hmc_kinetic* k, int64_t n_chains) {
  if (!t || n_chains < 0 || t->D < 1) return 0;
  const bool dense = t->kind == HMC_TARGET_DENSE;
  if (hmc::big_path(dense, t->D)) return hmc::big_workspace_bytes(n_chains, t->D, dense, !k || k->minv_full);
  if (!dense) return 0;
  return hmc::dense_workspace_bytes(n_chains, t->D);
}

int64_t hmc_random_workspace_size(const hmc_target* t, int64_t n_chains) {
  return hmc_random_workspace_size_ex(t, nullptr, n_chains);   // enough for either cov_p
}

int64_t hmc_nuts_workspace_size_ex(int32_t D, int64_t n_chains, int32_t d_max, int32_t iters_per_call,
                                   int32_t philox_momenta) {
  if (D < 1 || n_chains < 0 || d_max < 1 || d_max > hmc::kNutsDmaxMax || iters_per_call < 1) return 0;
  if (hmc::nuts_lock_path(D)) {   // philox_momenta 0: replay tapes, or a full cov_p (its fragments too)
    return (philox_momenta ? hmc::nuts_lock_ws_doubles(n_chains, D, d_max, false)
                           : hmc::nuts_lock_ws_doubles(n_chains, D, d_max, true)) *
           (int64_t)sizeof(double);
  }
  if (!hmc::dense_tiles(D)) return hmc::nuts_big_ws_doubles(n_chains, D, d_max) * (int64_t)sizeof(double);
  return hmc::nuts_ws_doubles(n_chains, D, d_max, philox_momenta ? iters_per_call : 0) * (int64_t)sizeof(double);
}

int64_t hmc_nuts_workspace_size(int32_t D, int64_t n_chains, int32_t d_max) {
  return std::max(hmc_nuts_workspace_size_ex(D, n_chains, d_max, 32, 1),
                  hmc_nuts_workspace_size_ex(D, n_chains, d_max, 32, 0));
}

// Bytes of NUTS workspace this call needs (0: nothing to run, -1: unsupported shape).
static int64_t nuts_need(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s) {
  if (s->iter_end <= s->iter_begin || s->n_chains == 0) return 0;
  // its Philox momenta drawn ahead (diagonal cov_p) for this call's iterations, or the tree vectors
  // of the kernel this call takes
  const int32_t pm = s->rng_mode == HMC_RNG_PHILOX && !k->minv_full ? 1 : 0;
  const int64_t need = hmc_nuts_workspace_size_ex(t->D, s->n_chains, s->d_max, s->iter_end - s->iter_begin, pm);
  return need > 0 ? need : -1;
}

hmc_status hmc_workspace_register(const void* workspace, int64_t bytes) {
  if (!workspace || bytes < 0) return fail(HMC_EINVAL, "hmc_workspace_register: null pointer or negative size");
  ws_record(workspace, bytes);
  return HMC_OK;
}

hmc_status hmc_chain_init_ws(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                             const double* q_start, hmc_state* st, int64_t order_bytes, void* stream) {
  if (hmc_status e = check_schedule(t, k, s, false)) return e;
  if (!st) return fail(HMC_EINVAL, "null state");
  if (!k) return fail(HMC_EINVAL, "null kinetic");
  const int64_t need = order_need(t, k, s, st);
  if (order_bytes < need)
    return fail(HMC_EINVAL, "hmc_chain_init_ws: state.order of %lld bytes, this call needs %lld "
                "(hmc_random_workspace_size_ex)", (long long)order_bytes, (long long)need);
  if (st->order) ws_record(st->order, order_bytes);
  return hmc_chain_init(t, k, s, r, q_start, st, stream);
}

hmc_status hmc_random_iters_ws(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                               hmc_state* st, int64_t order_bytes, void* stream) {
  if (hmc_status e = check_schedule(t, k, s, true)) return e;
  if (!st) return fail(HMC_EINVAL, "null state");
  if (!k) return fail(HMC_EINVAL, "null kinetic");
  const int64_t need = order_need(t, k, s, st);
  if (order_bytes < need)
    return fail(HMC_EINVAL, "hmc_random_iters_ws: state.order of %lld bytes, this call needs %lld "
                "(hmc_random_workspace_size_ex)", (long long)order_bytes, (long long)need);
  if (st->order) ws_record(st->order, order_bytes);
  return hmc_random_iters(t, k, s, r, st, stream);
}

hmc_status hmc_nuts_iters_ws(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                             hmc_state* st, void* workspace, int64_t workspace_bytes, void* stream) {
  if (hmc_status e = check_schedule(t, k, s, false)) return e;   // also rejects a NULL k
  if (s->d_max < 1 || s->d_max > hmc::kNutsDmaxMax) return fail(HMC_EINVAL, "d_max must be in [1, %d]", hmc::kNutsDmaxMax);
  const int64_t need = nuts_need(t, k, s);
  if (need < 0) return fail(HMC_EINVAL, "NUTS workspace: unsupported D=%d / d_max=%d", t->D, s->d_max);
  if (workspace_bytes < need)
    return fail(HMC_EINVAL, "NUTS workspace of %lld bytes; this call (D=%d, %lld chains, d_max=%d, %d iterations, "
                "%s momenta) needs %lld (hmc_nuts_workspace_size_ex)", (long long)workspace_bytes, t->D,
                (long long)s->n_chains, s->d_max, s->iter_end - s->iter_begin,
                s->rng_mode == HMC_RNG_PHILOX && !k->minv_full ? "Philox" : "no pre-drawn", (long long)need);
  ws_record(workspace, workspace_bytes);
  return hmc_nuts_iters(t, k, s, r, st, workspace, stream);
}

hmc_status hmc_nuts_iters(const hmc_target* t, const hmc_kinetic* k, const hmc_schedule* s, const hmc_replay* r,
                          hmc_state* st, void* workspace, void* stream) {
  if (hmc_status e = check_schedule(t, k, s, false)) return e;
  if (!st) return fail(HMC_EINVAL, "null state");
  if (hmc_status e = check_window(t, s, st)) return e;
  if (s->iter_begin < 1 || s->iter_end < s->iter_begin || s->iter_end > s->n_iter + 1)
    return fail(HMC_EINVAL, "iteration range must satisfy 1 <= begin <= end <= Niter+1");
  if (s->n_chains == 0) return HMC_OK;   // empty batch: zero-size buffers may be NULL
  if (!st->q || !st->E_prev) return fail(HMC_EINVAL, "null state");
  if (s->d_max < 1 || s->d_max > hmc::kNutsDmaxMax) return fail(HMC_EINVAL, "d_max must be in [1, %d]", hmc::kNutsDmaxMax);
  if (hmc_status e = check_mass(t, k, s)) return e;
  if (t->kind != HMC_TARGET_DENSE) return fail(HMC_ENOTSUP, "NUTS runs the dense kernel: pass prec as dense");
  const bool big = !hmc::dense_tiles(t->D);   // D > 128: hmc_nuts_big.hip
  const bool replay = s->rng_mode == HMC_RNG_REPLAY;
  if (replay && (!r || !r->p || !r->tape || r->tape_stride < 1)) return fail(HMC_EINVAL, "replay mode needs p and tape");
  if (s->n_chains == 0 || s->iter_end == s->iter_begin) return HMC_OK;
  if (!workspace) return fail(HMC_EINVAL, "null workspace");
  {
    const int64_t need = nuts_need(t, k, s);
    if (need < 0) return fail(HMC_EINVAL, "NUTS workspace: unsupported D=%d / d_max=%d", t->D, s->d_max);
    if (hmc_status e = ws_check(workspace, need, "hmc_nuts_iters: workspace")) return e;
  }
  const hmc::Layout lay{0, 0, 16, (t->D + 1) / 2};   // 16 chain slots per wave (debug stamps: one row per wave)
  hmc::RandArgs a = rand_args(t, k, s, replay ? r : nullptr, st, lay);
  a.d_max = s->d_max;
  a.on_dmax = s->on_dmax;
  a.ws = static_cast<double*>(workspace);
  if (replay) {
    a.tape = r->tape;
    a.tape_stride = r->tape_stride;
  }
  a.traj_q = nullptr;
  a.n_save = 0;
  if (big && hmc::nuts_lock_path(t->D))   // 128 < D <= 320: lockstep 16-chain blocks (any cov_p)
    return hip_status(hmc::launch_nuts_lock(a, s->fp_mode == HMC_MODE_EXACT, replay, (hipStream_t)stream),
                      "hmc_nuts_iters(lockstep)");
  if (big) return hip_status(hmc::launch_nuts_big(a, s->fp_mode == HMC_MODE_EXACT, replay, (hipStream_t)stream),
                             "hmc_nuts_iters(large D)");
  return hip_status(hmc::launch_nuts_iters(a, s->fp_mode == HMC_MODE_EXACT, replay, (hipStream_t)stream),
                    "hmc_nuts_iters");
}

hmc_status hmc_leapfrog(const hmc_target* t, const hmc_kinetic* k, int64_t n, const double* p, const double* q,
                        double* p_out, double* q_out, int32_t fp_mode, void* stream) {
  if (!t || !k || t->D < 1 || n < 0) return fail(HMC_EINVAL, "bad arguments");
  if (n > 0 && (!p || !q || !p_out || !q_out)) return fail(HMC_EINVAL, "null row pointers");
  if (p_out == p || q_out == q || p_out == q || q_out == p) return fail(HMC_EINVAL, "outputs alias inputs");
  hmc::RowArgs a{};
  a.n = n;
  a.D = t->D;
  a.dense = t->kind == HMC_TARGET_DENSE;
  a.q0 = t->q0;
  a.prec = t->prec;
  if (hmc_status e = check_mass(t, k, nullptr)) return e;
  a.minv = k->minv;
  a.minvf = k->minv_full;
  a.dtv = k->dt_vec;
  a.dt = k->dt;
  a.logc = t->logdet_const;
  a.p = p;
  a.q = q;
  a.po = p_out;
  a.qo = q_out;
  return hip_status(hmc::launch_leapfrog_rows(a, fp_mode == HMC_MODE_EXACT, (hipStream_t)stream), "hmc_leapfrog");
}

hmc_status hmc_energy(const hmc_target* t, const hmc_kinetic* k, int64_t n, const double* q, const double* p,
                      double* E_out, void* stream) {
  if (!t || !k || t->D < 1 || n < 0) return fail(HMC_EINVAL, "bad arguments");
  if (n > 0 && (!p || !q || !E_out)) return fail(HMC_EINVAL, "null row pointers");
  hmc::RowArgs a{};
  a.n = n;
  a.D = t->D;
  a.dense = t->kind == HMC_TARGET_DENSE;
  a.q0 = t->q0;
  a.prec = t->prec;
  if (hmc_status e = check_mass(t, k, nullptr)) return e;
  a.minv = k->minv;
  a.minvf = k->minv_full;
  a.logc = t->logdet_const;
  a.p = p;
  a.q = q;
  a.E = E_out;
  return hip_status(hmc::launch_energy_rows(a, (hipStream_t)stream), "hmc_energy");
}

hmc_status hmc_rng_normals(uint64_t seed, int64_t chain0, int64_t n, int32_t iteration, int32_t npairs, double* out,
                           void* stream) {
  if (n < 0 || npairs < 0 || iteration < 0) return fail(HMC_EINVAL, "bad arguments");
  if (n * npairs > 0 && !out) return fail(HMC_EINVAL, "null out");
  return hip_status(hmc::launch_rng_normals((uint32_t)seed, (uint32_t)(seed >> 32), chain0, n, iteration, npairs,
                                            out, (hipStream_t)stream),
                    "hmc_rng_normals");
}

hmc_status hmc_philox(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t k0, uint32_t k1, int64_t n,
                      uint32_t* out, void* stream) {
  if (n < 0 || (n > 0 && !out)) return fail(HMC_EINVAL, "bad arguments");
  return hip_status(hmc::launch_philox(make_uint4(x0, x1, x2, x3), k0, k1, n, out, (hipStream_t)stream),
                    "hmc_philox");
}

int64_t hmc_rowsum_work_size(int64_t rows, int32_t D) { return hmc::diag_rowsum_work(rows, D); }

int64_t hmc_variogram_work_size(int64_t n_chains, int32_t D, int32_t nlags) {
  return hmc::diag_variogram_work(n_chains, D, nlags);
}

hmc_status hmc_split_moments(const double* x, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                             int64_t base, int32_t n, int32_t D, double* mean_out, double* std_out, void* stream) {
  if (!x || !mean_out || !std_out || n_chains < 1 || n < 1 || D < 1) return fail(HMC_EINVAL, "bad arguments");
  return hip_status(hmc::launch_split_moments(x, n_chains, chain_stride, sample_stride, base, n, D, mean_out,
                                              std_out, (hipStream_t)stream),
                    "hmc_split_moments");
}

hmc_status hmc_rowsum(const double* x, int64_t n_outer, int64_t outer_stride, int64_t n_inner, int64_t inner_stride,
                      int64_t base, int32_t D, const double* center, double* work, double* out, void* stream) {
  if (!x || !work || !out || n_outer < 1 || n_inner < 1 || D < 1) return fail(HMC_EINVAL, "bad arguments");
  return hip_status(hmc::launch_rowsum(x, n_outer, outer_stride, n_inner, inner_stride, base, D, center, work, out,
                                       (hipStream_t)stream),
                    "hmc_rowsum");
}

hmc_status hmc_variogram(const double* x, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                         int64_t base, int32_t n, int32_t D, int32_t t0, int32_t t1, double* work, double* out,
                         void* stream) {
  if (!x || !work || !out || n_chains < 1 || n < 1 || D < 1 || t0 < 1 || t1 <= t0 || t1 - t0 > kMaxLags)
    return fail(HMC_EINVAL, "bad arguments (1 <= t0 < t1, t1 - t0 <= %d)", kMaxLags);
  if (!hmc::diag_view_ok(n_chains, chain_stride, sample_stride, n, D, 2, 0, 0)) return view_too_large("hmc_variogram");
  return hip_status(hmc::launch_variogram(x, n_chains, chain_stride, sample_stride, base, n, D, t0, t1, work, out,
                                          (hipStream_t)stream),
                    "hmc_variogram (the view must keep one chain's samples within 1 GiB, include/hmc.h)");
}

static bool conv_tmax_ok(int32_t t) { return t >= 1 && t <= kMaxLags; }

int64_t hmc_convergence_work_size(int64_t n_chains, int32_t D, int32_t tmax) {
  if (n_chains < 1 || D < 1 || !conv_tmax_ok(tmax)) return 0;
  return hmc::diag_conv_work(n_chains, D, tmax);
}

hmc_status hmc_convergence_sums(const double* x, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                                int64_t base, int32_t n, int32_t D, int32_t tmax, double* work, double* out,
                                void* stream) {
  if (!x || !work || !out || n_chains < 1 || n < 2 || D < 1) return fail(HMC_EINVAL, "bad arguments");
  if (!conv_tmax_ok(tmax)) return fail(HMC_EINVAL, "tmax must be in 1 .. %d", kMaxLags);
  if (!hmc::diag_view_ok(n_chains, chain_stride, sample_stride, n, D, 2, 0, 0))
    return view_too_large("hmc_convergence_sums");
  return hip_status(hmc::launch_conv_fused(x, n_chains, chain_stride, sample_stride, base, n, D, tmax, work, out,
                                           (hipStream_t)stream),
                    "hmc_convergence_sums");
}

hmc_status hmc_half_sums(const double* window, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                         int32_t D, int32_t wrap, int32_t slot0, int32_t n, int32_t tmax, double* work, double* out,
                         void* stream) {
  if (!window || !work || !out || n_chains < 1 || n < 2 || D < 1 || slot0 < 0 || wrap < 0 ||
      (wrap > 0 && (slot0 >= wrap || n > wrap)))
    return fail(HMC_EINVAL, "bad arguments");
  if (!conv_tmax_ok(tmax)) return fail(HMC_EINVAL, "tmax must be in 1 .. %d", kMaxLags);
  if (!hmc::diag_view_ok(n_chains, chain_stride, sample_stride, n, D, 1, wrap, slot0))
    return view_too_large("hmc_half_sums");
  return hip_status(hmc::launch_half_sums(window, n_chains, chain_stride, sample_stride, D, wrap, slot0, n, tmax, work,
                                          out, (hipStream_t)stream),
                    "hmc_half_sums");
}

int64_t hmc_stream_work_size(int64_t n_chains, int32_t D, int32_t tmax) {
  if (n_chains < 1 || D < 1 || (tmax != 8 && tmax != 16 && tmax != 32 && tmax != 64)) return 0;
  return hmc::diag_stream_groups(n_chains) * (int64_t)tmax * D;
}

hmc_status hmc_stream_accumulate(const double* window, int64_t n_chains, int64_t chain_stride, int64_t sample_stride,
                                 int32_t D, int32_t wrap, int32_t slot0, int32_t carry, int32_t rows, int64_t pos0,
                                 int32_t n_half, double* shift, double* s1, double* s2, int32_t tmax, double* work,
                                 double* vsum, void* stream) {
  if (!window || !shift || !s1 || !s2 || !work || !vsum || n_chains < 1 || D < 1 || rows < 0 || carry < 0 ||
      n_half < 2 || pos0 < 0 || wrap < 1 || slot0 < 0 || slot0 >= wrap || carry + rows > wrap)
    return fail(HMC_EINVAL, "bad arguments");
  if (tmax != 8 && tmax != 16 && tmax != 32 && tmax != 64) return fail(HMC_EINVAL, "tmax must be 8, 16, 32 or 64");
  if (carry < (pos0 < tmax ? pos0 : tmax)) return fail(HMC_EINVAL, "carry must be >= min(tmax, pos0)");
  if (rows == 0) return HMC_OK;
  return hip_status(hmc::launch_stream_accum(window, n_chains, chain_stride, sample_stride, D, wrap, slot0, carry, rows,
                                             pos0, n_half, shift, s1, s2, tmax, work, vsum, (hipStream_t)stream),
                    "hmc_stream_accumulate");
}

}  // extern "C"
