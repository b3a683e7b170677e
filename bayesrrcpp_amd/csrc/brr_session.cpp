// brr_session.cpp -- host driver and C ABI (include/brr.h) of the MI355X Gibbs sampler.
//
// One brr_session = one chain on one GPU (one column shard).  Everything numeric runs in the
// HIP kernels of brr_kernels.hip; the host only orders launches, moves data at the boundary,
// and (for the reference visit order only) replays glibc rand() + std::random_shuffle.
// There is no CPU compute fallback: without a usable HIP device every entry point fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>


#include <rccl/rccl.h>

#include "../../include/brr.h"
#include "brr_device.hpp"
#include "brr_launch.hpp"
#include "brr_rng.hpp"
#include "brr_sample.hpp"

using namespace brr;

namespace {

thread_local std::string g_last_error;

struct Logger {
  brr_log_fn fn = nullptr;
  void *user = nullptr;
  void operator()(const char *fmt, ...) const {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (fn) fn(buf, user); else fputs(buf, stderr);
  }
};

#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      set_error("HIP error %s at %s:%d: %s", hipGetErrorString(e_), __FILE__, __LINE__, \
                #expr);                                                                \
      return -2;                                                                       \
    }                                                                                  \
  } while (0)

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

// glibc rand() (random_r TYPE_3) from a fresh-process state, and libstdc++'s
// std::random_shuffle (/usr/include/c++/11/bits/stl_algo.h:4568-4582) -- the reference's
// visit order (BayesRv2.cpp:182), used by BRR_ORDER_REFERENCE.
struct GlibcRand {
  int32_t r[34];
  int idx = 0;
  void seed(uint32_t s) {
    int32_t x[344];
    if (s == 0) s = 1;
    x[0] = (int32_t)s;
    for (int i = 1; i < 31; ++i) {
      const int32_t hi = x[i - 1] / 127773, lo = x[i - 1] % 127773;
      int32_t word = 16807 * lo - 2836 * hi;
      if (word < 0) word += 2147483647;
      x[i] = word;
    }
    for (int i = 31; i < 34; ++i) x[i] = x[i - 31];
    for (int i = 34; i < 344; ++i) x[i] = (int32_t)((uint32_t)x[i - 31] + (uint32_t)x[i - 3]);
    for (int i = 0; i < 34; ++i) r[i] = x[310 + i];
    idx = 0;
  }
  int32_t next() {
    const int32_t v = (int32_t)((uint32_t)r[(idx + 3) % 34] + (uint32_t)r[(idx + 31) % 34]);
    r[idx] = v;
    idx = (idx + 1) % 34;
    return (int32_t)((uint32_t)v >> 1);
  }
  void shuffle(std::vector<int32_t> &a) {
    for (size_t i = 1; i < a.size(); ++i) {
      const size_t j = (size_t)(next() % (int32_t)(i + 1));
      if (i != j) std::swap(a[i], a[j]);
    }
  }
};

template <class T>
int dalloc(T **p, int64_t n) {
  *p = nullptr;
  if (n <= 0) n = 1;
  hipError_t e = hipMalloc((void **)p, sizeof(T) * (size_t)n);
  if (e != hipSuccess) {
    // clear the runtime's sticky last error: a later launcher that returns hipGetLastError() (e.g.
    // launch_slab_sentinels) would otherwise report this failed allocation as its own launch failure
    (void)hipGetLastError();
    set_error("hipMalloc(%lld bytes) failed: %s", (long long)(sizeof(T) * n), hipGetErrorString(e));
    return -2;
  }
  return 0;
}

}  // namespace

// sample output ring (brr_sample.hpp)
struct SampleRing {
  int depth = 0;
  hipStream_t cst = nullptr;  // copy stream (device -> pinned host)
  size_t bytes = 0, o_beta = 0, o_eps = 0, o_lam = 0, o_sgg = 0, o_alpha = 0, o_comp = 0;
  std::vector<char *> dbuf, hbuf;
  std::vector<hipEvent_t> ev_snap, ev_host;
  std::vector<char> busy;
  int next = 0, in_use = 0, max_in_use = 0;
  std::mutex mu;
  std::condition_variable cv;
};

struct brr_session {
  brr_options opt;
  Logger log;
  Dev d{};
  int device = 0;
  hipStream_t st = nullptr;
  hipStream_t st_side = nullptr;  // two-kernel fused sweep: the streaming kernel's stream
  hipEvent_t ev_go = nullptr, ev_done = nullptr;
  int sbase = 0, gbase[NPAR] = {}, abase = 0;  // hand-over counter epochs (see SyncWord)
  FusedCfg fused;       // fused persistent sweep (nsg == 0: per-block kernels)
  int64_t N = 0, M = 0, M_total = 0, col_offset = 0;
  int K = 1, G = 1, F = 0, B = 128, nb = 0, model = 0, NS = 0;
  int order_mode = BRR_ORDER_BLOCKED;
  int shard = 0, nshard = 1;
  int nex = 1, seg = 0;         // column shards: exchanges per sweep, the sweep's current segment
  int rshard = 0, nrshard = 1;  // exact row shards: this session's rank / count
  hipEvent_t ev_x = nullptr;    // row shards in one process (brr_group): cross-stream ordering
  int32_t iteration = 0;
  bool init_pending = false;  // column-shard restart between init_local and init_finish
  bool initialized = false, pi_given = false, need_reduce = false, have_y = false, have_x = false;
  bool x2bit = false;  // genotype storage: 2-bit codes (opt.x_storage == BRR_X_2BIT)
  int *cls_flags = nullptr;  // k_classes: [0] a column is not class-coded, [1] max classes per column
  uint8_t *gram_codes = nullptr;  // k_gram_int's input: class codes of the current Gram layout
  uint8_t *xcls = nullptr;        // REFERENCE order: column-major class codes (Dev::xcls)
  int gram_np_init = 0;           // the Gram kernel of the latest init (Dev::gram_np then)
  int ovs_last = 0;               // the latest fused launch ran the overlapped solver (brr_ovsolve.hpp)
  double mu0 = 0, sigmaE0 = 0;
  double *ex_eps = nullptr, *ex_stats = nullptr;  // exchange buffers (caller- or session-owned)
  bool ex_owned = false;
  std::vector<double> synth_y;  // this shard's X_causal beta_causal (synthetic cohort)
  ncclComm_t comm = nullptr;
  // reference visit order state (owned by the shuffle-ahead thread once it runs, RefAhead)
  GlibcRand grand;
  std::vector<int32_t> ref_order, ref_forder;
  // REFERENCE order: the next sweep's permutation is shuffled on a host thread while the device runs
  // the current sweep (the glibc stream does not depend on the chain); the sweep takes it
  struct RefAhead {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool want = false, have = false, stop = false;
    std::vector<int32_t> visit, forder;  // the next sweep's: this shard's visit order, fixedI
  } ahead;
  std::vector<int32_t> cur_visit, cur_forder;  // the current sweep's (alive while its copies are in flight)
  int32_t *ref_pin[2] = {nullptr, nullptr};  // pinned member buffers of upload_order
  hipEvent_t ref_ev[2] = {nullptr, nullptr};
  int ref_k = 0;
  bool ref_static = false;  // block sizes and in-block indices of the REFERENCE layout uploaded
  int census_failures = 0;  // fused sweeps whose residency census failed (the session then runs per block)
  // timing
  bool timing = false;
  bool prof_on = false;  // diagnostics timers on (scalar 102): the streaming kernel's diagnostics variant
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  // (start event index, kind: 0 = k_stream, 1 = k_solve, 2 = solver per sweep, >= 3: a marker-loop
  // launch over kind - 3 block positions -- the fused sweep, an exchange segment of it, the row-shard loop)
  std::vector<std::pair<size_t, int>> ev_pairs;
  double t_stream = 0, t_solve = 0, t_solve_sweep = 0;
  int64_t n_stream = 0, n_solve = 0, n_solve_sweep = 0;
  std::vector<void *> allocs;
  SampleRing ring;

  bool alloc_failed = false;  // after one failed allocation the rest are not attempted
  template <class T>
  int alloc(T **p, int64_t n) {
    if (alloc_failed) { *p = nullptr; return -2; }
    int rc = dalloc(p, n);
    if (rc == 0) allocs.push_back((void *)*p);
    else alloc_failed = true;
    return rc;
  }
  ~brr_session() {
    if (ahead.th.joinable()) {
      {
        std::lock_guard<std::mutex> lk(ahead.mu);
        ahead.stop = true;
      }
      ahead.cv.notify_all();
      ahead.th.join();
    }
    // nothing may still run on either stream when its buffers go (e.g. a streaming kernel left in
    // flight by a bounded solver timeout): both drain before any hipFree / hipEventDestroy
    if (st_side) (void)hipStreamSynchronize(st_side);
    if (st) (void)hipStreamSynchronize(st);
    brr::sample_ring_close(this);
    if (comm) (void)ncclCommDestroy(comm);
    for (void *p : allocs) (void)hipFree(p);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    if (ev_x) (void)hipEventDestroy(ev_x);
    if (ev_go) (void)hipEventDestroy(ev_go);
    if (ev_done) (void)hipEventDestroy(ev_done);
    if (gram_codes) (void)hipFree(gram_codes);
    if (xcls) (void)hipFree(xcls);
    for (int k = 0; k < 2; ++k) {
      if (ref_pin[k]) (void)hipHostFree(ref_pin[k]);
      if (ref_ev[k]) (void)hipEventDestroy(ref_ev[k]);
    }
    if (st_side) (void)hipStreamDestroy(st_side);
    if (st) (void)hipStreamDestroy(st);
  }
  hipEvent_t ev() {
    if (ev_used == ev_pool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      ev_pool.push_back(e);
    }
    return ev_pool[ev_used++];
  }
};

namespace {

int encode_layout(brr_session *s);

int rows_flagged(brr_session *s, int flags, const double *deps_in = nullptr) {
  HIPCHK(launch_rows(s->d, flags, deps_in, s->st));
  return 0;
}

int collect_timing(brr_session *s) {
  if (s->ev_pairs.empty()) return 0;
  HIPCHK(hipStreamSynchronize(s->st));
  for (auto &pr : s->ev_pairs) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, s->ev_pool[pr.first], s->ev_pool[pr.first + 1]));
    if (pr.second == 0) { s->t_stream += ms; s->n_stream++; }
    else if (pr.second == 1) { s->t_solve += ms; s->n_solve++; }
    else if (pr.second == 2) { s->t_solve_sweep += ms; s->n_solve_sweep++; }
    else { s->t_stream += ms; s->n_stream += pr.second - 3; }  // marker-loop launch: per block position
  }
  s->ev_pairs.clear();
  s->ev_used = 0;
  return 0;
}

// this column shard's markers (local indices) in the order the global reference permutation
// lists them (the unsharded case: the permutation itself)
std::vector<int32_t> shard_visit(const brr_session *s) {
  if (s->M_total == s->M && s->col_offset == 0) return s->ref_order;
  std::vector<int32_t> v;
  v.reserve((size_t)s->M);
  for (const int32_t m : s->ref_order)
    if (m >= s->col_offset && m < s->col_offset + s->M) v.push_back((int32_t)(m - s->col_offset));
  return v;
}

// The shuffle-ahead thread: one sweep's permutations per request, in the reference's order of draws
// (fixedI before markerI, BayesRv2Groups.cpp:216,227; markerI, BayesRv2.cpp:182), so the glibc stream is
// consumed exactly as a synchronous shuffle would.
void ref_ahead_run(brr_session *s) {
  auto &a = s->ahead;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(a.mu);
      a.cv.wait(lk, [&] { return a.want || a.stop; });
      if (a.stop) return;
    }
    if (s->F > 0) s->grand.shuffle(s->ref_forder);
    s->grand.shuffle(s->ref_order);
    std::vector<int32_t> v = shard_visit(s), f = s->ref_forder;
    {
      std::lock_guard<std::mutex> lk(a.mu);
      a.visit.swap(v);
      a.forder.swap(f);
      a.want = false;
      a.have = true;
    }
    a.cv.notify_all();
  }
}

// this sweep's REFERENCE permutations (into s->cur_visit / cur_forder), and the next sweep's shuffle
// started on the thread
void ref_take(brr_session *s) {
  auto &a = s->ahead;
  std::unique_lock<std::mutex> lk(a.mu);
  if (!a.th.joinable()) {
    a.want = true;
    a.th = std::thread(ref_ahead_run, s);
  }
  a.cv.wait(lk, [&] { return a.have; });
  s->cur_visit.swap(a.visit);
  s->cur_forder.swap(a.forder);
  a.have = false;
  a.want = true;  // the next sweep's, while this one runs on the device
  lk.unlock();
  a.cv.notify_all();
}

int upload_order(brr_session *s, const std::vector<int32_t> &order) {
  // positions s*B+i of the reference order; Gram blocks follow the positions.  Only the members change
  // from sweep to sweep: they go through two pinned buffers (the copy of the sweep before last has
  // landed before its buffer is refilled), so the host never waits for the device here and the next
  // sweep's shuffle overlaps the current sweep's kernels; the block sizes and in-block indices are
  // uploaded once.
  const size_t n = (size_t)s->nb * s->B;
  if (!s->ref_static) {
    std::vector<int32_t> gi(n, 0), bsz(s->nb), gb(s->nb);
    for (int b = 0; b < s->nb; ++b) {
      const int size = (int)std::min<int64_t>(s->B, s->M - (int64_t)b * s->B);
      bsz[b] = size;
      gb[b] = b;
      for (int i = 0; i < size; ++i) gi[(size_t)b * s->B + i] = i;
    }
    HIPCHK(hipMemcpyAsync(s->d.gidx, gi.data(), gi.size() * 4, hipMemcpyHostToDevice, s->st));
    HIPCHK(hipMemcpyAsync(s->d.bsz, bsz.data(), bsz.size() * 4, hipMemcpyHostToDevice, s->st));
    HIPCHK(hipMemcpyAsync(s->d.gblk, gb.data(), gb.size() * 4, hipMemcpyHostToDevice, s->st));
    HIPCHK(hipStreamSynchronize(s->st));  // host vectors go out of scope
    s->ref_static = true;
  }
  const int k = s->ref_k;
  s->ref_k ^= 1;
  if (!s->ref_pin[k]) {
    HIPCHK(hipHostMalloc((void **)&s->ref_pin[k], n * 4, hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&s->ref_ev[k], hipEventDisableTiming));
  } else {
    HIPCHK(hipEventSynchronize(s->ref_ev[k]));  // this buffer's previous copy has landed
  }
  int32_t *mem = s->ref_pin[k];
  for (int b = 0; b < s->nb; ++b) {
    const int size = (int)std::min<int64_t>(s->B, s->M - (int64_t)b * s->B);
    std::memcpy(mem + (size_t)b * s->B, order.data() + (size_t)b * s->B, sizeof(int32_t) * (size_t)size);
    std::fill(mem + (size_t)b * s->B + size, mem + (size_t)(b + 1) * s->B, 0);
  }
  HIPCHK(hipMemcpyAsync(s->d.member, mem, n * 4, hipMemcpyHostToDevice, s->st));
  HIPCHK(hipEventRecord(s->ref_ev[k], s->st));
  return 0;
}

// the pipeline's bounded device waits raise sc->err instead of hanging.  mid_sweep: called between
// the exchange segments of a column-sharded sweep (brr_session_sweep_local), whose later segments
// still run in the same sweep
int check_device_error(brr_session *s, bool mid_sweep = false) {
  HIPCHK(hipStreamSynchronize(s->st));
  std::vector<int> sy(SY_WORDS);
  HIPCHK(hipMemcpy(sy.data(), s->d.sync, sizeof(int) * SY_WORDS, hipMemcpyDeviceToHost));
  if (sy[SY_ERR]) {
    set_error("device pipeline protocol timed out (k_stream / k_solve hand-over): site %d, workgroup %d "
              "waited for %d, saw %d (iteration %d; published blocks %d, groups %d/%d)",
              sy[SY_ERR + 1], sy[SY_ERR + 4], sy[SY_ERR + 2], sy[SY_ERR + 3], (int)s->iteration, sy[SY_PEND],
              sy[SY_GDONE], sy[SY_GDONE + 32]);
    const unsigned long long *ts = reinterpret_cast<const unsigned long long *>(sy.data() + SY_TS);
    std::string msg = brr_last_error();
    char buf[512];
    std::snprintf(buf, sizeof buf, " [us from streamer start: census %.1f, solver entry %.1f, solver block-0 wait %.1f..%.1f, "
                  "publish %.1f, first block-2 wait %.1f, first timeout %.1f]",
                  (ts[1] - ts[0]) / 100.0, ((double)ts[2] - ts[0]) / 100.0, ((double)ts[3] - ts[0]) / 100.0,
                  ((double)ts[4] - ts[0]) / 100.0, ((double)ts[5] - ts[0]) / 100.0, ((double)ts[6] - ts[0]) / 100.0,
                  ((double)ts[7] - ts[0]) / 100.0);
    set_error("%s%s", msg.c_str(), buf);
    // the error is reported once: clear the flag so the session can go on.  A failed residency
    // census (site 5) left the sweep's marker loop undone but the state consistent (every
    // workgroup exited before touching it): later sweeps use the per-block kernels.
    HIPCHK(hipMemset(s->d.sync + SY_ERR, 0, sizeof(int) * 5));
    if (sy[SY_ERR + 1] == 5 && s->fused.nsg > 0) {
      s->fused = FusedCfg{};
      s->d.lag = 1;
      // the hand-over counters are cumulative epochs of one pipeline geometry (and the failed
      // sweep advanced none of them): start every epoch again from zero
      const int NC = s->B >= 128 ? s->B / 128 : 1;
      HIPCHK(hipMemset(s->d.sync, 0, sizeof(int) * SY_WORDS));
      HIPCHK(hipMemset(s->d.cnt1, 0, sizeof(int) * NPAR * s->d.NG * NC));
      // the per-block solve sums whole padded batches of slab2 rows: no fused-solver sentinels left
      HIPCHK(hipMemset(s->d.slab2, 0, sizeof(double) * NPAR * s->d.slab2_stride));
      // The sweep's remaining segments (exchange segments, from block position f1 on) run on the
      // per-block kernels with this sweep's epoch bases (Dev::sbase / gbase, set at segment 0):
      // rebase them so that the counters, now zero, read as if blocks [0, f1) had passed, and the
      // session's bases past this sweep.  Without a sweep in flight f1 = nb: the next sweep starts
      // every epoch at zero.
      int f1 = s->nb;
      if (mid_sweep) f1 = (int)((int64_t)s->nb * (s->seg + 1) / s->nex);  // end of the failed segment
      s->d.sbase = -f1;
      for (int k = 0; k < NPAR; ++k) s->d.gbase[k] = -((f1 + NPAR - 1 - k) / NPAR);  // blocks < f1 of ring index k
      s->sbase = s->d.sbase + s->nb;
      for (int k = 0; k < NPAR; ++k) s->gbase[k] = s->d.gbase[k] + (s->nb + NPAR - 1 - k) / NPAR;
      s->abase = 0;
      s->census_failures++;
      s->log("libbrr: fused sweep could not be made resident; using the per-block kernels\n");
    }
    return -3;
  }
  return 0;
}

int ensure_reduced(brr_session *s) {
  if (!s->need_reduce) return 0;
  // row shards: S1/S2 run over every shard's rows; a local reduce here would leave this shard's
  // partial sums marked as final.  coll_sweep_rows reduces and sums them across shards.
  if (s->nrshard > 1) return 0;
  s->need_reduce = false;
  return rows_flagged(s, H_ROW_REDUCE);
}

// block positions [seg0, seg1) of exchange segment e of E (whole blocks; the oracle splits a
// shard's positions the same way, oracle/brr_oracle.c seg_positions)
void seg_range(int nb, int e, int E, int *seg0, int *seg1) {
  *seg0 = (int)((int64_t)nb * e / E);
  *seg1 = (int)((int64_t)nb * (e + 1) / E);
}

int do_sweep_local(brr_session *s) {
  if (!s->initialized) { set_error("session not initialised (brr_session_init)"); return -1; }
  if (int rc = ensure_reduced(s)) return rc;
  const uint32_t it = (uint32_t)s->iteration;
  const bool sharded = s->nshard > 1;
  const bool last = s->seg == s->nex - 1;
  Dev &d = s->d;
  if (s->seg == 0) {
    HIPCHK(launch_sweep_start(d, it, s->st));
    if (int rc = rows_flagged(s, H_ROW_SHIFT | H_ROW_WRITE)) return rc;
    // visit order
    if (s->order_mode == BRR_ORDER_BLOCKED) {
      HIPCHK(launch_perm(d, it, s->shard, false, s->st));
    } else if (s->order_mode == BRR_ORDER_REFERENCE) {
      ref_take(s);  // fixedI and markerI of this sweep, shuffled ahead on the host thread
      if (s->F > 0)
        HIPCHK(hipMemcpyAsync(d.forder, s->cur_forder.data(), (size_t)s->F * 4, hipMemcpyHostToDevice, s->st));
      if (int rc = upload_order(s, s->cur_visit)) return rc;
      if (int rc = encode_layout(s)) return rc;
      HIPCHK(launch_gram(d, 0, d.gram, nullptr, s->st));
      HIPCHK(launch_gram(d, 1, d.xgram, d.xgramT, s->st));
      if (d.lag >= 2) HIPCHK(launch_gram(d, 2, d.xgram2, d.xgram2T, s->st));  // (the layout's blocks two apart)
    } else {
      HIPCHK(launch_perm(d, it, s->shard, true, s->st));
    }
    if (s->model == MODEL_GROUPS && s->F > 0)
      HIPCHK(launch_fixed(d, it, s->order_mode == BRR_ORDER_BLOCKED, s->st));
    if (sharded)
      if (int rc = rows_flagged(s, H_ROW_SNAPSHOT)) return rc;
    // epoch bases of the hand-over counters (cumulative over the session; fixed for the sweep's
    // segments, whose block positions continue the sweep's)
    d.sbase = s->sbase;
    for (int k = 0; k < NPAR; ++k) d.gbase[k] = s->gbase[k];
    s->sbase += s->nb;
    for (int k = 0; k < NPAR; ++k) s->gbase[k] += (s->nb + NPAR - 1 - k) / NPAR;  // blocks s with s % NPAR == k
    // per-marker constants of the sweep in visit order (every segment's positions)
    HIPCHK(launch_prep(d, it, s->st));
  }
  // this launch's block positions (the whole sweep, or exchange segment seg)
  int s0 = 0, s1 = s->nb;
  seg_range(s->nb, s->seg, s->nex, &s0, &s1);
  d.seg0 = s0;
  d.seg1 = s1;
  // the hot loop (lag-1 pipeline).  Fused: ONE persistent launch, workgroup 0 solves block s
  // while the streaming workgroups form block s+1's dots (device counters hand over).
  // Per-block fallback: stream(0), stream(1), solve(0), stream(2), solve(1), ... on the one
  // queue (every dependency ahead in queue order, the same device protocol never waits).
  double *ebuf[2] = {d.eps, d.eps2};
  const bool fused = s->fused.nsg > 0;
  if (s1 > s0 && fused) {
    d.abase = s->abase;  // residency census epoch of this launch
    s->abase += s->fused.nsg + 1 + s->fused.nred;
    Dev dp = d;
    dp.NG = s->fused.ngroups;  // (1: the reducers write every column's whole sum)
    dp.gtarget = s->fused.nred;
    dp.ngr = s->fused.narr;
    // the cross-Gram corrections in the reducers (Dev::rcorr), for every fused sweep: at B <= 128 C3
    // 10.42 -> 10.88 sweeps/s (profiles/r04g_ab.log), the Horseshoe at lag 2 15.2 -> 18.8 (its phase A
    // loses the 5.6 us correction of a dense list), C2 2-bit at lag 2 45.5 -> 50.7 in the driver's window
    // (profiles/r05i_ab.log); C2 f32 unchanged in the driver's window (32.1-32.5 ms), its steady marker
    // loop 30.8 -> 31.1 ms (profiles/r05j_ab.log) -- taken there too, so that both storages sum the
    // corrections in one association and keep bit-identical chains (the solver's own correction sums
    // in another: BRR_RED_CORR=0, diagnostics, matches the oracle to the same tolerance but not bit
    // for bit)
    {
      const char *rc = getenv("BRR_RED_CORR");
      dp.rcorr = rc ? (atoi(rc) != 0) : true;
      // the reducers' cross-Gram columns loaded before the lists are published: off by default (C4 at
      // lag 2 18.8 -> 14.7 sweeps/s, C3 12.45 -> 12.2, C1 / C3 at lag 1 within noise;
      // profiles/r05i_ab.log, r05g*); BRR_RED_PF=1 turns it on where the slices fit a reducer's LDS
      const char *pf = getenv("BRR_RED_PF");
      dp.rcpf = dp.rcorr && s->fused.rcpf && pf && pf[0] == '1';
      // BRR_RED_SPLIT=1: the newest list's correction in the solver (its own list, from its LDS), the
      // older ones in the reducers
      const char *sp = getenv("BRR_RED_SPLIT");
      dp.rcsplit = dp.rcorr && sp && sp[0] == '1';
      // the overlapped solver workgroup (brr_ovsolve.hpp; BayesR family at B = 128, lag <= 2): block
      // s+1's decisions, Gram block and cross-Gram corrections prepared while block s's chain runs; its
      // corrector forms every correction, so the reducers form none (rcorr = 0) and the dots wait for no
      // list publication.  On by default for Groups, where the hand-over it hides outweighs its slower
      // chain step: C3 12.63 -> 14.31 sweeps/s; off for V2 / restart, whose chain dominates: C1 229 -> 210,
      // REFERENCE order 8.5 -> 6.7 (profiles/r06k_ab.log, r06h_ab.log).  BRR_OVS=0|1
      // overrides
      const char *ov = getenv("BRR_OVS");
      // (default for Groups in BLOCKED order; REFERENCE order at lag 1 runs faster on the round-5 solver:
  // 11.5 against 8.5 sweeps/s at C2, profiles/r06s_ab.log, r06v_ab.log)
  dp.ovs = (ov ? ov[0] == '1' : (s->model == MODEL_GROUPS && s->order_mode == BRR_ORDER_BLOCKED)) &&
           ov_solver_ok(dp, s->fused);
      if (dp.ovs) dp.rcorr = dp.rcsplit = dp.rcpf = 0;
      s->ovs_last = dp.ovs;
    }
    dp.slab_storage = d.Xc != nullptr || d.xcodes != nullptr;  // streamers read blocks in storage order (2-bit, f32 code cache)
    FusedCfg fc = s->fused;
    fc.prof = s->prof_on ? 1 : 0;  // (the streaming kernel's diagnostics variant only while they are on)
    if (s->timing) {
      const size_t i0 = s->ev_used;
      hipEvent_t e0 = s->ev(), e1 = s->ev();
      HIPCHK(hipEventRecord(e0, s->st));
      HIPCHK(launch_sweep_fused(dp, it, fc, s->st, s->st_side, s->ev_go, s->ev_done));
      HIPCHK(hipEventRecord(e1, s->st));
      s->ev_pairs.push_back({i0, 3 + (s1 - s0)});
    } else {
      HIPCHK(launch_sweep_fused(dp, it, fc, s->st, s->st_side, s->ev_go, s->ev_done));
    }
  } else if (s1 > s0) {
    // eps buffers relative to the segment start: k_stream(b) reads ebuf[(b - s0) & 1]
    auto stream_b = [&](int b) -> int {
      const double *ein = ebuf[(b - s0) & 1];
      double *eout = ebuf[(b - s0 + 1) & 1];
      if (s->timing) {
        const size_t i0 = s->ev_used;
        hipEvent_t e0 = s->ev(), e1 = s->ev();
        HIPCHK(hipEventRecord(e0, s->st));
        HIPCHK(launch_stream(d, b, ein, eout, s->st));
        HIPCHK(hipEventRecord(e1, s->st));
        s->ev_pairs.push_back({i0, 0});
      } else {
        HIPCHK(launch_stream(d, b, ein, eout, s->st));
      }
      return 0;
    };
    auto solve_b = [&](int b) -> int {
      if (s->timing) {
        const size_t i2 = s->ev_used;
        hipEvent_t e2 = s->ev(), e3 = s->ev();
        HIPCHK(hipEventRecord(e2, s->st));
        HIPCHK(launch_solve(d, b, it, s->st));
        HIPCHK(hipEventRecord(e3, s->st));
        s->ev_pairs.push_back({i2, 1});
      } else {
        HIPCHK(launch_solve(d, b, it, s->st));
      }
      return 0;
    };
    for (int b = s0; b < s1; ++b) {
      if (int rc = stream_b(b)) return rc;
      if (b >= s0 + 1)
        if (int rc = solve_b(b - 1)) return rc;
    }
    if (int rc = solve_b(s1 - 1)) return rc;
  }
  // E_{s1-2} (written by the last k_stream) minus the changes of the last two blocks; the
  // fused sweep has already applied them and written eps
  const int ns = s1 - s0;
  const double *elast = (fused || ns == 0) ? d.eps : ebuf[ns & 1];
  const int sa = (!fused && ns >= 2) ? (s1 - 2) % NSLOT : -1, sb = (fused || ns == 0) ? -1 : (s1 - 1) % NSLOT;
  if (sharded) {
    if (!s->ex_eps || !s->ex_stats) { set_error("exchange buffers not set"); return -1; }
    Dev dx = d;
    dx.deps = s->ex_eps;
    HIPCHK(launch_rows(dx, H_ROW_PENDING | H_ROW_WRITE | H_ROW_DEPS, nullptr, s->st, elast, sa, sb));
  } else {
    HIPCHK(launch_rows(d, H_ROW_PENDING | H_ROW_WRITE | H_ROW_REDUCE, nullptr, s->st, elast, sa, sb));
  }
  if (last) {
    const int mode = s->model == MODEL_HORSESHOE ? H_MR_HS : H_MR_BAYESR;
    HIPCHK(launch_markers(d, mode, it, s->st));
    if (sharded)
      HIPCHK(hipMemcpyAsync(s->ex_stats, d.stats, sizeof(double) * s->NS, hipMemcpyDeviceToDevice, s->st));
  } else {
    // an earlier exchange segment: only the residual delta; the statistics follow the last
    HIPCHK(hipMemsetAsync(s->ex_stats, 0, sizeof(double) * s->NS, s->st));
  }
  return 0;
}

int do_sweep_finish(brr_session *s) {
  const uint32_t it = (uint32_t)s->iteration;
  const bool sharded = s->nshard > 1;
  if (sharded && s->seg < s->nex - 1) {
    // the next exchange segment starts from eps = eps_segment_start + sum of the shards' deltas
    if (int rc = rows_flagged(s, H_ROW_EXCHANGE | H_ROW_WRITE | H_ROW_SNAPSHOT, s->ex_eps)) return rc;
    s->seg++;
    return 0;
  }
  s->seg = 0;
  if (sharded) {
    if (int rc = rows_flagged(s, H_ROW_EXCHANGE | H_ROW_WRITE | H_ROW_REDUCE, s->ex_eps)) return rc;
    HIPCHK(launch_hyper(s->d, it, s->ex_stats, s->st));
  } else {
    HIPCHK(launch_hyper(s->d, it, s->d.stats, s->st));
  }
  s->iteration++;
  s->d.seg0 = 0;
  s->d.seg1 = s->nb;
  if (s->timing) return collect_timing(s);
  return 0;
}

template <class T>
int h2d(brr_session *s, T *dst, const T *src, int64_t n) {
  if (n <= 0) return 0;
  HIPCHK(hipMemcpyAsync(dst, src, sizeof(T) * (size_t)n, hipMemcpyHostToDevice, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  return 0;
}

template <class T>
int d2h(brr_session *s, T *dst, const T *src, int64_t n) {
  if (n <= 0) return 0;
  HIPCHK(hipStreamSynchronize(s->st));
  HIPCHK(hipMemcpy(dst, src, sizeof(T) * (size_t)n, hipMemcpyDeviceToHost));
  return 0;
}

// ---------------------------------------------------------------------------------------
// Exact row shards.  A Coll is the set of sessions one host thread drives: one
// session (single GPU; or one row shard of a multi-process RCCL job) or every member of an
// in-process brr_group.  coll_sum is the exchange step: the sum across row shards of a device
// buffer, in place, identical on every shard -- ncclAllReduce on the session stream (one process
// per GPU), or k_group_sum over the members' buffers in rank order (brr_group), ordered against
// the members' streams with events.  Without row shards it does nothing.
struct Coll {
  std::vector<brr_session *> ss;
  bool rows() const { return ss[0]->nrshard > 1; }
};

template <class Get>
int coll_sum(Coll &c, Get get, int64_t n) {
  if (!c.rows() || n <= 0) return 0;
  if (c.ss.size() == 1) {
    brr_session *s = c.ss[0];
    if (!s->comm) {
      set_error("row-sharded session without a communicator: brr_session_comm_init before init, or a brr_group");
      return -1;
    }
    double *b = get(s);
    const ncclResult_t r = ncclAllReduce(b, b, (size_t)n, ncclDouble, ncclSum, s->comm, s->st);
    if (r != ncclSuccess) { set_error("ncclAllReduce (row shards): %s", ncclGetErrorString(r)); return -2; }
    return 0;
  }
  brr_session *s0 = c.ss[0];
  GroupPtrs p{};
  p.n = (int)c.ss.size();
  for (size_t i = 0; i < c.ss.size(); ++i) {
    p.ptr[i] = get(c.ss[i]);
    if (i > 0) {
      HIPCHK(hipSetDevice(c.ss[i]->device));
      HIPCHK(hipEventRecord(c.ss[i]->ev_x, c.ss[i]->st));
      HIPCHK(hipSetDevice(s0->device));
      HIPCHK(hipStreamWaitEvent(s0->st, c.ss[i]->ev_x, 0));
    }
  }
  HIPCHK(hipSetDevice(s0->device));
  HIPCHK(launch_group_sum(p, n, s0->st));
  HIPCHK(hipEventRecord(s0->ev_x, s0->st));
  for (size_t i = 1; i < c.ss.size(); ++i) {
    HIPCHK(hipSetDevice(c.ss[i]->device));
    HIPCHK(hipStreamWaitEvent(c.ss[i]->st, s0->ev_x, 0));
  }
  return 0;
}

// f(s) for every session of the collective, on its device
template <class F>
int coll_each(Coll &c, F f) {
  for (brr_session *s : c.ss) {
    HIPCHK(hipSetDevice(s->device));
    if (int rc = f(s)) return rc;
  }
  return 0;
}

double *sc_sums(brr_session *s) { return &s->d.sc->S1; }  // S1, S2: adjacent in Scal

// Value classes of every column (k_classes) and the Gram kernel they allow: the exact integer
// k_gram_int when every column has at most 4 distinct values (genotypes, either storage) and B is
// a multiple of 64; else the FP64 k_gram.  BRR_GRAM_F64=1 forces the latter (diagnostics).
int prepare_classes(brr_session *s) {
  Dev &d = s->d;
  d.gram_np = 0;
  const char *f = getenv("BRR_GRAM_F64");
  if ((f && f[0] == '1') || s->B % 64 != 0 || s->M == 0) return 0;
  int fl[2] = {0, 0};
  HIPCHK(hipMemsetAsync(s->cls_flags, 0, sizeof(int) * 2, s->st));
  HIPCHK(launch_classes(d, s->cls_flags, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  HIPCHK(hipMemcpy(fl, s->cls_flags, sizeof fl, hipMemcpyDeviceToHost));
  if (fl[0] == 0 && fl[1] >= 1) d.gram_np = std::max(1, fl[1] - 1);
  if (d.gram_np > 0 && !s->gram_codes) {
    // the layout's class codes: N P / 4 bytes (without them, the FP64 kernel)
    if (hipMalloc(&s->gram_codes, (size_t)s->nb * s->B * d.ldc) != hipSuccess) {
      (void)hipGetLastError();
      s->gram_codes = nullptr;
      d.gram_np = 0;
    }
  }
  d.gram_codes = d.gram_np > 0 ? s->gram_codes : nullptr;
  s->gram_np_init = d.gram_np;
  // REFERENCE order re-encodes its layout every sweep: from column-major class codes made once here
  // (N P / 4 bytes; without the memory, from X itself as before)
  if (d.gram_np > 0 && s->order_mode == BRR_ORDER_REFERENCE && !s->xcls && !getenv("BRR_NO_XCLS")) {
    if (hipMalloc(&s->xcls, (size_t)s->M * d.ldc) != hipSuccess) {
      (void)hipGetLastError();
      s->xcls = nullptr;
    } else {
      HIPCHK(launch_xcls(d, s->xcls, s->st));
    }
  }
  d.xcls = s->xcls;
  return 0;
}

// Gram blocks of the current layout need its class codes first (k_gram_int)
int encode_layout(brr_session *s) {
  if (s->d.gram_np > 0 && !gram_reads_xcls(s->d)) HIPCHK(launch_encode_layout(s->d, s->st));
  return 0;
}

// BLOCKED / IDENTITY order: no Gram blocks after init, the class codes' memory is returned
int release_gram_codes(brr_session *s) {
  s->d.xcodes = nullptr;
  if (s->order_mode == BRR_ORDER_REFERENCE || !s->gram_codes) return 0;
  if (s->fused.nsg > 0 && s->fused.f32cc && s->d.gram_np > 0 && s->order_mode == BRR_ORDER_BLOCKED) {
    // f32 storage: the init layout's class codes are the storage-order codes the streamers' cache
    // is filled from (k_sweep_stream<2>)
    s->d.xcodes = s->gram_codes;
    return 0;
  }
  HIPCHK(hipStreamSynchronize(s->st));
  HIPCHK(hipFree(s->gram_codes));
  s->gram_codes = nullptr;
  s->d.gram_codes = nullptr;
  s->d.gram_np = 0;
  return 0;
}

// the Gram and cross-Gram blocks of the current layout (init; REFERENCE order: every sweep),
// summed over the row shards
int coll_grams(Coll &c) {
  if (int rc = coll_each(c, [](brr_session *s) -> int {
        Dev &d = s->d;
        if (int rc = encode_layout(s)) return rc;
        HIPCHK(launch_gram(d, 0, d.gram, nullptr, s->st));
        HIPCHK(launch_gram(d, 1, d.xgram, d.xgramT, s->st));  // cycle neighbours (b, b+1 mod nb)
        if (d.lag >= 2) HIPCHK(launch_gram(d, 2, d.xgram2, d.xgram2T, s->st));  // (b, b+2 mod nb)
        if (d.lag >= 3) HIPCHK(launch_gram(d, 3, d.xgram3, d.xgram3T, s->st));  // (b, b+3 mod nb)
        return 0;
      }))
    return rc;
  if (!c.rows()) return 0;
  const int64_t nbb = (int64_t)c.ss[0]->nb * c.ss[0]->B * c.ss[0]->B;
  if (int rc = coll_sum(c, [](brr_session *s) { return s->d.gram; }, nbb)) return rc;
  if (int rc = coll_sum(c, [](brr_session *s) { return s->d.xgram; }, nbb)) return rc;
  return coll_sum(c, [](brr_session *s) { return s->d.xgramT; }, nbb);
}

// last init step: hyper-parameter init draws from the (summed) statistics
int init_finish(brr_session *s, const double *stats) {
  if (int rc = release_gram_codes(s)) return rc;
  HIPCHK(launch_hyper_init(s->d, stats, s->pi_given, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  s->iteration = 0;
  s->initialized = true;
  s->init_pending = false;
  s->need_reduce = false;
  return 0;
}

int coll_init(Coll &c, int32_t seed) {
  for (brr_session *s : c.ss) {
    if (!s->have_x) { set_error("X not uploaded"); return -1; }
    if (s->model != MODEL_RESTART && !s->have_y) { set_error("Y not set"); return -1; }
  }
  // identity block layout -> Gram blocks and xsquared (BayesRv2.cpp:170)
  if (int rc = coll_each(c, [&](brr_session *s) -> int {
        s->d.seed = (uint64_t)(int64_t)seed;
        HIPCHK(launch_perm(s->d, 0, s->shard, true, s->st));
        return 0;
      }))
    return rc;
  if (int rc = coll_each(c, prepare_classes)) return rc;
  // 2-bit storage whose streamers keep no LDS code cache (B = 512): a column-major copy of the codes
  // (N M / 4 bytes) for the change-list apply -- a changed column then costs each streaming workgroup
  // 64 contiguous bytes per 256 rows instead of a byte of 64 16-B tile granules (C2: ~1.5 GB less
  // traffic per sweep).  BRR_XCM=0: off.
  if (int rc = coll_each(c, [](brr_session *s) -> int {
        Dev &d = s->d;
        const char *xe = getenv("BRR_XCM");
        if (!s->x2bit || s->fused.nsg == 0 || s->fused.ccache || (xe && xe[0] == '0')) return 0;
        if (!d.Xcm) {  // (optional: without the memory the apply reads the tiles, as before)
          uint8_t *p = nullptr;
          if (hipMalloc(&p, (size_t)d.ldc * s->M) != hipSuccess) {
            (void)hipGetLastError();
            return 0;
          }
          s->allocs.push_back(p);
          d.Xcm = p;
        }
        HIPCHK(launch_codes_cm(d, const_cast<uint8_t *>(d.Xcm), s->st));  // (every init: X may be new)
        return 0;
      }))
    return rc;
  if (int rc = coll_grams(c)) return rc;
  if (int rc = coll_each(c, [](brr_session *s) -> int {
        Dev &d = s->d;
        HIPCHK(launch_xsq(d, s->st));
        Scal sc{};
        if (s->model == MODEL_RESTART) { sc.mu = s->mu0; sc.sigmaE = s->sigmaE0; }
        if (s->model == MODEL_HORSESHOE) sc.c2 = d.hyp.c2_0;
        HIPCHK(hipMemcpyAsync(d.sc, &sc, sizeof sc, hipMemcpyHostToDevice, s->st));
        if (s->model != MODEL_RESTART) {
          HIPCHK(hipMemsetAsync(d.beta, 0, sizeof(double) * s->M, s->st));
          HIPCHK(hipMemsetAsync(d.comp, 0, sizeof(int) * s->M, s->st));
        }
        HIPCHK(hipMemsetAsync(d.sel, 0, s->M, s->st));
        HIPCHK(hipMemsetAsync(d.alpha, 0, sizeof(double) * std::max(s->F, 1), s->st));
        if (s->F > 0) {  // identity fixed-effect order (IDENTITY mode; REFERENCE overwrites per sweep)
          std::vector<int32_t> idf((size_t)s->F);
          for (int i = 0; i < s->F; ++i) idf[(size_t)i] = i;
          if (int rc = h2d(s, d.forder, idf.data(), s->F)) return rc;
        }
        if (s->model == MODEL_HORSESHOE) {
          std::vector<double> ones((size_t)s->M, 1.0);
          if (int rc = h2d(s, d.lambda, ones.data(), s->M)) return rc;
          if (int rc = h2d(s, d.hsv, ones.data(), s->M)) return rc;
        }
        return rows_flagged(s, (s->model == MODEL_RESTART ? 0 : (H_ROW_INIT_Y | H_ROW_WRITE)) | H_ROW_REDUCE);
      }))
    return rc;
  if (int rc = coll_sum(c, sc_sums, 2)) return rc;
  return coll_each(c, [](brr_session *s) -> int {
    Dev &d = s->d;
    const double *stats = d.stats;
    if (s->model == MODEL_RESTART) {
      // v(g, k) counts over every marker (BRv2Grstart.cpp:157-165): a row shard holds every
      // marker; column shards sum their local counts across shards first
      HIPCHK(launch_markers(d, H_MR_COUNT_ALL, 0, s->st));
      if (s->nshard > 1) {
        if (int rc = brr_session_exchange_buffers(s, nullptr, nullptr)) return rc;
        HIPCHK(hipMemcpyAsync(s->ex_stats, d.stats, sizeof(double) * s->NS, hipMemcpyDeviceToDevice, s->st));
        if (!s->comm) {  // brr_session_init_local: the caller sums the exchange statistics
          HIPCHK(hipStreamSynchronize(s->st));
          s->init_pending = true;
          return 0;
        }
        ncclResult_t r = ncclAllReduce(s->ex_stats, s->ex_stats, (size_t)s->NS, ncclDouble, ncclSum, s->comm, s->st);
        if (r != ncclSuccess) { set_error("ncclAllReduce failed: %s", ncclGetErrorString(r)); return -2; }
        stats = s->ex_stats;
      }
    }
    return init_finish(s, stats);
  });
}

// One exact sweep of row-sharded sessions (per-block kernels; the same operations as
// do_sweep_local + do_sweep_finish with the cross-shard sums inserted where a quantity runs over
// rows: residual sums, fixed-effect dots, each block's dots, and REFERENCE order's Gram blocks).
int coll_sweep_rows(Coll &c) {
  for (brr_session *s : c.ss)
    if (!s->initialized) { set_error("session not initialised"); return -1; }
  bool red = false;
  for (brr_session *s : c.ss) red |= s->need_reduce;
  if (red) {
    if (int rc = coll_each(c, [](brr_session *s) -> int {
          s->need_reduce = false;
          return rows_flagged(s, H_ROW_REDUCE);
        }))
      return rc;
    if (int rc = coll_sum(c, sc_sums, 2)) return rc;
  }
  brr_session *s0 = c.ss[0];
  const uint32_t it = (uint32_t)s0->iteration;
  if (int rc = coll_each(c, [&](brr_session *s) -> int {
        Dev &d = s->d;
        HIPCHK(launch_sweep_start(d, it, s->st));
        if (int rc = rows_flagged(s, H_ROW_SHIFT | H_ROW_WRITE)) return rc;
        if (s->order_mode == BRR_ORDER_BLOCKED) {
          HIPCHK(launch_perm(d, it, 0, false, s->st));
        } else if (s->order_mode == BRR_ORDER_REFERENCE) {
          ref_take(s);  // (a row shard holds every marker: its visit order is the whole permutation)
          if (s->F > 0)
            HIPCHK(hipMemcpyAsync(d.forder, s->cur_forder.data(), (size_t)s->F * 4, hipMemcpyHostToDevice, s->st));
          if (int rc = upload_order(s, s->cur_visit)) return rc;
        } else {
          HIPCHK(launch_perm(d, it, 0, true, s->st));
        }
        return 0;
      }))
    return rc;
  if (s0->order_mode == BRR_ORDER_REFERENCE)
    if (int rc = coll_grams(c)) return rc;
  if (s0->model == MODEL_GROUPS && s0->F > 0) {
    const bool dev_perm = s0->order_mode == BRR_ORDER_BLOCKED;
    for (int cf = 0; cf < s0->F; ++cf) {
      if (int rc = coll_each(c, [&](brr_session *s) -> int {
            HIPCHK(launch_fixed_row(s->d, it, cf, 0, dev_perm, s->st));
            return 0;
          }))
        return rc;
      if (int rc = coll_sum(c, [](brr_session *s) { return &s->d.sc->fx; }, 1)) return rc;
      if (int rc = coll_each(c, [&](brr_session *s) -> int {
            HIPCHK(launch_fixed_row(s->d, it, cf, 1, dev_perm, s->st));
            return 0;
          }))
        return rc;
    }
  }
  if (int rc = coll_each(c, [&](brr_session *s) -> int {
        Dev &d = s->d;
        d.sbase = s->sbase;
        for (int k = 0; k < NPAR; ++k) d.gbase[k] = s->gbase[k];
        d.abase = s->abase;
        s->sbase += s->nb;
        for (int k = 0; k < NPAR; ++k) s->gbase[k] += (s->nb + NPAR - 1 - k) / NPAR;
        HIPCHK(launch_prep(d, it, s->st));
        return 0;
      }))
    return rc;
  // the marker loop: stream(b), the block's dots summed over the shards, solve(b - 1) (lag-1
  // pipeline of the per-block kernels)
  const int nb = s0->nb;
  auto stream_b = [&](int b) {
    return coll_each(c, [&](brr_session *s) -> int {
      double *ebuf[2] = {s->d.eps, s->d.eps2};
      HIPCHK(launch_stream(s->d, b, ebuf[b & 1], ebuf[(b + 1) & 1], s->st));
      HIPCHK(launch_slab_total(s->d, b, s->st));
      return 0;
    });
  };
  auto solve_b = [&](int b) {
    return coll_each(c, [&](brr_session *s) -> int {
      Dev dp = s->d;
      dp.NG = 1;  // the summed dots are in slab2 row 0
      HIPCHK(launch_solve(dp, b, it, s->st));
      return 0;
    });
  };
  // instrumentation (one session): the whole marker loop between two events, per block position
  const bool timed = c.ss.size() == 1 && s0->timing;
  size_t ti = 0;
  if (timed) {
    ti = s0->ev_used;
    hipEvent_t e0 = s0->ev();
    (void)s0->ev();
    HIPCHK(hipEventRecord(e0, s0->st));
  }
  for (int b = 0; b < nb; ++b) {
    if (int rc = stream_b(b)) return rc;
    if (int rc = coll_sum(c, [b](brr_session *s) { return s->d.slab2 + (b % NPAR) * s->d.slab2_stride; }, s0->B))
      return rc;
    if (b >= 1)
      if (int rc = solve_b(b - 1)) return rc;
  }
  if (int rc = solve_b(nb - 1)) return rc;
  if (timed) {
    HIPCHK(hipEventRecord(s0->ev_pool[ti + 1], s0->st));
    s0->ev_pairs.push_back({ti, 3 + nb});
  }
  if (int rc = coll_each(c, [&](brr_session *s) -> int {
        Dev &d = s->d;
        double *ebuf[2] = {d.eps, d.eps2};
        const int sa = nb >= 2 ? (nb - 2) % NSLOT : -1, sb = (nb - 1) % NSLOT;
        HIPCHK(launch_rows(d, H_ROW_PENDING | H_ROW_WRITE | H_ROW_REDUCE, nullptr, s->st, ebuf[nb & 1], sa, sb));
        return 0;
      }))
    return rc;
  if (int rc = coll_sum(c, sc_sums, 2)) return rc;
  return coll_each(c, [&](brr_session *s) -> int {
    const int mode = s->model == MODEL_HORSESHOE ? H_MR_HS : H_MR_BAYESR;
    HIPCHK(launch_markers(s->d, mode, it, s->st));
    HIPCHK(launch_hyper(s->d, it, s->d.stats, s->st));
    s->iteration++;
    if (s->timing) return collect_timing(s);
    return 0;
  });
}

}  // namespace

// =======================================================================================
extern "C" {

void brr_options_default(brr_options *o) {
  std::memset(o, 0, sizeof *o);
  o->abi_version = BRR_ABI_VERSION;
  o->block_size = 0;  // automatic: 512 (V2, restart), 128 (Groups, Horseshoe)
  o->order_mode = BRR_ORDER_BLOCKED;
  o->shard_count = 1;
  o->row_shard_count = 1;
  o->exchanges_per_sweep = 0;  // automatic (column shards: E = 8, capped at the blocks per shard)
}

void brr_options_effective(const brr_options *in, brr_options *out) {
  if (out) *out = brr::options_from_caller(in);
}

const char *brr_last_error(void) { return g_last_error.c_str(); }

int brr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int brr_device_memory(int32_t device, int64_t *free_bytes, int64_t *total_bytes) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) { set_error("no HIP device available"); return -1; }
  if (device < 0 || device >= n) { set_error("device %d not present", device); return -1; }
  // a query only: the caller's current device is restored on every path
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = device;
  size_t f = 0, t = 0;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMemGetInfo(&f, &t);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("HIP error %s: %s (device memory query)", hipGetErrorName(e), hipGetErrorString(e));
    return -1;
  }
  if (free_bytes) *free_bytes = (int64_t)f;
  if (total_bytes) *total_bytes = (int64_t)t;
  return 0;
}

brr_session *brr_session_create(int32_t model, int64_t N, int64_t M, int64_t M_total,
                                int64_t col_offset, int32_t K, int32_t groups, int64_t F,
                                const brr_options *opt_in) {
  brr_options opt = brr::options_from_caller(opt_in);
  if (opt.row_shard_count < 1) opt.row_shard_count = 1;
  const bool rows = opt.row_shard_count > 1;
  const int64_t N_total = opt.N_total > 0 ? opt.N_total : N;
  if (rows) {
    if (opt.shard_count > 1) { set_error("row shards and column shards cannot be combined"); return nullptr; }
    if (opt.row_shard_count > GROUP_MAX) { set_error("row_shard_count > %d", GROUP_MAX); return nullptr; }
    if (opt.row_shard_rank < 0 || opt.row_shard_rank >= opt.row_shard_count) { set_error("bad row_shard_rank"); return nullptr; }
    if (opt.row_offset < 0 || opt.row_offset + N > N_total) { set_error("rows [row_offset, row_offset + N) outside N_total"); return nullptr; }
    if (M_total != M || col_offset != 0) { set_error("a row shard holds every marker (M_total == M, col_offset 0)"); return nullptr; }
  }
  if (model < 0 || model > 3) { set_error("bad model %d", model); return nullptr; }
  if (N < 1 || M < 1) { set_error("N and M must be >= 1"); return nullptr; }
  if (M_total < M) M_total = M;
  if (model == MODEL_HORSESHOE) K = 1;
  if (K < 1 || K > MAXK) { set_error("mixture components K=%d outside [1,%d]", K, MAXK); return nullptr; }
  if (model == MODEL_V2 || model == MODEL_HORSESHOE) groups = 1;
  if (groups < 1 || groups > MAXG) { set_error("groups=%d outside [1,%d]", groups, MAXG); return nullptr; }
  if (model != MODEL_GROUPS) F = 0;
  if (F < 0 || F > 1024) { set_error("fixed effects F=%lld outside [0,1024]", (long long)F); return nullptr; }
  // automatic block size: BayesRSamplerV2 / BRV2Grstart change few markers per block (long blocks
  // amortise the per-block hand-over); the Horseshoe resamples every marker and the Groups chain
  // keeps most markers in non-zero components (C3: 23 % change per sweep), so their serial chain
  // dominates and B = 128 keeps the whole Gram block in LDS (C3: 9.3 / 6.2 / 4.5 sweeps/s at
  // B = 128 / 256 / 512)
  // (small cohorts: the chain, not the stream, dominates every sampler -- C1, N = 2,000: 147 against
  // 90 sweeps/s at B = 128 / 512 -- so B = 128 below N = 32,768)
  // (row shards choose from the cohort's N_total: every shard must run the same B, and the same B
  // as the unsharded chain)
  // (REFERENCE order recomputes its Gram blocks every sweep, 2 P B N class-pair products: C2 4.0
  // against 1.8 sweeps/s at B = 128 / 512, profiles/r03_c2_reference_order_b*_intgram.log)
  int B = opt.block_size > 0 ? opt.block_size
                             : ((model == MODEL_HORSESHOE || model == MODEL_GROUPS || N_total < 32768 ||
                                 opt.order_mode == BRR_ORDER_REFERENCE)
                                    ? 128
                                    : 512);
  if (B % 64 != 0 || B > BMAX) { set_error("block_size=%d must be a multiple of 64 and <= %d", B, BMAX); return nullptr; }
  if (opt.shard_count < 1) opt.shard_count = 1;
  if (opt.shard_count > 1 && (col_offset % B) != 0) {
    set_error("col_offset must be a multiple of block_size when sharded");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    set_error("no HIP device available: the MI355X sampler has no CPU fallback");
    return nullptr;
  }
  if (opt.device < 0 || opt.device >= ndev) { set_error("device %d not present", opt.device); return nullptr; }
  brr_session *s = new brr_session();
  s->opt = opt;
  s->log.fn = opt.log;
  s->log.user = opt.log_userdata;
  s->device = opt.device;
  if (hipSetDevice(s->device) != hipSuccess) {
    set_error("cannot initialise HIP device %d", s->device);
    delete s;
    return nullptr;
  }
  // an earlier call's failure (e.g. another session's failed allocation) must not surface as this
  // session's error: the launchers report hipGetLastError()
  (void)hipGetLastError();
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, s->device);
  const int cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) {
    set_error("cannot create a stream on HIP device %d", s->device);
    delete s;
    return nullptr;
  }
  s->N = N; s->M = M; s->M_total = M_total; s->col_offset = col_offset;
  s->K = K; s->G = groups; s->F = (int)F; s->B = B; s->model = model;
  s->order_mode = opt.order_mode;
  s->shard = opt.shard_rank; s->nshard = opt.shard_count;
  // column shards: exchanges per sweep E.  0 (default) = automatic: E = 8, at most the blocks per
  // shard -- global quantities, so every shard runs the same E (the exchange is a collective).  A
  // segment's stale residual of the other S - 1 shards is then (S - 1) / (S E) < 1/8 of a sweep's
  // changes; the sigmaE bias grows about linearly in that fraction (+3.0 % at 8 shards and E = 1, +0.7 %
  // at 2 shards and E = 2, +0.13 % at 8 shards and E = 8: profiles/r03_shard_bias.jsonl,
  // profiles/r04_shard_bias_E_eq_S.jsonl), and 8 shards at E = 8 pass the distributional test against
  // the 1-shard chain.
  if (s->nshard > 1) {
    const int64_t nbt = (M_total + B - 1) / B;
    s->nex = opt.exchanges_per_sweep > 0 ? opt.exchanges_per_sweep
                                         : (int)std::max<int64_t>(1, std::min<int64_t>(8, nbt / s->nshard));
  } else {
    s->nex = 1;
  }
  s->rshard = rows ? opt.row_shard_rank : 0; s->nrshard = opt.row_shard_count;
  if (hipEventCreateWithFlags(&s->ev_x, hipEventDisableTiming) != hipSuccess) {
    set_error("cannot create an event on HIP device %d", s->device);
    delete s;
    return nullptr;
  }
  s->nb = (int)((M + B - 1) / B);
  s->NS = stats_size(groups, K);
  Dev &d = s->d;
  d.N = N; d.M = M; d.M_total = M_total; d.col_offset = col_offset;
  d.Ntot = N_total; d.row_offset = rows ? opt.row_offset : 0;
  d.ld = (N + SROWS - 1) / SROWS * SROWS;  // every streaming row tile inside the allocation (zero rows)
  d.K = K; d.G = groups; d.F = (int)F; d.B = B; d.nb = s->nb; d.model = model;
  d.seg0 = 0; d.seg1 = s->nb;  // block positions of a launch (exchange segments: a part)
  // streaming geometry: row tiles of SROWS rows (k_stream), NC = B/128 column chunks
  d.R = SROWS;
  d.RG = (int)((N + SROWS - 1) / SROWS);
  d.NG = (d.RG + STREAM_GROUP - 1) / STREAM_GROUP;
  const int NGpad = (d.NG + 31) / 32 * 32;  // k_solve reads slab2 in unconditional batches of 32
  const int NC = B >= 128 ? B / 128 : 1;
  d.gtarget = d.NG * NC;
  d.MRG = (int)((M + 255) / 256);
  const int64_t RGrows = (N + 255) / 256;
  int rc = 0;
  // genotype storage: f32 (default) or 2-bit codes + per-column value tables
  s->x2bit = opt.x_storage == BRR_X_2BIT;
  d.ldc = d.ld / 4;
  // Preflight: the big buffers against the device's free memory, before any of them is allocated.
  // A create that cannot fit (e.g. a 200 GB X while an earlier session still holds 250 GB) fails
  // here with its sizes in the message; BRR_NO_MEM_PREFLIGHT=1 skips it (tests: the allocation
  // failure path itself).
  if (!(getenv("BRR_NO_MEM_PREFLIGHT") && getenv("BRR_NO_MEM_PREFLIGHT")[0] == '1')) {
    size_t mfree = 0, mtotal = 0;
    if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess) {
      const double xb = s->x2bit ? (double)d.ldc * s->nb * B + 16.0 * M : 4.0 * (double)d.ld * M;
      // Gram sets: gram, xgram, xgramT, and for the fused sweep's lag 2 (3) the cross-Gram blocks of
      // blocks two (three) apart in both orientations -- the lag chosen below, before the fused
      // geometry is known (the per-block fallback runs lag 1 and leaves these unallocated: an over-count)
      const char *lg = getenv("BRR_LAG");
      const char *pb = getenv("BRR_PER_BLOCK");
      int lag_pre = 1;
      if (opt.order_mode == BRR_ORDER_BLOCKED && s->nb >= 4 && !rows && !(pb && pb[0] == '1') && !(lg && atoi(lg) < 2))
        lag_pre = (lg && atoi(lg) >= 3 && s->nb >= 5) ? 3 : 2;
      if (opt.order_mode == BRR_ORDER_REFERENCE && s->nb >= 4 && !rows && lg && atoi(lg) >= 2) lag_pre = 2;
      const double grams = (3.0 + 2.0 * (lag_pre - 1)) * 8.0 * (double)s->nb * B * B;
      // the integer Gram's class codes of the layout (N P / 4 bytes, during init; REFERENCE order keeps
      // them and a column-major copy for every sweep).  Without that memory init would fall back to
      // the FP64 Gram kernel, ~6x slower, so it is counted too.
      const double codes = (double)d.ldc * s->nb * B * (opt.order_mode == BRR_ORDER_REFERENCE ? 2.0 : 1.0);
      const double small = 8.0 * (double)d.ld * 3 + 8.0 * (double)s->nb * B * (3 + 2 * K) + 64.0 * M + 8.0 * N * std::max<int64_t>(F, 1);
      const double need = xb + grams + codes + small;
      if (need > (double)mfree) {
        set_error("device %d has %.2f GB free of %.2f GB: this session needs %.2f GB (X %.2f GB, %d Gram sets %.2f GB, "
                  "class codes %.2f GB, the rest %.2f GB)",
                  s->device, mfree / 1e9, mtotal / 1e9, need / 1e9, xb / 1e9, 1 + 2 * lag_pre, grams / 1e9, codes / 1e9,
                  small / 1e9);
        delete s;
        return nullptr;
      }
    }
  }
  if (s->x2bit) {
    rc |= s->alloc(const_cast<uint8_t **>(&d.Xc), d.ldc * s->nb * B);  // whole tiles of the last block
    rc |= s->alloc(const_cast<float **>(&d.xlut), 4 * M);
  } else {
    rc |= s->alloc(const_cast<float **>(&d.X), d.ld * M);
  }
  rc |= s->alloc(const_cast<double **>(&d.Y), N);
  rc |= s->alloc(const_cast<double **>(&d.fixed), N * std::max<int64_t>(F, 1));
  rc |= s->alloc(const_cast<double **>(&d.cva), (int64_t)groups * std::max(K - 1, 1));
  rc |= s->alloc(&d.eps, d.ld);  // padded to ld rows (zeros): k_stream loads 4 rows per lane
  rc |= s->alloc(&d.eps2, d.ld);  // k_stream double buffer
  rc |= s->alloc(&d.eps_start, d.ld);
  rc |= s->alloc(&d.beta, M);
  rc |= s->alloc(&d.xsq, M);
  rc |= s->alloc(&d.lambda, M);
  rc |= s->alloc(&d.hsv, M);
  rc |= s->alloc(&d.sigmaGG, groups);
  rc |= s->alloc(&d.pi, (int64_t)groups * K);
  rc |= s->alloc(&d.alpha, std::max<int64_t>(F, 1));
  rc |= s->alloc(&d.comp, M);
  rc |= s->alloc(&d.forder, std::max<int64_t>(F, 1));
  rc |= s->alloc(&d.sel, M);
  rc |= s->alloc(&d.cls_info, M);
  rc |= s->alloc(&d.cls_val, 4 * M);
  rc |= s->alloc(&d.cls_cnt, 4 * M);
  rc |= s->alloc(&s->cls_flags, 2);
  rc |= s->alloc(&d.gram, (int64_t)s->nb * B * B);
  rc |= s->alloc(&d.xgram, (int64_t)s->nb * B * B);
  rc |= s->alloc(&d.xgramT, (int64_t)s->nb * B * B);
  rc |= s->alloc(&d.member, (int64_t)s->nb * B);
  rc |= s->alloc(&d.gidx, (int64_t)s->nb * B);
  rc |= s->alloc(&d.bsz, s->nb);
  rc |= s->alloc(&d.gblk, s->nb);
  rc |= s->alloc(&d.blkorder, s->nb);
  d.slab1_stride = (int64_t)(d.RG + 1) * B;  // per-block: RG row tiles; fused: 2 nsg <= RG + 1 slices
  d.slab2_stride = (int64_t)NGpad * B;
  d.pend_stride = B + 16;
  rc |= s->alloc(&d.slab1, NPAR * d.slab1_stride);
  rc |= s->alloc(&d.slab2, NPAR * d.slab2_stride);
  rc |= s->alloc(&d.cnt1, NPAR * (int64_t)d.NG * NC);
  rc |= s->alloc(&d.sync, SY_WORDS);
  rc |= s->alloc(&d.pend_idx, NSLOT * d.pend_stride);
  rc |= s->alloc(&d.pend_pos, NSLOT * d.pend_stride);
  rc |= s->alloc(&d.pend_gi, NSLOT * d.pend_stride);
  rc |= s->alloc(&d.pend_bo, NSLOT * d.pend_stride);
  rc |= s->alloc(&d.pend_bn, NSLOT * d.pend_stride);
  rc |= s->alloc(&d.pend_n, 2 * NSLOT);  // [NSLOT] padded list lengths, [NSLOT] entries before the padding
  rc |= s->alloc(&d.trace, (int64_t)s->nb * 16 + 9216);  // + per-workgroup probes and totals
  d.nbB = (int64_t)s->nb * B;
  rc |= s->alloc(&d.mc, d.nbB * (3 + 2 * std::max(K, 1)));
  rc |= s->alloc(&d.rslab, 2 * RGrows);
  rc |= s->alloc(&d.rcnt, 1);
  rc |= s->alloc(&d.mslab, (int64_t)d.MRG * s->NS);
  rc |= s->alloc(&d.mcnt, 1);
  rc |= s->alloc(&d.stats, s->NS);
  rc |= s->alloc(&d.sc, 1);
  d.deps = nullptr;
  if (rc) { delete s; return nullptr; }
  d.gAssign = nullptr;
  // every buffer a kernel may read before writing is zeroed here (recycled device memory
  // holds the previous session's values): slab2 pad rows, member padding, pending list
  bool ok = hipMemsetAsync(d.cnt1, 0, sizeof(int) * NPAR * d.NG * NC, s->st) == hipSuccess &&
            hipMemsetAsync(d.sync, 0, sizeof(int) * SY_WORDS, s->st) == hipSuccess &&
            hipMemsetAsync(d.pend_gi, 0, sizeof(int) * NSLOT * d.pend_stride, s->st) == hipSuccess &&
            hipMemsetAsync(d.pend_n, 0, sizeof(int) * 6, s->st) == hipSuccess &&
            hipMemsetAsync(d.eps, 0, sizeof(double) * d.ld, s->st) == hipSuccess &&
            hipMemsetAsync(d.eps2, 0, sizeof(double) * d.ld, s->st) == hipSuccess &&
            hipMemsetAsync(d.slab2, 0, sizeof(double) * NPAR * d.slab2_stride, s->st) == hipSuccess &&
            hipMemsetAsync(d.member, 0, sizeof(int) * s->nb * B, s->st) == hipSuccess &&
            hipMemsetAsync(d.gidx, 0, sizeof(int) * s->nb * B, s->st) == hipSuccess &&
            hipMemsetAsync(d.pend_idx, 0, sizeof(int) * NSLOT * d.pend_stride, s->st) == hipSuccess &&
            hipMemsetAsync(d.pend_pos, 0, sizeof(int) * NSLOT * d.pend_stride, s->st) == hipSuccess &&
            hipMemsetAsync(d.pend_bo, 0, sizeof(double) * NSLOT * d.pend_stride, s->st) == hipSuccess &&
            hipMemsetAsync(d.pend_bn, 0, sizeof(double) * 3 * d.pend_stride, s->st) == hipSuccess &&
            hipMemsetAsync(d.rcnt, 0, sizeof(int), s->st) == hipSuccess &&
            hipMemsetAsync(d.mcnt, 0, sizeof(int), s->st) == hipSuccess &&
            hipMemsetAsync(d.sc, 0, sizeof(Scal), s->st) == hipSuccess &&
            hipMemsetAsync(d.stats, 0, sizeof(double) * s->NS, s->st) == hipSuccess &&
            (s->x2bit ? hipMemsetAsync(const_cast<uint8_t *>(d.Xc), 0xFF, (size_t)d.ldc * s->nb * B, s->st) == hipSuccess &&
                            hipMemsetAsync(const_cast<float *>(d.xlut), 0, sizeof(float) * 4 * M, s->st) == hipSuccess
                      : hipMemsetAsync(const_cast<float *>(d.X), 0, sizeof(float) * d.ld * M, s->st) == hipSuccess) &&
            hipMemsetAsync(d.alpha, 0, sizeof(double) * std::max<int64_t>(F, 1), s->st) == hipSuccess &&
            hipMemsetAsync(const_cast<double *>(d.fixed), 0, sizeof(double) * N * std::max<int64_t>(F, 1), s->st) == hipSuccess &&
            set_solve_lds_limit(B) == hipSuccess && hipStreamSynchronize(s->st) == hipSuccess;
  if (!ok) { set_error("device initialisation failed"); delete s; return nullptr; }
  if (groups > 1) {
    int *ga = nullptr;
    if (s->alloc(&ga, M)) { delete s; return nullptr; }
    (void)hipMemsetAsync(ga, 0, sizeof(int) * M, s->st);
    d.gAssign = ga;
  }
  // fused persistent sweep (one workgroup per CU, all resident); BRR_PER_BLOCK=1 forces the
  // per-block kernels, BRR_STREAM_WG=n caps the streaming workgroups (tests: several row tiles
  // per half-workgroup)
  {
    const char *pb = getenv("BRR_PER_BLOCK");
    const char *cap = getenv("BRR_STREAM_WG");
    // lag 2 (fused sweep, BLOCKED order, nb >= 4): the streamers apply block s-3's changes
    // before streaming block s, so a workgroup can run two blocks ahead of the solver and
    // per-block jitter among the streamers is absorbed; costs the cross-Gram blocks of blocks
    // two apart (2 nb B^2 f64 more, computed once at init) and a second correction -- in the
    // reducers where they correct the dots (Dev::rcorr, brr::session_sweep), else in the solver.
    // Chosen for the samplers that change few markers per block (V2, restart; C2 f32 26.3 -> 27.2
    // sweeps/s) in either storage, and for the Horseshoe, with the reducers' correction: C4 15.2 ->
    // 18.8 sweeps/s, C2 2-bit 45.5 -> 50.7 in the driver's window (profiles/r05i_ab.log; with the
    // correction in the solver lag 2 was 25 / 7 % slower than lag 1 there), and for Groups (C3 12.41 ->
    // 12.58, profiles/r05j_ab.log).  BRR_LAG=1|2 overrides.
    const char *lg = getenv("BRR_LAG");
    // REFERENCE order only on request (BRR_LAG=2): its third Gram set per sweep (the layout's blocks two
    // apart, ~14 ms with the fp4 Gram kernel) costs more than the deeper marker loop saves -- C2 in REFERENCE
    // order 11.5 (lag 1) against 10.4 (lag 2; 10.8 with the overlapped solver), profiles/r06v_ab.log
    const bool lag2_ok = (s->order_mode == BRR_ORDER_BLOCKED || (s->order_mode == BRR_ORDER_REFERENCE && lg)) && s->nb >= 4;
    d.lag = (lag2_ok && (lg ? atoi(lg) >= 2 : true)) ? 2 : 1;
    if (d.lag == 2 && lg && atoi(lg) >= 3 && s->nb >= 5 && s->order_mode == BRR_ORDER_BLOCKED) d.lag = 3;  // (diagnostics: BRR_LAG=3)
    // row shards: the per-block kernels (the cross-shard sum of a block's dots sits between its
    // streaming and its solve; the fused sweep's in-kernel hand-over is one device's)
    // 2-bit storage in REFERENCE order: the fused streamers read a block's code tiles in storage
    // order (whole column blocks), but a REFERENCE block holds arbitrary columns -- the per-block
    // kernels read each member column by index
    const bool ref2bit = s->x2bit && s->order_mode == BRR_ORDER_REFERENCE;
    // f32 storage in BLOCKED order: keep the streamed blocks' class codes in LDS (used when init
    // finds every column class-coded, and where LDS holds lag + 2 blocks of them) and apply the
    // change lists from them instead of re-reading X -- on by default for the Horseshoe, whose
    // lists hold every column of a block (C4 13.05 -> 14.1 sweeps/s with the round-4 apply tables
    // and reducers, profiles/r04i_ab.log; round 3: 13.87 -> 13.42), and for Groups (C3 12.24 -> 12.28
    // sweeps/s, same box, profiles/r05e_ab.log: no slower, and the apply no longer re-reads the changed
    // columns, 1.30x -> ~1.0x the algorithmic bytes); V2 / restart change few markers per block (C2: no
    // change).  BRR_F32_CODE_CACHE=0|1 overrides.
    const char *fcc = getenv("BRR_F32_CODE_CACHE");
    const bool f32cc = !s->x2bit && s->order_mode == BRR_ORDER_BLOCKED &&
                       (fcc ? fcc[0] == '1' : (model == MODEL_HORSESHOE || model == MODEL_GROUPS));
    if (rows || ref2bit || (pb && pb[0] == '1') || !fused_config(d, cus, cap ? atoi(cap) : 0, &s->fused, f32cc))
      s->fused = FusedCfg{};
    if (s->fused.nsg == 0) d.lag = 1;
    // the persistent solver polls its reduced dots against per-block sentinels (brr_kernels.hip
    // slab_sentinel): slot p starts with block p's
    if (s->fused.nsg > 0 && launch_slab_sentinels(d, (int)(d.slab2_stride / B), s->st) != hipSuccess) {
      set_error("cannot initialise the dot slots");
      delete s;
      return nullptr;
    }
    // lag 1 while the solver bounds the sweep: more than ~30 changed markers per block at C2's
    // 100,000 rows (the burn-in's first sweeps), scaled with the rows: a block's streaming time and a
    // change's solver cost both grow with them; BRR_LAG_SWITCH overrides the per-block count at
    // 100,000 rows.  Round 5, with the corrections in the reducers, the driver's window (sweeps 5-24)
    // at 8 / 15 / 30 / 60: 32.75 / 32.37 / 31.78 / 31.95 ms per step, C2 2-bit flat
    // (profiles/r05o_ab.log; round 3, with the corrections in the solver, 15 was the crossover,
    // profiles/r03_lagswitch_ab.log)
    {
      const char *ls = getenv("BRR_LAG_SWITCH");
      const double per_block = (ls ? atof(ls) : 30.0) * ((double)N / 1e5);
      // (BRR_LAG: that lag in every sweep after the first.  The Horseshoe and Groups keep lag 2 from the
      // second sweep on, the burn-in included: the Horseshoe changes every marker in every sweep, Groups ~25 of 128 per block, both
      // above the switch, and both gain from lag 2 with the reducers' correction)
      d.lag_thresh = (lg || model == MODEL_HORSESHOE || model == MODEL_GROUPS) ? 1e300 : per_block * s->nb;
    }
    // The streaming kernel's stream must never share a hardware queue with the session stream: a
    // solver kernel ahead of it in the same queue would wait (bounded, census site 5) for streaming
    // workgroups that cannot start.  HIP maps ordinary streams round-robin onto a small pool of
    // queues (GPU_MAX_HW_QUEUES, 4 on the box), so two streams of one session can land on one
    // queue once other streams come and go; a stream with a CU mask gets a queue of its own.
    std::vector<uint32_t> cu_all((size_t)(cus + 31) / 32, 0xFFFFFFFFu);
    if (s->fused.split && hipExtStreamCreateWithCUMask(&s->st_side, (uint32_t)cu_all.size(), cu_all.data()) != hipSuccess) {
      (void)hipGetLastError();
      s->st_side = nullptr;
    }
    if (s->fused.split &&
        ((!s->st_side && hipStreamCreateWithFlags(&s->st_side, hipStreamNonBlocking) != hipSuccess) ||
         hipEventCreateWithFlags(&s->ev_go, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming) != hipSuccess)) {
      set_error("cannot create the streaming kernel's stream / events");
      delete s;
      return nullptr;
    }
    if ((d.lag >= 2 && (s->alloc(&d.xgram2, (int64_t)s->nb * B * B) || s->alloc(&d.xgram2T, (int64_t)s->nb * B * B))) ||
        (d.lag >= 3 && (s->alloc(&d.xgram3, (int64_t)s->nb * B * B) || s->alloc(&d.xgram3T, (int64_t)s->nb * B * B)))) {
      delete s;
      return nullptr;
    }
  }
  // REFERENCE order: the permutation of ALL M_total markers (every column shard draws the same
  // glibc stream); a shard visits its own columns in that order (shard_visit)
  s->ref_order.resize((size_t)M_total);
  for (int64_t i = 0; i < M_total; ++i) s->ref_order[(size_t)i] = (int32_t)i;
  s->ref_forder.resize((size_t)std::max(s->F, 0));
  for (int i = 0; i < s->F; ++i) s->ref_forder[(size_t)i] = i;
  s->grand.seed(1);  // a fresh process: rand() unseeded == srand(1)
  return s;
}

void brr_session_destroy(brr_session *s) {
  if (!s) return;
  // an output still open (brr_session_output_open without _close, e.g. after an error in the
  // caller): join its writer thread and drain its rows before the sample ring goes away
  (void)brr_session_output_close(s, nullptr);
  delete s;
}

// 2-bit encoding of columns c0 .. c0+nc-1 of a host matrix (f64 or f32, leading dimension ldx):
// each column's distinct f32 values plus 0 (the padding rows) must number at most 4; codes are
// their ranks in ascending order (bit pattern order), so the device decodes exactly the f32
// values the f32 storage would hold.  Threads split the columns.  Returns the first offending
// column, or -1.
static int64_t encode_2bit(const void *X, bool f64, int64_t ldx, int64_t N, int64_t ldc, int64_t c0, int64_t nc,
                           uint8_t *codes, float *lut) {
  std::atomic<int64_t> bad{-1};
  auto work = [&](int64_t a, int64_t b) {
    for (int64_t j = a; j < b && bad.load() < 0; ++j) {
      const int64_t col = c0 + j;
      auto val = [&](int64_t i) -> float {
        return f64 ? (float)((const double *)X)[ldx * col + i] : ((const float *)X)[ldx * col + i];
      };
      uint32_t vals[4];
      int nv = 0;
      auto add = [&](uint32_t u) -> bool {
        for (int k = 0; k < nv; ++k)
          if (vals[k] == u) return true;
        if (nv == 4) return false;
        vals[nv++] = u;
        return true;
      };
      bool ok = add(0u);  // +0.0f: padding rows
      for (int64_t i = 0; i < N && ok; ++i) {
        const float v = val(i);
        uint32_t u;
        std::memcpy(&u, &v, 4);
        ok = add(u);
      }
      if (!ok) {
        int64_t exp = -1;
        bad.compare_exchange_strong(exp, col);
        return;
      }
      float fv[4];
      for (int k = 0; k < nv; ++k) std::memcpy(&fv[k], &vals[k], 4);
      // ascending value order (ties impossible: distinct bit patterns; -0 < +0 by pattern)
      std::sort(vals, vals + nv, [](uint32_t x, uint32_t y) {
        float a, b;
        std::memcpy(&a, &x, 4);
        std::memcpy(&b, &y, 4);
        return a < b || (a == b && x > y);
      });
      uint8_t zero_code = 0;
      for (int k = 0; k < nv; ++k) {
        std::memcpy(&lut[4 * j + k], &vals[k], 4);
        if (vals[k] == 0u) zero_code = (uint8_t)k;
      }
      for (int k = nv; k < 4; ++k) lut[4 * j + k] = 0.f;
      (void)fv;
      uint8_t *cc = codes + j * ldc;
      for (int64_t b4 = 0; b4 < ldc; ++b4) {
        uint32_t byte = 0;
        for (int k = 0; k < 4; ++k) {
          const int64_t i = 4 * b4 + k;
          uint32_t code = zero_code;
          if (i < N) {
            const float v = val(i);
            uint32_t u;
            std::memcpy(&u, &v, 4);
            for (int q = 0; q < nv; ++q)
              if (vals[q] == u) code = (uint32_t)q;
          }
          byte |= code << (2 * k);
        }
        cc[b4] = (uint8_t)byte;
      }
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::max(1u, std::thread::hardware_concurrency()),
                                                             (int64_t)16, nc}));
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t) pool.emplace_back(work, nc * t / nt, nc * (t + 1) / nt);
  for (auto &th : pool) th.join();
  return bad.load();
}

static int upload_x_any(brr_session *s, const void *X, bool f64, int64_t ldx) {
  if (!s || !X) { set_error("null argument"); return -1; }
  if (ldx < s->N) { set_error("ldx < N"); return -1; }
  HIPCHK(hipSetDevice(s->device));
  if (s->x2bit) {
    const int64_t ldc = s->d.ldc;
    const int64_t chunk_cols = std::max<int64_t>(1, std::min<int64_t>(s->M, (int64_t)(256ll << 20) / ldc));
    std::vector<uint8_t> codes((size_t)(ldc * chunk_cols));
    std::vector<float> lut((size_t)(4 * chunk_cols));
    uint8_t *stage = nullptr;  // column-major chunk on the device, scattered into the code tiles
    HIPCHK(hipMalloc(&stage, (size_t)(ldc * chunk_cols)));
    struct Free { uint8_t *p; ~Free() { (void)hipFree(p); } } free_stage{stage};
    for (int64_t c0 = 0; c0 < s->M; c0 += chunk_cols) {
      const int64_t nc = std::min<int64_t>(chunk_cols, s->M - c0);
      const int64_t bad = encode_2bit(X, f64, ldx, s->N, ldc, c0, nc, codes.data(), lut.data());
      if (bad >= 0) {
        set_error("column %lld has more than 3 distinct non-zero values: 2-bit genotype storage needs "
                  "genotype-coded columns (x_storage = BRR_X_F32 stores any matrix)", (long long)bad);
        return -1;
      }
      HIPCHK(hipMemcpy(stage, codes.data(), (size_t)(ldc * nc), hipMemcpyHostToDevice));
      HIPCHK(launch_codes_tile(stage, const_cast<uint8_t *>(s->d.Xc), c0, nc, ldc, s->B, s->st));
      HIPCHK(hipStreamSynchronize(s->st));
      HIPCHK(hipMemcpy(const_cast<float *>(s->d.xlut) + 4 * c0, lut.data(), sizeof(float) * 4 * nc,
                       hipMemcpyHostToDevice));
    }
    s->have_x = true;
    return 0;
  }
  const size_t esz = f64 ? 8 : 4;
  const int64_t chunk_cols = std::min<int64_t>(
      65535, std::max<int64_t>(1, (int64_t)(256ll << 20) / (int64_t)(esz * ldx)));  // grid.y limit
  void *stage = nullptr;
  HIPCHK(hipMalloc(&stage, esz * (size_t)ldx * (size_t)std::min<int64_t>(chunk_cols, s->M)));
  for (int64_t c0 = 0; c0 < s->M; c0 += chunk_cols) {
    const int64_t nc = std::min<int64_t>(chunk_cols, s->M - c0);
    hipError_t e = hipMemcpy(stage, (const char *)X + esz * (size_t)ldx * (size_t)c0, esz * (size_t)ldx * (size_t)nc,
                             hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = launch_cast_x(stage, f64, ldx, const_cast<float *>(s->d.X) + s->d.ld * c0, s->d.ld, s->N, nc, s->st);
    if (e == hipSuccess) e = hipStreamSynchronize(s->st);
    if (e != hipSuccess) {
      (void)hipFree(stage);
      set_error("X upload failed: %s", hipGetErrorString(e));
      return -2;
    }
  }
  (void)hipFree(stage);
  s->have_x = true;
  return 0;
}

int brr_session_upload_x_f64(brr_session *s, const double *X, int64_t ldx) { return upload_x_any(s, X, true, ldx); }
int brr_session_upload_x_f32(brr_session *s, const float *X, int64_t ldx) { return upload_x_any(s, X, false, ldx); }

// PLINK .bed body (SNP-major, after the 3 magic bytes): this shard's M columns of bytes_per_col
// >= ceil(N/4) bytes, sample i in bits 2(i&3).. of byte i>>2; codes 00 = two copies of allele 1,
// 10 = heterozygous, 11 = no copy, 01 = missing.  Genotype g = copies of allele 1; columns are
// standardised as R's scale() after mean imputation (vignettes/BayesRR.Rmd:92): mean over the
// observed samples, sd = sqrt(sum_observed (g - mean)^2 / (N - 1)), x = f32((g - mean) / sd), a
// missing sample gets x = 0; a column without variation is all 0.
int brr_session_upload_bed(brr_session *s, const uint8_t *bed, int64_t bytes_per_col) {
  if (!s || !bed) { set_error("null argument"); return -1; }
  const int64_t N = s->N, nbytes = (N + 3) / 4;
  if (bytes_per_col < nbytes) { set_error("bytes_per_col < ceil(N/4)"); return -1; }
  HIPCHK(hipSetDevice(s->device));
  const int64_t ldc = s->d.ldc;
  const int64_t chunk_cols = std::max<int64_t>(1, std::min<int64_t>(s->M, (int64_t)(256ll << 20) / ldc));
  std::vector<uint8_t> codes;
  std::vector<float> lut((size_t)(4 * chunk_cols)), xf;
  uint8_t *stage = nullptr;  // 2-bit: column-major chunk on the device, scattered into the code tiles
  if (s->x2bit) {
    codes.resize((size_t)(ldc * chunk_cols));
    HIPCHK(hipMalloc(&stage, (size_t)(ldc * chunk_cols)));
  } else {
    xf.resize((size_t)(s->d.ld * chunk_cols));
  }
  struct Free { uint8_t *p; ~Free() { if (p) (void)hipFree(p); } } free_stage{stage};
  static const double gval[4] = {2.0, 0.0 /* missing */, 1.0, 0.0};
  for (int64_t c0 = 0; c0 < s->M; c0 += chunk_cols) {
    const int64_t nc = std::min<int64_t>(chunk_cols, s->M - c0);
    for (int64_t j = 0; j < nc; ++j) {
      const uint8_t *src = bed + bytes_per_col * (c0 + j);
      int64_t cnt[4] = {0, 0, 0, 0};
      for (int64_t i = 0; i < N; ++i) cnt[(src[i >> 2] >> (2 * (i & 3))) & 3]++;
      const int64_t nobs = cnt[0] + cnt[2] + cnt[3];
      const double S = 2.0 * cnt[0] + cnt[2], Q = 4.0 * cnt[0] + cnt[2];
      const double mean = nobs > 0 ? S / (double)nobs : 0.0;
      const double ss = Q - S * mean;  // sum over observed samples of (g - mean)^2
      const bool flat = nobs < 2 || !(ss > 0.0) || N < 2;
      const double sd = flat ? 1.0 : std::sqrt(ss / (double)(N - 1));
      float *l = &lut[(size_t)(4 * j)];
      for (int c = 0; c < 4; ++c) l[c] = (flat || c == 1) ? 0.f : (float)((gval[c] - mean) / sd);
      if (s->x2bit) {
        uint8_t *dst = &codes[(size_t)(ldc * j)];
        std::memcpy(dst, src, (size_t)nbytes);
        if (N & 3) dst[nbytes - 1] = (uint8_t)((dst[nbytes - 1] & ((1u << (2 * (N & 3))) - 1u)) |
                                               (0x55u & ~((1u << (2 * (N & 3))) - 1u)));  // padding: code 01 -> 0
        std::memset(dst + nbytes, 0x55, (size_t)(ldc - nbytes));
      } else {
        float *dst = &xf[(size_t)(s->d.ld * j)];
        for (int64_t i = 0; i < s->d.ld; ++i) dst[i] = i < N ? l[(src[i >> 2] >> (2 * (i & 3))) & 3] : 0.f;
      }
    }
    if (s->x2bit) {
      HIPCHK(hipMemcpy(stage, codes.data(), (size_t)(ldc * nc), hipMemcpyHostToDevice));
      HIPCHK(launch_codes_tile(stage, const_cast<uint8_t *>(s->d.Xc), c0, nc, ldc, s->B, s->st));
      HIPCHK(hipStreamSynchronize(s->st));
      HIPCHK(hipMemcpy(const_cast<float *>(s->d.xlut) + 4 * c0, lut.data(), sizeof(float) * 4 * nc,
                       hipMemcpyHostToDevice));
    } else {
      HIPCHK(hipMemcpy(const_cast<float *>(s->d.X) + s->d.ld * c0, xf.data(), sizeof(float) * s->d.ld * nc,
                       hipMemcpyHostToDevice));
    }
  }
  s->have_x = true;
  return 0;
}

int brr_session_synthesize(brr_session *s, uint64_t ds, double h2, int64_t n_causal) {
  if (!s) return -1;
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(launch_synth_x(s->d, ds, s->st));
  s->have_x = true;
  // this shard's genetic values X_c beta_c over its causal columns
  if (n_causal < 1) n_causal = std::max<int64_t>(1, std::min<int64_t>(1000, s->M_total / 10));
  const double pc = (double)n_causal / (double)s->M_total;
  const double scale = std::sqrt(h2 / (double)n_causal);
  std::vector<int> cidx;
  std::vector<double> cb;
  for (int64_t jl = 0; jl < s->M; ++jl) {
    const int64_t j = s->col_offset + jl;
    if (uniform(ds, T_DATA_FREQ, (uint32_t)j, 0, 1) < pc) {
      cidx.push_back((int)jl);
      cb.push_back(normal(ds, T_DATA_FREQ, (uint32_t)j, 0, 2) * scale);
    }
  }
  int *dci = nullptr;
  double *dcb = nullptr, *dy = nullptr;
  const int nc = (int)cidx.size();
  HIPCHK(hipMalloc(&dci, sizeof(int) * std::max(nc, 1)));
  HIPCHK(hipMalloc(&dcb, sizeof(double) * std::max(nc, 1)));
  HIPCHK(hipMalloc(&dy, sizeof(double) * s->N));
  if (nc) {
    HIPCHK(hipMemcpy(dci, cidx.data(), sizeof(int) * nc, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dcb, cb.data(), sizeof(double) * nc, hipMemcpyHostToDevice));
  }
  HIPCHK(launch_synth_y(s->d, dci, dcb, nc, dy, s->st));
  s->synth_y.assign((size_t)s->N, 0.0);
  HIPCHK(hipStreamSynchronize(s->st));
  HIPCHK(hipMemcpy(s->synth_y.data(), dy, sizeof(double) * s->N, hipMemcpyDeviceToHost));
  (void)hipFree(dci); (void)hipFree(dcb); (void)hipFree(dy);
  if (s->nshard > 1 || s->nrshard > 1) return 0;  // Y needs every shard's genetic values: brr_session_synth_y
  return brr_session_synth_y(s, s->synth_y.data(), ds, h2);
}

int brr_session_synth_partial_y(brr_session *s, double *out) {
  if (!s || !out || s->synth_y.size() != (size_t)s->N) { set_error("no synthetic genetic values"); return -1; }
  std::memcpy(out, s->synth_y.data(), sizeof(double) * s->N);
  return 0;
}

int brr_session_synth_y(brr_session *s, const double *g_sum, uint64_t ds, double h2) {
  if (!s || !g_sum) return -1;
  // row shards: g_sum holds the genetic values of all N_total rows (row order); Y is
  // standardised over the cohort and this shard keeps its rows
  const int64_t NT = s->d.Ntot, r0 = s->d.row_offset;
  std::vector<double> y(g_sum, g_sum + NT);
  const double se = std::sqrt(1.0 - h2);
  double mean = 0.0;
  for (int64_t i = 0; i < NT; ++i) {
    y[(size_t)i] += se * normal(ds, T_DATA_NOISE, (uint32_t)i, 0, 0);
    mean += y[(size_t)i];
  }
  mean /= (double)NT;
  double ss = 0.0;
  for (int64_t i = 0; i < NT; ++i) ss += (y[(size_t)i] - mean) * (y[(size_t)i] - mean);
  const double sd = NT > 1 ? std::sqrt(ss / (double)(NT - 1)) : 1.0;
  for (auto &v : y) v = (v - mean) / (sd > 0 ? sd : 1.0);  // Y = scale(y)
  return brr_session_set_y(s, y.data() + r0);
}

int brr_session_set_y(brr_session *s, const double *Y) {
  if (!s || !Y) return -1;
  s->have_y = true;
  return h2d(s, const_cast<double *>(s->d.Y), Y, s->N);
}

int brr_session_set_fixed(brr_session *s, const double *fixed) {
  if (!s) return -1;
  if (s->F == 0) return 0;
  if (!fixed) return -1;
  return h2d(s, const_cast<double *>(s->d.fixed), fixed, s->N * s->F);
}

int brr_session_set_bayesr(brr_session *s, double sigma0, double v0E, double s02E, double v0G,
                           double s02G, const double *cva, const int32_t *gAssign) {
  if (!s) return -1;
  Hyper &h = s->d.hyp;
  h.sigma0 = sigma0; h.v0E = v0E; h.s02E = s02E; h.v0G = v0G; h.s02G = s02G;
  const int nc = s->K - 1;
  if (nc > 0) {
    if (!cva) { set_error("cva required"); return -1; }
    if (int rc = h2d(s, const_cast<double *>(s->d.cva), cva, (int64_t)s->G * nc)) return rc;
  }
  if (s->G > 1) {
    if (!gAssign) { set_error("gAssign required for groups > 1"); return -1; }
    for (int64_t m = 0; m < s->M; ++m)
      if (gAssign[m] < 0 || gAssign[m] >= s->G) { set_error("gAssign[%lld]=%d outside [0,%d)", (long long)m, gAssign[m], s->G); return -1; }
    if (int rc = h2d(s, const_cast<int *>(s->d.gAssign), (const int *)gAssign, s->M)) return rc;
  }
  if (!s->pi_given) {  // priorPi (BayesRv2Groups.cpp:170-175; SURVEY Appendix B for V2)
    std::vector<double> pi((size_t)s->G * s->K);
    for (int g = 0; g < s->G; ++g) {
      pi[(size_t)g * s->K] = 0.5;
      for (int k = 1; k < s->K; ++k) pi[(size_t)g * s->K + k] = 0.5 / s->K;
    }
    if (int rc = h2d(s, s->d.pi, pi.data(), (int64_t)pi.size())) return rc;
  }
  return 0;
}

int brr_session_set_horseshoe(brr_session *s, double A, double v0E, double s02E, double vL,
                              double vT, double c2, double vC, double sC) {
  if (!s) return -1;
  Hyper &h = s->d.hyp;
  h.A = A; h.v0E = v0E; h.s02E = s02E; h.vL = vL; h.vT = vT; h.c2_0 = c2; h.vC = vC; h.sC = sC;
  return 0;
}

int brr_session_set_restart(brr_session *s, double mu, const double *beta, double sigmaE,
                            const double *sigmaGG, const double *eps, const double *comp) {
  if (!s || !beta || !sigmaGG || !eps || !comp) { set_error("null argument"); return -1; }
  std::vector<int> c((size_t)s->M);
  for (int64_t m = 0; m < s->M; ++m) {
    const int k = (int)comp[m];  // Eigen indexes v(g, components(i)) with a double
    if (k < 0 || k >= s->K) { set_error("components[%lld]=%g outside [0,%d)", (long long)m, comp[m], s->K); return -1; }
    c[(size_t)m] = k;
  }
  s->mu0 = mu;
  s->sigmaE0 = sigmaE;
  int rc = h2d(s, s->d.beta, beta, s->M);
  rc = rc ? rc : h2d(s, s->d.comp, c.data(), s->M);
  rc = rc ? rc : h2d(s, s->d.sigmaGG, sigmaGG, s->G);
  rc = rc ? rc : h2d(s, s->d.eps, eps, s->N);
  return rc;
}

int brr_session_set_pi(brr_session *s, const double *pi) {
  if (!s || !pi) return -1;
  s->pi_given = true;
  return h2d(s, s->d.pi, pi, (int64_t)s->G * s->K);
}

int brr_session_init(brr_session *s, int32_t seed) {
  if (!s) return -1;
  if (s->model == MODEL_RESTART && s->nshard > 1 && !s->comm) {
    set_error("restart across column shards sums the component counts at init: brr_session_comm_init "
              "first, or drive brr_session_init_local / exchange / brr_session_init_finish yourself");
    return -1;
  }
  Coll c{{s}};
  return coll_init(c, seed);
}

int brr_session_init_local(brr_session *s, int32_t seed) {
  if (!s) return -1;
  if (s->comm) { set_error("init_local is for sessions without a communicator: use brr_session_init"); return -1; }
  Coll c{{s}};
  return coll_init(c, seed);
}

int brr_session_init_finish(brr_session *s) {
  if (!s) return -1;
  if (s->initialized) return 0;  // nothing was left to sum (not a column-sharded restart)
  if (!s->init_pending) { set_error("brr_session_init_local has not run"); return -1; }
  HIPCHK(hipSetDevice(s->device));
  return init_finish(s, s->ex_stats);
}

int brr_session_sweep(brr_session *s, int32_t n) { return brr::session_sweep(s, n, true); }

}  // extern "C"

int brr::session_sweep(brr_session *s, int n, bool check) {
  if (!s) return -1;
  if (s->nrshard > 1) {
    Coll c{{s}};
    for (int r = 0; r < n; ++r)
      if (int rc = coll_sweep_rows(c)) return rc;
    return check_device_error(s);
  }
  // BRR_EXCHANGE_LOOPBACK=1 (measurement): a column shard without a communicator sweeps as one rank of
  // a multi-GPU job whose other ranks changed nothing -- the exchange buffers already hold the sum
  // then -- so one GPU times a rank's real workload with every exchange segment, minus the collective
  // itself (bench.py --rank-of)
  static const bool loopback = getenv("BRR_EXCHANGE_LOOPBACK") && getenv("BRR_EXCHANGE_LOOPBACK")[0] == '1';
  if (s->nshard > 1 && !s->comm && !loopback) {
    set_error("sharded session without a communicator: brr_session_comm_init, or drive "
              "sweep_local / exchange / sweep_finish yourself");
    return -1;
  }
  HIPCHK(hipSetDevice(s->device));
  if (s->nshard > 1 && !s->comm)
    if (int rc = brr_session_exchange_buffers(s, nullptr, nullptr)) return rc;
  // BRR_SEGMENT_CHECK=0: no device check between exchange segments (measurement of its cost)
  static const bool seg_check = !(getenv("BRR_SEGMENT_CHECK") && getenv("BRR_SEGMENT_CHECK")[0] == '0');
  int seg_rc = 0;
  for (int r = 0; r < n; ++r) {
    for (int e = 0; e < s->nex; ++e) {
      const bool last = s->seg == s->nex - 1;
      if (int rc = do_sweep_local(s)) return rc;
      // an exchange segment before the sweep's last: the device check, as sweep_local's callers get it
      // (a failed census moves the sweep's later segments onto the per-block kernels instead of fused
      // launches whose census could no longer pass).  The error is returned after the loop: every rank
      // still takes part in every collective of the sweep.
      if (seg_check && s->nex > 1 && s->fused.nsg > 0 && !last)
        if (int rc = check_device_error(s, true)) seg_rc = rc;
      if (s->nshard > 1 && s->comm) {
        // the exchange step of the column-sharded sweep (E per sweep): the sum of the
        // residual deltas (N doubles) and, after the sweep's last segment only, of the marker
        // statistics (NS; zeros before), in place on the session stream -- one collective when the
        // two buffers are adjacent (the session's own, brr_session_exchange_buffers)
        ncclResult_t r1 = ncclSuccess, r2 = ncclSuccess;
        if (s->ex_stats == s->ex_eps + s->N) {
          r1 = ncclAllReduce(s->ex_eps, s->ex_eps, (size_t)(s->N + (last ? s->NS : 0)), ncclDouble, ncclSum, s->comm, s->st);
        } else {
          r1 = ncclAllReduce(s->ex_eps, s->ex_eps, (size_t)s->N, ncclDouble, ncclSum, s->comm, s->st);
          if (last) r2 = ncclAllReduce(s->ex_stats, s->ex_stats, (size_t)s->NS, ncclDouble, ncclSum, s->comm, s->st);
        }
        if (r1 != ncclSuccess || r2 != ncclSuccess) {
          set_error("ncclAllReduce failed: %s", ncclGetErrorString(r1 != ncclSuccess ? r1 : r2));
          return -2;
        }
      }
      if (int rc = do_sweep_finish(s)) return rc;
    }
  }
  if (check)
    if (int rc = check_device_error(s)) return rc;
  return seg_rc;
}

extern "C" {

int brr_comm_unique_id(void *out) {
  if (!out) return -1;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) { set_error("ncclGetUniqueId: %s", ncclGetErrorString(r)); return -2; }
  std::memcpy(out, &id, sizeof id);
  return 0;
}

int brr_session_comm_init(brr_session *s, const void *unique_id, int32_t nranks, int32_t rank) {
  if (!s || !unique_id) return -1;
  if (s->nrshard > 1) {  // row shards: only the communicator (no residual exchange buffers)
    if (nranks != s->nrshard || rank != s->rshard) {
      set_error("comm (%d ranks, rank %d) does not match the session's row shards (%d, %d)", nranks, rank,
                s->nrshard, s->rshard);
      return -1;
    }
    HIPCHK(hipSetDevice(s->device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof id);
    ncclResult_t r = ncclCommInitRank(&s->comm, nranks, id, rank);
    if (r != ncclSuccess) { set_error("ncclCommInitRank: %s", ncclGetErrorString(r)); s->comm = nullptr; return -2; }
    return 0;
  }
  if (nranks != s->nshard || rank != s->shard) {
    set_error("comm (%d ranks, rank %d) does not match the session's shards (%d, %d)", nranks, rank,
              s->nshard, s->shard);
    return -1;
  }
  HIPCHK(hipSetDevice(s->device));
  double *e = nullptr, *st = nullptr;
  if (int rc = brr_session_exchange_buffers(s, &e, &st)) return rc;
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof id);
  ncclResult_t r = ncclCommInitRank(&s->comm, nranks, id, rank);
  if (r != ncclSuccess) { set_error("ncclCommInitRank: %s", ncclGetErrorString(r)); s->comm = nullptr; return -2; }
  return 0;
}

int brr_session_exchange_sizes(brr_session *s, int64_t *n_eps, int64_t *n_stats) {
  if (!s) return -1;
  if (n_eps) *n_eps = s->N;
  if (n_stats) *n_stats = s->NS;
  return 0;
}

int brr_session_set_exchange(brr_session *s, double *dev_eps, double *dev_stats) {
  if (!s) return -1;
  s->ex_eps = dev_eps;
  s->ex_stats = dev_stats;
  return 0;
}

int brr_session_exchange_buffers(brr_session *s, double **dev_eps, double **dev_stats) {
  if (!s) return -1;
  if (!s->ex_eps || !s->ex_stats) {
    // one allocation, the statistics right after the residual deltas: a sweep's exchange is then
    // ONE ncclAllReduce of N + NS doubles (N alone after an earlier exchange segment)
    HIPCHK(hipSetDevice(s->device));
    if (s->alloc(&s->ex_eps, s->N + s->NS)) return -2;
    s->ex_stats = s->ex_eps + s->N;
    HIPCHK(hipMemset(s->ex_eps, 0, sizeof(double) * (s->N + s->NS)));
    s->ex_owned = true;
  }
  if (dev_eps) *dev_eps = s->ex_eps;
  if (dev_stats) *dev_stats = s->ex_stats;
  return 0;
}

int brr_session_exchange_copy(brr_session *s, int32_t dir, double *host_eps, double *host_stats) {
  if (!s || !s->ex_eps) { set_error("no exchange buffers"); return -1; }
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipStreamSynchronize(s->st));
  const hipMemcpyKind k = dir == 0 ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice;
  if (host_eps)
    HIPCHK(dir == 0 ? hipMemcpy(host_eps, s->ex_eps, sizeof(double) * s->N, k)
                    : hipMemcpy(s->ex_eps, host_eps, sizeof(double) * s->N, k));
  if (host_stats)
    HIPCHK(dir == 0 ? hipMemcpy(host_stats, s->ex_stats, sizeof(double) * s->NS, k)
                    : hipMemcpy(s->ex_stats, host_stats, sizeof(double) * s->NS, k));
  return 0;
}

int brr_session_sweep_local(brr_session *s) {
  if (!s) return -1;
  HIPCHK(hipSetDevice(s->device));
  int rc = do_sweep_local(s);
  // exchange buffers complete for the caller; a protocol timeout or failed residency census of
  // this launch is reported here (as brr_session_sweep does), not left for a later sweep to trip on
  if (rc == 0) rc = check_device_error(s, true);
  return rc;
}

int brr_session_sweep_finish(brr_session *s) {
  if (!s) return -1;
  HIPCHK(hipSetDevice(s->device));
  return do_sweep_finish(s);
}

int32_t brr_session_exchanges_per_sweep(brr_session *s) { return s ? s->nex : -1; }

int brr_session_get_scalar(brr_session *s, int32_t which, double *out) {
  if (!s || !out) return -1;
  HIPCHK(hipSetDevice(s->device));
  if (int rc = ensure_reduced(s)) return rc;
  Scal sc;
  if (int rc = d2h(s, &sc, s->d.sc, 1)) return rc;
  switch (which) {
    case BRR_MU: *out = sc.mu; return 0;
    case BRR_SIGMAE: *out = sc.sigmaE; return 0;
    case BRR_SIGMAF: *out = sc.sigmaF; return 0;
    case BRR_TAU: *out = sc.tau; return 0;
    case BRR_ETA: *out = sc.eta; return 0;
    case BRR_C2: *out = sc.c2; return 0;
    case BRR_SIGMAG: return d2h(s, out, s->d.sigmaGG, 1);
    case BRR_SUMSQ_BETA: return d2h(s, out, s->d.stats, 1);
    case 100: *out = (double)sc.n_slow; return 0;     // diagnostics (not in brr.h)
    case 101: *out = (double)sc.n_changed; return 0;
    case 102: *out = (double)sc.prof_on; return 0;
    case 104: *out = (double)s->fused.nsg; return 0;  // fused sweep: streaming workgroups (0 = per-block)
    case 105: *out = (double)(s->fused.ccache || s->d.xcodes != nullptr); return 0;  // fused sweep: code cache in LDS
    case 106: *out = (double)s->d.lag; return 0;  // pipeline lag
    case 107: *out = (double)s->gram_np_init; return 0;  // Gram kernel: class planes of k_gram_int (0 = FP64 k_gram)
    case 130: *out = (double)s->census_failures; return 0;  // residency census failures so far
    case 131: *out = (double)s->fused.nred; return 0;       // fused sweep: reducer workgroups (column slices)
    case 132: *out = (double)s->ovs_last; return 0;         // the latest fused launch ran the overlapped solver
    case 109: *out = (double)(s->fused.nsg > 0 ? s->fused.stnt : 0); return 0;  // threads per streaming workgroup
    case 108: *out = (double)(s->fused.nsg > 0 && sc.lag_next >= 2 ? s->d.lag : 1); return 0;  // the next sweep's pipeline lag
    case 110: case 111: case 112: case 113: case 114: case 115: case 116: case 117: case 118: case 119:
    case 120: case 121: case 122: case 123: case 124: case 125: case 126: case 127: case 128: case 129:
      *out = (double)sc.prof[which - 110]; return 0;
    default: set_error("unknown scalar %d", which); return -1;
  }
}

int brr_session_set_scalar(brr_session *s, int32_t which, double v) {
  if (!s) return -1;
  HIPCHK(hipSetDevice(s->device));
  Scal sc;
  if (int rc = d2h(s, &sc, s->d.sc, 1)) return rc;
  switch (which) {
    case BRR_MU: sc.mu = v; break;
    case BRR_SIGMAE: sc.sigmaE = v; break;
    case BRR_SIGMAF: sc.sigmaF = v; break;
    case BRR_TAU: sc.tau = v; break;
    case BRR_ETA: sc.eta = v; break;
    case BRR_C2: sc.c2 = v; break;
    case BRR_SIGMAG: return h2d(s, s->d.sigmaGG, &v, 1);
    case 102:  // diagnostics: k_solve phase timers on/off (resets the totals)
      sc.prof_on = v != 0.0;
      s->prof_on = sc.prof_on != 0;
      for (auto &x : sc.prof) x = 0;
      HIPCHK(hipMemsetAsync(s->d.trace, 0, sizeof(unsigned long long) * (16 * (size_t)s->nb + 9216), s->st));
      break;
    default: set_error("scalar %d not settable", which); return -1;
  }
  s->need_reduce = true;
  return h2d(s, s->d.sc, &sc, 1);
}

static int64_t rc_or(int rc, int64_t n) { return rc ? rc : n; }

int64_t brr_session_get_vector(brr_session *s, int32_t which, double *out) {
  if (!s) return -1;
  if (hipSetDevice(s->device) != hipSuccess) return -2;
  int64_t n = -1;
  switch (which) {
    case BRR_BETA: case BRR_COMP: case BRR_LAMBDA: case BRR_XSQ: case BRR_ORDER: case BRR_HSV: n = s->M; break;
    case BRR_EPS: n = s->N; break;
    case BRR_SIGMAGG: case BRR_BETAACUM: n = s->G; break;
    case BRR_PI: case BRR_VCOUNT: n = (int64_t)s->G * s->K; break;
    case BRR_ALPHA: n = s->F; break;
    case 200: n = s->M; break;  // diagnostics: column sums of the device X (not in brr.h)
    case 201: n = (int64_t)s->nb * 16 + 9216; break;  // diagnostics: per-block event trace (brr_kernels.hip TR_*)
    case 202: case 203: n = (int64_t)s->nb * s->B * s->B; break;  // diagnostics: the Gram / cross-Gram blocks
    default: set_error("unknown vector %d", which); return -1;
  }
  if (!out) return n;
  if (which == 201) {
    std::vector<unsigned long long> tr((size_t)n);
    if (int rc = d2h(s, tr.data(), s->d.trace, n)) return rc;
    for (int64_t i = 0; i < n; ++i) out[i] = (double)tr[(size_t)i];
    return n;
  }
  if (which == 202 || which == 203) return (rc_or(d2h(s, out, which == 202 ? s->d.gram : s->d.xgram, n), n));
  if (which == 200) {
    std::vector<float> x((size_t)(s->d.ld * s->M));
    if (s->x2bit) {
      std::vector<uint8_t> c((size_t)(s->d.ldc * s->nb * s->B));
      std::vector<float> l((size_t)(4 * s->M));
      if (int rc = d2h(s, c.data(), s->d.Xc, (int64_t)c.size())) return rc;
      if (int rc = d2h(s, l.data(), s->d.xlut, (int64_t)l.size())) return rc;
      for (int64_t j = 0; j < s->M; ++j)
        for (int64_t i = 0; i < s->d.ld; ++i)
          x[(size_t)(j * s->d.ld + i)] = l[(size_t)(4 * j + ((c[(size_t)((((j / s->B) * (s->B >> 4) + ((j % s->B) >> 4)) * s->d.ldc + (i >> 2)) * 16 + (j % s->B & 15))] >> (2 * (i & 3))) & 3))];
    } else if (int rc = d2h(s, x.data(), s->d.X, (int64_t)x.size())) {
      return rc;
    }
    for (int64_t j = 0; j < s->M; ++j) {
      double a = 0;
      for (int64_t i = 0; i < s->d.ld; ++i) a += std::fabs((double)x[(size_t)(j * s->d.ld + i)]);
      out[j] = a;
    }
    return n;
  }
  int rc = 0;
  switch (which) {
    case BRR_BETA: rc = d2h(s, out, s->d.beta, n); break;
    case BRR_EPS: rc = d2h(s, out, s->d.eps, n); break;
    case BRR_LAMBDA: rc = d2h(s, out, s->d.lambda, n); break;
    case BRR_HSV: rc = d2h(s, out, s->d.hsv, n); break;
    case BRR_XSQ: rc = d2h(s, out, s->d.xsq, n); break;
    case BRR_SIGMAGG: rc = d2h(s, out, s->d.sigmaGG, n); break;
    case BRR_PI: rc = d2h(s, out, s->d.pi, n); break;
    case BRR_ALPHA: rc = d2h(s, out, s->d.alpha, n); break;
    case BRR_BETAACUM: rc = d2h(s, out, s->d.stats + 2, n); break;
    case BRR_VCOUNT: rc = d2h(s, out, s->d.stats + 2 + s->G, n); break;
    case BRR_COMP: {
      std::vector<int> c((size_t)n);
      rc = d2h(s, c.data(), s->d.comp, n);
      for (int64_t i = 0; i < n; ++i) out[i] = c[(size_t)i];
      break;
    }
    case BRR_ORDER: {
      std::vector<int> mem((size_t)s->nb * s->B), bsz((size_t)s->nb);
      rc = d2h(s, mem.data(), s->d.member, (int64_t)mem.size());
      rc = rc ? rc : d2h(s, bsz.data(), s->d.bsz, s->nb);
      int64_t k = 0;
      for (int b = 0; b < s->nb; ++b)
        for (int i = 0; i < bsz[(size_t)b]; ++i) out[k++] = (double)(s->col_offset + mem[(size_t)b * s->B + i]);
      break;
    }
  }
  return rc ? rc : n;
}

int brr_session_set_vector(brr_session *s, int32_t which, const double *in) {
  if (!s || !in) return -1;
  HIPCHK(hipSetDevice(s->device));
  int rc = 0;
  switch (which) {
    case BRR_BETA: rc = h2d(s, s->d.beta, in, s->M); break;
    case BRR_EPS: rc = h2d(s, s->d.eps, in, s->N); s->need_reduce = true; break;
    case BRR_LAMBDA: rc = h2d(s, s->d.lambda, in, s->M); break;
    case BRR_SIGMAGG: rc = h2d(s, s->d.sigmaGG, in, s->G); break;
    case BRR_PI: rc = h2d(s, s->d.pi, in, (int64_t)s->G * s->K); break;
    case BRR_ALPHA: rc = h2d(s, s->d.alpha, in, s->F); break;
    case BRR_COMP: {
      std::vector<int> c((size_t)s->M);
      for (int64_t i = 0; i < s->M; ++i) c[(size_t)i] = (int)in[i];
      rc = h2d(s, s->d.comp, c.data(), s->M);
      break;
    }
    default: set_error("vector %d not settable", which); return -1;
  }
  return rc;
}

int brr_session_linear_predictor(brr_session *s, double *out) {
  if (!s || !out) { set_error("linear_predictor: null argument"); return -1; }
  if (!s->have_x) { set_error("linear_predictor: X not uploaded"); return -1; }
  double *tmp = nullptr;
  if (int rc = dalloc(&tmp, s->N)) return rc;
  int rc = 0;
  if (launch_linpred(s->d, tmp, s->st) != hipSuccess || hipStreamSynchronize(s->st) != hipSuccess ||
      hipMemcpy(out, tmp, sizeof(double) * (size_t)s->N, hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("linear_predictor: %s", hipGetErrorString(hipGetLastError()));
    rc = -2;
  }
  (void)hipFree(tmp);
  return rc;
}

int32_t brr_session_iteration(brr_session *s) { return s ? s->iteration : -1; }

int brr_session_set_timing(brr_session *s, int32_t on) {
  if (!s) return -1;
  if (int rc = collect_timing(s)) return rc;
  s->timing = on != 0;
  if (on) {
    s->t_stream = s->t_solve = s->t_solve_sweep = 0;
    s->n_stream = s->n_solve = s->n_solve_sweep = 0;
  }
  return 0;
}

int brr_session_timing(brr_session *s, double *stream_ms, int64_t *n_stream, double *solve_ms,
                       int64_t *n_solve) {
  if (!s) return -1;
  if (int rc = collect_timing(s)) return rc;
  if (stream_ms) *stream_ms = s->t_stream;
  if (n_stream) *n_stream = s->n_stream;
  // the persistent solver is timed per sweep: reported per block position (waits included)
  if (solve_ms) *solve_ms = s->t_solve + s->t_solve_sweep;
  if (n_solve) *n_solve = s->n_solve + s->n_solve_sweep * s->nb;
  return 0;
}

int64_t brr_session_block_size(brr_session *s) { return s ? s->B : -1; }

// ---------------------------------------------------------------------------------------
// In-process row-shard group
struct brr_group {
  Coll c;
};

brr_group *brr_group_create(brr_session *const *members, int32_t n) {
  if (!members || n < 1 || n > GROUP_MAX) { set_error("brr_group_create: 1 .. %d members", GROUP_MAX); return nullptr; }
  brr_group *g = new brr_group();
  for (int i = 0; i < n; ++i) {
    brr_session *s = members[i];
    if (!s || s->nrshard != n || s->rshard != i) {
      set_error("brr_group_create: member %d must be row shard %d of %d", i, i, n);
      delete g;
      return nullptr;
    }
    const brr_session *a = members[0];
    if (s->model != a->model || s->M != a->M || s->B != a->B || s->K != a->K || s->G != a->G || s->F != a->F ||
        s->order_mode != a->order_mode || s->d.Ntot != a->d.Ntot) {
      set_error("brr_group_create: member %d differs from member 0 (model, M, B, K, groups, F, order, N_total)", i);
      delete g;
      return nullptr;
    }
    if (s->device != a->device) {  // members on other GPUs: the sum kernel runs on member 0's device
      (void)hipSetDevice(a->device);
      const hipError_t e = hipDeviceEnablePeerAccess(s->device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        set_error("brr_group_create: no peer access from device %d to %d", a->device, s->device);
        delete g;
        return nullptr;
      }
      (void)hipGetLastError();
    }
    g->c.ss.push_back(s);
  }
  return g;
}

int brr_group_init(brr_group *g, int32_t seed) {
  if (!g) return -1;
  return coll_init(g->c, seed);
}

int brr_group_sweep(brr_group *g, int32_t n) {
  if (!g) return -1;
  for (int r = 0; r < n; ++r)
    if (int rc = coll_sweep_rows(g->c)) return rc;
  for (brr_session *s : g->c.ss) {
    HIPCHK(hipSetDevice(s->device));
    if (int rc = check_device_error(s)) return rc;
  }
  return 0;
}

void brr_group_destroy(brr_group *g) { delete g; }

int brr_session_synchronize(brr_session *s) {
  if (!s) return -1;
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipStreamSynchronize(s->st));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// Sample output ring (brr_sample.hpp)
namespace brr {

brr_options options_from_caller(const brr_options *in) {
  brr_options o;
  brr_options_default(&o);
  if (in) {
    // an older caller's struct: only the part its ABI had is read, the rest keeps the defaults.
    // exchanges_per_sweep = 0 means automatic (E = 8) for every ABI: ABI 3's header documented that
    // (with "query brr_session_exchanges_per_sweep() and run E rounds" for the hand-driven protocol),
    // and ABI 1 / 2 structs, which have no such field, get the default
    if (in->abi_version >= 3) o = *in;
    else if (in->abi_version == 2) std::memcpy(&o, in, offsetof(brr_options, exchanges_per_sweep));
    else std::memcpy(&o, in, offsetof(brr_options, row_shard_rank));
    o.abi_version = BRR_ABI_VERSION;
  }
  if (o.exchanges_per_sweep < 0) o.exchanges_per_sweep = 0;
  return o;
}

int sample_ring_open(brr_session *s, int depth) {
  sample_ring_close(s);
  SampleRing &r = s->ring;
  if (depth < 1) depth = 1;
  HIPCHK(hipSetDevice(s->device));
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  size_t o = al(sizeof(Scal));
  r.o_beta = o; o += al(8 * (size_t)s->M);
  r.o_eps = o; o += al(8 * (size_t)s->N);
  r.o_lam = o; o += s->model == MODEL_HORSESHOE ? al(8 * (size_t)s->M) : 0;
  r.o_sgg = o; o += al(8 * (size_t)s->G);
  r.o_alpha = o; o += al(8 * (size_t)std::max(s->F, 1));
  r.o_comp = o; o += al(4 * (size_t)s->M);
  r.bytes = o;
  HIPCHK(hipStreamCreateWithFlags(&r.cst, hipStreamNonBlocking));
  r.depth = depth;
  r.dbuf.assign(depth, nullptr);
  r.hbuf.assign(depth, nullptr);
  r.ev_snap.assign(depth, nullptr);
  r.ev_host.assign(depth, nullptr);
  r.busy.assign(depth, 0);
  r.next = r.in_use = r.max_in_use = 0;
  for (int i = 0; i < depth; ++i) {
    HIPCHK(hipMalloc((void **)&r.dbuf[i], r.bytes));
    HIPCHK(hipHostMalloc((void **)&r.hbuf[i], r.bytes, hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&r.ev_snap[i], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&r.ev_host[i], hipEventDisableTiming));
  }
  return 0;
}

int sample_ring_push(brr_session *s, int *slot_out) {
  SampleRing &r = s->ring;
  if (r.depth == 0) { set_error("sample ring not open"); return -1; }
  int slot;
  {
    std::unique_lock<std::mutex> lk(r.mu);
    r.cv.wait(lk, [&] { return !r.busy[r.next]; });  // back-pressure: the writer is r.depth rows behind
    slot = r.next;
    r.busy[slot] = 1;
    r.next = (r.next + 1) % r.depth;
    r.max_in_use = std::max(r.max_in_use, ++r.in_use);
  }
  // the snapshot and its copy; on any failure the claimed slot goes back to the ring (a failing
  // push must not shrink the ring until a later push blocks for ever)
  auto enqueue = [&]() -> int {
    HIPCHK(hipSetDevice(s->device));
    if (int rc = ensure_reduced(s)) return rc;
    char *d = r.dbuf[slot];
    const Dev &dv = s->d;
    auto cp = [&](size_t off, const void *src, size_t n) {
      return n ? hipMemcpyAsync(d + off, src, n, hipMemcpyDeviceToDevice, s->st) : hipSuccess;
    };
    HIPCHK(cp(0, dv.sc, sizeof(Scal)));
    HIPCHK(cp(r.o_beta, dv.beta, 8 * (size_t)s->M));
    HIPCHK(cp(r.o_eps, dv.eps, 8 * (size_t)s->N));
    if (s->model == MODEL_HORSESHOE) HIPCHK(cp(r.o_lam, dv.lambda, 8 * (size_t)s->M));
    HIPCHK(cp(r.o_sgg, dv.sigmaGG, 8 * (size_t)s->G));
    if (s->F > 0) HIPCHK(cp(r.o_alpha, dv.alpha, 8 * (size_t)s->F));
    HIPCHK(cp(r.o_comp, dv.comp, 4 * (size_t)s->M));
    HIPCHK(hipEventRecord(r.ev_snap[slot], s->st));
    HIPCHK(hipStreamWaitEvent(r.cst, r.ev_snap[slot], 0));
    HIPCHK(hipMemcpyAsync(r.hbuf[slot], d, r.bytes, hipMemcpyDeviceToHost, r.cst));
    HIPCHK(hipEventRecord(r.ev_host[slot], r.cst));
    return 0;
  };
  if (int rc = enqueue()) {
    sample_ring_release(s, slot);
    return rc;
  }
  *slot_out = slot;
  return 0;
}

int sample_ring_wait(brr_session *s, int slot, SampleView *v) {
  SampleRing &r = s->ring;
  HIPCHK(hipEventSynchronize(r.ev_host[slot]));
  const char *h = r.hbuf[slot];
  v->sc = reinterpret_cast<const Scal *>(h);
  v->beta = reinterpret_cast<const double *>(h + r.o_beta);
  v->eps = reinterpret_cast<const double *>(h + r.o_eps);
  v->lam = reinterpret_cast<const double *>(h + r.o_lam);
  v->sgg = reinterpret_cast<const double *>(h + r.o_sgg);
  v->alpha = reinterpret_cast<const double *>(h + r.o_alpha);
  v->comp = reinterpret_cast<const int32_t *>(h + r.o_comp);
  return 0;
}

void sample_ring_release(brr_session *s, int slot) {
  SampleRing &r = s->ring;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    r.busy[slot] = 0;
    --r.in_use;
  }
  r.cv.notify_all();
}

int sample_ring_max_in_use(brr_session *s) { return s->ring.max_in_use; }

void sample_ring_close(brr_session *s) {
  SampleRing &r = s->ring;
  if (r.depth == 0) return;
  (void)hipSetDevice(s->device);
  if (r.cst) (void)hipStreamSynchronize(r.cst);
  for (int i = 0; i < r.depth; ++i) {
    if (r.dbuf[i]) (void)hipFree(r.dbuf[i]);
    if (r.hbuf[i]) (void)hipHostFree(r.hbuf[i]);
    if (r.ev_snap[i]) (void)hipEventDestroy(r.ev_snap[i]);
    if (r.ev_host[i]) (void)hipEventDestroy(r.ev_host[i]);
  }
  if (r.cst) (void)hipStreamDestroy(r.cst);
  r.cst = nullptr;
  r.depth = 0;
  r.dbuf.clear(); r.hbuf.clear(); r.ev_snap.clear(); r.ev_host.clear(); r.busy.clear();
}

}  // namespace brr
