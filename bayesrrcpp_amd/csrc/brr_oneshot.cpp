// brr_oneshot.cpp -- the four drop-in entry points with the reference's signatures and file
// semantics (include/brr.h), built on the session API.
//
// Sample output replaces the reference's moodycamel::ConcurrentQueue<VectorXd> + writer
// section (src/BayesRv2.cpp:62,257-290): kept iterations are copied device->host into a row
// and handed to a writer thread that formats them like Eigen's
// IOFormat(StreamPrecision, DontAlignCols, ", ", ...) (6 significant digits, ", " separators,
// BayesRv2.cpp:72).  Unlike the reference the queue is always drained
// before returning and HorseshoeR writes every kept sample.
#include <hip/hip_runtime.h>

#include <charconv>
#include <chrono>
#include <map>
#include <memory>
#include <condition_variable>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/brr.h"
#include "brr_sample.hpp"

namespace {

struct Log {
  brr_log_fn fn = nullptr;
  void *user = nullptr;
  void operator()(const std::string &m) const {
    if (fn) fn(m.c_str(), user); else fputs(m.c_str(), stderr);
  }
};

// The writer thread: header strings and sample slots (brr_sample.hpp) in order.  A sample row is
// formatted straight from the slot's pinned host copy, then the slot is released to the sampler.
class CsvWriter {
 public:
  explicit CsvWriter(FILE *f) : f_(f), th_([this] { run(); }) {}
  ~CsvWriter() { close(); }
  void header(const std::string &h) { push({true, h, -1, 0}); }
  // the row layout of the session's model (BayesRv2.cpp:261-272, BayesRv2Groups.cpp:317,
  // BRv2Grstart.cpp:267, HorseshoeR.cpp:258)
  void bind(brr_session *s, int model, int64_t N, int64_t M, int G, int64_t F) {
    s_ = s; model_ = model; N_ = N; M_ = M; G_ = G; F_ = F;
  }
  void sample(int slot, int iteration) { push({false, std::string(), slot, iteration}); }
  int error() const { return err_; }
  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (done_) return;
      done_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();  // drain everything queued (the reference may drop rows)
  }
  // after close(): cut the file back to the headers and the first n sample rows (a failed chain keeps
  // only the rows of states a device check confirmed)
  void truncate_rows(int64_t n) {
    const int64_t off = n <= 0 ? hdr_end_ : row_end_[(size_t)std::min<int64_t>(n, (int64_t)row_end_.size()) - 1];
    fflush(f_);
    if (ftruncate(fileno(f_), (off_t)off) != 0) err_ = -3;
    fseek(f_, 0, SEEK_END);
  }

 private:
  struct Item { bool is_header; std::string h; int slot; int iteration; };
  void push(Item &&it) {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(it));
    cv_.notify_one();
  }
  void put(double v) {
    if (!first_) buf_ += ", ";
    first_ = false;
    // %g (6 significant digits, Eigen StreamPrecision, BayesRv2.cpp:72) without printf's
    // locale and parsing overhead: std::to_chars with the general format and precision 6 is
    // specified as printf("%.6g")
    const auto res = std::to_chars(num_, num_ + sizeof num_, v, std::chars_format::general, 6);
    buf_.append(num_, (size_t)(res.ptr - num_));
  }
  void put(const double *v, int64_t n) { for (int64_t i = 0; i < n; ++i) put(v[i]); }
  void format(const brr::SampleView &v, int iteration) {
    buf_.clear();
    first_ = true;
    put((double)iteration);
    put(v.sc->mu);
    put(v.beta, M_);
    put(v.sc->sigmaE);
    if (model_ == BRR_MODEL_HORSESHOE) {
      put(v.sc->tau);
      put(v.lam, M_);
      put(v.eps, N_);
      put(0.0);  // sample has 2M+4+N slots, 2M+N+3 values (HorseshoeR.cpp:157,258)
    } else {
      if (model_ == BRR_MODEL_V2) put(v.sgg[0]);
      for (int64_t i = 0; i < M_; ++i) put((double)v.comp[i]);
      if (model_ != BRR_MODEL_V2) put(v.sgg, G_);
      put(v.eps, N_);
      if (model_ == BRR_MODEL_GROUPS) {
        put(v.alpha, F_);
        put(v.sc->sigmaF);
      }
    }
    buf_ += '\n';
  }
  void run() {
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return done_ || !q_.empty(); });
        if (q_.empty()) return;
        it = std::move(q_.front());
        q_.pop_front();
      }
      if (it.is_header) {
        fputs(it.h.c_str(), f_);
        pos_ += (int64_t)it.h.size();
        hdr_end_ = pos_;
        continue;
      }
      brr::SampleView v;
      if (brr::sample_ring_wait(s_, it.slot, &v) != 0) {
        err_ = -2;
      } else {
        format(v, it.iteration);
        fwrite(buf_.data(), 1, buf_.size(), f_);
        pos_ += (int64_t)buf_.size();
      }
      row_end_.push_back(pos_);  // (a failed row leaves the offset unchanged)
      brr::sample_ring_release(s_, it.slot);
    }
  }
  FILE *f_;
  brr_session *s_ = nullptr;
  int model_ = 0, G_ = 1;
  int64_t N_ = 0, M_ = 0, F_ = 0;
  std::string buf_;
  char num_[40];
  bool first_ = true;
  int err_ = 0;
  int64_t pos_ = 0, hdr_end_ = 0;  // bytes written; end of the headers
  std::vector<int64_t> row_end_;   // file offset after each sample row, in order
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> q_;
  bool done_ = false;
  std::thread th_;
};

std::string hdr_v2(int64_t M, int64_t N) {  // BayesRv2.cpp:16-37
  std::string h = "iteration,mu,";
  for (int64_t i = 0; i < M; ++i) h += "beta[" + std::to_string(i + 1) + "],";
  h += "sigmaE,sigmaG,";
  for (int64_t i = 0; i < M; ++i) h += "comp[" + std::to_string(i + 1) + "],";
  for (int64_t i = 0; i < N - 1; ++i) h += "epsilon[" + std::to_string(i + 1) + "],";
  h += "epsilon[" + std::to_string(N) + "]\n";
  return h;
}

std::string hdr_groups(int64_t M, int64_t N, int G, int64_t F) {  // BayesRv2Groups.cpp:25-54
  std::string h = "iteration,mu,";
  for (int64_t i = 0; i < M; ++i) h += "beta[" + std::to_string(i + 1) + "],";
  h += "sigmaE,";
  for (int64_t i = 0; i < M; ++i) h += "comp[" + std::to_string(i + 1) + "],";
  for (int g = 0; g < G; ++g) h += "sigmaG[" + std::to_string(g + 1) + "],";
  for (int64_t i = 0; i < N - 1; ++i) h += "epsilon[" + std::to_string(i + 1) + "],";
  h += "epsilon[" + std::to_string(N) + "],";
  for (int64_t i = 0; i < F; ++i) h += "alpha[" + std::to_string(i + 1) + "],";
  h += "sigmaF\n";
  return h;
}

std::string hdr_hs(int64_t M, int64_t N) {  // HorseshoeR.cpp:279-291
  std::string h = "iteration,mu,";
  for (int64_t i = 0; i < M; ++i) h += "beta[" + std::to_string(i + 1) + "],";
  h += "sigmaE,tau,";
  for (int64_t i = 0; i < M; ++i) h += "lambda[" + std::to_string(i + 1) + "],";
  for (int64_t i = 0; i < N; ++i) h += "epsilon[" + std::to_string(i + 1) + "],";
  h += "\n";
  return h;
}

bool bad_iterations(int max_it, int burn_in, int thinning) {
  // BayesRv2.cpp:76; thinning < 1 would be a modulo by zero at :259 (SIGFPE) in the reference
  return max_it < burn_in || max_it < 1 || burn_in < 1 || thinning < 1;
}

const char *kIterMsg =
    "error: burn_in has to be a positive integer and smaller than the maximum number of iterations ";

void hyper_warnings(const Log &log, double sigma0, double v0E, double s02E, double v0G, double s02G,
                    const double *cva, int64_t n) {
  // BayesRv2.cpp:81-95 -- warnings only (the reference's `return` is commented out)
  if (sigma0 < 0 || v0E < 0 || s02E < 0 || v0G < 0 || s02G < 0) log("error: hyper parameters have to be positive");
  bool zero = false, neg = false;
  for (int64_t i = 0; i < n; ++i) { zero |= cva[i] == 0.0; neg |= cva[i] < 0.0; }
  if (zero) log("error: the zero component is already included in the model by default");
  if (neg) log("error: the variance of the components should be positive");
}

// BRR_TIMELINE=1: a host-side timeline of a one-shot call through the log callback -- one line per
// phase (milliseconds since the call began): open + header, session create, X upload, setters,
// init (Gram blocks), the chain (per 100 iterations: time in sweeps, in sample pushes), the writer's
// drain and the teardown.  Accounts for the end-to-end time of the drop-in path beside the session
// rate (bench.py --oneshot).
struct Timeline {
  bool on = false;
  Log log;
  std::chrono::steady_clock::time_point t0, last;
  explicit Timeline(const Log &l) : log(l) {
    const char *e = getenv("BRR_TIMELINE");
    on = e && e[0] == '1';
    t0 = last = std::chrono::steady_clock::now();
  }
  static double ms(std::chrono::steady_clock::duration d) {
    return std::chrono::duration<double, std::milli>(d).count();
  }
  void mark(const char *phase) {
    if (!on) return;
    const auto t = std::chrono::steady_clock::now();
    char b[160];
    snprintf(b, sizeof b, "timeline %-10s +%9.2f ms  at %9.2f ms\n", phase, ms(t - last), ms(t - t0));
    log(b);
    last = t;
  }
};
struct Run {
  int model;
  const char *out;
  int max_it, burn_in, thin;
  int64_t N, M;
  int G;
  int64_t F;
  Log log;
  bool verbose;
  Timeline *tl;  // the call's timeline (run_chain reports its per-100-iteration lines into it)
};

int fail(brr_session *s, const Log &log, int rc) {
  std::string m = std::string("brr: ") + brr_last_error() + "\n";
  log(m);
  if (s) brr_session_destroy(s);
  return rc < 0 ? rc : -1;
}

// the reference's sweep loop with sample emission (BayesRv2.cpp:171-278).  Kept iterations go
// through the session's sample ring: a device snapshot, an asynchronous copy to pinned memory
// and the writer thread, so the sampler never waits for a row's D2H copy or its formatting
// unless the writer is BRR_SAMPLE_RING (default 4) rows behind.
// *n_ok: the sample rows pushed up to the last device check that passed (on a failure the caller
// keeps only those rows in the file)
int run_chain(brr_session *s, const Run &r, CsvWriter *w, int64_t *n_ok) {
  *n_ok = 0;
  int64_t n_rows = 0;
  const char *rd = getenv("BRR_SAMPLE_RING");
  if (int rc = brr::sample_ring_open(s, rd ? atoi(rd) : 4)) return rc;
  w->bind(s, r.model, r.N, r.M, r.G, r.F);
  const auto t1 = std::chrono::steady_clock::now();
  const int every = r.max_it / 10;  // (int)std::ceil(max_iterations/10): integer division
  double t_sweep = 0, t_push = 0;
  int n_push = 0;
  for (int it = 0; it < r.max_it; ++it) {
    if (r.verbose && it > 0 && every > 0 && it % every == 0) {
      r.log("iteration: " + std::to_string(it) + "\n");
      if (r.model == BRR_MODEL_HORSESHOE) {
        double tau = 0, eta = 0, se = 0;
        brr_session_get_scalar(s, BRR_TAU, &tau);
        brr_session_get_scalar(s, BRR_ETA, &eta);
        brr_session_get_scalar(s, BRR_SIGMAE, &se);
        char b[160];
        snprintf(b, sizeof b, " tau %g\n eta %g\nsigmaE%g\n", tau, eta, se);
        r.log(b);
      }
    }
    const auto ta = std::chrono::steady_clock::now();
    // the device error check (stream sync + read-back) every 16 iterations and at the end: a per-sweep
    // sync left the device idle for the host's launches of every sweep (C1: 7.4 against 6.9 ms)
    const bool check = (it & 15) == 15 || it + 1 == r.max_it;
    if (int rc = brr::session_sweep(s, 1, check)) return rc;
    const auto tb = std::chrono::steady_clock::now();
    t_sweep += std::chrono::duration<double, std::milli>(tb - ta).count();
    if (it >= r.burn_in && it % r.thin == 0) {
      int slot = -1;
      if (int rc = brr::sample_ring_push(s, &slot)) return rc;
      w->sample(slot, it);
      ++n_rows;
      t_push += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count();
      ++n_push;
    }
    if (check) *n_ok = n_rows;  // this sweep's state (and its row) passed the device check
    if (r.tl && r.tl->on && ((it + 1) % 100 == 0 || it + 1 == r.max_it)) {
      char b[200];
      snprintf(b, sizeof b, "timeline chain it %d: sweeps %.2f ms, %d sample pushes %.2f ms\n", it + 1, t_sweep,
               n_push, t_push);
      r.tl->log(b);
      t_sweep = t_push = 0;
      n_push = 0;
    }
  }
  brr_session_synchronize(s);
  const auto t2 = std::chrono::steady_clock::now();
  r.log("duration: " + std::to_string((long long)std::chrono::duration_cast<std::chrono::seconds>(t2 - t1).count()) + "s\n");
  return 0;
}

brr_options opts_or_default(const brr_options *o) { return brr::options_from_caller(o); }


}  // namespace

extern "C" {

int brr_BayesRSamplerV2(const char *outputFile, int seed, int max_iterations, int burn_in,
                        int thinning, const double *X, int64_t N, int64_t M, const double *Y,
                        double sigma0, double v0E, double s02E, double v0G, double s02G,
                        const double *cva, int32_t n_cva, const brr_options *opt_in) {
  brr_options opt = opts_or_default(opt_in);
  Log log{opt.log, opt.log_userdata};
  Timeline tl(log);
  FILE *f = fopen(outputFile, "w");  // BayesRv2.cpp:69
  if (!f) { log(std::string("brr: cannot open ") + outputFile + "\n"); return -3; }
  CsvWriter w(f);
  w.header(hdr_v2(M, N));  // header before validation (:70 vs :76)
  if (bad_iterations(max_iterations, burn_in, thinning)) {
    log(kIterMsg);
    w.close(); fclose(f);
    return 1;
  }
  hyper_warnings(log, sigma0, v0E, s02E, v0G, s02G, cva, n_cva);
  tl.mark("open");
  brr_session *s = brr_session_create(BRR_MODEL_V2, N, M, M, 0, n_cva + 1, 1, 0, &opt);
  tl.mark("create");
  int rc = s ? 0 : -1;
  if (!rc) rc = brr_session_upload_x_f64(s, X, N);
  tl.mark("upload");
  if (!rc) rc = brr_session_set_y(s, Y);
  if (!rc) rc = brr_session_set_bayesr(s, sigma0, v0E, s02E, v0G, s02G, cva, nullptr);
  tl.mark("set");
  if (!rc) rc = brr_session_init(s, seed);
  tl.mark("init");
  Run r{BRR_MODEL_V2, outputFile, max_iterations, burn_in, thinning, N, M, 1, 0, log, opt.verbose != 0, &tl};
  int64_t n_ok = 0;
  if (!rc) rc = run_chain(s, r, &w, &n_ok);
  tl.mark("chain");
  w.close();
  if (rc) w.truncate_rows(n_ok);  // only rows of device-checked states stay
  fclose(f);
  tl.mark("drain");
  if (!rc && w.error()) rc = w.error();
  if (rc) return fail(s, log, rc);
  brr_session_destroy(s);
  tl.mark("destroy");
  return 0;
}

int brr_BayesRSamplerV2Groups(const char *outputFile, int seed, int max_iterations, int burn_in,
                              int thinning, const double *X, int64_t N, int64_t M,
                              const double *Y, double sigma0, double v0E, double s02E,
                              double v0G, double s02G, const double *cva, int32_t n_cva, int groups,
                              const int32_t *gAssign, const double *fixed, int64_t F,
                              const brr_options *opt_in) {
  brr_options opt = opts_or_default(opt_in);
  Log log{opt.log, opt.log_userdata};
  FILE *f = fopen(outputFile, "w");  // BayesRv2Groups.cpp:85 (empty until :113)
  if (!f) { log(std::string("brr: cannot open ") + outputFile + "\n"); return -3; }
  if (bad_iterations(max_iterations, burn_in, thinning)) {
    log(kIterMsg);
    fclose(f);
    return 1;
  }
  hyper_warnings(log, sigma0, v0E, s02E, v0G, s02G, cva, (int64_t)n_cva * groups);
  CsvWriter w(f);
  w.header(hdr_groups(M, N, groups, F));
  brr_session *s = brr_session_create(BRR_MODEL_GROUPS, N, M, M, 0, n_cva + 1, groups, F, &opt);
  int rc = s ? 0 : -1;
  if (!rc) rc = brr_session_upload_x_f64(s, X, N);
  if (!rc) rc = brr_session_set_y(s, Y);
  if (!rc) rc = brr_session_set_fixed(s, fixed);
  if (!rc) rc = brr_session_set_bayesr(s, sigma0, v0E, s02E, v0G, s02G, cva, gAssign);
  if (!rc) rc = brr_session_init(s, seed);
  Run r{BRR_MODEL_GROUPS, outputFile, max_iterations, burn_in, thinning, N, M, groups, F, log, opt.verbose != 0, nullptr};
  int64_t n_ok = 0;
  if (!rc) rc = run_chain(s, r, &w, &n_ok);
  w.close();
  if (rc) w.truncate_rows(n_ok);  // only rows of device-checked states stay
  fclose(f);
  if (!rc && w.error()) rc = w.error();
  if (rc) return fail(s, log, rc);
  brr_session_destroy(s);
  return 0;
}

int brr_BRV2Grstart(const char *outputFile, int seed, int max_iterations, int burn_in,
                    int thinning, double mu, const double *beta, double sigmaE,
                    const double *sigmaGG, const double *X, int64_t N, int64_t M,
                    const double *epsilon, const double *components, double sigma0, double v0E,
                    double s02E, double v0G, double s02G, const double *cva, int32_t n_cva,
                    int groups, const int32_t *gAssign, const brr_options *opt_in) {
  brr_options opt = opts_or_default(opt_in);
  Log log{opt.log, opt.log_userdata};
  FILE *f = fopen(outputFile, "w");  // BRv2Grstart.cpp:85; no header is ever written
  if (!f) { log(std::string("brr: cannot open ") + outputFile + "\n"); return -3; }
  if (bad_iterations(max_iterations, burn_in, thinning)) {
    log(kIterMsg);
    fclose(f);
    return 1;
  }
  hyper_warnings(log, sigma0, v0E, s02E, v0G, s02G, cva, (int64_t)n_cva * groups);
  CsvWriter w(f);
  brr_session *s = brr_session_create(BRR_MODEL_RESTART, N, M, M, 0, n_cva + 1, groups, 0, &opt);
  int rc = s ? 0 : -1;
  if (!rc) rc = brr_session_upload_x_f64(s, X, N);
  if (!rc) rc = brr_session_set_bayesr(s, sigma0, v0E, s02E, v0G, s02G, cva, gAssign);
  if (!rc) rc = brr_session_set_restart(s, mu, beta, sigmaE, sigmaGG, epsilon, components);
  if (!rc) rc = brr_session_init(s, seed);
  Run r{BRR_MODEL_RESTART, outputFile, max_iterations, burn_in, thinning, N, M, groups, 0, log, opt.verbose != 0, nullptr};
  int64_t n_ok = 0;
  if (!rc) rc = run_chain(s, r, &w, &n_ok);
  w.close();
  if (rc) w.truncate_rows(n_ok);  // only rows of device-checked states stay
  fclose(f);
  if (!rc && w.error()) rc = w.error();
  if (rc) return fail(s, log, rc);
  brr_session_destroy(s);
  return 0;
}

int brr_HorseshoeR(const char *outputFile, int seed, int max_iterations, int burn_in,
                   int thinning, const double *X, int64_t N, int64_t M, const double *Y,
                   double A, double v0E, double s02E, double vL, double vT, double c2,
                   double vC, double sC, const brr_options *opt_in) {
  brr_options opt = opts_or_default(opt_in);
  Log log{opt.log, opt.log_userdata};
  if (bad_iterations(max_iterations, burn_in, thinning)) {  // HorseshoeR.cpp:119-123 (stdout)
    log(kIterMsg);
    return 1;
  }
  FILE *f = fopen(outputFile, "w");
  if (!f) { log(std::string("brr: cannot open ") + outputFile + "\n"); return -3; }
  CsvWriter w(f);
  w.header(hdr_hs(M, N));
  brr_session *s = brr_session_create(BRR_MODEL_HORSESHOE, N, M, M, 0, 1, 1, 0, &opt);
  int rc = s ? 0 : -1;
  if (!rc) rc = brr_session_upload_x_f64(s, X, N);
  if (!rc) rc = brr_session_set_y(s, Y);
  if (!rc) rc = brr_session_set_horseshoe(s, A, v0E, s02E, vL, vT, c2, vC, sC);
  if (!rc) rc = brr_session_init(s, seed);
  if (!rc && opt.verbose) {
    double eta = 0, tau = 0;
    brr_session_get_scalar(s, BRR_ETA, &eta);
    brr_session_get_scalar(s, BRR_TAU, &tau);
    char b[128];
    snprintf(b, sizeof b, "initial eta %g\ninitial tau %g\n", eta, tau);
    log(b);
  }
  Run r{BRR_MODEL_HORSESHOE, outputFile, max_iterations, burn_in, thinning, N, M, 1, 0, log, opt.verbose != 0, nullptr};
  int64_t n_ok = 0;
  if (!rc) rc = run_chain(s, r, &w, &n_ok);
  w.close();
  if (rc) w.truncate_rows(n_ok);  // only rows of device-checked states stay
  fclose(f);
  if (!rc && w.error()) rc = w.error();
  if (rc) return fail(s, log, rc);
  brr_session_destroy(s);
  return 0;
}

// ---------------------------------------------------------------------------------------
// Sample output of a session: the one-shots' CSV pipeline for callers that drive
// sweeps themselves (bench.py's output-on run).  One writer per session, kept here.
namespace {
struct Output {
  FILE *f = nullptr;
  std::unique_ptr<CsvWriter> w;
};
std::mutex g_out_mu;
std::map<brr_session *, std::unique_ptr<Output>> g_out;
}  // namespace

int brr_session_output_open(brr_session *s, const char *path, int32_t model, int64_t N, int64_t M, int32_t groups,
                            int64_t F, int32_t header, int32_t ring_depth) {
  if (!s || !path) return -1;
  std::lock_guard<std::mutex> lk(g_out_mu);
  if (g_out.count(s)) return -1;
  auto o = std::make_unique<Output>();
  o->f = fopen(path, "w");
  if (!o->f) return -3;
  if (int rc = brr::sample_ring_open(s, ring_depth)) { fclose(o->f); return rc; }
  o->w = std::make_unique<CsvWriter>(o->f);
  if (header) {
    if (model == BRR_MODEL_V2) o->w->header(hdr_v2(M, N));
    else if (model == BRR_MODEL_GROUPS) o->w->header(hdr_groups(M, N, groups, F));
    else if (model == BRR_MODEL_HORSESHOE) o->w->header(hdr_hs(M, N));
  }
  o->w->bind(s, model, N, M, groups, F);
  g_out[s] = std::move(o);
  return 0;
}

int brr_session_output_sample(brr_session *s, int32_t iteration) {
  Output *o = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_out_mu);
    auto it = g_out.find(s);
    if (it == g_out.end()) return -1;
    o = it->second.get();
  }
  int slot = -1;
  if (int rc = brr::sample_ring_push(s, &slot)) return rc;
  o->w->sample(slot, iteration);
  return 0;
}

int brr_session_output_close(brr_session *s, int32_t *max_rows_in_flight) {
  std::unique_ptr<Output> o;
  {
    std::lock_guard<std::mutex> lk(g_out_mu);
    auto it = g_out.find(s);
    if (it == g_out.end()) return -1;
    o = std::move(it->second);
    g_out.erase(it);
  }
  o->w->close();
  const int err = o->w->error();
  fclose(o->f);
  if (max_rows_in_flight) *max_rows_in_flight = brr::sample_ring_max_in_use(s);
  brr::sample_ring_close(s);
  return err;
}

}  // extern "C"
