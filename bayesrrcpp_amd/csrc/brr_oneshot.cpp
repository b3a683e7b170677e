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

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/brr.h"

namespace {

struct Log {
  brr_log_fn fn = nullptr;
  void *user = nullptr;
  void operator()(const std::string &m) const {
    if (fn) fn(m.c_str(), user); else fputs(m.c_str(), stderr);
  }
};

class CsvWriter {
 public:
  explicit CsvWriter(FILE *f) : f_(f), th_([this] { run(); }) {}
  ~CsvWriter() { close(); }
  void header(const std::string &h) { std::lock_guard<std::mutex> lk(mu_); q_.push_back({true, h, {}}); cv_.notify_one(); }
  void row(std::vector<double> &&v) {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back({false, std::string(), std::move(v)});
    cv_.notify_one();
  }
  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (done_) return;
      done_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();  // drain everything queued (the reference may drop rows)
  }

 private:
  struct Item { bool is_header; std::string h; std::vector<double> v; };
  void run() {
    std::string buf;
    char num[40];
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return done_ || !q_.empty(); });
        if (q_.empty()) return;
        it = std::move(q_.front());
        q_.pop_front();
      }
      if (it.is_header) { fputs(it.h.c_str(), f_); continue; }
      buf.clear();
      for (size_t i = 0; i < it.v.size(); ++i) {
        if (i) buf += ", ";
        int n = snprintf(num, sizeof num, "%g", it.v[i]);
        buf.append(num, (size_t)n);
      }
      buf += '\n';
      fwrite(buf.data(), 1, buf.size(), f_);
    }
  }
  FILE *f_;
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

struct Run {
  int model;
  const char *out;
  int max_it, burn_in, thin;
  int64_t N, M;
  int G;
  int64_t F;
  Log log;
  bool verbose;
};

int fail(brr_session *s, const Log &log, int rc) {
  std::string m = std::string("brr: ") + brr_last_error() + "\n";
  log(m);
  if (s) brr_session_destroy(s);
  return rc < 0 ? rc : -1;
}

// the reference's sweep loop with sample emission (BayesRv2.cpp:171-278)
int run_chain(brr_session *s, const Run &r, CsvWriter *w) {
  const int64_t N = r.N, M = r.M;
  const int G = r.G;
  std::vector<double> beta((size_t)M), comp((size_t)M), eps((size_t)N), sgg((size_t)G), alpha((size_t)std::max<int64_t>(r.F, 1)),
      lam((size_t)M);
  const auto t1 = std::chrono::steady_clock::now();
  const int every = r.max_it / 10;  // (int)std::ceil(max_iterations/10): integer division
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
    if (int rc = brr_session_sweep(s, 1)) return rc;
    if (it >= r.burn_in && it % r.thin == 0) {
      double mu = 0, se = 0, sg = 0, tau = 0, sf = 0;
      if (brr_session_get_scalar(s, BRR_MU, &mu) || brr_session_get_scalar(s, BRR_SIGMAE, &se)) return -2;
      if (brr_session_get_vector(s, BRR_BETA, beta.data()) < 0 || brr_session_get_vector(s, BRR_EPS, eps.data()) < 0) return -2;
      std::vector<double> row;
      row.reserve((size_t)(2 * M + N + G + r.F + 8));
      row.push_back(it);
      row.push_back(mu);
      row.insert(row.end(), beta.begin(), beta.end());
      row.push_back(se);
      if (r.model == BRR_MODEL_HORSESHOE) {
        brr_session_get_scalar(s, BRR_TAU, &tau);
        if (brr_session_get_vector(s, BRR_LAMBDA, lam.data()) < 0) return -2;
        row.push_back(tau);
        row.insert(row.end(), lam.begin(), lam.end());
        row.insert(row.end(), eps.begin(), eps.end());
        row.push_back(0.0);  // sample has 2M+4+N slots, 2M+N+3 values (HorseshoeR.cpp:157,258)
      } else {
        if (brr_session_get_vector(s, BRR_COMP, comp.data()) < 0) return -2;
        if (r.model == BRR_MODEL_V2) {
          brr_session_get_scalar(s, BRR_SIGMAG, &sg);
          row.push_back(sg);
          row.insert(row.end(), comp.begin(), comp.end());
          row.insert(row.end(), eps.begin(), eps.end());
        } else {
          if (brr_session_get_vector(s, BRR_SIGMAGG, sgg.data()) < 0) return -2;
          row.insert(row.end(), comp.begin(), comp.end());
          row.insert(row.end(), sgg.begin(), sgg.end());
          row.insert(row.end(), eps.begin(), eps.end());
          if (r.model == BRR_MODEL_GROUPS) {
            if (r.F > 0 && brr_session_get_vector(s, BRR_ALPHA, alpha.data()) < 0) return -2;
            row.insert(row.end(), alpha.begin(), alpha.begin() + r.F);
            brr_session_get_scalar(s, BRR_SIGMAF, &sf);
            row.push_back(sf);
          }
        }
      }
      w->row(std::move(row));
    }
  }
  brr_session_synchronize(s);
  const auto t2 = std::chrono::steady_clock::now();
  r.log("duration: " + std::to_string((long long)std::chrono::duration_cast<std::chrono::seconds>(t2 - t1).count()) + "s\n");
  return 0;
}

brr_options opts_or_default(const brr_options *o) {
  brr_options r;
  if (o) r = *o; else brr_options_default(&r);
  return r;
}

}  // namespace

extern "C" {

int brr_BayesRSamplerV2(const char *outputFile, int seed, int max_iterations, int burn_in,
                        int thinning, const double *X, int64_t N, int64_t M, const double *Y,
                        double sigma0, double v0E, double s02E, double v0G, double s02G,
                        const double *cva, int32_t n_cva, const brr_options *opt_in) {
  brr_options opt = opts_or_default(opt_in);
  Log log{opt.log, opt.log_userdata};
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
  brr_session *s = brr_session_create(BRR_MODEL_V2, N, M, M, 0, n_cva + 1, 1, 0, &opt);
  int rc = s ? 0 : -1;
  if (!rc) rc = brr_session_upload_x_f64(s, X, N);
  if (!rc) rc = brr_session_set_y(s, Y);
  if (!rc) rc = brr_session_set_bayesr(s, sigma0, v0E, s02E, v0G, s02G, cva, nullptr);
  if (!rc) rc = brr_session_init(s, seed);
  Run r{BRR_MODEL_V2, outputFile, max_iterations, burn_in, thinning, N, M, 1, 0, log, opt.verbose != 0};
  if (!rc) rc = run_chain(s, r, &w);
  w.close();
  fclose(f);
  if (rc) return fail(s, log, rc);
  brr_session_destroy(s);
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
  Run r{BRR_MODEL_GROUPS, outputFile, max_iterations, burn_in, thinning, N, M, groups, F, log, opt.verbose != 0};
  if (!rc) rc = run_chain(s, r, &w);
  w.close();
  fclose(f);
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
  Run r{BRR_MODEL_RESTART, outputFile, max_iterations, burn_in, thinning, N, M, groups, 0, log, opt.verbose != 0};
  if (!rc) rc = run_chain(s, r, &w);
  w.close();
  fclose(f);
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
  Run r{BRR_MODEL_HORSESHOE, outputFile, max_iterations, burn_in, thinning, N, M, 1, 0, log, opt.verbose != 0};
  if (!rc) rc = run_chain(s, r, &w);
  w.close();
  fclose(f);
  if (rc) return fail(s, log, rc);
  brr_session_destroy(s);
  return 0;
}

}  // extern "C"
