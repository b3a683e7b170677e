// brr_ovsolve.hpp -- the overlapped persistent solver of the BayesR family at B = 128 (round 6).
// A fragment of brr_kernels.hip: included there inside namespace brr, after solver_role, and uses
// its helpers (Dev access, decide_pos, chain_redecide, refresh_arm, quot_rn, the sc1 hand-over).
//
// Reference: the per-marker mixture update, src/BayesRv2.cpp:186-245 (Groups
// src/BayesRv2Groups.cpp:232-298, restart src/BRv2Grstart.cpp:183-250).  The chain runs the same
// exact single-site Gibbs steps as solve_block's; what changes is WHEN the chain-independent work
// of a block runs.
//
// solve_block, per block s: constants, wait for the reduced dots (the reducers wait for block s-1's
// change list to subtract its cross-Gram correction), decisions, Gram block, the chain on wave 0, the
// write-back -- one after the other, so C3's block period is its ~12 us chain plus ~8 us of hand-over
// and preparation (profiles/r05k_prof_c3.log).  Here the eight waves of the solver workgroup take
// roles, and block s+1 is prepared while wave 0 runs block s's chain:
//   wave 0     block s's chain (chain_bayesr_ov); a change the corrector holds no row for (see wave 1)
//              goes into an LDS queue as it is made;
//   wave 1     the corrector: the cross-Gram corrections of block s+1's dots for the changes the
//              streamed dots have not seen -- block s's, corr_j = sum_{i changed in s} C_ij delta_i
//              (C = X_s^T X_{s+1}; the rows of the positions predicted to change are loaded into its
//              registers while the chain runs), and at lag 2 block s-1's -- so the reducers correct
//              nothing and the dots wait for no list publication;
//   wave 2     block s-1's write-back (its change list in Gram-index order, the publish, beta / comp /
//              sel), then positions 0-63 of block s+1's decisions;
//   wave 3     positions 64-127 of block s+1's decisions: every lane polls its reduced dot, reads its
//              constants from HBM and decides at num' = dot + x2 bo (block s's changes not yet in);
//              once the corrector is done, num = num' - corr, and the positions whose num left its
//              decision window are decided again at num, side by side (waves 2 and 3);
//   waves 5-7  block s+1's Gram block into the second LDS buffer as its upper triangle (row a holds
//              G(a, b) for the Gram indices b >= a rounded down to even: 65 KB instead of 128, every row
//              16-B aligned, so one 16-B LDS-DMA per row), so that two buffers fit beside the rest;
//   wave 4     idle (it shares wave 0's SIMD: any work there would take the chain's issue slots).
// At the block boundary wave 0 starts block s+1's chain from decisions at the exact num, as solve_block's
// chain does, so the steps and decisions are those of the exact sampler.
//
// Synchronisation inside the workgroup: one barrier per block (after every role's work for it), and
// LDS words with epochs (block indices, never reset) for the hand-overs inside a block:
// the queue count and "chain done" (wave 0 -> 1), "corrections done" (wave 1 -> 2, 3) and "set free"
// (wave 2 -> 3).  LDS
// operations of one wave complete in issue order, so data written before a word is visible to the wave
// that has read the word.  Every wait is bounded (the session's protocol error flag).

#ifndef BRR_OV_RC
#define BRR_OV_RC 32
#endif
#ifndef BRR_OV_SLEEP
#define BRR_OV_SLEEP 1  // s_sleep units between the LDS polls of the waves that wait beside the chain
#endif
constexpr int OVB = 128;                     // block size of the overlapped solver
constexpr int OV_TRI = OVB * (OVB + 2) / 2;  // stored entries of a Gram block: rows a, columns >= a & ~1
constexpr int OV_GS = OV_TRI;                // doubles per Gram buffer
constexpr int OV_KMAX = 4;                   // mixture components the constants area holds
constexpr int OV_SET_D = 7, OV_SET_I = 3;    // doubles / ints per position in a decision set
constexpr size_t OV_OFF_SET = (size_t)2 * OV_GS * 8;
constexpr size_t OV_SET_BYTES = (size_t)(OV_SET_D * 8 + OV_SET_I * 4) * OVB;
constexpr size_t OV_OFF_CONST = OV_OFF_SET + 2 * OV_SET_BYTES;
constexpr size_t OV_OFF_COR = OV_OFF_CONST + (size_t)(2 * OV_KMAX + 2) * 8 * OVB;  // K + (K-1) + 3 fields
constexpr size_t OV_OFF_QDL = OV_OFF_COR + 8 * OVB;
constexpr size_t OV_OFF_QGI = OV_OFF_QDL + 8 * OVB;
constexpr size_t OV_OFF_MISC = OV_OFF_QGI + 4 * OVB;
constexpr size_t OV_LDS = OV_OFF_MISC + 32 * 4;
static_assert(OV_LDS <= SOLVE_LDS_MAX - 64, "overlapped solver LDS");
enum OvFlag : int { OVF_QN = 0, OVF_QDONE = 1, OVF_FREE = 2, OVF_CDONE = 3, OVF_CREADY = 4 };

// A block's decision set (two, by block parity): written by the deciders (r0 = num', lo, hi, dsel,
// sdz, bo, fl, gi, m), read by the chain, which writes bn and (over fl) the selected components for the
// write-back.
struct OvSet {
  double *r0, *lo, *hi, *dsel, *sdz, *bo, *bn;
  int *fl, *gi, *m;
};
__device__ __forceinline__ OvSet ov_set(char *smem, int b) {
  double *p = reinterpret_cast<double *>(smem + OV_OFF_SET + (size_t)(b & 1) * OV_SET_BYTES);
  int *q = reinterpret_cast<int *>(p + OV_SET_D * OVB);
  return OvSet{p, p + OVB, p + 2 * OVB, p + 3 * OVB, p + 4 * OVB, p + 5 * OVB, p + 6 * OVB,
               q, q + OVB, q + 2 * OVB};
}
// the Gram triangle of block b: G(a, b) for Gram indices a <= b at ov_tri(b)[ov_row(a) + b].  Row a holds
// the columns (a & ~1) .. B-1 (an even start keeps every row 16-B aligned); it begins at the entries of the
// rows before it, sum_{a' < a} (B - (a' & ~1)) = 2m (B + 1 - m) for a = 2m (+ B - 2m for a = 2m + 1)
__device__ __forceinline__ double *ov_tri(char *smem, int b) {
  return reinterpret_cast<double *>(smem) + (size_t)(b & 1) * OV_GS;
}
__device__ __forceinline__ int ov_tstart(int a) {
  const int m = a >> 1;
  return 2 * m * (OVB + 1 - m) + ((a & 1) ? OVB - 2 * m : 0);
}
__device__ __forceinline__ int ov_row(int a) { return ov_tstart(a) - (a & ~1); }

typedef __attribute__((address_space(3))) int ov_lint;
typedef __attribute__((address_space(3))) double ov_ldbl;
__device__ __forceinline__ int ov_ld(const int *p) { return *(volatile const ov_lint *)p; }
__device__ __forceinline__ void ov_st(int *p, int v) { *(volatile ov_lint *)p = v; }

// bounded wait (a whole wave) until the epoch word reaches target
__device__ __forceinline__ void ov_wait(const Dev &d, const int *p, int target, int site) {
  for (uint32_t n = 0;; ++n) {
    if ((int)((unsigned)ov_ld(p) - (unsigned)target) >= 0) return;
    if ((n & 255) == 255 && ld_sc1_int(d.sync + SY_ERR)) return;  // another wait already failed
    if (n > SPIN_MAX) {
      if ((threadIdx.x & 63) == 0 && atomicCAS(d.sync + SY_ERR, 0, 1) == 0) {
        st_sc1_int(d.sync + SY_ERR + 1, site);
        st_sc1_int(d.sync + SY_ERR + 2, target);
        st_sc1_int(d.sync + SY_ERR + 3, ov_ld(p));
        st_sc1_int(d.sync + SY_ERR + 4, (int)blockIdx.x);
      }
      return;
    }
    __builtin_amdgcn_s_sleep(BRR_OV_SLEEP);
  }
}

// Decisions of block b, one position per lane (waves 2 and 3), in two passes.  The first, early in block
// b-1: the position's Gram index, member and old beta into the set, the reduced dot polled (the slot holds
// block b's sentinel until its reducer writes it) and re-armed with the sentinel of its next use, then the
// decision at num' = dot + x2 bo (block b-1's changes not yet in; constants from HBM, k_prep's per-sweep
// values -- solve_block reads the same ones from LDS -- kept in registers).  The second, once the
// corrector has block b-1's changes: num = num' - corr; a position whose t = num^2 left its window is
// decided again at num (the windows), all of them side by side, so the chain starts
// from decisions at the exact num as solve_block's does.
struct OvPos {
  bool in;
  int gi, m;
  double bo, x2, p, z, r;
  double av[MAXK], dv[MAXK];  // a_k, D_k (k >= 1 at dv[k - 1])
};

__device__ __forceinline__ void ov_decision(const Dev &d, const OvPos &P, double r, double sigmaE, OvSet st, int pos) {
#pragma clang fp contract(off)
  const FastDec o = decide_pos(d, r, P.av, P.dv, 1, sigmaE, P.p, P.x2, P.m);
  double dsel = 1.0;
#pragma unroll
  for (int k = 1; k < MAXK; ++k)
    if (!o.ex && o.k == k) dsel = P.dv[k - 1];
  const bool likely = o.ex || !(o.k == FALLTHROUGH || (o.k == 0 && P.bo == 0.0));
  st.fl[pos] = (o.k & 0xFF) | (o.ex ? PF_EX : 0) | (likely ? PF_LIKELY : 0);
  st.r0[pos] = r;
  st.lo[pos] = o.lo;
  st.hi[pos] = o.hi;
  st.dsel[pos] = dsel;
  st.sdz[pos] = sqrt(sigmaE / dsel) * P.z;  // rnorm(muk, sqrt(sigmaE/denom)) noise
}

__device__ __forceinline__ OvPos ov_decide(const Dev &d, int b, int pos, OvSet st, double sigmaE,
                                           unsigned long long *twait) {
#pragma clang fp contract(off)
  OvPos P;
  const int bs = d.bsz[b];
  P.in = pos < bs;
  const int64_t S = d.nbB;
  const int64_t q = (int64_t)b * OVB + pos;
  const double *mc = d.mc;
  P.gi = P.in ? d.gidx[q] : 0;
  P.m = P.in ? d.member[q] : 0;
  P.bo = P.in ? mc[MC_BO * S + q] : 0.0;
  P.x2 = P.in ? mc[MC_XSQ * S + q] : 1.0;
  P.p = P.in ? mc[MC_P * S + q] : 0.5;
  P.z = P.in ? mc[MC_Z * S + q] : 0.0;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    P.av[k] = P.in && k < d.K ? mc[(MC_A + k) * S + q] : 0.0;
    P.dv[k] = P.in && k + 1 < d.K ? mc[(MC_A + d.K + k) * S + q] : 1.0;
  }
  st.gi[pos] = P.gi;
  st.m[pos] = P.m;
  st.bo[pos] = P.bo;
  // the dots are by visit position, or by in-block storage index (2-bit codes / the f32 code cache)
  const int sidx = P.in && d.slab_storage ? P.gi : pos;
  const int par = b % NPAR;
  double *slab2 = d.slab2 + par * d.slab2_stride;
  const unsigned long long sent = slab_sentinel(d.sbase + b);
  const uint64_t tw0 = twait ? wall_clock64() : 0;
  double dsum = 0.0;
  for (int g0 = 0; g0 < d.NG; g0 += 16) {
    unsigned long long v[16];
    for (uint32_t n = 0;; ++n) {
      bool ready = true;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        v[u] = g0 + u < d.NG ? ld_sc1_u64(slab2 + (int64_t)(g0 + u) * OVB + sidx) : 0ull;
        ready = ready && v[u] != sent;
      }
      if (ready) break;
      if (((n & 255) == 255 && ld_sc1_int(d.sync + SY_ERR)) || n > SPIN_MAX) {
        if (atomicCAS(d.sync + SY_ERR, 0, 1) == 0) {
          st_sc1_int(d.sync + SY_ERR + 1, 3);
          st_sc1_int(d.sync + SY_ERR + 2, d.sbase + b);
          st_sc1_int(d.sync + SY_ERR + 3, g0);
          st_sc1_int(d.sync + SY_ERR + 4, (int)blockIdx.x);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) dsum += __longlong_as_double((long long)v[u]);
  }
  if (twait && (threadIdx.x & 63) == 0) *twait += wall_clock64() - tw0;
  // this lane alone read its slot column: it gets the sentinel of the block that uses the slots next
  // (b + NPAR in this sweep, else block b % NPAR of the next; that block's reducer writes only after
  // this solver has published later blocks' lists, so these stores land first)
  const int nxt = b + NPAR < d.nb ? d.sbase + b + NPAR : d.sbase + d.nb + b % NPAR;
  const unsigned long long ns = slab_sentinel(nxt);
  for (int g = 0; g < d.NG; ++g) st_sc1_u64(slab2 + (int64_t)g * OVB + sidx, ns);
  // num' = x . (eps + x b_old) without block b-1's changes (BayesRv2.cpp:191-193)
  P.r = dsum + P.x2 * P.bo;
  if (P.in) ov_decision(d, P, P.r, sigmaE, st, pos);
  return P;
}

// the second pass (after the corrector's flag): num = num' - corr, re-decided where the window was left
// (when OV_FOLD_MIN or more of the wave's positions left theirs; else the chain re-decides them)
constexpr int OV_FOLD_MIN = 3;
__device__ __forceinline__ void ov_fold(const Dev &d, const OvPos &P, int pos, OvSet st, const double *Lcor,
                                        double sigmaE) {
#pragma clang fp contract(off)
  if (!P.in) return;
  const double r = P.r - Lcor[P.gi];
  const double t = r * r;
  const int fl = st.fl[pos];
  const bool left = !(fl & PF_EX) && !(t >= st.lo[pos] && t <= st.hi[pos]);
  // (one or two positions of the wave: the chain's re-decision, ~0.7 us each, costs less than this
  // pass's ~1.5 us; C1 leaves ~13 per block, C3 ~2)
  if (left && __popcll(__ballot(left)) >= OV_FOLD_MIN) ov_decision(d, P, r, sigmaE, st, pos);
  else st.r0[pos] = r;
}

// Block b's Gram block as the triangle (waves 5-7, wave w of nw): row a (B - (a & ~1) doubles, contiguous
// in HBM and in LDS) is one 16-B LDS-DMA wave instruction.  Retired by each wave's vmcnt(0) before the
// barrier; no other wave's data is needed, so it starts with the block.
__device__ __forceinline__ void ov_load_gram(const Dev &d, int b, double *tri, int w, int nw) {
  const double *src = d.gram + (int64_t)d.gblk[b] * OVB * OVB;
  const int lane = threadIdx.x & 63;
  for (int a = w; a < OVB; a += nw) {
    const int a0 = a & ~1;
    if (2 * lane < OVB - a0)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + (int64_t)a * OVB + a0 + 2 * lane),
                                       (__attribute__((address_space(3))) void *)(tri + ov_tstart(a)), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A block's change list kept in the corrector's registers for the next block (lag 2): lane l holds
// entries l and l + 64 (Gram index, delta), in position order.
struct OvStash {
  int g0 = 0, g1 = 0, n = 0;
  double d0 = 0.0, d1 = 0.0;
};

constexpr int OV_RC = BRR_OV_RC;  // cross-Gram rows the corrector holds in registers (likely positions; 40 spilled)

// The corrector (wave 1): block s+1's dots minus the changes the streamed dots have not seen, so that the
// reducers correct nothing (Dev::rcorr = 0) and the dots wait for no list publication:
//   at lag 2 block s-1's changes (C2 = X_{s-1}^T X_{s+1}), from the registers the last block left them in,
//   summed at the start of the block;
//   block s's changes (C = X_s^T X_{s+1}): the cross-Gram rows of the first OV_RC positions the decisions
//   predict to change are loaded into registers while the chain runs, and when it ends each is scaled by
//   its position's delta (zero if it did not change), in position order; a change no register holds (a
//   position re-decided into a change, or predicted past the first OV_RC) is pushed by the chain into an
//   LDS queue and summed here as it comes, in chain order.
// corr = (held + queued) + older.  Lane l owns block s+1's Gram indices 2l, 2l+1 (one 16-B load of each
// cross-Gram row).  After the chain the queue area is its scratch.
__device__ __forceinline__ void ov_correct(const Dev &d, int s, int s0, int lag, OvStash &ost, OvSet st,
                                           const int *qn, const int *qdone, double *qdl, int *qgi, double *Lcor,
                                           unsigned long long *ttail) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int bs = d.bsz[s];
  const int gp = d.gblk[s], gb = d.gblk[s + 1];
  const double *C = gb == (gp + 1) % d.nb ? d.xgram + (int64_t)gp * OVB * OVB : d.xgramT + (int64_t)gb * OVB * OVB;
  auto rowld = [&](const double *Cx, int g) __attribute__((always_inline)) -> double2 {
    return *reinterpret_cast<const double2 *>(Cx + (int64_t)g * OVB + 2 * lane);
  };
  // the likely positions of block s (the decisions' prediction), in position order: the chain holds the
  // same rule (chain_bayesr_ov)
  const int f0 = lane < bs ? st.fl[lane] : 0, f1 = lane + 64 < bs ? st.fl[lane + 64] : 0;
  const uint64_t lk0 = __ballot(f0 & PF_LIKELY), lk1 = __ballot(f1 & PF_LIKELY);
  double2 row[OV_RC];
  {
    uint64_t m0 = lk0, m1 = lk1;
#pragma unroll
    for (int r = 0; r < OV_RC; ++r) {
      const int p = m0 ? __builtin_ctzll(m0) : (m1 ? 64 + __builtin_ctzll(m1) : -1);
      if (m0) m0 &= m0 - 1; else if (m1) m1 &= m1 - 1;
      row[r] = p >= 0 ? rowld(C, st.gi[max(p, 0)]) : make_double2(0.0, 0.0);
    }
  }
  // the older list (lag 2): block s-1's changes against block s+1
  double b0 = 0.0, b1 = 0.0;
  if (lag >= 2 && s - 1 >= s0) {
    const int gp2 = d.gblk[s - 1];
    const double *C2 = gb == (gp2 + 2) % d.nb ? d.xgram2 + (int64_t)gp2 * OVB * OVB : d.xgram2T + (int64_t)gb * OVB * OVB;
    for (int e0 = 0; e0 < ost.n; e0 += 8) {
      double2 cv[8];
      double dl[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + min(u, ost.n - e0 - 1);
        dl[u] = readlane_f64(e < 64 ? ost.d0 : ost.d1, e & 63);
        cv[u] = rowld(C2, __builtin_amdgcn_readlane(e < 64 ? ost.g0 : ost.g1, e & 63));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u < ost.n) {
          b0 += cv[u].x * dl[u];
          b1 += cv[u].y * dl[u];
        }
    }
  }
  // the queued changes, as the chain pushes them, until it ends
  double c0 = 0.0, c1 = 0.0;
  int nd = 0;
  uint64_t tdone = 0;
  for (uint32_t n = 0;; ++n) {
    const bool done = ov_ld(qdone) == s + 1;  // (read before the count: the count is then final)
    if (done && ttail && !tdone) tdone = wall_clock64();
    const int v = ov_ld(qn);
    const int nq = (v >> 9) == s ? (v & 511) : 0;
    while (nd < nq) {
      const int nb8 = min(8, nq - nd);
      double2 cv[8];
      double dl[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = nd + min(u, nb8 - 1);
        dl[u] = qdl[e];
        cv[u] = rowld(C, qgi[e]);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nb8) {
          c0 += cv[u].x * dl[u];
          c1 += cv[u].y * dl[u];
        }
      nd += nb8;
    }
    if (done) break;
    if ((n & 255) == 255 && ld_sc1_int(d.sync + SY_ERR)) break;
    if (n > SPIN_MAX) {
      if (lane == 0 && atomicCAS(d.sync + SY_ERR, 0, 1) == 0) {
        st_sc1_int(d.sync + SY_ERR + 1, 10);
        st_sc1_int(d.sync + SY_ERR + 2, s);
        st_sc1_int(d.sync + SY_ERR + 4, (int)blockIdx.x);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(BRR_OV_SLEEP);
  }
  // the held rows, scaled by their positions' deltas (this lane's two positions, read by readlane)
  const double dl0 = lane < bs ? st.bn[lane] - st.bo[lane] : 0.0;
  const double dl1 = lane + 64 < bs ? st.bn[lane + 64] - st.bo[lane + 64] : 0.0;
  double a0 = 0.0, a1 = 0.0;
  {
    uint64_t m0 = lk0, m1 = lk1;
#pragma unroll
    for (int r = 0; r < OV_RC; ++r) {
      const int p = m0 ? __builtin_ctzll(m0) : (m1 ? 64 + __builtin_ctzll(m1) : -1);
      if (m0) m0 &= m0 - 1; else if (m1) m1 &= m1 - 1;
      if (p >= 0) {
        const double dl = readlane_f64(p < 64 ? dl0 : dl1, p & 63);  // (0 where the position did not change)
        a0 += row[r].x * dl;
        a1 += row[r].y * dl;
      }
    }
  }
  Lcor[2 * lane] = (a0 + c0) + b0;
  Lcor[2 * lane + 1] = (a1 + c1) + b1;
  if (ttail && lane == 0 && tdone) *ttail += wall_clock64() - tdone;
}

// block s's changes, in position order, kept for block s+2's correction (lag 2; after the corrections are
// handed over, off the block boundary's path; the queue area as scratch)
__device__ __forceinline__ void ov_stash(const Dev &d, int s, OvSet st, double *qdl, int *qgi, OvStash &ost) {
  const int lane = threadIdx.x & 63;
  const int bs = d.bsz[s];
  const double dl0 = lane < bs ? st.bn[lane] - st.bo[lane] : 0.0;
  const double dl1 = lane + 64 < bs ? st.bn[lane + 64] - st.bo[lane + 64] : 0.0;
  const uint64_t ch0 = __ballot(dl0 != 0.0), ch1 = __ballot(dl1 != 0.0);
  const uint64_t below = (1ull << lane) - 1ull;
  {
    const int e0 = __popcll(ch0 & below), e1 = __popcll(ch0) + __popcll(ch1 & below);
    if (dl0 != 0.0) { qgi[e0] = st.gi[lane]; qdl[e0] = dl0; }
    if (dl1 != 0.0) { qgi[e1] = st.gi[lane + 64]; qdl[e1] = dl1; }
  }
  const int nch = __popcll(ch0) + __popcll(ch1);
  ost.n = nch;
  ost.g0 = lane < nch ? qgi[lane] : 0;
  ost.d0 = lane < nch ? qdl[lane] : 0.0;
  ost.g1 = lane + 64 < nch ? qgi[lane + 64] : 0;
  ost.d1 = lane + 64 < nch ? qdl[lane + 64] : 0.0;
}

// Block w's write-back (wave 2): its change list in Gram-index (storage) order -- the order of
// solve_block's write-back, so the lists are the same -- then the publish and the marker state.  The
// position of each Gram index goes where the set's windows were (no longer read).
__device__ __forceinline__ void ov_writeback(const Dev &d, int w, OvSet st) {
  const int lane = threadIdx.x & 63;
  const int bs = d.bsz[w];
  int *Lpg = reinterpret_cast<int *>(st.lo);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int pos = lane + 64 * c;
    if (pos < bs) Lpg[st.gi[pos]] = pos;  // (one wave: its LDS writes complete before its reads below)
  }
  const int pslot = w % NSLOT;
  int *pidx = d.pend_idx + pslot * d.pend_stride, *pgi = d.pend_gi + pslot * d.pend_stride;
  int *ppos = d.pend_pos + pslot * d.pend_stride;
  double *pbo = d.pend_bo + pslot * d.pend_stride, *pbn = d.pend_bn + pslot * d.pend_stride;
  int base = 0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int gi = lane + 64 * c;
    const int pos = gi < bs ? Lpg[gi] : 0;
    int changed = 0, m = 0;
    double bnv = 0.0, bov = 0.0;
    if (gi < bs) {
      m = st.m[pos];
      bnv = st.bn[pos];
      bov = st.bo[pos];
      changed = bnv != bov;
    }
    const uint64_t bal = __ballot(changed);
    if (changed) {
      const int idx = base + __popcll(bal & ((1ull << lane) - 1ull));
      st_sc1_int(pidx + idx, m);
      st_sc1_int(pgi + idx, gi);
      st_sc1_int(ppos + idx, pos);
      st_sc1(pbo + idx, bov);
      st_sc1(pbn + idx, bnv);
    }
    base += __popcll(bal);
  }
  const int npend = base;
  const int npad = (npend + 15) & ~15;  // lists are read in batches of 8 / 16
  if (npend + lane < npad) {            // neutral padding: eps + x*0 - x*0 == eps exactly, delta = 0
    st_sc1_int(pidx + npend + lane, 0);
    st_sc1_int(pgi + npend + lane, 0);
    st_sc1_int(ppos + npend + lane, 0);
    st_sc1(pbo + npend + lane, 0.0);
    st_sc1(pbn + npend + lane, 0.0);
  }
  if (lane == 0) {
    st_sc1_int(d.pend_n + pslot, npad);
    st_sc1_int(d.pend_n + NSLOT + pslot, npend);
  }
  // publish (the only storing wave drains its sc1 stores, then the count: MI355X_MICROARCH.md
  // "Valid forms")
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    __hip_atomic_store(d.sync + SY_PEND, d.sbase + w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == 0) stamp(d.sync, 5);
    if (npend) atomicAdd(&d.sc->n_changed, (unsigned long long)npend);
  }
  // the block's state for later sweeps (BayesRv2.cpp:226-245), off the streamers' path
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int pos = lane + 64 * c;
    if (pos < bs) {
      const int m = st.m[pos];
      d.beta[m] = st.bn[pos];
      const int ks = st.fl[pos];  // (the chain's selected component)
      if (ks != FALLTHROUGH) d.comp[m] = ks;
      d.sel[m] = ks != FALLTHROUGH;
    }
  }
}

// Block s's chain (wave 0): chain_bayesr_resident_blk's steps (sub-blocks of 64 positions, lane l
// holding positions l + 64 q) on the decision set, with the Gram triangle; the changes the corrector holds
// no row for into its queue.  The per-component constants (re-decisions, the exact formula) arrive by
// wave 4's LDS-DMA, waited for at their first use.
template <int B>
__device__ __forceinline__ void chain_bayesr_ov(const Dev &d, int s, double sigmaE, OvSet st, const double *La,
                                                const double *Lden, const double *Lp, const double *Lx2,
                                                const double *Lz, const double *tri, double *qdl, int *qgi, int *qn,
                                                int *qdone, const int *cready, bool prof) {
#pragma clang fp contract(off)
  constexpr int NS = B / 64;
  const int lane = threadIdx.x & 63;
  const int bs = d.bsz[s];
  double r[NS], lo[NS], hi[NS], dv[NS], iv[NS], sz[NS], bo[NS], bn[NS];
  int gg[NS], ks[NS], tl[NS];  // tl: this lane's positions' triangle rows (G(g, gif) for gif > g)
  uint32_t act = 0, win = 0, valid = 0, exb = 0;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane + 64 * q;
    const bool in = pos < bs;
    const int fl = in ? st.fl[pos] : 0;
    gg[q] = in ? st.gi[pos] : 0;
    tl[q] = ov_row(gg[q]);
    r[q] = in ? st.r0[pos] : 0.0;  // (num: block s-1's changes folded in by the deciders' second pass)
    lo[q] = in ? st.lo[pos] : 1.0;
    hi[q] = in ? st.hi[pos] : -1.0;
    dv[q] = in ? st.dsel[pos] : 1.0;
    iv[q] = 1.0 / dv[q];
    sz[q] = in ? st.sdz[pos] : 0.0;
    bo[q] = in ? st.bo[pos] : 0.0;
    bn[q] = bo[q];
    ks[q] = fl & 0xFF;
    const double tt = r[q] * r[q];
    valid |= (uint32_t)in << q;
    act |= (uint32_t)(in && (fl & PF_LIKELY)) << q;
    exb |= (uint32_t)(in && (fl & PF_EX)) << q;
    win |= (uint32_t)(in && tt >= lo[q] && tt <= hi[q]) << q;
  }
  // the positions whose cross-Gram row the corrector holds: the first OV_RC predicted ones in position order
  uint32_t held = 0;
  {
    const uint64_t l0 = __ballot(act & 1u), l1 = __ballot((act >> 1) & 1u);
    const uint64_t below = (1ull << lane) - 1ull;
    held |= (uint32_t)((act & 1u) && __popcll(l0 & below) < OV_RC);
    held |= (uint32_t)(((act >> 1) & 1u) && __popcll(l0) + __popcll(l1 & below) < OV_RC) << 1;
  }
  int nslow = 0, nsteps = 0, nref = 0, nq = 0;
  bool cw = false;  // the constants' LDS-DMA waited for
  uint64_t tslow = 0;
  const uint64_t tl0 = prof ? wall_clock64() : 0;
  static_for<NS>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    constexpr uint32_t bk = 1u << k;
    if (64 * k >= bs) return;
    int i = 64 * k;
    int np = 0, ppos = 0;  // this sub-block's changes: lane c holds change c's Gram index
    double pdl = 0.0;      // and its delta
    while (true) {
      const bool mine = (lane + 64 * k >= i) && ((valid & (act | ~win | exb) & bk) != 0);
      const double qv = quot_rn(r[k], dv[k], iv[k]) + sz[k];
      const double bnl = ks[k] == 0 ? 0.0 : (ks[k] == FALLTHROUGH ? bo[k] : qv);
      const int fastl = (int)(((win & ~exb) >> k) & 1u);
      const uint64_t bal = __ballot(mine);
      if (!bal) break;
      const int L = __builtin_ctzll(bal);
      const int first = 64 * k + L;  // wave-uniform
      const int gif = __builtin_amdgcn_readlane(gg[k], L);
      double delta;
      if (__builtin_expect(__builtin_amdgcn_readlane(fastl, L) != 0, 1)) {
        delta = readlane_f64(bnl - bo[k], L);
        bn[k] = lane == L ? bnl : bn[k];
      } else {
        const uint64_t ts0 = prof ? wall_clock64() : 0;
        if (!cw) {  // (wave 4's LDS-DMA of this block's constants, issued when the last chain ended)
          ov_wait(d, cready, s, 16);
          cw = true;
        }
        const double rf = readlane_f64(r[k], L);
        const bool exf = (__builtin_amdgcn_readlane((int)exb, L) >> k) & 1;
        if (!exf) {
          // outside its window: re-decide at the current num (as chain_bayesr_resident_blk)
          const double arm = refresh_arm(rf, Lden + first, B, d.K, sigmaE, Lz[first]);
          const double pf = Lp[first], x2f = Lx2[first];
          const int mf = st.m[first];
          FastDec o = chain_redecide(d, rf, La + first, Lden + first, B, sigmaE, pf, x2f, mf);
          const double bof = readlane_f64(bo[k], L);
          const bool lk = o.ex || !(o.k == FALLTHROUGH || (o.k == 0 && bof == 0.0));
          if (lane == L) {
            lo[k] = o.lo; hi[k] = o.hi; ks[k] = o.k;
            act = (act & ~bk) | ((uint32_t)lk << k);
            win = (win & ~bk) | ((uint32_t)(!o.ex) << k);
            exb = (exb & ~bk) | ((uint32_t)o.ex << k);
          }
          ++nref;
          if (o.ex || !lk) {
            if (prof) tslow += wall_clock64() - ts0;
            continue;
          }
          const double bnr = o.k == 0 ? 0.0 : readlane_f64(arm, o.k);
          bn[k] = lane == L ? bnr : bn[k];
          delta = bnr - bof;
          if (prof) tslow += wall_clock64() - ts0;
        } else {
          const double bof = readlane_f64(bo[k], L);
          const int m = st.m[first];
          const int g = d.gAssign ? d.gAssign[m] : 0;
          Decision dc = decide_bayesr_ool(rf, Lx2[first], sigmaE, d.sigmaGG[g], d.pi + (int64_t)g * d.K, d.cva + g, d.G,
                                          d.K, Lp[first], false);
          const double bnf = dc.k == 0 ? 0.0 : (dc.k == FALLTHROUGH ? bof : rf / dc.denom + sqrt(sigmaE / dc.denom) * Lz[first]);
          if (lane == L) { bn[k] = bnf; ks[k] = dc.k; }
          delta = bnf - bof;
          ++nslow;
          if (prof) tslow += wall_clock64() - ts0;
        }
      }
      // the sub-block's later positions subtract G delta now (G(gif, g) from the triangle: row gif when g >
      // gif, else row g); the later sub-blocks' positions at the flush
      {
        const int tg = __builtin_amdgcn_readlane(tl[k], L);  // (= ov_row(gif))
        const double g = tri[gg[k] > gif ? tg + gg[k] : tl[k] + gif];
        const bool later = lane > L && (valid & bk);
        r[k] = later ? r[k] - g * delta : r[k];
        const double tt = r[k] * r[k];
        win = (win & ~bk) | ((uint32_t)(tt >= lo[k] && tt <= hi[k]) << k);
      }
      if (delta != 0.0 && !((__builtin_amdgcn_readlane((int)held, L) >> k) & 1)) {
        // a change whose row the corrector does not hold: into its queue
        if (lane == 0) {
          ((ov_ldbl *)qdl)[nq] = delta;
          ((ov_lint *)qgi)[nq] = gif;
        }
        ++nq;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) ov_st(qn, (s << 9) | nq);
      }
      if (k + 1 < NS && delta != 0.0) {  // (a zero delta subtracts exactly nothing)
        ppos = lane == np ? gif : ppos;
        pdl = lane == np ? delta : pdl;
        ++np;
      }
      i = first + 1;
      ++nsteps;
    }
    if constexpr (k + 1 < NS) {
      // flush: this sub-block's changes, in chain order, into every later position
      for (int c = 0; c < np; ++c) {
        const int gc = __builtin_amdgcn_readlane(ppos, c);
        const double dc = readlane_f64(pdl, c);
        const int tg = ov_row(gc);
#pragma unroll
        for (int q = k + 1; q < NS; ++q) r[q] = r[q] - tri[gg[q] > gc ? tg + gg[q] : tl[q] + gc] * dc;
      }
#pragma unroll
      for (int q = k + 1; q < NS; ++q) {
        const double tt = r[q] * r[q];
        win = (win & ~(1u << q)) | ((uint32_t)(((valid >> q) & 1u) && tt >= lo[q] && tt <= hi[q]) << q);
      }
    }
  });
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int pos = lane + 64 * q;
    if (pos < bs) { st.bn[pos] = bn[q]; st.fl[pos] = ks[q]; }
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (lane == 0) ov_st(qdone, s + 1);
  if (lane == 0 && nslow) atomicAdd(&d.sc->n_slow, (unsigned long long)nslow);
  if (prof && lane == 0) {
    atomicAdd(&d.sc->prof[6], (unsigned long long)nsteps);
    atomicAdd(&d.sc->prof[7], (unsigned long long)nref);
    atomicAdd(&d.sc->prof[8], (unsigned long long)tslow);
    atomicAdd(&d.sc->prof[9], (unsigned long long)(wall_clock64() - tl0));
  }
}

// The chain as a called function (BRR_OV_CHAIN_CALL=1): its own register allocation, its LDS operands as
// address-space-3 pointers (as chain_hs_call)
#ifndef BRR_OV_CHAIN_CALL
#define BRR_OV_CHAIN_CALL 0
#endif
template <int B>
__device__ __attribute__((noinline)) void chain_bayesr_ov_call(
    const Dev &d, int s, double sigmaE, BRR_LDS double *r0, BRR_LDS double *lo, BRR_LDS double *hi, BRR_LDS double *dsel,
    BRR_LDS double *sdz, BRR_LDS double *bo, BRR_LDS double *bn, BRR_LDS int *fl, BRR_LDS int *gi, BRR_LDS int *m,
    BRR_LDS const double *La, BRR_LDS const double *Lden, BRR_LDS const double *Lp, BRR_LDS const double *Lx2,
    BRR_LDS const double *Lz, BRR_LDS const double *tri, BRR_LDS double *qdl, BRR_LDS int *qgi, BRR_LDS int *qn,
    BRR_LDS int *qdone, BRR_LDS const int *cready, bool prof) {
  const OvSet st{from_lds(r0), from_lds(lo), from_lds(hi), from_lds(dsel), from_lds(sdz), from_lds(bo), from_lds(bn),
                 from_lds(fl), from_lds(gi), from_lds(m)};
  chain_bayesr_ov<B>(d, s, sigmaE, st, from_lds(La), from_lds(Lden), from_lds(Lp), from_lds(Lx2), from_lds(Lz),
                     from_lds(tri), from_lds(qdl), from_lds(qgi), from_lds(qn), from_lds(qdone), from_lds(cready), prof);
}

// Block b's per-component constants (the chain's re-decisions and exact formula): one 1-KiB LDS-DMA per
// field (a_k, D_k, p, x2, z), issued by wave 4
__device__ __forceinline__ void ov_consts_dma(const Dev &d, int b, double *Lc) {
  const int lane = threadIdx.x & 63;
  const int K = d.K, KD = K > 1 ? K - 1 : 0, nf = K + KD + 3;
  const int64_t S = d.nbB, q0 = (int64_t)b * OVB;
  for (int f = 0; f < nf; ++f) {
    const int mf = f < K + KD ? MC_A + f : f == K + KD ? MC_P : f == K + KD + 1 ? MC_XSQ : MC_Z;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(d.mc + mf * S + q0 + 2 * lane),
                                     (__attribute__((address_space(3))) void *)(Lc + (int64_t)f * OVB), 16, 0, 0);
  }
}
__device__ __forceinline__ void ov_consts(const Dev &d, int s, bool nxt, double *Lc, int *misc) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's DMA of block s's constants)
  if ((threadIdx.x & 63) == 0) ov_st(misc + OVF_CREADY, s);
  if (nxt) {
    ov_wait(d, misc + OVF_QDONE, s + 1, 17);  // chain s no longer reads them
    ov_consts_dma(d, s + 1, Lc);
  }
}

// The persistent solver workgroup, overlapped form (Dev::ovs; BayesR family, B = 128, K <= 4).
// Diagnostics (prof_on): [0] wave 0's time between two chains (the block boundary: what the
// preparation did not hide), [2] the chains, [3] the write-backs, [10] the corrector's tail after a
// chain, [13] the deciders' wait for their dots, [15] the Gram loads; [5] blocks.
template <int B>
__device__ __forceinline__ void solver_role_ov(const Dev &d, uint32_t it, char *smem) {
  static_assert(B == OVB, "the overlapped solver runs at B = 128");
  (void)it;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int K = d.K, KD = K > 1 ? K - 1 : 0;
  double *Lc = reinterpret_cast<double *>(smem + OV_OFF_CONST);
  const double *La = Lc, *Lden = Lc + (int64_t)K * B, *Lp = Lc + (int64_t)(K + KD) * B, *Lx2 = Lp + B, *Lz = Lx2 + B;
  double *Lcor = reinterpret_cast<double *>(smem + OV_OFF_COR);
  double *qdl = reinterpret_cast<double *>(smem + OV_OFF_QDL);
  int *qgi = reinterpret_cast<int *>(smem + OV_OFF_QGI);
  int *misc = reinterpret_cast<int *>(smem + OV_OFF_MISC);
  const bool prof = d.sc->prof_on;
  const double sigmaE = d.sc->sigmaE;
  const int s0 = d.seg0, s1 = d.seg1;
  unsigned long long *pf = prof ? d.sc->prof : nullptr;
  if (t < 32) misc[t] = -(1 << 24);  // epochs below every block index
  __syncthreads();
  // prologue: block s0's decision set (no newer changes than its dots: num' is num), Gram triangle and
  // constants
  if (wv == 4) {
    ov_consts_dma(d, s0, Lc);
    lds_barrier();
  } else {
  if (wv == 2 || wv == 3) {
    (void)ov_decide(d, s0, (wv - 2) * 64 + lane, ov_set(smem, s0), sigmaE, nullptr);
  } else if (wv >= 5) {
    ov_load_gram(d, s0, ov_tri(smem, s0), wv - 5, 3);
  }
  __syncthreads();
  }
  uint64_t tprev = 0;
  const int lag = sweep_lag(d);
  OvStash ost;  // (wave 1) the last block's change list
  for (int s = s0; s < s1; ++s) {
    const bool nxt = s + 1 < s1;
    if (wv == 0) {
      const uint64_t tc0 = prof ? wall_clock64() : 0;
      const uint64_t tcs0 = prof ? __builtin_amdgcn_s_memtime() : 0;
#if BRR_OV_CHAIN_CALL
      {
        const OvSet st = ov_set(smem, s);
        chain_bayesr_ov_call<B>(d, s, sigmaE, to_lds(st.r0), to_lds(st.lo), to_lds(st.hi), to_lds(st.dsel), to_lds(st.sdz),
                                to_lds(st.bo), to_lds(st.bn), to_lds(st.fl), to_lds(st.gi), to_lds(st.m), to_lds(La),
                                to_lds(Lden), to_lds(Lp), to_lds(Lx2), to_lds(Lz), to_lds((const double *)ov_tri(smem, s)),
                                to_lds(qdl), to_lds(qgi), to_lds(misc + OVF_QN), to_lds(misc + OVF_QDONE),
                                to_lds((const int *)(misc + OVF_CREADY)), prof);
      }
#else
      chain_bayesr_ov<B>(d, s, sigmaE, ov_set(smem, s), La, Lden, Lp, Lx2, Lz, ov_tri(smem, s), qdl, qgi, misc + OVF_QN,
                         misc + OVF_QDONE, misc + OVF_CREADY, prof);
#endif
      if (prof && lane == 0) {
        const uint64_t tc1 = wall_clock64();
        const uint64_t tcs = __builtin_amdgcn_s_memtime() - tcs0;  // shader clocks of the chain
        atomicAdd(&pf[11], (unsigned long long)tcs);
        atomicAdd(&pf[12], (unsigned long long)tcs);
        atomicAdd(&pf[2], (unsigned long long)(tc1 - tc0));
        if (s > s0) atomicAdd(&pf[0], (unsigned long long)(tc0 - tprev));
        atomicAdd(&pf[5], 1ull);
        unsigned long long *tr = d.trace + (int64_t)s * 16;
        tr[TR_SOLVE0] = tc0;
        tr[TR_GDONE_SEEN] = tc0;
        tr[TR_CHAIN] = tc1;
        tprev = tc1;
      }
    } else if (wv == 1) {
      if (nxt) {
        ov_correct(d, s, s0, lag, ost, ov_set(smem, s), misc + OVF_QN, misc + OVF_QDONE, qdl, qgi, Lcor,
                   pf ? &pf[10] : nullptr);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) ov_st(misc + OVF_CDONE, s);
        if (lag >= 2) ov_stash(d, s, ov_set(smem, s), qdl, qgi, ost);
      }
    } else if (wv == 2 || wv == 3) {
      if (wv == 2) {
        if (s > s0) {
          const uint64_t tw0 = prof ? wall_clock64() : 0;
          ov_writeback(d, s - 1, ov_set(smem, s - 1));
          if (prof && lane == 0) {
            const uint64_t tw1 = wall_clock64();
            atomicAdd(&pf[3], (unsigned long long)(tw1 - tw0));
            d.trace[(int64_t)(s - 1) * 16 + TR_PUB] = tw1;
          }
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) ov_st(misc + OVF_FREE, s);  // block s-1's set is free for block s+1
      } else if (nxt) {
        ov_wait(d, misc + OVF_FREE, s, 12);
      }
      if (nxt) {
        const int pos = (wv - 2) * 64 + lane;
        const OvPos P = ov_decide(d, s + 1, pos, ov_set(smem, s + 1), sigmaE, pf && wv == 2 ? &pf[13] : nullptr);
        ov_wait(d, misc + OVF_CDONE, s, 13);  // block s's changes are in the corrector's sums
        const uint64_t tf0 = prof ? wall_clock64() : 0;
        ov_fold(d, P, pos, ov_set(smem, s + 1), Lcor, sigmaE);
        if (prof && wv == 2 && lane == 0) atomicAdd(&pf[14], (unsigned long long)(wall_clock64() - tf0));
      }
    } else if (wv >= 5) {
      if (nxt) {
        const uint64_t tg0 = prof ? wall_clock64() : 0;
        ov_load_gram(d, s + 1, ov_tri(smem, s + 1), wv - 5, 3);
        if (prof && wv == 5 && lane == 0) atomicAdd(&pf[15], (unsigned long long)(wall_clock64() - tg0));
      }
    } else {
      // wave 4 (wave 0's SIMD: only a few instructions): block s's constants have landed -- the flag the
      // chain's first re-decision waits for -- then, once the chain ends, block s+1's go into the area
      ov_consts(d, s, nxt, Lc, misc);
      lds_barrier();  // (no vmcnt wait: the DMA stays in flight across the barrier)
      continue;
    }
    __syncthreads();
  }
  if (wv == 2) ov_writeback(d, s1 - 1, ov_set(smem, s1 - 1));
}
