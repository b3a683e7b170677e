// brr_device.hpp -- data layout shared by the HIP kernels and the host session.
//
// HBM layout (one session = one GPU = one column shard):
//   X        f32, column-major, ld = roundup(N, 256) rows (1-KiB aligned columns, zero rows
//            beyond N, so a streaming row tile never leaves the allocation); the only
//            large array: streamed once per sweep by k_stream.
//   Xc+xlut  alternative genotype storage: 2-bit codes (a byte = 4 consecutive rows of
//            one column, PLINK .bed packing) in tiles, and a 4-entry f32 value table per column.
//            Tile order: column block b (B columns), group of 16 columns, row quad g (nq = ld/4 =
//            ldc quads), 16 bytes = the group's 16 columns at that quad: byte of (b B + i, g) at
//            ((b B/16 + i/16) nq + g) 16 + i%16 (code_off).  A streaming lane reads 16 columns x 4
//            rows with one 16-byte load and a wave 1 KiB contiguous.  The decoded values are the
//            f32 values the X storage would hold, so every kernel computes on bit-identical
//            inputs; a sweep reads N P / 4 bytes instead of 4 N P.
//   eps,eps2 f64 [ld] residual (Y - mu - X beta), double-buffered across k_stream launches.
//   beta,xsq f64 [M]; comp int32 [M]; sel uint8 [M] (marker selected a component this sweep)
//   gram     f64 [nb][B][B] block Gram matrices X_b^T X_b of the fixed column blocks (for
//            class-coded columns the exact dot products, correctly rounded: k_gram_int).
//   xgram    f64 [nb][B][B] cross-Gram X_b^T X_{b+1 mod nb} of cycle neighbours; xgramT its
//            transposes (rows indexed by block b+1).  Consecutive blocks of a sweep are cycle
//            neighbours (visit order = rotation of the block cycle, either direction).
//   member   int32 [nb*B] marker at (block position s, slot i); gidx = its row in the Gram.
//   mc       f64 [fields][nb*B] per-marker constants of the sweep in visit order (k_prep).
//   slab1/2  f64 partial dot products (2-level deterministic reduction, see k_stream), two
//            copies (block parity): k_stream(s+1) runs while k_solve(s) reads copy s & 1.
//   pend_*   changed markers of a block (three slots, block mod 3): written by k_solve(s),
//            read by k_solve(s+1) (cross-Gram correction) and k_stream(s+2) (residual update).
#pragma once
#include <stdint.h>

namespace brr {

constexpr int MAXK = 8;         // mixture components incl. zero
constexpr int MAXG = 64;        // groups
constexpr int BMAX = 512;       // marker block (Gram rows are staged in LDS on demand)
constexpr int SROWS = 256;      // k_stream rows per workgroup (64 lanes x 4 rows: 1 KiB per column)
constexpr int STREAM_GROUP = 16;  // k_stream workgroups per first-level reduction group
constexpr int FALLTHROUGH = 255;  // no component selected (700-guard, BayesRv2.cpp:216-242)

enum Model : int { MODEL_V2 = 0, MODEL_GROUPS = 1, MODEL_RESTART = 2, MODEL_HORSESHOE = 3 };

// In-process row-shard group (brr_group): the members' copies of one buffer, rank order.
constexpr int GROUP_MAX = 16;
struct GroupPtrs {
  double *ptr[GROUP_MAX];
  int n;
};

// Device-resident scalar state of a chain.
struct Scal {
  double mu, mu_prev, sigmaE, sigmaF, tau, eta, c2;
  double S1;   // sum(eps + mu)   (BayesRv2.cpp:177-178 operand), from the latest row pass
  double S2;   // ||eps||^2        (BayesRv2.cpp:251 operand)
  double fx;   // row shards: this shard's part of a fixed-effect dot (BayesRv2Groups.cpp:220), summed across shards
  int lag_next;  // pipeline lag of the next fused sweep: 2 = Dev::lag, else 1 (set by k_hyper, see Dev::lag_thresh)
  int pad1;
  unsigned long long n_slow;     // diagnostics: serial steps that needed the exact re-evaluation
  unsigned long long n_changed;  // markers whose beta changed (session total)
  unsigned long long nch_mark;   // n_changed at the end of the previous sweep
  int prof_on;                   // diagnostics: k_solve phase timers on
  int pad2;
  unsigned long long prof[20];   // k_solve phase totals (wall_clock64 ticks, 100 MHz), counters;
                                 // [16]: streamer boundaries served by the list prefetch
};

struct Hyper {
  double sigma0, v0E, s02E, v0G, s02G;   // BayesR family
  double A, vL, vT, c2_0, vC, sC;         // Horseshoe
};

// Hand-over words of the stream / solve pipeline (MI355X_MICROARCH.md "Valid forms"): a block
// of their own, each word on its own 128-B line, zeroed by hipMemsetAsync when the session is
// created and afterwards only touched by agent-scope atomics / sc1 accesses.  Counts are
// cumulative over the session (epochs), so nothing is ever reset inside a kernel.
enum SyncWord : int {
  SY_PEND = 0,     // blocks whose k_solve has published its change list (session total)
  SY_GDONE = 32,   // + 32 * (s % NPAR): level-2 reduction groups completed (session total)
  SY_ERR = 160,    // a bounded wait expired; SY_ERR + 1..4: site, target, value seen, workgroup
  SY_ARRIVE = 192, // persistent streamer workgroups that started (session total)
  SY_TS = 224,     // diagnostics: 64-bit wall-clock stamps (see brr_session.cpp)
  SY_WORDS = 256
};

// Pipeline rings: partial-dot slabs, their arrival counters and reduction counts cycle over
// NPAR blocks (block s uses s % NPAR); change lists over NSLOT slots (s % NSLOT).  With a lag
// of L blocks (streamers apply block s-1-L's changes before streaming block s; the solver
// corrects block s's dots for blocks s-1 .. s-L through cross-Gram blocks) the streamers run
// at most L blocks ahead of the solver: NPAR >= L + 1, NSLOT >= L + 2.
constexpr int NPAR = 4;
constexpr int NSLOT = 5;
constexpr int LAG_MAX = 3;

// Stats vector (reduced over markers, summed across shards):
//   [0] sum beta^2  [1] sum beta^2/lambda  [2 .. 2+G) betaAcum[g]  [2+G .. 2+G+G*K) v[g][k]
__host__ __device__ inline int stats_size(int G, int K) { return 2 + G + G * K; }

// Everything a kernel needs: dimensions, hyper-parameters and device pointers (by value).
struct Dev {
  int64_t N, ld, M, M_total, col_offset;
  int64_t Ntot, row_offset;  // row shards: cohort rows and this shard's first row (else N, 0)
  int K, G, F, B, nb, model, R, RG, NG, MRG;
  int seg0, seg1;   // block positions of the current marker-loop launch(es): [seg0, seg1) (the
                    // sweep: [0, nb); a column-shard exchange segment: a part, brr_options)
  int gtarget;      // reduction groups k_solve(s) waits for (per-block: NG * NC; persistent: NG)
  int ngr;          // (fused sweep) arrival groups of the streaming workgroups: the stride of cnt1
  int rcorr;        // (fused sweep) the reducers subtract the cross-Gram corrections from the dots they
                    // write (reduce_role); the solver's phase A then forms none
  int rcsplit;      // (rcorr) the solver corrects for the newest list (block s-1: its own, in its LDS) and the
                    // reducers for the older ones only, so the dots need not wait for the newest publication
  int rcpf;         // (rcorr) the reducers load their columns of those cross-Gram blocks into LDS before the
                    // lists are published
  int slab_storage; // the partial dots are indexed by in-block storage index, not visit position
                    // (fused sweep on 2-bit code tiles)
  int ovs;          // (fused sweep, BayesR family, B = 128) the overlapped solver workgroup (brr_ovsolve.hpp):
                    // block s+1 prepared while block s's chain runs; its corrector forms every cross-Gram
                    // correction (rcorr = 0)
  uint64_t seed;
  Hyper hyp;
  const float *X;      // f32 storage (x_storage BRR_X_F32), else nullptr
  const uint8_t *Xc;   // 2-bit genotype codes (BRR_X_2BIT), else nullptr: column j at Xc + j ldc,
                       // row i in bits 2(i&3)..2(i&3)+1 of byte i>>2 (PLINK .bed packing)
  const float *xlut;   // [M][4] value of each code of column j (padding rows decode to 0)
  const uint8_t *Xcm;  // 2-bit storage, fused sweep without an LDS code cache: the codes column-major (ldc
                       // bytes per column, PLINK packing; k_codes_cm), read by the change-list apply, else nullptr
  int64_t ldc;         // bytes per code column = ld / 4
  // value classes of every column (k_classes): the distinct values of its N rows, ascending, when a
  // column has at most 4 of them (genotype columns, in either storage) -- the integer Gram kernel
  // (k_gram_int) counts class pairs on the i8 matrix cores and forms each Gram entry exactly
  int *cls_info;       // [M] ncls (bits 0-2; 0 = not class-coded) | code -> class map << 8 (2-bit storage)
  float *cls_val;      // [M][4] class values, ascending (classes >= ncls: 0)
  int *cls_cnt;        // [M][4] real rows in each class
  int gram_np;         // k_gram_int's explicit class planes (1..3); 0 = the f64 matrix-core k_gram
  uint8_t *gram_codes; // k_gram_int's input: [nb][B/16][ldc][16] class codes of the current layout (k_encode_layout)
  const uint8_t *xcls;   // REFERENCE order: every column's class codes, column-major (ldc bytes per column;
                        // k_xcls), the source of each sweep's layout encoding (k_encode_gather), else nullptr
  const uint8_t *xcodes; // f32 storage, BLOCKED order: the class codes in storage order (gram_codes of the
                        // init layout), the source of the streamers' code cache (k_sweep_stream<2>), else nullptr
  const double *Y, *fixed, *cva;
  const int *gAssign;
  double *eps, *eps2, *eps_start, *deps, *beta, *xsq, *lambda, *hsv, *sigmaGG, *pi, *alpha;
  double *mc;       // per-position constants, field f at mc + f * nbB (see MC_* in brr_kernels.hip)
  int64_t nbB;      // nb * B
  int *comp, *forder;
  uint8_t *sel;
  double *gram, *xgram, *xgramT;
  double *xgram2, *xgram2T;  // lag >= 2: X_b^T X_{b+2 mod nb} and its transpose (else nullptr)
  double *xgram3, *xgram3T;  // lag 3: X_b^T X_{b+3 mod nb} and its transpose (else nullptr)
  int lag;                   // pipeline lag L (1 or 2, see NPAR): the fused sweep's largest (LDS layout)
  double lag_thresh;         // changes in a sweep above which the next fused sweep runs lag 1: its solver
                             // is then the bottleneck (burn-in), and lag 1 halves its cross-Gram work
  int *member, *gidx, *bsz, *gblk, *blkorder;
  double *slab1, *slab2;   // [2][RG*B], [2][NGpad*B]
  int *cnt1;                // [2][NG*NC] level-2 arrival counters (k_stream), cumulative
  int *sync;                // SyncWord block
  int sbase;                // blocks published before this sweep (SY_PEND epoch base)
  int gbase[NPAR];          // blocks of each ring index before this sweep (SY_GDONE / cnt1 epochs)
  int abase;                // persistent streamer arrivals before this sweep (SY_ARRIVE epoch)
  int64_t slab1_stride, slab2_stride, pend_stride;
  int *pend_idx, *pend_gi;  // [NSLOT][B+16]
  int *pend_pos;            // [NSLOT][B+16] visit position of each change within its block
  double *pend_bo, *pend_bn;
  int *pend_n;              // [NSLOT] padded counts (multiple of 16), then [NSLOT] counts before the padding
  double *rslab;
  int *rcnt;
  double *mslab;
  int *mcnt;
  double *stats;
  unsigned long long *trace;  // diagnostics: [nb][16] wall-clock events of the last traced sweep
  Scal *sc;
};

}  // namespace brr
