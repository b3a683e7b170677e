// brr_launch.hpp -- host-callable launch wrappers for the kernels in brr_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "brr_device.hpp"

namespace brr {

enum RowFlagsHost : int {
  H_ROW_SHIFT = 1, H_ROW_PENDING = 2, H_ROW_WRITE = 4, H_ROW_SNAPSHOT = 8, H_ROW_DEPS = 16,
  H_ROW_EXCHANGE = 32, H_ROW_REDUCE = 64, H_ROW_INIT_Y = 128
};
enum MarkerModeHost : int { H_MR_BAYESR = 0, H_MR_HS = 1, H_MR_COUNT_ALL = 2 };

hipError_t launch_synth_x(const Dev &d, uint64_t ds, hipStream_t st);
hipError_t launch_synth_y(const Dev &d, const int *cidx, const double *cb, int nc, double *y, hipStream_t st);
hipError_t launch_cast_x(const void *src, bool is_f64, int64_t lds, float *dst, int64_t ldd,
                         int64_t N, int64_t M, hipStream_t st);
hipError_t launch_codes_cm(const Dev &d, uint8_t *xcm, hipStream_t st);
hipError_t launch_codes_tile(const uint8_t *src, uint8_t *Xc, int64_t c0, int64_t nc, int64_t ldc, int B,
                             hipStream_t st);
hipError_t launch_classes(const Dev &d, int *flags, hipStream_t st);
hipError_t launch_encode_layout(const Dev &d, hipStream_t st);  // class codes of the layout (Dev::gram_codes)
hipError_t launch_xcls(const Dev &d, uint8_t *xcls, hipStream_t st);  // column-major class codes (REFERENCE order)
// Gram blocks: k_gram_int (exact, i8 matrix cores) when Dev::gram_np > 0, else k_gram (FP64 MFMA)
hipError_t launch_gram(const Dev &d, int shift, double *G, double *GT, hipStream_t st);
// the Gram blocks come from Dev::xcls (REFERENCE order, k_gram_fp4): no layout encoding needed
bool gram_reads_xcls(const Dev &d);
hipError_t launch_xsq(const Dev &d, hipStream_t st);
hipError_t launch_rows(const Dev &d, int flags, const double *deps_in, hipStream_t st,
                       const double *eps_in = nullptr, int slot_a = -1, int slot_b = -1);
hipError_t launch_sweep_start(const Dev &d, uint32_t it, hipStream_t st);
hipError_t launch_noop(hipStream_t st);
hipError_t launch_perm(const Dev &d, uint32_t it, int shard, bool identity, hipStream_t st);
hipError_t launch_fixed(const Dev &d, uint32_t it, bool perm_on_device, hipStream_t st);
hipError_t launch_stream(const Dev &d, int s, const double *eps_in, double *eps_out, hipStream_t st);
// row shards
hipError_t launch_fixed_row(const Dev &d, uint32_t it, int cf, int phase, bool perm_on_device, hipStream_t st);
hipError_t launch_slab_total(const Dev &d, int s, hipStream_t st);
hipError_t launch_group_sum(const GroupPtrs &p, int64_t n, hipStream_t st);
hipError_t launch_prep(const Dev &d, uint32_t it, hipStream_t st);
struct FusedCfg {
  int nsg = 0, rpw = 0, npass = 0, nslot = 0, ngroups = 0, nred = 0, narr = 0;
  int ccache = 0;  // the streamers keep the last blocks' code tiles in LDS (2-bit storage; f32: see f32cc)
  int f32cc = 0;   // f32 storage: room for the class-code cache (used when Dev::xcodes is set: k_sweep_stream<2>)
  int split = 0;   // solver and streaming workgroups as two kernels side by side (else one k_sweep)
  int pfe = 0;     // (split, f32 storage) list entries the streamers can prefetch before a boundary (0: off)
  int stnt = 512;  // (split) threads per streaming / reducing workgroup (1024: 2-bit codes at B >= 256)
  int rcpf = 0;    // a reducer's LDS holds its cross-Gram slices (Dev::rcpf)
  int prof = 0;    // (split) launch the streaming kernel's diagnostics variant (Scal::prof_on is set)
  size_t lds = 0;     // solver workgroup's dynamic LDS (one kernel: every workgroup's)
  size_t st_lds = 0;  // (split) streaming / reducing workgroups' dynamic LDS
};
bool fused_config(const Dev &d, int cus, int max_wg, FusedCfg *cfg, bool f32cc = false);
bool ov_solver_ok(const Dev &d, const FusedCfg &c);
// split: the solver kernel on st, the streaming kernel on st_side (ev_go / ev_done order them
// against st); otherwise one k_sweep grid on st (BRR_FUSED_SINGLE=1: the PMC passes' form)
hipError_t launch_sweep_fused(const Dev &d, uint32_t it, const FusedCfg &c, hipStream_t st, hipStream_t st_side,
                              hipEvent_t ev_go, hipEvent_t ev_done);
hipError_t launch_solve(const Dev &d, int s, uint32_t it, hipStream_t st);
hipError_t set_solve_lds_limit(int B);
size_t solve_lds_bytes(int B, int K);
hipError_t launch_linpred(const Dev &d, double *out, hipStream_t st);
hipError_t launch_slab_sentinels(const Dev &d, int nrow, hipStream_t st);  // fused solver's dot slots (epoch p in slot p)
hipError_t launch_markers(const Dev &d, int mode, uint32_t it, hipStream_t st);
hipError_t launch_hyper(const Dev &d, uint32_t it, const double *stats, hipStream_t st);
hipError_t launch_hyper_init(const Dev &d, const double *stats, bool pi_given, hipStream_t st);

}  // namespace brr
