// Fused PrimalDualSplitting iteration for 2-D images (one launch per iteration) and the
// device-side loop control that replaces the reference's host loop.
//
// Replaces, for the problem family of the PDS headline benchmark,
//   PrimalDualSplitting.update_iterand      pycsou/opt/proxalgs.py:343-355
//   PrimalDualSplitting.update_diagnostics  pycsou/opt/proxalgs.py:366-394
//   GenericIterativeAlgorithm.iterate loop  pycsou/core/solver.py:55-76
// with F = 1/2 ||Conv x - y||^2 (Conv separable, centred taps), 1/2 ||x - y||^2, 0, or a
// precomputed gradient buffer; K = Gradient(kind='forward'); H = lam*L1 / lam*L21 (pixel
// groups); G = Null / NonNegativeOrthant / Segment.  The tile kernel is in pds_tile.hpp.
#include "pds_host.hpp"
#include "pds_pt.hpp"

namespace pcs {

// ---------------------------------------------------------------- loop control
__global__ void k_ctrl_init(Ctrl* c, int min_iter, int max_iter, double thr, int has_dual, int hist_len) {
  c->it = 0;
  c->min_iter = min_iter;
  c->max_iter = max_iter;
  c->thr = thr;
  c->has_dual = has_dual;
  c->hist_len = hist_len;
  c->pend = c->pad1 = 0;
  const double inf = __builtin_huge_val();
  c->stopped = !((0 <= min_iter) || (0 <= max_iter && inf > thr));
}

// Sum [np][4] partials in a fixed order (deterministic): 1024 threads, 4 independent
// 32-B loads in flight per thread per trip.
constexpr int kRedThreads = 1024;

__device__ __forceinline__ void sum_partials(const double* __restrict__ part, int64_t np, double (&v)[4]) {
  const double4* p4 = reinterpret_cast<const double4*>(part);
  double4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = make_double4(0.0, 0.0, 0.0, 0.0);
  for (int64_t i = threadIdx.x; i < np; i += 4 * kRedThreads) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = i + u * kRedThreads;
      if (j < np) {
        const double4 q = p4[j];
        a[u].x += q.x; a[u].y += q.y; a[u].z += q.z; a[u].w += q.w;
      }
    }
  }
  v[0] = (a[0].x + a[1].x) + (a[2].x + a[3].x);
  v[1] = (a[0].y + a[1].y) + (a[2].y + a[3].y);
  v[2] = (a[0].z + a[1].z) + (a[2].z + a[3].z);
  v[3] = (a[0].w + a[1].w) + (a[2].w + a[3].w);
}

__global__ __launch_bounds__(kRedThreads) void k_reduce_partials(const double* __restrict__ part, int64_t np,
                                                                 double* __restrict__ sums) {
  __shared__ double red[4 * (kRedThreads / 64)];
  double v[4];
  sum_partials(part, np, v);
  block_sum<4>(v, red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) sums[k] = v[k];
  }
}

__global__ void k_finalize(const double* __restrict__ sums, Ctrl* c, double* hist) {
  if (c->stopped) return;
  finalize_from(sums, c, hist);
}

__global__ __launch_bounds__(kRedThreads) void k_reduce_finalize(const double* __restrict__ part, int64_t np, Ctrl* c,
                                                                 double* hist) {
  __shared__ double red[4 * (kRedThreads / 64)];
  double v[4];
  sum_partials(part, np, v);  // loads issued before the (dependent) stop-flag test
  if (c->stopped) return;     // uniform: the whole block leaves together
  block_sum<4>(v, red);
  if (threadIdx.x == 0) finalize_from(v, c, hist);
}

// k iterations' norm sums gathered from `world` ranks as [world][k][4] (the deep-halo slab loop's one
// all-gather per chunk): iteration j's rank rows summed exactly as k_reduce_finalize sums a contiguous
// [world][4] (lane r holds rank r's row, then the block tree), then the loop control, in iteration order.
// Thread 0 alone runs finalize_from and tests the stop flag it wrote itself; iterations after a stop are
// not recorded (solver.py:65-66).
__global__ __launch_bounds__(kRedThreads) void k_reduce_finalize_k(const double* __restrict__ g, int world, int k,
                                                                   Ctrl* c, double* hist) {
  __shared__ double red[4 * (kRedThreads / 64)];
  for (int j = 0; j < k; ++j) {
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if ((int)threadIdx.x < world) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = g[((int64_t)threadIdx.x * k + j) * 4 + q];
    }
    block_sum<4>(v, red);
    if (threadIdx.x == 0 && !c->stopped) finalize_from(v, c, hist);
    __syncthreads();  // red reused by the next iteration's tree
  }
}

__global__ __launch_bounds__(kFinLanes) void k_finalize_pending(const double* __restrict__ part, int64_t np, Ctrl* c,
                                                                double* hist) {
  __shared__ double red[4 * (kFinLanes / 64)];
  __shared__ int flag[1];
  finalize_pending(part, np, c, hist, false, red, flag);
}

// ---------------------------------------------------------------- host dispatch (planning: pds_host.hpp)
template <typename T, int FK, int H>
static int launch_pds2d(const pcs_pds2d_args* a, hipStream_t st) {
  constexpr int TH = Tile<T>::TH, NT = Tile<T>::NT;
  const int tiles_x = (int)((a->n1 + 63) / 64);
  const int tiles_y = (int)((a->rows + TH - 1) / TH);
  const int64_t ntiles = (int64_t)tiles_x * tiles_y;
  if (ntiles > 0x7fffffff) return PCS_EUNSUPPORTED;
  const Slab s = make_slab(a);
  const Params<T> P = make_params<T>(a);
  k_pds2d<T, FK, H, TH, NT><<<(unsigned)ntiles + fin_extra(a), NT, 0, st>>>(
      (const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, (const T*)a->y, (const T*)a->gbuf, (const T*)a->taps0,
      (const T*)a->taps1, a->half, s, P, a->hkind, a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a),
      tiles_x, (int)ntiles, tiles_x, 0);
  return launch_status();
}

// ---- fp32 pointwise grad F (NULL / DENOISE / GRADBUF): the row-marching kernel of pds_pt.hpp
static int pt_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pds2d_pt<PCS_F_DENOISE, PCS_H_L21>, 256, 0) !=
            hipSuccess ||
        nb < 1)
      nb = 4;
    (void)hipGetLastError();
    // 2 workgroups per CU (fewer, longer row segments) although 5 fit: C2 2048^2 with the deferred
    // finalization 41.6-43.1 K it/s at 512 workgroups against 40.6-41.2 at 768, 38.7-38.9 at 640, 37.9-38.5 at
    // 384 and 39.4-39.5 at 1024-1280 (profiles/r5_slots_sweep.txt); 768 with the in-launch reduction
    // (profiles/r1_c2_pt_grid_sweep.txt)
    slots = cus * (nb < 2 ? nb : 2);
    const char* e = getenv("PCS_PT_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

// tasks = 64-column strips x row segments of >= 4 steps, about one wave of resident blocks
static bool pt_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p) {
  const int tiles_x = (int)((a->n1 + PtGeom::TW - 1) / PtGeom::TW);
  if (tiles_x < 2) return false;
  plan_bands(rb, PtGeom::TS, tiles_x, pt_slots(), 4, p);
  return true;
}

static bool use_pt(const pcs_pds2d_args* a) {
  static int disabled = -1;  // PCS_NO_MARCH=1: diagnostics, force the tile kernel
  if (disabled < 0) disabled = getenv("PCS_NO_MARCH") != nullptr;
  if (disabled) return false;
  if (a->dtype != PCS_F32 || !make_slab(a).vec) return false;
  if (a->fkind != PCS_F_NULL && a->fkind != PCS_F_DENOISE && a->fkind != PCS_F_GRADBUF) return false;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return false;
  const int64_t hmax = a->halo_x > a->halo_z ? (a->halo_x > a->halo_y ? a->halo_x : a->halo_y)
                                             : (a->halo_z > a->halo_y ? a->halo_z : a->halo_y);
  if (!(a->n0 < (1LL << 30) && (a->rows + 2 * hmax) * a->n1 * 4 <= (1LL << 30))) return false;
  MarchPlan p;
  return pt_plan(a, full_bands(a), &p);
}

template <int FK, int HK>
static int launch_pt(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  MarchPlan p;
  if (!pt_plan(a, rb, &p)) return PCS_EINVAL;
  if (p.ntasks == 0) return PCS_OK;
  const Slab s64 = make_slab(a);
  const Slab32 s{(int)s64.n0, (int)s64.n1, (int)s64.row0, (int)s64.rows, s64.hx, s64.hy, s64.hz, s64.vec};
  const Params<float> P = make_params<float>(a);
  const float* g = FK == PCS_F_DENOISE ? (const float*)a->y : FK == PCS_F_GRADBUF ? (const float*)a->gbuf : nullptr;
  k_pds2d_pt<FK, HK><<<(unsigned)p.ntasks + fin_extra(a), 256, 0, st>>>((const float*)a->x, (float*)a->xn, (const float*)a->z,
                                                         (float*)a->zn, g, s, P, a->gkind, a->partials,
                                                         (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a), p.tiles_x, p.bd,
                                                         p.ntasks);
  return launch_status();
}

static int64_t bands_nblocks(const pcs_pds2d_args* a, RowBands rb);

template <int FK>
static int launch_pt(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  return a->hkind == PCS_H_L21 ? launch_pt<FK, PCS_H_L21>(a, rb, st) : launch_pt<FK, PCS_H_L1>(a, rb, st);
}

// the row-marching families (march, pt, smarch) take row bands; the tile kernel runs whole slabs only
static int pds2d_bands(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  if (use_nm64(a)) return launch_nmarch64(a, rb, st);
  if (use_smarch(a)) return a->dtype == PCS_F64 ? sm_launch<double>(a, rb, st) : sm_launch<float>(a, rb, st);
  if (use_march(a)) return launch_march(a, rb, st);
  if (a->kkind != PCS_K_GRAD_FORWARD) return PCS_EUNSUPPORTED;
  if (a->fkind == PCS_F_DENOISE) return launch_pt<PCS_F_DENOISE>(a, rb, st);
  if (a->fkind == PCS_F_GRADBUF) return launch_pt<PCS_F_GRADBUF>(a, rb, st);
  return launch_pt<PCS_F_NULL>(a, rb, st);
}

template <typename T>
static int pds2d(const pcs_pds2d_args* a, hipStream_t st) {
  if (use_nm64(a) || use_smarch(a) || use_march(a)) return pds2d_bands(a, full_bands(a), st);
  if (a->kkind != PCS_K_GRAD_FORWARD) return PCS_EUNSUPPORTED;
  if (use_pt(a)) return pds2d_bands(a, full_bands(a), st);
  switch (a->fkind) {
    case PCS_F_NULL: return launch_pds2d<T, PCS_F_NULL, 0>(a, st);
    case PCS_F_DENOISE: return launch_pds2d<T, PCS_F_DENOISE, 0>(a, st);
    case PCS_F_GRADBUF: return launch_pds2d<T, PCS_F_GRADBUF, 0>(a, st);
    case PCS_F_SEPCONV:
      switch (tier_for(a->half)) {
        case 3: return launch_pds2d<T, PCS_F_SEPCONV, 3>(a, st);
        case 7: return launch_pds2d<T, PCS_F_SEPCONV, 7>(a, st);
        case 11: return launch_pds2d<T, PCS_F_SEPCONV, 11>(a, st);
        case 15: return launch_pds2d<T, PCS_F_SEPCONV, 15>(a, st);
        default: return PCS_EUNSUPPORTED;
      }
    default: return PCS_EINVAL;
  }
}

static int64_t bands_nblocks(const pcs_pds2d_args* a, RowBands rb) {
  MarchPlan p;
  if (use_nm64(a)) {
    nm64_plan(a, rb, &p);
    return (int64_t)p.ntasks;
  }
  if (use_smarch(a)) {
    sm_plan(a, rb, &p);
    return (int64_t)p.ntasks;
  }
  if (use_march(a)) {
    if (tier_for(a->half) == 3) march_plan<3>(a, rb, &p);
    else march_plan<7>(a, rb, &p);
    return (int64_t)p.ntasks;
  }
  if (a->kkind != PCS_K_GRAD_FORWARD) return -1;
  if (use_pt(a)) {
    pt_plan(a, rb, &p);
    return (int64_t)p.ntasks;
  }
  return -1;
}

static int needed_halo_x(int fkind, int half) {
  if (fkind != PCS_F_SEPCONV) return 1;  // CONV2D: checked against conv_tier in check_args
  const int t = tier_for(half);
  return t < 0 ? -1 : 2 * t + 1;
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_pds2d_halo_x(int half) { return 1 + 2 * tier_for(half < 0 ? 0 : half); }

int pcs_pds2d_ntaps_len(int half) {
  const int t = tier_for(half < 0 ? 0 : half);
  return (t == 3 || t == 7) ? 64 + 32 * t : -1;
}

// a CONV2D call = its two correlation passes + the GRADBUF step of these arguments
static pcs_pds2d_args step_args(const pcs_pds2d_args* a) {
  pcs_pds2d_args b = *a;
  if (b.fkind == PCS_F_CONV2D) b.fkind = PCS_F_GRADBUF;
  return b;
}

// grad F = Conv^T (Conv x - y) of a general Convolve2D over the stored rows clipped to the image:
// r = Conv x - y -> rbuf, g = Conv^T r -> gbuf (pcs_conv2d_planned; y, rbuf, gbuf in x's layout)
static int conv2d_prepass(const pcs_pds2d_args* a, hipStream_t st) {
  int64_t lo, hi;
  window_rows(a, a->halo_x, &lo, &hi);
  const int64_t off = (lo + a->halo_x) * a->n1 * (a->dtype == PCS_F32 ? 4 : 8);
  const char* xb = (const char*)a->x + off;
  const char* yb = (const char*)a->y + off;
  char* rb = (char*)a->rbuf + off;
  char* gb = (char*)const_cast<void*>(a->gbuf) + off;
  int rc = pcs_conv2d_planned(a->dtype, xb, rb, hi - lo, a->n1, a->conv_fwd, a->conv_tier, yb, -1.0, st);
  if (rc == PCS_OK) rc = pcs_conv2d_planned(a->dtype, rb, gb, hi - lo, a->n1, a->conv_adj, a->conv_tier, nullptr, 0.0, st);
  return rc;
}

int64_t pcs_pds2d_nblocks(const pcs_pds2d_args* a) {
  if (a && a->fkind == PCS_F_CONV2D) {
    const pcs_pds2d_args b = step_args(a);
    return pcs_pds2d_nblocks(&b);
  }
  if (!a || a->rows < 1 || a->n1 < 1) return -1;
  if (use_nm64(a) || use_smarch(a) || a->kkind != PCS_K_GRAD_FORWARD) return bands_nblocks(a, full_bands(a));
  if (use_march(a) || use_pt(a)) return bands_nblocks(a, full_bands(a));
  const int th = a->dtype == PCS_F64 ? Tile<double>::TH : Tile<float>::TH;
  return ((a->n1 + 63) / 64) * ((a->rows + th - 1) / th);
}

int64_t pcs_pds2d_ws_bytes(const pcs_pds2d_args* a) {
  const int64_t nb = pcs_pds2d_nblocks(a);
  return nb < 0 ? -1 : red_ws_bytes(nb);
}

static int check_args(const pcs_pds2d_args* a) {
  if (!a || !a->x || !a->xn || !a->z || !a->zn || !a->partials) return PCS_EINVAL;
  if (a->hist && (!a->ws || !a->ctrl || !aligned16(a->ws) || !aligned16(a->partials))) return PCS_EINVAL;
  if (a->hist && a->fin_partials == a->partials) return PCS_EINVAL;  // the two arrays of deferred finalization
  if (!a->hist && a->sums_out &&
      (!a->ws || !aligned16(a->ws) || !aligned16(a->partials) || a->n_pre < 0 || a->n_pre > 0x7fffffff ||
       (a->n_pre > 0 && !a->pre_partials)))
    return PCS_EINVAL;
  if (a->n0 < 1 || a->n1 < 1 || a->rows < 1 || a->row0 < 0 || a->row0 + a->rows > a->n0) return PCS_EINVAL;
  const bool multi = a->rows < a->n0;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return PCS_EINVAL;
  if (a->gkind < PCS_G_NULL || a->gkind > PCS_G_SEGMENT) return PCS_EINVAL;
  if (!(a->sigma > 0) || !(a->step0 != 0) || !(a->step1 != 0)) return PCS_EINVAL;
  if (a->kkind < PCS_K_GRAD_FORWARD || a->kkind > PCS_K_LAPLACIAN) return PCS_EINVAL;
  if (a->kkind == PCS_K_LAPLACIAN && a->hkind != PCS_H_L1) return PCS_EINVAL;  // one component: L21 == L1
  if (a->kkind != PCS_K_GRAD_FORWARD && a->rows < a->n0 &&
      (a->halo_x < 2 || a->halo_z < 4 || (a->fkind != PCS_F_NULL && a->halo_y < 2)))
    return PCS_EINVAL;
  if (a->fkind == PCS_F_CONV2D) {  // two planned correlations over the stored window, then GRADBUF
    if (!a->conv_fwd || !a->conv_adj || !a->rbuf || !a->gbuf || !a->y || a->halo_y != a->halo_x) return PCS_EINVAL;
    if (a->conv_tier < 3 || !(a->conv_tier & 1) || (multi && a->halo_x < a->conv_tier + 1)) return PCS_EINVAL;
  }
  if (a->fkind == PCS_F_SEPCONV && a->kkind != PCS_K_GRAD_FORWARD && multi &&
      (a->halo_y != a->halo_x || a->halo_x < 2 + 2 * tier_for(a->half)))
    return PCS_EINVAL;
  if ((a->fkind == PCS_F_DENOISE || a->fkind == PCS_F_SEPCONV) && !a->y) return PCS_EINVAL;
  if (a->fkind == PCS_F_GRADBUF && !a->gbuf) return PCS_EINVAL;
  if (a->fkind == PCS_F_SEPCONV && (!a->taps0 || !a->taps1 || a->half < 0)) return PCS_EINVAL;
  if (a->mkind != PCS_M_NONE) {  // the masked block: whole images, F = 0, the row march only
    if (a->mkind != PCS_M_L1LOSS || a->fkind != PCS_F_NULL || multi || !a->ym || !a->zm || !a->zmn) return PCS_EINVAL;
    if (!use_smarch(a)) return PCS_EUNSUPPORTED;
  }
  const int hxn = needed_halo_x(a->fkind, a->half);
  if (hxn < 0) return PCS_EUNSUPPORTED;
  if (multi && (a->halo_x < hxn || a->halo_z < 1 ||
                ((a->fkind == PCS_F_SEPCONV) && a->halo_y < tier_for(a->half) + 1) ||
                ((a->fkind == PCS_F_DENOISE || a->fkind == PCS_F_GRADBUF) && a->halo_y < 1)))
    return PCS_EINVAL;
  return PCS_OK;
}

static bool bands_ok(const pcs_pds2d_args* a, int64_t ra0, int64_t rb0, int64_t ra1, int64_t rb1) {
  return 0 <= ra0 && ra0 <= rb0 && rb0 <= ra1 && ra1 <= rb1 && rb1 <= a->rows;
}

int64_t pcs_pds2d_nblocks_bands(const pcs_pds2d_args* a, int64_t ra0, int64_t rb0, int64_t ra1, int64_t rb1) {
  if (check_args(a) != PCS_OK || !bands_ok(a, ra0, rb0, ra1, rb1)) return -1;
  return bands_nblocks(a, RowBands{ra0, rb0, ra1, rb1});
}

int pcs_pds2d_step_bands(const pcs_pds2d_args* a, int64_t ra0, int64_t rb0, int64_t ra1, int64_t rb1,
                         hipStream_t st) {
  const int rc = check_args(a);
  if (rc != PCS_OK) return rc;
  if (a->hist || !bands_ok(a, ra0, rb0, ra1, rb1)) return PCS_EINVAL;
  if (a->fkind == PCS_F_CONV2D) return PCS_EUNSUPPORTED;  // its correlation passes run once per iteration
  if (!(use_nm64(a) || use_smarch(a) || use_march(a) || (a->kkind == PCS_K_GRAD_FORWARD && use_pt(a))))
    return PCS_EUNSUPPORTED;
  return pds2d_bands(a, RowBands{ra0, rb0, ra1, rb1}, st);
}

int pcs_pds2d_supported(const pcs_pds2d_args* a) {
  if (check_args(a) != PCS_OK) return 0;
  if (a->fkind == PCS_F_CONV2D) {
    const pcs_pds2d_args b = step_args(a);
    return pcs_pds2d_supported(&b);
  }
  if (a->kkind != PCS_K_GRAD_FORWARD) return (use_nm64(a) || use_smarch(a) || use_march(a)) ? 1 : 0;
  if (use_nm64(a) || use_smarch(a) || use_march(a) || use_pt(a)) return 1;
  return (a->dtype == PCS_F32 || a->dtype == PCS_F64) && (a->fkind != PCS_F_SEPCONV || tier_for(a->half) > 0) ? 1 : 0;
}

int pcs_pds2d_path(const pcs_pds2d_args* a) {
  if (check_args(a) != PCS_OK) return -1;
  if (a->fkind == PCS_F_CONV2D) {
    const pcs_pds2d_args b = step_args(a);
    return pcs_pds2d_supported(&b) ? PCS_PATH_CONV2D : -1;
  }
  if (use_nm64(a)) return PCS_PATH_NM64;
  if (use_smarch(a)) return a->fkind == PCS_F_SEPCONV ? PCS_PATH_SMARCH_NX : PCS_PATH_SMARCH;
  if (use_march(a)) return use_nmarch(a) ? PCS_PATH_NMARCH : PCS_PATH_MARCH;
  if (a->kkind != PCS_K_GRAD_FORWARD) return -1;
  if (use_pt(a)) return PCS_PATH_PT;
  return pcs_pds2d_supported(a) ? PCS_PATH_TILE : -1;
}

int pcs_pds2d_step(const pcs_pds2d_args* a, hipStream_t st) {
  int rc = check_args(a);
  if (rc != PCS_OK) return rc;
  if (a->fkind == PCS_F_CONV2D) {
    rc = conv2d_prepass(a, st);
    if (rc != PCS_OK) return rc;
    const pcs_pds2d_args b = step_args(a);
    return pcs_pds2d_step(&b, st);
  }
  if (a->dtype == PCS_F32) return pds2d<float>(a, st);
  if (a->dtype == PCS_F64) return pds2d<double>(a, st);
  return PCS_EINVAL;
}

// n consecutive iterations launched back to back from the host (no graph): iteration i reads
// (x, z) when i is even and (xn, zn) when odd and writes the other pair, so after an even n the
// iterate is back in (x, z).  Needs the in-kernel loop control (hist): after the stopping rule
// fires the remaining launches return at once, exactly as in a captured graph.
int pcs_pds2d_run(const pcs_pds2d_args* a, int64_t n, hipStream_t st) {
  if (!a || n < 0 || !a->hist) return PCS_EINVAL;
  pcs_pds2d_args b = *a;
  for (int64_t i = 0; i < n; ++i) {
    if (i % 2) {
      b.x = a->xn, b.xn = const_cast<void*>(a->x), b.z = a->zn, b.zn = const_cast<void*>(a->z);
      b.zm = a->zmn, b.zmn = const_cast<void*>(a->zm);
      if (a->fin_partials) b.partials = const_cast<double*>(a->fin_partials), b.fin_partials = a->partials;
    } else {
      b.x = a->x, b.xn = a->xn, b.z = a->z, b.zn = a->zn;
      b.zm = a->zm, b.zmn = a->zmn;
      b.partials = a->partials, b.fin_partials = a->fin_partials;
    }
    const int rc = pcs_pds2d_step(&b, st);
    if (rc != PCS_OK) return rc;
  }
  return PCS_OK;
}

int64_t pcs_ctrl_bytes(void) { return 64; }

#ifdef PCS_STAMPS
// diagnostic build only: copy the march kernel's per-segment stamp totals to the host
int pcs_debug_stamps(void* host, int64_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pcs_stamps), (size_t)bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : PCS_ELAUNCH;
}
#endif

int pcs_ctrl_init2(void* ctrl, int min_iter, int max_iter, double thr, int has_dual, int hist_len, hipStream_t st) {
  if (!ctrl || hist_len < 2) return PCS_EINVAL;
  k_ctrl_init<<<1, 1, 0, st>>>((Ctrl*)ctrl, min_iter, max_iter, thr, has_dual, hist_len);
  return launch_status();
}

int pcs_ctrl_init(void* ctrl, int min_iter, int max_iter, double thr, int has_dual, hipStream_t st) {
  const int n = (min_iter > max_iter ? min_iter : max_iter) + 1;
  return pcs_ctrl_init2(ctrl, min_iter, max_iter, thr, has_dual, 2 * (n > 0 ? n : 1) + 2, st);
}

int pcs_reduce_partials(const double* part, int64_t np, double* sums, hipStream_t st) {
  if (!part || !sums || np < 1 || !aligned16(part)) return PCS_EINVAL;
  k_reduce_partials<<<1, kRedThreads, 0, st>>>(part, np, sums);
  return launch_status();
}

int pcs_pds_finalize(const double* sums, void* ctrl, double* hist, hipStream_t st) {
  if (!sums || !ctrl || !hist) return PCS_EINVAL;
  k_finalize<<<1, 1, 0, st>>>(sums, (Ctrl*)ctrl, hist);
  return launch_status();
}

int pcs_pds_finalize_pending(const double* part, int64_t np, void* ctrl, double* hist, hipStream_t st) {
  if (!part || !ctrl || !hist || np < 1) return PCS_EINVAL;
  k_finalize_pending<<<1, kFinLanes, 0, st>>>(part, np, (Ctrl*)ctrl, hist);
  return launch_status();
}

int pcs_pds_reduce_finalize_k(const double* gathered, int world, int k, void* ctrl, double* hist, hipStream_t st) {
  if (!gathered || !ctrl || !hist || world < 1 || world > kRedThreads || k < 1) return PCS_EINVAL;
  // one wave when the ranks fit in it: the same sums as the 1024-thread tree (the other waves add zeros),
  // a fraction of its barriers per iteration
  k_reduce_finalize_k<<<1, world <= 64 ? 64 : kRedThreads, 0, st>>>(gathered, world, k, (Ctrl*)ctrl, hist);
  return launch_status();
}

int pcs_pds_reduce_finalize(const double* part, int64_t np, void* ctrl, double* hist, hipStream_t st) {
  if (!part || !ctrl || !hist || np < 1 || !aligned16(part)) return PCS_EINVAL;
  k_reduce_finalize<<<1, kRedThreads, 0, st>>>(part, np, (Ctrl*)ctrl, hist);
  return launch_status();
}

}  // extern "C"
