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
#include "pds_march.hpp"
#include "pds_nmarch.hpp"
#include "pds_pt.hpp"
#include "pds_smarch.hpp"

namespace pcs {

// ---------------------------------------------------------------- loop control
__global__ void k_ctrl_init(Ctrl* c, int min_iter, int max_iter, double thr, int has_dual, int hist_len) {
  c->it = 0;
  c->min_iter = min_iter;
  c->max_iter = max_iter;
  c->thr = thr;
  c->has_dual = has_dual;
  c->hist_len = hist_len;
  c->pad0 = c->pad1 = 0;
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

// ---------------------------------------------------------------- host dispatch
template <typename T>
struct Tile {
  static constexpr int TH = 31;  // U region = 32 rows
  static constexpr int NT = 256;
};
template <>
struct Tile<double> {
  static constexpr int TH = 15;
  static constexpr int NT = 256;
};

static int tier_for(int half) {
  if (half <= 3) return 3;
  if (half <= 7) return 7;
  if (half <= 11) return 11;
  if (half <= 15) return 15;
  return -1;
}

static bool aligned16(const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; }

static Slab make_slab(const pcs_pds2d_args* a) {
  const int vec = (a->n1 % 4 == 0) && aligned16(a->x) && aligned16(a->xn) && aligned16(a->z) && aligned16(a->zn) &&
                  aligned16(a->y) && aligned16(a->gbuf);
  return Slab{a->n0, a->n1, a->row0, a->rows, a->halo_x, a->halo_y, a->halo_z, vec};
}

template <typename T>
static Params<T> make_params(const pcs_pds2d_args* a) {
  Params<T> P;
  P.tau = (T)a->tau;
  P.sigma = (T)a->sigma;
  P.inv_sigma = (T)(1.0 / a->sigma);
  P.rho = (T)a->rho;
  P.omr = (T)(1.0 - a->rho);
  const double t_h = (1.0 / a->sigma) * a->lam;  // ProxFuncPostComp: tau*scale with tau = 1/sigma
  P.t_h = (T)t_h;
  P.inv_t_h = (T)(1.0 / t_h);
  P.lam = (T)a->lam;
  P.inv_step0 = (T)(1.0 / a->step0);
  P.inv_step1 = (T)(1.0 / a->step1);
  P.unit0 = a->step0 == 1.0;
  P.unit1 = a->step1 == 1.0;
  P.seg_a = (T)a->seg_a;
  P.seg_b = (T)a->seg_b;
  return P;
}

static RedOut red_out(const pcs_pds2d_args* a) {
  return a->hist ? RedOut{nullptr, nullptr, 0} : RedOut{a->sums_out, a->pre_partials, (int)a->n_pre};
}

template <typename T, int FK, int H>
static int launch_pds2d(const pcs_pds2d_args* a, hipStream_t st) {
  constexpr int TH = Tile<T>::TH, NT = Tile<T>::NT;
  const int tiles_x = (int)((a->n1 + 63) / 64);
  const int tiles_y = (int)((a->rows + TH - 1) / TH);
  const int64_t ntiles = (int64_t)tiles_x * tiles_y;
  if (ntiles > 0x7fffffff) return PCS_EUNSUPPORTED;
  const Slab s = make_slab(a);
  const Params<T> P = make_params<T>(a);
  k_pds2d<T, FK, H, TH, NT><<<(unsigned)ntiles, NT, 0, st>>>(
      (const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, (const T*)a->y, (const T*)a->gbuf, (const T*)a->taps0,
      (const T*)a->taps1, a->half, s, P, a->hkind, a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a),
      tiles_x, (int)ntiles, tiles_x, 0);
  return launch_status();
}

// ---- fp32 separable conv, tiers 3 and 7: the row-marching kernel (pds_march.hpp) on every
// 64-column strip, reduction + loop control in its last workgroups
constexpr int kMarchNT = 256;
constexpr int kNMarchNT = 256;

struct MarchPlan {
  int tiles_x;  // 64-column strips
  Bands bd;     // row segments of the launch's bands
  int ntasks;   // strips x segments
};

// own-row bands [ra0, rb0) and [ra1, rb1) of a launch (0 <= ra0 <= rb0 <= ra1 <= rb1 <= rows)
struct RowBands {
  int64_t ra0, rb0, ra1, rb1;
};
static RowBands full_bands(const pcs_pds2d_args* a) { return RowBands{0, a->rows, a->rows, a->rows}; }

// Segments of TS-row steps over the bands: about `slots / tiles_x` segments in all (one wave of
// resident workgroups), at least one per non-empty band, at most one per `min_steps` steps.
static void plan_bands(RowBands rb, int TS, int tiles_x, int slots, int min_steps, MarchPlan* p) {
  if (rb.rb0 == rb.ra0) rb = RowBands{rb.ra1, rb.rb1, rb.rb1, rb.rb1};
  const int64_t L0 = rb.rb0 - rb.ra0, L1 = rb.rb1 - rb.ra1;
  const int64_t steps = (L0 + TS - 1) / TS + (L1 + TS - 1) / TS;
  const int64_t bands = (L0 > 0) + (L1 > 0);
  int64_t nseg = slots / tiles_x;
  const int64_t max_seg = (steps + min_steps - 1) / min_steps;
  nseg = nseg > max_seg ? max_seg : nseg;
  nseg = nseg < bands ? bands : nseg;
  nseg = nseg < 1 ? 1 : nseg;
  const int64_t seg_len = ((steps + nseg - 1) / nseg) * TS;
  const int64_t n0 = (L0 + seg_len - 1) / seg_len, n1 = (L1 + seg_len - 1) / seg_len;
  p->tiles_x = tiles_x;
  p->bd = Bands{(int)seg_len, (int)n0, (int)rb.ra0, (int)rb.rb0, (int)rb.ra1, (int)rb.rb1};
  p->ntasks = (int)(tiles_x * (n0 + n1));
}

// resident workgroups of the march kernel on the whole device (queried once)
template <int H>
static int march_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pds2d_march<float, H, PCS_H_L21, kMarchNT>, kMarchNT,
                                                     0) != hipSuccess ||
        nb < 1)
      nb = 3;
    (void)hipGetLastError();
    slots = cus * nb;
  }
  return slots;
}

// One march task = one 64-column strip x one row segment; as many segments as fill the
// device in one wave of resident workgroups.  False for narrow images (the tile kernel).
template <int H>
static bool march_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p);

// the normal-operator march kernel (pds_nmarch.hpp): fp32 separable tiers 3 / 7 with the host's
// Conv^T y and N tables; images of at least 64 x 64 (the edge bands of N never overlap).  Backward /
// centred K too (its GEN geometry) unless PCS_NMARCH_GEN=0, when the last strip keeps its column
// c0 - 1 out of N_h's right edge band (n1 - c0_last > H); else those K take the stencil march
static bool nmarch_gen_enabled() {
  const char* e = getenv("PCS_NMARCH_GEN");  // read per call (tests and the A/B switch it)
  return e == nullptr || atoi(e) != 0;
}
static bool use_nmarch(const pcs_pds2d_args* a) {
  if (!(a->cty != nullptr && a->ntaps != nullptr && aligned16(a->cty) && a->n0 >= 64 && a->n1 >= 64)) return false;
  if (a->kkind == PCS_K_GRAD_FORWARD) return true;
  if (a->kkind != PCS_K_GRAD_BACKWARD && a->kkind != PCS_K_GRAD_CENTERED) return false;
  const int64_t last = a->n1 - 64 * ((a->n1 + 63) / 64 - 1);  // width of the last 64-column strip
  return nmarch_gen_enabled() && last > tier_for(a->half);
}

template <int H>
static int nmarch_slots(bool gen) {
  static int slots_f = 0, slots_g = 0;
  int& slots = gen ? slots_g : slots_f;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    const hipError_t oe =
        gen ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &nb, k_pds2d_nmarch_gen<float, H, PCS_H_L21, kNMarchNT, PCS_CENTERED>, kNMarchNT, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pds2d_nmarch<float, H, PCS_H_L21, kNMarchNT>,
                                                           kNMarchNT, 0);
    if (oe != hipSuccess ||
        nb < 1)
      nb = 3;
    (void)hipGetLastError();
    slots = cus * nb;
    const char* e = getenv("PCS_NMARCH_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

template <int H>
static bool march_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p) {
  const bool nm = use_nmarch(a);
  const int tw = nm ? NMarch<H>::TW : March<H>::TW;
  const int tiles_x = (int)((a->n1 + tw - 1) / tw);
  if (tiles_x < 2) return false;
  plan_bands(rb, March<H>::TS, tiles_x, nm ? nmarch_slots<H>(a->kkind != PCS_K_GRAD_FORWARD) : march_slots<H>(), 1, p);
  return true;
}

static bool use_march(const pcs_pds2d_args* a) {
  static int disabled = -1;  // PCS_NO_MARCH=1: diagnostics, force the tile kernel
  if (disabled < 0) disabled = getenv("PCS_NO_MARCH") != nullptr;
  if (disabled) return false;
  const int t = tier_for(a->half);
  if (a->dtype != PCS_F32 || a->fkind != PCS_F_SEPCONV || (t != 3 && t != 7) || !make_slab(a).vec) return false;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return false;
  if (a->kkind != PCS_K_GRAD_FORWARD && !use_nmarch(a)) return false;  // only the normal-operator march is general
  const int64_t hmax = a->halo_x > a->halo_z ? (a->halo_x > a->halo_y ? a->halo_x : a->halo_y)
                                             : (a->halo_z > a->halo_y ? a->halo_z : a->halo_y);
  // 32-bit indexing and buffer views of at most 2^30 bytes (pds_march.hpp kOOB)
  if (!(a->n0 < (1LL << 30) && (a->rows + 2 * hmax) * a->n1 * 4 <= (1LL << 30))) return false;
  MarchPlan p;
  return t == 3 ? march_plan<3>(a, full_bands(a), &p) : march_plan<7>(a, full_bands(a), &p);
}

template <int H, int HK>
static int launch_march(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  MarchPlan p;
  if (!march_plan<H>(a, rb, &p)) return PCS_EINVAL;
  if (p.ntasks == 0) return PCS_OK;
  const Slab s64 = make_slab(a);
  const Slab32 s{(int)s64.n0, (int)s64.n1, (int)s64.row0, (int)s64.rows, s64.hx, s64.hy, s64.hz, s64.vec};
  const Params<float> P = make_params<float>(a);
  if (use_nmarch(a) && a->kkind != PCS_K_GRAD_FORWARD) {
    auto kern = a->kkind == PCS_K_GRAD_BACKWARD ? k_pds2d_nmarch_gen<float, H, HK, kNMarchNT, PCS_BACKWARD>
                                                : k_pds2d_nmarch_gen<float, H, HK, kNMarchNT, PCS_CENTERED>;
    kern<<<(unsigned)p.ntasks, kNMarchNT, 0, st>>>((const float*)a->x, (float*)a->xn, (const float*)a->z, (float*)a->zn,
                                                   (const float*)a->cty, (const float*)a->ntaps, s, P, a->gkind,
                                                   a->edge, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a),
                                                   p.tiles_x, p.bd, p.ntasks);
    return launch_status();
  }
  if (use_nmarch(a)) {
    k_pds2d_nmarch<float, H, HK, kNMarchNT><<<(unsigned)p.ntasks, kNMarchNT, 0, st>>>(
        (const float*)a->x, (float*)a->xn, (const float*)a->z, (float*)a->zn, (const float*)a->cty,
        (const float*)a->ntaps, s, P, a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a), p.tiles_x,
        p.bd, p.ntasks);
    return launch_status();
  }
  if (a->kkind != PCS_K_GRAD_FORWARD) return PCS_EUNSUPPORTED;
  k_pds2d_march<float, H, HK, kMarchNT><<<(unsigned)p.ntasks, kMarchNT, 0, st>>>(
      (const float*)a->x, (float*)a->xn, (const float*)a->z, (float*)a->zn, (const float*)a->y,
      (const float*)a->taps0, (const float*)a->taps1, a->half, s, P, a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist,
      a->ws, red_out(a), p.tiles_x, p.bd, p.ntasks);
  return launch_status();
}

template <int H>
static int launch_march(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  return a->hkind == PCS_H_L21 ? launch_march<H, PCS_H_L21>(a, rb, st) : launch_march<H, PCS_H_L1>(a, rb, st);
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
    // 3 workgroups per CU (fewer, longer row segments) although 5 fit: C2 2048^2 measured
    // 29.9 us/iteration at 768 workgroups against 35.7 at 1024-2560 and 30.8 at 512
    // (profiles/r1_c2_pt_grid_sweep.txt)
    slots = cus * (nb < 3 ? nb : 3);
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
  k_pds2d_pt<FK, HK><<<(unsigned)p.ntasks, 256, 0, st>>>((const float*)a->x, (float*)a->xn, (const float*)a->z,
                                                         (float*)a->zn, g, s, P, a->gkind, a->partials,
                                                         (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a), p.tiles_x, p.bd,
                                                         p.ntasks);
  return launch_status();
}

static int64_t bands_nblocks(const pcs_pds2d_args* a, RowBands rb);

// persistent form: all n iterations in one launch; the grid must be co-resident
template <int FK, int HK>
static int launch_pt_loop(const pcs_pds2d_args* a, int64_t n, unsigned* bar, hipStream_t st) {
  int dev = 0, cus = 0, nb = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pds2d_pt_loop<FK, HK>, 256, 0) != hipSuccess)
    return PCS_ELAUNCH;
  const int tiles_x = (int)((a->n1 + PtGeom::TW - 1) / PtGeom::TW);
  // the occupancy query can over-report by one block/CU for SGPR-heavy kernels: at most 4
  // blocks of 256 threads per CU for a grid that must be co-resident
  nb = nb > 3 ? 3 : nb;  // and 3 per CU is the fastest grid of the per-launch kernel too
  if (tiles_x < 2 || nb < 1) return PCS_EUNSUPPORTED;
  // one wave of this kernel's resident workgroups, and never more tasks than the per-launch
  // plan that sized the caller's partials / ws buffers (pcs_pds2d_nblocks, pt_slots())
  const int slots = cus * nb < pt_slots() ? cus * nb : pt_slots();
  MarchPlan p;
  plan_bands(full_bands(a), PtGeom::TS, tiles_x, slots, 4, &p);
  if (p.ntasks < 1 || (int64_t)p.ntasks > (int64_t)cus * nb || (int64_t)p.ntasks > bands_nblocks(a, full_bands(a)))
    return PCS_EUNSUPPORTED;
  // fresh barrier state for every launch: a timed-out barrier of an earlier launch (sticky
  // flag, stranded arrival count) cannot leak into this one
  if (hipMemsetAsync(bar, 0, (size_t)pcs_grid_bar_bytes(), st) != hipSuccess) return PCS_ELAUNCH;
  const Slab s64 = make_slab(a);
  const Slab32 s{(int)s64.n0, (int)s64.n1, (int)s64.row0, (int)s64.rows, s64.hx, s64.hy, s64.hz, s64.vec};
  const Params<float> P = make_params<float>(a);
  const float* g = FK == PCS_F_DENOISE ? (const float*)a->y : FK == PCS_F_GRADBUF ? (const float*)a->gbuf : nullptr;
  k_pds2d_pt_loop<FK, HK><<<(unsigned)p.ntasks, 256, 0, st>>>(
      (float*)a->x, (float*)a->xn, (float*)a->z, (float*)a->zn, g, s, P, a->gkind, a->partials, (Ctrl*)a->ctrl,
      a->hist, a->ws, bar, (int)n, p.tiles_x, p.bd, p.ntasks);
  return launch_status();
}

template <int FK>
static int launch_pt_loop(const pcs_pds2d_args* a, int64_t n, unsigned* bar, hipStream_t st) {
  return a->hkind == PCS_H_L21 ? launch_pt_loop<FK, PCS_H_L21>(a, n, bar, st)
                               : launch_pt_loop<FK, PCS_H_L1>(a, n, bar, st);
}

template <int FK>
static int launch_pt(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  return a->hkind == PCS_H_L21 ? launch_pt<FK, PCS_H_L21>(a, rb, st) : launch_pt<FK, PCS_H_L1>(a, rb, st);
}

// ---- fp32 general-stencil K (backward / centred Gradient, Laplacian) with a pointwise grad F:
// the row-marching kernel of pds_smarch.hpp (PCS_SM_FWD=1 also routes the forward Gradient
// through it: diagnostics / A-B against pds_pt.hpp)
static bool sm_forward() {
  const char* e = getenv("PCS_SM_FWD");  // read per call (tests switch it)
  return e != nullptr && atoi(e) != 0;
}

// 16-row halves per step of the march (SMarch RS): 2 = 32-row steps (twice the loads in flight per
// barrier, half the steps; the Laplacian's single z component leaves the LDS for 64-row rings at 3
// workgroups / CU).  Measured (tools/sm_probe.py, profiles/r4_sm_rs_ab.txt): Laplacian 2048^2 28.7 us
// either way, 4096^2 82.0 against 76.6 us; centred 31.0 against 29.6-29.9 us at 2048^2 -- the 2048^2
// time is not the per-step latency.  Default 1; PCS_SM_RS=2 (read once) for every fp32 K (parity
// green at RS = 2 for every smarch case, profiles/r4_sm_rs_ab.txt)
static int sm_rs(const pcs_pds2d_args* a) {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("PCS_SM_RS");
    env = e ? atoi(e) : 0;
  }
  if (a->dtype != PCS_F32) return 1;
  return env == 2 ? 2 : 1;
}

// resident workgroups (<= 3 per CU: fewer, longer row segments, as the pt kernel), queried once per
// kernel shape: RS = 1 takes the centred-K kernel's occupancy for every K (rings of the same size or
// smaller), RS = 2 its own K's
template <typename T, int KK, int RS>
static int sm_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    constexpr int QK = RS == 1 ? PCS_CENTERED : KK;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, k_pds2d_smarch<T, QK, PCS_F_DENOISE, QK == SK_LAP ? PCS_H_L1 : PCS_H_L21, RS>, 256, 0) != hipSuccess ||
        nb < 1)
      nb = sizeof(T) == 4 ? 3 : 2;
    (void)hipGetLastError();
    slots = cus * (nb < 3 ? nb : 3);
    // fp64: three rounds of the resident workgroups (later ones start as earlier ones finish), with
    // segments of >= 8 steps (sm_plan).  fp64 C3 4096^2: 3326-3379 it/s against 3194-3219 at one round,
    // 3139-3226 at four or six (profiles/r4_f64_step_slots.txt)
    if (sizeof(T) == 8) slots *= 3;
    const char* e = getenv("PCS_SM_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

static int sm_slots_for(const pcs_pds2d_args* a, int rs) {
  if (a->dtype == PCS_F64) return sm_slots<double, PCS_CENTERED, 1>();
  if (rs == 1) return sm_slots<float, PCS_CENTERED, 1>();
  switch (a->kkind) {
    case PCS_K_GRAD_FORWARD: return sm_slots<float, PCS_FORWARD, 2>();
    case PCS_K_GRAD_BACKWARD: return sm_slots<float, PCS_BACKWARD, 2>();
    case PCS_K_LAPLACIAN: return sm_slots<float, SK_LAP, 2>();
    default: return sm_slots<float, PCS_CENTERED, 2>();
  }
}

static bool sm_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p) {
  const int tiles_x = (int)((a->n1 + 63) / 64);
  if (tiles_x < 2) return false;
  const int rs = sm_rs(a);
  // at least 4 16-row halves per segment (2 steps of 32 rows); fp64 at least 8 steps
  plan_bands(rb, 16 * rs, tiles_x, sm_slots_for(a, rs), a->dtype == PCS_F64 ? 8 : 4 / rs, p);
  return true;
}

// F = (1/2)||Conv x - y||^2, Conv separable, with a non-forward K: grad F = N x - Conv^T y, N x by the
// in-plane normal-operator kernel into gbuf (pcs_conv2d_sep_ata_planes on the whole image: two
// composite-tap passes), then the march step reads gbuf and cty -- whole images only
// local rows [lo, hi) of the stored window (halo h) clipped to the image
static void window_rows(const pcs_pds2d_args* a, int h, int64_t* lo, int64_t* hi) {
  *lo = -h > -a->row0 ? -h : -a->row0;
  *hi = a->rows + h < a->n0 - a->row0 ? a->rows + h : a->n0 - a->row0;
}

static bool sm_normal(const pcs_pds2d_args* a) {
  if (a->fkind != PCS_F_SEPCONV || !a->cty || !a->gbuf || !aligned16(a->cty) || a->halo_y != a->halo_x) return false;
  if (a->half < 0 || a->half > 7 || !a->taps0 || !a->taps1) return false;
  int64_t lo, hi;
  window_rows(a, a->halo_x, &lo, &hi);
  // shape / tap validation only (nplanes 0): any non-null input will do before x is bound
  return pcs_conv2d_sep_ata_planes(a->dtype, a->x ? a->x : a->cty, const_cast<void*>(a->gbuf), 0, hi - lo, a->n1,
                                   a->taps0, 2 * a->half + 1, a->half, a->taps1, 2 * a->half + 1, a->half,
                                   nullptr) == PCS_OK;
}

static bool use_march(const pcs_pds2d_args* a);
// sep_ata.hip: N x - sub by the two-pass normal-operator kernel (PCS_EUNSUPPORTED: taps / layout it does not take)
int sep_normal_minus(int dt, const void* in, void* out, const void* sub, int64_t np, int64_t n1, int64_t n2,
                     const void* ha, int ka, int offa, const void* hb, int kb, int offb, hipStream_t st);

// fp64 (the reference's default dtype): every K kind, the forward Gradient included, takes this march
// (the forward-only fp32 kernels pds_pt.hpp / pds_nmarch.hpp have no fp64 form)
static bool use_smarch(const pcs_pds2d_args* a) {
  if (a->kkind == PCS_K_GRAD_FORWARD && !sm_forward() && a->dtype != PCS_F64 && a->mkind == PCS_M_NONE) return false;
  // separable PSF with backward / centred K: the fused normal-operator march (one launch) when it applies
  if (a->kkind != PCS_K_GRAD_FORWARD && a->fkind == PCS_F_SEPCONV && use_march(a)) return false;
  if (a->kkind < PCS_K_GRAD_FORWARD || a->kkind > PCS_K_LAPLACIAN) return false;
  if ((a->dtype != PCS_F32 && a->dtype != PCS_F64) || !make_slab(a).vec) return false;
  if (a->fkind != PCS_F_NULL && a->fkind != PCS_F_DENOISE && a->fkind != PCS_F_GRADBUF &&
      !((a->kkind != PCS_K_GRAD_FORWARD || a->dtype == PCS_F64) && sm_normal(a)))
    return false;
  if (a->mkind != PCS_M_NONE && (a->fkind != PCS_F_NULL || !aligned16(a->ym) || !aligned16(a->zm) || !aligned16(a->zmn)))
    return false;
  if (a->hkind != PCS_H_L1 && (a->hkind != PCS_H_L21 || a->kkind == PCS_K_LAPLACIAN)) return false;
  const int64_t hmax = a->halo_x > a->halo_z ? (a->halo_x > a->halo_y ? a->halo_x : a->halo_y)
                                             : (a->halo_z > a->halo_y ? a->halo_z : a->halo_y);
  const int64_t esz = a->dtype == PCS_F64 ? 8 : 4;
  // 32-bit indexing; every buffer view (z: one per component) at most 2^30 bytes (kOOB)
  if (!(a->n0 < (1LL << 30) && (a->rows + 2 * hmax) * a->n1 * esz <= (1LL << 30))) return false;
  MarchPlan p;
  return sm_plan(a, full_bands(a), &p);
}

template <typename T>
static SParamsT<T> make_sparams(const pcs_pds2d_args* a) {
  SParamsT<T> Q;
  Q.ih20 = (T)(1.0 / (a->step0 * a->step0));
  Q.ih21 = (T)(1.0 / (a->step1 * a->step1));
  Q.w0 = (T)a->w0;
  Q.w1 = (T)a->w1;
  Q.edge = a->edge != 0;
  return Q;
}

template <typename T, int KK, int FK, int HK>
static int launch_smarch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  MarchPlan p;
  if (!sm_plan(a, rb, &p)) return PCS_EINVAL;
  if (p.ntasks == 0) return PCS_OK;
  const Slab s64 = make_slab(a);
  const Slab32 s{(int)s64.n0, (int)s64.n1, (int)s64.row0, (int)s64.rows, s64.hx, s64.hy, s64.hz, s64.vec};
  const Params<T> P = make_params<T>(a);
  const T* g = FK == PCS_F_DENOISE                       ? (const T*)a->y
               : (FK == PCS_F_GRADBUF || FK == SM_F_NB) ? (const T*)a->gbuf
                                                        : nullptr;
  const T* b = FK == SM_F_NB ? (const T*)a->cty : nullptr;
  if constexpr (FK == SM_F_MASK) g = (const T*)a->ym;
  const T* mi = FK == SM_F_MASK ? (const T*)a->zm : nullptr;
  T* mo = FK == SM_F_MASK ? (T*)a->zmn : nullptr;
  auto* kern = k_pds2d_smarch<T, KK, FK, HK, 1>;
  if constexpr (sizeof(T) == 4)
    if (sm_rs(a) == 2) kern = k_pds2d_smarch<T, KK, FK, HK, 2>;
  kern<<<(unsigned)p.ntasks, 256, 0, st>>>((const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, g, b, mi, mo, s, P,
                                           make_sparams<T>(a), a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws,
                                           red_out(a), p.tiles_x, p.bd, p.ntasks);
  return launch_status();
}

template <typename T, int KK, int FK>
static int launch_smarch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  if constexpr (KK == SK_LAP) return launch_smarch<T, KK, FK, PCS_H_L1>(a, rb, st);
  else
    return a->hkind == PCS_H_L21 ? launch_smarch<T, KK, FK, PCS_H_L21>(a, rb, st)
                                 : launch_smarch<T, KK, FK, PCS_H_L1>(a, rb, st);
}

template <typename T, int KK>
static int launch_smarch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  if (a->fkind == PCS_F_SEPCONV) {  // N x -> gbuf on the stored rows (clipped to the image), then the
    // step with grad F = gbuf - cty; whole slabs only (the N x pass runs once per iteration).  The
    // forward Gradient comes here in fp64 only (fp32 has the fused normal-operator march)
    if ((KK == PCS_FORWARD && sizeof(T) == 4) || rb.ra0 != 0 || rb.rb0 != a->rows) return PCS_EUNSUPPORTED;
    int64_t lo, hi;
    window_rows(a, a->halo_x, &lo, &hi);
    const int64_t off = (lo + a->halo_x) * a->n1;
    // grad F = N x - Conv^T y formed by the normal-operator kernel itself (it reads Conv^T y as it stores): the
    // step then reads one buffer (7 words instead of 8; the same subtraction, bit for bit).  PCS_NX_SUB=0
    // (read once): N x alone and the subtraction in the step
    static int nx_sub = -1;
    if (nx_sub < 0) {
      const char* e = getenv("PCS_NX_SUB");
      nx_sub = e == nullptr || atoi(e) != 0;
    }
    if (nx_sub) {
      const int rs = sep_normal_minus(a->dtype, (const T*)a->x + off, (T*)const_cast<void*>(a->gbuf) + off,
                                      (const T*)a->cty + off, 1, hi - lo, a->n1, a->taps0, 2 * a->half + 1, a->half,
                                      a->taps1, 2 * a->half + 1, a->half, st);
      if (rs == PCS_OK) return launch_smarch<T, KK, PCS_F_GRADBUF>(a, rb, st);
      if (rs != PCS_EUNSUPPORTED) return rs;
    }
    const int rc = pcs_conv2d_sep_ata_planes(a->dtype, (const T*)a->x + off, (T*)const_cast<void*>(a->gbuf) + off, 1,
                                             hi - lo, a->n1, a->taps0, 2 * a->half + 1, a->half, a->taps1,
                                             2 * a->half + 1, a->half, st);
    if (rc != PCS_OK) return rc;
    return launch_smarch<T, KK, SM_F_NB>(a, rb, st);
  }
  if (a->mkind == PCS_M_L1LOSS) return launch_smarch<T, KK, SM_F_MASK>(a, rb, st);
  if (a->fkind == PCS_F_DENOISE) return launch_smarch<T, KK, PCS_F_DENOISE>(a, rb, st);
  if (a->fkind == PCS_F_GRADBUF) return launch_smarch<T, KK, PCS_F_GRADBUF>(a, rb, st);
  return launch_smarch<T, KK, PCS_F_NULL>(a, rb, st);
}

template <typename T>
static int launch_smarch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  switch (a->kkind) {
    case PCS_K_GRAD_FORWARD: return launch_smarch<T, PCS_FORWARD>(a, rb, st);
    case PCS_K_GRAD_BACKWARD: return launch_smarch<T, PCS_BACKWARD>(a, rb, st);
    case PCS_K_GRAD_CENTERED: return launch_smarch<T, PCS_CENTERED>(a, rb, st);
    case PCS_K_LAPLACIAN: return launch_smarch<T, SK_LAP>(a, rb, st);
    default: return PCS_EINVAL;
  }
}

static int launch_smarch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  return a->dtype == PCS_F64 ? launch_smarch<double>(a, rb, st) : launch_smarch<float>(a, rb, st);
}

// the row-marching families (march, pt, smarch) take row bands; the tile kernel runs whole slabs only
static int pds2d_bands(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  if (use_smarch(a)) return launch_smarch(a, rb, st);
  if (use_march(a)) return tier_for(a->half) == 3 ? launch_march<3>(a, rb, st) : launch_march<7>(a, rb, st);
  if (a->kkind != PCS_K_GRAD_FORWARD) return PCS_EUNSUPPORTED;
  if (a->fkind == PCS_F_DENOISE) return launch_pt<PCS_F_DENOISE>(a, rb, st);
  if (a->fkind == PCS_F_GRADBUF) return launch_pt<PCS_F_GRADBUF>(a, rb, st);
  return launch_pt<PCS_F_NULL>(a, rb, st);
}

template <typename T>
static int pds2d(const pcs_pds2d_args* a, hipStream_t st) {
  if (use_smarch(a) || use_march(a)) return pds2d_bands(a, full_bands(a), st);
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
  if (use_smarch(a) || a->kkind != PCS_K_GRAD_FORWARD) return bands_nblocks(a, full_bands(a));
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
  if (!(use_smarch(a) || use_march(a) || (a->kkind == PCS_K_GRAD_FORWARD && use_pt(a)))) return PCS_EUNSUPPORTED;
  return pds2d_bands(a, RowBands{ra0, rb0, ra1, rb1}, st);
}

int pcs_pds2d_supported(const pcs_pds2d_args* a) {
  if (check_args(a) != PCS_OK) return 0;
  if (a->fkind == PCS_F_CONV2D) {
    const pcs_pds2d_args b = step_args(a);
    return pcs_pds2d_supported(&b);
  }
  if (a->kkind != PCS_K_GRAD_FORWARD) return (use_smarch(a) || use_march(a)) ? 1 : 0;
  if (use_smarch(a) || use_march(a) || use_pt(a)) return 1;
  return (a->dtype == PCS_F32 || a->dtype == PCS_F64) && (a->fkind != PCS_F_SEPCONV || tier_for(a->half) > 0) ? 1 : 0;
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
    } else {
      b.x = a->x, b.xn = a->xn, b.z = a->z, b.zn = a->zn;
      b.zm = a->zm, b.zmn = a->zmn;
    }
    const int rc = pcs_pds2d_step(&b, st);
    if (rc != PCS_OK) return rc;
  }
  return PCS_OK;
}

// The same n iterations as pcs_pds2d_run in ONE launch of the pointwise-F row-marching kernel
// (fp32 NULL / DENOISE / GRADBUF families), a grid barrier per iteration in place of the
// kernel boundary.  `bar`: pcs_grid_bar_bytes() device bytes, zeroed once before first use.
// PCS_EUNSUPPORTED when the problem is not of that family or its grid is not co-resident.
int pcs_pds2d_run_persistent(const pcs_pds2d_args* a, int64_t n, void* bar, hipStream_t st) {
  if (!a || n < 0 || n > 0x7fffffff || !a->hist || !bar || !aligned16(bar)) return PCS_EINVAL;
  const int rc = check_args(a);
  if (rc != PCS_OK) return rc;
  if (a->rows != a->n0 || a->kkind != PCS_K_GRAD_FORWARD || use_smarch(a) || use_march(a) || !use_pt(a))
    return PCS_EUNSUPPORTED;
  if (n == 0) return PCS_OK;
  unsigned* b = (unsigned*)bar;
  if (a->fkind == PCS_F_DENOISE) return launch_pt_loop<PCS_F_DENOISE>(a, n, b, st);
  if (a->fkind == PCS_F_GRADBUF) return launch_pt_loop<PCS_F_GRADBUF>(a, n, b, st);
  return launch_pt_loop<PCS_F_NULL>(a, n, b, st);
}

int64_t pcs_grid_bar_bytes(void) { return 512; }

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

int pcs_pds_reduce_finalize(const double* part, int64_t np, void* ctrl, double* hist, hipStream_t st) {
  if (!part || !ctrl || !hist || np < 1 || !aligned16(part)) return PCS_EINVAL;
  k_reduce_finalize<<<1, kRedThreads, 0, st>>>(part, np, (Ctrl*)ctrl, hist);
  return launch_status();
}

}  // extern "C"
