// Host-side planning shared by the fused 2-D step's translation units (pds.hip: the ABI, loop control,
// tile and pointwise-F kernels; pds_nm.hip: the separable-PSF row marches; pds_sm32.hip / pds_sm64.hip:
// the general-stencil march per element type).  Kernels are instantiated only in the unit that launches
// them, so the units compile in parallel.
#pragma once

#include "pds_march.hpp"
#include "pds_nmarch.hpp"
#include "pds_smarch.hpp"

namespace pcs {

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
  return a->hist ? RedOut{nullptr, nullptr, 0, a->fin_partials}
                 : RedOut{a->sums_out, a->pre_partials, (int)a->n_pre, nullptr};
}
// workgroups a step launch adds ahead of its tasks (the deferred finalizer slots, pds_ctrl.hpp)
static unsigned fin_extra(const pcs_pds2d_args* a) {
  return a->hist && a->fin_partials ? (unsigned)kFinBlocks : 0u;
}

// ---- fp32 separable conv, tiers 3 and 7: the row-marching kernel (pds_march.hpp) on every
// 64-column strip, reduction + loop control in its last workgroups
constexpr int kMarchNT = 256;
constexpr int kNMarchNT = 256;

struct MarchPlan {
  int tiles_x;  // 64-column strips
  Bands bd;     // row segments of the launch's bands
  int ntasks;   // strips x segments
  StripSplit sp{-1, 0, 0, 0, {0, 0, 0}, Bands{16, 0, 0, 0, 0, 0}};  // border strips on shorter segments (sm_plan)
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

// occupancy-derived grids of the kernels of other units (queried once each)
int march_slots_h(int H);                // pds_nm.hip: k_pds2d_march, tiers 3 / 7
int nmarch_slots_h(int H, bool gen);     // pds_nm.hip: k_pds2d_nmarch(_gen)
template <typename T> int sm_slots();    // pds_sm32.hip / pds_sm64.hip: k_pds2d_smarch
// launches of the other units
int launch_march(const pcs_pds2d_args* a, RowBands rb, hipStream_t st);                      // pds_nm.hip
template <typename T> int sm_launch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st);  // pds_sm*.hip

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
static bool march_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p) {
  const bool nm = use_nmarch(a);
  const int tw = nm ? NMarch<H>::TW : March<H>::TW;
  const int tiles_x = (int)((a->n1 + tw - 1) / tw);
  if (tiles_x < 2) return false;
  plan_bands(rb, March<H>::TS, tiles_x, nm ? nmarch_slots_h(H, a->kkind != PCS_K_GRAD_FORWARD) : march_slots_h(H), 1, p);
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

// ---- fp32 general-stencil K (backward / centred Gradient, Laplacian) with a pointwise grad F:
// the row-marching kernel of pds_smarch.hpp (PCS_SM_FWD=1 also routes the forward Gradient
// through it: diagnostics / A-B against pds_pt.hpp)
static bool sm_forward() {
  const char* e = getenv("PCS_SM_FWD");  // read per call (tests switch it)
  return e != nullptr && atoi(e) != 0;
}

static int sm_slots_for(const pcs_pds2d_args* a) {
  if (a->dtype == PCS_F64) return sm_slots<double>();
  // the masked block (CPS inpainting: z_m and y read, z_m' written on top of the denoising march's words) runs
  // best at two workgroups per CU: 2048^2 35.9-36.5 K it/s against 34.5 at three, 32.0-32.2 at 2.5 (the other
  // fp32 K keep three: Laplacian 39.8-40.6 K at two against 41.4-41.5; profiles/r5_slots_sweep.txt)
  static const bool forced = getenv("PCS_SM_SLOTS") != nullptr;
  const int s = sm_slots<float>();
  return a->mkind != PCS_M_NONE && !forced ? s / 3 * 2 : s;
}

// the fused fp64 normal-operator march (pds_nm64.hip): fp64, separable PSF of tier 3 / 7 with the host's
// Conv^T y and fp64 N tables, Gradient K of any kind, H = lam L1 / L21; PCS_NM64=0 (read per call): the split
// form (N x by k_sep2d_nrmm into the gradient buffer, then the stencil march)
int nm64_slots();
bool nm64_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p);
int launch_nmarch64(const pcs_pds2d_args* a, RowBands rb, hipStream_t st);
static bool use_nm64(const pcs_pds2d_args* a) {
  const char* e = getenv("PCS_NM64");
  if (e != nullptr && atoi(e) == 0) return false;
  if (a->dtype != PCS_F64 || a->fkind != PCS_F_SEPCONV || a->mkind != PCS_M_NONE) return false;
  if (!a->cty || !a->ntaps || !aligned16(a->cty) || a->half < 0) return false;
  if (a->kkind != PCS_K_GRAD_FORWARD && a->kkind != PCS_K_GRAD_BACKWARD && a->kkind != PCS_K_GRAD_CENTERED) return false;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return false;
  const int t = tier_for(a->half);
  if ((t != 3 && t != 7) || !make_slab(a).vec || a->n0 < 64 || a->n1 < 128) return false;
  // slabs: x rows 2H + 1 past the own rows (the PV windows of the U rows one past them), b one, z one
  // (forward K) / two
  if (a->rows < a->n0 &&
      (a->halo_x < 2 * t + 1 || a->halo_y < 1 || a->halo_z < (a->kkind == PCS_K_GRAD_FORWARD ? 1 : 2)))
    return false;
  const int64_t hmax = a->halo_x > a->halo_z ? (a->halo_x > a->halo_y ? a->halo_x : a->halo_y)
                                             : (a->halo_z > a->halo_y ? a->halo_z : a->halo_y);
  if (!(a->n0 < (1LL << 30) && (a->rows + 2 * hmax) * a->n1 * 8 <= (1LL << 30))) return false;
  MarchPlan p;
  return nm64_plan(a, full_bands(a), &p);
}

static bool sm_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p) {
  const int tiles_x = (int)((a->n1 + 63) / 64);
  if (tiles_x < 2) return false;
  // segments of at least 4 16-row steps (fp64: 8)
  const int slots = sm_slots_for(a);
  plan_bands(rb, 16, tiles_x, slots, a->dtype == PCS_F64 ? 8 : 4, p);
  // fp32, one band, backward / centred K or the Laplacian: the border strips (the first, and the last ones
  // whose 4-column margin reaches past n1 - 3) run the column edge rules on every element, so in the one-round
  // grid their tasks end the launch -- 2048^2 Laplacian 23.9 us against 19.3 with interior arithmetic
  // everywhere (profiles/r5_sm_allci_ab.txt).  They get shorter segments (a step count scaled by r), within
  // the same slots.  PCS_SM_SPLIT=0 (read once): one segmentation for every strip
  static const int split_on = [] {
    const char* e = getenv("PCS_SM_SPLIT");
    return e == nullptr || atoi(e) != 0;
  }();
  const bool one_band = rb.rb0 == rb.ra0 || rb.rb1 == rb.ra1;
  if (!split_on || a->dtype != PCS_F32 || !one_band || tiles_x < 4 || a->kkind == PCS_K_GRAD_FORWARD) return true;
  const double r = a->kkind == PCS_K_LAPLACIAN ? 0.8 : 0.85;  // border / interior task steps
  if (rb.rb0 == rb.ra0) rb = RowBands{rb.ra1, rb.rb1, rb.rb1, rb.rb1};
  const int64_t L = rb.rb0 - rb.ra0, steps = (L + 15) / 16;
  int nright = 0;
  for (int j = tiles_x - 1; j >= 1 && 64 * j + 70 > a->n1; --j) ++nright;
  const int nbs = 1 + nright, iw = tiles_x - nbs;
  if (nbs > 3 || iw < 1) return true;
  // only where the split keeps the interior segments as they were (4096^2: it would lengthen them 22 -> 24
  // steps and measured 0.5-1 % slower; 2048^2 keeps 6: Laplacian 23.7 -> 20.0 us, centred 25.3 -> 24.6)
  const int64_t li0 = p->bd.seg_len / 16;
  for (int64_t li = 4; li <= li0; ++li) {
    const int64_t lb = (int64_t)(li * r);
    if (lb < 2 || lb >= li) continue;
    const int64_t ni = (steps + li - 1) / li, nb = (steps + lb - 1) / lb;
    if (iw * ni + nbs * nb > slots) continue;
    p->bd = Bands{(int)(16 * li), (int)((L + 16 * li - 1) / (16 * li)), (int)rb.ra0, (int)rb.rb0, (int)rb.rb0, (int)rb.rb0};
    p->sp.bdb = Bands{(int)(16 * lb), (int)((L + 16 * lb - 1) / (16 * lb)), (int)rb.ra0, (int)rb.rb0, (int)rb.rb0,
                      (int)rb.rb0};
    p->sp.nint = iw * p->bd.nseg0;
    p->sp.ilo = 1;
    p->sp.iw = iw;
    p->sp.nbs = nbs;
    p->sp.bs[0] = 0;
    for (int k = 1; k < nbs; ++k) p->sp.bs[k] = tiles_x - k;
    p->ntasks = p->sp.nint + nbs * p->sp.bdb.nseg0;
    return true;
  }
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

}  // namespace pcs
