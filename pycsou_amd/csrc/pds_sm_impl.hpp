// The general-stencil row march of the fused 2-D step (pds_smarch.hpp): its grid and launches for one
// element type, instantiated by pds_sm32.hip (fp32) and pds_sm64.hip (fp64) -- planning: pds_host.hpp.
#pragma once

#include "pds_host.hpp"

namespace pcs {

// resident workgroups (<= 3 per CU: fewer, longer row segments, as the pt kernel), queried once per element
// type on the centred-K kernel (every K's rings are the same size or smaller)
template <typename T>
int sm_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pds2d_smarch<T, PCS_CENTERED, PCS_F_DENOISE, PCS_H_L21>,
                                                     256, 0) != hipSuccess ||
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
  k_pds2d_smarch<T, KK, FK, HK><<<(unsigned)p.ntasks + fin_extra(a), 256, 0, st>>>((const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, g, b, mi, mo, s, P,
                                           make_sparams<T>(a), a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws,
                                           red_out(a), p.tiles_x, p.bd, p.ntasks, p.sp);
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
int sm_launch(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  switch (a->kkind) {
    case PCS_K_GRAD_FORWARD: return launch_smarch<T, PCS_FORWARD>(a, rb, st);
    case PCS_K_GRAD_BACKWARD: return launch_smarch<T, PCS_BACKWARD>(a, rb, st);
    case PCS_K_GRAD_CENTERED: return launch_smarch<T, PCS_CENTERED>(a, rb, st);
    case PCS_K_LAPLACIAN: return launch_smarch<T, SK_LAP>(a, rb, st);
    default: return PCS_EINVAL;
  }
}


}  // namespace pcs
