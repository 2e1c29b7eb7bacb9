// The separable-PSF row marches of the fused 2-D step (fp32, tiers 3 / 7): k_pds2d_march (four
// 15-tap passes) and the normal-operator marches k_pds2d_nmarch / k_pds2d_nmarch_gen (grad F = N x -
// Conv^T y, pds_nmarch.hpp) -- their grids and launches (planning: pds_host.hpp).
#include "pds_host.hpp"

namespace pcs {

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

int march_slots_h(int H) { return H == 3 ? march_slots<3>() : march_slots<7>(); }
int nmarch_slots_h(int H, bool gen) { return H == 3 ? nmarch_slots<3>(gen) : nmarch_slots<7>(gen); }

template <int H, int HK>
static int launch_march_k(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  MarchPlan p;
  if (!march_plan<H>(a, rb, &p)) return PCS_EINVAL;
  if (p.ntasks == 0) return PCS_OK;
  const Slab s64 = make_slab(a);
  const Slab32 s{(int)s64.n0, (int)s64.n1, (int)s64.row0, (int)s64.rows, s64.hx, s64.hy, s64.hz, s64.vec};
  const Params<float> P = make_params<float>(a);
  if (use_nmarch(a) && a->kkind != PCS_K_GRAD_FORWARD) {
    auto kern = a->kkind == PCS_K_GRAD_BACKWARD ? k_pds2d_nmarch_gen<float, H, HK, kNMarchNT, PCS_BACKWARD>
                                                : k_pds2d_nmarch_gen<float, H, HK, kNMarchNT, PCS_CENTERED>;
    kern<<<(unsigned)p.ntasks + fin_extra(a), kNMarchNT, 0, st>>>((const float*)a->x, (float*)a->xn, (const float*)a->z, (float*)a->zn,
                                                   (const float*)a->cty, (const float*)a->ntaps, s, P, a->gkind,
                                                   a->edge, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a),
                                                   p.tiles_x, p.bd, p.ntasks);
    return launch_status();
  }
  if (use_nmarch(a)) {
    k_pds2d_nmarch<float, H, HK, kNMarchNT><<<(unsigned)p.ntasks + fin_extra(a), kNMarchNT, 0, st>>>(
        (const float*)a->x, (float*)a->xn, (const float*)a->z, (float*)a->zn, (const float*)a->cty,
        (const float*)a->ntaps, s, P, a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a), p.tiles_x,
        p.bd, p.ntasks);
    return launch_status();
  }
  if (a->kkind != PCS_K_GRAD_FORWARD) return PCS_EUNSUPPORTED;
  k_pds2d_march<float, H, HK, kMarchNT><<<(unsigned)p.ntasks + fin_extra(a), kMarchNT, 0, st>>>(
      (const float*)a->x, (float*)a->xn, (const float*)a->z, (float*)a->zn, (const float*)a->y,
      (const float*)a->taps0, (const float*)a->taps1, a->half, s, P, a->gkind, a->partials, (Ctrl*)a->ctrl, a->hist,
      a->ws, red_out(a), p.tiles_x, p.bd, p.ntasks);
  return launch_status();
}

template <int H>
static int launch_march_k(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  return a->hkind == PCS_H_L21 ? launch_march_k<H, PCS_H_L21>(a, rb, st) : launch_march_k<H, PCS_H_L1>(a, rb, st);
}

int launch_march(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  return tier_for(a->half) == 3 ? launch_march_k<3>(a, rb, st) : launch_march_k<7>(a, rb, st);
}

}  // namespace pcs
