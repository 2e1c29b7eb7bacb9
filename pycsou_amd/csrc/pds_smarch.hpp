// Row-marching fused 2-D PDS step for a GENERAL finite-difference K (fp32 / fp64, pointwise grad F):
//   K = Gradient(kind = 'backward' | 'centered' | 'forward', edge, sampling)   (pycsou/linop/diff.py:777-882;
//       'centered' is the reference's default), z = [D0 x; D1 x]
//   K = Laplacian(weights, sampling, edge) = w0 D2_0 + w1 D2_1                (diff.py:885-957), z = K x
// F = NULL (0), DENOISE (grad F = x - y), GRADBUF (grad F read from g) or, for a separable blur,
// grad F = N x - Conv^T y with N x from a buffer (SM_F_NB, below), H = lam L1 / lam L21.
// PrimalDualSplitting.update_iterand / update_diagnostics (pycsou/opt/proxalgs.py:343-394):
//   x_t = prox_G((x - tau grad F) - tau K^T z),  u = 2 x_t - x,  x' = rho x_t + (1 - rho) x
//   z'  = rho H.fenchel_prox(z + sigma K u, sigma) + (1 - rho) z
//
// The forward-Gradient row march (pds_pt.hpp) generalised to stencils that reach one sample
// both ways (two at the image edges for the Laplacian's one-sided rows).  One workgroup
// (256 threads: 4 rows x 16 four-column groups per wave) owns a 64-column strip of a row segment
// [s0, s1) and marches down it 16 rows per step (a = s0 + 16 k):
//   top   land z rows [a + ZHI - 15, a + ZHI] (loaded during the previous step) in the z ring;
//         issue the next step's z loads
//   U     rows [a+1, a+16]: K^T z from the z ring, x_t, u -> u ring, x' -> HBM.  Every item also
//         computes a fifth column: c0 - 1 (group 0) or c + 4 (the rest; group 15's is c0 + 64),
//         the u columns K u of the strip's edge columns reaches
//   Z     rows [a, a+16): K u from the u ring, fenchel prox, relaxation, z' -> HBM
// The next step's x and y|g load at the top of the step too, into the second of two register
// sets (the march is unrolled by two steps), so every load has a whole step to land.
// z and u live in 32-row LDS rings (row r in slot r & 31; columns [c0 - 4, c0 + 68)), so every
// z row is read from HBM once per strip, every u row computed once; x and y|g are read once.
// HBM traffic per pixel: x, y|g, z (D components) in; x', z' out -- (3 + 2 D) words when F reads
// a buffer (7 for the gradients, 5 for the Laplacian), plus the strips' 4-column halos of z.
// A one-row-deep prologue (rows s0 - 2 .. s0 of u, masked loads) starts each segment.
// Per element the stencils are stencil.hpp's (same operation order), 1/h applied as a
// multiplication (exact for unit sampling).  Global accesses go through buffer descriptors
// (hardware range check: rows / columns outside the image or the stored slab read 0).
#pragma once

#include <type_traits>

#include "pds_march.hpp"
#include "stencil.hpp"

namespace pcs {

// cache-policy bits of the x' / z' stores: 16 = sc1 (written through, not left dirty in L2):
// 2048^2 30.5-30.6 against 31.9-32.0 us per iteration back to back with plain stores, nt (2)
// 30.9 / 34.7 (tools/sm_probe.py, profiles/r3_sm_store_policy.jsonl); diagnostics builds override
#ifndef PCS_SM_SAUX
#define PCS_SM_SAUX 16
#endif
// fp64: a 4-column group is two 16-B stores 16 B apart, so each store instruction covers every other
// 16-B chunk of the wave's span; written through (sc1) those halves leave as partial lines -- PMC
// WRITE_SIZE 2.0x the bytes (profiles/r4_prof_c3f64_*) -- so fp64 stores are plain (L2 merges the halves)
#ifndef PCS_SM_SAUX64
#define PCS_SM_SAUX64 0
#endif

// waves per SIMD the register budget targets (diagnostics builds override; 1 = no constraint)
#ifndef PCS_SM_WPE
#define PCS_SM_WPE 1
#endif

// wave priority 3 while a step's loads issue (as pds_pt.hpp); PCS_SM_PRIO=0 (diagnostics) drops it
#ifndef PCS_SM_PRIO
#define PCS_SM_PRIO 1
#endif

enum { SK_LAP = 3 };  // KK: PCS_FORWARD / PCS_BACKWARD / PCS_CENTERED (2 components) or the Laplacian (1)
// FK beyond the public kinds: grad F = g - b with g = N x = Conv^T Conv x from a buffer (the in-plane
// normal-operator kernel, pcs_conv2d_sep_ata_planes) and b = Conv^T y (formed once per problem);
// SM_F_MASK: F = 0 and a masked data-fidelity block in K / H (below)
enum { SM_F_NB = 16, SM_F_MASK = 32 };

// SM_F_MASK: K = LinOpVStack(Masking, K_s), H = ProxFuncHStack(L1Loss(y), lam * L1 | L21) -- the reference
// notebook's TV-LAD inpainting (pycsou/linop/base.py:159-279, func/base.py:21-89, func/loss.py:222-268,
// solved by ChambollePockSplitting, opt/proxalgs.py:628-716).  The masked dual block z_m is held expanded
// to the image (0 where the mask is False), y expanded with NaN where the mask is False (gsrc), so the
// block is pointwise and lives in the U phase alone:
//   K^T z = (0 + M^T z_m) + K_s^T z_s                        (LinOpStack.adjoint accumulation order)
//   z_m'  = w - sigma ((prox_l1(w / sigma - y, 1 / sigma)) + y),  w = z_m + sigma u   (masked pixels)
// (ProximableFunctional.fenchel_prox of the stack, core/functional.py:176-207, with the L1Loss prox
// ProxFuncPreComp(L1Norm, 1, -y): prox_l1(v + (-y), tau) - (-y)).  msrc / mdst: z_m in / out.

// the stencils on a 5-sample window: stencil.hpp (sw_d1_fwd / sw_d1_adj / sw_d2_fwd / sw_d2_adj)

// stencil-specific parameters (the rest is Params<T>)
template <typename T>
struct SParamsT {
  T ih20, ih21, w0, w1;  // 1 / sampling^2 per axis, Laplacian weights
  int edge;
};
using SParams = SParamsT<float>;

// 16-row steps, 32-row rings (32-row steps with 64-row rings measured no faster at 2048^2 and slower at
// 4096^2, profiles/r4_sm_rs_ab.txt; z rows landed with the segment prologue's, profiles/r3_ck44_ze_ab.txt:
// no change -- both removed in round 5)
template <int KK>
struct SMarch {
  static constexpr int TW = 64, TS = 16, D = KK == SK_LAP ? 1 : 2;
  // z rows [a + ZLO, a + ZHI] feed step a (U rows a+1..a+16 reach ZR rows up, ZD down; the Z
  // rows a..a+15 read their own z)
  static constexpr int ZHI = KK == SK_LAP ? 18 : KK == PCS_FORWARD ? 16 : 17;
  // rows of u above a segment the first Z rows read (the prologue computes them) and the z rows
  // above those that u needs
  static constexpr int UPRO = KK == SK_LAP ? 2 : 1, ZPRO = UPRO + (KK == SK_LAP ? 2 : 1);
  // u / z windows along axis 0 (offsets -2..+2 from the row): which rows each phase reads
  static constexpr bool UWIN(int k) {  // U phase: z rows r - 2 + k
    return KK == SK_LAP ? true : KK == PCS_FORWARD ? (k == 1 || k == 2) : KK == PCS_BACKWARD ? (k == 2 || k == 3)
                                                                                             : (k >= 1 && k <= 3);
  }
  static constexpr bool ZWIN(int k) {  // Z phase: u rows r - 2 + k
    return KK == SK_LAP ? true : KK == PCS_FORWARD ? (k == 2 || k == 3) : KK == PCS_BACKWARD ? (k == 1 || k == 2)
                                                                                             : (k >= 1 && k <= 3);
  }
  // K u reaches left / right along axis 1 (the neighbour groups the Z phase reads; the U phase
  // reads both, its fifth column lying on either side)
  static constexpr bool Z_L = KK != PCS_FORWARD, Z_R = KK != PCS_BACKWARD;  // u[c-1] / u[c+1]
  static constexpr int RING = 32, WZ = TW + 12, GZ = 18;  // ring rows of columns [c0 - 4, c0 + 68) (+ pad: 19 slots)
  static constexpr int RM = RING - 1;
  static constexpr int NZN = TS * GZ;                     // z items per component per step
  static constexpr int O_Z = 0, O_U = D * RING * WZ, SZ = O_U + RING * WZ;
};

// T = float or double: the same geometry (4-column groups, 64-column strips, 16-row steps); an fp64
// group is two 16-B accesses and the rings take twice the LDS (58 KB for a Gradient K)
template <typename T, int KK, int FK, int HK, bool CI>
__device__ __forceinline__ void smarch_task(const T* __restrict__ x, T* __restrict__ xn,
                                            const T* __restrict__ z, T* __restrict__ zn,
                                            const T* __restrict__ gsrc, const T* __restrict__ bsrc,
                                            const T* __restrict__ msrc, T* __restrict__ mdst,
                                            const Slab32& s, const Params<T>& P,
                                            const SParamsT<T>& Q, int gk, int s0, int s1, int c0, T* sm,
                                            double (&part)[4], int stop_raw) {
  constexpr uint32_t ES = sizeof(T);
  constexpr int SAUX = sizeof(T) == 4 ? PCS_SM_SAUX : PCS_SM_SAUX64;
  using M = SMarch<KK>;
  constexpr int NT = 256, TS = M::TS, TW = M::TW, WZ = M::WZ, GZ = M::GZ, D = M::D, RING = M::RING, RM = M::RM;
  constexpr int KZ = cdiv(M::NZN, NT);
  T* ZR = sm + M::O_Z;  // component d, row r: ZR + d * RING * WZ + (r & RM) * WZ; column c at c - c0 + 4
  T* UR = sm + M::O_U;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hb = tid >> 5, l5 = tid & 31;
  const int ui = 2 * hb + lane_grp(l5), ug = lane_idx(l5);  // both phases: row ui of the step, group ug
  const int n0 = s.n0, n1 = s.n1, edge = Q.edge;
  const int zstride = (s.rows + 2 * s.hz) * n1;
  const View vx = make_view(x, s, s.hx, ES), vg = make_view(gsrc != nullptr ? gsrc : x, s, s.hy, ES),
             vb = make_view(bsrc != nullptr ? bsrc : x, s, s.hy, ES),
             vm = make_view(msrc != nullptr ? msrc : x, s, s.hx, ES);
  View vz[D];
#pragma unroll
  for (int d = 0; d < D; ++d) vz[d] = make_view(z + d * zstride, s, s.hz, ES);
  const uint32_t pitch = (uint32_t)n1 * ES;
  const Rsrc rxn = rsrc_of(xn, (uint32_t)(s.rows + 2 * s.hx) * pitch);
  const Rsrc rmn = rsrc_of(mdst != nullptr ? mdst : xn, FK == SM_F_MASK ? (uint32_t)(s.rows + 2 * s.hx) * pitch : 0u);
  Rsrc rzn[D];
#pragma unroll
  for (int d = 0; d < D; ++d) rzn[d] = rsrc_of(zn + d * zstride, (uint32_t)zstride * ES);
#define PCS_WAVE_ON(k, N) ((k) * NT + wv * 64 < (N))
#define PCS_ITEM(k, N) min((k) * NT + tid, (N) - 1)

  // rings start zeroed: the columns no item writes (c0 - 4 .. c0 - 2, c0 + 65 ..) read as 0
  {
    const G4<T> zero = {{T(0), T(0), T(0), T(0)}};
    for (int i = tid; i < M::SZ / 4; i += NT) st4(sm + 4 * i, zero);
  }
  const int c = c0 + 4 * ug;
  const int ce = ug == 0 ? c - 1 : c + 4;             // the item's fifth column
  const int lc = 4 + 4 * ug, lce = ug == 0 ? 3 : lc + 4;  // their ring columns
  const bool ext_st = ug == 0 || ug == TW / 4 - 1;   // fifth columns K u reads: c0 - 1, c0 + 64
  // only groups 0 and 15 keep their fifth column: the others' fifth-column loads carry kOOB (no memory
  // request; computed from zeros, never stored).  PCS_SM_E5=0: every group loads it
#ifndef PCS_SM_E5
#define PCS_SM_E5 1
#endif
  const uint32_t co_c = col_off(c, n1, ES), co_e = (!PCS_SM_E5 || ext_st) ? col_off(ce, n1, ES) : kOOB;
  // CI: the strip and its 4-column margins lie >= 2 columns inside the image (no column edge rule)
  const bool cin = CI || c < n1, ce_in = CI || (unsigned)ce < (unsigned)n1;
  uint32_t co_z[KZ];
  int rr_z[KZ], lo_z[KZ];
#pragma unroll
  for (int k = 0; k < KZ; ++k) {
    const int e = PCS_ITEM(k, M::NZN), g = e - (e / GZ) * GZ;
    rr_z[k] = e / GZ;
    lo_z[k] = 4 * g;
    co_z[k] = col_off(c0 - 4 + 4 * g, n1, ES);
  }
  // x, y|g (and b) of the U items in two register sets: the set of step k + 1 loads at the top of
  // step k, a whole step before the U phase that reads it (PB: the set, a compile-time index)
  G4<T> zr[D][KZ], xr[2], gr[2], br[2], mr[2];
  T xe[2], ge[2], be[2], me[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) xe[i] = ge[i] = be[i] = me[i] = T(0);
  // z rows [a + ZHI - 15, a + ZHI] (rows below rmin read as 0)
  auto loads_z = [&](int a, int rmin) {
    auto& dst = zr;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int k = 0; k < KZ; ++k) {
        const int r = a + M::ZHI - 15 + rr_z[k];
        dst[d][k] = bload4t<T>(vz[d].r, (r < rmin ? kOOB : vz[d].row_off(r)) + co_z[k]);
      }
  };
  auto land_z = [&](int a) {
    const auto& src = zr;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int k = 0; k < KZ; ++k)
        if (PCS_WAVE_ON(k, M::NZN))
          st4(ZR + d * RING * WZ + ((a + M::ZHI - 15 + rr_z[k]) & RM) * WZ + lo_z[k], src[d][k]);
  };
  // x and y|g of U row a + 1 + ui: the group and the fifth column (PB: the register set)
  auto loads_x = [&](auto pb, int a, int rmin) {
    constexpr int PB = decltype(pb)::value;
    const int r = a + 1 + ui;
    const uint32_t ro = r < rmin ? kOOB : vx.row_off(r);
    xr[PB] = bload4t<T>(vx.r, ro + co_c);
    xe[PB] = bload1t<T>(vx.r, ro + co_e);
    if constexpr (FK == SM_F_MASK) {  // y (NaN = unmasked) on the own columns; z_m on both
      const uint32_t rg = r < rmin ? kOOB : vg.row_off(r);
      gr[PB] = bload4t<T>(vg.r, rg + co_c);
      const uint32_t rm = r < rmin ? kOOB : vm.row_off(r);
      mr[PB] = bload4t<T>(vm.r, rm + co_c);
      me[PB] = bload1t<T>(vm.r, rm + co_e);
    } else if constexpr (FK != PCS_F_NULL) {
      const uint32_t rg = r < rmin ? kOOB : vg.row_off(r);
      gr[PB] = bload4t<T>(vg.r, rg + co_c);
      ge[PB] = bload1t<T>(vg.r, rg + co_e);
    }
    if constexpr (FK == SM_F_NB) {
      const uint32_t rb = r < rmin ? kOOB : vb.row_off(r);
      br[PB] = bload4t<T>(vb.r, rb + co_c);
      be[PB] = bload1t<T>(vb.r, rb + co_e);
    }
  };

  // ---- U: x_t, u on row lr = a + 1 + ui, columns c .. c + 3 and ce; x' on own cells
  // RI (std::true_type / false_type): every row of the step lies >= 2 rows inside the image
  auto uphase = [&](auto ri, auto pb, int a) {
    constexpr bool RI = decltype(ri)::value;
    constexpr int PB = decltype(pb)::value;
    const int lr = a + 1 + ui, gr_ = s.row0 + lr;
    const T* Z0 = ZR;
    const T* Z1 = ZR + (D - 1) * RING * WZ;  // the axis-1 component (the Laplacian's only one)
    G4<T> v0[5];
    T ve[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const T* row = Z0 + ((lr - 2 + k) & RM) * WZ;
      if (M::UWIN(k)) {
        v0[k] = lds4(row + lc);
        ve[k] = row[lce];
      } else {
        v0[k] = G4<T>{{T(0), T(0), T(0), T(0)}};
        ve[k] = T(0);
      }
    }
    const T* hrow = Z1 + (lr & RM) * WZ;
    const G4<T> hl = lds4(hrow + lc - 4);
    const G4<T> hc = D == 2 ? lds4(hrow + lc) : v0[2];
    const G4<T> hr = lds4(hrow + lc + 4);
    const T hv[12] = {hl.v[0], hl.v[1], hl.v[2], hl.v[3], hc.v[0], hc.v[1],
                      hc.v[2], hc.v[3], hr.v[0], hr.v[1], hr.v[2], hr.v[3]};
    const bool rrow = RI || (unsigned)gr_ < (unsigned)n0;
    const bool own = lr >= s0 && lr < s1 && rrow && cin;
    G4<T> uo, xo, mo;
    T ue = T(0), sdx = T(0), sx = T(0), sdm = T(0), sm2 = T(0);
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int i1 = m < 4 ? c + m : ce;
      T w0[5], w1[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        w0[k] = m < 4 ? v0[k].v[m] : ve[k];
        w1[k] = m < 4 ? hv[2 + m + k] : (ug == 0 ? hv[1 + k] : hv[6 + k]);
      }
      T kt;
      if constexpr (KK == SK_LAP) {
        kt = pcs_fma(Q.w0 * Q.ih20, sw_d2_adj<RI>(w0, gr_, n0, edge), (Q.w1 * Q.ih21) * sw_d2_adj<CI>(w1, i1, n1, edge));
      } else {  // VStack rmatvec: D0^T z0 + D1^T z1
        kt = pcs_fma(sw_d1_adj<KK, RI>(w0, gr_, n0, edge), P.inv_step0,
                    sw_d1_adj<KK, CI>(w1, i1, n1, edge) * P.inv_step1);
      }
      if constexpr (FK == SM_F_MASK) kt = (m < 4 ? mr[PB].v[m] : me[PB]) + kt;  // (0 + M^T z_m) + K_s^T z_s
      const T xv = m < 4 ? xr[PB].v[m] : xe[PB];
      T gf = T(0);
      if constexpr (FK == PCS_F_DENOISE) gf = xv - (m < 4 ? gr[PB].v[m] : ge[PB]);  // (2 (x + (-y))) 0.5, exact
      else if constexpr (FK == PCS_F_GRADBUF) gf = m < 4 ? gr[PB].v[m] : ge[PB];
      else if constexpr (FK == SM_F_NB) gf = (m < 4 ? gr[PB].v[m] : ge[PB]) - (m < 4 ? br[PB].v[m] : be[PB]);
      const T xt = prox_g((xv - P.tau * gf) - P.tau * kt, gk, P.seg_a, P.seg_b);
      const bool in = rrow && (m < 4 ? cin : ce_in);
      const T u = in ? (T(2) * xt - xv) : T(0);
      if (m < 4) {
        uo.v[m] = u;
        const T xnew = pcs_fma(P.rho, xt, P.omr * xv);
        xo.v[m] = xnew;
        const T dx = xv - xnew;
        sdx += dx * dx;
        sx += xv * xv;
        if constexpr (FK == SM_F_MASK) {  // the masked block's z_m', pointwise (K u = M u here)
          const T yv = gr[PB].v[m], zmv = mr[PB].v[m];
          const T w = zmv + P.sigma * u;
          const T a = w * P.inv_sigma + (-yv);  // ProxFuncPreComp: v + (-y)
          const T pl = a - P.inv_sigma * clip1(a * P.sigma);  // prox_l1(a, 1 / sigma)
          const T zt = w - P.sigma * (pl - (-yv));
          const T zo = (yv == yv) ? pcs_fma(P.rho, zt, P.omr * zmv) : T(0);  // NaN y: not sampled
          mo.v[m] = zo;
          const T dm = zmv - zo;
          sdm += dm * dm;
          sm2 += zmv * zmv;
        }
      } else {
        ue = u;
      }
    }
    if (own) {
      part[0] += (double)sdx;
      part[1] += (double)sx;
      if constexpr (FK == SM_F_MASK) {
        part[2] += (double)sdm;
        part[3] += (double)sm2;
      }
    }
    if constexpr (FK == SM_F_MASK) bstore4t<T, SAUX>(rmn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_c, mo);
    T* urow = UR + (lr & RM) * WZ;
    st4(urow + lc, uo);
    if (ext_st) urow[lce] = ue;
    bstore4t<T, SAUX>(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_c, xo);
  };

  // ---- Z: z' on row lr = a + ui, columns c .. c + 3
  auto zphase = [&](auto ri, int a) {
    constexpr bool RI = decltype(ri)::value;
    const int lr = a + ui, gr_ = s.row0 + lr;
    G4<T> v0[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      v0[k] = M::ZWIN(k) ? lds4(UR + ((lr - 2 + k) & RM) * WZ + lc) : G4<T>{{T(0), T(0), T(0), T(0)}};
    const T* hrow = UR + (lr & RM) * WZ;
    const G4<T> zero = {{T(0), T(0), T(0), T(0)}};
    const G4<T> hl = M::Z_L ? lds4(hrow + lc - 4) : zero;
    const G4<T> hc = v0[2];
    const G4<T> hr = M::Z_R ? lds4(hrow + lc + 4) : zero;
    const T hv[12] = {hl.v[0], hl.v[1], hl.v[2], hl.v[3], hc.v[0], hc.v[1],
                      hc.v[2], hc.v[3], hr.v[0], hr.v[1], hr.v[2], hr.v[3]};
    G4<T> zv[D];
#pragma unroll
    for (int d = 0; d < D; ++d) zv[d] = lds4(ZR + d * RING * WZ + (lr & RM) * WZ + lc);
    const bool own = lr >= s0 && lr < s1 && (RI || (unsigned)gr_ < (unsigned)n0) && cin;
    G4<T> o[D];
    T sdz = T(0), sz = T(0);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int i1 = c + m;
      T w0[5], w1[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        w0[k] = v0[k].v[m];
        w1[k] = hv[2 + m + k];
      }
      T ku[D];
      if constexpr (KK == SK_LAP) {  // w0 D2_0 u + w1 D2_1 u (pylops Laplacian matvec)
        ku[0] = pcs_fma(Q.w0, sw_d2_fwd<RI>(w0, gr_, n0, Q.ih20, edge), Q.w1 * sw_d2_fwd<CI>(w1, i1, n1, Q.ih21, edge));
      } else {
        ku[0] = sw_d1_fwd<KK, RI>(w0, gr_, n0, P.inv_step0, edge);
        ku[D - 1] = sw_d1_fwd<KK, CI>(w1, i1, n1, P.inv_step1, edge);
      }
      T w[D], v[D], zt[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        w[d] = zv[d].v[m] + P.sigma * ku[d];
        v[d] = w[d] * P.inv_sigma;
      }
      if constexpr (D == 2 && HK == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
        T f = T(1) - P.t_h * fast_rsqrt(pcs_fma(v[0], v[0], v[D - 1] * v[D - 1]));
        f = f > T(0) ? f : T(0);
#pragma unroll
        for (int d = 0; d < D; ++d) zt[d] = w[d] - P.sigma * (f * v[d]);
      } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
#pragma unroll
        for (int d = 0; d < D; ++d) zt[d] = w[d] - P.sigma * (v[d] - P.t_h * clip1(v[d] * P.inv_t_h));
      }
#pragma unroll
      for (int d = 0; d < D; ++d) {
        o[d].v[m] = pcs_fma(P.rho, zt[d], P.omr * zv[d].v[m]);
        const T ed = zv[d].v[m] - o[d].v[m];
        sdz += ed * ed;
        sz += zv[d].v[m] * zv[d].v[m];
      }
    }
    if (own) {
      part[2] += (double)sdz;
      part[3] += (double)sz;
    }
    const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_c;
#pragma unroll
    for (int d = 0; d < D; ++d) bstore4t<T, SAUX>(rzn[d], off, o[d]);
  };

  // prologue: u on rows [s0 - UPRO, s0] (a 16-row pseudo-step at a = s0 - TS whose loads skip the
  // rows it does not need, register set 0 half 0), x' on row s0
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  const int nsteps = (s1 - s0 + TS - 1) / TS;
  loads_z(s0 - TS, s0 - M::ZPRO);
  loads_x(P0{}, s0 - TS, s0 - M::UPRO);
  lds_barrier();  // rings zeroed
  land_z(s0 - TS);
  if (nsteps > 0) {
    loads_z(s0, -(1 << 30));
    loads_x(P1{}, s0, -(1 << 30));
  }
  if (stop_raw) return;  // loop already stopped (solver.py:65-66): loads issued, nothing stored
  lds_barrier();
  uphase(std::false_type{}, P0{}, s0 - TS);
  // step k reads register set PB = (k + 1) & 1 and loads the other one for step k + 1
  auto step = [&](auto pb, int k) {
    constexpr int PB = decltype(pb)::value;
    const int a = s0 + k * TS;
    // rows [a, a + 16] at >= 2 rows from both image edges (uniform)
    const bool ri = s.row0 + a >= 2 && s.row0 + a + TS + 3 <= n0;
    lds_barrier();  // the previous step's Z phase is done with the rings
    land_z(a);
    if (PCS_SM_PRIO) __builtin_amdgcn_s_setprio(3);  // the step's loads issue ahead of other waves' VALU
    if (k + 1 < nsteps) {
      loads_z(a + TS, -(1 << 30));
      loads_x(std::integral_constant<int, 1 - PB>{}, a + TS, -(1 << 30));
    }
    if (PCS_SM_PRIO) __builtin_amdgcn_s_setprio(0);
    lds_barrier();
    // U reads only the z ring; the Z rows read u rows up to their last row + 1 (+ 2 on the image's
    // first row only), all written by this step's U phase or earlier
    if (ri) uphase(std::true_type{}, pb, a);
    else uphase(std::false_type{}, pb, a);
    lds_barrier();
    if (ri) zphase(std::true_type{}, a);
    else zphase(std::false_type{}, a);
  };
  for (int k = 0; k < nsteps; k += 2) {
    step(P1{}, k);
    if (k + 1 < nsteps) step(P0{}, k + 1);
  }
#undef PCS_WAVE_ON
#undef PCS_ITEM
}

template <typename T, int KK, int FK, int HK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PCS_SM_WPE))) void k_pds2d_smarch(const T* __restrict__ x, T* __restrict__ xn,
                                                       const T* __restrict__ z, T* __restrict__ zn,
                                                       const T* __restrict__ gsrc,
                                                       const T* __restrict__ bsrc, const T* __restrict__ msrc,
                                                       T* __restrict__ mdst, Slab32 s, Params<T> P,
                                                       SParamsT<T> Q, int gk, double* __restrict__ partials, Ctrl* ctrl,
                                                       double* hist, void* ws, RedOut ro, int tiles_x, Bands bd,
                                                       int ntasks, StripSplit sp) {
  __shared__ __attribute__((aligned(16))) T sm[SMarch<KK>::SZ];
  __shared__ double red[4 * 4];
  __shared__ int flag[2];
  if (fin_slot(ro, ntasks, ctrl, hist, red, flag)) return;  // deferred finalization (pds_ctrl.hpp)
  const int stop_raw = stop_flag_early(ctrl, ro);  // consumed in the task (PCS_DEFER_STOP)
  const bool stopped = !stop_deferred(ro) && stop_requested(ctrl, ro, flag);
  if (stopped && ro.sums == nullptr) return;  // loop already stopped (solver.py:65-66)
  int task;
  {  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> adjacent strips of a segment
    const int b = (int)blockIdx.x - fin_shift(ro), q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  int strip, s0, s1;
  if (sp.nint < 0) {  // one segmentation for every strip
    const int seg = task / tiles_x;
    strip = task - seg * tiles_x;
    band_rows(bd, seg, s0, s1);
  } else if (task < sp.nint) {  // interior strips
    const int seg = task / sp.iw;
    strip = sp.ilo + task - seg * sp.iw;
    band_rows(bd, seg, s0, s1);
  } else {  // border strips, shorter segments
    const int b = task - sp.nint, seg = b / sp.nbs, j = b - seg * sp.nbs;
    strip = j == 0 ? sp.bs[0] : (j == 1 ? sp.bs[1] : sp.bs[2]);
    band_rows(sp.bdb, seg, s0, s1);
  }
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  const int c0 = strip * SMarch<KK>::TW;
  if (!stopped) {
#ifndef PCS_SM_ALLCI  // diagnostics (timing only, wrong border columns): every strip on the interior form
#define PCS_SM_ALLCI 0
#endif
    if (PCS_SM_ALLCI || (c0 >= 4 && c0 + SMarch<KK>::TW + 6 <= s.n1))  // columns [c0 - 2, c0 + 66) >= 2 inside: no column edge rule
      smarch_task<T, KK, FK, HK, true>(x, xn, z, zn, gsrc, bsrc, msrc, mdst, s, P, Q, gk, s0, s1, c0, sm, part,
                                           stop_raw);
    else
      smarch_task<T, KK, FK, HK, false>(x, xn, z, zn, gsrc, bsrc, msrc, mdst, s, P, Q, gk, s0, s1, c0, sm, part,
                                            stop_raw);
  }
  if (stop_raw) return;  // the task returned before any store
  block_sum<4>(part, red);
  publish_partials(part, partials, ntasks, ws, ctrl, hist, flag, ro);
}

}  // namespace pcs
