// Row-marching fused 2-D PDS step for a pointwise grad F (fp32): F = NULL (0), DENOISE
// (grad F = x - y, SquaredL2Loss without an operator) or GRADBUF (grad F precomputed in g).
//
// The march kernel (pds_march.hpp) without its convolution passes: one workgroup owns a
// 64-column strip of a row segment [s0, s1) and steps down it 16 rows at a time.  Step k
// (a = s0 + 16k):
//   top   issue loads: x and y|g on rows [a+1, a+17) (one 4-group + the next column per thread),
//         z0 / z1 rows [a, a+16] -> registers
//   land  z -> Z0 / Z1 (LDS)
//   P45   x_t = prox_G(x - tau grad F - tau K^T z), u = 2 x_t - x on rows [a+1, a+16] and columns
//         [c0, c0+65) -> 17-row u ring; x' on own cells
//   P6    z' = rho fenchel(z + sigma K u) + (1 - rho) z on rows [a, a+16)
// Row s0's u comes from a one-row prologue.  Same arithmetic per pixel as the tile kernel.
// Reference: PrimalDualSplitting.update_iterand (pycsou/opt/proxalgs.py:343-355), grad of
// (1/2) SquaredL2Loss = (2 (x + (-y))) 0.5 (core/map.py:609-610).
#pragma once

#include "pds_march.hpp"

namespace pcs {

// wave priority 3 while a step's loads issue (as pds_nmarch.hpp): C2 29.8-30.1 against
// 30.2-30.4 us per iteration (3 alternating reps, tools/c2_ab.sh); PCS_PT_PRIO=0 drops it
#ifndef PCS_PT_PRIO
#define PCS_PT_PRIO 1
#endif
// cache-policy bits of the per-launch kernel's x' / z' stores (16 = sc1: written through, not left dirty in L2)
// C2 2048^2: 31.4 against 32.3 us per iteration, C3 4096^2: 112.7 against 113.9 us (two alternating
// reps each, profiles/r3_store_policy_ab.txt)
#ifndef PCS_PT_SAUX
#define PCS_PT_SAUX 16
#endif

struct PtGeom {
  static constexpr int TW = 64, TS = 16, UROWS = TS + 1, WG = TW + 4, GG = WG / 4;
  static constexpr int NZ0 = UROWS * GG, NZ1 = UROWS * (GG + 1);
  static constexpr int O_U = 0, SZ_U = UROWS * WG;  // u ring: row r in slot (r - s0) % 17
  static constexpr int O_Z0 = O_U + SZ_U, SZ_Z0 = UROWS * WG;
  static constexpr int O_Z1 = O_Z0 + SZ_Z0, SZ_Z1 = UROWS * (WG + 4);
  static constexpr int SZ = O_Z1 + SZ_Z1;
};

template <int FK, int HK, int SAUX = 0>
__device__ __forceinline__ void pt_task(const float* __restrict__ x, float* __restrict__ xn,
                                        const float* __restrict__ z, float* __restrict__ zn,
                                        const float* __restrict__ gsrc, const Slab32& s, const Params<float>& P, int gk,
                                        int s0, int s1, int c0, float* sm, double (&part)[4]) {
  using T = float;
  using M = PtGeom;
  constexpr int NT = 256, TS = M::TS, TW = M::TW, WG = M::WG, GG = M::GG;
  constexpr int KZ0 = cdiv(M::NZ0, NT), KZ1 = cdiv(M::NZ1, NT);
  T* U = sm + M::O_U;
  T* Z0 = sm + M::O_Z0;
  T* Z1 = sm + M::O_Z1;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hb = tid >> 5, l5 = tid & 31, lgrp = lane_grp(l5), lidx = lane_idx(l5);
  const int n0 = s.n0, n1 = s.n1;
  const int zstride = (s.rows + 2 * s.hz) * n1;
  const View vx = make_view(x, s, s.hx), vz0 = make_view(z, s, s.hz), vz1 = make_view(z + zstride, s, s.hz);
  const View vg = make_view(gsrc != nullptr ? gsrc : x, s, s.hy);
  const uint32_t pitch = (uint32_t)n1 * 4u;
  const Rsrc rxn = rsrc_of(xn, (uint32_t)(s.rows + 2 * s.hx) * pitch);
  const Rsrc rzn0 = rsrc_of(zn, (uint32_t)zstride * 4u), rzn1 = rsrc_of(zn + zstride, (uint32_t)zstride * 4u);
#define PCS_WAVE_ON(k, N) ((k) * NT + wv * 64 < (N))
#define PCS_ITEM(k, N) min((k) * NT + tid, (N) - 1)

  const int ui = 2 * hb + lgrp, ug = lidx;  // P45 / P6: row ui of the step, column group ug
  const int ucg = c0 + 4 * ug;
  // column c + 4 is kept by group 15 only: the other groups' fifth-column loads carry kOOB (no memory
  // request; their fifth column is computed from zeros and dropped).  PCS_PT_E5=0: every group loads it
#ifndef PCS_PT_E5
#define PCS_PT_E5 1
#endif
  const uint32_t co_u = col_off(ucg, n1),
                 co_e = (!PCS_PT_E5 || ug == TW / 4 - 1) ? col_off(ucg + 4, n1) : kOOB;
  uint32_t co_z0[KZ0], co_z1[KZ1];
  int rr_z0[KZ0], rr_z1[KZ1];
  // bit 2: U group in; 3: U column c + 4 in; 4: U group is the last
  const int flags = ((ucg < n1) << 2) | ((ucg + 4 < n1) << 3) | ((ucg == n1 - 4) << 4);
#pragma unroll
  for (int k = 0; k < KZ0; ++k) {
    const int e = PCS_ITEM(k, M::NZ0);
    rr_z0[k] = e / GG;
    co_z0[k] = col_off(c0 + 4 * (e - (e / GG) * GG), n1);
  }
#pragma unroll
  for (int k = 0; k < KZ1; ++k) {
    const int e = PCS_ITEM(k, M::NZ1);
    rr_z1[k] = e / (GG + 1);
    co_z1[k] = col_off(c0 - 4 + 4 * (e - (e / (GG + 1)) * (GG + 1)), n1);
  }
  G4<T> xr, gr, zr0[KZ0], zr1[KZ1];
  T xre = T(0), gre = T(0);
  // loads of step a, in two parts so that each is issued as soon as its registers are free:
  // z rows [a, a + TS] right after the previous step's z landed in LDS, x and y|g on the P45
  // row a + 1 + ui right after the previous step's P45 used them
  auto loads_z = [&](int a) {
#pragma unroll
    for (int k = 0; k < KZ0; ++k) zr0[k] = bload4(vz0.r, vz0.row_off(a + rr_z0[k]) + co_z0[k]);
#pragma unroll
    for (int k = 0; k < KZ1; ++k) zr1[k] = bload4(vz1.r, vz1.row_off(a + rr_z1[k]) + co_z1[k]);
  };
  auto loads_x = [&](int a) {
    const uint32_t ro = vx.row_off(a + 1 + ui);
    xr = bload4(vx.r, ro + co_u);
    xre = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vx.r, (int)(ro + co_e), 0, 0));
    if constexpr (FK != PCS_F_NULL) {
      const uint32_t rg = vg.row_off(a + 1 + ui);
      gr = bload4(vg.r, rg + co_u);
      gre = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vg.r, (int)(rg + co_e), 0, 0));
    }
  };
  auto land_z = [&]() {
#pragma unroll
    for (int k = 0; k < KZ0; ++k)
      if (PCS_WAVE_ON(k, M::NZ0)) st4(Z0 + 4 * PCS_ITEM(k, M::NZ0), zr0[k]);
#pragma unroll
    for (int k = 0; k < KZ1; ++k)
      if (PCS_WAVE_ON(k, M::NZ1)) st4(Z1 + 4 * PCS_ITEM(k, M::NZ1), zr1[k]);
  };
  // ---- P45 on row lr = a + 1 + ui (columns c .. c + 4; column c + 4 is stored by group 15 only)
  auto p45 = [&](int a, int fl, int ub) {
    const int i = ui, g = ug;
    const int lr = a + 1 + i, gr_ = s.row0 + lr;
    int slot = i + 1 + ub;
    slot = slot >= 17 ? slot - 17 : slot;
    const G4<T> za = lds4(Z0 + i * WG + 4 * g);                   // z0[lr - 1]
    const G4<T> zb = lds4(Z0 + (i + 1) * WG + 4 * g);             // z0[lr]
    const G4<T> z1a = lds4(Z1 + (i + 1) * (WG + 4) + 4 * g);      // z1[lr][c - 4 .. c - 1]
    const G4<T> z1b = lds4(Z1 + (i + 1) * (WG + 4) + 4 * g + 4);  // z1[lr][c .. c + 3]
    const T zae = Z0[i * WG + 4 * g + 4], zbe = Z0[(i + 1) * WG + 4 * g + 4];
    const T z1e = Z1[(i + 1) * (WG + 4) + 4 * g + 8];
    const bool r_last = gr_ >= n0 - 1, r_first = gr_ <= 0;
    const bool rrow = gr_ < n0 && lr <= s.rows;
    const bool cin = (fl >> 2) & 1, cin_e = (fl >> 3) & 1, clast = (fl >> 4) & 1;
    const bool own = lr >= s0 && lr < s1 && gr_ < n0 && cin;
    G4<T> uo, xo;
    T ue = T(0), sdx = T(0), sx = T(0);
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const T xv = m < 4 ? xr.v[m] : xre;
      T gd = T(0);
      if constexpr (FK == PCS_F_DENOISE) gd = xv - (m < 4 ? gr.v[m] : gre);  // (2 (x + (-y))) 0.5, exact
      else if constexpr (FK == PCS_F_GRADBUF) gd = m < 4 ? gr.v[m] : gre;
      const T zl = (m == 0) ? z1a.v[3] : z1b.v[m - 1];
      const T zr = m < 4 ? z1b.v[m] : z1e;
      T d0 = r_first ? T(0) : (m < 4 ? za.v[m] : zae);
      if (!r_last) d0 -= (m < 4 ? zb.v[m] : zbe);
      const T d1 = zl - ((m == 3 && clast) ? T(0) : zr);
      const T xt = prox_g((xv - P.tau * gd) - P.tau * (d0 * P.inv_step0 + d1 * P.inv_step1), gk, P.seg_a, P.seg_b);
      const bool in = rrow && (m < 4 ? cin : cin_e);
      const T u = in ? (T(2) * xt - xv) : T(0);
      if (m < 4) {
        uo.v[m] = u;
        const T xnew = P.rho * xt + P.omr * xv;
        xo.v[m] = xnew;
        const T dx = xv - xnew;
        sdx += dx * dx;
        sx += xv * xv;
      } else {
        ue = u;
      }
    }
    if (own) {
      part[0] += (double)sdx;
      part[1] += (double)sx;
    }
    st4(U + slot * WG + 4 * g, uo);
    if (g == TW / 4 - 1) U[slot * WG + TW] = ue;
    bstore4<SAUX>(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_u, xo);
  };
  // ---- P6: z' on row lr = a + ui
  auto p6 = [&](int a, int fl, int ub) {
    const int i = ui, g = ug;
    const int lr = a + i, gr_ = s.row0 + lr;
    int sl0 = i + ub, sl1 = i + 1 + ub;
    sl0 = sl0 >= 17 ? sl0 - 17 : sl0;
    sl1 = sl1 >= 17 ? sl1 - 17 : sl1;
    const G4<T> uc = lds4(U + sl0 * WG + 4 * g);
    const G4<T> ud = lds4(U + sl1 * WG + 4 * g);
    const G4<T> zv0 = lds4(Z0 + i * WG + 4 * g);
    const G4<T> zv1 = lds4(Z1 + i * (WG + 4) + 4 * g + 4);
    const T une = U[sl0 * WG + 4 * g + 4];
    const bool cin = (fl >> 2) & 1, clast = (fl >> 4) & 1;
    const bool r_last = gr_ >= n0 - 1;
    const bool own = lr < s1 && gr_ < n0 && cin;
    G4<T> o0, o1;
    T sdz = T(0), sz = T(0);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const T uright = (m < 3) ? uc.v[m + 1] : une;
      const T d0 = r_last ? T(0) : (ud.v[m] - uc.v[m]);
      const T d1 = (m == 3 && clast) ? T(0) : (uright - uc.v[m]);
      const T w0v = zv0.v[m] + P.sigma * (d0 * P.inv_step0), w1v = zv1.v[m] + P.sigma * (d1 * P.inv_step1);
      const T v0 = w0v * P.inv_sigma, v1 = w1v * P.inv_sigma;
      T zt0, zt1;
      if (HK == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
        T f = T(1) - P.t_h * fast_rsqrt(v0 * v0 + v1 * v1);
        f = f > T(0) ? f : T(0);
        zt0 = w0v - P.sigma * (f * v0);
        zt1 = w1v - P.sigma * (f * v1);
      } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
        zt0 = w0v - P.sigma * (v0 - P.t_h * clip1(v0 * P.inv_t_h));
        zt1 = w1v - P.sigma * (v1 - P.t_h * clip1(v1 * P.inv_t_h));
      }
      o0.v[m] = P.rho * zt0 + P.omr * zv0.v[m];
      o1.v[m] = P.rho * zt1 + P.omr * zv1.v[m];
      const T e0 = zv0.v[m] - o0.v[m], e1 = zv1.v[m] - o1.v[m];
      sdz += e0 * e0 + e1 * e1;
      sz += zv0.v[m] * zv0.v[m] + zv1.v[m] * zv1.v[m];
    }
    if (own) {
      part[2] += (double)sdz;
      part[3] += (double)sz;
    }
    const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_u;
    bstore4<SAUX>(rzn0, off, o0);
    bstore4<SAUX>(rzn1, off, o1);
  };

  // prologue: u on row s0 (step a = s0 - TS, row TS - 1 of its P45), x' on row s0
  const int nsteps = (s1 - s0 + TS - 1) / TS;
  loads_z(s0 - TS);
  loads_x(s0 - TS);
  land_z();
  if (nsteps > 0) loads_z(s0);
  lds_barrier();
  p45(s0 - TS, launder(flags), 1);
  if (nsteps > 0) loads_x(s0);
  int ub = 0;
  for (int k = 0; k < nsteps; ++k) {
    const int a = s0 + k * TS;
    const int fl = launder(flags);
    lds_barrier();  // previous P6 done with Z, U rows
    land_z();
#if PCS_PT_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
    if (k + 1 < nsteps) loads_z(a + TS);  // next step's z flies during this step's P45 and P6
#if PCS_PT_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    lds_barrier();
    p45(a, fl, ub);
#if PCS_PT_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
    if (k + 1 < nsteps) loads_x(a + TS);  // next step's x, y|g during this step's P6
#if PCS_PT_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    lds_barrier();
    p6(a, fl, ub);
    ub = ub == 0 ? 16 : ub - 1;
  }
#undef PCS_WAVE_ON
#undef PCS_ITEM
}

template <int FK, int HK>
__global__ __launch_bounds__(256) void k_pds2d_pt(const float* __restrict__ x, float* __restrict__ xn,
                                                   const float* __restrict__ z, float* __restrict__ zn,
                                                   const float* __restrict__ gsrc, Slab32 s, Params<float> P, int gk,
                                                   double* __restrict__ partials, Ctrl* ctrl, double* hist, void* ws,
                                                   RedOut ro, int tiles_x, Bands bd, int ntasks) {
  __shared__ __attribute__((aligned(16))) float sm[PtGeom::SZ];
  __shared__ double red[4 * 4];
  __shared__ int flag[2];
  if (fin_slot(ro, ntasks, ctrl, hist, red, flag)) return;  // deferred finalization (pds_ctrl.hpp)
  const bool stopped = stop_requested(ctrl, ro, flag);
  if (stopped && ro.sums == nullptr) return;  // loop already stopped (solver.py:65-66)
  int task;
  {  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> adjacent strips of a segment
    const int b = (int)blockIdx.x - fin_shift(ro), q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int seg = task / tiles_x, strip = task - seg * tiles_x;
  int s0, s1;
  band_rows(bd, seg, s0, s1);
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (!stopped) pt_task<FK, HK, PCS_PT_SAUX>(x, xn, z, zn, gsrc, s, P, gk, s0, s1, strip * PtGeom::TW, sm, part);
  block_sum<4>(part, red);
  publish_partials(part, partials, ntasks, ws, ctrl, hist, flag, ro);
}

}  // namespace pcs
