// Tile kernel of the fused 2-D PDS iteration (see pds.hip for the algorithm map).
//
// One workgroup = one TH x 64 output tile.  With forward differences, z' on the tile
// needs u = 2 x_t - x on the tile plus one row below and one column to the right (the
// "U region", HG x WG); x_t there needs grad F and K^T z.
//   X  = x on the U region grown by 2H rows / 2*RU4(H) cols      (HBM -> regs -> LDS)
//   A  = row-conv(X)               forward blur along axis 1      (P1)
//   R  = col-conv(A) - y, 0 outside the image (residual h*x - y)  (P2)
//   B  = col-corr(R)               adjoint blur along axis 0      (P3)
//   Gd = row-corr(B) = Conv^T r  = grad F on the U region         (P4)
//   x_t, u on the U region (U in LDS); x' on the tile -> HBM      (P5)
//   z' = rho * fenchel(z + sigma K u) + (1-rho) z on the tile     (P6)
// MI355X specifics:
//  * every global access is a 16-B-per-lane group load issued in one batch (X and the
//    P2 residual's y at entry; z, x (and y/g) for the update right after X lands), so
//    each wave keeps 5-10 loads in flight; z lands in LDS (reused buffers) so K^T z and
//    K u neighbour reads are LDS reads;
//  * tiles whose whole footprint is inside the image take an `interior` instantiation
//    with no bounds logic (uniform branch per workgroup);
//  * LDS passes work on 4-wide column groups (16-B ds_read_b128 per lane); row passes
//    walk items column-major over odd slot pitches (25/21/17 slots) so the 16 lanes of
//    every b128 lane group hit 16 distinct 16-B slots: conflict-free;
//  * no divisions in the inner update: 1/h, 1/sigma, 1/t are precomputed, unit steps
//    skip the scaling (exact), the L21 group norm uses rsqrt.
#pragma once

#include "common.hpp"
#include "pds_ctrl.hpp"

// Diagnostics only: bit k skips phase k (0 P1, 1 P2, 2 P3, 3 P4, 4 P5, 5 P6, 6 X->LDS,
// 7 z->LDS) so rocprof counters can be attributed to phases.  Results are wrong.
#ifndef PCS_ABLATE
#define PCS_ABLATE 0
#endif
#define PCS_ON(bit) (!(PCS_ABLATE & (1 << (bit))))

namespace pcs {

template <int V>
struct RU4 {
  static constexpr int value = (V + 3) / 4 * 4;
};
constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <typename T>
struct G4 {
  T v[4];
};

template <typename T>
__device__ __forceinline__ G4<T> ld4(const T* p);
template <>
__device__ __forceinline__ G4<float> ld4<float>(const float* p) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  return {{q.x, q.y, q.z, q.w}};
}
template <>
__device__ __forceinline__ G4<double> ld4<double>(const double* p) {
  const double2 a = reinterpret_cast<const double2*>(p)[0];
  const double2 b = reinterpret_cast<const double2*>(p)[1];
  return {{a.x, a.y, b.x, b.y}};
}
// LDS group read that stays ONE ds_read_b128: without `volatile` hipcc narrows a
// 16-B read whose first/last element is unused into ds_read2_b32 pairs at odd offsets
// (2-4 way bank conflicts).
template <typename T>
__device__ __forceinline__ G4<T> lds4(const T* p);
template <>
__device__ __forceinline__ G4<float> lds4<float>(const float* p) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const volatile f4* lds_f4;
  const f4 q = *(lds_f4)(p);
  return {{q.x, q.y, q.z, q.w}};
}
template <>
__device__ __forceinline__ G4<double> lds4<double>(const double* p) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const volatile d2* lds_d2;
  const d2 a = ((lds_d2)(p))[0];
  const d2 b = ((lds_d2)(p))[1];
  return {{a.x, a.y, b.x, b.y}};
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const G4<T>& g);
template <>
__device__ __forceinline__ void st4<float>(float* p, const G4<float>& g) {
  *reinterpret_cast<float4*>(p) = make_float4(g.v[0], g.v[1], g.v[2], g.v[3]);
}
template <>
__device__ __forceinline__ void st4<double>(double* p, const G4<double>& g) {
  reinterpret_cast<double2*>(p)[0] = make_double2(g.v[0], g.v[1]);
  reinterpret_cast<double2*>(p)[1] = make_double2(g.v[2], g.v[3]);
}

// Slab geometry: local arrays hold rows [row0 - halo, row0 + rows + halo) of the n0 x n1 image.
struct Slab {
  int64_t n0, n1, row0, rows;
  int hx, hy, hz;  // halo rows stored in x/xn, y/gbuf, z/zn
  int vec;         // n1 % 4 == 0 and 16-B aligned bases: 4-groups are whole-in or whole-out
};

// 4 consecutive columns [c, c+4) of local row lr; zeros outside the image / stored rows.
template <typename T, bool INT>
__device__ __forceinline__ G4<T> gload4(const T* __restrict__ a, const Slab& s, int halo, int64_t lr, int64_t c) {
  if (INT) return ld4(a + (lr + halo) * s.n1 + c);
  G4<T> g = {{T(0), T(0), T(0), T(0)}};
  const int64_t gr = s.row0 + lr;
  if (gr < 0 || gr >= s.n0 || lr < -halo || lr >= s.rows + halo) return g;
  const T* row = a + (lr + halo) * s.n1;
  if (s.vec) {
    if (c >= 0 && c + 3 < s.n1) g = ld4(row + c);
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (c + m >= 0 && c + m < s.n1) g.v[m] = row[c + m];
  }
  return g;
}

// ---------------------------------------------------------------- LDS passes
// Row pass: out[r][j] = sum_t w[t'] in[r][j + SH + t] (t' = REV ? 2H-t : t), 4-groups,
// items column-major (consecutive lanes -> consecutive rows of one group).
template <typename T, int H, bool REV, int NT>
__device__ __forceinline__ void row_pass(const T* __restrict__ in, int pin, T* __restrict__ out, int pout, int rows,
                                         int ngroups, const T (&w)[2 * H + 1]) {
  constexpr int H4 = RU4<H>::value;
  constexpr int NV = 1 + H4 / 2;
  constexpr int SH = H4 - H;
  const int items = rows * ngroups;
  for (int it = threadIdx.x; it < items; it += NT) {
    const int g = it / rows, r = it - g * rows;
    T v[4 * NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const G4<T> t4 = lds4(in + r * pin + 4 * g + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = t4.v[e];
    }
    G4<T> o;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T acc = T(0);
#pragma unroll
      for (int t = 0; t < 2 * H + 1; ++t) acc += w[REV ? 2 * H - t : t] * v[m + SH + t];
      o.v[m] = acc;
    }
    st4(out + r * pout + 4 * g, o);
  }
}

// Column pass for one item: rows [i0, i0+RR) of group g: acc[m] = sum_t w[t'] in[i0+m+t][4g..].
template <typename T, int H, int RR, bool REV>
__device__ __forceinline__ void col_item(const T* __restrict__ in, int pin, int in_rows, int i0, int g,
                                         const T (&w)[2 * H + 1], G4<T> (&acc)[RR]) {
  constexpr int NT = 2 * H + 1;
#pragma unroll
  for (int m = 0; m < RR; ++m)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[m].v[e] = T(0);
#pragma unroll
  for (int k = 0; k < RR + NT - 1; ++k) {
    if (i0 + k < in_rows) {
      const G4<T> v = lds4(in + (i0 + k) * pin + 4 * g);
#pragma unroll
      for (int m = 0; m < RR; ++m) {
        const int t = k - m;
        if (t >= 0 && t < NT) {
          const T wt = w[REV ? NT - 1 - t : t];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[m].v[e] += wt * v.v[e];
        }
      }
    }
  }
}

template <typename T>
struct Params {
  T tau, sigma, inv_sigma, rho, omr, t_h, inv_t_h, inv_step0, inv_step1, seg_a, seg_b;
  T lam;  // H = lam * L1 / L21 (the normal-operator kernel's fenchel step: clip / scale by lam)
  int unit0, unit1;  // step == 1: skip the scaling (exact)
};

template <typename T>
__device__ __forceinline__ T prox_g(T v, int gk, T a, T b) {
  if (gk == PCS_G_NONNEG) return (v < T(0)) ? T(0) : v;  // math/prox.py:295-297
  if (gk == PCS_G_SEGMENT) {                             // math/prox.py:340-343
    v = (v < a) ? a : v;
    return (v > b) ? b : v;
  }
  return v;
}

__device__ __forceinline__ float fast_rsqrt(float v) { return __builtin_amdgcn_rsqf(v); }
// fp64: v_rsq_f64 and two Newton steps (each squares the relative error: ~1 ulp) instead of 1.0 / sqrt(v),
// an IEEE square root and an IEEE division (~25 fp64 instructions on the fenchel prox's path).  v = 0 and
// v = +inf keep the hardware's exact +inf / 0 (a Newton step would turn them into NaN)
__device__ __forceinline__ double fast_rsqrt(double v) {
  const double y0 = __builtin_amdgcn_rsq(v);
  const double h = 0.5 * v;
  double y = y0 * __builtin_fma(-h * y0, y0, 1.5);
  y = y * __builtin_fma(-h * y, y, 1.5);
  return (v == 0.0 || v == __builtin_huge_val()) ? y0 : y;
}

template <typename T>
struct TileGeom {
  int64_t t0, c0;
};

// ---------------------------------------------------------------- tile body
template <typename T, int FK, int H, int TH, int NT, bool INT>
__device__ __forceinline__ void pds2d_tile(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                           T* __restrict__ zn, const T* __restrict__ y, const T* __restrict__ gbuf,
                                           const T (&w0)[2 * H + 1], const T (&w1)[2 * H + 1], const Slab& s,
                                           const Params<T>& P, int hk, int gk, int64_t t0, int64_t c0, T* bufX,
                                           T* bufA, double (&part)[4]) {
  constexpr bool CONV = (FK == PCS_F_SEPCONV);
  constexpr int TW = 64;
  constexpr int H4 = RU4<H>::value;
  constexpr int HG = TH + 1, WG = TW + 4, GG = WG / 4;         // U region rows [t0, t0+TH], cols [c0, c0+WG)
  constexpr int HR = HG + 2 * H, WR = WG + 2 * H4, GR = WR / 4;  // R region
  constexpr int HX = HG + 4 * H, WX = WG + 4 * H4, GX = WX / 4;  // X region
  constexpr int NZ0 = (HG + 1) * GG, NZ1 = HG * (GG + 1);      // Z0 rows [t0-1, t0+TH]; Z1 cols [c0-4, c0+WG)
  constexpr int SZ_U = HG * WG;
  constexpr int PX = CONV ? cdiv(HX * GX, NT) : 1;
  constexpr int PZ = cdiv(NZ0 + NZ1, NT);
  constexpr int PU = cdiv(HG * GG, NT);
  constexpr int RR2 = CONV ? cdiv(HR, NT / GR) : 1;
  constexpr int RR3 = CONV ? cdiv(HG, NT / GR) : 1;
  static_assert(!CONV || cdiv(HR, RR2) * GR <= NT, "P2 must fit one round");
  static_assert(!CONV || cdiv(HG, RR3) * GR <= NT, "P3 must fit one round");

  const int tid = threadIdx.x;
  const int64_t n0 = s.n0, n1 = s.n1;
  const int64_t zstride = (s.rows + 2 * s.hz) * n1;
  T* Gd = bufX;
  T* Z0 = CONV ? bufX + SZ_U : bufX;
  T* U = bufA;
  T* Z1 = bufA + SZ_U;

  G4<T> yr[RR2];
  const bool p2_on = CONV && tid < cdiv(HR, RR2) * GR;
  const int p2_i0 = (tid / GR) * RR2, p2_g = tid - (tid / GR) * GR;
  if constexpr (CONV) {
    // ---- stage X (HBM -> regs in one batch) and the y this thread's P2 item subtracts
    G4<T> xr[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int e = tid + k * NT;
      if (e < HX * GX) {
        const int r = e / GX, g = e - r * GX;
        xr[k] = gload4<T, INT>(x, s, s.hx, t0 - 2 * H + r, c0 - 2 * H4 + 4 * g);
      }
    }
    if (p2_on) {
#pragma unroll
      for (int m = 0; m < RR2; ++m) yr[m] = gload4<T, INT>(y, s, s.hy, t0 - H + p2_i0 + m, c0 - H4 + 4 * p2_g);
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int e = tid + k * NT;
      if (PCS_ON(6) && e < HX * GX) st4(bufX + 4 * e, xr[k]);  // dense rows: pitch WX = 4 GX
    }
    __syncthreads();
  }

  // ---- prefetch z (both components) and x (+ y / g) on the U region; consumed after the conv passes
  G4<T> zr[PZ];
#pragma unroll
  for (int k = 0; k < PZ; ++k) {
    const int e = tid + k * NT;
    if (e < NZ0) {
      const int r = e / GG, g = e - r * GG;
      zr[k] = gload4<T, INT>(z, s, s.hz, t0 - 1 + r, c0 + 4 * g);
    } else if (e < NZ0 + NZ1) {
      const int f = e - NZ0, r = f / (GG + 1), g = f - r * (GG + 1);
      zr[k] = gload4<T, INT>(z + zstride, s, s.hz, t0 + r, c0 - 4 + 4 * g);
    }
  }
  G4<T> xu[PU], yu[PU];
#pragma unroll
  for (int k = 0; k < PU; ++k) {
    const int e = tid + k * NT;
    if (e < HG * GG) {
      const int r = e / GG, g = e - r * GG;
      xu[k] = gload4<T, INT>(x, s, s.hx, t0 + r, c0 + 4 * g);
      if constexpr (FK == PCS_F_DENOISE) yu[k] = gload4<T, INT>(y, s, s.hy, t0 + r, c0 + 4 * g);
      if constexpr (FK == PCS_F_GRADBUF) yu[k] = gload4<T, INT>(gbuf, s, s.hy, t0 + r, c0 + 4 * g);
    }
  }

  if constexpr (CONV) {
    // P1: A = forward row conv of X on the R columns                (bufX -> bufA)
    if (PCS_ON(0)) row_pass<T, H, true, NT>(bufX, WX, bufA, WR, HX, GR, w1);
    __syncthreads();
    // P2: R = forward col conv of A - y, zero outside the image      (bufA -> bufX)
    if (PCS_ON(1) && p2_on) {
      G4<T> acc[RR2];
      col_item<T, H, RR2, true>(bufA, WR, HX, p2_i0, p2_g, w0, acc);
#pragma unroll
      for (int m = 0; m < RR2; ++m) {
        const int i = p2_i0 + m;
        if (i < HR) {
          if (INT) {
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[m].v[e] = acc[m].v[e] - yr[m].v[e];
          } else {
            const int64_t gr = s.row0 + t0 - H + i;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int64_t c = c0 - H4 + 4 * p2_g + e;
              const bool in = (gr >= 0 && gr < n0 && c >= 0 && c < n1);
              // r = Conv x - y   (grad = Conv^T((2*(r + (-y)))*0.5), map.py:609-610: exact)
              acc[m].v[e] = in ? (acc[m].v[e] - yr[m].v[e]) : T(0);
            }
          }
          st4(bufX + i * WR + 4 * p2_g, acc[m]);
        }
      }
    }
    __syncthreads();
    // P3: B = adjoint col pass of R: B[i] = sum_s w0[s] R[i + s]    (bufX -> bufA)
    if (PCS_ON(2) && tid < cdiv(HG, RR3) * GR) {
      const int i0 = (tid / GR) * RR3, g = tid - (tid / GR) * GR;
      G4<T> acc[RR3];
      col_item<T, H, RR3, false>(bufX, WR, HR, i0, g, w0, acc);
#pragma unroll
      for (int m = 0; m < RR3; ++m)
        if (i0 + m < HG) st4(bufA + (i0 + m) * WR + 4 * g, acc[m]);
    }
    __syncthreads();
    // P4: Gd = adjoint row pass of B on the U columns                (bufA -> bufX[0, SZ_U))
    if (PCS_ON(3)) row_pass<T, H, false, NT>(bufA, WR, Gd, WG, HG, GG, w1);
    __syncthreads();
  }

  // ---- land z in LDS (Z0 in bufX after Gd, Z1 in bufA after U)
#pragma unroll
  for (int k = 0; k < PZ; ++k) {
    const int e = tid + k * NT;
    if (!PCS_ON(7)) continue;
    if (e < NZ0) {
      st4(Z0 + 4 * e, zr[k]);  // dense, pitch WG
    } else if (e < NZ0 + NZ1) {
      st4(Z1 + 4 * (e - NZ0), zr[k]);  // dense, pitch WG + 4
    }
  }
  __syncthreads();

  // ---- P5: primal update on the U region; x' on the tile
#pragma unroll
  for (int k = 0; k < PU; ++k) {
    const int e = tid + k * NT;
    if (!PCS_ON(4) || e >= HG * GG) continue;
    const int i = e / GG, g = e - i * GG;
    const int64_t lr = t0 + i, gr = s.row0 + lr;
    G4<T> gd;
    if constexpr (CONV) gd = lds4(Gd + i * WG + 4 * g);
    const G4<T> za = lds4(Z0 + i * WG + 4 * g);             // z0[lr-1]
    const G4<T> zb = lds4(Z0 + (i + 1) * WG + 4 * g);       // z0[lr]
    const G4<T> z1a = lds4(Z1 + i * (WG + 4) + 4 * g);      // z1[c-4 .. c-1]
    const G4<T> z1b = lds4(Z1 + i * (WG + 4) + 4 * g + 4);  // z1[c .. c+3]
    const bool r_last = INT ? false : (gr >= n0 - 1), r_first = INT ? false : (gr <= 0);
    G4<T> uo, xo;
    bool own_all = (i < TH) && (4 * g < TW);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t c = c0 + 4 * g + m;
      const T xv = xu[k].v[m];
      T gf;
      if constexpr (FK == PCS_F_NULL) gf = T(0);
      else if constexpr (FK == PCS_F_DENOISE) gf = xv - yu[k].v[m];
      else if constexpr (FK == PCS_F_SEPCONV) gf = gd.v[m];
      else gf = yu[k].v[m];
      // K^T z for forward differences, VStack order: (0 + D0^T z0) + D1^T z1
      const T zl = (m == 0) ? z1a.v[3] : z1b.v[m - 1];
      T d0 = r_first ? T(0) : za.v[m];
      if (!r_last) d0 -= zb.v[m];
      T d1 = (INT || c > 0) ? zl : T(0);
      if (INT || c < n1 - 1) d1 -= z1b.v[m];
      const T a0 = P.unit0 ? d0 : d0 * P.inv_step0;
      const T a1 = P.unit1 ? d1 : d1 * P.inv_step1;
      const T xt = prox_g((xv - P.tau * gf) - P.tau * (a0 + a1), gk, P.seg_a, P.seg_b);
      bool in = true;
      if (!INT) in = (gr >= 0 && gr < n0 && c < n1 && lr <= s.rows);
      uo.v[m] = in ? (T(2) * xt - xv) : T(0);
      const T xnew = P.rho * xt + P.omr * xv;
      xo.v[m] = xnew;
      bool own = (i < TH) && (4 * g + m < TW);
      if (!INT) own = own && in && lr < s.rows;
      own_all = own_all && own;
      if (own) {
        const double dx = (double)xv - (double)xnew;
        part[0] += dx * dx;
        part[1] += (double)xv * (double)xv;
      }
    }
    st4(U + i * WG + 4 * g, uo);
    T* xrow = xn + (lr + s.hx) * n1;
    if (own_all && (INT || s.vec)) {
      st4(xrow + c0 + 4 * g, xo);
    } else if (i < TH) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t c = c0 + 4 * g + m;
        if (gr >= 0 && gr < n0 && c < n1 && (4 * g + m) < TW && lr < s.rows) xrow[c] = xo.v[m];
      }
    }
  }
  __syncthreads();

  // ---- P6: dual update on the tile
  constexpr int PD = cdiv(TH * (TW / 4), NT);
#pragma unroll
  for (int k = 0; k < PD; ++k) {
    const int e = tid + k * NT;
    if (!PCS_ON(5) || e >= TH * (TW / 4)) continue;
    const int i = e / (TW / 4), g = e - i * (TW / 4);
    const int64_t lr = t0 + i, gr = s.row0 + lr;
    if (!INT && (lr >= s.rows || gr >= n0)) continue;
    const G4<T> uc = lds4(U + i * WG + 4 * g);
    const G4<T> un = lds4(U + i * WG + 4 * g + 4);
    const G4<T> ud = lds4(U + (i + 1) * WG + 4 * g);
    const G4<T> zv0 = lds4(Z0 + (i + 1) * WG + 4 * g);
    const G4<T> zv1 = lds4(Z1 + i * (WG + 4) + 4 * g + 4);
    const bool r_last = INT ? false : (gr >= n0 - 1);
    G4<T> o0, o1;
    bool all_in = true;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t c = c0 + 4 * g + m;
      const bool cin = INT || c < n1;
      all_in = all_in && cin;
      const T uright = (m < 3) ? uc.v[m + 1] : un.v[0];
      T d0 = r_last ? T(0) : (ud.v[m] - uc.v[m]);
      T d1 = (INT || c < n1 - 1) ? (uright - uc.v[m]) : T(0);
      const T ku0 = P.unit0 ? d0 : d0 * P.inv_step0;
      const T ku1 = P.unit1 ? d1 : d1 * P.inv_step1;
      const T w0v = zv0.v[m] + P.sigma * ku0, w1v = zv1.v[m] + P.sigma * ku1;
      const T v0 = w0v * P.inv_sigma, v1 = w1v * P.inv_sigma;
      T zt0, zt1;
      if (hk == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
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
      if (cin) {
        const double e0 = (double)zv0.v[m] - (double)o0.v[m], e1 = (double)zv1.v[m] - (double)o1.v[m];
        part[2] += e0 * e0 + e1 * e1;
        part[3] += (double)zv0.v[m] * (double)zv0.v[m] + (double)zv1.v[m] * (double)zv1.v[m];
      }
    }
    T* r0 = zn + (lr + s.hz) * n1;
    T* r1 = r0 + zstride;
    if (all_in && (INT || s.vec)) {
      st4(r0 + c0 + 4 * g, o0);
      st4(r1 + c0 + 4 * g, o1);
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t c = c0 + 4 * g + m;
        if (c < n1) {
          r0[c] = o0.v[m];
          r1[c] = o1.v[m];
        }
      }
    }
  }
}

// ---------------------------------------------------------------- kernel
template <typename T, int FK, int H, int TH, int NT>
__global__ __launch_bounds__(NT) void k_pds2d(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                               T* __restrict__ zn, const T* __restrict__ y,
                                               const T* __restrict__ gbuf, const T* __restrict__ taps0,
                                               const T* __restrict__ taps1, int half, Slab s, Params<T> P, int hk,
                                               int gk, double* __restrict__ partials, Ctrl* ctrl,
                                               double* hist, void* ws, RedOut ro, int tiles_x, int ntiles, int bl,
                                               int tx_shift) {
  constexpr bool CONV = (FK == PCS_F_SEPCONV);
  constexpr int TW = 64;
  constexpr int H4 = RU4<H>::value;
  constexpr int HG = TH + 1, WG = TW + 4;
  constexpr int HX = HG + 4 * H, WX = WG + 4 * H4, WR = WG + 2 * H4;
  constexpr int SZ_Z0 = (HG + 1) * WG, SZ_Z1 = HG * (WG + 4), SZ_U = HG * WG;
  constexpr int SZX = CONV ? (HX * WX > SZ_U + SZ_Z0 ? HX * WX : SZ_U + SZ_Z0) : SZ_Z0;
  constexpr int SZA = CONV ? (HX * WR > SZ_U + SZ_Z1 ? HX * WR : SZ_U + SZ_Z1) : SZ_U + SZ_Z1;
  __shared__ __attribute__((aligned(16))) T bufX[SZX];
  __shared__ __attribute__((aligned(16))) T bufA[SZA];
  __shared__ double red[4 * (NT / 64)];
  __shared__ int flag[2];
  if (fin_slot(ro, ntiles, ctrl, hist, red, flag)) return;  // deferred finalization (pds_ctrl.hpp)

  const bool stopped = stop_requested(ctrl, ro, flag);
  if (stopped && ro.sums == nullptr) return;  // loop already stopped (solver.py:65-66)

  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> give them adjacent tiles.
  int tile;
  {
    const int b = (int)blockIdx.x - fin_shift(ro), q = ntiles / 8, r = ntiles % 8, xcd = b % 8, k = b / 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int ty = tile / tiles_x, txs = tile - ty * tiles_x;
  const int tx = txs < bl ? txs : txs + tx_shift;  // strip subset: [0, bl) and the right-most strips
  const int64_t t0 = (int64_t)ty * TH, c0 = (int64_t)tx * TW;

  T w0[2 * H + 1], w1[2 * H + 1];
#pragma unroll
  for (int t = 0; t < 2 * H + 1; ++t) {  // centred taps, zero-padded from `half` to the tier H
    const bool ok = CONV && (t - H >= -half) && (t - H <= half);
    w0[t] = ok ? taps0[t - H + half] : T(0);
    w1[t] = ok ? taps1[t - H + half] : T(0);
  }

  // interior: the tile's whole footprint (loads and boundary stencil cases) is inside the
  // image and the stored rows -> no bounds logic
  const int rh = CONV ? 2 * H : 1;
  const int ch = CONV ? 2 * H4 : 4;
  const int hmin = min(s.hx, min(s.hy, s.hz));
  const bool interior = s.vec && (s.row0 + t0 - rh >= 1) && (s.row0 + t0 + TH + rh <= s.n0 - 2) &&
                        (t0 - rh >= -hmin) && (t0 + TH + rh <= s.rows - 1 + hmin) && (t0 + TH <= s.rows - 1) &&
                        (c0 - ch >= 0) && (c0 + WG + ch <= s.n1 - 1);
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (stopped) {
  } else if (interior)
    pds2d_tile<T, FK, H, TH, NT, true>(x, xn, z, zn, y, gbuf, w0, w1, s, P, hk, gk, t0, c0, bufX, bufA, part);
  else
    pds2d_tile<T, FK, H, TH, NT, false>(x, xn, z, zn, y, gbuf, w0, w1, s, P, hk, gk, t0, c0, bufX, bufA, part);
  block_sum<4>(part, red);
  // single launch per iteration: last workgroups reduce (+ finalize) in-kernel, or deferred
  publish_partials(part, partials, ntiles, ws, ctrl, hist, flag, ro);
}

}  // namespace pcs
