// Fused PrimalDualSplitting step for 2-D images with a general finite-difference K:
//   K = Gradient(kind='forward' | 'backward' | 'centered', edge)      (pycsou/linop/diff.py:777-882)
//   K = Laplacian(weights, step, edge)                                (pycsou/linop/diff.py:885-957)
// and a pointwise grad F (F = 0, (1/2)||x - y||^2, or g read from a buffer -- e.g. Conv^T(Conv x - y)
// of a non-separable PSF from pcs_conv2d_planned):
//   x_t = prox_G((x - tau g) - tau K^T z),  u = 2 x_t - x
//   z_t = H.fenchel_prox(z + sigma K u, sigma)      H = lam*L1, or lam*L21 over the gradient components
//   z'  = rho z_t + (1-rho) z ;  x' = rho x_t + (1-rho) x
// plus the four norm partials of update_diagnostics and the in-kernel loop control --
// PrimalDualSplitting.update_iterand / update_diagnostics (pycsou/opt/proxalgs.py:343-394).
//
// One workgroup owns a 32 x 64 tile.  z' on the tile needs K u on it, i.e. u on the tile grown by
// 2 rows / columns (the Laplacian's one-sided edge rows reach two samples; the centred and the
// one-sided first-order stencils reach one), and u there needs K^T z, i.e. z on the tile grown by
// 4 rows / columns.  Phases:
//   loads   z region (40 x 72 per component) -> LDS; x, g of the U region (36 x 72) -> registers
//   U       K^T z (LDS), x_t, u -> LDS; x' on the tile -> HBM (16-B groups)
//   Z       K u (LDS), fenchel prox, relaxation; z' on the tile -> HBM
// The per-element stencils are stencil.hpp's (the standalone operators' operation order), so the
// fused step and the generic per-operator path agree to rounding.  Every global access is a
// 16-B group when n1 % 4 == 0 (groups are then wholly inside or outside the image).
#include "pds_tile.hpp"
#include "stencil.hpp"

namespace pcs {

enum { KK_LAP = 3 };  // KK: PCS_FORWARD / PCS_BACKWARD / PCS_CENTERED gradients, or the Laplacian

// phase barriers: LDS-only (s_waitcnt lgkmcnt(0) + s_barrier) by default -- no wave reads global
// data another wave of the launch wrote, so the x' stores of the U phase need not have landed
// before the Z phase (__syncthreads' release fence would wait for them); PCS_GEN_LDSBAR=0 restores it
#ifndef PCS_GEN_LDSBAR
#define PCS_GEN_LDSBAR 1
#endif
#if PCS_GEN_LDSBAR
#define PCS_GEN_BARRIER() lds_barrier()
#else
#define PCS_GEN_BARRIER() __syncthreads()
#endif
#ifndef PCS_GEN_TR
#define PCS_GEN_TR 32
#endif
struct GenG {
  static constexpr int TR = PCS_GEN_TR, TC = 64, NT = 256;
  static constexpr int CW = TC + 8, CG = CW / 4;  // LDS columns [c0 - 4, c0 + TC + 4)
  static constexpr int ZR = TR + 8, UR = TR + 4;  // Z rows [r0 - 4, r0 + TR + 4), U rows [r0 - 2, r0 + TR + 2)
  static constexpr int NZI = ZR * CG, NUI = UR * CG, NOI = TR * (TC / 4);
  static constexpr int KZ = cdiv(NZI, NT), KU = cdiv(NUI, NT), KO = cdiv(NOI, NT);
};

template <typename T>
struct GenP {
  T tau, sigma, inv_sigma, rho, omr, t_h, inv_t_h, h0, h1, w0, w1, h20, h21, seg_a, seg_b;
  T ih0, ih1, ih20, ih21;  // reciprocals for the interior path
};

struct GenGeo {
  int n0, n1, tiles1, edge;
};

// 4 columns [c, c + 4) of row r of an n0 x n1 array; zeros outside
template <typename T, bool VEC>
__device__ __forceinline__ G4<T> gen_ld4(const T* __restrict__ a, int n0, int n1, int r, int c) {
  G4<T> g = {{T(0), T(0), T(0), T(0)}};
  if ((unsigned)r >= (unsigned)n0) return g;
  const T* row = a + (int64_t)r * n1;
  if constexpr (VEC) {
    if (c >= 0 && c < n1) g = ld4(row + c);
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (c + m >= 0 && c + m < n1) g.v[m] = row[c + m];
  }
  return g;
}
template <typename T, bool VEC>
__device__ __forceinline__ void gen_st4(T* __restrict__ a, int n1, int r, int c, const G4<T>& g) {
  T* p = a + (int64_t)r * n1 + c;
  if constexpr (VEC) {
    st4(p, g);
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (c + m < n1) p[m] = g.v[m];
  }
}

// K^T z at image pixel (i0, i1); Z holds the components (comp stride zcs), l = local index
template <typename T, int KK>
__device__ __forceinline__ T gen_kt(const T* Z, int zcs, int l, int i0, int i1, int n0, int n1, const GenP<T>& P,
                                    int edge) {
  constexpr int CW = GenG::CW;
  if constexpr (KK == KK_LAP) {  // w0 D2_0^T z + w1 D2_1^T z (pylops Laplacian rmatvec)
    return P.w0 * d2_adj_core<T, int>(Z, l, CW, i0, n0, P.h20, edge) +
           P.w1 * d2_adj_core<T, int>(Z, l, 1, i1, n1, P.h21, edge);
  } else {  // VStack rmatvec: y = 0; y += D0^T z0; y += D1^T z1
    T acc = T(0);
    acc += d1_adj_core<T, int>(Z, l, CW, i0, n0, P.h0, KK, edge);
    acc += d1_adj_core<T, int>(Z + zcs, l, 1, i1, n1, P.h1, KK, edge);
    return acc;
  }
}

// Interior stencils (every pixel of the U region and the tile at >= 2 samples from the image
// edges, i.e. no edge rule can apply): branch-free, 1/h as a multiplication (exact for unit steps).
template <typename T, int KK>
__device__ __forceinline__ T gen_kt_int(const T* Z, int zcs, int l, const GenP<T>& P) {
  constexpr int CW = GenG::CW;
  if constexpr (KK == KK_LAP) {
    T a0 = Z[l + CW] * P.ih20;
    a0 -= (T(2) * Z[l]) * P.ih20;
    a0 += Z[l - CW] * P.ih20;
    T a1 = Z[l + 1] * P.ih21;
    a1 -= (T(2) * Z[l]) * P.ih21;
    a1 += Z[l - 1] * P.ih21;
    return P.w0 * a0 + P.w1 * a1;
  } else {
    const T* Z1 = Z + zcs;
    T a0, a1;
    if constexpr (KK == PCS_FORWARD) {
      a0 = -(Z[l] * P.ih0) + Z[l - CW] * P.ih0;
      a1 = -(Z1[l] * P.ih1) + Z1[l - 1] * P.ih1;
    } else if constexpr (KK == PCS_BACKWARD) {
      a0 = -(Z[l + CW] * P.ih0) + Z[l] * P.ih0;
      a1 = -(Z1[l + 1] * P.ih1) + Z1[l] * P.ih1;
    } else {
      a0 = -((T(0.5) * Z[l + CW]) * P.ih0) + (T(0.5) * Z[l - CW]) * P.ih0;
      a1 = -((T(0.5) * Z1[l + 1]) * P.ih1) + (T(0.5) * Z1[l - 1]) * P.ih1;
    }
    return (T(0) + a0) + a1;
  }
}
template <typename T, int KK>
__device__ __forceinline__ void gen_ku_int(const T* U, int l, const GenP<T>& P, T* ku) {
  constexpr int CW = GenG::CW;
  if constexpr (KK == KK_LAP) {
    ku[0] = P.w0 * ((U[l + CW] - T(2) * U[l] + U[l - CW]) * P.ih20) + P.w1 * ((U[l + 1] - T(2) * U[l] + U[l - 1]) * P.ih21);
  } else if constexpr (KK == PCS_FORWARD) {
    ku[0] = (U[l + CW] - U[l]) * P.ih0;
    ku[1] = (U[l + 1] - U[l]) * P.ih1;
  } else if constexpr (KK == PCS_BACKWARD) {
    ku[0] = (U[l] - U[l - CW]) * P.ih0;
    ku[1] = (U[l] - U[l - 1]) * P.ih1;
  } else {
    ku[0] = (T(0.5) * U[l + CW] - T(0.5) * U[l - CW]) * P.ih0;
    ku[1] = (T(0.5) * U[l + 1] - T(0.5) * U[l - 1]) * P.ih1;
  }
}

template <typename T, int KK, int FK, bool VEC, bool INT>
__device__ __forceinline__ void gen_tile(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                         T* __restrict__ zn, const T* __restrict__ gsrc, const GenGeo& geo,
                                         const GenP<T>& P, int hk, int gk, int r0, int c0, T* Z, T* U,
                                         double (&part)[4]) {
  using G = GenG;
  constexpr int D = (KK == KK_LAP) ? 1 : 2, CW = G::CW, CG = G::CG, NT = G::NT, ZS = G::ZR * G::CW;
  constexpr bool LV = VEC || INT;  // interior tiles: every group of the regions is inside the image
  const int n0 = geo.n0, n1 = geo.n1, edge = geo.edge;
  const int64_t N = (int64_t)n0 * n1;
  const int tid = threadIdx.x;
  auto ld = [&](const T* a, int r, int c) -> G4<T> {
    if constexpr (INT && VEC) return ld4(a + (int64_t)r * n1 + c);
    else return gen_ld4<T, LV && VEC>(a, n0, n1, r, c);
  };

  // ---- loads: z region -> registers -> LDS; x (and g) of the U items -> registers
  G4<T> xr[G::KU], gr[G::KU];
  {
    G4<T> zr[D][G::KZ];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int k = 0; k < G::KZ; ++k) {
        const int e = min(k * NT + tid, G::NZI - 1), rr = e / CG, g = e - rr * CG;
        zr[d][k] = ld(z + d * N, r0 - 4 + rr, c0 - 4 + 4 * g);
      }
#pragma unroll
    for (int k = 0; k < G::KU; ++k) {
      const int e = min(k * NT + tid, G::NUI - 1), rr = e / CG, g = e - rr * CG;
      xr[k] = ld(x, r0 - 2 + rr, c0 - 4 + 4 * g);
      if constexpr (FK != PCS_F_NULL) gr[k] = ld(gsrc, r0 - 2 + rr, c0 - 4 + 4 * g);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int k = 0; k < G::KZ; ++k) {
        const int e = k * NT + tid;
        if (e < G::NZI) st4(Z + d * ZS + 4 * e, zr[d][k]);  // row rr, group g at rr * CW + 4 g = 4 e
      }
  }
  PCS_GEN_BARRIER();
  // ---- U items: x_t, u on rows [r0 - 2, r0 + TR + 2) x columns [c0 - 2, c0 + TC + 2); x' on the tile
#pragma unroll
  for (int k = 0; k < G::KU; ++k) {
    const int e = k * NT + tid;
    if (e < G::NUI) {
      const int rr = e / CG, g = e - rr * CG;
      const int i0 = r0 - 2 + rr, cb = c0 - 4 + 4 * g;
      const int lz = (rr + 2) * CW + 4 * g;  // Z local index of (i0, cb)
      const bool own = rr >= 2 && rr < 2 + G::TR && g >= 1 && g <= G::TC / 4 && i0 < n0 && cb < n1;
      G4<T> uo, xo;
      T sdx = T(0), sx = T(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int i1 = cb + m;
        // interior tiles: every column of the item is in the image (the two outside the U region
        // compute unused values from in-bounds LDS neighbours)
        const bool in = INT || ((unsigned)i0 < (unsigned)n0 && (unsigned)i1 < (unsigned)n1 && i1 >= c0 - 2 &&
                                i1 < c0 + G::TC + 2);
        T u = T(0), xnew = T(0), xv = xr[k].v[m];
        if (in) {
          T gf = T(0);
          if constexpr (FK == PCS_F_DENOISE) gf = xv - gr[k].v[m];  // (2 (x + (-y))) 0.5, exact
          else if constexpr (FK == PCS_F_GRADBUF) gf = gr[k].v[m];
          T kt;
          if constexpr (INT) kt = gen_kt_int<T, KK>(Z, ZS, lz + m, P);
          else kt = gen_kt<T, KK>(Z, ZS, lz + m, i0, i1, n0, n1, P, edge);
          const T xt = prox_g((xv - P.tau * gf) - P.tau * kt, gk, P.seg_a, P.seg_b);
          u = T(2) * xt - xv;
          xnew = P.rho * xt + P.omr * xv;
        }
        const T dx = xv - xnew;
        sdx += (in && i1 < n1) ? dx * dx : T(0);
        sx += (in && i1 < n1) ? xv * xv : T(0);
        uo.v[m] = u;
        xo.v[m] = xnew;
      }
      st4(U + rr * CW + 4 * g, uo);
      if (own) {
        part[0] += (double)sdx;
        part[1] += (double)sx;
        gen_st4<T, LV && VEC>(xn, n1, i0, cb, xo);
      }
    }
  }
  PCS_GEN_BARRIER();
  // ---- z' on the tile
#pragma unroll
  for (int k = 0; k < G::KO; ++k) {
    const int e = k * NT + tid;
    if (e < G::NOI) {
      const int rr = e / (G::TC / 4), g = e - rr * (G::TC / 4);
      const int i0 = r0 + rr, cb = c0 + 4 * g;
      if (INT || (i0 < n0 && cb < n1)) {
        const int lu = (rr + 2) * CW + 4 * (g + 1), lz = (rr + 4) * CW + 4 * (g + 1);
        G4<T> o[D];
        T sdz = T(0), sz = T(0);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int i1 = cb + m;
          T ku[D], zv[D];
          if constexpr (INT) {
            gen_ku_int<T, KK>(U, lu + m, P, ku);
          } else if constexpr (KK == KK_LAP) {  // w0 D2_0 u + w1 D2_1 u (pylops Laplacian matvec)
            ku[0] = P.w0 * d2_fwd_core<T, int>(U, lu + m, CW, i0, n0, P.h20, edge) +
                    P.w1 * d2_fwd_core<T, int>(U, lu + m, 1, i1, n1, P.h21, edge);
          } else {
            ku[0] = d1_fwd_core<T, int>(U, lu + m, CW, i0, n0, P.h0, KK, edge);
            ku[1] = d1_fwd_core<T, int>(U, lu + m, 1, i1, n1, P.h1, KK, edge);
          }
          T w[D], v[D], zt[D];
#pragma unroll
          for (int d = 0; d < D; ++d) {
            zv[d] = Z[d * ZS + lz + m];
            w[d] = zv[d] + P.sigma * ku[d];
            v[d] = w[d] * P.inv_sigma;
          }
          if (D == 2 && hk == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
            T f = T(1) - P.t_h * fast_rsqrt(v[0] * v[0] + v[D - 1] * v[D - 1]);
            f = f > T(0) ? f : T(0);
#pragma unroll
            for (int d = 0; d < D; ++d) zt[d] = w[d] - P.sigma * (f * v[d]);
          } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
#pragma unroll
            for (int d = 0; d < D; ++d) zt[d] = w[d] - P.sigma * (v[d] - P.t_h * clip1(v[d] * P.inv_t_h));
          }
          const bool cm = INT || i1 < n1;
#pragma unroll
          for (int d = 0; d < D; ++d) {
            o[d].v[m] = P.rho * zt[d] + P.omr * zv[d];
            const T ed = zv[d] - o[d].v[m];
            sdz += cm ? ed * ed : T(0);
            sz += cm ? zv[d] * zv[d] : T(0);
          }
        }
        part[2] += (double)sdz;
        part[3] += (double)sz;
#pragma unroll
        for (int d = 0; d < D; ++d) gen_st4<T, LV && VEC>(zn + d * N, n1, i0, cb, o[d]);
      }
    }
  }
}

template <typename T, int KK, int FK, bool VEC>
__global__ __launch_bounds__(GenG::NT) void k_pds2d_gen(const T* __restrict__ x, T* __restrict__ xn,
                                                         const T* __restrict__ z, T* __restrict__ zn,
                                                         const T* __restrict__ gsrc, GenGeo geo, GenP<T> P, int hk,
                                                         int gk, double* __restrict__ partials, Ctrl* ctrl,
                                                         double* hist, void* ws, int ntasks) {
  using G = GenG;
  constexpr int D = (KK == KK_LAP) ? 1 : 2;
  __shared__ __attribute__((aligned(16))) T Z[D * G::ZR * G::CW];
  __shared__ __attribute__((aligned(16))) T U[G::UR * G::CW];
  __shared__ double red[4 * (G::NT / 64)];
  __shared__ int flag[2];
  if (ctrl != nullptr && ctrl->stopped != 0) return;  // loop already stopped (solver.py:65-66)
  int task;
  {  // XCD-aware bijective remap: consecutive tiles of a row share an XCD (their halo lines)
    const int b = blockIdx.x, q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int ty = task / geo.tiles1, tx = task - ty * geo.tiles1;
  const int r0 = ty * G::TR, c0 = tx * G::TC;
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  // interior tile (uniform): the U region and the tile are >= 2 samples inside the image and the
  // regions' loads are all in bounds -> no edge rule, no bounds check
  const bool interior = r0 >= 4 && r0 + G::TR + 4 <= geo.n0 && c0 >= 4 && c0 + G::TC + 4 <= geo.n1;
  if (interior)
    gen_tile<T, KK, FK, VEC, true>(x, xn, z, zn, gsrc, geo, P, hk, gk, r0, c0, Z, U, part);
  else
    gen_tile<T, KK, FK, VEC, false>(x, xn, z, zn, gsrc, geo, P, hk, gk, r0, c0, Z, U, part);
  block_sum<4>(part, red);
  if (hist != nullptr) {
    reduce_and_finalize(part, partials, ntasks, ws, ctrl, hist, flag);
  } else if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) partials[(int64_t)blockIdx.x * 4 + k] = part[k];
  }
}

// ---------------------------------------------------------------- host side
static int64_t gen_tiles(const pcs_pds2d_stencil_args* a) {
  return ((a->n0 + GenG::TR - 1) / GenG::TR) * ((a->n1 + GenG::TC - 1) / GenG::TC);
}

static bool gen_aligned(const void* q) { return q == nullptr || ((uintptr_t)q & 15) == 0; }

template <typename T, int KK, int FK, bool VEC>
static int gen_launch(const pcs_pds2d_stencil_args* a, const void* x, void* xn, const void* z, void* zn,
                      hipStream_t st) {
  GenGeo geo;
  geo.n0 = (int)a->n0;
  geo.n1 = (int)a->n1;
  geo.tiles1 = (int)((a->n1 + GenG::TC - 1) / GenG::TC);
  geo.edge = a->edge;
  GenP<T> P;
  P.tau = (T)a->tau;
  P.sigma = (T)a->sigma;
  P.inv_sigma = (T)(1.0 / a->sigma);
  P.rho = (T)a->rho;
  P.omr = (T)(1.0 - a->rho);
  const double t_h = (1.0 / a->sigma) * a->lam;  // ProxFuncPostComp: tau*scale with tau = 1/sigma
  P.t_h = (T)t_h;
  P.inv_t_h = (T)(1.0 / t_h);
  P.h0 = (T)a->step0;
  P.h1 = (T)a->step1;
  P.w0 = (T)a->w0;
  P.w1 = (T)a->w1;
  P.h20 = (T)(a->step0 * a->step0);
  P.h21 = (T)(a->step1 * a->step1);
  P.ih0 = (T)(1.0 / a->step0);
  P.ih1 = (T)(1.0 / a->step1);
  P.ih20 = (T)(1.0 / (a->step0 * a->step0));
  P.ih21 = (T)(1.0 / (a->step1 * a->step1));
  P.seg_a = (T)a->seg_a;
  P.seg_b = (T)a->seg_b;
  const int ntasks = (int)gen_tiles(a);
  k_pds2d_gen<T, KK, FK, VEC><<<(unsigned)ntasks, GenG::NT, 0, st>>>(
      (const T*)x, (T*)xn, (const T*)z, (T*)zn, (const T*)a->g, geo, P, a->hkind, a->gkind, a->partials,
      (Ctrl*)a->ctrl, a->hist, a->ws, ntasks);
  return launch_status();
}

template <typename T, int KK, bool VEC>
static int gen_fk(const pcs_pds2d_stencil_args* a, const void* x, void* xn, const void* z, void* zn, hipStream_t st) {
  switch (a->fkind) {
    case PCS_F_NULL: return gen_launch<T, KK, PCS_F_NULL, VEC>(a, x, xn, z, zn, st);
    case PCS_F_DENOISE: return gen_launch<T, KK, PCS_F_DENOISE, VEC>(a, x, xn, z, zn, st);
    case PCS_F_GRADBUF: return gen_launch<T, KK, PCS_F_GRADBUF, VEC>(a, x, xn, z, zn, st);
    default: return PCS_EINVAL;
  }
}

template <typename T, bool VEC>
static int gen_kk(const pcs_pds2d_stencil_args* a, const void* x, void* xn, const void* z, void* zn, hipStream_t st) {
  switch (a->kkind) {
    case PCS_K_GRAD_FORWARD: return gen_fk<T, PCS_FORWARD, VEC>(a, x, xn, z, zn, st);
    case PCS_K_GRAD_BACKWARD: return gen_fk<T, PCS_BACKWARD, VEC>(a, x, xn, z, zn, st);
    case PCS_K_GRAD_CENTERED: return gen_fk<T, PCS_CENTERED, VEC>(a, x, xn, z, zn, st);
    case PCS_K_LAPLACIAN: return gen_fk<T, KK_LAP, VEC>(a, x, xn, z, zn, st);
    default: return PCS_EINVAL;
  }
}

static int gen_step(const pcs_pds2d_stencil_args* a, const void* x, void* xn, const void* z, void* zn,
                    hipStream_t st) {
  const bool vec = a->n1 % 4 == 0 && gen_aligned(x) && gen_aligned(xn) && gen_aligned(z) && gen_aligned(zn) &&
                   gen_aligned(a->g);
  if (a->dtype == PCS_F32) return vec ? gen_kk<float, true>(a, x, xn, z, zn, st) : gen_kk<float, false>(a, x, xn, z, zn, st);
  return vec ? gen_kk<double, true>(a, x, xn, z, zn, st) : gen_kk<double, false>(a, x, xn, z, zn, st);
}

static int gen_check(const pcs_pds2d_stencil_args* a) {
  if (!a || !a->x || !a->xn || !a->z || !a->zn || !a->partials) return PCS_EINVAL;
  if (a->dtype != PCS_F32 && a->dtype != PCS_F64) return PCS_EINVAL;
  if (a->n0 < 1 || a->n1 < 1) return PCS_EINVAL;
  if (a->n0 >= (1LL << 30) || a->n1 >= (1LL << 30) || gen_tiles(a) >= (1LL << 31)) return PCS_EUNSUPPORTED;
  if (a->kkind < PCS_K_GRAD_FORWARD || a->kkind > PCS_K_LAPLACIAN) return PCS_EINVAL;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return PCS_EINVAL;
  if (a->kkind == PCS_K_LAPLACIAN && a->hkind != PCS_H_L1) return PCS_EINVAL;  // one component: L21 == L1
  if (a->gkind < PCS_G_NULL || a->gkind > PCS_G_SEGMENT) return PCS_EINVAL;
  if (a->fkind != PCS_F_NULL && a->fkind != PCS_F_DENOISE && a->fkind != PCS_F_GRADBUF) return PCS_EINVAL;
  if (a->fkind != PCS_F_NULL && !a->g) return PCS_EINVAL;
  if (!(a->sigma > 0) || !(a->lam > 0) || a->step0 == 0 || a->step1 == 0) return PCS_EINVAL;
  if (a->hist && (!a->ws || !a->ctrl || !gen_aligned(a->ws) || !gen_aligned(a->partials))) return PCS_EINVAL;
  return PCS_OK;
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int64_t pcs_pds2d_stencil_nblocks(const pcs_pds2d_stencil_args* a) {
  if (!a || a->n0 < 1 || a->n1 < 1) return -1;
  return gen_tiles(a);
}

int64_t pcs_pds2d_stencil_ws_bytes(const pcs_pds2d_stencil_args* a) {
  const int64_t nb = pcs_pds2d_stencil_nblocks(a);
  return nb < 0 ? -1 : red_ws_bytes(nb);
}

int pcs_pds2d_stencil_step(const pcs_pds2d_stencil_args* a, hipStream_t st) {
  const int rc = gen_check(a);
  return rc != PCS_OK ? rc : gen_step(a, a->x, a->xn, a->z, a->zn, st);
}

int pcs_pds2d_stencil_run(const pcs_pds2d_stencil_args* a, int64_t n, hipStream_t st) {
  const int rc = gen_check(a);
  if (rc != PCS_OK) return rc;
  if (n < 0 || !a->hist) return PCS_EINVAL;
  for (int64_t i = 0; i < n; ++i) {
    const bool odd = i & 1;
    const int r = odd ? gen_step(a, a->xn, const_cast<void*>(a->x), a->zn, const_cast<void*>(a->z), st)
                      : gen_step(a, a->x, a->xn, a->z, a->zn, st);
    if (r != PCS_OK) return r;
  }
  return PCS_OK;
}

}  // extern "C"
