// Fused PrimalDualSplitting iteration for 2-D images (one launch per iteration).
//
// Replaces, for the problem family of the PDS headline benchmark,
//   PrimalDualSplitting.update_iterand      pycsou/opt/proxalgs.py:343-355
//   PrimalDualSplitting.update_diagnostics  pycsou/opt/proxalgs.py:366-394
//   GenericIterativeAlgorithm.iterate loop  pycsou/core/solver.py:55-76
// with F = 1/2 ||Conv x - y||^2 (Conv separable, centred taps), 1/2 ||x - y||^2, 0, or a
// precomputed gradient buffer; K = Gradient(kind='forward'); H = lam*L1 / lam*L21 (pixel
// groups); G = Null / NonNegativeOrthant / Segment.
//
// Design (MI355X): the iteration reads x, y, z once and writes x', z' once -- the
// compulsory (2d+3) N words -- by recomputing, per 64 x TH output tile, everything
// the tile depends on inside LDS:
//   X  = x on the tile grown by 1+2H rows / CX cols          (global -> LDS)
//   A  = row-conv(X)          (forward conv, along axis 1)   (LDS -> LDS)
//   R  = col-conv(A) - y, zero outside the image (= residual r = h*x - y)
//   B  = col-corr(R)          (adjoint conv, along axis 0)
//   Gd = row-corr(B)          (= Conv^T r = grad F on the tile grown by one ring)
//   x_t, u = 2x_t - x on the grown tile (U in LDS), x' on the tile  -> HBM
//   z' = rho * fenchel(z + sigma K u) + (1-rho) z on the tile       -> HBM
// Every LDS pass works on 4-wide column groups (one 16-B ds_read per lane, lanes on
// consecutive 16-B slots: conflict-free), taps are compile-time-indexed registers, the
// column passes keep a rolling RR-row register window, so each LDS value feeds up to
// 4*RR FMAs.  Blocks are remapped so that each XCD sweeps a contiguous band of tiles
// (halo re-reads hit that XCD's L2).
#include "common.hpp"

namespace pcs {

template <int V>
struct RU4 {
  static constexpr int value = (V + 3) / 4 * 4;
};

template <typename T>
__device__ __forceinline__ void lds_ld4(const T* p, T (&v)[4]);
template <>
__device__ __forceinline__ void lds_ld4<float>(const float* p, float (&v)[4]) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
}
template <>
__device__ __forceinline__ void lds_ld4<double>(const double* p, double (&v)[4]) {
  const double2 a = reinterpret_cast<const double2*>(p)[0];
  const double2 b = reinterpret_cast<const double2*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}
template <typename T>
__device__ __forceinline__ void lds_st4(T* p, const T (&v)[4]);
template <>
__device__ __forceinline__ void lds_st4<float>(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void lds_st4<double>(double* p, const double (&v)[4]) {
  reinterpret_cast<double2*>(p)[0] = make_double2(v[0], v[1]);
  reinterpret_cast<double2*>(p)[1] = make_double2(v[2], v[3]);
}

// Slab geometry shared by all passes.
struct Slab {
  int64_t n0, n1, row0, rows;
  int hx, hy, hz;  // halo rows stored in x/xn, y/gbuf, z/zn
};

// Global element (local row lr, col c) of a slab array with `halo` stored halo rows;
// zero outside the image or outside the stored rows.
template <typename T>
__device__ __forceinline__ T gload(const T* __restrict__ a, const Slab& s, int halo, int64_t lr, int64_t c) {
  const int64_t gr = s.row0 + lr;
  if (gr < 0 || gr >= s.n0 || c < 0 || c >= s.n1 || lr < -halo || lr >= s.rows + halo) return T(0);
  return a[(lr + halo) * s.n1 + c];
}

// ---------------------------------------------------------------- LDS passes
// Row pass: out[r][j] = sum_t w[t] * in[r][j + SH + t], j in 4-groups, SH = H4 - H.
template <typename T, int H, bool REV>
__device__ __forceinline__ void row_pass(const T* __restrict__ in, int pin, T* __restrict__ out, int pout, int rows,
                                         int ngroups, const T (&w)[2 * H + 1]) {
  constexpr int H4 = RU4<H>::value;
  constexpr int NV = 1 + H4 / 2;  // 4-groups loaded per item
  constexpr int SH = H4 - H;
  const int items = rows * ngroups;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int r = it / ngroups, g = it - r * ngroups;
    T v[4 * NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      T t4[4];
      lds_ld4(in + r * pin + 4 * g + 4 * q, t4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = t4[e];
    }
    T o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T acc = T(0);
#pragma unroll
      for (int t = 0; t < 2 * H + 1; ++t) acc += w[REV ? 2 * H - t : t] * v[m + SH + t];
      o[m] = acc;
    }
    lds_st4(out + r * pout + 4 * g, o);
  }
}

// Column pass: out[i][j] = sum_t w[t] * in[i + t][j] for i < out_rows, rolling RR-row window.
// Epi(i, j0, o[4]) post-processes the 4 outputs of row i, columns j0..j0+3 before the store.
template <typename T, int H, int RR, bool REV, typename Epi>
__device__ __forceinline__ void col_pass(const T* __restrict__ in, int pin, T* __restrict__ out, int pout,
                                         int out_rows, int ngroups, const T (&w)[2 * H + 1], Epi epi) {
  constexpr int NT = 2 * H + 1;
  const int chunks = (out_rows + RR - 1) / RR;
  const int items = chunks * ngroups;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int c = it / ngroups, g = it - c * ngroups;
    const int i0 = c * RR;
    T acc[RR][4];
#pragma unroll
    for (int m = 0; m < RR; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[m][e] = T(0);
#pragma unroll
    for (int k = 0; k < RR + NT - 1; ++k) {
      // rows beyond out_rows + NT - 1 only feed outputs that are never stored
      if (i0 + k < out_rows + NT - 1) {
        T v[4];
        lds_ld4(in + (i0 + k) * pin + 4 * g, v);
#pragma unroll
        for (int m = 0; m < RR; ++m) {
          const int t = k - m;
          if (t >= 0 && t < NT) {
            const T wt = w[REV ? NT - 1 - t : t];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[m][e] += wt * v[e];
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < RR; ++m) {
      if (i0 + m < out_rows) {
        epi(i0 + m, 4 * g, acc[m]);
        lds_st4(out + (i0 + m) * pout + 4 * g, acc[m]);
      }
    }
  }
}

struct NoEpi {
  template <typename T>
  __device__ void operator()(int, int, T (&)[4]) const {}
};

template <typename T>
struct Params {
  T tau, sigma, rho, omr, lam_over_sigma, step0, step1, seg_a, seg_b;
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

// ---------------------------------------------------------------- fused kernel
// FK: PCS_F_*.  H: separable half width tier (FK == PCS_F_SEPCONV), else 0.  TH: tile rows.
template <typename T, int FK, int H, int TH>
__global__ __launch_bounds__(256) void k_pds2d(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                                T* __restrict__ zn, const T* __restrict__ y,
                                                const T* __restrict__ gbuf, const T* __restrict__ taps0,
                                                const T* __restrict__ taps1, int half, Slab s, Params<T> P, int hk,
                                                int gk, double* __restrict__ partials,
                                                const int32_t* __restrict__ ctrl, int tiles_x, int ntiles) {
  constexpr int TW = 64;
  constexpr int H4 = RU4<H>::value;
  constexpr int CG = 4, CR = CG + H4, CX = CR + H4;
  constexpr int WG = TW + 2 * CG, WR = TW + 2 * CR, WX = TW + 2 * CX;
  constexpr int HG = TH + 2, HR = HG + 2 * H, HXR = HG + 4 * H;
  constexpr int SZ1 = (FK == PCS_F_SEPCONV) ? (HXR * WX > HG * WG ? HXR * WX : HG * WG) : 4;
  constexpr int SZ2 = (FK == PCS_F_SEPCONV) ? HXR * WR : HG * WG;
  __shared__ __attribute__((aligned(16))) T buf1[SZ1];
  __shared__ __attribute__((aligned(16))) T buf2[SZ2];
  __shared__ double red[4 * 4];

  if (ctrl != nullptr && ctrl[1] != 0) return;  // loop already stopped (solver.py:65-66)

  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> give them adjacent tiles.
  int tile;
  {
    const int b = blockIdx.x, q = ntiles / 8, r = ntiles % 8, xcd = b % 8, k = b / 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int64_t t0 = (int64_t)ty * TH;          // first local row of the tile
  const int64_t c0 = (int64_t)tx * TW;          // first column of the tile
  const int64_t n0 = s.n0, n1 = s.n1;

  // ---- grad F on the G region (rows t0-1 .. t0+TH, cols c0-CG .. c0+TW+CG) ----
  T* U = (FK == PCS_F_SEPCONV) ? buf2 : buf2;  // U lives in buf2 in every mode
  T* Gd = buf1;                                 // only used by SEPCONV
  if constexpr (FK == PCS_F_SEPCONV) {
    constexpr int NT = 2 * H + 1;
    T w0[NT], w1[NT];  // centred taps, zero-padded from `half` to the tier H
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int sidx = t - H + half;
      const bool ok = (t - H >= -half) && (t - H <= half);
      w0[t] = ok ? taps0[sidx] : T(0);
      w1[t] = ok ? taps1[sidx] : T(0);
    }
    // X: global -> LDS (zero outside image / stored rows)
    const int64_t xr0 = t0 - 1 - 2 * H, xc0 = c0 - CX;
    for (int e = threadIdx.x; e < HXR * (WX / 4); e += blockDim.x) {
      const int r = e / (WX / 4), g = e - r * (WX / 4);
      T v[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) v[m] = gload(x, s, s.hx, xr0 + r, xc0 + 4 * g + m);
      lds_st4(buf1 + r * WX + 4 * g, v);
    }
    __syncthreads();
    // A = forward row conv of X on the R columns: out[c] = sum_s w1[s] X[c - s]
    row_pass<T, H, true>(buf1, WX, buf2, WR, HXR, WR / 4, w1);
    __syncthreads();
    // R = forward col conv of A - y, zero outside the image
    {
      const int64_t rr0 = t0 - 1 - H, rc0 = c0 - CR;
      const Slab sl = s;
      auto epi = [&](int i, int j0, T(&o)[4]) {
        const int64_t lr = rr0 + i, gr = sl.row0 + lr;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int64_t c = rc0 + j0 + m;
          const bool in = (gr >= 0 && gr < sl.n0 && c >= 0 && c < sl.n1);
          // r = Conv x - y   (grad = Conv^T((2*(r + (-y)))*0.5), map.py:609-610; exact)
          o[m] = in ? (o[m] - gload(y, sl, sl.hy, lr, c)) : T(0);
        }
      };
      col_pass<T, H, 6, true>(buf2, WR, buf1, WR, HR, WR / 4, w0, epi);
    }
    __syncthreads();
    // B = adjoint col pass of R (correlation): B[i] = sum_s w0[s] R[i + s]
    col_pass<T, H, 6, false>(buf1, WR, buf2, WR, HG, WR / 4, w0, NoEpi{});
    __syncthreads();
    // Gd = adjoint row pass of B on the G columns
    row_pass<T, H, false>(buf2, WR, Gd, WG, HG, WG / 4, w1);
    __syncthreads();
  }

  // ---- primal update on the G region; x' on the tile ----
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  const T* z0 = z;
  const T* z1 = z + (s.rows + 2 * s.hz) * n1;
  for (int e = threadIdx.x; e < HG * (WG / 4); e += blockDim.x) {
    const int i = e / (WG / 4), g = e - i * (WG / 4);
    const int64_t lr = t0 - 1 + i, gr = s.row0 + lr;
    T uo[4];
    T gdv[4];
    if constexpr (FK == PCS_F_SEPCONV) lds_ld4(Gd + i * WG + 4 * g, gdv);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t c = c0 - CG + 4 * g + m;
      const bool in = (gr >= 0 && gr < n0 && c >= 0 && c < n1 && lr >= -1 && lr <= s.rows);
      T u = T(0);
      if (in) {
        const T xv = x[(lr + s.hx) * n1 + c];
        T gf;
        if constexpr (FK == PCS_F_NULL) gf = T(0);
        else if constexpr (FK == PCS_F_DENOISE) gf = xv - y[(lr + s.hy) * n1 + c];
        else if constexpr (FK == PCS_F_SEPCONV) gf = gdv[m];
        else gf = gbuf[(lr + s.hy) * n1 + c];
        // K^T z for forward differences, VStack order: (0 + D0^T z0) + D1^T z1
        T a0 = T(0), a1 = T(0);
        if (gr < n0 - 1) a0 -= z0[(lr + s.hz) * n1 + c] / P.step0;
        if (gr > 0) a0 += z0[(lr - 1 + s.hz) * n1 + c] / P.step0;
        if (c < n1 - 1) a1 -= z1[(lr + s.hz) * n1 + c] / P.step1;
        if (c > 0) a1 += z1[(lr + s.hz) * n1 + c - 1] / P.step1;
        const T ktz = a0 + a1;
        const T xt = prox_g((xv - P.tau * gf) - P.tau * ktz, gk, P.seg_a, P.seg_b);
        u = T(2) * xt - xv;
        const bool own = (i >= 1 && i <= TH && (4 * g + m) >= CG && (4 * g + m) < CG + TW && lr < s.rows);
        if (own) {
          const T xnew = P.rho * xt + P.omr * xv;
          xn[(lr + s.hx) * n1 + c] = xnew;
          const double dx = (double)xv - (double)xnew;
          part[0] += dx * dx;
          part[1] += (double)xv * (double)xv;
        }
      }
      uo[m] = u;
    }
    lds_st4(U + i * WG + 4 * g, uo);
  }
  __syncthreads();

  // ---- dual update on the tile ----
  const T t_h = P.lam_over_sigma;
  T* zn0 = zn;
  T* zn1 = zn + (s.rows + 2 * s.hz) * n1;
  for (int e = threadIdx.x; e < TH * TW; e += blockDim.x) {
    const int i = e / TW, j = e - i * TW;
    const int64_t lr = t0 + i, gr = s.row0 + lr, c = c0 + j;
    if (lr >= s.rows || gr >= n0 || c >= n1) continue;
    const T uc = U[(i + 1) * WG + CG + j];
    const T ku0 = (gr < n0 - 1) ? (U[(i + 2) * WG + CG + j] - uc) / P.step0 : T(0);
    const T ku1 = (c < n1 - 1) ? (U[(i + 1) * WG + CG + j + 1] - uc) / P.step1 : T(0);
    const int64_t zi = (lr + s.hz) * n1 + c;
    const T zv0 = z0[zi], zv1 = z1[zi];
    const T w0v = zv0 + P.sigma * ku0, w1v = zv1 + P.sigma * ku1;
    T zt0, zt1;
    if (hk == PCS_H_L21) {  // w - sigma * (fac * (w/sigma)), penalty.py:551-557
      const T v0 = w0v / P.sigma, v1 = w1v / P.sigma;
      const T nrm = sqrt(v0 * v0 + v1 * v1);
      T f = T(1) - t_h / nrm;
      f = f > T(0) ? f : T(0);
      zt0 = w0v - P.sigma * (f * v0);
      zt1 = w1v - P.sigma * (f * v1);
    } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
      const T v0 = w0v / P.sigma, v1 = w1v / P.sigma;
      zt0 = w0v - P.sigma * (v0 - t_h * clip1(v0 / t_h));
      zt1 = w1v - P.sigma * (v1 - t_h * clip1(v1 / t_h));
    }
    const T zn0v = P.rho * zt0 + P.omr * zv0;
    const T zn1v = P.rho * zt1 + P.omr * zv1;
    zn0[zi] = zn0v;
    zn1[zi] = zn1v;
    const double d0 = (double)zv0 - (double)zn0v, d1 = (double)zv1 - (double)zn1v;
    part[2] += d0 * d0 + d1 * d1;
    part[3] += (double)zv0 * (double)zv0 + (double)zv1 * (double)zv1;
  }
  block_sum<4>(part, red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) partials[(int64_t)blockIdx.x * 4 + k] = part[k];
  }
}

// ---------------------------------------------------------------- loop control
struct Ctrl {
  int32_t it, stopped, min_iter, max_iter, has_dual, hist_len, pad0, pad1;
  double thr;
  double pad2;
};
static_assert(sizeof(Ctrl) == 48, "ctrl layout");

__global__ void k_ctrl_init(Ctrl* c, int min_iter, int max_iter, double thr, int has_dual, int hist_len) {
  c->it = 0;
  c->min_iter = min_iter;
  c->max_iter = max_iter;
  c->thr = thr;
  c->has_dual = has_dual;
  c->hist_len = hist_len;
  const double inf = __builtin_huge_val();
  c->stopped = !((0 <= min_iter) || (0 <= max_iter && inf > thr));
}

__device__ __forceinline__ void finalize_from(const double* v, Ctrl* c, double* hist) {
  const int it = c->it;
  const double inf = __builtin_huge_val();
  // update_diagnostics: ||old - new|| / ||old||, inf if ||old|| == 0 (proxalgs.py:372-383)
  const double rp = (v[1] == 0.0) ? inf : sqrt(v[0]) / sqrt(v[1]);
  const double rd = (v[3] == 0.0) ? inf : sqrt(v[2]) / sqrt(v[3]);
  if (2 * it + 1 < c->hist_len) {
    hist[2 * it] = rp;
    hist[2 * it + 1] = rd;
  }
  const int nx = it + 1;
  c->it = nx;
  // while ((iter <= max_iter) and (stopping_metric() > thr)) or (iter <= min_iter)
  const bool run = (nx <= c->min_iter) || (nx <= c->max_iter && rp > c->thr);
  if (!run || 2 * nx + 1 >= c->hist_len) c->stopped = 1;
}

__global__ __launch_bounds__(256) void k_reduce_partials(const double* __restrict__ part, int64_t np,
                                                         double* __restrict__ sums) {
  __shared__ double red[4 * 4];
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < np; i += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += part[i * 4 + k];
  }
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

__global__ __launch_bounds__(256) void k_reduce_finalize(const double* __restrict__ part, int64_t np, Ctrl* c,
                                                         double* hist) {
  __shared__ double red[4 * 4];
  if (c->stopped) return;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < np; i += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += part[i * 4 + k];
  }
  block_sum<4>(v, red);
  if (threadIdx.x == 0) finalize_from(v, c, hist);
}

// ---------------------------------------------------------------- host dispatch
template <typename T>
static int tile_rows() { return sizeof(T) == 4 ? 32 : 16; }

static int tier_for(int half) {
  if (half <= 3) return 3;
  if (half <= 7) return 7;
  if (half <= 11) return 11;
  if (half <= 15) return 15;
  return -1;
}

template <typename T, int FK, int H>
static int launch_pds2d(const pcs_pds2d_args* a, hipStream_t st) {
  constexpr int TH = sizeof(T) == 4 ? 32 : 16;
  const int tiles_x = (int)((a->n1 + 63) / 64);
  const int tiles_y = (int)((a->rows + TH - 1) / TH);
  const int64_t ntiles = (int64_t)tiles_x * tiles_y;
  if (ntiles > 0x7fffffff) return PCS_EUNSUPPORTED;
  Slab s{a->n0, a->n1, a->row0, a->rows, a->halo_x, a->halo_y, a->halo_z};
  Params<T> P;
  P.tau = (T)a->tau;
  P.sigma = (T)a->sigma;
  P.rho = (T)a->rho;
  P.omr = (T)(1.0 - a->rho);
  P.lam_over_sigma = (T)((1.0 / a->sigma) * a->lam);
  P.step0 = (T)a->step0;
  P.step1 = (T)a->step1;
  P.seg_a = (T)a->seg_a;
  P.seg_b = (T)a->seg_b;
  k_pds2d<T, FK, H, TH><<<(unsigned)ntiles, 256, 0, st>>>(
      (const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, (const T*)a->y, (const T*)a->gbuf, (const T*)a->taps0,
      (const T*)a->taps1, a->half, s, P, a->hkind, a->gkind, a->partials, a->ctrl, tiles_x, (int)ntiles);
  return launch_status();
}

template <typename T>
static int pds2d(const pcs_pds2d_args* a, hipStream_t st) {
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

static int needed_halo_x(int fkind, int half) {
  if (fkind != PCS_F_SEPCONV) return 1;
  const int t = tier_for(half);
  return t < 0 ? -1 : 1 + 2 * t;
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_pds2d_halo_x(int half) { return 1 + 2 * tier_for(half < 0 ? 0 : half); }

int64_t pcs_pds2d_nblocks(const pcs_pds2d_args* a) {
  if (!a) return -1;
  const int th = a->dtype == PCS_F64 ? 16 : 32;
  return ((a->n1 + 63) / 64) * ((a->rows + th - 1) / th);
}

int pcs_pds2d_step(const pcs_pds2d_args* a, hipStream_t st) {
  if (!a || !a->x || !a->xn || !a->z || !a->zn || !a->partials) return PCS_EINVAL;
  if (a->n0 < 1 || a->n1 < 1 || a->rows < 1 || a->row0 < 0 || a->row0 + a->rows > a->n0) return PCS_EINVAL;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return PCS_EINVAL;
  if (a->gkind < PCS_G_NULL || a->gkind > PCS_G_SEGMENT) return PCS_EINVAL;
  if ((a->fkind == PCS_F_DENOISE || a->fkind == PCS_F_SEPCONV) && !a->y) return PCS_EINVAL;
  if (a->fkind == PCS_F_GRADBUF && !a->gbuf) return PCS_EINVAL;
  if (a->fkind == PCS_F_SEPCONV && (!a->taps0 || !a->taps1 || a->half < 0)) return PCS_EINVAL;
  const int hxn = needed_halo_x(a->fkind, a->half);
  if (hxn < 0) return PCS_EUNSUPPORTED;
  const bool multi = a->rows < a->n0;
  if (multi && (a->halo_x < hxn || a->halo_z < 2 ||
                ((a->fkind == PCS_F_SEPCONV) && a->halo_y < 1 + tier_for(a->half)) ||
                ((a->fkind == PCS_F_DENOISE || a->fkind == PCS_F_GRADBUF) && a->halo_y < 1)))
    return PCS_EINVAL;
  if (a->dtype == PCS_F32) return pds2d<float>(a, st);
  if (a->dtype == PCS_F64) return pds2d<double>(a, st);
  return PCS_EINVAL;
}

int64_t pcs_ctrl_bytes(void) { return 64; }

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
  if (!part || !sums || np < 1) return PCS_EINVAL;
  k_reduce_partials<<<1, 256, 0, st>>>(part, np, sums);
  return launch_status();
}

int pcs_pds_finalize(const double* sums, void* ctrl, double* hist, hipStream_t st) {
  if (!sums || !ctrl || !hist) return PCS_EINVAL;
  k_finalize<<<1, 1, 0, st>>>(sums, (Ctrl*)ctrl, hist);
  return launch_status();
}

int pcs_pds_reduce_finalize(const double* part, int64_t np, void* ctrl, double* hist, hipStream_t st) {
  if (!part || !ctrl || !hist || np < 1) return PCS_EINVAL;
  k_reduce_finalize<<<1, 256, 0, st>>>(part, np, (Ctrl*)ctrl, hist);
  return launch_status();
}

}  // extern "C"
