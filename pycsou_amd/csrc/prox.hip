// Proximal operators, projections, vector algebra and deterministic reductions.
//
// Replaces the NumPy bodies of pycsou/func/base.py:239-240 (LpNorm.prox),
// pycsou/func/penalty.py:23-131, 480-668 (L2/SquaredL2/L1/L21 norms, indicator
// projections), pycsou/core/functional.py:207, 264-265 (fenchel_prox, lambda*f),
// pycsou/math/prox.py:167-343 (ball / orthant / segment projections) and the
// np.linalg.norm calls of proxalgs.py:366-394.  All are HBM-bound streaming
// kernels: grid-stride loops, one element per thread per trip.
#include "common.hpp"

namespace pcs {

#define PCS_GRID_LOOP(p, n) \
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < (n); p += (int64_t)gridDim.x * blockDim.x)

template <typename T>
__device__ __forceinline__ T prox_l1_el(T v, T t) {
  // x - tau * proj_linfty_ball(x / tau, 1)
  return v - t * clip1(v / t);
}

template <typename T>
__global__ void k_prox_l1(const T* __restrict__ x, T* __restrict__ out, int64_t n, T tau) {
  PCS_GRID_LOOP(p, n) out[p] = prox_l1_el(x[p], tau);
}

template <typename T>
__global__ void k_fenchel_l1(const T* __restrict__ w, T* __restrict__ out, int64_t n, T sigma, T t) {
  // w - sigma * prox(w / sigma, t), t = (1/sigma)*lam
  PCS_GRID_LOOP(p, n) {
    const T v = w[p];
    out[p] = v - sigma * prox_l1_el(v / sigma, t);
  }
}

template <typename T>
__device__ __forceinline__ T l21_fac(T nrm, T t) {
  // clip(1 - tau / ||x_g||, 0, None); tau/0 = inf -> 0 (penalty.py:554)
  const T f = T(1) - t / nrm;
  return f > T(0) ? f : T(0);
}

template <typename T>
__global__ void k_prox_l21_pixel(const T* __restrict__ x, T* __restrict__ out, int64_t npix, int d, T tau) {
  PCS_GRID_LOOP(p, npix) {
    T s = T(0);
    for (int k = 0; k < d; ++k) {
      const T v = x[k * npix + p];
      s += v * v;
    }
    const T f = l21_fac(sqrt(s), tau);
    for (int k = 0; k < d; ++k) out[k * npix + p] = f * x[k * npix + p];
  }
}

template <typename T>
__global__ void k_fenchel_l21_pixel(const T* __restrict__ w, T* __restrict__ out, int64_t npix, int d, T sigma,
                                    T t) {
  PCS_GRID_LOOP(p, npix) {
    T s = T(0);
    for (int k = 0; k < d; ++k) {
      const T v = w[k * npix + p] / sigma;
      s += v * v;
    }
    const T f = l21_fac(sqrt(s), t);
    for (int k = 0; k < d; ++k) {
      const T wv = w[k * npix + p];
      out[k * npix + p] = wv - sigma * (f * (wv / sigma));
    }
  }
}

template <typename T>
__global__ void k_group_sumsq(const T* __restrict__ x, const int32_t* __restrict__ gid, int64_t n,
                              double* __restrict__ acc) {
  PCS_GRID_LOOP(p, n) {
    const double v = (double)x[p];
    atomicAdd(&acc[gid[p]], v * v);
  }
}

// deterministic group sums (ABI 10): the members of group g are x[order[off[g] .. off[g+1])] in ascending
// element order (a stable argsort of the labels, formed once by the host), summed in that order in fp64 by
// one thread per group (short groups) or by one wave per group (lane-strided partial sums, then a fixed
// butterfly) -- the same sums on every run, unlike the atomic form above
template <typename T>
__global__ void k_group_sumsq_thread(const T* __restrict__ x, const int32_t* __restrict__ order,
                                     const int64_t* __restrict__ off, int64_t ngroups, double* __restrict__ acc) {
  PCS_GRID_LOOP(g, ngroups) {
    double s = 0.0;
    for (int64_t k = off[g]; k < off[g + 1]; ++k) {
      const double v = (double)x[order[k]];
      s += v * v;
    }
    acc[g] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_group_sumsq_wave(const T* __restrict__ x, const int32_t* __restrict__ order,
                                                          const int64_t* __restrict__ off, int64_t ngroups,
                                                          double* __restrict__ acc) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < ngroups; g += nw) {
    double s = 0.0;
    for (int64_t k = off[g] + lane; k < off[g + 1]; k += 64) {
      const double v = (double)x[order[k]];
      s += v * v;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if (lane == 0) acc[g] = s;
  }
}

template <typename T>
__global__ void k_group_scale(const T* __restrict__ x, const int32_t* __restrict__ gid, int64_t n,
                              const double* __restrict__ acc, T tau, T* __restrict__ out) {
  PCS_GRID_LOOP(p, n) {
    const T f = l21_fac((T)sqrt(acc[gid[p]]), tau);
    out[p] = f * x[p];
  }
}

template <typename T>
__global__ void k_prox_l2(const T* __restrict__ x, T* __restrict__ out, int64_t n, T tau, const double* __restrict__ ss) {
  // LpNorm.prox with proj_l2_ball (func/base.py:239-240, math/prox.py:207-210):
  //   v = x/tau ; out = x - tau * (||v|| <= 1 ? v : (1*v)/||v||)
  const T nv = (T)(sqrt(*ss) / (double)tau);
  PCS_GRID_LOOP(p, n) {
    const T v = x[p] / tau;
    out[p] = x[p] - tau * ((nv <= T(1)) ? v : v / nv);
  }
}

template <typename T>
__global__ void k_prox_sql2(const T* __restrict__ x, T* __restrict__ out, int64_t n, T den) {
  PCS_GRID_LOOP(p, n) out[p] = x[p] / den;
}

template <typename T>
__global__ void k_proj_nonneg(const T* __restrict__ x, T* __restrict__ out, int64_t n) {
  PCS_GRID_LOOP(p, n) {
    const T v = x[p];
    out[p] = (v < T(0)) ? T(0) : v;
  }
}

template <typename T>
__global__ void k_proj_segment(const T* __restrict__ x, T* __restrict__ out, int64_t n, T a, T b) {
  PCS_GRID_LOOP(p, n) {
    T v = x[p];
    v = (v < a) ? a : v;
    out[p] = (v > b) ? b : v;
  }
}

template <typename T>
__global__ void k_axpby(const T* __restrict__ x, const T* __restrict__ y, T* __restrict__ out, int64_t n, T a, T b) {
  if (y) {
    PCS_GRID_LOOP(p, n) out[p] = a * x[p] + b * y[p];
  } else {
    PCS_GRID_LOOP(p, n) out[p] = a * x[p];
  }
}

template <typename T>
__global__ void k_sub2(const T* __restrict__ x, const T* __restrict__ y, const T* __restrict__ w, T* __restrict__ out,
                       int64_t n, T a, T b) {
  PCS_GRID_LOOP(p, n) out[p] = (x[p] - a * y[p]) - b * w[p];
}

template <typename T>
__global__ void k_mul(const T* __restrict__ x, const T* __restrict__ d, T* __restrict__ out, int64_t n) {
  PCS_GRID_LOOP(p, n) out[p] = d[p] * x[p];
}

constexpr int kRedBlocks = 1024;

// both sums of one relative improvement in one pass: part[b] = (sum (a-b)^2, sum a^2) of block b
template <typename T>
__global__ __launch_bounds__(256) void k_relsums_stage1(const T* __restrict__ old, const T* __restrict__ nw,
                                                        int64_t n, double* __restrict__ part) {
  __shared__ double sm[8];
  double v[2] = {0.0, 0.0};
  PCS_GRID_LOOP(p, n) {
    const double a = (double)old[p], dd = a - (double)nw[p];
    v[0] += dd * dd;
    v[1] += a * a;
  }
  block_sum<2>(v, sm);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = v[0];
    part[2 * blockIdx.x + 1] = v[1];
  }
}

__global__ __launch_bounds__(256) void k_relsums_stage2(const double* __restrict__ part, int np,
                                                        double* __restrict__ out) {
  __shared__ double sm[8];
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    v[0] += part[2 * i];
    v[1] += part[2 * i + 1];
  }
  block_sum<2>(v, sm);
  if (threadIdx.x == 0) {
    out[0] = v[0];
    out[1] = v[1];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_reduce_stage1(int kind, const T* __restrict__ x, const T* __restrict__ y,
                                                       int64_t n, double* __restrict__ part) {
  __shared__ double sm[4];
  double v[1] = {0.0};
  PCS_GRID_LOOP(p, n) {
    const double a = (double)x[p];
    switch (kind) {
      case 0: v[0] += a * a; break;
      case 1: v[0] += fabs(a); break;
      case 2: { const double dd = a - (double)y[p]; v[0] += dd * dd; } break;
      default: v[0] += a * (double)y[p]; break;
    }
  }
  block_sum<1>(v, sm);
  if (threadIdx.x == 0) part[blockIdx.x] = v[0];
}

__global__ __launch_bounds__(256) void k_reduce_stage2(const double* __restrict__ part, int np,
                                                       double* __restrict__ out) {
  __shared__ double sm[4];
  double v[1] = {0.0};
  for (int i = threadIdx.x; i < np; i += blockDim.x) v[0] += part[i];
  block_sum<1>(v, sm);
  if (threadIdx.x == 0) *out = v[0];
}

template <typename T>
static int reduce(int kind, const void* x, const void* y, int64_t n, double* out, void* ws, hipStream_t st) {
  if (!out || !ws || n < 0 || kind < 0 || kind > 3) return PCS_EINVAL;
  if (n > 0 && (!x || (kind >= 2 && !y))) return PCS_EINVAL;
  const unsigned g = grid_for(n, 256, kRedBlocks);
  k_reduce_stage1<T><<<g, 256, 0, st>>>(kind, (const T*)x, (const T*)y, n, (double*)ws);
  k_reduce_stage2<<<1, 256, 0, st>>>((const double*)ws, (int)g, out);
  return launch_status();
}

// One fused AcceleratedProximalGradientDescent.update_iterand + update_diagnostics
// (pycsou/opt/proxalgs.py:586-601, 612-622) given g = grad F(x) (computed by F's operators):
//   x_t = G.prox(x - tau g, tau)        G: null / NonNegativeOrthant / Segment / lam*L1Norm
//   x'  = x_t + a (x_t - aux)           aux = previous x_t ('past_aux'), a = (t_old - 1) / t
// plus per-block partials of ||x - x'||^2 and ||x||^2 (stage 2: k_apgd_sums, fixed order).
template <typename T>
__global__ __launch_bounds__(256) void k_apgd_step(const T* __restrict__ x, const T* __restrict__ g,
                                                   const T* __restrict__ aux, T* __restrict__ xn, T* __restrict__ auxn,
                                                   int64_t n, T tau, T a, int gk, T thr, T sa, T sb,
                                                   double* __restrict__ part) {
  __shared__ double sm[8];
  double v[2] = {0.0, 0.0};
  PCS_GRID_LOOP(p, n) {
    const T xv = x[p];
    T w = xv - tau * g[p];
    if (gk == PCS_APGD_G_L1) {
      w = prox_l1_el(w, thr);  // lam*L1: prox(x, tau*lam)  (functional.py:264-265, base.py:239-240)
    } else if (gk == PCS_G_NONNEG) {
      w = (w < T(0)) ? T(0) : w;  // math/prox.py:295-297
    } else if (gk == PCS_G_SEGMENT) {
      w = (w < sa) ? sa : w;  // math/prox.py:340-343
      w = (w > sb) ? sb : w;
    }
    const T xnew = w + a * (w - aux[p]);
    auxn[p] = w;
    xn[p] = xnew;
    const double d = (double)xv - (double)xnew;
    v[0] += d * d;
    v[1] += (double)xv * (double)xv;
  }
  block_sum<2>(v, sm);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = v[0];
    part[2 * blockIdx.x + 1] = v[1];
  }
}

__global__ __launch_bounds__(256) void k_apgd_sums(const double* __restrict__ part, int np, double* __restrict__ out) {
  __shared__ double sm[8];
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    v[0] += part[2 * i];
    v[1] += part[2 * i + 1];
  }
  block_sum<2>(v, sm);
  if (threadIdx.x == 0) {
    out[0] = v[0];
    out[1] = v[1];
  }
}

}  // namespace pcs

using namespace pcs;

#define PCS_DISPATCH(dt, ...)                            \
  do {                                                   \
    if ((dt) == PCS_F32) {                               \
      using T = float;                                   \
      __VA_ARGS__;                                       \
    } else if ((dt) == PCS_F64) {                        \
      using T = double;                                  \
      __VA_ARGS__;                                       \
    } else {                                             \
      return PCS_EINVAL;                                 \
    }                                                    \
  } while (0)

extern "C" {

int pcs_prox_l1(int dt, const void* x, void* out, int64_t n, double tau, hipStream_t st) {
  if (!x || !out || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_prox_l1<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (T*)out, n, (T)tau));
  return launch_status();
}

int pcs_fenchel_l1(int dt, const void* w, void* out, int64_t n, double sigma, double lam, hipStream_t st) {
  if (!w || !out || n < 0) return PCS_EINVAL;
  const double t = (1.0 / sigma) * lam;
  PCS_DISPATCH(dt, k_fenchel_l1<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)w, (T*)out, n, (T)sigma, (T)t));
  return launch_status();
}

int pcs_prox_l21_pixel(int dt, const void* x, void* out, int64_t npix, int d, double tau, hipStream_t st) {
  if (!x || !out || npix < 0 || d < 1) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_prox_l21_pixel<T><<<grid_for(npix, 256), 256, 0, st>>>((const T*)x, (T*)out, npix, d, (T)tau));
  return launch_status();
}

int pcs_fenchel_l21_pixel(int dt, const void* w, void* out, int64_t npix, int d, double sigma, double lam,
                          hipStream_t st) {
  if (!w || !out || npix < 0 || d < 1) return PCS_EINVAL;
  const double t = (1.0 / sigma) * lam;
  PCS_DISPATCH(dt, k_fenchel_l21_pixel<T><<<grid_for(npix, 256), 256, 0, st>>>((const T*)w, (T*)out, npix, d,
                                                                                (T)sigma, (T)t));
  return launch_status();
}

int pcs_prox_l21_labels(int dt, const void* x, void* out, int64_t n, const int32_t* gid, int64_t ngroups, double tau,
                        void* ws, hipStream_t st) {
  if (!x || !out || !gid || !ws || n < 0 || ngroups < 1) return PCS_EINVAL;
  if (hipMemsetAsync(ws, 0, sizeof(double) * (size_t)ngroups, st) != hipSuccess) return PCS_ELAUNCH;
  PCS_DISPATCH(dt, k_group_sumsq<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, gid, n, (double*)ws);
               k_group_scale<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, gid, n, (const double*)ws, (T)tau,
                                                                  (T*)out));
  return launch_status();
}

int pcs_prox_l21_groups(int dt, const void* x, void* out, int64_t n, const int32_t* gid, int64_t ngroups,
                        const int32_t* order, const int64_t* off, int64_t maxlen, double tau, void* ws, hipStream_t st) {
  if (!x || !out || !gid || !order || !off || !ws || n < 0 || ngroups < 1 || maxlen < 0) return PCS_EINVAL;
  if (maxlen <= 32) {
    PCS_DISPATCH(dt, k_group_sumsq_thread<T><<<grid_for(ngroups, 256), 256, 0, st>>>((const T*)x, order, off, ngroups,
                                                                                    (double*)ws));
  } else {
    const int64_t nb = (ngroups + 3) / 4;
    PCS_DISPATCH(dt, k_group_sumsq_wave<T><<<(unsigned)(nb < 65536 ? nb : 65536), 256, 0, st>>>(
                         (const T*)x, order, off, ngroups, (double*)ws));
  }
  PCS_DISPATCH(dt, k_group_scale<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, gid, n, (const double*)ws, (T)tau,
                                                                      (T*)out));
  return launch_status();
}

int pcs_prox_l2(int dt, const void* x, void* out, int64_t n, double tau, const double* ss, hipStream_t st) {
  if (!x || !out || !ss || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_prox_l2<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (T*)out, n, (T)tau, ss));
  return launch_status();
}

int pcs_prox_sql2(int dt, const void* x, void* out, int64_t n, double tau, hipStream_t st) {
  if (!x || !out || n < 0) return PCS_EINVAL;
  const double den = 1.0 + 2.0 * tau;
  PCS_DISPATCH(dt, k_prox_sql2<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (T*)out, n, (T)den));
  return launch_status();
}

int pcs_proj_nonneg(int dt, const void* x, void* out, int64_t n, hipStream_t st) {
  if (!x || !out || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_proj_nonneg<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (T*)out, n));
  return launch_status();
}

int pcs_proj_segment(int dt, const void* x, void* out, int64_t n, double a, double b, hipStream_t st) {
  if (!x || !out || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_proj_segment<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (T*)out, n, (T)a, (T)b));
  return launch_status();
}

int pcs_axpby(int dt, const void* x, const void* y, void* out, int64_t n, double a, double b, hipStream_t st) {
  if (!x || !out || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_axpby<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (const T*)y, (T*)out, n, (T)a, (T)b));
  return launch_status();
}

int pcs_mul(int dt, const void* x, const void* d, void* out, int64_t n, hipStream_t st) {
  if (!x || !d || !out || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_mul<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (const T*)d, (T*)out, n));
  return launch_status();
}

int pcs_rel_sums(int dt, const void* old, const void* nw, int64_t n, double* out_dev, void* ws, hipStream_t st) {
  if (!old || !nw || !out_dev || !ws || n < 0) return PCS_EINVAL;
  const unsigned g = grid_for(n, 256, kRedBlocks / 2);
  PCS_DISPATCH(dt, k_relsums_stage1<T><<<g, 256, 0, st>>>((const T*)old, (const T*)nw, n, (double*)ws));
  k_relsums_stage2<<<1, 256, 0, st>>>((const double*)ws, (int)g, out_dev);
  return launch_status();
}

int pcs_sub2(int dt, const void* x, const void* y, const void* w, void* out, int64_t n, double a, double b,
             hipStream_t st) {
  if (!x || !y || !w || !out || n < 0) return PCS_EINVAL;
  PCS_DISPATCH(dt, k_sub2<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)x, (const T*)y, (const T*)w, (T*)out, n,
                                                               (T)a, (T)b));
  return launch_status();
}

int64_t pcs_reduce_ws_bytes(void) { return (int64_t)sizeof(double) * 2 * kRedBlocks; }

int pcs_apgd_step(int dt, const void* x, const void* g, const void* aux, void* xn, void* aux_n, int64_t n, double tau,
                  double a, int gkind, double lam, double seg_a, double seg_b, double* sums_dev, void* ws,
                  hipStream_t st) {
  if (!x || !g || !aux || !xn || !aux_n || !sums_dev || !ws || n < 0) return PCS_EINVAL;
  if (gkind != PCS_G_NULL && gkind != PCS_G_NONNEG && gkind != PCS_G_SEGMENT && gkind != PCS_APGD_G_L1)
    return PCS_EINVAL;
  if (xn == x || xn == aux || aux_n == x || aux_n == aux || xn == aux_n) return PCS_EINVAL;
  if (gkind == PCS_APGD_G_L1 && !(tau * lam > 0)) return PCS_EINVAL;
  const unsigned gr = grid_for(n, 256, kRedBlocks);
  PCS_DISPATCH(dt, k_apgd_step<T><<<gr, 256, 0, st>>>((const T*)x, (const T*)g, (const T*)aux, (T*)xn, (T*)aux_n, n,
                                                       (T)tau, (T)a, gkind, (T)(tau * lam), (T)seg_a, (T)seg_b,
                                                       (double*)ws));
  k_apgd_sums<<<1, 256, 0, st>>>((const double*)ws, (int)gr, sums_dev);
  return launch_status();
}

int pcs_reduce(int dt, int kind, const void* x, const void* y, int64_t n, double* out, void* ws, hipStream_t st) {
  if (dt == PCS_F32) return reduce<float>(kind, x, y, n, out, ws, st);
  if (dt == PCS_F64) return reduce<double>(kind, x, y, n, out, ws, st);
  return PCS_EINVAL;
}

}  // extern "C"
