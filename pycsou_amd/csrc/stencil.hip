// Finite-difference operators: FirstDerivative / SecondDerivative / Gradient / Laplacian.
//
// Replaces the PyLops 1.x arithmetic behind pycsou/linop/diff.py:128 (FirstDerivative),
// :218 (SecondDerivative), :882 (Gradient = VStack of FirstDerivative) and :957
// (Laplacian = w0*D2_0 + w1*D2_1).
// Each output element is produced by one thread; neighbour loads are coalesced along
// the contiguous axis and re-used through L1/L2.  The per-element operation order follows
// the NumPy slicing order of PyLops 1.x so that fp64 results agree to the last ulp or two.
#include "common.hpp"
#include "stencil.hpp"

namespace pcs {

struct Geo3 {
  int64_t n[3];   // dims padded to 3 (leading 1s)
  int64_t s[3];   // C-order strides
  int64_t N;
};

static bool make_geo(int ndim, const int64_t* dims, Geo3& g) {
  if (ndim < 1 || ndim > 3 || dims == nullptr) return false;
  int pad = 3 - ndim;
  for (int i = 0; i < 3; ++i) g.n[i] = (i < pad) ? 1 : dims[i - pad];
  for (int i = 0; i < 3; ++i)
    if (g.n[i] < 1) return false;
  g.s[2] = 1;
  g.s[1] = g.n[2];
  g.s[0] = g.n[1] * g.n[2];
  g.N = g.n[0] * g.n[1] * g.n[2];
  return true;
}

// One axis of an N-D C-order array as the middle axis of (outer, n_axis, inner): a derivative
// along that axis sees only the sample's position on it, so any ndim maps onto the 3-D kernels
// with axis index 1 (PyLops 1.x FirstDerivative / SecondDerivative take any ndim).
static constexpr int kMaxDims = 32;
static bool make_geo_axis(int ndim, const int64_t* dims, int axis, Geo3& g) {
  if (ndim < 1 || ndim > kMaxDims || dims == nullptr || axis < 0 || axis >= ndim) return false;
  int64_t outer = 1, inner = 1;
  for (int i = 0; i < ndim; ++i) {
    if (dims[i] < 1) return false;
    if (i < axis) outer *= dims[i];
    if (i > axis) inner *= dims[i];
  }
  const int64_t d3[3] = {outer, dims[axis], inner};
  return make_geo(3, d3, g);
}

__device__ __forceinline__ int64_t coord(const Geo3& g, int64_t p, int a) { return (p / g.s[a]) % g.n[a]; }

// D_a x / D_a^T y at p (stencil.hpp cores with the axis geometry of g)
template <typename T>
__device__ __forceinline__ T d1_fwd_at(const T* __restrict__ x, const Geo3& g, int64_t p, int a, T h, int kind,
                                       int edge) {
  return d1_fwd_core<T, int64_t>(x, p, g.s[a], coord(g, p, a), g.n[a], h, kind, edge);
}
template <typename T>
__device__ __forceinline__ T d1_adj_at(const T* __restrict__ y, const Geo3& g, int64_t p, int a, T h, int kind,
                                       int edge) {
  return d1_adj_core<T, int64_t>(y, p, g.s[a], coord(g, p, a), g.n[a], h, kind, edge);
}

template <typename T>
__global__ void k_deriv1_fwd(const T* __restrict__ x, T* __restrict__ out, Geo3 g, int a, T h, int kind, int edge) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x)
    out[p] = d1_fwd_at(x, g, p, a, h, kind, edge);
}

template <typename T>
__global__ void k_deriv1_adj(const T* __restrict__ y, T* __restrict__ out, Geo3 g, int a, T h, int kind, int edge) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x)
    out[p] = d1_adj_at(y, g, p, a, h, kind, edge);
}

// out += D_a^T y: one Gradient block of an N-D (ndim > 3) adjoint, accumulated in axis order as
// k_grad_adj does (VStack rmatvec sums the blocks in order)
template <typename T>
__global__ void k_deriv1_adj_acc(const T* __restrict__ y, T* __restrict__ out, Geo3 g, int a, T h, int kind,
                                 int edge) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x)
    out[p] = out[p] + d1_adj_at(y, g, p, a, h, kind, edge);
}

template <typename T>
__global__ void k_grad_fwd(const T* __restrict__ x, T* __restrict__ out, Geo3 g, int nd, T h0, T h1, T h2, int kind,
                           int edge) {
  const T hs[3] = {h0, h1, h2};
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x) {
    for (int k = 0; k < nd; ++k) out[k * g.N + p] = d1_fwd_at(x, g, p, 3 - nd + k, hs[k], kind, edge);
  }
}

template <typename T>
__global__ void k_grad_adj(const T* __restrict__ z, T* __restrict__ out, Geo3 g, int nd, T h0, T h1, T h2, int kind,
                           int edge) {
  const T hs[3] = {h0, h1, h2};
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x) {
    T acc = T(0);
    for (int k = 0; k < nd; ++k) acc += d1_adj_at(z + k * g.N, g, p, 3 - nd + k, hs[k], kind, edge);
    out[p] = acc;
  }
}

// SecondDerivative (pylops 1.x) along axis a at p, and its adjoint
template <typename T>
__device__ __forceinline__ T d2_fwd_at(const T* __restrict__ x, const Geo3& g, int64_t p, int a, T h2, int edge) {
  return d2_fwd_core<T, int64_t>(x, p, g.s[a], coord(g, p, a), g.n[a], h2, edge);
}
template <typename T>
__device__ __forceinline__ T d2_adj_at(const T* __restrict__ y, const Geo3& g, int64_t p, int a, T h2, int edge) {
  return d2_adj_core<T, int64_t>(y, p, g.s[a], coord(g, p, a), g.n[a], h2, edge);
}

template <typename T>
__global__ void k_deriv2(const T* __restrict__ x, T* __restrict__ out, Geo3 g, int a, T h2, int edge, int adj) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x)
    out[p] = adj ? d2_adj_at(x, g, p, a, h2, edge) : d2_fwd_at(x, g, p, a, h2, edge);
}

template <typename T>
__global__ void k_lap(const T* __restrict__ x, T* __restrict__ out, Geo3 g, T w0, T w1, T h20, T h21, int edge,
                      int adj) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < g.N; p += (int64_t)gridDim.x * blockDim.x) {
    if (!adj)
      out[p] = w0 * d2_fwd_at(x, g, p, 1, h20, edge) + w1 * d2_fwd_at(x, g, p, 2, h21, edge);
    else
      out[p] = w0 * d2_adj_at(x, g, p, 1, h20, edge) + w1 * d2_adj_at(x, g, p, 2, h21, edge);
  }
}

template <typename T>
static int deriv1(bool adj, const void* in, void* out, int ndim, const int64_t* dims, int axis, double step, int kind,
                  int edge, hipStream_t st) {
  Geo3 g;
  if (!make_geo_axis(ndim, dims, axis, g) || kind < 0 || kind > 2 || !in || !out) return PCS_EINVAL;
  const unsigned grid = grid_for(g.N, 256);
  if (!adj)
    k_deriv1_fwd<T><<<grid, 256, 0, st>>>((const T*)in, (T*)out, g, 1, (T)step, kind, edge);
  else
    k_deriv1_adj<T><<<grid, 256, 0, st>>>((const T*)in, (T*)out, g, 1, (T)step, kind, edge);
  return launch_status();
}

// Gradient of an array with more than 3 axes: one launch per axis block (forward: block k of the
// stacked output; adjoint: the first block written, the others accumulated in axis order)
template <typename T>
static int grad_nd(bool adj, const T* in, T* out, int ndim, const int64_t* dims, const double* steps, int kind,
                   int edge, hipStream_t st) {
  Geo3 g;
  for (int k = 0; k < ndim; ++k)
    if (!make_geo_axis(ndim, dims, k, g)) return PCS_EINVAL;
  const unsigned grid = grid_for(g.N, 256);
  for (int k = 0; k < ndim; ++k) {
    make_geo_axis(ndim, dims, k, g);
    if (!adj)
      k_deriv1_fwd<T><<<grid, 256, 0, st>>>(in, out + k * g.N, g, 1, (T)steps[k], kind, edge);
    else if (k == 0)
      k_deriv1_adj<T><<<grid, 256, 0, st>>>(in, out, g, 1, (T)steps[k], kind, edge);
    else
      k_deriv1_adj_acc<T><<<grid, 256, 0, st>>>(in + k * g.N, out, g, 1, (T)steps[k], kind, edge);
    const int rc = launch_status();
    if (rc != PCS_OK) return rc;
  }
  return PCS_OK;
}

template <typename T>
static int grad(bool adj, const void* in, void* out, int ndim, const int64_t* dims, const double* steps, int kind,
                int edge, hipStream_t st) {
  if (ndim > 3 && kind >= 0 && kind <= 2 && in && out && steps)
    return grad_nd<T>(adj, (const T*)in, (T*)out, ndim, dims, steps, kind, edge, st);
  Geo3 g;
  if (!make_geo(ndim, dims, g) || kind < 0 || kind > 2 || !in || !out || !steps) return PCS_EINVAL;
  const T h0 = (T)steps[0], h1 = ndim > 1 ? (T)steps[1] : T(1), h2 = ndim > 2 ? (T)steps[2] : T(1);
  const unsigned grid = grid_for(g.N, 256);
  if (!adj)
    k_grad_fwd<T><<<grid, 256, 0, st>>>((const T*)in, (T*)out, g, ndim, h0, h1, h2, kind, edge);
  else
    k_grad_adj<T><<<grid, 256, 0, st>>>((const T*)in, (T*)out, g, ndim, h0, h1, h2, kind, edge);
  return launch_status();
}

template <typename T>
static int deriv2(bool adj, const void* in, void* out, int ndim, const int64_t* dims, int axis, double step, int edge,
                  hipStream_t st) {
  Geo3 g;
  if (!make_geo_axis(ndim, dims, axis, g) || !in || !out) return PCS_EINVAL;
  k_deriv2<T><<<grid_for(g.N, 256), 256, 0, st>>>((const T*)in, (T*)out, g, 1, (T)(step * step), edge, adj ? 1 : 0);
  return launch_status();
}

template <typename T>
static int lap(bool adj, const void* in, void* out, const int64_t* dims, const double* w, const double* steps, int edge,
               hipStream_t st) {
  Geo3 g;
  if (!make_geo(2, dims, g) || !in || !out || !w || !steps) return PCS_EINVAL;
  const double h20 = steps[0] * steps[0], h21 = steps[1] * steps[1];
  k_lap<T><<<grid_for(g.N, 256), 256, 0, st>>>((const T*)in, (T*)out, g, (T)w[0], (T)w[1], (T)h20, (T)h21, edge,
                                               adj ? 1 : 0);
  return launch_status();
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_abi_version(void) { return 10; }  // 10: pcs_prox_l21_groups (deterministic label sums); 9: pcs_slab2d_deep_* (communication-avoiding slab loop), pcs_pds_reduce_finalize_k; 8: pcs_pds2d_args fin_partials, pcs_pds_finalize_pending; 7: the persistent 2-D loop (pcs_pds2d_run_persistent, pcs_grid_bar_bytes) removed; 6: pcs_pds2d_args mkind, ym, zm, zmn; 2: pcs_pds2d_args gained kkind, edge, w0, w1; 3: conv_fwd, conv_adj, conv_tier, rbuf; 4: pcs_pds3d_args kkind, edge; 5: pcs_pds3d_args conv0_*

int pcs_deriv1_fwd(int dt, const void* x, void* out, int ndim, const int64_t* dims, int axis, double step, int kind,
                   int edge, hipStream_t st) {
  if (dt == PCS_F32) return deriv1<float>(false, x, out, ndim, dims, axis, step, kind, edge, st);
  if (dt == PCS_F64) return deriv1<double>(false, x, out, ndim, dims, axis, step, kind, edge, st);
  return PCS_EINVAL;
}

int pcs_deriv1_adj(int dt, const void* y, void* out, int ndim, const int64_t* dims, int axis, double step, int kind,
                   int edge, hipStream_t st) {
  if (dt == PCS_F32) return deriv1<float>(true, y, out, ndim, dims, axis, step, kind, edge, st);
  if (dt == PCS_F64) return deriv1<double>(true, y, out, ndim, dims, axis, step, kind, edge, st);
  return PCS_EINVAL;
}

int pcs_deriv2_fwd(int dt, const void* x, void* out, int ndim, const int64_t* dims, int axis, double step, int edge,
                   hipStream_t st) {
  if (dt == PCS_F32) return deriv2<float>(false, x, out, ndim, dims, axis, step, edge, st);
  if (dt == PCS_F64) return deriv2<double>(false, x, out, ndim, dims, axis, step, edge, st);
  return PCS_EINVAL;
}

int pcs_deriv2_adj(int dt, const void* y, void* out, int ndim, const int64_t* dims, int axis, double step, int edge,
                   hipStream_t st) {
  if (dt == PCS_F32) return deriv2<float>(true, y, out, ndim, dims, axis, step, edge, st);
  if (dt == PCS_F64) return deriv2<double>(true, y, out, ndim, dims, axis, step, edge, st);
  return PCS_EINVAL;
}

int pcs_grad_fwd(int dt, const void* x, void* out, int ndim, const int64_t* dims, const double* steps, int kind,
                 int edge, hipStream_t st) {
  if (dt == PCS_F32) return grad<float>(false, x, out, ndim, dims, steps, kind, edge, st);
  if (dt == PCS_F64) return grad<double>(false, x, out, ndim, dims, steps, kind, edge, st);
  return PCS_EINVAL;
}

int pcs_grad_adj(int dt, const void* z, void* out, int ndim, const int64_t* dims, const double* steps, int kind,
                 int edge, hipStream_t st) {
  if (dt == PCS_F32) return grad<float>(true, z, out, ndim, dims, steps, kind, edge, st);
  if (dt == PCS_F64) return grad<double>(true, z, out, ndim, dims, steps, kind, edge, st);
  return PCS_EINVAL;
}

int pcs_lap_fwd(int dt, const void* x, void* out, const int64_t* dims, const double* w, const double* steps, int edge,
                hipStream_t st) {
  if (dt == PCS_F32) return lap<float>(false, x, out, dims, w, steps, edge, st);
  if (dt == PCS_F64) return lap<double>(false, x, out, dims, w, steps, edge, st);
  return PCS_EINVAL;
}

int pcs_lap_adj(int dt, const void* y, void* out, const int64_t* dims, const double* w, const double* steps, int edge,
                hipStream_t st) {
  if (dt == PCS_F32) return lap<float>(true, y, out, dims, w, steps, edge, st);
  if (dt == PCS_F64) return lap<double>(true, y, out, dims, w, steps, edge, st);
  return PCS_EINVAL;
}

}  // extern "C"
