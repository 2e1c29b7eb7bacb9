// Sampling operators: Masking / DownSampling / SubSampling (pycsou/linop/sampling.py:25-391).
//
// Forward  y = x[idx]                  (Masking.__call__ x[sampling_bool], sampling.py:192-193;
//                                       SubSampling -> pylops.Restriction.matvec)
// Adjoint  x = 0; x[idx] = y           (Masking.adjoint, sampling.py:195-198; Restriction.rmatvec)
// The host turns the boolean mask / index list into int32 gather indices once.  The adjoint is
// written as a gather too: out[p] = inv[p] >= 0 ? y[inv[p]] : 0 with inv the inverse map
// (last index wins for repeated indices, as NumPy's fancy assignment does), so every output
// element is written exactly once by one thread: coalesced stores, no zero-fill pass, no races.
// HBM-bound: idx/inv (4 B) + data per element, grid-stride, one element per thread per trip.
#include "common.hpp"

namespace pcs {

template <typename T>
__global__ void k_gather(const T* __restrict__ x, const int32_t* __restrict__ idx, T* __restrict__ out, int64_t m) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = x[idx[i]];
}

template <typename T>
__global__ void k_gather_or_zero(const T* __restrict__ y, const int32_t* __restrict__ inv, T* __restrict__ out,
                                 int64_t n) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t j = inv[p];
    out[p] = j >= 0 ? y[j] : T(0);
  }
}

template <typename T>
static int gather(const void* x, const int32_t* idx, void* out, int64_t m, hipStream_t st) {
  if (m == 0) return PCS_OK;
  k_gather<T><<<grid_for(m, 256), 256, 0, st>>>((const T*)x, idx, (T*)out, m);
  return launch_status();
}

template <typename T>
static int gather_or_zero(const void* y, const int32_t* inv, void* out, int64_t n, hipStream_t st) {
  if (n == 0) return PCS_OK;
  k_gather_or_zero<T><<<grid_for(n, 256), 256, 0, st>>>((const T*)y, inv, (T*)out, n);
  return launch_status();
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_gather(int dt, const void* x, const int32_t* idx, void* out, int64_t m, hipStream_t st) {
  if (m < 0 || (m > 0 && (!x || !idx || !out))) return PCS_EINVAL;
  if (dt == PCS_F32) return gather<float>(x, idx, out, m, st);
  if (dt == PCS_F64) return gather<double>(x, idx, out, m, st);
  return PCS_EINVAL;
}

int pcs_gather_or_zero(int dt, const void* y, const int32_t* inv, void* out, int64_t n, hipStream_t st) {
  if (n < 0 || (n > 0 && (!inv || !out))) return PCS_EINVAL;
  if (dt == PCS_F32) return gather_or_zero<float>(y, inv, out, n, st);
  if (dt == PCS_F64) return gather_or_zero<double>(y, inv, out, n, st);
  return PCS_EINVAL;
}

}  // extern "C"
