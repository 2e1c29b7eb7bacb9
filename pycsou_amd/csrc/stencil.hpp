// Per-element PyLops 1.x finite-difference stencils (pycsou/linop/diff.py:128 FirstDerivative,
// :218 SecondDerivative; the arithmetic behind :882 Gradient and :957 Laplacian), shared by the
// standalone operators (stencil.hip) and the fused stencil PDS step (pds_gen.hip), so both
// produce the same per-element operation order.  `a` is any array (HBM or LDS), p the element,
// s the stride along the axis, i the element's coordinate along it and n the axis length.
// Operation order follows the NumPy slicing of PyLops 1.x.
#pragma once

#include "common.hpp"

namespace pcs {

// D x at p (FirstDerivative._matvec_{forward,backward,centered})
template <typename T, typename I>
__device__ __forceinline__ T d1_fwd_core(const T* __restrict__ x, I p, I s, I i, I n, T h, int kind, int edge) {
  if (kind == PCS_FORWARD) {
    return (i < n - 1) ? (x[p + s] - x[p]) / h : T(0);
  } else if (kind == PCS_BACKWARD) {
    return (i > 0) ? (x[p] - x[p - s]) / h : T(0);
  }
  if (i > 0 && i < n - 1) return (T(0.5) * x[p + s] - T(0.5) * x[p - s]) / h;
  if (!edge || n < 2) return T(0);
  return (i == 0) ? (x[p + s] - x[p]) / h : (x[p] - x[p - s]) / h;
}

// (D^T y) at p (FirstDerivative._rmatvec_*), accumulation order of the slicing code
template <typename T, typename I>
__device__ __forceinline__ T d1_adj_core(const T* __restrict__ y, I p, I s, I i, I n, T h, int kind, int edge) {
  T acc = T(0);
  if (kind == PCS_FORWARD) {
    if (i < n - 1) acc -= y[p] / h;
    if (i > 0) acc += y[p - s] / h;
  } else if (kind == PCS_BACKWARD) {
    if (i < n - 1) acc -= y[p + s] / h;
    if (i > 0) acc += y[p] / h;
  } else {
    if (i <= n - 3) acc -= (T(0.5) * y[p + s]) / h;
    if (i >= 2) acc += (T(0.5) * y[p - s]) / h;
    if (edge && n >= 2) {
      if (i == 0) acc -= y[p] / h;
      if (i == 1) acc += y[p - s] / h;
      if (i == n - 2) acc -= y[p + s] / h;
      if (i == n - 1) acc += y[p] / h;
    }
  }
  return acc;
}

// SecondDerivative x at p (h2 = sampling^2)
template <typename T, typename I>
__device__ __forceinline__ T d2_fwd_core(const T* __restrict__ x, I p, I s, I i, I n, T h2, int edge) {
  if (i > 0 && i < n - 1) return (x[p + s] - T(2) * x[p] + x[p - s]) / h2;
  if (!edge || n < 3) return T(0);
  if (i == 0) return (x[p] - T(2) * x[p + s] + x[p + 2 * s]) / h2;
  return (x[p - 2 * s] - T(2) * x[p - s] + x[p]) / h2;
}

// SecondDerivative^T y at p
template <typename T, typename I>
__device__ __forceinline__ T d2_adj_core(const T* __restrict__ y, I p, I s, I i, I n, T h2, int edge) {
  T acc = T(0);
  if (i <= n - 3) acc += y[p + s] / h2;
  if (i >= 1 && i <= n - 2) acc -= (T(2) * y[p]) / h2;
  if (i >= 2) acc += y[p - s] / h2;
  if (edge && n >= 3) {
    if (i == 0) acc += y[p] / h2;
    if (i == 1) acc -= (T(2) * y[p - s]) / h2;
    if (i == 2) acc += y[p - 2 * s] / h2;
    if (i == n - 3) acc += y[p + 2 * s] / h2;
    if (i == n - 2) acc -= (T(2) * y[p + s]) / h2;
    if (i == n - 1) acc += y[p] / h2;
  }
  return acc;
}

}  // namespace pcs
