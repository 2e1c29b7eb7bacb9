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

// ---- the same stencils on a 5-sample window w[k] = a[i + k - 2] along one axis (the fused
// row- and plane-marching steps: pds_smarch.hpp, pds3d.hip);
// INT: the sample is known to lie >= 2 samples inside the axis (no edge rule applies).  hipcc
// contracts a * b + c freely (-ffp-contract=fast ignores the fp pragmas), so every formula here is
// written with no mul feeding an add -- (difference) * step, or an explicit fma -- and the interior
// and the edge instantiations of a sample give the same bits: a pixel's result does not depend on
// which row step or slab it falls in (slabs are bitwise equal to the whole image)
__device__ __forceinline__ float pcs_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double pcs_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

template <int KIND, bool INT, typename T>
__device__ __forceinline__ T sw_d1_fwd(const T (&w)[5], int i, int n, T ih, int edge) {
  if constexpr (KIND == PCS_FORWARD) {
    const T c = (w[3] - w[2]) * ih;
    return (INT || i < n - 1) ? c : T(0);
  } else if constexpr (KIND == PCS_BACKWARD) {
    const T c = (w[2] - w[1]) * ih;
    return (INT || i > 0) ? c : T(0);
  } else {
    const T c = (w[3] - w[1]) * (T(0.5) * ih);
    if constexpr (INT) return c;
    const T e = (i == 0) ? (w[3] - w[2]) * ih : (w[2] - w[1]) * ih;
    return (i > 0 && i < n - 1) ? c : ((edge && n >= 2) ? e : T(0));
  }
}
// The adjoints return the stencil sum in sample units (the caller scales by 1/h): only adds and the
// exact halving/doubling happen in here, so contraction has nothing to choose between
template <int KIND, bool INT, typename T>
__device__ __forceinline__ T sw_d1_adj(const T (&w)[5], int i, int n, int edge) {
  if constexpr (KIND == PCS_FORWARD) {  // -w[2] [i < n-1] + w[1] [i > 0]
    const T t2 = (INT || i < n - 1) ? w[2] : T(0);
    const T t1 = (INT || i > 0) ? w[1] : T(0);
    return t1 - t2;
  } else if constexpr (KIND == PCS_BACKWARD) {
    const T t3 = (INT || i < n - 1) ? w[3] : T(0);
    const T t2 = (INT || i > 0) ? w[2] : T(0);
    return t2 - t3;
  } else {
    const T t3 = (INT || i <= n - 3) ? w[3] : T(0);
    const T t1 = (INT || i >= 2) ? w[1] : T(0);
    T acc = T(0.5) * (t1 - t3);
    if constexpr (!INT) {  // only rows within 2 of an edge, which INT never covers
      // selects in the rules' order (n = 2, 3 apply several), the uniform edge test folded into each:
      // an `if (edge ...)` here is a scalar branch per sample and axis, which splits the plane march's
      // unrolled item loops into basic blocks of ~8 instructions (k_pds3d_gen's border tiles ran 1.5x
      // their interior time, profiles/r5_g3d_edge_ab.txt)
      const bool e = edge && n >= 2;
      acc = (e && i == 0) ? acc - w[2] : acc;
      acc = (e && i == 1) ? acc + w[1] : acc;
      acc = (e && i == n - 2) ? acc - w[3] : acc;
      acc = (e && i == n - 1) ? acc + w[2] : acc;
    }
    return acc;
  }
}
template <bool INT, typename T>
__device__ __forceinline__ T sw_d2_fwd(const T (&w)[5], int i, int n, T ih2, int edge) {
  const T c = ((w[3] - T(2) * w[2]) + w[1]) * ih2;  // 2 w exact: contracting the inner sub is exact
  if constexpr (INT) return c;
  const T e = (i == 0) ? ((w[2] - T(2) * w[3]) + w[4]) * ih2 : ((w[0] - T(2) * w[1]) + w[2]) * ih2;
  return (i > 0 && i < n - 1) ? c : ((edge && n >= 3) ? e : T(0));
}
template <bool INT, typename T>
__device__ __forceinline__ T sw_d2_adj(const T (&w)[5], int i, int n, int edge) {
  const T t3 = (INT || i <= n - 3) ? w[3] : T(0);
  const T t2 = (INT || (i >= 1 && i <= n - 2)) ? w[2] : T(0);
  const T t1 = (INT || i >= 2) ? w[1] : T(0);
  T acc = (t3 - T(2) * t2) + t1;
  if constexpr (!INT) {  // selects in the rules' order, the edge test folded in (sw_d1_adj)
    const bool e = edge && n >= 3;
    acc = (e && i == 0) ? acc + w[2] : acc;
    acc = (e && i == 1) ? acc - T(2) * w[1] : acc;
    acc = (e && i == 2) ? acc + w[0] : acc;
    acc = (e && i == n - 3) ? acc + w[4] : acc;
    acc = (e && i == n - 2) ? acc - T(2) * w[3] : acc;
    acc = (e && i == n - 1) ? acc + w[2] : acc;
  }
  return acc;
}

}  // namespace pcs
