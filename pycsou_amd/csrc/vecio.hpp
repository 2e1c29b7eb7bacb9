// 16-byte vector I/O helpers shared by the separable-convolution kernels (conv.hip, sep_ata.hip).
#pragma once

#include "common.hpp"

namespace pcs {

template <typename T>
struct V16 {  // 16 bytes of T
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};
template <typename T>
__device__ __forceinline__ V16<T> ldv(const T* p) {
  V16<T> r;
  *reinterpret_cast<uint4*>(r.v) = *reinterpret_cast<const uint4*>(p);
  return r;
}
template <typename T>
__device__ __forceinline__ void stv(T* p, const V16<T>& r) {
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(r.v);
}

template <typename T>
struct Q4 {
  T v[4];
};
template <typename T>
__device__ __forceinline__ Q4<T> ldq(const T* p) {  // 4 elements, 16-B aligned
  Q4<T> r;
  constexpr int VN = V16<T>::N;
#pragma unroll
  for (int h = 0; h < 4 / VN; ++h) {
    const V16<T> v = ldv(p + h * VN);
#pragma unroll
    for (int e = 0; e < VN; ++e) r.v[h * VN + e] = v.v[e];
  }
  return r;
}
// LDS read of 4 elements that stays whole 16-B ds_read_b128 (volatile, LDS address space):
// otherwise hipcc narrows a read whose edge elements are unused into ds_read2_b32 pairs
// (32-bank, 2-4 way conflicts)
template <typename T>
__device__ __forceinline__ Q4<T> ldsq(const T* p) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const volatile u4* lds_u4;
  Q4<T> r;
  constexpr int VN = V16<T>::N;
#pragma unroll
  for (int h = 0; h < 4 / VN; ++h) {
    const u4 v = ((lds_u4)(p))[h];
    __builtin_memcpy(r.v + h * VN, &v, 16);
  }
  return r;
}
template <typename T>
__device__ __forceinline__ void stq(T* p, const Q4<T>& r) {
  constexpr int VN = V16<T>::N;
#pragma unroll
  for (int h = 0; h < 4 / VN; ++h) {
    V16<T> v;
#pragma unroll
    for (int e = 0; e < VN; ++e) v.v[e] = r.v[h * VN + e];
    stv(p + h * VN, v);
  }
}

}  // namespace pcs
