// Direct 'same' zero-boundary convolutions (general PSF / taps).
//
// Replaces pylops.signalprocessing.Convolve2D / Convolve1D (1.x) behind
// pycsou/linop/conv.py:294 and :163, which call scipy.signal.convolve / correlate.
//   out[i] = sum_j h[j] x[i + off - j]          (convolution, forward)
// The adjoint (correlation) is the same call with the flipped filter and
// off' = k-1-off (the host side caches the flipped copy).
//
// conv2d: LDS-tiled.  A 256-thread block owns a TH x 64 output tile; the input
// apron (TH+kh-1) x (64+kw-1) and the PSF are staged in LDS once, each thread
// accumulates a column of TH/4 outputs with a rolling register window over the
// apron rows so every LDS value read feeds up to TH/4 FMAs.
#include "common.hpp"

namespace pcs {

constexpr int kConvTW = 64;   // tile width (one wave of columns)
constexpr int kConvTH = 32;   // tile height
constexpr int kConvRPT = kConvTH / 4;  // rows per thread (4 row groups of 64 threads)
constexpr int kConvMaxK = 31;  // max kh, kw of the LDS-tiled kernel (LDS <= 64 KiB at fp64)

template <typename T>
__global__ __launch_bounds__(256) void k_conv2d(const T* __restrict__ x, T* __restrict__ out, int64_t n0,
                                                 int64_t n1, const T* __restrict__ psf, int kh, int kw, int off0,
                                                 int off1, const T* __restrict__ b, T beta) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const int AH = kConvTH + kh - 1, AW = kConvTW + kw - 1;
  const int AP = AW | 1;  // odd pitch: column reads are bank-conflict free
  T* ap = sm;             // apron  [AH][AP]
  T* hp = sm + AH * AP;   // psf    [kh][kw]
  const int64_t r0 = (int64_t)blockIdx.y * kConvTH, c0 = (int64_t)blockIdx.x * kConvTW;
  // apron origin: input row for tile row 0 and tap j0 = kh-1 is r0 + off0 - (kh-1)
  const int64_t ar = r0 + off0 - (kh - 1), ac = c0 + off1 - (kw - 1);
  for (int i = threadIdx.x; i < kh * kw; i += blockDim.x) hp[i] = psf[i];
  for (int e = threadIdx.x; e < AH * AW; e += blockDim.x) {
    const int rr = e / AW, cc = e - rr * AW;
    const int64_t gr = ar + rr, gc = ac + cc;
    ap[rr * AP + cc] = (gr >= 0 && gr < n0 && gc >= 0 && gc < n1) ? x[gr * n1 + gc] : T(0);
  }
  __syncthreads();
  const int tc = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int rbase = tg * kConvRPT;
  T acc[kConvRPT];
#pragma unroll
  for (int m = 0; m < kConvRPT; ++m) acc[m] = T(0);
  // out[rbase+m][tc] = sum_{j0,j1} h[j0][j1] * ap[rbase + m + kh-1-j0][tc + kw-1-j1]
  for (int j1 = 0; j1 < kw; ++j1) {
    const int col = tc + kw - 1 - j1;
    for (int q = 0; q < kConvRPT + kh - 1; ++q) {
      const T v = ap[(rbase + q) * AP + col];
#pragma unroll
      for (int m = 0; m < kConvRPT; ++m) {
        const int j0 = m + kh - 1 - q;
        if (j0 >= 0 && j0 < kh) acc[m] += hp[j0 * kw + j1] * v;
      }
    }
  }
  const int64_t gc = c0 + tc;
  if (gc < n1) {
#pragma unroll
    for (int m = 0; m < kConvRPT; ++m) {
      const int64_t gr = r0 + rbase + m;
      if (gr < n0) {
        T o = acc[m];
        if (b) o = o + beta * b[gr * n1 + gc];
        out[gr * n1 + gc] = o;
      }
    }
  }
}

// Fallback for very large PSFs: one thread per output, taps from global (cached).
template <typename T>
__global__ void k_conv2d_big(const T* __restrict__ x, T* __restrict__ out, int64_t n0, int64_t n1,
                             const T* __restrict__ psf, int kh, int kw, int off0, int off1, const T* __restrict__ b,
                             T beta) {
  const int64_t N = n0 * n1;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = p / n1, j = p - i * n1;
    T acc = T(0);
    for (int j0 = 0; j0 < kh; ++j0) {
      const int64_t r = i + off0 - j0;
      if (r < 0 || r >= n0) continue;
      for (int j1 = 0; j1 < kw; ++j1) {
        const int64_t c = j + off1 - j1;
        if (c >= 0 && c < n1) acc += psf[j0 * kw + j1] * x[r * n1 + c];
      }
    }
    if (b) acc = acc + beta * b[p];
    out[p] = acc;
  }
}

// conv1d along axis a of a (padded) 3-D array: out[p] = sum_t h[t] x[p + (off-t) s_a].
template <typename T>
__global__ void k_conv1d(const T* __restrict__ x, T* __restrict__ out, int64_t N, int64_t na, int64_t sa,
                         const T* __restrict__ h, int k, int off) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = (p / sa) % na;
    T acc = T(0);
    for (int t = 0; t < k; ++t) {
      const int64_t q = i + off - t;
      if (q >= 0 && q < na) acc += h[t] * x[p + (off - t) * sa];
    }
    out[p] = acc;
  }
}

template <typename T>
static int conv2d(const void* x, void* out, int64_t n0, int64_t n1, const void* psf, int kh, int kw, int off0,
                  int off1, const void* b, double beta, hipStream_t st) {
  if (!x || !out || !psf || n0 < 1 || n1 < 1 || kh < 1 || kw < 1 || off0 < 0 || off0 >= kh || off1 < 0 ||
      off1 >= kw)
    return PCS_EINVAL;
  if (kh <= kConvMaxK && kw <= kConvMaxK) {
    const int AH = kConvTH + kh - 1, AW = kConvTW + kw - 1, AP = AW | 1;
    const size_t lds = sizeof(T) * (size_t)(AH * AP + kh * kw);
    dim3 grid((unsigned)((n1 + kConvTW - 1) / kConvTW), (unsigned)((n0 + kConvTH - 1) / kConvTH));
    if (grid.y > 65535) return PCS_EUNSUPPORTED;
    k_conv2d<T><<<grid, 256, lds, st>>>((const T*)x, (T*)out, n0, n1, (const T*)psf, kh, kw, off0, off1,
                                        (const T*)b, (T)beta);
  } else {
    k_conv2d_big<T><<<grid_for(n0 * n1, 256), 256, 0, st>>>((const T*)x, (T*)out, n0, n1, (const T*)psf, kh, kw,
                                                            off0, off1, (const T*)b, (T)beta);
  }
  return launch_status();
}

template <typename T>
static int conv1d(const void* x, void* out, int ndim, const int64_t* dims, int axis, const void* taps, int k, int off,
                  hipStream_t st) {
  if (!x || !out || !taps || !dims || ndim < 1 || ndim > 3 || axis < 0 || axis >= ndim || k < 1 || off < 0 ||
      off >= k)
    return PCS_EINVAL;
  int64_t N = 1, sa = 1;
  for (int i = 0; i < ndim; ++i) N *= dims[i];
  for (int i = axis + 1; i < ndim; ++i) sa *= dims[i];
  k_conv1d<T><<<grid_for(N, 256), 256, 0, st>>>((const T*)x, (T*)out, N, dims[axis], sa, (const T*)taps, k, off);
  return launch_status();
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_conv2d(int dt, const void* x, void* out, int64_t n0, int64_t n1, const void* psf, int kh, int kw, int off0,
               int off1, const void* b, double beta, hipStream_t st) {
  if (dt == PCS_F32) return conv2d<float>(x, out, n0, n1, psf, kh, kw, off0, off1, b, beta, st);
  if (dt == PCS_F64) return conv2d<double>(x, out, n0, n1, psf, kh, kw, off0, off1, b, beta, st);
  return PCS_EINVAL;
}

int pcs_conv1d(int dt, const void* x, void* out, int ndim, const int64_t* dims, int axis, const void* taps, int k,
               int off, hipStream_t st) {
  if (dt == PCS_F32) return conv1d<float>(x, out, ndim, dims, axis, taps, k, off, st);
  if (dt == PCS_F64) return conv1d<double>(x, out, ndim, dims, axis, taps, k, off, st);
  return PCS_EINVAL;
}

}  // extern "C"
