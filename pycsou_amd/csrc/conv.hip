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
#include "vecio.hpp"

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

// ---- fast paths for taps k <= 15 (zero-padded to 15: out[j] = sum_{t<15} h'[t] x[j + off - t])
constexpr int kC1K = 15;

// Strided axis (stride sa >= 16 B, 16-B aligned rows): a thread owns 16 B of consecutive inner
// elements and RUN consecutive outputs along the axis; every input row it streams feeds up to
// 15 outputs held in registers (coalesced 16-B loads, each input read once per run).
template <typename T, int RUN>
__global__ __launch_bounds__(256) void k_conv1d_strided(const T* __restrict__ x, T* __restrict__ out, int64_t outer,
                                                         int64_t na, int64_t sa, const T* __restrict__ taps, int k,
                                                         int off) {
  constexpr int VN = V16<T>::N;
  T h[kC1K];
#pragma unroll
  for (int t = 0; t < kC1K; ++t) h[t] = t < k ? taps[t] : T(0);
  const int64_t ng = sa / VN, nrun = (na + RUN - 1) / RUN;
  const int64_t total = outer * nrun * ng;
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cg = id % ng, rest = id / ng, jr = rest % nrun, o = rest / nrun;
    const int64_t j0 = jr * RUN;
    const T* xb = x + o * na * sa + cg * VN;
    T acc[RUN][VN];
#pragma unroll
    for (int m = 0; m < RUN; ++m)
#pragma unroll
      for (int e = 0; e < VN; ++e) acc[m][e] = T(0);
    // input row u = j0 + off - (15-1) + q feeds output m with tap t = m + 14 - q
#pragma unroll
    for (int q = 0; q < RUN + kC1K - 1; ++q) {
      const int64_t u = j0 + off - (kC1K - 1) + q;
      V16<T> v;
      if (u >= 0 && u < na) {
        v = ldv(xb + u * sa);
      } else {
#pragma unroll
        for (int e = 0; e < VN; ++e) v.v[e] = T(0);
      }
#pragma unroll
      for (int m = 0; m < RUN; ++m) {
        const int t = m + kC1K - 1 - q;
        if (t >= 0 && t < kC1K) {
#pragma unroll
          for (int e = 0; e < VN; ++e) acc[m][e] += h[t] * v.v[e];
        }
      }
    }
    T* ob = out + o * na * sa + cg * VN;
#pragma unroll
    for (int m = 0; m < RUN; ++m) {
      if (j0 + m < na) {
        V16<T> r;
#pragma unroll
        for (int e = 0; e < VN; ++e) r.v[e] = acc[m][e];
        stv(ob + (j0 + m) * sa, r);
      }
    }
  }
}

// Contiguous axis (stride 1): TPR threads own a TPR*16-byte segment of one row (staged in LDS
// with a 16-B aligned halo of >= 14 elements each side); a 256-thread block holds 256/TPR such
// row segments (short rows: several rows per block, no idle lanes).  Thread i of a segment
// computes the 16 B of outputs at 16*i from 16-B LDS reads.  SHIFT = (16 + off - 14) mod VN
// selects the window alignment at compile time.
template <typename T, int SHIFT, int TPR>
__global__ __launch_bounds__(256) void k_conv1d_contig(const T* __restrict__ x, T* __restrict__ out, int64_t rows,
                                                        int64_t na, const T* __restrict__ taps, int k, int off) {
  constexpr int VN = V16<T>::N;
  constexpr int SEG = TPR * VN;         // outputs per row segment
  constexpr int RPB = 256 / TPR;        // row segments per block
  constexpr int HALO = 16;              // elements (multiple of VN, >= 14)
  constexpr int SP = SEG + 2 * HALO + 2 * VN;  // LDS elements per segment
  constexpr int NW = (VN + kC1K - 1 + SHIFT + VN - 1) / VN;  // 16-B reads per window
  __shared__ __attribute__((aligned(16))) T sm[RPB * SP];
  T h[kC1K];
#pragma unroll
  for (int t = 0; t < kC1K; ++t) h[t] = t < k ? taps[t] : T(0);
  const int64_t nseg = (na + SEG - 1) / SEG;
  const int sub = threadIdx.x / TPR, i = threadIdx.x - sub * TPR;
  const int64_t task = (int64_t)blockIdx.x * RPB + sub;
  const int64_t r = task / nseg, sgi = task - r * nseg;
  const bool live = r < rows;
  const int64_t c0 = sgi * SEG;
  const T* xr = x + (live ? r : 0) * na;
  T* ss = sm + sub * SP;
  // stage [c0 - HALO, c0 + SEG + HALO) (zero outside the row), 16 B per thread-load
  for (int e = i; e < (SEG + 2 * HALO) / VN; e += TPR) {
    const int64_t c = c0 - HALO + (int64_t)e * VN;
    V16<T> v;
    if (c >= 0 && c + VN <= na) {
      v = ldv(xr + c);
    } else {
#pragma unroll
      for (int q = 0; q < VN; ++q) v.v[q] = (c + q >= 0 && c + q < na) ? xr[c + q] : T(0);
    }
    stv(ss + e * VN, v);
  }
  __syncthreads();
  if (!live) return;
  // outputs j = c0 + VN*i + m read inputs j + off - t, t < 15: LDS index
  // VN*i + m + HALO + off - 14 + (14 - t); window start (aligned) base = VN*i + ((HALO + off - 14) & ~(VN-1))
  const int start = HALO + off - (kC1K - 1);  // >= 2 since off >= 0
  const int abase = VN * i + (start & ~(VN - 1));
  T w[NW * VN];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    V16<T> v;  // whole ds_read_b128 (volatile LDS read: no narrowing into ds_read2_b32)
    {
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) const volatile u4* lds_u4;
      const u4 raw = *(lds_u4)(ss + abase + q * VN);
      __builtin_memcpy(v.v, &raw, 16);
    }
#pragma unroll
    for (int e = 0; e < VN; ++e) w[q * VN + e] = v.v[e];
  }
  V16<T> o;
#pragma unroll
  for (int m = 0; m < VN; ++m) {
    T acc = T(0);
#pragma unroll
    for (int t = 0; t < kC1K; ++t) acc += h[t] * w[SHIFT + m + (kC1K - 1 - t)];
    o.v[m] = acc;
  }
  const int64_t j = c0 + VN * i;
  if (j + VN <= na) {
    stv(out + r * na + j, o);
  } else {
#pragma unroll
    for (int m = 0; m < VN; ++m)
      if (j + m < na) out[r * na + j + m] = o.v[m];
  }
}

template <typename T, int TPR>
static void launch_contig(const T* x, T* out, int64_t rows, int64_t na, const T* taps, int k, int off, hipStream_t st) {
  constexpr int VN = V16<T>::N;
  const int64_t nseg = (na + TPR * VN - 1) / (TPR * VN);
  const unsigned g = (unsigned)((rows * nseg + 256 / TPR - 1) / (256 / TPR));
  switch ((16 + off - (kC1K - 1)) & (VN - 1)) {
    case 0: k_conv1d_contig<T, 0, TPR><<<g, 256, 0, st>>>(x, out, rows, na, taps, k, off); break;
    case 1: k_conv1d_contig<T, 1, TPR><<<g, 256, 0, st>>>(x, out, rows, na, taps, k, off); break;
    case 2: k_conv1d_contig<T, 2, TPR><<<g, 256, 0, st>>>(x, out, rows, na, taps, k, off); break;
    default: k_conv1d_contig<T, 3, TPR><<<g, 256, 0, st>>>(x, out, rows, na, taps, k, off); break;
  }
}

// VP adjacent voxels per thread (one VP-wide load / store per plane and array): the same per-voxel sums
template <typename T, int VP>
struct alignas(sizeof(T) * VP) C0Vec {
  T v[VP];
};
template <typename T, int KT, int VP>
__global__ __launch_bounds__(256) void k_conv0_rta(const T* __restrict__ tin, const T* __restrict__ y, T* __restrict__ s,
                                                   int64_t nsub, int64_t plane, const T* __restrict__ taps, int k,
                                                   int off, int64_t img_lo, int64_t img_hi, int64_t q0, int64_t q1) {
  using V = C0Vec<T, VP>;
  const int64_t pos = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VP;  // plane % VP == 0 (host)
  if (pos >= plane) return;
  T h[KT], hf[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    h[t] = t < k ? taps[t] : T(0);
    hf[t] = t < k ? taps[k - 1 - t] : T(0);
  }
  const int64_t p0 = q0 + k - 2 * KT + 1;  // first plane loaded: both windows full at the first output
  const int64_t nsteps = (q1 + k - 2) - p0 + 1;
  const int64_t nblk = (nsteps + KT - 1) / KT;
  const int64_t lo = img_lo > 0 ? img_lo : 0, hi = img_hi < nsub ? img_hi : nsub;
  T tw[KT][VP], rw[KT][VP];
  V tl[KT], yl[KT];
#pragma unroll
  for (int u = 0; u < KT; ++u)
#pragma unroll
    for (int m = 0; m < VP; ++m) tw[u][m] = rw[u][m] = T(0);
  auto load_blk = [&](int64_t b, V (&tv)[KT], V (&yv)[KT]) {
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int64_t p = p0 + b * KT + u, pr = p - off;
      const bool tin_ok = p >= 0 && p < nsub, y_ok = pr >= lo && pr < hi;
      const V a = *reinterpret_cast<const V*>(tin + (tin_ok ? p : 0) * plane + pos);
      const V c = *reinterpret_cast<const V*>(y + (y_ok ? pr : lo) * plane + pos);
#pragma unroll
      for (int m = 0; m < VP; ++m) {
        tv[u].v[m] = tin_ok ? a.v[m] : T(0);
        yv[u].v[m] = y_ok ? c.v[m] : T(0);
      }
    }
  };
  if (nblk > 0) load_blk(0, tl, yl);
  for (int64_t b = 0; b < nblk; ++b) {
    V tn[KT], yn[KT];
    if (b + 1 < nblk) load_blk(b + 1, tn, yn);
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int64_t p = p0 + b * KT + u, pr = p - off, q = p - k + 1;
      V out;
#pragma unroll
      for (int m = 0; m < VP; ++m) {
        tw[u][m] = tl[u].v[m];
        T acc = T(0);
#pragma unroll
        for (int t = 0; t < KT; ++t) acc += h[t] * tw[(u - t + KT) % KT][m];
        rw[u][m] = (pr >= lo && pr < hi) ? acc - yl[u].v[m] : T(0);
        T sacc = T(0);
#pragma unroll
        for (int t = 0; t < KT; ++t) sacc += hf[t] * rw[(u - t + KT) % KT][m];
        out.v[m] = sacc;
      }
      if (q >= q0 && q < q1) *reinterpret_cast<V*>(s + q * plane + pos) = out;
    }
    if (b + 1 < nblk) {
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        tl[u] = tn[u];
        yl[u] = yn[u];
      }
    }
  }
}

// fp32 voxels per thread of the axis-0 pass (diagnostics builds override): 2 = 8-B loads / stores, 512 voxels
// (2 KB) of a plane per workgroup
#ifndef PCS_CONV0_VP32
#define PCS_CONV0_VP32 2
#endif

template <typename T>
static int conv0_rta(const void* t, const void* y, void* s, int64_t nsub, int64_t plane, const void* taps, int k, int off,
                     int64_t img_lo, int64_t img_hi, int64_t q0, int64_t q1, hipStream_t st) {
  if (!t || !y || !s || !taps || nsub < 1 || plane < 1 || k < 1 || k > kC1K || off < 0 || off >= k || q0 < 0 ||
      q1 > nsub || q0 > q1)
    return PCS_EINVAL;
  if (q0 == q1) return PCS_OK;
  constexpr int VPW = sizeof(T) == 4 ? PCS_CONV0_VP32 : 1;
  const bool wide = VPW > 1 && plane % VPW == 0 && ((uintptr_t)t | (uintptr_t)y | (uintptr_t)s) % (VPW * sizeof(T)) == 0;
  const int vp = wide ? VPW : 1;
  const unsigned g = (unsigned)((plane / vp + 255) / 256);
  auto go = [&](auto kt, auto vpc) {
    constexpr int KT = decltype(kt)::value, VP = decltype(vpc)::value;
    k_conv0_rta<T, KT, VP><<<g, 256, 0, st>>>((const T*)t, (const T*)y, (T*)s, nsub, plane, (const T*)taps, k, off,
                                              img_lo, img_hi, q0, q1);
  };
  using K7 = std::integral_constant<int, 7>;
  using K15 = std::integral_constant<int, kC1K>;
  using V1 = std::integral_constant<int, 1>;
  using VW = std::integral_constant<int, VPW>;
  if (k <= 7) {
    if (wide) go(K7{}, VW{});
    else go(K7{}, V1{});
  } else {
    if (wide) go(K15{}, VW{});
    else go(K15{}, V1{});
  }
  return launch_status();
}

// ---- two Convolve1D along axes 1 and 2 of every plane of a 3-D array in one pass
// (the in-plane part of a separable 3-D blur, pycsou/linop/conv.py:20-164):
//   VFIRST:  out = C_b(C_a(in)),   !VFIRST: out = C_a(C_b(in)),
// C_a along axis 1 (taps ha, ka, offa), C_b along axis 2 (taps hb, kb, offb), zero boundary.
// A block computes a TY x 64 tile of one plane: the input tile with its halo (TY + 14 rows,
// 64 + 32 columns, zeros outside the plane) is staged in LDS once, the first pass writes an LDS
// intermediate, the second pass writes the output: 2 sub-volume passes instead of 4.  Each
// output is the same t-ascending sum as pcs_conv1d's.
constexpr int64_t kSep2DBlocks = 1024;

// vertical pass over an LDS buffer: acc[r] = sum_t ha[t] rows[i + r + KT - 1 - t] at column c;
// each of the RB + KT - 1 rows is read once, bottom up (t ascending per output, as pcs_conv1d)
template <typename T, int RB, int KT>
__device__ __forceinline__ void sep_vpass(const T* buf, int pitch, int i, int c, const T (&ha)[KT], Q4<T> (&acc)[RB]) {
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[r].v[m] = T(0);
#pragma unroll
  for (int j = RB + KT - 2; j >= 0; --j) {
    const Q4<T> v = ldsq(buf + (i + j) * pitch + c);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int t = r + KT - 1 - j;
      if (t >= 0 && t < KT) {
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[r].v[m] += ha[t] * v.v[m];
      }
    }
  }
}

template <typename T>
struct Sep2D {
  static constexpr int KT = kC1K, TX = 64, CH = 16, WC = TX + 2 * CH, GC = WC / 4;
  static constexpr int TY = sizeof(T) == 4 ? 32 : 16, NR = TY + KT - 1;
};

template <typename T, int SHIFT, bool VFIRST, bool VEC>
__global__ __launch_bounds__(256) void k_sep2d(const T* __restrict__ in, T* __restrict__ out, int64_t nplanes, int64_t n1,
                                               int64_t n2, const T* __restrict__ ha_, int ka, int offa,
                                               const T* __restrict__ hb_, int kb, int offb) {
  using S = Sep2D<T>;
  constexpr int KT = S::KT, TX = S::TX, CH = S::CH, WC = S::WC, GC = S::GC, TY = S::TY, NR = S::NR;
  constexpr int SZ_IN = NR * WC, SZ_MID = VFIRST ? TY * WC : NR * TX;
  __shared__ __attribute__((aligned(16))) T sm[SZ_IN + SZ_MID];
  T* tin = sm;
  T* mid = sm + SZ_IN;
  T ha[KT], hb[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    ha[t] = t < ka ? ha_[t] : T(0);
    hb[t] = t < kb ? hb_[t] : T(0);
  }
  const int64_t ty = (n1 + TY - 1) / TY, tx = (n2 + TX - 1) / TX, ntiles = nplanes * ty * tx;
  const int tid = threadIdx.x;
  constexpr bool vec = VEC;
  // persistent blocks: tile b + gridDim.x's input is loaded into registers while tile b computes
  // stage rows [i0 + offa - 14, i0 + TY + offa), columns [j0 - 16, j0 + 80)
  constexpr int NL = (NR * GC + 255) / 256;
  Q4<T> q[NL];
  // tile b: plane b / (ty tx), then column strip, row tile fastest (vertical neighbours, which
  // share 14 halo rows, are consecutive)
  auto tile_of = [&](int64_t b, int64_t& pl, int64_t& i0, int64_t& j0) {
    pl = b / (ty * tx);
    const int64_t rem = b - pl * (ty * tx), sj = rem / ty;
    i0 = (rem - sj * ty) * TY;
    j0 = sj * TX;
  };
  auto load_tile = [&](int64_t b) {
    int64_t pl, i0, j0;
    tile_of(b, pl, i0, j0);
    const T* src = in + pl * n1 * n2;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = min(l * 256 + tid, NR * GC - 1);
      const int rl = e / GC, g = e - (e / GC) * GC;
      const int64_t gi = i0 + offa - (KT - 1) + rl, gc = j0 - CH + 4 * g;
      const bool rin = gi >= 0 && gi < n1;
      // branch-free (clamped address + select): a load inside a divergent branch makes the
      // compiler wait for it before the next one is issued
      if (VEC) {
        const bool ok = rin && gc >= 0 && gc + 4 <= n2;
        const Q4<T> v = ldq(src + (ok ? gi * n2 + gc : 0));
#pragma unroll
        for (int m = 0; m < 4; ++m) q[l].v[m] = ok ? v.v[m] : T(0);
      } else {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const bool ok = rin && gc + m >= 0 && gc + m < n2;
          const T v = src[ok ? gi * n2 + gc + m : 0];
          q[l].v[m] = ok ? v : T(0);
        }
      }
    }
  };
  // horizontal window: outputs at tile column c (multiple of 4) read tile columns
  // c + CH + offb - 14 + (14 - t); aligned start c + ((CH + offb - 14) & ~3), SHIFT the rest
  constexpr int NW = (4 + KT - 1 + SHIFT + 3) / 4;
  const int hb0 = (CH + offb - (KT - 1)) & ~3;
  auto hpass = [&](const T* row, int c, Q4<T>& o) {  // row: LDS row base; c: first output col in the row's frame
    T w[NW * 4];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const Q4<T> v = ldsq(row + c + hb0 + 4 * u);
#pragma unroll
      for (int e = 0; e < 4; ++e) w[4 * u + e] = v.v[e];
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T acc = T(0);
#pragma unroll
      for (int t = 0; t < KT; ++t) acc += hb[t] * w[SHIFT + m + (KT - 1 - t)];
      o.v[m] = acc;
    }
  };
  // LDS lane maps: every 16-lane ds_read_b128 group reads 16 distinct 16-B slots of one row
  const int half = tid >> 5, l5 = tid & 31, lgrp = lane_grp(l5), lidx = lane_idx(l5);
  // XCD-aware persistent schedule: the blocks of one XCD (b % 8) walk one contiguous eighth of
  // the tile order together, so halo rows re-read by a neighbour tile hit that XCD's L2
  int64_t first = blockIdx.x, stride = gridDim.x, last = ntiles;
  if (gridDim.x % 8 == 0) {
    const int64_t xcd = blockIdx.x % 8, nbx = gridDim.x / 8;
    first = xcd * ntiles / 8 + blockIdx.x / 8;
    last = (xcd + 1) * ntiles / 8;
    stride = nbx;
  }
  int64_t b = first;
  if (b < last) load_tile(b);
  for (; b < last; b += stride) {
    int64_t pl, i0, j0;
    tile_of(b, pl, i0, j0);
    T* dst = out + pl * n1 * n2;
    auto store = [&](int i, int c, const Q4<T>& o) {  // tile row i, tile col c (multiple of 4)
      const int64_t gi = i0 + i, gc = j0 + c;
      if (gi >= n1) return;
      if (vec && gc + 4 <= n2) {
        stq(dst + gi * n2 + gc, o);
      } else {
#pragma unroll
        for (int m = 0; m < 4; ++m)
          if (gc + m < n2) dst[gi * n2 + gc + m] = o.v[m];
      }
    };
    __syncthreads();  // the previous tile's passes are done with tin / mid
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = l * 256 + tid;
      if (e < NR * GC) stq(tin + (e / GC) * WC + 4 * (e - (e / GC) * GC), q[l]);
    }
    __syncthreads();
    if (b + stride < last) load_tile(b + stride);
    if (VFIRST) {
      // mid[i][c] (i < TY, all WC columns) = vertical pass: 32 lanes per block of RB rows
      constexpr int RB = TY / 8;
      for (int rb = half; rb < TY / RB; rb += 8) {
        const int g = row_lane_group<GC>(l5);
        Q4<T> acc[RB];
        sep_vpass<T, RB, KT>(tin, WC, rb * RB, 4 * g, ha, acc);
#pragma unroll
        for (int r = 0; r < RB; ++r) stq(mid + (rb * RB + r) * WC + 4 * g, acc[r]);
      }
      __syncthreads();
      for (int i = 2 * half + lgrp; i < TY; i += 16) {
        Q4<T> o;
        hpass(mid + i * WC, 4 * lidx, o);
        store(i, 4 * lidx, o);
      }
    } else {
      // mid[r][c] (all NR rows, TX columns) = horizontal pass
      for (int r = 2 * half + lgrp; r < NR; r += 16) {
        Q4<T> o;
        hpass(tin + r * WC, 4 * lidx, o);
        stq(mid + r * TX + 4 * lidx, o);
      }
      __syncthreads();
      constexpr int RB = 2;
      for (int rb = 2 * half + lgrp; rb < TY / RB; rb += 16) {
        Q4<T> acc[RB];
        sep_vpass<T, RB, KT>(mid, TX, rb * RB, 4 * lidx, ha, acc);
#pragma unroll
        for (int r = 0; r < RB; ++r) store(rb * RB + r, 4 * lidx, acc[r]);
      }
    }
  }
}

// ---- row-marching separable in-plane convolution (horizontal pass first) ----------------
// A workgroup owns a 128-column strip of a plane and marches down a range of its rows, 16 rows
// per step.  Each input row segment (148 columns from the aligned start of the tap window,
// zeros outside the plane) is loaded from HBM once per strip, staged in LDS, its horizontal
// pass (taps hb) lands in a 32-row LDS ring, and the vertical pass (taps ha) of 16 output rows
// reads the ring: no vertical halo is recomputed (k_sep2d re-reads and re-filters 14 halo rows
// per 32-row tile).  Work: tasks = (plane, row segment, strip), strip fastest, the segment count
// from a cost model (waves of resident workgroups x (rows + 14-row prologue) per task), run by
// a persistent loop (each task restarts the march).  The
// XCD-aware map gives the blocks of one XCD consecutive tasks at any moment, i.e. neighbouring
// strips of the same rows: the 128-B lines of the 20 halo columns they share are read from HBM
// once and hit the XCD's L2 for the neighbour (PMC: 1.43x the input bytes when neighbouring
// strips ran at different rows).  Sums are k_sep2d's (t ascending per output).
template <typename T>
struct SepM {
  // fp32: 32 rows per step (one step's loads must cover the HBM latency: ~19 KB per block in
  // flight); fp64: 16 rows (LDS: 3 blocks per CU)
  static constexpr int KT = kC1K, TX = 128, G = TX / 4, GI = G + 5, WI = 4 * GI;
  static constexpr int RS = sizeof(T) == 4 ? 32 : 16, RING = 2 * RS, RB = RS / 8, NH = RS / 8;
  static constexpr int NL = (RS * GI + 255) / 256;
  static_assert(RS + KT - 1 <= RING && (RING & (RING - 1)) == 0, "ring holds the 14 rows above a step");
  static_assert(G == 32 && (RS / RB) * G == 256, "one vertical item (RB rows) and NH horizontal rows per thread");
};

struct SepCur {  // a step of the march: task t (plane, segment, strip), rows [a, b), step s of ns
  int64_t t, plane;
  int strip, a, b, s, ns;
};

template <typename T, int SHIFT, bool VEC>
__global__ __launch_bounds__(256) void k_sep2d_march(const T* __restrict__ in, T* __restrict__ out, int n1, int n2,
                                                     int nstrips, int nseg, int seg_len, int64_t ntasks,
                                                     const T* __restrict__ ha_, int ka, int offa,
                                                     const T* __restrict__ hb_, int kb, int S0) {
  using S = SepM<T>;
  constexpr int KT = S::KT, TX = S::TX, GI = S::GI, WI = S::WI, RS = S::RS, RING = S::RING, RB = S::RB, NL = S::NL,
                NH = S::NH;
  constexpr int NW = (SHIFT + KT + 3 + 3) / 4;  // Q4 slots of one horizontal window
  __shared__ __attribute__((aligned(16))) T stg[RS * WI];
  __shared__ __attribute__((aligned(16))) T ring[RING * TX];
  T ha[KT], hb[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    ha[t] = t < ka ? ha_[t] : T(0);
    hb[t] = t < kb ? hb_[t] : T(0);
  }
  // XCD-aware task map: XCD x (blocks b % 8 == x, nbx of them) owns a contiguous share of the
  // task list proportional to nbx; its k-th block takes lo + k, lo + k + nbx, ... so that the
  // blocks running together on one XCD work on consecutive tasks
  int64_t t0, t_end, t_stride;
  {
    const int64_t b = blockIdx.x, nb = gridDim.x, xcd = b % 8, k = b / 8, q = nb / 8, r = nb % 8;
    const int64_t nbx = q + (xcd < r ? 1 : 0);
    const int64_t before = xcd * q + (xcd < r ? xcd : r);  // blocks of the XCDs below x
    const int64_t lo = ntasks * before / nb, hi = ntasks * (before + nbx) / nb;
    t0 = lo + k;
    t_end = hi;
    t_stride = nbx;
  }
  if (t0 >= t_end) return;
  const int tid = threadIdx.x, g = tid & 31, hrow = tid >> 5;
  auto task_at = [&](int64_t t) {  // the first step of task t
    SepCur c;
    c.t = t;
    const int64_t per_plane = (int64_t)nseg * nstrips;
    c.plane = t / per_plane;
    const int rem = (int)(t - c.plane * per_plane), seg = rem / nstrips;
    c.strip = rem - seg * nstrips;
    c.a = seg * seg_len;
    c.b = min(n1, c.a + seg_len);
    c.s = 0;
    c.ns = (c.b - c.a + KT - 1 + RS - 1) / RS;
    return c;
  };
  Q4<T> q[NL];
  // loads of step c: input rows k = s RS + rr (global row a + offa - 14 + k) of the piece
  auto prefetch = [&](const SepCur& c) {
    const int j0 = c.strip * TX;
    const T* src = in + c.plane * (int64_t)n1 * n2;
    const int kmax = c.b - c.a + KT - 2;  // last input row any output of [a, b) reads
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = min(l * 256 + tid, RS * GI - 1);
      const int rr = e / GI, qq = e - (e / GI) * GI;
      const int k = c.s * RS + rr, gi = c.a + offa - (KT - 1) + k, gc = j0 + S0 + 4 * qq;
      const bool rin = gi >= 0 && gi < n1 && k <= kmax;
      if (VEC) {
        const bool ok = rin && gc >= 0 && gc + 4 <= n2;
        const Q4<T> v = ldq(src + (ok ? (int64_t)gi * n2 + gc : 0));
#pragma unroll
        for (int m = 0; m < 4; ++m) q[l].v[m] = ok ? v.v[m] : T(0);
      } else {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const bool ok = rin && gc + m >= 0 && gc + m < n2;
          const T v = src[ok ? (int64_t)gi * n2 + gc + m : 0];
          q[l].v[m] = ok ? v : T(0);
        }
      }
    }
  };
  SepCur cur = task_at(t0);
  prefetch(cur);
  for (;;) {
    // staging <- the landed rows of this step (slot e = row * GI + group: pitch WI)
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = l * 256 + tid;
      if (e < RS * GI) stq(stg + 4 * e, q[l]);
    }
    lds_barrier();  // staging landed; the previous step's vertical pass is done with the ring
    SepCur nxt = cur;
    bool more = true;
    if (cur.s + 1 < cur.ns) {
      nxt.s = cur.s + 1;
    } else {
      more = cur.t + t_stride < t_end;
      if (more) nxt = task_at(cur.t + t_stride);
    }
    if (more) prefetch(nxt);
    // horizontal pass: rows hrow + 8 h of the step, output group g -> ring slot of row k
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int i = hrow + 8 * h;
      T w[NW * 4];
#pragma unroll
      for (int u = 0; u < NW; ++u) {
        const Q4<T> v = ldsq(stg + i * WI + 4 * (g + u));
#pragma unroll
        for (int e = 0; e < 4; ++e) w[4 * u + e] = v.v[e];
      }
      Q4<T> o;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        T acc = T(0);
#pragma unroll
        for (int t = 0; t < KT; ++t) acc += hb[t] * w[SHIFT + m + (KT - 1 - t)];
        o.v[m] = acc;
      }
      stq(ring + ((cur.s * RS + i) & (RING - 1)) * TX + 4 * g, o);
    }
    lds_barrier();
    // vertical pass: output rows a - 14 + s RS + 2 hrow + r read ring rows k - 14 .. k
    {
      const int r0 = RB * hrow, kb0 = cur.s * RS + r0 - (KT - 1);
      Q4<T> acc[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[r].v[m] = T(0);
#pragma unroll
      for (int j = RB + KT - 2; j >= 0; --j) {
        const Q4<T> v = ldsq(ring + ((kb0 + j) & (RING - 1)) * TX + 4 * g);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int t = r + KT - 1 - j;
          if (t >= 0 && t < KT) {
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[r].v[m] += ha[t] * v.v[m];
          }
        }
      }
      const int gc = cur.strip * TX + 4 * g;
      T* dst = out + cur.plane * (int64_t)n1 * n2;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int o = cur.a - (KT - 1) + cur.s * RS + r0 + r;
        if (o < cur.a || o >= cur.b) continue;
        if (VEC) {
          if (gc < n2) stq(dst + (int64_t)o * n2 + gc, acc[r]);
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (gc + m < n2) dst[(int64_t)o * n2 + gc + m] = acc[r].v[m];
        }
      }
    }
    if (!more) break;
    cur = nxt;
  }
}

// resident workgroups of k_sep2d_march<T> on the device (queried once per type)
template <typename T>
static int sep_march_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sep2d_march<T, 0, true>, 256, 0) != hipSuccess || nb < 1)
      nb = 2;
    (void)hipGetLastError();
    slots = cus * nb;
    const char* e = getenv("PCS_SEP2D_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

template <typename T>
static void launch_sep2d_march(const void* in, void* out, int64_t np, int64_t n1, int64_t n2, const void* ha, int ka,
                               int offa, const void* hb, int kb, int offb, hipStream_t st) {
  using S = SepM<T>;
  const int64_t nstrips = (n2 + S::TX - 1) / S::TX, pieces = np * nstrips;
  const int d = offb - (S::KT - 1);  // first tap-window column relative to the output column
  const int S0 = d >= 0 ? 0 : -((-d + 3) / 4) * 4, shift = d - S0;
  const int64_t slots = sep_march_slots<T>();
  // row segments: the count that minimises (waves of resident workgroups) x (rows per task +
  // the 14-row prologue), segments of >= 32 rows (thin sub-volumes -- the boundary bands of
  // the multi-GPU schedule -- get few long segments, large volumes about 8+ tasks per block)
  const int64_t max_seg = n1 / 32 > 1 ? n1 / 32 : 1;
  int64_t nseg = 1, best = -1;
  for (int64_t c = 1; c <= max_seg; ++c) {
    const int64_t len = (n1 + c - 1) / c, waves = (pieces * c + slots - 1) / slots;
    const int64_t cost = waves * (len + S::KT - 1);
    if (best < 0 || cost < best) {
      best = cost;
      nseg = c;
    }
  }
  const int64_t seg_len = (n1 + nseg - 1) / nseg;
  nseg = (n1 + seg_len - 1) / seg_len;
  const int64_t ntasks = pieces * nseg;
  const int64_t grid = ntasks < slots ? ntasks : slots;
  auto args = [&](auto kern) {
    kern<<<(unsigned)grid, 256, 0, st>>>((const T*)in, (T*)out, (int)n1, (int)n2, (int)nstrips, (int)nseg,
                                         (int)seg_len, ntasks, (const T*)ha, ka, offa, (const T*)hb, kb, S0);
  };
  const bool vec = n2 % 4 == 0;
  switch (shift) {
    case 0: vec ? args(k_sep2d_march<T, 0, true>) : args(k_sep2d_march<T, 0, false>); break;
    case 1: vec ? args(k_sep2d_march<T, 1, true>) : args(k_sep2d_march<T, 1, false>); break;
    case 2: vec ? args(k_sep2d_march<T, 2, true>) : args(k_sep2d_march<T, 2, false>); break;
    default: vec ? args(k_sep2d_march<T, 3, true>) : args(k_sep2d_march<T, 3, false>); break;
  }
}

template <typename T, bool VFIRST>
static void launch_sep2d(const void* in, void* out, int64_t np, int64_t n1, int64_t n2, const void* ha, int ka, int offa,
                         const void* hb, int kb, int offb, hipStream_t st) {
  using S = Sep2D<T>;
  const int64_t nt = np * ((n1 + S::TY - 1) / S::TY) * ((n2 + S::TX - 1) / S::TX);
  // persistent: ~4 blocks per CU, a multiple of 8 (XCDs) when the tiles allow
  static int64_t cap = 0;
  if (cap == 0) {  // PCS_SEP2D_BLOCKS: diagnostics override of the persistent grid
    const char* e = getenv("PCS_SEP2D_BLOCKS");
    cap = e ? atoll(e) : kSep2DBlocks;
    if (cap < 8) cap = kSep2DBlocks;
  }
  const unsigned g = (unsigned)(nt >= cap ? cap : nt);
  auto args = [&](auto kern) {
    kern<<<g, 256, 0, st>>>((const T*)in, (T*)out, np, n1, n2, (const T*)ha, ka, offa, (const T*)hb, kb, offb);
  };
  if (n2 % 4 == 0) {
    switch ((S::CH + offb - (S::KT - 1)) & 3) {
      case 0: args(k_sep2d<T, 0, VFIRST, true>); break;
      case 1: args(k_sep2d<T, 1, VFIRST, true>); break;
      case 2: args(k_sep2d<T, 2, VFIRST, true>); break;
      default: args(k_sep2d<T, 3, VFIRST, true>); break;
    }
  } else {
    switch ((S::CH + offb - (S::KT - 1)) & 3) {
      case 0: args(k_sep2d<T, 0, VFIRST, false>); break;
      case 1: args(k_sep2d<T, 1, VFIRST, false>); break;
      case 2: args(k_sep2d<T, 2, VFIRST, false>); break;
      default: args(k_sep2d<T, 3, VFIRST, false>); break;
    }
  }
}

template <typename T>
static int sep2d(const void* in, void* out, int64_t np, int64_t n1, int64_t n2, const void* ha, int ka, int offa,
                 const void* hb, int kb, int offb, int vfirst, hipStream_t st) {
  using S = Sep2D<T>;
  if (!in || !out || !ha || !hb || np < 0 || n1 < 1 || n2 < 1 || ka < 1 || ka > kC1K || kb < 1 || kb > kC1K || offa < 0 ||
      offa >= ka || offb < 0 || offb >= kb || in == out)
    return PCS_EINVAL;
  if ((uintptr_t)in % 16 || (uintptr_t)out % 16) return PCS_EINVAL;
  if (np == 0) return PCS_OK;
  if (np * ((n1 + S::TY - 1) / S::TY) * ((n2 + S::TX - 1) / S::TX) >= (1LL << 31)) return PCS_EUNSUPPORTED;
  static int mode = -1;  // PCS_SEP2D_TILE=1: the tile kernel for the H-first order (diagnostics)
  if (mode < 0) {
    const char* e = getenv("PCS_SEP2D_TILE");
    mode = (e && e[0] == '1') ? 1 : 0;
  }
  if (vfirst)
    launch_sep2d<T, true>(in, out, np, n1, n2, ha, ka, offa, hb, kb, offb, st);
  else if (mode == 0 && n1 < (1LL << 30) && n2 < (1LL << 30))
    launch_sep2d_march<T>(in, out, np, n1, n2, ha, ka, offa, hb, kb, offb, st);
  else
    launch_sep2d<T, false>(in, out, np, n1, n2, ha, ka, offa, hb, kb, offb, st);
  return launch_status();
}

template <typename T>
static int conv1d(const void* x, void* out, int ndim, const int64_t* dims, int axis, const void* taps, int k, int off,
                  hipStream_t st) {
  // any ndim: the axis is the middle one of (outer, dims[axis], sa)
  if (!x || !out || !taps || !dims || ndim < 1 || ndim > 32 || axis < 0 || axis >= ndim || k < 1 || off < 0 ||
      off >= k)
    return PCS_EINVAL;
  int64_t N = 1, sa = 1, outer = 1;
  for (int i = 0; i < ndim; ++i) {
    if (dims[i] < 1) return PCS_EINVAL;
    N *= dims[i];
  }
  for (int i = axis + 1; i < ndim; ++i) sa *= dims[i];
  for (int i = 0; i < axis; ++i) outer *= dims[i];
  constexpr int VN = V16<T>::N;
  const bool al = ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0);
  if (k <= kC1K && al && sa > 1 && sa % VN == 0) {
    constexpr int RUN = sizeof(T) == 4 ? 16 : 8;
    const int64_t work = outer * ((dims[axis] + RUN - 1) / RUN) * (sa / VN);
    k_conv1d_strided<T, RUN><<<grid_for(work, 256, 1u << 20), 256, 0, st>>>(
        (const T*)x, (T*)out, outer, dims[axis], sa, (const T*)taps, k, off);
    return launch_status();
  }
  if (k <= kC1K && al && sa == 1 && dims[axis] % VN == 0) {
    const int64_t rows = outer, na = dims[axis];
    if (rows * ((na + VN * 64 - 1) / (VN * 64)) < (1LL << 31)) {
      // threads per row segment: the fewest (64 / 128 / 256) that cover the row, else 256
      if (na <= 64 * VN)
        launch_contig<T, 64>((const T*)x, (T*)out, rows, na, (const T*)taps, k, off, st);
      else if (na <= 128 * VN)
        launch_contig<T, 128>((const T*)x, (T*)out, rows, na, (const T*)taps, k, off, st);
      else
        launch_contig<T, 256>((const T*)x, (T*)out, rows, na, (const T*)taps, k, off, st);
      return launch_status();
    }
  }
  k_conv1d<T><<<grid_for(N, 256), 256, 0, st>>>((const T*)x, (T*)out, N, dims[axis], sa, (const T*)taps, k, off);
  return launch_status();
}

int corr2d_raw(int dt, const void* x, void* out, int64_t n0, int64_t n1, const void* psf, int kh, int kw, int off0,
               int off1, const void* b, double beta, hipStream_t st);  // corr2d.hip

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_conv2d(int dt, const void* x, void* out, int64_t n0, int64_t n1, const void* psf, int kh, int kw, int off0,
               int off1, const void* b, double beta, hipStream_t st) {
  if (x && x == out) return PCS_EINVAL;  // the stencil reads neighbours of every output
  if ((dt == PCS_F32 || dt == PCS_F64) && x && out && psf) {
    // odd square centred PSFs (3..15, 31): the register-blocked marching kernel (corr2d.hip)
    const int rc = corr2d_raw(dt, x, out, n0, n1, psf, kh, kw, off0, off1, b, beta, st);
    if (rc != PCS_EUNSUPPORTED) return rc;
  }
  if (dt == PCS_F32) return conv2d<float>(x, out, n0, n1, psf, kh, kw, off0, off1, b, beta, st);
  if (dt == PCS_F64) return conv2d<double>(x, out, n0, n1, psf, kh, kw, off0, off1, b, beta, st);
  return PCS_EINVAL;
}

int pcs_conv2d_sep_planes(int dt, const void* in, void* out, int64_t nplanes, int64_t n1, int64_t n2, const void* ha,
                          int ka, int offa, const void* hb, int kb, int offb, int vfirst, hipStream_t st) {
  if (dt == PCS_F32) return sep2d<float>(in, out, nplanes, n1, n2, ha, ka, offa, hb, kb, offb, vfirst, st);
  if (dt == PCS_F64) return sep2d<double>(in, out, nplanes, n1, n2, ha, ka, offa, hb, kb, offb, vfirst, st);
  return PCS_EINVAL;
}

int pcs_conv0_residual_adjoint(int dt, const void* t, const void* y, void* s, int64_t nsub, int64_t plane,
                               const void* taps, int k, int off, int64_t img_lo, int64_t img_hi, int64_t q0, int64_t q1,
                               hipStream_t st) {
  if (dt == PCS_F32) return conv0_rta<float>(t, y, s, nsub, plane, taps, k, off, img_lo, img_hi, q0, q1, st);
  if (dt == PCS_F64) return conv0_rta<double>(t, y, s, nsub, plane, taps, k, off, img_lo, img_hi, q0, q1, st);
  return PCS_EINVAL;
}

int pcs_conv1d(int dt, const void* x, void* out, int ndim, const int64_t* dims, int axis, const void* taps, int k,
               int off, hipStream_t st) {
  if (dt == PCS_F32) return conv1d<float>(x, out, ndim, dims, axis, taps, k, off, st);
  if (dt == PCS_F64) return conv1d<double>(x, out, ndim, dims, axis, taps, k, off, st);
  return PCS_EINVAL;
}

}  // extern "C"
