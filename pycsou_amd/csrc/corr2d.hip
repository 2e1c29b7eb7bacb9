// Fast general (non-separable) Convolve2D: register-blocked, row-marching direct
// correlation for PSFs up to 31 x 31.
//
// Replaces pylops.signalprocessing.Convolve2D (1.x) behind pycsou/linop/conv.py:294
// (forward = zero-boundary 'same' convolution, conv.py:243-260; adjoint = correlation,
// conv.py:266-278).  Every call is written as one correlation with a packed K x K window
// centred at Kc = K/2 (K odd, the "tier"):
//
//     out[r][c] = sum_{i,j < K} w[i][j] * x[r - Kc + i][c - Kc + j]   (x = 0 outside the image)
//
// forward:  w = flip(h')  where h' is h zero-padded into K x K with its offset at Kc,
// adjoint:  w = h'.  (pcs_conv2d_plan_pack builds w on the host; pcs_conv2d feeds an odd square
// centred PSF straight in, reading it flipped.)
//
// Kernel shape (gfx950): a 256-thread workgroup owns a strip of TW = 4*C columns and marches
// down a row segment TH = 64 rows at a time.  Each thread accumulates C consecutive outputs of
// one row (C*sizeof(T) = 64 B: 16 fp32 / 8 fp64) in registers.  The input rows live in an LDS
// ring of RS >= TH + K - 1 rows, each loaded from HBM once per strip segment.  For window row
// q the thread reads its C + K - 1 inputs (ds_read_b128) and does C*K FMAs with the K taps of
// row q, which are wave-uniform: one scalar-load row per q, held in SGPRs (one SGPR operand per
// v_fma), the next row loaded while the current one is in use.  The next window row's inputs
// are likewise read from LDS while the current one is consumed (an explicit lgkmcnt(0) at the
// top of each step, so the prefetch is never waited for early).  FMA : LDS-word = C*K : C+K-1
// (fp32, K = 15: 240 : 30).
// LDS banking: a b128 lane group (16 lanes) = 4 consecutive rows x 4 column chunks of 64 B; the
// row pitch is 16 B (mod 64 B) and the ring a multiple of 16 rows, so the 16 lanes hit 16
// distinct 16-B bank slots for every vector of the window -- conflict-free.
// The next block's input rows are loaded into registers before the current block is computed
// and written to the ring after it.  Tasks = strips x row segments sized so one launch fills
// the CUs once; the blockIdx -> task map is XCD-aware (neighbouring strips of a segment share
// their halo columns in one XCD's L2).
#include <type_traits>

#include "common.hpp"

// diagnostics variants (PCS_LIB_PATH builds, tools/conv2d_bench.py): register prefetch of the
// next block's rows (PRE).  Measured on 4096^2 fp32 (r2 session): SGPR taps (scalar loads),
// single-buffered input rows, 3-4 waves/SIMD register budgets and a one-burst read schedule
// were all equal or slower than this configuration (96.5-116 us against 97-98 us for k = 15).
#ifndef PCS_CORR_PRE
#define PCS_CORR_PRE 1
#endif
// spread the next row's LDS reads through the current row's FMAs (sched_group_barrier)
// instead of issuing them as one burst ahead of the FMAs
#ifndef PCS_CORR_SPREAD
#define PCS_CORR_SPREAD 1
#endif
#ifndef PCS_CORR_SPREAD_DIV
#define PCS_CORR_SPREAD_DIV 2
#endif
// ablations (timing only, wrong results): 1 = no FMAs, 2 = no ring fill
#ifndef PCS_CORR_ABLATE
#define PCS_CORR_ABLATE 0
#endif

namespace pcs {

namespace corr2d {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct V16 {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

// tier K (odd) and its packed-row stride (elements)
__host__ __device__ constexpr int row_stride(int K) { return K <= 15 ? 16 : 32; }

template <typename T, int K>
struct Cfg {
  static constexpr int V = 16 / sizeof(T);  // elements per 16 B
  static constexpr int C = 64 / sizeof(T);  // output columns per thread (4 vectors)
  static constexpr int TPR = 4;             // threads per row
  static constexpr int TW = TPR * C;        // strip width
  static constexpr int TH = 64;             // rows per marching block (one per thread group of 4)
  static constexpr int Kc = K / 2;
  static constexpr int LEFT = (Kc + V - 1) / V * V;  // LDS col 0 = strip col 0 - LEFT (16-B aligned)
  static constexpr int NB = (LEFT + C + Kc + V - 1) / V;  // b128 reads per thread per window row
  static constexpr int WIN = NB * V;
  static constexpr int PL = (TW - C) + WIN;  // logical row width (elements)
  static constexpr int PV = PL / V;          // 16-B vectors landed per row
  // physical pitch: >= PL, = 16 B mod 64 B (b128 conflict-free over 4 consecutive rows)
  static constexpr int PB = ((PL * (int)sizeof(T) + 47) / 64) * 64 + 16;
  static constexpr int P = PB / (int)sizeof(T);
  static constexpr int RS = (TH + K - 1 + 15) / 16 * 16;  // ring rows, multiple of 16
  static constexpr int KP = (K + V - 1) / V * V;  // taps per row in LDS (16-B multiple)
  static constexpr int RING_BYTES = RS * PB;
  static constexpr int LDS_BYTES = RING_BYTES + K * KP * (int)sizeof(T);
  static constexpr int NPRE = (TH * PV + 255) / 256;  // prefetch vectors per thread per block
};

// Ring fill helpers: vector e of a set of `rows` consecutive window rows starting at window row
// gw0 (global row g = gbase + gw), LDS cols [0, P) = global cols [cbase, cbase + P).
template <typename T, bool VEC>
__device__ __forceinline__ V16<T> load_vec(const T* __restrict__ x, int64_t n0, int64_t n1, int64_t g, int64_t gc) {
  V16<T> v;
  constexpr int V = 16 / sizeof(T);
  if (VEC) {
    if (g >= 0 && g < n0 && gc >= 0 && gc < n1) {
      *reinterpret_cast<uint4*>(v.v) = *reinterpret_cast<const uint4*>(x + g * n1 + gc);
    } else {
#pragma unroll
      for (int t = 0; t < V; ++t) v.v[t] = T(0);
    }
  } else {
    const bool rok = g >= 0 && g < n0;
#pragma unroll
    for (int t = 0; t < V; ++t) {
      const int64_t c = gc + t;
      v.v[t] = (rok && c >= 0 && c < n1) ? x[g * n1 + c] : T(0);
    }
  }
  return v;
}

template <typename T>
__device__ __forceinline__ void st_lds(T* p, const V16<T>& v) {
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(v.v);
}

__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }

template <typename T, int K, bool FLIP>
__device__ __forceinline__ T tap(const T* __restrict__ w, int ws, int i, int j) {
  return FLIP ? w[(K - 1 - i) * ws + (K - 1 - j)] : w[i * ws + j];
}

}  // namespace corr2d

// x: n0 x n1 image; out: n0 x n1; w: K rows of stride ws (FLIP: read w[K-1-i][K-1-j]);
// out = corr(x, w) + beta * b (b may be null).  Tasks: strips x segments, segment = seg rows.
template <typename T, int K, bool FLIP, bool VEC>
__global__ __launch_bounds__(256) void k_corr2d(const T* __restrict__ x, T* __restrict__ out, int64_t n0, int64_t n1,
                                                 const T* __restrict__ w, int ws, const T* __restrict__ b, T beta,
                                                 int64_t seg, int nstrips, int ntasks) {
  using Cf = corr2d::Cfg<T, K>;
  constexpr int V = Cf::V, C = Cf::C, TW = Cf::TW, TH = Cf::TH, Kc = Cf::Kc, LEFT = Cf::LEFT, NB = Cf::NB;
  constexpr int WIN = Cf::WIN, P = Cf::P, PV = Cf::PV, RS = Cf::RS, NPRE = Cf::NPRE;
  constexpr int KP = Cf::KP;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* ring = reinterpret_cast<T*>(smem_raw);
  T* tl = reinterpret_cast<T*>(smem_raw + Cf::RING_BYTES);  // taps [K][KP], correlation order

  int task = blockIdx.x;
  {  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> adjacent strips of a segment
    const int bb = blockIdx.x, qq = ntasks / 8, rr = ntasks % 8, xcd = bb % 8, kk = bb / 8;
    task = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + kk;
  }
  const int strip = task % nstrips;
  const int64_t sg = task / nstrips;
  const int64_t r0 = sg * seg;
  if (r0 >= n0) return;
  const int64_t r1 = min(n0, r0 + seg);
  const int64_t c0 = (int64_t)strip * TW;
  const int64_t cbase = c0 - LEFT;  // global col of LDS col 0
  const int64_t gbase = r0 - Kc;    // global row of window row 0
  const int nblk = (int)((r1 - r0 + TH - 1) / TH);

  // thread roles: b128 lane group (16 lanes) = 4 rows x 4 column chunks
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l5 = lane & 31;
  const int grp = (lane >> 5) * 2 + lane_grp(l5), idx = lane_idx(l5);
  const int trow = wv * 16 + grp * 4 + (idx >> 2);  // row in the block
  const int chunk = idx & 3;

  // ---- prologue: taps into LDS (zero columns past K), window rows [0, K-1) into ring slots 0..K-2
  for (int e = threadIdx.x; e < K * KP; e += 256) {
    const int i = e / KP, j = e - i * KP;
    tl[e] = j < K ? corr2d::tap<T, K, FLIP>(w, ws, i, j) : T(0);
  }
  for (int e = threadIdx.x; e < (K - 1) * PV; e += 256) {
    const int rr = e / PV, cv = e - rr * PV;
    corr2d::st_lds(ring + rr * P + cv * V, corr2d::load_vec<T, VEC>(x, n0, n1, gbase + rr, cbase + cv * V));
  }
  // block 0's new rows (window rows K-1 .. K-2+TH) into registers
  corr2d::V16<T> pre[NPRE];
  auto issue = [&](int blk) {
    const int64_t gw0 = (int64_t)blk * TH + (K - 1);
#pragma unroll
    for (int m = 0; m < NPRE; ++m) {
      const int e = threadIdx.x + m * 256;
      if (e < TH * PV) {
        const int rr = e / PV, cv = e - rr * PV;
        pre[m] = corr2d::load_vec<T, VEC>(x, n0, n1, gbase + gw0 + rr, cbase + cv * V);
      }
    }
  };
  if (PCS_CORR_PRE && PCS_CORR_ABLATE != 2) issue(0);

  for (int blk = 0; blk < nblk; ++blk) {
    if (!PCS_CORR_PRE && PCS_CORR_ABLATE != 2) issue(blk);
    {  // land the prefetched rows: window rows blk*TH + K-1 + rr -> ring slot mod RS
      const int s0 = (int)(((int64_t)blk * TH + (K - 1)) % RS);
#pragma unroll
      for (int m = 0; m < NPRE; ++m) {
        const int e = threadIdx.x + m * 256;
        if (e < TH * PV) {
          const int rr = e / PV, cv = e - rr * PV;
          int s = s0 + rr;
          if (s >= RS) s -= RS;
          corr2d::st_lds(ring + s * P + cv * V, pre[m]);
        }
      }
    }
    lds_barrier();
    if (PCS_CORR_PRE && PCS_CORR_ABLATE != 2 && blk + 1 < nblk) issue(blk + 1);

    const int64_t g = r0 + (int64_t)blk * TH + trow;  // this thread's output row
    // a wave whose 16 rows all lie past the segment skips the arithmetic
    if (r0 + (int64_t)blk * TH + wv * 16 < r1) {
      T acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = T(0);
      // fp32: b of this thread's outputs, loaded ahead of the FMAs (its latency was exposed at the store:
      // the fused-residual forward pass 0.0996 against 0.0886 ms for the plain adjoint, 4096^2 k = 15); fp64
      // keeps the load at the store (the 16 more registers would halve its occupancy)
      constexpr bool BPRE = sizeof(T) == 4;
      const int64_t gc = c0 + chunk * C;
      T bq[C];
      if (BPRE && b) {
#pragma unroll
        for (int c = 0; c < C; ++c) bq[c] = T(0);
        if (g < r1) {
          if (VEC) {
#pragma unroll
            for (int t = 0; t < C / V; ++t)
              if (gc + t * V < n1) {
                const corr2d::V16<T> bv = *reinterpret_cast<const corr2d::V16<T>*>(b + g * n1 + gc + t * V);
#pragma unroll
                for (int c = 0; c < V; ++c) bq[t * V + c] = bv.v[c];
              }
          } else {
#pragma unroll
            for (int c = 0; c < C; ++c)
              if (gc + c < n1) bq[c] = b[g * n1 + gc + c];
          }
        }
      }
      // ring slot of window row q = (blk*TH + trow + q) mod RS
      int s = (int)(((int64_t)blk * TH + trow) % RS);
      const T* lcol = ring + chunk * C;
      auto rd = [&](T (&dst)[WIN], int slot) {
        const T* p = lcol + slot * P;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          *reinterpret_cast<corr2d::u32x4*>(dst + t * V) = *reinterpret_cast<const corr2d::u32x4*>(p + t * V);
        }
      };
      auto fmas = [&](const T (&in)[WIN], const T (&h)[KP]) {
        if (PCS_CORR_ABLATE == 1) {
          acc[0] += in[LEFT] * h[0];
          return;
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int c = 0; c < C; ++c) acc[c] = corr2d::fma_t(h[j], in[LEFT - Kc + c + j], acc[c]);
      };
      // the window elements outside [LEFT-Kc, LEFT+C+Kc) are never used: an empty asm use of them
      // (after the step's FMAs, when the prefetch is needed next anyway) keeps every 16-B LDS
      // read whole (ds_read_b128 instead of narrowed, misaligned pieces)
      auto keep = [&](const T (&in)[WIN]) {
#pragma unroll
        for (int t = 0; t < WIN; ++t)
          if (t < LEFT - Kc || t >= LEFT + C + Kc) asm volatile("" ::"v"(in[t]));
      };
      // taps of window row q: LDS broadcast reads (every lane the same address)
      auto rdt = [&](T (&dst)[KP], int q) {
        const T* p = tl + q * KP;
#pragma unroll
        for (int t = 0; t < KP / V; ++t)
          *reinterpret_cast<corr2d::u32x4*>(dst + t * V) = *reinterpret_cast<const corr2d::u32x4*>(p + t * V);
      };
      // one LDS read, then GV FMAs, NR times (NR = the step's reads), over the first half of
      // this row's FMAs: the reads for the next row stream beside them and the second half
      // covers their latency
      auto spread = [&]() {
        constexpr int NR = NB + KP / V;
        constexpr int GV = C * K / (PCS_CORR_SPREAD_DIV * NR);
        if (PCS_CORR_SPREAD) {
#pragma unroll
          for (int t = 0; t < NR; ++t) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x002, GV, 0);  // VALU
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      T ia[WIN], ib[WIN], ha[KP], hb[KP];
      rd(ia, s);
      rdt(ha, 0);
      // two window rows per trip, the next row's inputs and taps read while the current row's
      // FMAs run (K odd: the last row after the loop).  spread() pins the schedule: left alone,
      // the machine scheduler sinks the prefetch reads to just before their use, so the next
      // row's LDS latency would not overlap this row's FMAs.
#pragma unroll 1
      for (int q = 0; q < K - 1; q += 2) {
        // everything this half consumes was requested a half-step ago: wait for it before
        // requesting the next row, so no wait inside the FMAs covers the fresh requests
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (++s == RS) s = 0;
        rd(ib, s);
        rdt(hb, q + 1);
        if (!PCS_CORR_SPREAD) __builtin_amdgcn_sched_barrier(0);
        fmas(ia, ha);
        spread();
        keep(ib);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (++s == RS) s = 0;
        rd(ia, s);
        rdt(ha, q + 2);
        if (!PCS_CORR_SPREAD) __builtin_amdgcn_sched_barrier(0);
        fmas(ib, hb);
        spread();
        keep(ia);
      }
      fmas(ia, ha);
      // ---- store (optionally + beta * b)
      if (g < r1) {
        if (VEC) {
#pragma unroll
          for (int t = 0; t < C / V; ++t) {
            if (gc + t * V < n1) {
              corr2d::V16<T> o;
#pragma unroll
              for (int c = 0; c < V; ++c) o.v[c] = acc[t * V + c];
              if (b) {
                corr2d::V16<T> bv;
                if (BPRE) {
#pragma unroll
                  for (int c = 0; c < V; ++c) bv.v[c] = bq[t * V + c];
                } else {
                  bv = *reinterpret_cast<const corr2d::V16<T>*>(b + g * n1 + gc + t * V);
                }
#pragma unroll
                for (int c = 0; c < V; ++c) o.v[c] = o.v[c] + beta * bv.v[c];
              }
              *reinterpret_cast<uint4*>(out + g * n1 + gc + t * V) = *reinterpret_cast<const uint4*>(o.v);
            }
          }
        } else {
#pragma unroll
          for (int c = 0; c < C; ++c) {
            if (gc + c < n1) {
              T o = acc[c];
              if (b) o = o + beta * (BPRE ? bq[c] : b[g * n1 + gc + c]);
              out[g * n1 + gc + c] = o;
            }
          }
        }
      }
    }
    lds_barrier();  // every read of the ring is done before the next landing overwrites it
  }
}

// (Round 5 built a matrix-core form of this correlation -- v_mfma_f32_16x16x4_f32 with the taps as A and
// one input row as B, bit-exact with this kernel -- and measured it slower: 0.096 against 0.089 ms per 4096^2
// pass, profiles/r5_corr_mfma_ab.txt.  Removed from the library in round 6; the source is in git history
// (commit e6cd0fe, k_corr2d_mf).)

namespace corr2d {

// smallest supported odd tier K with K/2 >= every one-sided extent of the PSF
static int tier(int kh, int kw, int off0, int off1) {
  if (kh < 1 || kw < 1 || off0 < 0 || off0 >= kh || off1 < 0 || off1 >= kw) return PCS_EINVAL;
  const int ext = max(max(off0, kh - 1 - off0), max(off1, kw - 1 - off1));
  static const int tiers[] = {3, 5, 7, 9, 11, 13, 15, 31};
  for (int t : tiers)
    if (t / 2 >= ext) return t;
  return PCS_EUNSUPPORTED;
}

template <typename T, int K, bool FLIP, bool VEC>
static int slots_for() {
  static const int slots = [] {
    int dev = 0, cus = 256, nb = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_corr2d<T, K, FLIP, VEC>, 256,
                                                     Cfg<T, K>::LDS_BYTES) != hipSuccess ||
        nb < 1)
      nb = 1;
    const char* e = getenv("PCS_CORR_ROUNDS");  // diagnostics: rounds of the resident workgroups
    const int rounds = e && atoi(e) > 0 ? atoi(e) : 1;
    return cus * nb * rounds;
  }();
  return slots;
}

template <typename T, int K, bool FLIP, bool VEC>
static int launch(const T* x, T* out, int64_t n0, int64_t n1, const T* w, int ws, const T* b, T beta, hipStream_t st) {
  using Cf = Cfg<T, K>;
  const int64_t nstrips = (n1 + Cf::TW - 1) / Cf::TW;
  const int64_t slots = slots_for<T, K, FLIP, VEC>();
  // segments per strip: fill the resident slots once; a segment keeps >= TH/2 rows (halo cost)
  int64_t segs = slots / nstrips;
  if (segs < 1) segs = 1;
  int64_t seg = (n0 + segs - 1) / segs;
  const int64_t min_seg = Cf::TH / 2;
  if (seg < min_seg) seg = min_seg;
  seg = (seg + 7) / 8 * 8;
  segs = (n0 + seg - 1) / seg;
  const int64_t ntasks = nstrips * segs;
  if (ntasks > 0x7fffffff) return PCS_EUNSUPPORTED;
  k_corr2d<T, K, FLIP, VEC><<<(unsigned)ntasks, 256, Cf::LDS_BYTES, st>>>(x, out, n0, n1, w, ws, b, beta, seg,
                                                                            (int)nstrips, (int)ntasks);
  return launch_status();
}

template <typename T, bool FLIP>
static int dispatch(int K, const void* x, void* out, int64_t n0, int64_t n1, const void* w, int ws, const void* b,
                    double beta, hipStream_t st) {
  const bool vec = n1 % (16 / (int64_t)sizeof(T)) == 0 && ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0) &&
                   (!b || (uintptr_t)b % 16 == 0);
  const T* xx = (const T*)x;
  T* oo = (T*)out;
  const T* ww = (const T*)w;
  const T* bb = (const T*)b;
  const T be = (T)beta;
#define PCS_CORR_CASE(KK)                                                                  \
  case KK:                                                                                 \
    return vec ? launch<T, KK, FLIP, true>(xx, oo, n0, n1, ww, ws, bb, be, st)          \
               : launch<T, KK, FLIP, false>(xx, oo, n0, n1, ww, ws, bb, be, st);
  switch (K) {
    PCS_CORR_CASE(3)
    PCS_CORR_CASE(5)
    PCS_CORR_CASE(7)
    PCS_CORR_CASE(9)
    PCS_CORR_CASE(11)
    PCS_CORR_CASE(13)
    PCS_CORR_CASE(15)
    PCS_CORR_CASE(31)
    default: return PCS_EUNSUPPORTED;
  }
#undef PCS_CORR_CASE
}

}  // namespace corr2d

// Used by pcs_conv2d (conv.hip) for odd square centred PSFs: forward = correlation with the
// PSF read flipped.  Returns PCS_EUNSUPPORTED if the shape is not such a tier.
int corr2d_raw(int dt, const void* x, void* out, int64_t n0, int64_t n1, const void* psf, int kh, int kw, int off0,
               int off1, const void* b, double beta, hipStream_t st) {
  if (kh != kw || kh % 2 == 0 || off0 != kh / 2 || off1 != kw / 2) return PCS_EUNSUPPORTED;
  const int K = corr2d::tier(kh, kw, off0, off1);
  if (K != kh) return PCS_EUNSUPPORTED;
  if (n0 < 1 || n1 < 1) return PCS_EINVAL;
  return dt == PCS_F32 ? corr2d::dispatch<float, true>(K, x, out, n0, n1, psf, kw, b, beta, st)
                       : corr2d::dispatch<double, true>(K, x, out, n0, n1, psf, kw, b, beta, st);
}

}  // namespace pcs

extern "C" {

int pcs_conv2d_plan_tier(int kh, int kw, int off0, int off1) { return pcs::corr2d::tier(kh, kw, off0, off1); }

int64_t pcs_conv2d_plan_bytes(int dtype, int kh, int kw, int off0, int off1) {
  const int K = pcs::corr2d::tier(kh, kw, off0, off1);
  if (K < 0) return K;
  if (dtype != PCS_F32 && dtype != PCS_F64) return PCS_EINVAL;
  return (int64_t)K * pcs::corr2d::row_stride(K) * (dtype == PCS_F32 ? 4 : 8);
}

int pcs_conv2d_plan_pack(int dtype, const double* psf, int kh, int kw, int off0, int off1, int adjoint,
                         void* plan_host) {
  const int K = pcs::corr2d::tier(kh, kw, off0, off1);
  if (K < 0) return K;
  if (!psf || !plan_host || (dtype != PCS_F32 && dtype != PCS_F64)) return PCS_EINVAL;
  const int ws = pcs::corr2d::row_stride(K), Kc = K / 2;
  const int s0 = Kc - off0, s1 = Kc - off1;  // h'[i + s0][j + s1] = h[i][j]
  for (int i = 0; i < K; ++i)
    for (int j = 0; j < ws; ++j) {
      double v = 0.0;
      if (j < K) {
        // forward: w = flip(h'), adjoint: w = h'
        const int ip = adjoint ? i : K - 1 - i, jp = adjoint ? j : K - 1 - j;
        const int hi = ip - s0, hj = jp - s1;
        if (hi >= 0 && hi < kh && hj >= 0 && hj < kw) v = psf[hi * kw + hj];
      }
      if (dtype == PCS_F32)
        reinterpret_cast<float*>(plan_host)[i * ws + j] = (float)v;
      else
        reinterpret_cast<double*>(plan_host)[i * ws + j] = v;
    }
  return PCS_OK;
}

int pcs_conv2d_planned(int dtype, const void* x, void* out, int64_t n0, int64_t n1, const void* plan, int tier,
                       const void* b, double beta, hipStream_t stream) {
  if (!x || !out || !plan || n0 < 1 || n1 < 1 || x == out || (b && b == out)) return PCS_EINVAL;
  if (tier < 3 || tier % 2 == 0) return PCS_EINVAL;
  const int ws = pcs::corr2d::row_stride(tier);
  if (dtype == PCS_F32) return pcs::corr2d::dispatch<float, false>(tier, x, out, n0, n1, plan, ws, b, beta, stream);
  if (dtype == PCS_F64) return pcs::corr2d::dispatch<double, false>(tier, x, out, n0, n1, plan, ws, b, beta, stream);
  return PCS_EINVAL;
}

}  // extern "C"
