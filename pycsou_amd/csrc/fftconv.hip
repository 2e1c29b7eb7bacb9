// FFT-domain Convolve2D (pycsou/linop/conv.py:167-295 with method='fft', the reference default:
// scipy.signal.fftconvolve(mode='same') at pycsou's offset) for PSFs too wide for the direct
// register-blocked correlation (corr2d.hip, <= 31 taps).  The cost no longer grows with the PSF:
//   forward  out[i] = sum_j h[j] x[i + off - j]      = y_full[i + off]
//   adjoint  out[i] = sum_j h[j] x[i - off + j]      = circular correlation at i - off
// both exact (no wrap-around) on zero-padded P0 x P1 grids with P >= block + k - 1 (overlap-add):
//   scatter x into blocks of b0 x b1 (each zero-padded to P0 x P1) -> batched R2C -> multiply by H
//   (or conj H) -> batched C2R -> crop: out[i] = sum over the (at most 2 x 2) blocks whose
//   linear-convolution support holds i of block[i +- off - origin] (+ beta b)
// Blocks keep every transform length small enough for rocFFT's one-kernel sizes (the whole
// 4096^2 image at 63 taps needs 4374-point transforms: two-level, transposes; 2048-blocks need
// 2160).  H = the R2C of the zero-padded PSF times 1 / (P0 P1), formed once per plan.  The transforms are
// rocFFT's (library FFTs, BASELINE configs[2] "via rocFFT"); padding, spectrum product and crop
// are the kernels below (HBM-bound, 16-B groups where the rows allow).  Every call is stream
// ordered with no allocation or host synchronisation, so it is hipGraph-capturable.
#include <rocfft/rocfft.h>

#include <stdlib.h>

#include <new>

#include "common.hpp"

namespace pcs {

struct FftConv {
  int dtype;
  int64_t n0, n1, P0, P1, H1;  // image, padded grid of one block, P1 / 2 + 1 spectrum columns
  int64_t b0, b1, nb0, nb1;    // block size and counts (overlap-add)
  int kh, kw, off0, off1;
  rocfft_plan fwd = nullptr, inv = nullptr;
  rocfft_execution_info info = nullptr;
  void* work = nullptr;
  size_t work_bytes = 0;
  void* pad = nullptr;   // real P0 x P1
  void* spec = nullptr;  // complex P0 x H1
  void* hf = nullptr;    // complex P0 x H1: spectrum of the padded PSF / (P0 P1)
};

// smallest even n' >= n whose prime factors are 2, 3, 5, 7 (rocFFT radices); PCS_FFT_GRID=<m>
// (diagnostics) forces m when m >= n
static int64_t fft_size(int64_t n) {
  const char* e = getenv("PCS_FFT_GRID");
  if (e && atoll(e) >= n) return atoll(e);
  for (int64_t m = n + (n & 1);; m += 2) {
    int64_t r = m;
    for (int p : {2, 3, 5, 7})
      while (r % p == 0) r /= p;
    if (r == 1) return m;
  }
}

// block (q0, q1) of x (rows [q0 b0, q0 b0 + b0), columns [q1 b1, ...) of the image) at the top-left
// of its zero-padded P0 x P1 grid; blocks are stored one after the other
template <typename T>
__global__ void k_fft_pad(const T* __restrict__ x, T* __restrict__ pad, int64_t n0, int64_t n1, int64_t P0,
                          int64_t P1, int64_t b0, int64_t b1, int64_t nb1, int64_t nblk) {
  const int64_t per = P0 * P1, total = nblk * per;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = i / per, e = i - q * per, r = e / P1, c = e - r * P1;
    const int64_t q0 = q / nb1, q1 = q - q0 * nb1;
    const int64_t gr = q0 * b0 + r, gc = q1 * b1 + c;
    pad[i] = (r < b0 && c < b1 && gr < n0 && gc < n1) ? x[gr * n1 + gc] : T(0);
  }
}

// spec *= hf (or conj(hf)) for every block, complex interleaved (hf: one block's spectrum)
template <typename T, bool CONJ>
__global__ void k_fft_mul(T* __restrict__ spec, const T* __restrict__ hf, int64_t n, int64_t per) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i % per;
    const T a = spec[2 * i], b = spec[2 * i + 1];
    const T c = hf[2 * k], d = CONJ ? -hf[2 * k + 1] : hf[2 * k + 1];
    spec[2 * i] = a * c - b * d;
    spec[2 * i + 1] = a * d + b * c;
  }
}

// out[i] = sum over blocks q of blk_q[(i + s - origin_q) mod P] for i + s - origin_q in [lo, lo + b + k - 1)
// (forward: s = off, lo = 0; adjoint: s = -off, lo = -(k - 1)) (+ beta b[i])
template <typename T>
__global__ void k_fft_crop(const T* __restrict__ pad, T* __restrict__ out, const T* __restrict__ b, T beta, int64_t n0,
                           int64_t n1, int64_t P0, int64_t P1, int64_t s0, int64_t s1, int64_t b0, int64_t b1,
                           int64_t nb0, int64_t nb1, int64_t lo0, int64_t lo1, int64_t len0, int64_t len1) {
  const int64_t total = n0 * n1, per = P0 * P1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n1, c = i - r * n1;
    const int64_t t0 = r + s0, t1 = c + s1;  // block q contributes at t - origin_q in [lo, lo + len)
    // candidate block rows: origin in (t0 - lo0 - len0, t0 - lo0]
    int64_t qa0 = (t0 - lo0 - len0) / b0 + 1, qb0 = (t0 - lo0) / b0;
    if (t0 - lo0 - len0 < 0) qa0 = 0;
    if (t0 - lo0 < 0) qb0 = -1;
    qb0 = qb0 < nb0 - 1 ? qb0 : nb0 - 1;
    int64_t qa1 = (t1 - lo1 - len1) / b1 + 1, qb1 = (t1 - lo1) / b1;
    if (t1 - lo1 - len1 < 0) qa1 = 0;
    if (t1 - lo1 < 0) qb1 = -1;
    qb1 = qb1 < nb1 - 1 ? qb1 : nb1 - 1;
    T v = T(0);
    for (int64_t q0 = qa0; q0 <= qb0; ++q0) {
      int64_t m0 = t0 - q0 * b0;
      m0 = m0 < 0 ? m0 + P0 : m0;
      for (int64_t q1 = qa1; q1 <= qb1; ++q1) {
        int64_t m1 = t1 - q1 * b1;
        m1 = m1 < 0 ? m1 + P1 : m1;
        v += pad[(q0 * nb1 + q1) * per + m0 * P1 + m1];
      }
    }
    if (b != nullptr) v += beta * b[i];
    out[i] = v;
  }
}

// block length along an axis of n samples: at most PCS_FFT_BLOCK (default 2048; 0 = no blocks)
static int64_t fft_block(int64_t n) {
  const char* e = getenv("PCS_FFT_BLOCK");
  const int64_t bmax = e ? atoll(e) : 2048;
  return (bmax > 0 && n > bmax) ? bmax : n;
}

static unsigned fgrid(int64_t n) { return grid_for(n, 256, 256 * 16); }

static int fft_exec(FftConv* f, rocfft_plan p, void* in, void* out, hipStream_t st) {
  if (rocfft_execution_info_set_stream(f->info, st) != rocfft_status_success) return PCS_ELAUNCH;
  void* ib[1] = {in};
  void* ob[1] = {out};
  return rocfft_execute(p, ib, ob, f->info) == rocfft_status_success ? launch_status() : PCS_ELAUNCH;
}

template <typename T>
static int fft_apply(FftConv* f, const T* x, T* out, int adjoint, const T* b, double beta, hipStream_t st) {
  const int64_t nblk = f->nb0 * f->nb1;
  k_fft_pad<T><<<fgrid(nblk * f->P0 * f->P1), 256, 0, st>>>(x, (T*)f->pad, f->n0, f->n1, f->P0, f->P1, f->b0, f->b1,
                                                             f->nb1, nblk);
  int rc = launch_status();
  if (rc == PCS_OK) rc = fft_exec(f, f->fwd, f->pad, f->spec, st);
  if (rc != PCS_OK) return rc;
  const int64_t per = f->P0 * f->H1, ns = nblk * per;
  if (adjoint)
    k_fft_mul<T, true><<<fgrid(ns), 256, 0, st>>>((T*)f->spec, (const T*)f->hf, ns, per);
  else
    k_fft_mul<T, false><<<fgrid(ns), 256, 0, st>>>((T*)f->spec, (const T*)f->hf, ns, per);
  rc = launch_status();
  if (rc == PCS_OK) rc = fft_exec(f, f->inv, f->spec, f->pad, st);
  if (rc != PCS_OK) return rc;
  const int64_t s0 = adjoint ? -f->off0 : f->off0, s1 = adjoint ? -f->off1 : f->off1;
  const int64_t lo0 = adjoint ? -(f->kh - 1) : 0, lo1 = adjoint ? -(f->kw - 1) : 0;
  k_fft_crop<T><<<fgrid(f->n0 * f->n1), 256, 0, st>>>((const T*)f->pad, out, b, (T)beta, f->n0, f->n1, f->P0, f->P1, s0,
                                                      s1, f->b0, f->b1, f->nb0, f->nb1, lo0, lo1, f->b0 + f->kh - 1,
                                                      f->b1 + f->kw - 1);
  return launch_status();
}

static void fft_free(FftConv* f) {
  if (!f) return;
  if (f->fwd) rocfft_plan_destroy(f->fwd);
  if (f->inv) rocfft_plan_destroy(f->inv);
  if (f->info) rocfft_execution_info_destroy(f->info);
  for (void* p : {f->work, f->pad, f->spec, f->hf})
    if (p) (void)hipFree(p);
  delete f;
}

static bool fft_setup_once() {
  static int ok = -1;
  if (ok < 0) ok = rocfft_setup() == rocfft_status_success;
  return ok == 1;
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int64_t pcs_fftconv2d_grid(int64_t n, int k) { return (n < 1 || k < 1) ? -1 : fft_size(fft_block(n) + k - 1); }

int pcs_fftconv2d_create(int dtype, int64_t n0, int64_t n1, const double* h, int kh, int kw, int off0, int off1,
                         void** handle) {
  if (!handle) return PCS_EINVAL;
  *handle = nullptr;
  if ((dtype != PCS_F32 && dtype != PCS_F64) || !h || n0 < 1 || n1 < 1 || kh < 1 || kw < 1 || off0 < 0 ||
      off0 >= kh || off1 < 0 || off1 >= kw)
    return PCS_EINVAL;
  if (!fft_setup_once()) return PCS_ELAUNCH;
  FftConv* f = new (std::nothrow) FftConv();
  if (!f) return PCS_ELAUNCH;
  f->dtype = dtype;
  f->n0 = n0, f->n1 = n1, f->kh = kh, f->kw = kw, f->off0 = off0, f->off1 = off1;
  f->b0 = fft_block(n0);
  f->b1 = fft_block(n1);
  f->nb0 = (n0 + f->b0 - 1) / f->b0;
  f->nb1 = (n1 + f->b1 - 1) / f->b1;
  f->P0 = fft_size(f->b0 + kh - 1);
  f->P1 = fft_size(f->b1 + kw - 1);
  f->H1 = f->P1 / 2 + 1;
  const int64_t nblk = f->nb0 * f->nb1;
  const size_t es = dtype == PCS_F32 ? 4 : 8;
  const rocfft_precision prec = dtype == PCS_F32 ? rocfft_precision_single : rocfft_precision_double;
  const size_t len[2] = {(size_t)f->P1, (size_t)f->P0};  // innermost first
  bool ok = rocfft_plan_create(&f->fwd, rocfft_placement_notinplace, rocfft_transform_type_real_forward, prec, 2, len,
                               (size_t)nblk, nullptr) == rocfft_status_success &&
            rocfft_plan_create(&f->inv, rocfft_placement_notinplace, rocfft_transform_type_real_inverse, prec, 2, len,
                               (size_t)nblk, nullptr) == rocfft_status_success &&
            rocfft_execution_info_create(&f->info) == rocfft_status_success;
  rocfft_plan h1 = nullptr;  // the PSF spectrum: one block's transform
  ok = ok && rocfft_plan_create(&h1, rocfft_placement_notinplace, rocfft_transform_type_real_forward, prec, 2, len, 1,
                                nullptr) == rocfft_status_success;
  size_t w0 = 0, w1 = 0, w2 = 0;
  ok = ok && rocfft_plan_get_work_buffer_size(f->fwd, &w0) == rocfft_status_success &&
       rocfft_plan_get_work_buffer_size(f->inv, &w1) == rocfft_status_success &&
       rocfft_plan_get_work_buffer_size(h1, &w2) == rocfft_status_success;
  f->work_bytes = w0 > w1 ? w0 : w1;
  f->work_bytes = f->work_bytes > w2 ? f->work_bytes : w2;
  ok = ok && (f->work_bytes == 0 || hipMalloc(&f->work, f->work_bytes) == hipSuccess) &&
       (f->work_bytes == 0 ||
        rocfft_execution_info_set_work_buffer(f->info, f->work, f->work_bytes) == rocfft_status_success) &&
       hipMalloc(&f->pad, (size_t)(nblk * f->P0 * f->P1) * es) == hipSuccess &&
       hipMalloc(&f->spec, (size_t)(nblk * f->P0 * f->H1) * 2 * es) == hipSuccess &&
       hipMalloc(&f->hf, (size_t)(f->P0 * f->H1) * 2 * es) == hipSuccess;

  if (ok) {  // H = R2C(zero-padded PSF) / (P0 P1), on the null stream, synchronised (setup only)
    const double scale = 1.0 / ((double)f->P0 * (double)f->P1);
    const int64_t np = f->P0 * f->P1;
    if (dtype == PCS_F32) {
      float* hp = new (std::nothrow) float[np];
      ok = hp != nullptr;
      if (ok) {
        for (int64_t i = 0; i < np; ++i) hp[i] = 0.f;
        for (int r = 0; r < kh; ++r)
          for (int c = 0; c < kw; ++c) hp[r * f->P1 + c] = (float)(h[r * kw + c] * scale);
        ok = hipMemcpy(f->pad, hp, (size_t)np * es, hipMemcpyHostToDevice) == hipSuccess;
        delete[] hp;
      }
    } else {
      double* hp = new (std::nothrow) double[np];
      ok = hp != nullptr;
      if (ok) {
        for (int64_t i = 0; i < np; ++i) hp[i] = 0.0;
        for (int r = 0; r < kh; ++r)
          for (int c = 0; c < kw; ++c) hp[r * f->P1 + c] = h[r * kw + c] * scale;
        ok = hipMemcpy(f->pad, hp, (size_t)np * es, hipMemcpyHostToDevice) == hipSuccess;
        delete[] hp;
      }
    }
    ok = ok && fft_exec(f, h1, f->pad, f->hf, nullptr) == PCS_OK && hipDeviceSynchronize() == hipSuccess;
  }
  if (h1) rocfft_plan_destroy(h1);
  if (!ok) {
    fft_free(f);
    return PCS_ELAUNCH;
  }
  *handle = f;
  return PCS_OK;
}

int pcs_fftconv2d_apply(void* handle, const void* x, void* out, int adjoint, const void* b, double beta,
                        hipStream_t st) {
  FftConv* f = (FftConv*)handle;
  if (!f || !x || !out || x == out) return PCS_EINVAL;
  if (f->dtype == PCS_F32) return fft_apply<float>(f, (const float*)x, (float*)out, adjoint, (const float*)b, beta, st);
  return fft_apply<double>(f, (const double*)x, (double*)out, adjoint, (const double*)b, beta, st);
}

int pcs_fftconv2d_destroy(void* handle) {
  fft_free((FftConv*)handle);
  return PCS_OK;
}

}  // extern "C"
