// FFT-domain Convolve2D (pycsou/linop/conv.py:167-295 with method='fft', the reference default:
// scipy.signal.fftconvolve(mode='same') at pycsou's offset) for PSFs too wide for the direct
// register-blocked correlation (corr2d.hip, <= 31 taps).  The cost no longer grows with the PSF:
//   forward  out[i] = sum_j h[j] x[i + off - j]      = y_full[i + off]
//   adjoint  out[i] = sum_j h[j] x[i - off + j]      = circular correlation at i - off
// both exact (no wrap-around) on a zero-padded P0 x P1 grid with P >= n + k - 1:
//   pad x -> R2C -> multiply by H (or conj H) -> C2R -> crop (+ beta b)
// H = the R2C of the zero-padded PSF times 1 / (P0 P1), formed once per plan.  The transforms are
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
  int64_t n0, n1, P0, P1, H1;  // image, padded grid, P1 / 2 + 1 spectrum columns
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

template <typename T>
__global__ void k_fft_pad(const T* __restrict__ x, T* __restrict__ pad, int64_t n0, int64_t n1, int64_t P0,
                          int64_t P1) {
  const int64_t total = P0 * P1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / P1, c = i - r * P1;
    pad[i] = (r < n0 && c < n1) ? x[r * n1 + c] : T(0);
  }
}

// spec *= hf (or conj(hf)), complex interleaved
template <typename T, bool CONJ>
__global__ void k_fft_mul(T* __restrict__ spec, const T* __restrict__ hf, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const T a = spec[2 * i], b = spec[2 * i + 1];
    const T c = hf[2 * i], d = CONJ ? -hf[2 * i + 1] : hf[2 * i + 1];
    spec[2 * i] = a * c - b * d;
    spec[2 * i + 1] = a * d + b * c;
  }
}

// out[i][j] = pad[(i + s0) mod P0][(j + s1) mod P1] (+ beta b[i][j])
template <typename T>
__global__ void k_fft_crop(const T* __restrict__ pad, T* __restrict__ out, const T* __restrict__ b, T beta, int64_t n0,
                           int64_t n1, int64_t P0, int64_t P1, int64_t s0, int64_t s1) {
  const int64_t total = n0 * n1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n1, c = i - r * n1;
    int64_t pr = r + s0, pc = c + s1;
    pr = pr < 0 ? pr + P0 : (pr >= P0 ? pr - P0 : pr);
    pc = pc < 0 ? pc + P1 : (pc >= P1 ? pc - P1 : pc);
    T v = pad[pr * P1 + pc];
    if (b != nullptr) v += beta * b[i];
    out[i] = v;
  }
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
  k_fft_pad<T><<<fgrid(f->P0 * f->P1), 256, 0, st>>>(x, (T*)f->pad, f->n0, f->n1, f->P0, f->P1);
  int rc = launch_status();
  if (rc == PCS_OK) rc = fft_exec(f, f->fwd, f->pad, f->spec, st);
  if (rc != PCS_OK) return rc;
  const int64_t ns = f->P0 * f->H1;
  if (adjoint)
    k_fft_mul<T, true><<<fgrid(ns), 256, 0, st>>>((T*)f->spec, (const T*)f->hf, ns);
  else
    k_fft_mul<T, false><<<fgrid(ns), 256, 0, st>>>((T*)f->spec, (const T*)f->hf, ns);
  rc = launch_status();
  if (rc == PCS_OK) rc = fft_exec(f, f->inv, f->spec, f->pad, st);
  if (rc != PCS_OK) return rc;
  const int64_t s0 = adjoint ? -f->off0 : f->off0, s1 = adjoint ? -f->off1 : f->off1;
  k_fft_crop<T><<<fgrid(f->n0 * f->n1), 256, 0, st>>>((const T*)f->pad, out, b, (T)beta, f->n0, f->n1, f->P0, f->P1, s0,
                                                      s1);
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

int64_t pcs_fftconv2d_grid(int64_t n, int k) { return (n < 1 || k < 1) ? -1 : fft_size(n + k - 1); }

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
  f->P0 = fft_size(n0 + kh - 1);
  f->P1 = fft_size(n1 + kw - 1);
  f->H1 = f->P1 / 2 + 1;
  const size_t es = dtype == PCS_F32 ? 4 : 8;
  const rocfft_precision prec = dtype == PCS_F32 ? rocfft_precision_single : rocfft_precision_double;
  const size_t len[2] = {(size_t)f->P1, (size_t)f->P0};  // innermost first
  bool ok = rocfft_plan_create(&f->fwd, rocfft_placement_notinplace, rocfft_transform_type_real_forward, prec, 2, len,
                               1, nullptr) == rocfft_status_success &&
            rocfft_plan_create(&f->inv, rocfft_placement_notinplace, rocfft_transform_type_real_inverse, prec, 2, len,
                               1, nullptr) == rocfft_status_success &&
            rocfft_execution_info_create(&f->info) == rocfft_status_success;
  size_t w0 = 0, w1 = 0;
  ok = ok && rocfft_plan_get_work_buffer_size(f->fwd, &w0) == rocfft_status_success &&
       rocfft_plan_get_work_buffer_size(f->inv, &w1) == rocfft_status_success;
  f->work_bytes = w0 > w1 ? w0 : w1;
  ok = ok && (f->work_bytes == 0 || hipMalloc(&f->work, f->work_bytes) == hipSuccess) &&
       (f->work_bytes == 0 ||
        rocfft_execution_info_set_work_buffer(f->info, f->work, f->work_bytes) == rocfft_status_success) &&
       hipMalloc(&f->pad, (size_t)(f->P0 * f->P1) * es) == hipSuccess &&
       hipMalloc(&f->spec, (size_t)(f->P0 * f->H1) * 2 * es) == hipSuccess &&
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
    ok = ok && fft_exec(f, f->fwd, f->pad, f->hf, nullptr) == PCS_OK && hipDeviceSynchronize() == hipSuccess;
  }
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
