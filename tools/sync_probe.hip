// Cost of cross-stream synchronisation between dependent kernels on one GPU (diagnostics for
// the slab loop schedule): a chain of N streaming kernels (each ~25 us) on stream A, with
//   none     : plain back-to-back launches
//   event    : hipEventRecord(A) + hipStreamWaitEvent(B) + a tiny kernel on B every launch
//   waitval  : hipStreamWriteValue32(A) + hipStreamWaitValue32(B) + a tiny kernel on B
//   pingpong : A waits on B's previous tiny kernel (event) before each launch
//   two      : two kernels per iteration on A (a long one, then a short one), no sync
//   twosync  : the same, the short one waits for B's tiny kernel of the previous iteration
//              (recorded while A ran the long kernel), then A records for B
// Prints us per iteration for each mode.
//   hipcc --offload-arch=gfx950 -O3 tools/sync_probe.hip -o build/sync_probe && ./build/sync_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void k_stream(const float4* __restrict__ a, float4* __restrict__ b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float4 v = a[i];
    v.x += 1.f;
    b[i] = v;
  }
}
__global__ void k_tiny(float* p) {
  if (threadIdx.x == 0) p[0] += 1.f;
}

int main() {
  const long n = 16L << 20;  // 16 Mi float4 = 256 MiB read + 256 MiB write... too long; use 4 Mi
  const long m = 4L << 20;
  float4 *a, *b;
  float* t;
  unsigned* flag;
  CK(hipMalloc(&a, n * sizeof(float4)));
  CK(hipMalloc(&b, n * sizeof(float4)));
  CK(hipMalloc(&t, 64));
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(a, 0, n * sizeof(float4)));
  CK(hipMemset(flag, 0, 64));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  hipEvent_t e0, e1, ev, evb;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&evb, hipEventDisableTiming));
  const int N = 400;
  const char* names[] = {"none", "event", "waitval", "pingpong", "two", "twosync"};
  for (int mode = 0; mode < 6; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipMemset(flag, 0, 64));
      CK(hipEventRecord(e0, A));
      for (int i = 0; i < N; ++i) {
        if (mode == 3 && i > 0) CK(hipStreamWaitEvent(A, evb, 0));
        k_stream<<<2048, 256, 0, A>>>(a, b, m);
        if (mode >= 4) {
          if (mode == 5 && i > 0) CK(hipStreamWaitEvent(A, evb, 0));
          k_stream<<<256, 256, 0, A>>>(a, b, m / 16);
          if (mode == 5) {
            CK(hipEventRecord(ev, A));
            CK(hipStreamWaitEvent(B, ev, 0));
            k_tiny<<<1, 64, 0, B>>>(t);
            CK(hipEventRecord(evb, B));
          }
        }
        if (mode == 1 || mode == 3) {
          CK(hipEventRecord(ev, A));
          CK(hipStreamWaitEvent(B, ev, 0));
          k_tiny<<<1, 64, 0, B>>>(t);
          if (mode == 3) CK(hipEventRecord(evb, B));
        } else if (mode == 2) {
          CK(hipStreamWriteValue32(A, flag, (unsigned)(i + 1), 0));
          CK(hipStreamWaitValue32(B, flag, (unsigned)(i + 1), hipStreamWaitValueGte, 0xffffffffu));
          k_tiny<<<1, 64, 0, B>>>(t);
        }
      }
      CK(hipEventRecord(e1, A));
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 1) printf("%-9s %.2f us/iter\n", names[mode], ms * 1e3f / N);
    }
  }
  return 0;
}
